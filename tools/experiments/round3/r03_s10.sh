set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s10_mpn.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s10_c3.json 2>/dev/null && \
PEMP_NO_SUM_TABLE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s10_c3_off.json 2>/dev/null && \
timeout -k 10 200 python bench.py --workload c3knn10 --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s10_knn.json 2>/dev/null && \
PEMP_NO_SUM_TABLE=1 timeout -k 10 200 python bench.py --workload c3knn10 --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s10_knn_off.json 2>/dev/null && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s10_kstats -o run -- \
  python bench.py --workload c3knn10 --no-cpu-baseline --no-roofline --steps 10 --streams 1 > gpurun_out/r03s10_kstats.log 2>&1
