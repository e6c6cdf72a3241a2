set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s18_mpn.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03s18_c3.json 2> gpurun_out/r03s18_c3.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --workload c3knn10 > gpurun_out/r03s18_knn.json 2> gpurun_out/r03s18_knn.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s18_stats -o run -- \
  python bench.py --workload c3knn10 --no-cpu-baseline --no-roofline --steps 10 --streams 1 > gpurun_out/r03s18_stats.log 2>&1
