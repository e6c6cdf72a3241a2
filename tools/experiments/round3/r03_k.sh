set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread -k "symmetric or golden or oracle" > gpurun_out/r03k_mpn.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --workload c3knn10 --steps 20 > gpurun_out/r03k_knn10.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline --workload c2 --steps 50 > gpurun_out/r03k_c2.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline --workload c2fp32 --steps 50 > gpurun_out/r03k_c2fp32.json 2>/dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03k_c2trace -o run -- \
  python bench.py --workload c2 --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03k_c2trace.log 2>&1
python tools/trace_report.py gpurun_out/r03k_c2trace/run_kernel_trace.csv 12 > gpurun_out/r03k_c2trace_report.md
