set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread -k "symmetric or oracle" > gpurun_out/r03q_mpn.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03q_ktrace -o run -- \
  python bench.py --workload c3knn10 --no-cpu-baseline --no-roofline --steps 10 --streams 1 > gpurun_out/r03q_ktrace.log 2>&1
python tools/trace_report.py gpurun_out/r03q_ktrace/run_kernel_trace.csv 6 > gpurun_out/r03q_ktrace_report.md
PEMP_NO_SYM_PREPARE=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03q_ktrace_nosym -o run -- \
  python bench.py --workload c3knn10 --no-cpu-baseline --no-roofline --steps 10 --streams 1 > gpurun_out/r03q_ktrace_nosym.log 2>&1
python tools/trace_report.py gpurun_out/r03q_ktrace_nosym/run_kernel_trace.csv 6 > gpurun_out/r03q_ktrace_nosym_report.md
timeout -k 10 200 python bench.py --workload c3knn10 --no-cpu-baseline --steps 20 > gpurun_out/r03q_knn.json 2>/dev/null
PEMP_NO_SYM_PREPARE=1 timeout -k 10 200 python bench.py --workload c3knn10 --no-cpu-baseline --steps 20 > gpurun_out/r03q_knn_nosym.json 2>/dev/null
