set -e
export TMPDIR=/tmp
PEMP_HOST_TRACE=1 timeout -k 10 120 python tools/host_trace.py c3 > gpurun_out/r03l_ht_c3.txt 2>&1
PEMP_HOST_TRACE=1 timeout -k 10 120 python tools/host_trace.py c2 > gpurun_out/r03l_ht_c2.txt 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03l_ktrace -o run -- \
  python bench.py --workload c3knn10 --no-cpu-baseline --no-roofline --steps 10 --streams 1 > gpurun_out/r03l_ktrace.log 2>&1
python tools/trace_report.py gpurun_out/r03l_ktrace/run_kernel_trace.csv 6 > gpurun_out/r03l_ktrace_report.md
