set -e
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 > gpurun_out/r03e_c3.json 2> gpurun_out/r03e_c3.err
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03e_trace -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03e_trace.log 2>&1
python tools/trace_report.py gpurun_out/r03e_trace/run_kernel_trace.csv 12 > gpurun_out/r03e_trace_report.md
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03e_ktrace -o run -- \
  python bench.py --workload c3knn10 --no-cpu-baseline --no-roofline --steps 10 --streams 1 > gpurun_out/r03e_ktrace.log 2>&1
python tools/trace_report.py gpurun_out/r03e_ktrace/run_kernel_trace.csv 6 > gpurun_out/r03e_ktrace_report.md
timeout -k 10 120 python tools/diag/host_timeline.py > gpurun_out/r03e_host.txt 2>&1
