set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03b_mpn.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03b_trace -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03b_trace.log 2>&1
python tools/trace_report.py gpurun_out/r03b_trace/run_kernel_trace.csv 12 > gpurun_out/r03b_trace_report.md
