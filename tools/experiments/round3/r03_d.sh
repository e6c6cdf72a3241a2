set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03d_mpn.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03d_c3.json 2> gpurun_out/r03d_c3.err
timeout -k 10 300 python bench.py --no-cpu-baseline --workload c3knn10 > gpurun_out/r03d_c3knn10.json 2> gpurun_out/r03d_c3knn10.err
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03d_trace -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 --streams 1 > gpurun_out/r03d_trace.log 2>&1
python tools/trace_report.py gpurun_out/r03d_trace/run_kernel_trace.csv 12 > gpurun_out/r03d_trace_report.md
