set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread -k "symmetric or oracle" > gpurun_out/r03m_mpn.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03m_ktrace -o run -- \
  python bench.py --workload c3knn10 --no-cpu-baseline --no-roofline --steps 10 --streams 1 > gpurun_out/r03m_ktrace.log 2>&1
python tools/trace_report.py gpurun_out/r03m_ktrace/run_kernel_trace.csv 6 > gpurun_out/r03m_ktrace_report.md
PEMP_SERIAL_PRELUDE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03m_c3_serialprelude.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03m_c3.json 2>/dev/null
