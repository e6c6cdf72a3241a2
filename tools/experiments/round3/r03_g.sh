set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03g_mpn.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03g_c3.json 2>/dev/null
PEMP_NO_FUSED_NODE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 > gpurun_out/r03g_c3_nofuse.json 2>/dev/null
timeout -k 10 200 python bench.py --no-cpu-baseline --workload c3knn10 --steps 20 > gpurun_out/r03g_knn10.json 2>/dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03g_ktrace -o run -- \
  python bench.py --workload c3knn10 --no-cpu-baseline --no-roofline --steps 10 --streams 1 > gpurun_out/r03g_ktrace.log 2>&1
python tools/trace_report.py gpurun_out/r03g_ktrace/run_kernel_trace.csv 6 > gpurun_out/r03g_ktrace_report.md
PEMP_LIB=build_ab/libpemp_stamps.so timeout -k 10 200 python tools/edge_timeline.py 0 2 > gpurun_out/r03g_timeline.txt 2>&1
