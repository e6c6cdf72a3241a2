set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s6_mpn.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s6_c3.json 2>/dev/null && \
STAMP_OUT=gpurun_out/r03s6_st PEMP_LIB=build_ab/libpemp_stamps.so timeout -k 10 200 python tools/edge_timeline.py 0 > gpurun_out/r03s6_timeline.txt 2>&1
