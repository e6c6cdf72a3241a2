set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s11_graph.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s11_c3.json 2>/dev/null && \
PEMP_LIB=build_ab/libpemp_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s11_c3_base.json 2>/dev/null
