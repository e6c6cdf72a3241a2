set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s3_mpn.log 2>&1 && \
AB_ARGS="--no-roofline" bash tools/ab_env.sh base:PEMP_LIB=build_ab/libpemp_base.so new: base2:PEMP_LIB=build_ab/libpemp_base.so new2: > gpurun_out/r03s3_ab.txt 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r03s3_c3.json 2>/dev/null && \
STAMP_OUT=gpurun_out/r03s3_st PEMP_LIB=build_ab/libpemp_stamps.so timeout -k 10 200 python tools/edge_timeline.py 0 2 > gpurun_out/r03s3_timeline.txt 2>&1
