set -e
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/r03i_base.json 2>/dev/null
PEMP_LIB=build_ab/libpemp_noq0.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/r03i_noq0.json 2>/dev/null
PEMP_LIB=build_ab/libpemp_stamps.so timeout -k 10 200 python tools/edge_timeline.py 0 > gpurun_out/r03i_tl_base.txt 2>&1
