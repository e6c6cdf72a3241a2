set -e
export TMPDIR=/tmp
PEMP_LIB=build_ab/libpemp_stamps.so timeout -k 10 200 python tools/edge_timeline.py 0 1 2 > gpurun_out/r03c_timeline.txt 2>&1
