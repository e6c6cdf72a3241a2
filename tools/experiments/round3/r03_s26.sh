# host-side cProfile of the serial step (c2, c3)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python tools/host_cprofile.py c2 > gpurun_out/r03s26_c2.txt 2>&1 || exit 1
timeout -k 10 200 python tools/host_cprofile.py c3 > gpurun_out/r03s26_c3.txt 2>&1 || exit 1
