# round 5, call kk: cProfile of the end-to-end leg at c3 and c2 (tools/e2e_cprofile.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python tools/e2e_cprofile.py c3 60 > gpurun_out/r05kk_c3.txt 2>&1 &&
timeout -k 10 240 python tools/e2e_cprofile.py c2 200 > gpurun_out/r05kk_c2.txt 2>&1
