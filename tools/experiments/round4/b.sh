# round 4, call b: edge-pass variants (asm scans + attention-weight fold, fast exp/rcp, gather order, priority)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/mpn_ab.py --workload c3 base scan noscan fast gfirst prio all > gpurun_out/r04b_mpnab_c3.log 2>&1 && \
timeout -k 10 200 python tools/mpn_ab.py --workload c3knn10 base scan all > gpurun_out/r04b_mpnab_knn10.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_mpn.py tests/test_gpu_dist.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r04b_gpu_tests.log 2>&1
echo rc=$?
tail -3 gpurun_out/r04b_gpu_tests.log
