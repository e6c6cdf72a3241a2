# round 4, call j: per-type parallel scan of the symmetric prepare; node_table tiles per workgroup (4 / 2 / 1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -q --timeout 200 --timeout-method thread > gpurun_out/r04j_mpn.log 2>&1
echo "mpn tests rc=$? $(tail -1 gpurun_out/r04j_mpn.log)"
timeout -k 10 300 python tools/mpn_ab.py --workload c3knn10 prev default tbl2 tbl1 > gpurun_out/r04j_ab_knn10.log 2>&1
echo "ab knn rc=$?"
timeout -k 10 300 python tools/mpn_ab.py --workload c3 default tbl2 tbl1 > gpurun_out/r04j_ab_c3.log 2>&1
echo "ab c3 rc=$?"
