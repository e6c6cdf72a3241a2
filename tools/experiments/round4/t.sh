# round 4, call t: node update fused into the node-table launch — MPN suite, c2 / c3 / c3knn10 A/B against the
# separate launches (build_ab/libpemp_nosum.so)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpn.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/r04t_tests.log)"
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--workload c2 --steps 200" timeout -k 10 600 bash tools/ab.sh default nosum
mv gpurun_out/ab_default.log gpurun_out/ab_c2_default.log; mv gpurun_out/ab_nosum.log gpurun_out/ab_c2_nosum.log
AB_ARGS="--workload c3 --steps 30" timeout -k 10 600 bash tools/ab.sh default nosum
