# round 4, call ac: fused node update + table with 2 / 4 / 5 column blocks per wave (fewer groups re-reading the
# aggregates) vs the two launches (default at c3 / c3knn10): MPN suite on cb4, then one-stream A/B on c3knn10 and c3
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PEMP_LIB=$PWD/build_ab/libpemp_cb4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mpn.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04ac_tests.log 2>&1
rc=$?
echo "tests(cb4) rc=$rc $(tail -1 gpurun_out/r04ac_tests.log)"
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--workload c3knn10 --steps 20 --streams 1" timeout -k 10 700 bash tools/ab.sh default cb2 cb4 cb5 default
for v in default cb2 cb4 cb5; do cp gpurun_out/ab_$v.log gpurun_out/ab_knn_$v.log; done
AB_ARGS="--workload c3 --steps 30 --streams 1" timeout -k 10 600 bash tools/ab.sh default cb4 cb5 default
