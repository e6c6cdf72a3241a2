# round 4, call x: lean NMS predicates (positive-threshold test, per-lane max for the ranking mark) and VOP2 DPP
# horizontal maxima — graph suite, then c3 A/B against the previous tree (old) and without the DPP maxima (nodpp)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04x_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/r04x_tests.log)"
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--workload c3 --steps 30 --streams 1" timeout -k 10 600 bash tools/ab.sh default old nodpp default old
