# round 4, call l: 4-columns-per-lane NMS (nms_quads_kernel) — graph suite (detection parity incl. edge cases),
# then the c3 bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/r04l_tests.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --no-cpu-baseline > gpurun_out/r04l_c3.log 2> gpurun_out/r04l_c3.err
echo "bench rc=$?"
