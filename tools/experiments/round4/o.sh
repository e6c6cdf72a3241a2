# round 4, call o: fused select + emit: rank-based top-k, one-word relaxed publication — graph suite (incl. detection edge cases and the
# two-kernel path on a large plane), c3 bench, phase clocks
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/r04o_tests.log)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --no-cpu-baseline > gpurun_out/r04o_c3.log 2> gpurun_out/r04o_c3.err
echo "bench rc=$?"
PEMP_LIB=$PWD/build_ab/libpemp_clocks.so timeout -k 10 200 python bench.py --workload c3 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04o_clocks.log 2>&1
echo "clocks rc=$?"
timeout -k 10 300 python -u bench.py --workload c2 --steps 50 --no-cpu-baseline > gpurun_out/r04o_c2.log 2> gpurun_out/r04o_c2.err
echo "c2 rc=$?"
