# round 4, call p: capacity-mode MPN (bind_mpn) — MPN + graph suites, then c2 / c2fp32 / c3 bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpn.py tests/test_gpu_graph.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04p_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/r04p_tests.log)"
[ $rc -eq 0 ] || exit $rc
for wl in c2 c2fp32 c3; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 50 --no-cpu-baseline > gpurun_out/r04p_$wl.log 2> gpurun_out/r04p_$wl.err
  echo "$wl rc=$?"
done
