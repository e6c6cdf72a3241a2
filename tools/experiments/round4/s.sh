# round 4, call s: capacity-mode forward replayed as a HIP graph — MPN + graph suites, c2 host profile, c2 / c3 A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpn.py tests/test_gpu_graph.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04s_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/r04s_tests.log)"
[ $rc -eq 0 ] || exit $rc
PEMP_CAP=1 timeout -k 10 200 python tools/host_cprofile.py c2 > gpurun_out/r04s_host_cap.txt 2>&1
echo "host rc=$? $(grep wall gpurun_out/r04s_host_cap.txt)"
AB_ARGS="--workload c2 --steps 200" timeout -k 10 600 bash tools/ab_env.sh c2g: c2nog:PEMP_NO_GRAPHS=1 c2nocap:PEMP_NO_CAP_MPN=1 c2g2:
AB_ARGS="--workload c3 --steps 30" timeout -k 10 600 bash tools/ab_env.sh c3g: c3nocap:PEMP_NO_CAP_MPN=1
