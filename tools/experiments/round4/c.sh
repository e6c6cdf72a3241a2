# round 4, call c: GPU suite on the new edge-pass defaults; MPN A/B vs the round-3 pass; c3 and c5ms bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r04c_gpu_tests.log 2>&1
echo tests_rc=$?
timeout -k 10 300 python tools/mpn_ab.py --workload c3 base default noprio slowmath > gpurun_out/r04c_mpnab_c3.log 2>&1 && \
timeout -k 10 200 python bench.py --workload c3 --steps 20 > gpurun_out/r04c_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c5ms --steps 10 --warmup 3 > gpurun_out/r04c_c5ms.log 2>&1
echo rc=$?
tail -3 gpurun_out/r04c_gpu_tests.log
