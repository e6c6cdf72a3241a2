# round 4, call a: GPU suite on the phase-A tree, the c5ms workload, MPN A/B baseline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04a_gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c5ms --steps 10 --warmup 3 > gpurun_out/r04a_c5ms.log 2>&1 && \
timeout -k 10 300 python tools/mpn_ab.py --workload c3 default > gpurun_out/r04a_mpnab.log 2>&1
echo rc=$?
tail -3 gpurun_out/r04a_gpu_tests.log
