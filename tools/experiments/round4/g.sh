# round 4, call g: GPU suite on the tree (asm scans on the folded f16x3 path only, e2e grouping API); bench c3, c5ms
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/r04g_gpu_tests.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/r04g_gpu_tests.log)"; grep FAILED gpurun_out/r04g_gpu_tests.log | head -8
timeout -k 10 400 python -u bench.py --workload c3 --steps 20 > gpurun_out/r04g_c3.log 2> gpurun_out/r04g_c3.err
echo "c3 rc=$?"
timeout -k 10 400 python -u bench.py --workload c5ms --steps 10 --warmup 3 > gpurun_out/r04g_c5ms.log 2> gpurun_out/r04g_c5ms.err
echo "c5ms rc=$?"
