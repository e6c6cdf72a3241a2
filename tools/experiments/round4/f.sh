# round 4, call f: the asm scans with the trailing DPP guard, bf16x3 + full MPN suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -q --timeout 200 --timeout-method thread > gpurun_out/r04f_mpn.log 2>&1
echo "rc=$? $(tail -1 gpurun_out/r04f_mpn.log)"; grep FAILED gpurun_out/r04f_mpn.log | head -5
