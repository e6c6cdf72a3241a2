# round 5, call a: GPU suite with the graph-capture fixes; the asm-vs-compiler scan check on the bf16x3 goldens
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05a_gpu_tests.log 2>&1
echo "suite rc=$? $(tail -1 gpurun_out/r05a_gpu_tests.log)"
PEMP_LIB=$PWD/build_ab/libpemp_asmchk.so timeout -k 10 120 python -u -m pytest tests/test_gpu_mpn.py -q -s -k "golden and attn and bf16x3" --timeout 100 --timeout-method thread > gpurun_out/r05a_asmchk.log 2>&1
echo "asmchk rc=$? $(tail -1 gpurun_out/r05a_asmchk.log)"
grep -c ASMCHK gpurun_out/r05a_asmchk.log || true
