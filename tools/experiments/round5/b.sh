# round 5, call b: capacity-mode regression debug; asm-scan bisection variants on the bf16x3 goldens; GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug/cap_mode_debug.py > gpurun_out/r05b_capdbg.log 2>&1
echo "capdbg rc=$?"; cat gpurun_out/r05b_capdbg.log | tail -20
for v in asmall asmall_drain asmall_vol asmall_tail; do
  PEMP_LIB=$PWD/build_ab/libpemp_$v.so timeout -k 10 120 python -u -m pytest tests/test_gpu_mpn.py -q -k "golden and attn and bf16x3" --timeout 100 --timeout-method thread > gpurun_out/r05b_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/r05b_$v.log)"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05b_gpu_tests.log 2>&1
echo "suite rc=$? $(tail -1 gpurun_out/r05b_gpu_tests.log)"; grep FAILED gpurun_out/r05b_gpu_tests.log | head
