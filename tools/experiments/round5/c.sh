# round 5, call c: capacity-mode debug; asm check variants (poison on mismatch / asm present but results dropped)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTHONPATH=$PWD timeout -k 10 120 python -u tools/debug/cap_mode_debug.py > gpurun_out/r05c_capdbg.log 2>&1
echo "capdbg rc=$?"; tail -25 gpurun_out/r05c_capdbg.log
for v in chk_poison chk_usecomp; do
  PEMP_LIB=$PWD/build_ab/libpemp_$v.so timeout -k 10 120 python -u -m pytest tests/test_gpu_mpn.py -q -s -k "golden and attn_t3 and bf16x3" --timeout 100 --timeout-method thread > gpurun_out/r05c_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/r05c_$v.log)"; grep "AssertionError: assert" gpurun_out/r05c_$v.log | head -3; grep -c ASMCHK gpurun_out/r05c_$v.log
done
