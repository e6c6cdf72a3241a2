# round 4, call e: which asm scan breaks bf16x3 (and does f16x3 break without the attention-weight fold)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in nomax nosum nofold; do
  export PEMP_LIB=$PWD/build_ab/libpemp_$v.so
  timeout -k 10 120 python -u -m pytest tests/test_gpu_mpn.py -q -k "golden and attn_t3" --timeout 100 --timeout-method thread > gpurun_out/r04e_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/r04e_$v.log)"; grep FAILED gpurun_out/r04e_$v.log | head -5
done
