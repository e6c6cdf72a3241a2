# round 5, call e: asm-scan race hunt (LDS zeroed at start / inputs pinned); the GPU suite with the test fixes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in asmall asmall_zero asmall_opq; do
  PEMP_LIB=$PWD/build_ab/libpemp_$lib.so timeout -k 10 60 python -u tools/debug/determinism.py mpn_attn_t3 bf16x3 10 | sed "s/^/$lib /"
  PEMP_LIB=$PWD/build_ab/libpemp_$lib.so timeout -k 10 60 python -u tools/debug/determinism.py mpn_attn_t3 fp32 10 | sed "s/^/$lib /"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05e_gpu_tests.log 2>&1
echo "suite rc=$? $(tail -1 gpurun_out/r05e_gpu_tests.log)"; grep FAILED gpurun_out/r05e_gpu_tests.log | head
