# round 6: the seg_sum17_asm question. Determinism of ten forwards of one golden graph with the
# asm sums in every attention instantiation (asmall: the known timing-dependent build), the same with the DPP moved
# from the v_fmac_f32 onto a v_mov_b32 into a temporary (asmall_nofmacdpp), the default build and the build without
# asm sums (nosums); then the cost of the asm sums in the default f16x3 path (isolated MPN at c3 / c3knn10).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06b}
for lib in default asmall asmall_nofmacdpp nosums; do
  if [ $lib = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$lib.so; fi
  for prec in bf16x3 f16x3 fp32; do
    timeout -k 10 90 python -u tools/debug/determinism.py mpn_attn_t3 $prec 10 2>&1 | tail -1 | sed "s/^/$lib /" || exit 1
  done
done | tee gpurun_out/${T}_determinism.txt
unset PEMP_LIB
for wl in c3 c3knn10; do
  timeout -k 10 300 python tools/mpn_ab.py --workload $wl --iters 40 default nosums default nosums > gpurun_out/${T}_ab_$wl.txt 2>&1 || exit 1
  cat gpurun_out/${T}_ab_$wl.txt
done
