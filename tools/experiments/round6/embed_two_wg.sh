# Edge embedding with two workgroups per CU (build_ab/libpemp_e<W>x2.so: W waves each, its own LDS image, the register
# target W x 2 / 4 waves per SIMD) against the in-tree one (16 waves, one per CU): c3 and c3knn10 lines, two rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c3knn10; do
  for round in 1 2; do
    AB_ARGS="--no-backbone --workload $wl" bash tools/ab.sh default e10x2 e8x2 e12x2 | sed "s/^/$wl r$round /" || exit 1
  done
done
