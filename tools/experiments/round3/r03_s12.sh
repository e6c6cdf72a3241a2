set -o pipefail
export TMPDIR=/tmp
for v in pc5 pc8 def; do
  if [ $v = def ]; then L=""; else L=build_ab/libpemp_$v.so; fi
  PEMP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s12_$v.json 2>/dev/null || exit 1
done
