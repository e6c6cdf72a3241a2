set -o pipefail
export TMPDIR=/tmp
for v in def pc5 def pc5 def pc5; do
  if [ $v = def ]; then L=""; else L=build_ab/libpemp_$v.so; fi
  PEMP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s14_$v.json 2>/dev/null || exit 1
  python - $v >> gpurun_out/r03s14.txt <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/r03s14_{v}.json").read().strip().splitlines()[-1])
print(v, d["ms_per_step"], d["kernel_avg_us"]["detect_nms"])
PY
done
