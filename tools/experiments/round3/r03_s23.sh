set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s23_mpn.log 2>&1 || exit 1
for v in new base new base; do
  if [ $v = base ]; then L=build_ab/libpemp_base.so; else L=""; fi
  PEMP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --streams 1 > gpurun_out/r03s23_$v.json 2>/dev/null || exit 1
  python - $v >> gpurun_out/r03s23.txt <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/r03s23_{v}.json").read().strip().splitlines()[-1])
print(v, d["ms_per_step"], "edge", d["roofline"]["avg_launch_us"], "head", d["kernel_avg_us"]["edge_step_head"])
PY
done
