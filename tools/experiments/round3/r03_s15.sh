set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s15_mpn.log 2>&1 || exit 1
for v in def pc5 def pc5; do
  if [ $v = def ]; then L=""; else L=build_ab/libpemp_$v.so; fi
  PEMP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s15_$v.json 2>/dev/null || exit 1
  python - $v >> gpurun_out/r03s15.txt <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/r03s15_{v}.json").read().strip().splitlines()[-1])
k = d["kernel_avg_us"]
print(v, d["ms_per_step"], "nms", k["detect_nms"], "edge", d["roofline"]["avg_launch_us"], "head", k["edge_step_head"])
PY
done
