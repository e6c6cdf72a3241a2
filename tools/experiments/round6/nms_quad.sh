# Split dense NMS (nms_quad_kernel, 4 columns per lane): detection / graph GPU tests, then the c3 line with the quad
# pass and with the strip kernel (PEMP_NMS_QUAD=0), alternating; detect_nms / detect_select_emit from kernel_avg_us.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06q}
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_graph.log 2>&1 || { tail -40 gpurun_out/${T}_graph.log; exit 1; }
echo "graph tests: $(tail -1 gpurun_out/${T}_graph.log)"
for round in 1 2; do
  for q in 1 0; do
    PEMP_NMS_QUAD=$q timeout -k 10 200 python bench.py --no-cpu-baseline --no-backbone --steps 20 > gpurun_out/${T}_b${q}_${round}.log 2>&1 || { tail -20 gpurun_out/${T}_b${q}_${round}.log; exit 1; }
    python - "$q" "gpurun_out/${T}_b${q}_${round}.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d["kernel_avg_us"]
print("quad", sys.argv[1], d["value"], d["ms_per_step"], "serial", d.get("value_serial_steps"), "nms", k.get("detect_nms"), "emit", k.get("detect_select_emit"), "frac", d["roofline"]["frac"])
PY
  done
done
