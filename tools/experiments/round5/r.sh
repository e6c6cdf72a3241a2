# round 5, call r: embedding image DMA after the first gather; 32-bit / multiply-shift index division in the graph
# builds: graph + MPN parity, per-shape times, c3 / c2 lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_mpn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05r_tests.log 2>&1
rc=$?; echo "graph+mpn tests rc=$rc $(tail -1 gpurun_out/r05r_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r05r_tests.log | head; exit 1; }
for wl in c3 c3knn10 c2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05r_${wl}_trace -o run -- \
      python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/r05r_${wl}_trace.log 2>&1 || exit 1
  python tools/trace_step_stats.py gpurun_out/r05r_${wl}_trace/run_kernel_trace.csv 25 > gpurun_out/r05r_${wl}_steps.md || exit 1
  echo "== $wl"; grep -E "embed|fused_fully|pack_nodes|edge_features|sum of" gpurun_out/r05r_${wl}_steps.md
done
for wl in c3 c2; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/r05r_$wl.json 2> gpurun_out/r05r_$wl.err || exit 1
  python - "$wl" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05r_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d.get('value_serial_steps'))
PY
done
