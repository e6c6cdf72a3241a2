# round 6: construct_graph_start / PendingGraph.result -- bench steps pipelined (step i + 1 queued before step i is
# collected) and the e2e leg's count wait overlapped with the previous batch's host stages. Graph GPU tests, then
# alternating bench lines with and without the pipelining (PEMP_BENCH_NO_PIPELINE=1: round 5's loop).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06d}
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -k "pipelined or reentrant or capacity" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "tests $(tail -1 gpurun_out/${T}_tests.log)"
for wl in ${WLS:-c3 c2 c3knn10}; do
  for v in pipe old pipe old; do
    if [ $v = old ]; then export PEMP_BENCH_NO_PIPELINE=1; else unset PEMP_BENCH_NO_PIPELINE; fi
    timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-backbone > gpurun_out/${T}_${wl}_$v.json 2> gpurun_out/${T}_${wl}_$v.err || exit 1
    python - "$T" "$wl" "$v" <<'PY'
import json, sys
T, wl, v = sys.argv[1:]
d = json.loads(open(f"gpurun_out/{T}_{wl}_{v}.json").read().strip().splitlines()[-1])
e = d.get("e2e") or {}
print(wl, v, "value", d["value"], "ms", d["ms_per_step"], "serial", d["value_serial_steps"], "S", d["config"]["batches_in_flight"],
      "probe", d.get("schedule_probe"), "e2e", e.get("images_per_sec"), e.get("stage_host_ms_per_batch"), flush=True)
PY
  done
done
