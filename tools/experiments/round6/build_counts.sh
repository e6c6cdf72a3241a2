# round 6: the capacity graph build writes the batch's (N, E, overflow) for the capacity-mode MPN
# (PEMP_BUILD_WRITE_COUNTS / PEMP_MPN_COUNTS_IN_OFFSETS): no cap_counts launch on the step's critical path.
# MPN + graph GPU tests, a c3 / c2 step trace, then alternating bench lines against PEMP_NO_BUILD_COUNTS=1.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpn.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "tests $(tail -1 gpurun_out/${T}_tests.log)"
for wl in c3 c2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_${wl}_trace -o run -- \
      python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/${T}_${wl}_trace.log 2>&1 || exit 1
  python tools/step_timeline.py gpurun_out/${T}_${wl}_trace/run_kernel_trace.csv > gpurun_out/${T}_${wl}_step_timeline.txt || exit 1
  tail -1 gpurun_out/${T}_${wl}_step_timeline.txt
done
for wl in c3 c2; do
  for v in new old new old; do
    if [ $v = old ]; then export PEMP_NO_BUILD_COUNTS=1; else unset PEMP_NO_BUILD_COUNTS; fi
    timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-backbone > gpurun_out/${T}_${wl}_$v.json 2> gpurun_out/${T}_${wl}_$v.err || exit 1
    python - "$T" "$wl" "$v" <<'PY'
import json, sys
T, wl, v = sys.argv[1:]
d = json.loads(open(f"gpurun_out/{T}_{wl}_{v}.json").read().strip().splitlines()[-1])
print(wl, v, "value", d["value"], "ms", d["ms_per_step"], "serial", d["value_serial_steps"], "S", d["config"]["batches_in_flight"],
      "mpn_ms", d["mpn_ms_per_step"], "e2e", (d.get("e2e") or {}).get("images_per_sec"), flush=True)
PY
  done
done
unset PEMP_NO_BUILD_COUNTS
