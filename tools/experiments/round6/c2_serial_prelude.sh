# round 6: at c2 (one image, ~22k edges) the prelude's fork / join cross-stream waits (7 + 11 us in the c2 step
# timeline) against the overlap they buy: PEMP_SERIAL_PRELUDE=1 (everything on the launch stream) vs the default,
# a c2 step trace each, then alternating bench lines for c2 and c2fp32
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06k}
for v in default serial; do
  if [ $v = default ]; then unset PEMP_SERIAL_PRELUDE; else export PEMP_SERIAL_PRELUDE=1; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_c2_${v}_trace -o run -- \
      python bench.py --workload c2 --profile-steps --steps 20 --warmup 5 > gpurun_out/${T}_c2_${v}_trace.log 2>&1 || exit 1
  python tools/step_timeline.py gpurun_out/${T}_c2_${v}_trace/run_kernel_trace.csv > gpurun_out/${T}_c2_${v}_step_timeline.txt || exit 1
  echo "$v c2 $(tail -1 gpurun_out/${T}_c2_${v}_step_timeline.txt)"
done
for wl in c2 c2fp32; do
  for v in default serial default serial default serial; do
    if [ $v = default ]; then unset PEMP_SERIAL_PRELUDE; else export PEMP_SERIAL_PRELUDE=1; fi
    timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-backbone > gpurun_out/${T}_${wl}_$v.json 2> gpurun_out/${T}_${wl}_$v.err || exit 1
    python - "$T" "$wl" "$v" <<'PY'
import json, sys
T, wl, v = sys.argv[1:]
d = json.loads(open(f"gpurun_out/{T}_{wl}_{v}.json").read().strip().splitlines()[-1])
print(wl, v, "value", d["value"], "ms", d["ms_per_step"], "serial", d["value_serial_steps"], "mpn_ms", d["mpn_ms_per_step"], flush=True)
PY
  done
done
unset PEMP_SERIAL_PRELUDE
