# Batch-step entry (pemp_step_fully_cap): GPU suite, then c2 / c2fp32 / c3 lines and the host timing of the step with
# the entry and without it (PEMP_STEP_ENTRY=0), alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06s}
PEMP_STEP_ENTRY=1 timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gt.log 2>&1; rc=$?
echo "suite rc $rc: $(tail -1 gpurun_out/${T}_gt.log)"
[ $rc -le 1 ] || exit 1
for round in 1 2; do
  for wl in c2 c2fp32 c3; do
    for v in entry noentry; do
      if [ $v = entry ]; then export PEMP_STEP_ENTRY=1; else export PEMP_STEP_ENTRY=0; fi
      timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-backbone --steps 20 > gpurun_out/${T}_${wl}_${v}_$round.log 2>&1 || { tail -20 gpurun_out/${T}_${wl}_${v}_$round.log; exit 1; }
      python - "$wl $v" "gpurun_out/${T}_${wl}_${v}_$round.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "serial", d.get("value_serial_steps"), "e2e", d.get("e2e_images_per_sec"), "e2e_stages", d.get("e2e", {}).get("stage_host_ms_per_batch"))
PY
    done
  done
done
export PEMP_STEP_ENTRY=1
for wl in c2 c3; do
  timeout -k 10 200 python tools/step_host_timing.py $wl 300 bench > gpurun_out/${T}_host_$wl.log 2>&1 || { tail -5 gpurun_out/${T}_host_$wl.log; exit 1; }
  head -3 gpurun_out/${T}_host_$wl.log
done
