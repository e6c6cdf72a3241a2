# e2e leg (bench.py e2e_pipeline: the GPU part on a high-priority stream) with the batch-step entry on and off
# (PEMP_STEP_ENTRY=0), alternating; c3 and c2.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06e}
for round in 1 2; do
  for wl in c3 c2; do
    for v in 1 0; do
      PEMP_STEP_ENTRY=$v timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-backbone --steps 20 > gpurun_out/${T}_${wl}_${v}_$round.log 2>&1 || { tail -20 gpurun_out/${T}_${wl}_${v}_$round.log; exit 1; }
      python - "$wl entry=$v" "gpurun_out/${T}_${wl}_${v}_$round.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "e2e", d.get("e2e_images_per_sec"), d.get("e2e", {}).get("stage_host_ms_per_batch"))
PY
    done
  done
done
