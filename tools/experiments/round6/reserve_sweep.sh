# CU reservation of the edge passes / embedding (PEMP_RESERVE_CUS) on the round-6 tree (batch-step entry): c3 and
# c3knn10 lines for 0 / 32 / 64 / 96 reserved CUs, two alternating rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c3knn10; do
  for round in 1 2; do
    for r in 64 0 32 96; do
      PEMP_RESERVE_CUS=$r timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-backbone --steps 20 > gpurun_out/r06r_${wl}_${r}_$round.log 2>&1 || exit 1
      python - "$wl reserve=$r r$round" "gpurun_out/r06r_${wl}_${r}_$round.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], "serial", d.get("value_serial_steps"), "probe", d.get("schedule_probe"))
PY
    done
  done
done
