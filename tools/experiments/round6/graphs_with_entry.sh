# Capacity-mode forward replayed from HIP graphs (PEMP_GRAPHS=1) with the batch-step entry: c2 and c3 lines against
# direct launches, two alternating rounds; the graph counters of each run (captures / launches / refused).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2; do
  for wl in c2 c3; do
    for g in 0 1; do
      PEMP_GRAPHS=$g timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-backbone --steps 40 > gpurun_out/r06gr_${wl}_${g}_$round.log 2>&1 || exit 1
      python - "$wl graphs=$g r$round" "gpurun_out/r06gr_${wl}_${g}_$round.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], "serial", d.get("value_serial_steps"), "probe", d.get("schedule_probe"), d.get("capacity_graphs"))
PY
    done
  done
done
