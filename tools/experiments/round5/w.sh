# round 5, call w: PEMP_RESERVE_CUS sweep 0 / 64 / 96 / 128, alternating, c3 and c3knn10 (two batches in flight)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c3knn10; do
  for r in 0 64 96 128 0 64 96 128; do
    PEMP_RESERVE_CUS=$r timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-roofline --steps 40 --streams 2 > gpurun_out/r05w_${wl}_$r.json 2> gpurun_out/r05w_${wl}_$r.err || exit 1
    python - "$wl" "$r" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05w_{sys.argv[1]}_{sys.argv[2]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'reserve', sys.argv[2], d['value'], d['ms_per_step'], d.get('value_serial_steps'))
PY
  done
done
