# round 5, call dd: PEMP_RESERVE_CUS 32 / 48 / 64 / 80 / 96 at c3, four rounds interleaved (two streams)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2 3 4; do
  for r in 32 48 64 80 96; do
    PEMP_RESERVE_CUS=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 40 --streams 2 > gpurun_out/r05dd_${r}_$k.json 2> gpurun_out/r05dd_${r}_$k.err || exit 1
  done
done
python - <<'PY'
import json, statistics
for r in (32, 48, 64, 80, 96):
    v = [json.loads(open(f'gpurun_out/r05dd_{r}_{k}.json').read().strip().splitlines()[-1])['value'] for k in (1, 2, 3, 4)]
    print(r, [round(x) for x in v], 'median', round(statistics.median(v)))
PY
