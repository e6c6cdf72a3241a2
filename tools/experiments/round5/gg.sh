# round 5, call gg: c2 with HIP graphs on / off (PEMP_NO_GRAPHS), one and two streams, three interleaved rounds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2 3; do
  for s in 1 2; do
    timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --no-roofline --no-backbone --steps 200 --streams $s > gpurun_out/r05gg_g_s${s}_$k.json 2>/dev/null &&
    PEMP_NO_GRAPHS=1 timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --no-roofline --no-backbone --steps 200 --streams $s > gpurun_out/r05gg_ng_s${s}_$k.json 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json, statistics
for t in ('g', 'ng'):
    for s in (1, 2):
        v = [json.loads(open(f'gpurun_out/r05gg_{t}_s{s}_{k}.json').read().strip().splitlines()[-1])['ms_per_step'] for k in (1, 2, 3)]
        print(t, 'streams', s, v, 'median', statistics.median(v))
PY
