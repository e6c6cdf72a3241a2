# round 5, call ii: c3 and c3knn10 with HIP graphs on / off (PEMP_NO_GRAPHS), two streams, three interleaved rounds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2 3; do
  for w in c3 c3knn10; do
    timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-roofline --no-backbone --steps 60 --streams 2 > gpurun_out/r05ii_g_${w}_$k.json 2>/dev/null &&
    PEMP_NO_GRAPHS=1 timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-roofline --no-backbone --steps 60 --streams 2 > gpurun_out/r05ii_ng_${w}_$k.json 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json, statistics
for w in ('c3', 'c3knn10'):
    for t in ('g', 'ng'):
        v = [json.loads(open(f'gpurun_out/r05ii_{t}_{w}_{k}.json').read().strip().splitlines()[-1])['value'] for k in (1, 2, 3)]
        print(w, t, [round(x) for x in v], 'median', round(statistics.median(v)))
PY
