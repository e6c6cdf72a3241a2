# round 5, call ll: end-to-end leg with the GPU parts alternating between two streams (c3, c5, c2, c3knn10)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in c3 c5 c2 c3knn10; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-backbone > gpurun_out/r05ll_$w.json 2> gpurun_out/r05ll_$w.err || exit 1
done
python - <<'PY'
import json
for w in ('c3', 'c5', 'c2', 'c3knn10'):
    d = json.loads(open(f'gpurun_out/r05ll_{w}.json').read().strip().splitlines()[-1])
    e = d['e2e']
    print(w, d['value'], 'e2e', e['images_per_sec'], 'serial', e['serial_images_per_sec'], 'persons', e['persons_per_batch'], e['stage_host_ms_per_batch'])
PY
