# round 5, call mm: end-to-end leg with the GPU parts on one vs two alternating streams (PEMP_E2E_STREAMS), two rounds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2; do
  for w in c3 c3knn10; do
    for s in 1 2; do
      PEMP_E2E_STREAMS=$s timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-backbone --steps 40 > gpurun_out/r05mm_${w}_s${s}_$k.json 2> gpurun_out/r05mm_${w}_s${s}_$k.err || exit 1
    done
  done
done
python - <<'PY'
import json
for w in ('c3', 'c3knn10'):
    for s in (1, 2):
        for k in (1, 2):
            d = json.loads(open(f'gpurun_out/r05mm_{w}_s{s}_{k}.json').read().strip().splitlines()[-1])
            e = d['e2e']
            print(w, 'streams', s, k, 'e2e', e['images_per_sec'], e['stage_host_ms_per_batch'])
PY
