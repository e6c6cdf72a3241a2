# round 5, call rr: the edge prelude side stream at the highest stream priority (PEMP_SIDE_PRIO=1 build), c3 / c3knn10 / c5,
# two rounds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2; do
  for w in c3 c3knn10 c5; do
    for v in default sideprio; do
      if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-roofline --no-backbone --steps 60 > gpurun_out/r05rr_${w}_${v}_$k.json 2> gpurun_out/r05rr_${w}_${v}_$k.err || exit 1
    done
  done
done
unset PEMP_LIB
python - <<'PY'
import json
for w in ('c3', 'c3knn10', 'c5'):
    for v in ('default', 'sideprio'):
        r = []
        for k in (1, 2):
            d = json.loads(open(f'gpurun_out/r05rr_{w}_{v}_{k}.json').read().strip().splitlines()[-1])
            r.append((round(d['value']), round(d.get('value_serial_steps') or 0), d['mpn_ms_per_step']))
        print(w, v, r)
PY
