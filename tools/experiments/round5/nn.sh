# round 5, call nn: node-table tiles per workgroup (PEMP_TBL_TILES 1 / 2 / 4 default / 8) at c3knn10 and c3, two rounds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2; do
  for w in c3knn10 c3; do
    for v in default tbl1 tbl2 tbl8; do
      if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-roofline --no-backbone --steps 40 > gpurun_out/r05nn_${w}_${v}_$k.json 2> gpurun_out/r05nn_${w}_${v}_$k.err || exit 1
    done
  done
done
unset PEMP_LIB
python - <<'PY'
import json
for w in ('c3knn10', 'c3'):
    for v in ('default', 'tbl1', 'tbl2', 'tbl8'):
        r = []
        for k in (1, 2):
            d = json.loads(open(f'gpurun_out/r05nn_{w}_{v}_{k}.json').read().strip().splitlines()[-1])
            r.append((round(d['value']), d['mpn_ms_per_step']))
        print(w, v, r)
PY
