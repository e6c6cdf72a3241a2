# round 5, call oo: node-table 2 tiles per workgroup as the default: GPU suite, smoke, c3knn10 / c3 / c2 lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05oo_gt.log 2>&1 || { tail -30 gpurun_out/r05oo_gt.log; exit 1; }
echo "suite ok $(tail -1 gpurun_out/r05oo_gt.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05oo_smoke.log 2>&1 || exit 1
echo "smoke ok"
for w in c3knn10 c3 c2; do
  timeout -k 10 300 python bench.py --workload $w --no-backbone > gpurun_out/r05oo_$w.json 2> gpurun_out/r05oo_$w.err || exit 1
done
python - <<'PY'
import json
for w in ('c3knn10', 'c3', 'c2'):
    d = json.loads(open(f'gpurun_out/r05oo_{w}.json').read().strip().splitlines()[-1])
    print(w, d['value'], d['ms_per_step'], 'mpn', d['mpn_ms_per_step'], 'frac', d['roofline']['frac'], 'e2e', d['e2e_images_per_sec'], d['kernel_avg_us'].get('node_table'))
PY
