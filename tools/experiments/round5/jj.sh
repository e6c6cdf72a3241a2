# round 5, call jj: the MPN GPU tests with graphs opt-in and the unbind logit lists, then c2 / c3 lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05jj_tests.txt 2>&1 &&
for k in 1 2; do
  timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --no-roofline --no-backbone --steps 200 > gpurun_out/r05jj_c2_$k.json 2>/dev/null &&
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --no-backbone --steps 60 > gpurun_out/r05jj_c3_$k.json 2>/dev/null || exit 1
done
tail -2 gpurun_out/r05jj_tests.txt
python - <<'PY'
import json
for w in ('c2', 'c3'):
    for k in (1, 2):
        d = json.loads(open(f'gpurun_out/r05jj_{w}_{k}.json').read().strip().splitlines()[-1])
        print(w, k, d['value'], d['ms_per_step'], d.get('schedule_probe'), d.get('capacity_graphs'))
PY
