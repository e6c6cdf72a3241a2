# round 5, call ff: host-side breakdown of the c2 step with per-C-call times, HIP graphs on and off (PEMP_NO_GRAPHS),
# and the c2 line both ways
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python tools/step_host_timing.py c2 300 > gpurun_out/r05ff_c2.txt 2>&1 &&
PEMP_NO_GRAPHS=1 timeout -k 10 240 python tools/step_host_timing.py c2 300 > gpurun_out/r05ff_c2_nographs.txt 2>&1 &&
for k in 1 2; do
  timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --no-roofline --no-backbone --steps 100 > gpurun_out/r05ff_c2_g_$k.json 2>/dev/null &&
  PEMP_NO_GRAPHS=1 timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --no-roofline --no-backbone --steps 100 > gpurun_out/r05ff_c2_ng_$k.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for t in ('g', 'ng'):
    for k in (1, 2):
        d = json.loads(open(f'gpurun_out/r05ff_c2_{t}_{k}.json').read().strip().splitlines()[-1])
        print(t, k, d['value'], d['ms_per_step'], d.get('schedule_probe'))
PY
