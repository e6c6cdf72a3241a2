# round 5, call pp: the schedule probe with >= 20 ms trials: c2 twice, c2fp32, c3; the two-rank bench test
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r05pp_dist.log 2>&1 || { tail -20 gpurun_out/r05pp_dist.log; exit 1; }
tail -1 gpurun_out/r05pp_dist.log
for w in c2 c2fp32 c2 c3; do
  timeout -k 10 300 python bench.py --workload $w --no-backbone --no-cpu-baseline --no-roofline > gpurun_out/r05pp_$w.json 2> gpurun_out/r05pp_$w.err || exit 1
  python -c "
import json; d = json.loads(open('gpurun_out/r05pp_$w.json').read().strip().splitlines()[-1])
print('$w', d['value'], d['ms_per_step'], d.get('value_serial_steps'), d['schedule_probe'])"
done
