# round 5, call u: the finishing chained on the grouping thread (GroupingJob.then): pose parity, the c3 e2e leg
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pose.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05u_pose_tests.log 2>&1
rc=$?; echo "pose tests rc=$rc $(tail -1 gpurun_out/r05u_pose_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r05u_pose_tests.log | head; exit 1; }
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05u_c3_$i.json 2> gpurun_out/r05u_c3_$i.err || exit 1
python - $i <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05u_c3_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print('c3', d['value'], d.get('value_serial_steps'), json.dumps(d['e2e']))
PY
done
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/r05u_c5.json 2> gpurun_out/r05u_c5.err || exit 1
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r05u_c5.json').read().strip().splitlines()[-1])
print('c5', d['value'], json.dumps(d['e2e']))
PY
