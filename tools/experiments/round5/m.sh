# round 5, call m: GAEC with split weight / edition triangles and compact edge lists: pose parity, host timing,
# c5 grouping and e2e legs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pose.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05m_pose_tests.log 2>&1
rc=$?; echo "pose tests rc=$rc $(tail -1 gpurun_out/r05m_pose_tests.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/gaec_bench.py 1 502 36 1 50 || exit 1
timeout -k 10 120 python tools/gaec_bench.py 8 153 9 1 50 || exit 1
timeout -k 10 120 python tools/gaec_bench.py 8 153 9 16 50 || exit 1
timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/r05m_c5.json 2> gpurun_out/r05m_c5.err || exit 1
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r05m_c5.json').read().strip().splitlines()[-1])
print(d['value'], d.get('value_serial_steps'), json.dumps(d['pose_grouping']), json.dumps(d['e2e']))
PY
