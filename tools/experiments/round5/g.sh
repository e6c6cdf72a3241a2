# round 5, call g: pose GPU tests (refine skips detected joints), c3 bench (e2e)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pose.py -q --timeout 120 --timeout-method thread > gpurun_out/r05g_pose_tests.log 2>&1
echo "pose tests rc=$? $(tail -1 gpurun_out/r05g_pose_tests.log)"
timeout -k 10 300 python bench.py > gpurun_out/r05g_c3.json 2> gpurun_out/r05g_c3.err; echo "c3 rc=$?"
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r05g_c3.json').read().strip().splitlines()[-1])
print(d['value'], d['value_serial_steps'], d['e2e'])
print(d['pose_grouping'])
PY
