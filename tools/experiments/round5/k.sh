# round 5, call k: batched finishing (pemp_pose_finish_batch) + grouping host part on the library thread:
# pose parity, then the c3 e2e leg and its host profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pose.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05k_pose_tests.log 2>&1
rc=$?; echo "pose tests rc=$rc $(tail -1 gpurun_out/r05k_pose_tests.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/e2e_cprofile.py c3 50 > gpurun_out/r05k_e2e_cprofile2.txt 2>&1 || exit 1
sed -n 2p gpurun_out/r05k_e2e_cprofile2.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05k_c3.json 2> gpurun_out/r05k_c3.err || exit 1
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r05k_c3.json').read().strip().splitlines()[-1])
print(d['value'], d.get('value_serial_steps'), json.dumps(d['e2e']))
PY
