# round 5, call v: one-workgroup-per-CU launches (edge passes, embedding) leaving PEMP_RESERVE_CUS CUs to the other
# batch in flight: MPN parity at 32 reserved, then c3 / c3knn10 throughput for 0 / 16 / 32 / 64
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PEMP_RESERVE_CUS=32 timeout -k 10 500 python -u -m pytest tests/test_gpu_mpn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05v_mpn_tests.log 2>&1
rc=$?; echo "mpn tests (32 reserved) rc=$rc $(tail -1 gpurun_out/r05v_mpn_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r05v_mpn_tests.log | head; exit 1; }
for wl in c3 c3knn10; do
  for r in 0 16 32 64 0 32; do
    PEMP_RESERVE_CUS=$r timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-roofline --steps 40 > gpurun_out/r05v_${wl}_$r.json 2> gpurun_out/r05v_${wl}_$r.err || exit 1
    python - "$wl" "$r" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05v_{sys.argv[1]}_{sys.argv[2]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'reserve', sys.argv[2], d['value'], d['ms_per_step'], d.get('value_serial_steps'), d.get('schedule_probe'))
PY
  done
done
