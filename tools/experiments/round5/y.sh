# round 5, call y: the NMS strip kernel leaving PEMP_NMS_RESERVE_CUS CUs free (0 / 32 / 64), c3 and c3knn10 lines
# (alternating), detection parity at 64
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PEMP_NMS_RESERVE_CUS=64 timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py -q -x -k "detect or golden" --timeout 120 --timeout-method thread > gpurun_out/r05y2_tests.log 2>&1
rc=$?; echo "graph tests (NMS 64 reserved) rc=$rc $(tail -1 gpurun_out/r05y2_tests.log)"; [ $rc -eq 0 ] || exit 1
for wl in c3 c3knn10; do
  for r in 0 32 64 0 32 64; do
    PEMP_NMS_RESERVE_CUS=$r timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-roofline --steps 40 --streams 2 > gpurun_out/r05y2_${wl}_$r.json 2> gpurun_out/r05y2_${wl}_$r.err || exit 1
    python - "$wl" "$r" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05y2_{sys.argv[1]}_{sys.argv[2]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'nms reserve', sys.argv[2], d['value'], d['ms_per_step'], d.get('value_serial_steps'))
PY
  done
done
