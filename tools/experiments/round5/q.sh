# round 5, call q: + the image DMA issued after the first tile gather: MPN parity, per-shape times
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_mpn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05q_mpn_tests.log 2>&1
rc=$?; echo "mpn tests rc=$rc $(tail -1 gpurun_out/r05q_mpn_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r05q_mpn_tests.log | head; exit 1; }
for wl in c3 c3knn10 c2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05q_${wl}_trace -o run -- \
      python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/r05q_${wl}_trace.log 2>&1 || exit 1
  python tools/trace_step_stats.py gpurun_out/r05q_${wl}_trace/run_kernel_trace.csv 25 > gpurun_out/r05q_${wl}_steps.md || exit 1
  echo "== $wl"; grep -E "embed|sum of" gpurun_out/r05q_${wl}_steps.md
done
for wl in c3 c2; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/r05q_$wl.json 2> gpurun_out/r05q_$wl.err || exit 1
  python - "$wl" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05q_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d.get('value_serial_steps'))
PY
done
