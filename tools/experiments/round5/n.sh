# round 5, call n: graph-stage host preparation before the detection launch, MPN capacity call split into
# prepare / launch: graph + MPN parity, batch-1 (c2) and c3 lines, a c2 step trace for the host gaps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_mpn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05n_tests.log 2>&1
rc=$?; echo "graph+mpn tests rc=$rc $(tail -1 gpurun_out/r05n_tests.log)"; [ $rc -eq 0 ] || exit 1
for wl in c2 c2fp32 c3; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/r05n_$wl.json 2> gpurun_out/r05n_$wl.err || exit 1
  python - "$wl" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05n_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d.get('value_serial_steps'), d.get('e2e', {}).get('images_per_sec'))
PY
done
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05n_c2_trace -o run -- \
    python bench.py --workload c2 --profile-steps --steps 20 --warmup 5 > gpurun_out/r05n_c2_trace.log 2>&1 || exit 1
python tools/trace_step_stats.py gpurun_out/r05n_c2_trace/run_kernel_trace.csv 25 > gpurun_out/r05n_c2_steps.md || exit 1
tail -1 gpurun_out/r05n_c2_steps.md
