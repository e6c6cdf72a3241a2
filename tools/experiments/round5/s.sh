# round 5, call s: graph build + MPN in one capacity-mode call / HIP graph (pemp_mpn_forward_fully_cap_built):
# graph + MPN parity, c2 / c3 lines, c2 step timeline; NMS counts from per-row ballots (c3 NMS time)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_mpn.py tests/test_gpu_pose.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05s_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r05s_tests.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r05s_tests.log | head; exit 1; }
for wl in c2 c2fp32 c3; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/r05s_$wl.json 2> gpurun_out/r05s_$wl.err || exit 1
  python - "$wl" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05s_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d.get('value_serial_steps'), d.get('schedule_probe'), d.get('capacity_graphs'))
PY
done
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05s_c2_trace -o run -- \
    python bench.py --workload c2 --profile-steps --steps 20 --warmup 5 > gpurun_out/r05s_c2_trace.log 2>&1 || exit 1
python tools/step_timeline.py gpurun_out/r05s_c2_trace/run_kernel_trace.csv
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05s_c3_trace -o run -- \
    python bench.py --workload c3 --profile-steps --steps 20 --warmup 5 > gpurun_out/r05s_c3_trace.log 2>&1 || exit 1
python tools/trace_step_stats.py gpurun_out/r05s_c3_trace/run_kernel_trace.csv 25 > gpurun_out/r05s_c3_steps.md || exit 1
grep -E "nms|plane_emit|sum of" gpurun_out/r05s_c3_steps.md
