# round 5, call i: fused node update + table (node_sum_table_kernel), parity + per-shape time + A/B over the
# column blocks per wave (PEMP_NST_BPW; -1 = the two launches it replaces)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mpn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05i_mpn_tests.log 2>&1
rc=$?; echo "mpn tests rc=$rc $(tail -1 gpurun_out/r05i_mpn_tests.log)"; [ $rc -eq 0 ] || exit 1
for wl in c3knn10 c3; do
  for b in -1 5 3 2; do
    PEMP_NST_BPW=$b timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05i_${wl}_b$b -o run -- \
        python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/r05i_${wl}_b$b.log 2>&1 || exit 1
    echo "== $wl bpw=$b"
    python tools/trace_step_stats.py gpurun_out/r05i_${wl}_b$b/run_kernel_trace.csv 25 > gpurun_out/r05i_${wl}_b$b.md || exit 1
    grep -E "node_|sum of" gpurun_out/r05i_${wl}_b$b.md
  done
done
for wl in c3knn10 c3; do
  for b in -1 5; do
    PEMP_NST_BPW=$b timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/r05i_${wl}_b$b.json 2> gpurun_out/r05i_${wl}_b$b.err || exit 1
    python - "$wl" "$b" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05i_{sys.argv[1]}_b{sys.argv[2]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], d['value'], d.get('value_serial_steps'), d.get('mpn_ms_per_step'))
PY
  done
done
