# round 5, call h: embedding in the f16x3 domain (parity + time + SQ), c3 bench with the three-stage e2e leg
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mpn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05h_mpn_tests.log 2>&1
echo "mpn tests rc=$? $(tail -1 gpurun_out/r05h_mpn_tests.log)"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05h_c3_trace -o run -- \
    python bench.py --workload c3 --profile-steps --steps 20 --warmup 5 > gpurun_out/r05h_c3_trace.log 2>&1 || exit 1
python tools/trace_step_stats.py gpurun_out/r05h_c3_trace/run_kernel_trace.csv 25 | head -8
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-include-regex "edge_embed" --output-format csv -d gpurun_out/r05h_sq1 -o pmc -- python bench.py --workload c3 --profile-steps --steps 3 --warmup 1 > gpurun_out/r05h_sq1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r05h_c3.json 2> gpurun_out/r05h_c3.err; echo "c3 rc=$?"
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r05h_c3.json').read().strip().splitlines()[-1])
print(d['value'], d['value_serial_steps'], d['e2e'])
PY
