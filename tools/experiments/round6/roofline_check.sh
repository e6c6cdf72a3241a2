# rocprofv3 kernel trace + stats of the bench command (c3, no backbone / CPU legs): the middle edge pass's
# back-to-back launches of the roofline phase (tools/trace_kernel_runs.py) against the line's roofline.avg_launch_us
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06f}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_rl -o run -- \
    python bench.py --no-backbone --no-cpu-baseline > gpurun_out/${T}_rl.json 2> gpurun_out/${T}_rl.err || exit 1
python tools/trace_kernel_runs.py gpurun_out/${T}_rl/run_kernel_trace.csv "edge_step_kernel<0, 0, 2, 1, 1>" 8 > gpurun_out/${T}_rl_runs.txt || exit 1
cat gpurun_out/${T}_rl_runs.txt
python tools/rocprof_summary.py gpurun_out/${T}_rl/run_kernel_stats.csv > gpurun_out/${T}_rl_stats.md || exit 1
tail -1 gpurun_out/${T}_rl.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('line', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
find gpurun_out -type f \( -name "*kernel_trace.csv" -o -name "*.db" \) -size +1M -delete
