# Two batches in flight at c3 (bench.py --profile-steps --streams 2): kernel trace, overlap and idle time
# (tools/two_stream_timeline.py), with the batch-step entry.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06t}
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_c3s2 -o run -- \
    python bench.py --workload c3 --profile-steps --streams 2 --steps 30 --warmup 5 > gpurun_out/${T}_c3s2.log 2>&1 || exit 1
python tools/two_stream_timeline.py gpurun_out/${T}_c3s2/run_kernel_trace.csv > gpurun_out/${T}_c3s2_overlap.txt || exit 1
cat gpurun_out/${T}_c3s2_overlap.txt
find gpurun_out -type f \( -name "*kernel_trace.csv" -o -name "*.db" \) -size +1M -delete
