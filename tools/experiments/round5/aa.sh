# round 5, call aa: where two batches in flight still serialise: c3 and c3knn10 kernel traces with two streams
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c3knn10; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05aa_${wl} -o run -- \
      python bench.py --workload $wl --profile-steps --streams 2 --steps 20 --warmup 6 > gpurun_out/r05aa_${wl}.log 2>&1 || exit 1
  echo "== $wl $(grep profile_steps gpurun_out/r05aa_${wl}.log | tail -1)"
  python tools/two_stream_timeline.py gpurun_out/r05aa_${wl}/run_kernel_trace.csv || exit 1
done
