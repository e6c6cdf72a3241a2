# round-6 closing evidence, part C: per-shape step traces (c3, c3knn10, c2), one bench line per workload (the default
# c3 run with the CPU baseline and the backbone leg), the two-rank rehearsal on one card
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06z}
for wl in c3 c3knn10 c2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_${wl}_trace -o run -- \
      python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/${T}_${wl}_trace.log 2>&1 || exit 1
  python tools/trace_step_stats.py gpurun_out/${T}_${wl}_trace/run_kernel_trace.csv 25 > gpurun_out/${T}_${wl}_step_kernels.md || exit 1
  python tools/step_timeline.py gpurun_out/${T}_${wl}_trace/run_kernel_trace.csv > gpurun_out/${T}_${wl}_step_timeline.txt || exit 1
done
echo "traces ok"
timeout -k 10 400 python bench.py > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
echo "c3 ok"
for wl in c3knn10 c5ms c2 c2fp32 c5; do
  timeout -k 10 300 python bench.py --workload $wl --no-backbone > gpurun_out/${T}_$wl.json 2> gpurun_out/${T}_$wl.err || exit 1
  echo "$wl ok"
done
PEMP_SHARE_DEVICE=1 PEMP_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline --no-backbone > gpurun_out/${T}_dist2.json 2> gpurun_out/${T}_dist2.err || exit 1
echo "dist2 ok"
# keep the merge-back under its 64 MiB cap: the raw traces / counter dumps were summarised above
find gpurun_out -type f \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*.db" \) -size +1M -delete
