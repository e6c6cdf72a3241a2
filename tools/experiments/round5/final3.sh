# round-5 closing evidence after the host-time changes and the 2-tile node table (no other kernel changed, so the
# PMC / SQ / MFMA passes of final.sh stand for the edge passes, NMS and embedding): GPU suite, smoke, the c3 / c3knn10 / c2
# step traces, one bench line per workload, the two-rank rehearsal on one card
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05f3}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gt.log 2>&1 || { tail -30 gpurun_out/${T}_gt.log; exit 1; }
echo "suite ok $(tail -1 gpurun_out/${T}_gt.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
echo "smoke ok"
for wl in c3 c3knn10 c2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_${wl}_trace -o run -- \
      python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/${T}_${wl}_trace.log 2>&1 || exit 1
  python tools/trace_step_stats.py gpurun_out/${T}_${wl}_trace/run_kernel_trace.csv 25 > gpurun_out/${T}_${wl}_step_kernels.md || exit 1
  python tools/step_timeline.py gpurun_out/${T}_${wl}_trace/run_kernel_trace.csv > gpurun_out/${T}_${wl}_step_timeline.txt || exit 1
done
echo "traces ok"
timeout -k 10 300 python bench.py > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
echo "c3 ok"
for wl in c3knn10 c5ms c2 c2fp32 c5; do
  timeout -k 10 300 python bench.py --workload $wl > gpurun_out/${T}_$wl.json 2> gpurun_out/${T}_$wl.err || exit 1
  echo "$wl ok"
done
PEMP_SHARE_DEVICE=1 PEMP_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline > gpurun_out/${T}_dist2.json 2> gpurun_out/${T}_dist2.err || exit 1
echo "dist2 ok"
