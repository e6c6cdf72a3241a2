# round-4 final evidence (final tree): GPU suite, smoke, kernel stats + PMC traffic (c3, c3knn10; merged into the box copy of
# profiles/pmc_latest.json before the bench lines read it), SQ counters of the edge passes and the NMS, one bench
# line per workload, the two-rank rehearsal on one card
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04f_gt.log 2>&1 || exit 1
echo "suite ok $(tail -1 gpurun_out/r04f_gt.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1 || exit 1
echo "smoke ok"
bash tools/gpu_profile.sh r04f c3 || exit 1
cp gpurun_out/r04f_pmc_latest.json profiles/pmc_latest.json
bash tools/gpu_profile.sh r04fk c3knn10 || exit 1
cp gpurun_out/r04fk_pmc_latest.json profiles/pmc_latest.json
echo "profiles ok"
bash tools/pmc_edge.sh r04f_sqedge 'edge_step_kernel' > gpurun_out/r04f_sq_edge.txt 2>&1 || exit 1
bash tools/pmc_edge.sh r04f_sqnms 'nms_strips_kernel|plane_emit_kernel' > gpurun_out/r04f_sq_detect.txt 2>&1 || exit 1
echo "sq ok"
timeout -k 10 300 python bench.py > gpurun_out/r04f_c3.json 2> gpurun_out/r04f_c3.err || exit 1
echo "c3 ok"
for wl in c3knn10 c5ms c2 c2fp32 c5; do
  timeout -k 10 300 python bench.py --workload $wl > gpurun_out/r04f_$wl.json 2> gpurun_out/r04f_$wl.err || exit 1
  echo "$wl ok"
done
PEMP_SHARE_DEVICE=1 PEMP_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline > gpurun_out/r04f_dist2.json 2> gpurun_out/r04f_dist2.err || exit 1
echo "dist2 ok"
for wl in c3 c3knn10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f1_${wl} -o run -- \
    python bench.py --workload $wl --streams 1 --no-cpu-baseline --steps 20 > gpurun_out/r04f1_${wl}.json 2> gpurun_out/r04f1_${wl}.err || exit 1
  echo "1-stream $wl ok"
done
