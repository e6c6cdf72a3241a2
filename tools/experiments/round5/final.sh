# round-5 final evidence (final tree): GPU suite, smoke, kernel stats + PMC traffic (c3, c3knn10; merged into the box
# copy of profiles/pmc_latest.json before the bench lines read it), MFMA-busy SQ pass (profiles/mfma_latest.json), SQ
# counters of the passes, NMS and embedding, per-shape step traces (c3, c3knn10, c2), one bench line per workload, the
# two-rank rehearsal on one card
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05z}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gt.log 2>&1 || { tail -30 gpurun_out/${T}_gt.log; exit 1; }
echo "suite ok $(tail -1 gpurun_out/${T}_gt.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
echo "smoke ok"
bash tools/gpu_profile.sh ${T} c3 || exit 1
cp gpurun_out/${T}_pmc_latest.json profiles/pmc_latest.json
bash tools/gpu_profile.sh ${T}k c3knn10 || exit 1
cp gpurun_out/${T}k_pmc_latest.json profiles/pmc_latest.json
echo "pmc ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex 'edge_step|edge_embed|node_' \
  --output-format csv -d gpurun_out/${T}_mfma_c3 -o pmc -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline \
  > gpurun_out/${T}_mfma_c3.log 2>&1 || exit 1
python tools/mfma_util.py gpurun_out/${T}_mfma_c3/pmc_counter_collection.csv --merge profiles/mfma_latest.json --workload c3 > gpurun_out/${T}_mfma_c3.txt || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex 'edge_step|edge_embed|node_' \
  --output-format csv -d gpurun_out/${T}_mfma_c3knn10 -o pmc -- python bench.py --workload c3knn10 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline \
  > gpurun_out/${T}_mfma_c3knn10.log 2>&1 || exit 1
python tools/mfma_util.py gpurun_out/${T}_mfma_c3knn10/pmc_counter_collection.csv --merge profiles/mfma_latest.json --workload c3knn10 > gpurun_out/${T}_mfma_c3knn10.txt || exit 1
cp profiles/mfma_latest.json gpurun_out/${T}_mfma_latest.json
echo "mfma ok"
bash tools/pmc_edge.sh ${T}_sqedge 'edge_step_kernel' > gpurun_out/${T}_sq_edge.txt 2>&1 || exit 1
bash tools/pmc_edge.sh ${T}_sqnms 'nms_strips_kernel|plane_emit_kernel' > gpurun_out/${T}_sq_detect.txt 2>&1 || exit 1
bash tools/pmc_edge.sh ${T}_sqemb 'edge_embed_kernel' > gpurun_out/${T}_sq_embed.txt 2>&1 || exit 1
echo "sq ok"
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
