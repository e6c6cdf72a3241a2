# round-6 closing evidence, part A (final tree): GPU suite, smoke, kernel-trace stats + PMC traffic (c3, c3knn10;
# merged into the box copy of profiles/pmc_latest.json), MFMA busy (all SIMDs and the SIMDs the grid uses) for the
# edge passes, the edge embedding and the node kernels (profiles/mfma_latest.json)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06z}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gt.log 2>&1 || { tail -30 gpurun_out/${T}_gt.log; exit 1; }
echo "suite ok $(tail -1 gpurun_out/${T}_gt.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
echo "smoke ok"
bash tools/gpu_profile.sh ${T} c3 || exit 1
cp gpurun_out/${T}_pmc_latest.json profiles/pmc_latest.json
bash tools/gpu_profile.sh ${T}k c3knn10 || exit 1
cp gpurun_out/${T}k_pmc_latest.json profiles/pmc_latest.json
echo "pmc ok"
for wl in c3 c3knn10; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex 'edge_step|edge_embed|node_' \
    --output-format csv -d gpurun_out/${T}_mfma_$wl -o pmc -- python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-roofline \
    > gpurun_out/${T}_mfma_$wl.log 2>&1 || exit 1
  python tools/mfma_util.py gpurun_out/${T}_mfma_$wl/pmc_counter_collection.csv --merge profiles/mfma_latest.json --workload $wl > gpurun_out/${T}_mfma_$wl.txt || exit 1
done
cp profiles/mfma_latest.json gpurun_out/${T}_mfma_latest.json
echo "mfma ok"
# keep the merge-back under its 64 MiB cap: the raw traces / counter dumps were summarised above
find gpurun_out -type f \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*.db" \) -size +1M -delete
