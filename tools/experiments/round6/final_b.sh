# round-6 closing evidence, part B: SQ counters (wave-cycle breakdown, instruction mix, LDS, L2 hit) of every kernel in
# the c3 step -- edge passes, edge embedding, detection, node kernels, graph build and preparation
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06z}
bash tools/pmc_edge.sh ${T}_sqedge 'edge_step_kernel' > gpurun_out/${T}_sq_edge.txt 2>&1 || exit 1
bash tools/pmc_edge.sh ${T}_sqemb 'edge_embed_kernel' > gpurun_out/${T}_sq_embed.txt 2>&1 || exit 1
bash tools/pmc_edge.sh ${T}_sqnms 'nms_strips_kernel|plane_emit_kernel' > gpurun_out/${T}_sq_detect.txt 2>&1 || exit 1
bash tools/pmc_edge.sh ${T}_sqnode 'node_rows_kernel|node_table_kernel' > gpurun_out/${T}_sq_node.txt 2>&1 || exit 1
bash tools/pmc_edge.sh ${T}_sqgraph 'fused_fully_graph_kernel|fully_prepare_kernel|edge_ranges_kernel|cap_counts_kernel' > gpurun_out/${T}_sq_graph.txt 2>&1 || exit 1
echo "sq ok"
# keep the merge-back under its 64 MiB cap: the raw traces / counter dumps were summarised above
find gpurun_out -type f \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*.db" \) -size +1M -delete
