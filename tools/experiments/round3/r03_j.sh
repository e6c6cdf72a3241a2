set -e
export TMPDIR=/tmp
bash tools/pmc_edge.sh r03j 'edge_step|edge_embed' > gpurun_out/r03j_pmc_report.txt 2>&1
bash tools/pmc_sq.sh r03jsq 'edge_step|edge_embed'
python tools/pmc_report.py gpurun_out/r03jsq_sq/pmc_counter_collection.csv > gpurun_out/r03j_sq_report.txt
