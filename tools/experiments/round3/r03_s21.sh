set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 bash tools/pmc_edge.sh r03s21 'nms_strips|edge_step_kernel<0, 1|edge_embed' > gpurun_out/r03s21_pmc_report.txt 2>&1
