set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 bash tools/pmc_edge.sh r03s7 'edge_step' > gpurun_out/r03s7_pmc_report.txt 2>&1
