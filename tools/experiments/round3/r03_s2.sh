set -o pipefail
export TMPDIR=/tmp
PEMP_LIB=build_ab/libpemp_stamps.so timeout -k 10 200 python tools/edge_timeline.py 0 1 2 > gpurun_out/r03s2_timeline.txt 2>&1 && \
timeout -k 10 400 bash tools/pmc_edge.sh r03s2 'edge_step|edge_embed' > gpurun_out/r03s2_pmc_report.txt 2>&1
