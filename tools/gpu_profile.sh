#!/bin/bash
# usage (GPU box): tools/gpu_profile.sh <tag> [workload] [extra bench args...]
# rocprofv3 kernel-trace stats of the bench command, then separate PMC passes (FETCH_SIZE, WRITE_SIZE) over
# the edge-pass, embedding and NMS kernels, merged into profiles/pmc_latest.json under (workload, edges).
# Outputs under gpurun_out/<tag>_*.
set -e
tag=$1
wl=${2:-c3}
shift; shift || true
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_stats -o run -- \
  python bench.py --workload $wl --no-cpu-baseline --steps 20 "$@" > gpurun_out/${tag}_stats.log 2>&1
rx='edge_step|nms_strips|edge_embed|node_|mpn_|fully_prepare|knn_'
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$rx" --output-format csv -d gpurun_out/${tag}_pmc_fetch -o pmc -- \
  python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-roofline "$@" > gpurun_out/${tag}_pmc_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$rx" --output-format csv -d gpurun_out/${tag}_pmc_write -o pmc -- \
  python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-roofline "$@" > gpurun_out/${tag}_pmc_write.log 2>&1
cp profiles/pmc_latest.json gpurun_out/${tag}_pmc_latest.json
python tools/pmc_json.py gpurun_out/${tag}_pmc_latest.json --bench-log gpurun_out/${tag}_pmc_fetch.log \
  gpurun_out/${tag}_pmc_*/pmc_counter_collection.csv > gpurun_out/${tag}_pmc.json
