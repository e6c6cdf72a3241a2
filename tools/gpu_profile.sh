#!/bin/bash
# usage (GPU box): tools/gpu_profile.sh <tag>
# rocprofv3 kernel-trace stats of the default bench command, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) over the edge-pass and NMS kernels. Outputs under gpurun_out/<tag>_*.
set -e
tag=$1
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_stats -o run -- \
  python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${tag}_stats.log 2>&1
rx='edge_step|nms_strips|edge_embed|node_step|mpn_'
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$rx" --output-format csv -d gpurun_out/${tag}_pmc_fetch -o pmc -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/${tag}_pmc_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$rx" --output-format csv -d gpurun_out/${tag}_pmc_write -o pmc -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/${tag}_pmc_write.log 2>&1
python tools/pmc_json.py gpurun_out/${tag}_pmc.json gpurun_out/${tag}_pmc_*/pmc_counter_collection.csv > /dev/null
# refine (pose finishing): kernel stats and HBM passes of its own
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_refine_stats -o run -- \
  python tools/refine_prof.py 9 > gpurun_out/${tag}_refine_stats.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex refine_argmax --output-format csv -d gpurun_out/${tag}_refine_pmc_fetch -o pmc -- \
  python tools/refine_prof.py 9 > gpurun_out/${tag}_refine_pmc_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex refine_argmax --output-format csv -d gpurun_out/${tag}_refine_pmc_write -o pmc -- \
  python tools/refine_prof.py 9 > gpurun_out/${tag}_refine_pmc_write.log 2>&1
