#!/bin/bash
# usage (GPU box): tools/pmc_sq.sh <tag> [regex]  -> SQ stall-breakdown counters of the matching kernels
# (one pass of 8 SQ counters over a short bench; the library picked by $PEMP_LIB if set)
set -e
tag=$1; rx=${2:-edge_step|nms_strips|edge_embed}
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA \
  --kernel-include-regex "$rx" --output-format csv -d gpurun_out/${tag}_sq -o pmc -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/${tag}_sq.log 2>&1
