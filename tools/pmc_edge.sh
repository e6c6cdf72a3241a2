#!/bin/bash
# usage (GPU box): tools/pmc_edge.sh <tag> <kernel-regex>  -- several PMC passes (one run each)
set -e
export TMPDIR=/tmp
tag=$1; rx=$2
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "$rx" --output-format csv -d gpurun_out/${tag}_p$i -o pmc -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/${tag}_p$i.log 2>&1
done
python tools/pmc_report.py gpurun_out/${tag}_p*/pmc_counter_collection.csv
