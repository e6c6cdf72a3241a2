#!/bin/bash
# usage (GPU box): tools/trace_step.sh <tag>  -> gpurun_out/<tag>_trace/ + report on stdout
set -e
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$1_trace -o run -- \
  python bench.py --no-cpu-baseline --no-roofline --steps 20 > gpurun_out/$1_trace.log 2>&1
python tools/trace_report.py gpurun_out/$1_trace/run_kernel_trace.csv 12 > gpurun_out/$1_trace_report.md
cat gpurun_out/$1_trace_report.md
