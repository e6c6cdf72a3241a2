#!/bin/bash
# usage: tools/pmc_pass.sh <outdir> <kernel-regex> <counter...>   (GPU box; separate run per counter set)
# honours PEMP_LIB (A/B library variants under build_ab/)
set -e
out=$1; shift; rx=$1; shift
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$rx" --output-format csv -d "$out" -o pmc -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > "$out.log" 2>&1
