#!/bin/bash
# usage (GPU box): tools/ab.sh default old nopf ...  -> one short bench per library variant
# (build_ab/libpemp_<v>.so; "default" = the in-tree library). Prints value + per-kernel us.
for v in "$@"; do
  if [ "$v" = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 $AB_ARGS > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{v}.log").read().strip().splitlines()[-1])
k = d["kernel_avg_us"] or {}
print(v, d["value"], " ".join(f"{a}={b}" for a, b in sorted(k.items())))
PY
done
