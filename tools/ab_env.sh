#!/bin/bash
# usage (GPU box): tools/ab_env.sh name:VAR=val,VAR2=val ... -> one short bench per environment
# ("name:" alone = defaults). Prints value + per-kernel us. Extra bench args via $AB_ARGS.
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
    timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 $AB_ARGS > gpurun_out/ab_$name.log 2>&1 ) \
    || { echo "$name failed"; tail -5 gpurun_out/ab_$name.log; exit 1; }
  python - "$name" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{v}.log").read().strip().splitlines()[-1])
k = d["kernel_avg_us"] or {}
print(v, d["value"], d.get("dtype"), " ".join(f"{a}={b}" for a, b in sorted(k.items())), flush=True)
PY
done
