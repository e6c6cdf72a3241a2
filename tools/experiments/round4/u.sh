# round 4, call u: c2 A/B, fused node update + table (default) vs separate (nosum), alternating x3, 400 steps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in default nosum; do
    if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --workload c2 --steps 400 --streams 1 > gpurun_out/r04u_${v}_$i.log 2>&1 || { echo "$v failed"; exit 1; }
    python -c "import json; r=json.loads(open('gpurun_out/r04u_${v}_$i.log').read().strip().splitlines()[-1]); print('$v $i', r['value'], r['ms_per_step'])"
  done
done
