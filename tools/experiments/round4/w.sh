# round 4, call w: batches in flight (streams 1..4) at c3, and the c2 line twice
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 2 3 4 1 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --workload c3 --steps 40 --streams $s > gpurun_out/r04w_s$s.log 2>&1 || exit 1
  python -c "import json; r=json.loads(open('gpurun_out/r04w_s$s.log').read().strip().splitlines()[-1]); print('streams $s', r['value'], r['ms_per_step'])"
done
