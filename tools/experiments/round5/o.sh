# round 5, call o: batches in flight (--streams 1..4) at c3 and c3knn10
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c3knn10; do
  for s in 1 2 3 4; do
    timeout -k 10 200 python bench.py --workload $wl --streams $s --no-cpu-baseline --no-roofline --steps 40 > gpurun_out/r05o_${wl}_s$s.json 2> gpurun_out/r05o_${wl}_s$s.err || exit 1
    python - "$wl" "$s" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05o_{sys.argv[1]}_s{sys.argv[2]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'streams', sys.argv[2], d['value'], d['ms_per_step'])
PY
  done
done
