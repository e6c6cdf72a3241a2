# round 5, call z: batches in flight 2 vs 3 with the CU reservation (c3, c3knn10, c5), alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c3knn10 c5; do
  for s in 2 3 2 3; do
    timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-roofline --steps 40 --streams $s > gpurun_out/r05z2_${wl}_$s.json 2> gpurun_out/r05z2_${wl}_$s.err || exit 1
    python - "$wl" "$s" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05z2_{sys.argv[1]}_{sys.argv[2]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'streams', sys.argv[2], d['value'], d['ms_per_step'])
PY
  done
done
