# Batch-1 lines (c2, c2fp32) with 200 timed steps (a 20-step region at batch 1 lasts 3-4 ms and one host hiccup moves it)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c2 c2fp32; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-backbone --steps 200 --warmup 20 > gpurun_out/r06b_$wl.json 2> gpurun_out/r06b_$wl.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/r06b_$wl.json').read().strip().splitlines()[-1]); print('$wl', d['value'], d['ms_per_step'], d['value_serial_steps'], d['schedule_probe'])"
done
