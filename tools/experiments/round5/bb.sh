# round 5, call bb: the backbone leg's dtype / layout / MIOpen find mode
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "bf16 nchw NORMAL" "f16 nchw NORMAL" "bf16 nhwc NORMAL" "f16 nhwc NORMAL" "bf16 nchw FAST"; do
  set -- $cfg
  PEMP_BB_DTYPE=$1 PEMP_BB_LAYOUT=$2 MIOPEN_FIND_MODE=$3 timeout -k 10 600 python bench.py --backbone --no-cpu-baseline --no-roofline --steps 10 > gpurun_out/r05bb_$1_$2_$3.json 2> gpurun_out/r05bb_$1_$2_$3.err || exit 1
  python - "$1" "$2" "$3" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/r05bb_{sys.argv[1]}_{sys.argv[2]}_{sys.argv[3]}.json').read().strip().splitlines()[-1])
print(sys.argv[1:], json.dumps(d['backbone']))
PY
done
