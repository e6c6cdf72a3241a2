# closing check of the final tree: GPU suite, smoke, the default bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06g}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gt.log 2>&1 || { tail -30 gpurun_out/${T}_gt.log; exit 1; }
echo "suite: $(tail -1 gpurun_out/${T}_gt.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
echo "smoke: $(tail -1 gpurun_out/${T}_smoke.log)"
timeout -k 10 400 python bench.py > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
tail -1 gpurun_out/${T}_c3.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'], d['e2e_images_per_sec'], d['roofline']['frac'], d['cpu_baseline']['value'])"
