# round 5, call cc: the c3knn10 MFMA-busy pass (merged into profiles/mfma_latest.json beside c3's) and its line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=r05cc
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-include-regex 'edge_step|edge_embed|node_' \
  --output-format csv -d gpurun_out/${T}_mfma_c3knn10 -o pmc -- python bench.py --workload c3knn10 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline \
  > gpurun_out/${T}_mfma_c3knn10.log 2>&1 || exit 1
python tools/mfma_util.py gpurun_out/${T}_mfma_c3knn10/pmc_counter_collection.csv --merge profiles/mfma_latest.json --workload c3knn10 > gpurun_out/${T}_mfma_c3knn10.txt || exit 1
cp profiles/mfma_latest.json gpurun_out/${T}_mfma_latest.json
cat gpurun_out/${T}_mfma_c3knn10.txt | head -20
timeout -k 10 400 python bench.py --workload c3knn10 > gpurun_out/${T}_c3knn10.json 2> gpurun_out/${T}_c3knn10.err || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/${T}_c3knn10.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline'].get('mfma_busy'), d['roofline']['frac'], (d.get('backbone') or {}).get('ms_per_batch'))
"
