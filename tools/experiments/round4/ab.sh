# round 4, call ab: fully_prepare with ballot-ranked type lists (default) vs the per-node counting loop (oldprep):
# MPN suite (bit-identity of the fast prepare), then c2 / c3 one-stream A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mpn.py tests/test_gpu_graph.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04ab_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/r04ab_tests.log)"
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in default oldprep; do
    if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --workload c2 --steps 400 --streams 1 > gpurun_out/r04ab_${v}_$i.log 2>&1 || { echo "$v failed"; exit 1; }
    python -c "import json; r=json.loads(open('gpurun_out/r04ab_${v}_$i.log').read().strip().splitlines()[-1]); print('c2 $v $i', r['value'], r['ms_per_step'], r['kernel_avg_us']['mpn_prepare'])"
  done
done
unset PEMP_LIB
AB_ARGS="--workload c3 --steps 30 --streams 1" timeout -k 10 600 bash tools/ab.sh default oldprep
