# round 5, call tt: fully_prepare count loop with its type loads batched 8 per thread: MPN + graph GPU tests, A/B against
# the previous commit (build_ab/libpemp_base.so) at c3 / c2 (mpn_prepare kernel time from the library profiler)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_mpn.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05tt_tests.log 2>&1 || { tail -30 gpurun_out/r05tt_tests.log; exit 1; }
tail -1 gpurun_out/r05tt_tests.log
for w in c3 c2; do
  for v in default base; do
    if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
    timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-backbone --steps 40 > gpurun_out/r05tt_${w}_$v.json 2> gpurun_out/r05tt_${w}_$v.err || exit 1
    python -c "
import json; d = json.loads(open('gpurun_out/r05tt_${w}_$v.json').read().strip().splitlines()[-1])
print('$w', '$v', d['value'], d.get('value_serial_steps'), d['mpn_ms_per_step'], 'prepare us', d['kernel_avg_us'].get('mpn_prepare'))"
  done
done
