# round 4, call d: bisect the bf16x3 golden failure over library variants; then the bench with the e2e leg
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default base noscan noprio slowmath; do
  if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
  timeout -k 10 120 python -u -m pytest tests/test_gpu_mpn.py -q -k "bf16x3" --timeout 100 --timeout-method thread > gpurun_out/r04d_bf16_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/r04d_bf16_$v.log)"
done
unset PEMP_LIB
timeout -k 10 400 python -u bench.py --workload c3 --steps 20 > gpurun_out/r04d_c3.log 2> gpurun_out/r04d_c3.err
echo bench_rc=$?
