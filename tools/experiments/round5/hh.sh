# round 5, call hh: the c2 step timed three ways (tools/step_host_timing.py plain / stream / bench), HIP graphs on / off
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2; do
  for m in plain stream bench; do
    timeout -k 10 120 python tools/step_host_timing.py c2 400 $m > gpurun_out/r05hh_g_${m}_$k.txt 2>&1 &&
    PEMP_NO_GRAPHS=1 timeout -k 10 120 python tools/step_host_timing.py c2 400 $m > gpurun_out/r05hh_ng_${m}_$k.txt 2>&1 || exit 1
  done
done
grep -h "us_per_step" gpurun_out/r05hh_*.txt
