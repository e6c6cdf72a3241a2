# round 5, call ee: host-side breakdown of the timed step at c2 and c3 (tools/step_host_timing.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python tools/step_host_timing.py c2 300 > gpurun_out/r05ee_c2.txt 2>&1 &&
timeout -k 10 240 python tools/step_host_timing.py c3 100 > gpurun_out/r05ee_c3.txt 2>&1
