set -o pipefail
export TMPDIR=/tmp
PEMP_HOST_TRACE=1 timeout -k 10 120 python tools/host_trace.py c3 > gpurun_out/r03s24_ht.txt 2>&1
