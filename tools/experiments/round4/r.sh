# round 4, call r: host time of the c2 step, capacity mode off / on (cProfile + wall per step)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_cprofile.py c2 > gpurun_out/r04r_host_nocap.txt 2>&1
echo "nocap rc=$?"
PEMP_CAP=1 timeout -k 10 200 python tools/host_cprofile.py c2 > gpurun_out/r04r_host_cap.txt 2>&1
echo "cap rc=$?"
timeout -k 10 200 python tools/host_cprofile.py c2 > gpurun_out/r04r_host_nocap2.txt 2>&1
echo "nocap2 rc=$?"
PEMP_CAP=1 timeout -k 10 200 python tools/host_cprofile.py c2 > gpurun_out/r04r_host_cap2.txt 2>&1
echo "cap2 rc=$?"
