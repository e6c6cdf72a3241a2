# round 4, call h: rocprofv3 stats + PMC traffic of c3 on the committed tree; bench lines c5ms, c3knn10, c2, c2fp32
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 560 bash tools/gpu_profile.sh r04h c3 --streams 1 > gpurun_out/r04h_profile.log 2>&1
echo "profile rc=$?"
for wl in c5ms c3knn10 c2 c2fp32; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 20 > gpurun_out/r04h_$wl.log 2> gpurun_out/r04h_$wl.err
  echo "$wl rc=$?"
done
