# bench lines per workload (traffic from the committed profiles/pmc_latest.json)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/r03g_c3.json 2> gpurun_out/r03g_c3.err || exit 1
for wl in c3knn10 c2 c2fp32 c5; do
  timeout -k 10 300 python bench.py --workload $wl > gpurun_out/r03g_$wl.json 2> gpurun_out/r03g_$wl.err || exit 1
done
