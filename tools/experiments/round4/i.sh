# round 4, call i: bench lines c3 (e2e), c5ms, c3knn10, c2, c2fp32; SQ + LDS counters of the edge passes (c3)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c5ms c3knn10 c2 c2fp32; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 20 > gpurun_out/r04i_$wl.log 2> gpurun_out/r04i_$wl.err
  echo "$wl rc=$?"
done
timeout -k 10 500 bash tools/pmc_edge.sh r04i_edge "edge_step" > gpurun_out/r04i_pmc_edge.txt 2>&1
echo "pmc rc=$?"
