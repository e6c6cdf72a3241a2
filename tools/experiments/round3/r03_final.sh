# round-3 final evidence: GPU suite, smoke, kernel stats + PMC traffic (c3, c3knn10; merged into the box copy of
# profiles/pmc_latest.json before the bench lines read it), then one bench line per workload
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03z_gt.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03z_smoke.log 2>&1 || exit 1
bash tools/gpu_profile.sh r03z c3 || exit 1
cp gpurun_out/r03z_pmc_latest.json profiles/pmc_latest.json
bash tools/gpu_profile.sh r03zk c3knn10 || exit 1
cp gpurun_out/r03zk_pmc_latest.json profiles/pmc_latest.json
timeout -k 10 300 python bench.py > gpurun_out/r03z_c3.json 2> gpurun_out/r03z_c3.err || exit 1
for wl in c3knn10 c2 c2fp32 c5; do
  timeout -k 10 300 python bench.py --workload $wl > gpurun_out/r03z_$wl.json 2> gpurun_out/r03z_$wl.err || exit 1
done
