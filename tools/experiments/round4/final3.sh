# round-4 closing check after the knn bit-row prepare: GPU suite, smoke, c3 and c3knn10 bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04g_gt.log 2>&1 || { tail -30 gpurun_out/r04g_gt.log; exit 1; }
echo "suite ok $(tail -1 gpurun_out/r04g_gt.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04g_smoke.log 2>&1 || exit 1
echo "smoke ok"
for wl in c3 c3knn10; do
  timeout -k 10 300 python bench.py --workload $wl > gpurun_out/r04g_$wl.json 2> gpurun_out/r04g_$wl.err || exit 1
  echo "$wl ok"
done
