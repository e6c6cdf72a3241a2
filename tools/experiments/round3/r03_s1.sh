set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03s1_gt.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s1_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r03s1_bench.json 2> gpurun_out/r03s1_bench.err && \
timeout -k 10 300 python bench.py --workload c3knn10 > gpurun_out/r03s1_knn10.json 2> gpurun_out/r03s1_knn10.err && \
bash tools/gpu_profile.sh r03s1 c3
