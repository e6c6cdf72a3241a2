set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_gt.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
