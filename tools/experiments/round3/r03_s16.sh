set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s16_graph.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s16_stats -o run -- \
  python bench.py --no-cpu-baseline --steps 20 --streams 1 > gpurun_out/r03s16_stats.log 2>&1
