set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06q2_graph.log 2>&1 || { tail -40 gpurun_out/r06q2_graph.log; exit 1; }
echo "graph tests: $(tail -1 gpurun_out/r06q2_graph.log)"
for round in 1 2; do
  PEMP_NMS_QUAD=0 timeout -k 10 120 python tools/nms_bench.py c3 || exit 1
  PEMP_NMS_QUAD=1 timeout -k 10 120 python tools/nms_bench.py c3 || exit 1
done
