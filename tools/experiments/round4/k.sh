# round 4, call k: NMS access-pattern microbenchmark; fused select + emit and the symmetric scan (graph + MPN
# suites); MPN A/B on c3knn10
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/ubench/nms_pattern.hip -o /tmp/nmsp && \
timeout -k 10 60 /tmp/nmsp > gpurun_out/r04k_nms_pattern.txt 2>&1
echo "ubench rc=$?"
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_mpn.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/r04k_tests.log)"
timeout -k 10 200 python tools/mpn_ab.py --workload c3knn10 default > gpurun_out/r04k_ab_knn10.log 2>&1
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --no-cpu-baseline > gpurun_out/r04k_c3.log 2> gpurun_out/r04k_c3.err
echo "bench rc=$?"
