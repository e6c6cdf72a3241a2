# knn bit-row prepare (pemp_mpn_forward_knn): parity tests, then c3knn10 with and without it (bench lines and the
# one-stream kernel trace)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mpn.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "knn_rows or symmetric or knn" > gpurun_out/kp_t.log 2>&1 || { tail -40 gpurun_out/kp_t.log; exit 1; }
echo "tests ok $(tail -1 gpurun_out/kp_t.log)"
timeout -k 10 300 python bench.py --workload c3knn10 --no-cpu-baseline > gpurun_out/kp_on.json 2> gpurun_out/kp_on.err || exit 1
PEMP_NO_KNN_PREPARE=1 timeout -k 10 300 python bench.py --workload c3knn10 --no-cpu-baseline > gpurun_out/kp_off.json 2> gpurun_out/kp_off.err || exit 1
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp1 -o run -- \
  python bench.py --workload c3knn10 --streams 1 --no-cpu-baseline --steps 20 > gpurun_out/kp1.json 2> gpurun_out/kp1.err || exit 1
echo "trace ok"
