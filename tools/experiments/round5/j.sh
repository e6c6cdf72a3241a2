# round 5, call j: node_sum_table_kernel / node_table_kernel with XCD-local column groups (PEMP_NODE_XCD),
# A/B over PEMP_NST_BPW (-1 = node_rows + node_table)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mpn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r05j_mpn_tests.log 2>&1
rc=$?; echo "mpn tests rc=$rc $(tail -1 gpurun_out/r05j_mpn_tests.log)"; [ $rc -eq 0 ] || exit 1
for wl in c3knn10 c3; do
  for cfg in "-1 0" "-1 1" "5 1" "3 1" "2 1"; do
    set -- $cfg; b=$1; x=$2
    PEMP_NST_BPW=$b PEMP_NODE_XCD=$x timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05j_${wl}_b${b}_x$x -o run -- \
        python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/r05j_${wl}_b${b}_x$x.log 2>&1 || exit 1
    echo "== $wl bpw=$b xcd=$x"
    python tools/trace_step_stats.py gpurun_out/r05j_${wl}_b${b}_x$x/run_kernel_trace.csv 25 > gpurun_out/r05j_${wl}_b${b}_x$x.md || exit 1
    grep -E "node_|sum of" gpurun_out/r05j_${wl}_b${b}_x$x.md
  done
done
