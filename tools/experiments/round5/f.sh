# round 5, call f: per-shape kernel traces of the serial step (c3, c3knn10, c2), SQ counters of the edge embedding
# and passes, bench lines c3 / c3knn10
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c3 c3knn10 c2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05f_${wl}_trace -o run -- \
    python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/r05f_${wl}_trace.log 2>&1 || exit 1
  echo "$wl $(tail -1 gpurun_out/r05f_${wl}_trace.log)"
  python tools/trace_step_stats.py gpurun_out/r05f_${wl}_trace/run_kernel_trace.csv 25 | head -30
done
rx='edge_step|edge_embed|nms_strips|node_'
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-include-regex "$rx" --output-format csv -d gpurun_out/r05f_sq1 -o pmc -- python bench.py --workload c3 --profile-steps --steps 3 --warmup 1 > gpurun_out/r05f_sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "$rx" --output-format csv -d gpurun_out/r05f_sq2 -o pmc -- python bench.py --workload c3 --profile-steps --steps 3 --warmup 1 > gpurun_out/r05f_sq2.log 2>&1 || exit 1
echo sq ok
timeout -k 10 300 python bench.py > gpurun_out/r05f_c3.json 2> gpurun_out/r05f_c3.err; echo "c3 rc=$?"
timeout -k 10 300 python bench.py --workload c3knn10 > gpurun_out/r05f_c3knn10.json 2> gpurun_out/r05f_c3knn10.err; echo "c3knn10 rc=$?"
