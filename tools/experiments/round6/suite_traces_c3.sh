# round 6: GPU suite + smoke on the current tree, per-shape step trace of c3, and the default c3 bench line
# (usage: TAG=r06a bash tools/experiments/round6/suite_traces_c3.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06a}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gt.log 2>&1 || { tail -30 gpurun_out/${T}_gt.log; exit 1; }
echo "suite ok $(tail -1 gpurun_out/${T}_gt.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
echo "smoke ok"
for wl in ${WLS:-c3}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_${wl}_trace -o run -- \
      python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/${T}_${wl}_trace.log 2>&1 || exit 1
  python tools/trace_step_stats.py gpurun_out/${T}_${wl}_trace/run_kernel_trace.csv 25 > gpurun_out/${T}_${wl}_step_kernels.md || exit 1
done
echo "traces ok"
timeout -k 10 300 python bench.py > gpurun_out/${T}_c3.json 2> gpurun_out/${T}_c3.err || exit 1
echo "c3 ok"
