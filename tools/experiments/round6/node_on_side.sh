# round 6: the first node step (node embedding + node table) on the prelude side stream and the edge prelude (order,
# ranges, embedding) on the launch stream (PEMP_NODE_ON_SIDE, default) vs round 5's split (nodeside0): MPN GPU tests,
# a c3 / c2 serial step trace each, alternating bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06i}
timeout -k 10 500 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "tests $(tail -1 gpurun_out/${T}_tests.log)"
for v in default nodeside0; do
  if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
  for wl in c3 c2; do
    timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_${wl}_${v}_trace -o run -- \
        python bench.py --workload $wl --profile-steps --steps 20 --warmup 5 > gpurun_out/${T}_${wl}_${v}_trace.log 2>&1 || exit 1
    python tools/step_timeline.py gpurun_out/${T}_${wl}_${v}_trace/run_kernel_trace.csv > gpurun_out/${T}_${wl}_${v}_step_timeline.txt || exit 1
    echo "$v $wl $(tail -1 gpurun_out/${T}_${wl}_${v}_step_timeline.txt)"
  done
done
for wl in c3 c3knn10 c2; do
  for v in default nodeside0 default nodeside0; do
    if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
    timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-backbone > gpurun_out/${T}_${wl}_$v.json 2> gpurun_out/${T}_${wl}_$v.err || exit 1
    python - "$T" "$wl" "$v" <<'PY'
import json, sys
T, wl, v = sys.argv[1:]
d = json.loads(open(f"gpurun_out/{T}_{wl}_{v}.json").read().strip().splitlines()[-1])
print(wl, v, "value", d["value"], "ms", d["ms_per_step"], "serial", d["value_serial_steps"], "S", d["config"]["batches_in_flight"],
      "mpn_ms", d["mpn_ms_per_step"], "e2e", (d.get("e2e") or {}).get("images_per_sec"), flush=True)
PY
  done
done
unset PEMP_LIB
