# round 6: the middle steps' node update fused into a WIDE node-table launch (16 waves = 256 table columns per
# workgroup: the tile's aggregates summed once per 256 columns instead of per 64). MPN GPU tests, then the isolated
# MPN A/B against the same tree without it (nowide: separate node_rows SUM + node_table launches at c3 / c3knn10) and
# with 8-wave workgroups (wide8); then c3 / c3knn10 bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06e}
timeout -k 10 500 python -u -m pytest tests/test_gpu_mpn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "tests $(tail -1 gpurun_out/${T}_tests.log)"
for wl in c3knn10 c3 c5; do
  timeout -k 10 300 python tools/mpn_ab.py --workload $wl --iters 40 default nowide wide8 default nowide wide8 > gpurun_out/${T}_ab_$wl.txt 2>&1 || exit 1
  cat gpurun_out/${T}_ab_$wl.txt
done
for wl in c3knn10 c3; do
  for v in default nowide default nowide; do
    if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
    timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-backbone > gpurun_out/${T}_${wl}_$v.json 2> gpurun_out/${T}_${wl}_$v.err || exit 1
    python - "$T" "$wl" "$v" <<'PY'
import json, sys
T, wl, v = sys.argv[1:]
d = json.loads(open(f"gpurun_out/{T}_{wl}_{v}.json").read().strip().splitlines()[-1])
e = d.get("e2e") or {}
print(wl, v, "value", d["value"], "ms", d["ms_per_step"], "serial", d["value_serial_steps"], "mpn_ms", d["mpn_ms_per_step"],
      "e2e", e.get("images_per_sec"), e.get("stage_host_ms_per_batch"), flush=True)
PY
  done
done
unset PEMP_LIB
