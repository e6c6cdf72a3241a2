# round 6: the edge passes' workgroups placed XCD-local by target range (PEMP_XCD_MAP 2, xcd_map_fill) against round
# 5's contiguous run of types per XCD (xcd1): isolated MPN A/B, then PMC FETCH_SIZE of the edge passes for both
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06h}
for wl in c3 c3knn10 c5; do
  timeout -k 10 300 python tools/mpn_ab.py --workload $wl --iters 40 default xcd1 default xcd1 > gpurun_out/${T}_ab_$wl.txt 2>&1 || exit 1
  cat gpurun_out/${T}_ab_$wl.txt
done
for v in default xcd1; do
  if [ $v = default ]; then unset PEMP_LIB; else export PEMP_LIB=$PWD/build_ab/libpemp_$v.so; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'edge_step' --output-format csv -d gpurun_out/${T}_fetch_$v -o pmc -- \
    python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/${T}_fetch_$v.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'edge_step' --output-format csv -d gpurun_out/${T}_write_$v -o pmc -- \
    python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/${T}_write_$v.log 2>&1 || exit 1
  python - "$T" "$v" <<'PY'
import csv, sys, collections
T, v = sys.argv[1:]
for cn, f in (("FETCH_SIZE", f"gpurun_out/{T}_fetch_{v}/pmc_counter_collection.csv"), ("WRITE_SIZE", f"gpurun_out/{T}_write_{v}/pmc_counter_collection.csv")):
    d = collections.defaultdict(float); k = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != cn: continue
        d[r["Dispatch_Id"]] += float(r["Counter_Value"]); k[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0][-40:]
    by = collections.defaultdict(list)
    for i, x in d.items(): by[k[i]].append(x * (2 if cn == "FETCH_SIZE" else 1) / 1024)
    for name, xs in sorted(by.items()):
        xs.sort(); print(v, cn, name, "median MB", round(xs[len(xs)//2], 2), "n", len(xs), flush=True)
PY
done
unset PEMP_LIB
