"""PMC HBM traffic per dispatch (rocprofv3 FETCH_SIZE / WRITE_SIZE passes) -> JSON for bench.py.

usage: python tools/pmc_json.py <out.json> --bench-log <log of one pass> gpurun_out/<tag>_pmc_*/pmc_counter_collection.csv
FETCH_SIZE is doubled (gfx950: it counts 64 B per 128-B request, MI355X_MICROARCH.md HBM section);
both counters are KB per dispatch. Keys are kernel names without template arguments' spaces.
Entries are keyed by (workload, edges): the bench line the passes ran (its JSON line in --bench-log)
names both, and bench.py reports `traffic` only for a run of the same workload and edge count.
An existing out.json keeps its other entries; one with the same key is replaced.
"""
import collections
import csv
import json
import os
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    m = re.match(r"([\w:]+(?:<[^()]*?>)?)\(", name)
    return (m.group(1) if m else name).replace(" ", "")


def bench_key(log):
    for line in open(log):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            rec = json.loads(line)
            cfg = rec["config"]
            return cfg["workload"].split(":")[0], int(cfg["edges_per_gpu"]), int(cfg["nodes_per_gpu"])
    raise SystemExit(f"no bench JSON line in {log}")


def main(argv):
    out = argv[0]
    i = argv.index("--bench-log")
    log = argv[i + 1]
    paths = argv[1:i] + argv[i + 2:]
    workload, edges, nodes = bench_key(log)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        f = cs.get("FETCH_SIZE")
        w = cs.get("WRITE_SIZE")
        if not f or not w:
            continue
        fb = 2 * 1024 * sum(f) / len(f)
        wb = 1024 * sum(w) / len(w)
        res[k] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "bytes": round(fb + wb),
                  "dispatches": len(f), "correction": "FETCH_SIZE x2 (gfx950), KB -> B"}
    runs = []
    if os.path.exists(out):
        try:
            runs = json.load(open(out)).get("runs", [])
        except ValueError:
            runs = []
    runs = [r for r in runs if (r["workload"], r["edges"]) != (workload, edges)]
    runs.append({"workload": workload, "edges": edges, "nodes": nodes, "source": paths, "kernels": res})
    json.dump({"runs": runs}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
