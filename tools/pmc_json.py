"""PMC HBM traffic per dispatch (rocprofv3 FETCH_SIZE / WRITE_SIZE passes) -> JSON for bench.py.

usage: python tools/pmc_json.py <out.json> gpurun_out/<tag>_pmc_*/pmc_counter_collection.csv
FETCH_SIZE is doubled (gfx950: it counts 64 B per 128-B request, MI355X_MICROARCH.md HBM section);
both counters are KB per dispatch. Keys are kernel names without template arguments' spaces.
"""
import collections
import csv
import json
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    m = re.match(r"([\w:]+(?:<[^()]*?>)?)\(", name)
    return (m.group(1) if m else name).replace(" ", "")


def main(out, paths):
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
    json.dump({"source": paths, "kernels": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
