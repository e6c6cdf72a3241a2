"""MFMA utilisation per kernel from a rocprofv3 --pmc CSV holding SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE.

util = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles), kernel cycles = GRBM_GUI_ACTIVE / XCDs
(rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'; SQ_VALU_MFMA_BUSY_CYCLES
is summed over every SIMD and counts 16 cycles per v_mfma_f32_16x16x32_{f16,bf16}, calibrated with
tools/ubench/mfma_peak.hip, where the counter figure equals the event-timed TFLOP/s over the peak at the clock
the same counters give). 256 CUs x 4 SIMDs, 8 XCDs.
Two figures per kernel: mfma_busy over all 1,024 SIMDs, and mfma_busy_used over the SIMDs of the CUs the grid
occupies, 4 x min(256, workgroups) (the edge passes and the edge embedding run one workgroup per CU on 192 CUs
under the CU reservation, so their busy fraction on the SIMDs they actually use is 256/192 x the first figure).
usage: python tools/mfma_util.py pmc_counter_collection.csv [kernel-regex] [--json]
       python tools/mfma_util.py pmc_counter_collection.csv --merge profiles/mfma_latest.json --workload c3
       (adds / replaces the workload's run in the bench's source file)"""
import csv
import json
import re
import sys
from collections import defaultdict

SIMDS, XCDS = 1024, 8


CUS = SIMDS // 4


def per_dispatch(path, rx=None):
    d = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        if rx and not re.search(rx, r["Kernel_Name"]):
            continue
        k = (r["Dispatch_Id"])
        d[k][r["Counter_Name"]] = d[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
        try:   # workgroups of the dispatch -> CUs it can occupy
            d[k]["_wgs"] = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
        except (KeyError, ValueError):
            pass
    return d, names


def summarize(path, rx=None):
    d, names = per_dispatch(path, rx)
    by = defaultdict(list)
    for k, v in d.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and v.get("GRBM_GUI_ACTIVE"):
            cyc = v["GRBM_GUI_ACTIVE"] / XCDS
            cus = min(CUS, max(1, int(v.get("_wgs", CUS))))
            by[names[k]].append((v["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc), cyc, v.get("SQ_INSTS_MFMA", 0.0), cus))
    out = {}
    for n, vals in by.items():
        vals.sort()
        med = vals[len(vals) // 2]
        out[n] = {"mfma_busy": round(med[0], 4), "mfma_busy_used": round(med[0] * CUS / med[3], 4), "cus_used": med[3],
                  "dispatches": len(vals), "kernel_cycles_median": round(med[1]), "mfma_insts_median": med[2]}
    return out


def merge(path, workload, res, source):
    try:
        doc = json.load(open(path))
    except (OSError, ValueError):
        doc = {"formula": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), median over dispatches; "
                          "mfma_busy_used: the same over 4 x cus_used SIMDs, cus_used = min(256, workgroups)",
               "runs": []}
    doc["runs"] = [r for r in doc["runs"] if r.get("workload") != workload]
    doc["runs"].append({"workload": workload, "source": source, "kernels": res})
    json.dump(doc, open(path, "w"), indent=1)


if __name__ == "__main__":
    argv = sys.argv[1:]
    opts = {}
    for key in ("--merge", "--workload"):
        if key in argv:
            i = argv.index(key)
            opts[key] = argv[i + 1]
            del argv[i:i + 2]
    args = [a for a in argv if not a.startswith("--")]
    res = summarize(args[0], args[1] if len(args) > 1 else None)
    if "--merge" in opts:
        merge(opts["--merge"], opts["--workload"], res, args[0])
    if "--json" in sys.argv:
        print(json.dumps(res, indent=1))
    else:
        for n, v in sorted(res.items(), key=lambda kv: -kv[1]["mfma_busy"]):
            print(f"{v['mfma_busy']:7.4f} used {v['mfma_busy_used']:7.4f} ({v['cus_used']} CUs)  n={v['dispatches']:<4d} "
                  f"cycles={v['kernel_cycles_median']:<9d} {n[:100]}")
