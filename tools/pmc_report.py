"""Average rocprofv3 PMC counters per dispatch, per kernel, over one or more counter_collection CSVs.

usage: python tools/pmc_report.py gpurun_out/pmc_*/pmc_counter_collection.csv

FETCH_SIZE is reported raw and x2 (the gfx950 correction of MI355X_MICROARCH.md: FETCH_SIZE counts
64 B per 128-B request) -- both in KB per dispatch as rocprofv3 defines the counter.
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    m = re.match(r"([\w:]+(?:<[^()]*?>)?)\(", name)
    return (m.group(1) if m else name)[:70]


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(f"## {k}")
        for c, v in sorted(cs.items()):
            avg = sum(v) / len(v)
            extra = f"   (x2 corrected: {2 * avg:,.0f})" if c == "FETCH_SIZE" else ""
            print(f"  {c:28s} {avg:18,.0f}  n={len(v)}{extra}")
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            w = d["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    print(f"  {c + ' / WAVE_CYCLES':40s} {d[c] / w:.3f}")
        # (MFMA utilisation: tools/mfma_util.py, from SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE; the former
        # MFMA_BUSY / (BUSY_CYCLES x 4) ratio here was not a utilisation and read above 1)


if __name__ == "__main__":
    main(sys.argv[1:])
