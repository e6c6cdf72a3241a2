"""Per-kernel medians of a `bench.py --profile-steps` rocprofv3 kernel trace (every launch in it is a step kernel:
warmup + K serial steps on one stream), grouped by (kernel, grid size) so that shapes stay apart; `per step` = the
kernel's total over the trace / (warmup + K).
usage: python tools/trace_step_stats.py <run_kernel_trace.csv> <steps incl. warmup> [--md]"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:70]


def main(path, steps, md=False):
    rows = list(csv.DictReader(open(path)))
    g = defaultdict(list)
    for r in rows:
        if not r["Kernel_Name"].startswith(("void pemp", "pemp")):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]))].append(d)
    items = sorted(g.items(), key=lambda kv: -sum(kv[1]))
    tot = sum(sum(v) for v in g.values()) / steps
    if md:
        print("| kernel | grid | launches | median us | mean us | us per step |")
        print("|---|---|---|---|---|---|")
    for (k, grid), v in items:
        row = (k, grid, len(v), statistics.median(v), statistics.mean(v), sum(v) / steps)
        if md:
            print(f"| `{row[0]}` | {row[1]} | {row[2]} | {row[3]:.2f} | {row[4]:.2f} | {row[5]:.2f} |")
        else:
            print(f"{row[3]:8.2f} {row[4]:8.2f} {row[5]:8.2f}  n={row[2]:<5d} grid={row[1]:<8d} {row[0]}")
    print(f"\nsum of pemp kernel time per step: {tot:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), "--md" in sys.argv)
