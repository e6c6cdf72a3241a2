"""Per-kernel averages and the timeline of one pipeline step from a rocprofv3 kernel trace.

usage: python tools/trace_report.py gpurun_out/<dir>/run_kernel_trace.csv [step_index]
A step starts at an nms_strips_kernel launch; gaps are GPU idle time between kernels.
"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    m = re.match(r"([\w:]+(?:<[^()]*?>)?)\(", n)
    return (m.group(1) if m else n)[:60]


def main(path, step=10):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    agg = collections.defaultdict(list)
    for r in rows:
        agg[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("| kernel | calls | avg us | min us |")
    print("|---|---:|---:|---:|")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"| `{k}` | {len(v)} | {sum(v) / len(v):.2f} | {min(v):.2f} |")
    idx = [i for i, r in enumerate(rows) if "nms_strips" in r["Kernel_Name"]]
    if len(idx) > step + 1:
        i0, i1 = idx[step], idx[step + 1]
        t0 = prev = int(rows[i0]["Start_Timestamp"])
        print(f"\nstep {step} timeline (us): start, gap before, duration, kernel")
        busy = 0.0
        for r in rows[i0:i1]:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{(st - t0) / 1e3:8.1f} {(st - prev) / 1e3:7.1f} {(en - st) / 1e3:7.1f}  {short(r['Kernel_Name'])}")
            busy += (en - st) / 1e3
            prev = en
        total = (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3
        print(f"step {total:.1f} us, kernels busy {busy:.1f} us, idle {total - busy:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
