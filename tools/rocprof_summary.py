"""Condense a rocprofv3 ``*_kernel_stats.csv`` into a short table (kernel, calls, avg/min/max us, share).

usage: python tools/rocprof_summary.py gpurun_out/prof_r01/run_kernel_stats.csv > profiles/r01_kernel_stats.md
"""
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    m = re.match(r"([\w:]+(?:<[^()]*?>)?)\(", name)
    return (m.group(1) if m else name)[:80]


def main(path):
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"source: `{path}`\n")
    print("| kernel | calls | avg us | min us | max us | total ms | share |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
              f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
              f"{float(r['TotalDurationNs']) / 1e6:.3f} | {100 * float(r['TotalDurationNs']) / total:.1f}% |")


if __name__ == "__main__":
    main(sys.argv[1])
