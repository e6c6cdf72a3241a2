"""One step's kernel timeline from a rocprofv3 --kernel-trace CSV of `bench.py --profile-steps` (steps start at the
NMS kernel): start offset, duration and the idle gap before each kernel, for the median-span step, plus the median
step span and period. usage: python tools/step_timeline.py run_kernel_trace.csv [first_kernel_substring]"""
import csv
import re
import statistics
import sys


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "").replace("pemp::", "")
    return re.sub(r"\(.*$", "", name)[:60]


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "nms_"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    steps = [rows[a:b] for a, b in zip(starts, starts[1:])]
    if not steps:
        raise SystemExit("no steps found")
    spans = [max(k[1] for k in s) - s[0][0] for s in steps]
    periods = [steps[i + 1][0][0] - steps[i][0][0] for i in range(len(steps) - 1)]
    med = statistics.median(spans)
    s = min(steps, key=lambda st: abs((max(k[1] for k in st) - st[0][0]) - med))
    t0, prev_end = s[0][0], s[0][0]
    for a, b, n in s:
        gap = (a - prev_end) / 1e3
        print(f"{(a - t0) / 1e3:8.2f} {'(gap %.2f)' % gap if gap > 1 else '':>12} {(b - a) / 1e3:7.2f}  {n}")
        prev_end = max(prev_end, b)
    print(f"median step span {med / 1e3:.1f} us, median step period {statistics.median(periods) / 1e3:.1f} us, "
          f"kernel time in the step {sum(b - a for a, b, _ in s) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
