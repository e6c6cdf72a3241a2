"""Overlap of two batches in flight from a rocprofv3 --kernel-trace CSV of `bench.py --profile-steps --streams 2`:
per (stream, kernel) the time it ran with nothing else on the GPU, and how much of the window the GPU had exactly one
/ two kernels running. usage: python tools/two_stream_timeline.py run_kernel_trace.csv [skip_first_us]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "").replace("pemp::", "")
    return re.sub(r"\(.*$", "", name)[:48]


rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        if "pemp" not in r["Kernel_Name"]:
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
rows.sort()
t0 = rows[0][0] + int(float(sys.argv[2]) * 1e3) if len(sys.argv) > 2 else rows[len(rows) // 4][0]
rows = [r for r in rows if r[0] >= t0]
events = sorted([(a, 1, i) for i, (a, b, n) in enumerate(rows)] + [(b, -1, i) for i, (a, b, n) in enumerate(rows)])
active, last, busy = set(), events[0][0], defaultdict(float)
alone = defaultdict(float)
for t, d, i in events:
    dt = t - last
    busy[min(len(active), 3)] += dt
    if len(active) == 1:
        alone[rows[next(iter(active))][2]] += dt
    last = t
    if d > 0:
        active.add(i)
    else:
        active.discard(i)
span = events[-1][0] - events[0][0]
print(f"window {span / 1e3:.1f} us: idle {busy[0] / span:.1%}, one kernel {busy[1] / span:.1%}, "
      f"two {busy[2] / span:.1%}, three+ {busy[3] / span:.1%}")
tot = defaultdict(float)
for a, b, n in rows:
    tot[n] += b - a
print("kernel | total us | alone us")
for n in sorted(tot, key=lambda k: -alone[k])[:16]:
    print(f"{n} | {tot[n] / 1e3:.1f} | {alone[n] / 1e3:.1f}")
