"""Merge tools/host_trace.py output ([py] and [ht] lines, CLOCK_MONOTONIC ns) into one host timeline."""
import sys

ev = []
for line in open(sys.argv[1]):
    p = line.split()
    if line.startswith("[py]"):
        ev.append((int(p[1]), " ".join(p[2:])))
    elif line.startswith("[ht]"):
        ev.append((int(p[1]), "launch @mpn/graph/detect line " + p[3]))
ev.sort()
t0 = ev[0][0]
prev = t0
for t, name in ev:
    print(f"{(t - t0) / 1e3:9.1f}  +{(t - prev) / 1e3:7.1f}  {name}")
    prev = t
