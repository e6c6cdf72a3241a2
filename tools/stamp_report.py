"""Per-workgroup / per-SIMD balance of one stamped edge pass (tools/edge_timeline.py with STAMP_OUT=prefix).
usage: python tools/stamp_report.py gpurun_out/<prefix>_pass0.npy [NW]"""
import sys

import numpy as np

s = np.load(sys.argv[1]).astype(np.int64)
NW = int(sys.argv[2]) if len(sys.argv) > 2 else 16
t0 = s[:, 0][s[:, 0] > 0].min()
us = np.where(s > 0, (s - t0) / 100.0, np.nan)
G = s.shape[0] // NW
ex = us[:, 15].reshape(G, NW)
nt = np.sum(np.isfinite(us[:, 3:15:3]), 1).reshape(G, NW)
pct = lambda v: " ".join(f"{x:6.2f}" for x in np.nanpercentile(v, [0, 10, 50, 90, 100]))
print("WG exit (max over waves)  ", pct(np.nanmax(ex, 1)))
print("WG tiles (<=4 per wave counted) hist", np.bincount(nt.sum(1)))
simd = np.array([[nt[g, np.arange(NW) % 4 == k].sum() for k in range(4)] for g in range(G)])
print("SIMD tiles hist", np.bincount(simd.ravel()))
last = np.nanmax(np.where(np.isfinite(us[:, 5:15:3]), us[:, 5:15:3], np.nan), 1).reshape(G, NW)   # last stamped tile done
print("wave last-tile-done        ", pct(last.ravel()))
print("mean last-tile-done by wave", np.round(np.nanmean(last, 0), 1))
for i in range(4):
    st, dn = us[:, 3 + 3 * i], us[:, 5 + 3 * i]
    if np.isfinite(st).any():
        print(f"tile{i}: start {pct(st)} | dur {pct(dn - st)}")
