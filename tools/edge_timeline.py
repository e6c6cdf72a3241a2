"""Diagnostic: per-wave phase timeline of one edge pass (needs the -DPEMP_STAMPS library,
build_ab/libpemp_stamps.so, selected with PEMP_LIB). Usage: python tools/edge_timeline.py [pass]
Stamps (s_memrealtime, 100 MHz): 0 entry, 1 weights staged, 2 wave range known, per tile i < 4:
3+3i tile start, 4+3i first rows arrived, 5+3i tile done; 15 exit."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import pemp_amd  # noqa: E402
from pemp_amd import _lib, config as pcfg  # noqa: E402

wl = dict(bench.WORKLOADS[os.environ.get("WL", "c3")])
dev = torch.device("cuda:0")
gc = pcfg.inference_gc_config(wl["graph"], 5, False)
hm, feats, tags = bench.make_inputs(wl, 0, dev)
model, _ = bench.make_model(wl, dev)
if os.environ.get("PREC"):
    model.precision = os.environ["PREC"]
L = _lib.lib()
for _ in range(3):
    out, pe, pn, pc = bench.run_step(wl, gc, model, hm, feats, tags, dev)
torch.cuda.synchronize()
x, ea, ei, types = out[0], out[1], out[2], out[7][:, 2]
fn = L.pemp_diag_stamps
fn.restype, fn.argtypes = ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int32]
nw = 256 * 16
for pas in [int(a) for a in (sys.argv[1:] or ["0", "2"])]:
    buf = torch.zeros(nw * 16, dtype=torch.int64, device=dev)
    fn(buf.data_ptr(), pas)
    with torch.no_grad():
        model(x, ea, ei, node_types=types)
    torch.cuda.synchronize()
    fn(None, -1)
    s = buf.view(nw, 16).cpu().numpy().astype(np.int64)
    if os.environ.get("STAMP_OUT"):
        np.save(f"{os.environ['STAMP_OUT']}_pass{pas}.npy", s)
    live = s[:, 0] > 0
    s = s[live]
    t0 = s[:, 0].min()
    us = np.where(s > 0, (s - t0) / 100.0, np.nan)
    print(f"== pass {pas}: {live.sum()} waves stamped, kernel span {np.nanmax(us):.2f} us")
    pct = lambda v: " ".join(f"{np.nanpercentile(v, q):7.2f}" for q in (0, 10, 50, 90, 100)) if np.isfinite(v).any() else "-"
    print("            min    p10    p50    p90    max (us)")
    names = {0: "entry", 1: "staged", 2: "range", 15: "exit"}
    for k in (0, 1, 2, 15):
        print(f"{names[k]:>9} {pct(us[:, k])}")
    for i in range(4):
        st, da, dn = us[:, 3 + 3 * i], us[:, 4 + 3 * i], us[:, 5 + 3 * i]
        print(f"tile{i} start {pct(st)}")
        print(f"   load lat {pct(da - st)}")
        print(f"   compute  {pct(dn - da)}")
    ntiles = np.sum(np.isfinite(us[:, 3:15:3]), 1)
    print("tiles/wave (<=4 stamped):", np.bincount(ntiles))
    sys.stdout.flush()
