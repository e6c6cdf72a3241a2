"""cProfile of the host side of the bench step (GPU box): which Python functions the graph constructor and
the MPN forward spend their host time in. usage: python tools/host_cprofile.py [workload]
(PEMP_CAP=1: the model bound to the graph constructor, capacity mode, as bench.py runs fully-graph workloads)"""
import time
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
dev = torch.device("cuda", 0)
gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
hm, feats, tags = bench.make_inputs(wl, 0, dev)
model, _ = bench.make_model(wl, dev)
if os.environ.get("PEMP_CAP"):
    bench.pemp_amd.bind_mpn(model)
for _ in range(5):
    bench.run_step(wl, gc, model, hm, feats, tags, dev)
torch.cuda.synchronize()
with torch.no_grad():
    t0 = time.perf_counter()
    for _ in range(200):
        bench.run_step(wl, gc, model, hm, feats, tags, dev)
    torch.cuda.synchronize()
    print(f"wall per step (serial, no profiler): {(time.perf_counter() - t0) / 200 * 1e3:.4f} ms", flush=True)
for _ in range(5):
    bench.run_step(wl, gc, model, hm, feats, tags, dev)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
with torch.no_grad():
    for _ in range(50):
        bench.run_step(wl, gc, model, hm, feats, tags, dev)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(25)
