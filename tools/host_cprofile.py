"""cProfile of the host side of the bench step (GPU box): which Python functions the graph constructor and
the MPN forward spend their host time in. usage: python tools/host_cprofile.py [workload]"""
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
st.sort_stats("tottime").print_stats(30)
