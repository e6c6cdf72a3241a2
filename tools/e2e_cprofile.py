"""cProfile of bench.py's end-to-end leg (GPU box): where the host time of the pipelined construct_graph -> MPN ->
grouping -> finishing loop goes. usage: python tools/e2e_cprofile.py [workload] [steps]"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
wl = bench.WORKLOADS[name]
dev = torch.device("cuda", 0)
gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
hm, feats, tags = bench.make_inputs(wl, 0, dev)
model, _ = bench.make_model(wl, dev)
if wl["graph"] == "fully":
    bench.pemp_amd.bind_mpn(model)
rec = bench.e2e_pipeline(wl, gc, model, hm, feats, tags, dev, steps, 5, 1)
print(rec, flush=True)
pr = cProfile.Profile()
pr.enable()
bench.e2e_pipeline(wl, gc, model, hm, feats, tags, dev, steps, 5, 1)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(60)
# where the queueing stages spend it (callees of the pose / constructor entry points)
st.sort_stats("cumulative").print_callees("finish_batch_start|group_persons_start|_construct|gpu_part")
