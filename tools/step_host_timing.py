"""Host-side breakdown of bench.py's timed step (GPU box): how long run_step spends before the detection launch, in
the count wait, after it, and in the model call, plus a cProfile of the loop. usage:
python tools/step_host_timing.py [workload] [steps]"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from importlib import import_module  # noqa: E402

gcm = import_module("pemp_amd.graph_constructor")

name = sys.argv[1] if len(sys.argv) > 1 else "c2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
mode = sys.argv[3] if len(sys.argv) > 3 else "plain"   # plain | stream (inside torch.cuda.stream) | bench (bench.run_step)
wl = bench.WORKLOADS[name]
dev = torch.device("cuda", 0)
gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
hm, feats, tags = bench.make_inputs(wl, 0, dev)
model, _ = bench.make_model(wl, dev)
if wl["graph"] == "fully":
    bench.pemp_amd.bind_mpn(model)
bench._lib.lib()

acc = {"wait": 0.0, "cg": 0.0, "model": 0.0}
orig_wait = gcm.NaiveGraphConstructor._wait_counts


def timed_wait(counts, d):
    t = time.perf_counter()
    r = orig_wait(counts, d)
    acc["wait"] += time.perf_counter() - t
    return r


gcm.NaiveGraphConstructor._wait_counts = staticmethod(timed_wait)

L = bench._lib.lib()
for fn in ("pemp_detect", "pemp_fully_graph_build_cap", "pemp_mpn_forward_fully_cap"):
    acc[fn] = 0.0

    def wrap(f, name):
        def w(*a):
            t = time.perf_counter()
            r = f(*a)
            acc[name] += time.perf_counter() - t
            return r
        return w
    setattr(L, fn, wrap(getattr(L, fn), fn))


def step_plain():
    t0 = time.perf_counter()
    out = bench.pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                              factor_list=None, masks=None, device=dev, testing=True, heatmaps=None,
                                              num_joints=wl["J"]).construct_graph()
    t1 = time.perf_counter()
    model(out[0], out[1], out[2], node_types=out[7][:, 2])
    t2 = time.perf_counter()
    acc["cg"] += t1 - t0
    acc["model"] += t2 - t1


s0 = torch.cuda.current_stream(dev)


def step_stream():
    with torch.cuda.stream(s0):
        step_plain()


def step_bench():
    bench.run_step(wl, gc, model, hm, feats, tags, dev)


step = {"plain": step_plain, "stream": step_stream, "bench": step_bench}[mode]


for _ in range(20):
    step()
torch.cuda.synchronize()
for k in acc:
    acc[k] = 0.0
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
us = {k: round(v / steps * 1e6, 1) for k, v in acc.items()}
print({"workload": name, "mode": mode, "us_per_step": round(dt / steps * 1e6, 1), "construct_graph_us": us["cg"],
       "of_which_count_wait_us": us["wait"], "model_call_us": us["model"],
       "c_calls_us": {k: us[k] for k in us if k.startswith("pemp_")}}, flush=True)

# the host cost alone: the same step with the GPU work already done (a synchronize before each step)
for k in acc:
    acc[k] = 0.0
t0 = time.perf_counter()
for _ in range(steps):
    torch.cuda.synchronize()
    step()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
us = {k: round(v / steps * 1e6, 1) for k, v in acc.items()}
print({"synced_steps_us": round(dt / steps * 1e6, 1), "construct_graph_us": us["cg"],
       "of_which_count_wait_us": us["wait"], "model_call_us": us["model"],
       "c_calls_us": {k: us[k] for k in us if k.startswith("pemp_")}}, flush=True)

pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
