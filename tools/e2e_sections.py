"""finish_batch_start and group_persons_start section timing (GPU box): wraps numpy / torch / ctypes entry points used
by the two functions with perf_counter accumulators by monkeypatching, runs the e2e leg, prints per-batch µs."""
import collections, os, sys, time
sys.path.insert(0, os.getcwd())
import torch, numpy as np
import bench
from pemp_amd import pose as pp
acc = collections.defaultdict(float); cnt = collections.defaultdict(int)
def wrap(mod, name, label):
    f = getattr(mod, name)
    def g(*a, **k):
        t = time.perf_counter(); r = f(*a, **k); acc[label] += time.perf_counter() - t; cnt[label] += 1; return r
    setattr(mod, name, g)
for n in ("fill_mean", "_maps", "_check_coords", "_to_host_async", "_start"):
    wrap(pp, n, n)
wrap(pp, "finish_batch_start", "finish_batch_start")
wrap(pp, "group_persons_start", "group_persons_start")
wl = bench.WORKLOADS["c3"]; dev = torch.device("cuda", 0)
gc = bench.pcfg.inference_gc_config("fully", 5, False)
hm, feats, tags = bench.make_inputs(wl, 0, dev)
model, _ = bench.make_model(wl, dev); bench.pemp_amd.bind_mpn(model)
bench.e2e_pipeline(wl, gc, model, hm, feats, tags, dev, 20, 5, 1)
acc.clear(); cnt.clear()
rec = bench.e2e_pipeline(wl, gc, model, hm, feats, tags, dev, 50, 5, 1)
print(rec["images_per_sec"], rec["stage_host_ms_per_batch"])
for k in sorted(acc, key=lambda k: -acc[k]):
    print(f"{k:24s} {acc[k] / cnt[k] * 1e6:8.1f} us x {cnt[k]}")
