"""The e2e leg of bench.py alone, interleaved over variants in one process (the leg is bound by host Python and its
spread between runs and boxes is large): groupings in flight (bench.E2E_DEPTH) x launches first (bench.E2E_EARLY), or
with E2E_AB_ENTRY=1
batch-step entry on / off (graph_constructor._STEP_ENTRY) x depth 1 / 2, alternating.
usage: python tools/e2e_ab.py [workload] [rounds]
-> one line per (variant, round) and the per-variant medians"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import pemp_amd  # noqa: E402
from importlib import import_module  # noqa: E402

gcm = import_module("pemp_amd.graph_constructor")
name = sys.argv[1] if len(sys.argv) > 1 else "c3"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
wl = bench.WORKLOADS[name]
dev = torch.device("cuda:0")
gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
hm, feats, tags = bench.make_inputs(wl, 0, dev)
model, _ = bench.make_model(wl, dev)
if wl["graph"] == "fully":
    pemp_amd.bind_mpn(model)
for _ in range(3):
    bench.run_step(wl, gc, model, hm, feats, tags, dev)
torch.cuda.synchronize()
res = {}
variants = [(e, d, 1) for e in (True, False) for d in (1, 2)] if os.environ.get("E2E_AB_ENTRY") else \
    [(True, 1, 0), (True, 2, 0), (True, 1, 1), (True, 2, 1), (True, 3, 1)]
for r in range(rounds):
    for entry, depth, early in variants:
        gcm._STEP_ENTRY = entry
        bench.E2E_DEPTH = depth
        bench.E2E_EARLY = bool(early)
        rec = bench.e2e_pipeline(wl, gc, model, hm, feats, tags, dev, 20, 5, 1)
        key = f"entry={int(entry)} depth={depth} early={early}"
        res.setdefault(key, []).append(rec["images_per_sec"])
        print(name, key, r, rec["images_per_sec"], rec["stage_host_ms_per_batch"], flush=True)
for k, v in res.items():
    print(name, k, "median", round(statistics.median(v), 1), "all", v, flush=True)
