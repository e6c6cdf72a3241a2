"""The frontend_heatmaps leg of bench.py alone (detection on reference-op maps vs the projected front-end).
usage: python tools/frontend_detect.py [workload] -> one JSON line (PEMP_LIB selects the library)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

wl_name = sys.argv[1] if len(sys.argv) > 1 else "c3"
wl = bench.WORKLOADS[wl_name]
dev = torch.device("cuda:0")
gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
_, feats, _ = bench.make_inputs(wl, 0, dev)
res = bench.frontend_heatmaps(wl, gc, feats, dev)
res["workload"] = wl_name
res["lib"] = os.environ.get("PEMP_LIB", "default")
print(json.dumps(res), flush=True)
