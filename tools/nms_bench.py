"""Isolated timing of the detection stages at a bench workload's shape: back-to-back pemp_detect calls with only the
NMS pass (stages = PEMP_DETECT_NMS) and with the whole detection, HIP events on the launch stream.
usage: python tools/nms_bench.py [workload] [reps] -> one JSON line (PEMP_NMS_QUAD / PEMP_LIB select the variant)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import pemp_amd  # noqa: E402,F401
from pemp_amd import _lib  # noqa: E402

wl_name = sys.argv[1] if len(sys.argv) > 1 else "c3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
wl = bench.WORKLOADS[wl_name]
dev = torch.device("cuda:0")
hm, _, _ = bench.make_inputs(wl, 0, dev)
B, J, H, W = hm.shape
L = _lib.lib()
st = _lib.stream(dev)
topk, thr, pool = 5, 0.1, 5
ws = torch.empty(L.pemp_detect_workspace_size(B, J, H, W, topk), dtype=torch.uint8, device=dev)
cap = 512
det = torch.empty(B, cap, 3, dtype=torch.int64, device=dev)
dsc = torch.empty(B, cap, dtype=torch.float32, device=dev)
n_det = torch.empty(B, dtype=torch.int32, device=dev)


def call(stages):
    _lib.check(L.pemp_detect(_lib.ptr(hm), None, B, J, H, W, pool, thr, 1, topk, stages, _lib.ptr(ws), ws.numel(),
                             _lib.ptr(det), _lib.ptr(dsc), _lib.ptr(n_det), cap, None, st))


out = {"workload": wl_name, "quad": os.environ.get("PEMP_NMS_QUAD", "default"), "bytes": hm.numel() * 4}
# cold: the 256 MB Infinity Cache (MALL) holds most of a 223 MB batch between back-to-back calls; a 1 GiB copy
# between calls evicts it, as the MPN's traffic does inside a step (events around each call only)
scrub = torch.empty(2, 512 << 20, dtype=torch.uint8, device=dev)
s0 = torch.cuda.current_stream(dev)
for name, stages in (("nms", 1), ("detect", 3)):
    ts = []
    for i in range(reps // 2 + 3):
        scrub[1].copy_(scrub[0])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s0)
        call(stages)
        b.record(s0)
        b.synchronize()
        if i >= 3:
            ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    out[name + "_cold_us"] = round(ts[len(ts) // 2], 2)
for name, stages in (("nms", 1), ("detect", 3)):
    for _ in range(5):
        call(stages)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream(dev)
    e0.record(s)
    for _ in range(reps):
        call(stages)
    e1.record(s)
    e1.synchronize()
    out[name + "_us"] = round(e0.elapsed_time(e1) * 1000 / reps, 2)
out["nms_TBs"] = round(out["bytes"] / out["nms_us"] / 1e6, 3)
out["nms_cold_TBs"] = round(out["bytes"] / out["nms_cold_us"] / 1e6, 3)
out["n_det"] = n_det.tolist()
print(json.dumps(out), flush=True)
