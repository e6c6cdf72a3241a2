"""Host time between consecutive kernel launches inside the library (GPU box), one bench step:
PEMP_HOST_TRACE=1 PEMP_LIB=build_ab/libpemp_ht.so python tools/host_trace.py [workload], on a diagnostics
build of the library (tools/build_variant.sh ht common.hip -DPEMP_HOST_TRACE, and mpn.hip / graph.hip the same way). Python-side marks: construct_graph entry/exit,
count wait, model.forward entry/exit."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pemp_amd import _lib  # noqa: E402
from pemp_amd import graph_constructor as gcm  # noqa: E402

wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
dev = torch.device("cuda", 0)
gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
hm, feats, tags = bench.make_inputs(wl, 0, dev)
model, _ = bench.make_model(wl, dev)
L = _lib.lib()
dump = L.pemp_host_trace_dump
dump.restype = ctypes.c_int
for _ in range(5):
    bench.run_step(wl, gc, model, hm, feats, tags, dev)
torch.cuda.synchronize()
dump()
marks = []
pc = time.perf_counter_ns
orig_wait = gcm.NaiveGraphConstructor._wait_counts


def wait(counts, d):
    marks.append(("wait_counts enter", pc()))
    r = orig_wait(counts, d)
    marks.append(("wait_counts exit", pc()))
    return r


gcm.NaiveGraphConstructor._wait_counts = staticmethod(wait)
orig_fwd = type(model).forward


def fwd(self, *a, **k):
    marks.append(("forward enter", pc()))
    r = orig_fwd(self, *a, **k)
    marks.append(("forward exit", pc()))
    return r


type(model).forward = fwd
for rep in range(3):
    marks.clear()
    torch.cuda.synchronize()
    dump()
    t0 = pc()
    marks.append(("step start", t0))
    with torch.no_grad():
        bench.run_step(wl, gc, model, hm, feats, tags, dev)
    marks.append(("step host end", pc()))
    torch.cuda.synchronize()
    marks.append(("gpu idle", pc()))
    if rep == 2:
        for name, t in marks:
            print(f"[py] {t} {name}", flush=True)
        sys.stdout.flush()
        dump()
