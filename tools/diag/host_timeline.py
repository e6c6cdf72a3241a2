"""Host timeline of one bench step (GPU box): every libpemp call, the count-copy event wait and the
MPN forward entry, as microseconds from the step start. Shows where the host sits on the critical
path between the graph build and the first MPN kernel."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from pemp_amd import _lib  # noqa: E402
from pemp_amd import graph_constructor as gcm  # noqa: E402

LOG = []
pc = time.perf_counter


class Proxy:
    def __init__(self, L):
        self._L = L

    def __getattr__(self, name):
        fn = getattr(self._L, name)
        if not callable(fn):
            return fn

        def w(*a):
            t0 = pc()
            r = fn(*a)
            LOG.append((name, t0, pc()))
            return r
        return w


def main():
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["c3"]
    gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
    hm, feats, tags = bench.make_inputs(wl, 0, dev)
    model, _ = bench.make_model(wl, dev)
    for _ in range(5):
        bench.run_step(wl, gc, model, hm, feats, tags, dev)
    torch.cuda.synchronize()
    _lib._LIB = Proxy(_lib.lib())
    orig_wait = gcm.NaiveGraphConstructor._wait_counts

    def wait(counts, d):
        t0 = pc(); r = orig_wait(counts, d); LOG.append(("wait_counts", t0, pc()))
        return r
    gcm.NaiveGraphConstructor._wait_counts = staticmethod(wait)
    orig_fwd = type(model).forward

    def fwd(self, *a, **k):
        LOG.append(("model.forward enter", pc(), pc()))
        r = orig_fwd(self, *a, **k)
        LOG.append(("model.forward exit", pc(), pc()))
        return r
    type(model).forward = fwd
    for rep in range(6):
        LOG.clear()
        torch.cuda.synchronize()
        t0 = pc()
        bench.run_step(wl, gc, model, hm, feats, tags, dev)
        t1 = pc()
        torch.cuda.synchronize()
        t2 = pc()
        if rep == 5:
            for name, a, b in LOG:
                print(f"{(a - t0) * 1e6:8.1f} {(b - a) * 1e6:7.1f}  {name}")
            print(f"host step {(t1 - t0) * 1e6:.1f} us, until GPU idle {(t2 - t0) * 1e6:.1f} us")


if __name__ == "__main__":
    main()
