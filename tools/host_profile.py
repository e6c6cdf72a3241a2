"""Host-side (Python) cost of one pipeline step, per section, on the GPU box.

Times construct_graph() and the MPN forward with time.perf_counter around each call, plus
micro-costs of the building blocks (torch.empty on the device, a ctypes call, a D2H count
read-back). No device synchronisation inside the timed sections except the read-back itself.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pemp_amd import _lib  # noqa: E402


def timeit(fn, n=200):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t) / n
    torch.cuda.synchronize()
    return dt * 1e6


def main():
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["c3"]
    gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
    hm, feats, tags = bench.make_inputs(wl, 0, dev)
    model, _ = bench.make_model(wl, dev)
    L = _lib.lib()
    out, *_ = bench.run_step(wl, gc, model, hm, feats, tags, dev)
    x, ea, ei, types = out[0], out[1], out[2], out[7][:, 2]
    n = torch.empty(8, dtype=torch.int32, device=dev)
    print(f"torch.empty (device)         {timeit(lambda: torch.empty(1000, 128, device=dev)):8.1f} us")
    print(f"tensor.view/narrow           {timeit(lambda: x.narrow(0, 0, 10)):8.1f} us")
    print(f"ctypes pemp_abi_version      {timeit(lambda: L.pemp_abi_version()):8.1f} us")
    print(f"D2H 8 ints (.cpu())          {timeit(lambda: n.cpu(), 100):8.1f} us")
    print(f"current_stream ptr           {timeit(lambda: _lib.stream()):8.1f} us")
    with torch.no_grad():
        print(f"model forward (host+launch)  {timeit(lambda: model(x, ea, ei, node_types=types), 50):8.1f} us")
        print(f"model._weights               {timeit(lambda: model._weights(dev)):8.1f} us")
    cg = lambda: bench.pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                                      factor_list=None, masks=None, device=dev, testing=True,
                                                      heatmaps=None, num_joints=wl["J"]).construct_graph()
    print(f"construct_graph (incl. sync) {timeit(cg, 50):8.1f} us")
    print(f"full step                    {timeit(lambda: bench.run_step(wl, gc, model, hm, feats, tags, dev), 50):8.1f} us")


if __name__ == "__main__":
    main()
