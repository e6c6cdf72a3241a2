"""Host-side cost of each part of one pipeline step (GPU box): construct_graph pieces and the MPN
forward pieces, timed with perf_counter over many repetitions (the GPU runs the same work, so
results are "host cost when the host is the bottleneck")."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pemp_amd import _lib  # noqa: E402


def t(fn, n=300):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    return dt


def main():
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["c3"]
    gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
    hm, feats, tags = bench.make_inputs(wl, 0, dev)
    model, _ = bench.make_model(wl, dev)
    L = _lib.lib()
    out, *_ = bench.run_step(wl, gc, model, hm, feats, tags, dev)
    x, ea, ei, types = out[0], out[1], out[2], out[7][:, 2]
    N, E = x.shape[0], ei.shape[1]
    ws = model._ws.get(0, dev)
    desc = model._desc_ref
    fw = model._weights(dev)
    st = _lib.stream(dev)
    rows = [
        ("_lib.stream(dev)", lambda: _lib.stream(dev)),
        ("model._weights", lambda: model._weights(dev)),
        ("torch.empty x3", lambda: (torch.empty(2, E, device=dev), torch.empty(2, N, device=dev),
                                    torch.empty(2, N, 17, device=dev))),
        ("workspace_size", lambda: L.pemp_mpn_workspace_size(desc, N, E)),
        ("pemp_mpn_prepare (5 launches)", lambda: L.pemp_mpn_prepare(desc, ei.data_ptr(), types.data_ptr(), N, E,
                                                                    ws.data_ptr(), ws.numel(), st)),
        ("pemp_mpn_forward (rest)", lambda: L.pemp_mpn_forward(desc, fw.struct_ref, x.data_ptr(), ea.data_ptr(),
                                                               ei.data_ptr(), types.data_ptr(), N, E,
                                                               ws.data_ptr() + 0, ws.data_ptr(), ws.data_ptr(),
                                                               ws.data_ptr(), ws.numel(), st)),
        ("model forward (all)", lambda: model(x, ea, ei, node_types=types)),
        ("out[7][:, 2]", lambda: out[7][:, 2]),
    ]
    with torch.no_grad():
        for name, fn in rows:
            print(f"{name:34s} {t(fn, 100):8.1f} us", flush=True)
    cg = lambda: bench.pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                                      factor_list=None, masks=None, device=dev, testing=True,
                                                      heatmaps=None, num_joints=wl["J"]).construct_graph()
    print(f"{'construct_graph (incl. sync)':34s} {t(cg, 50):8.1f} us")
    print(f"{'full step':34s} {t(lambda: bench.run_step(wl, gc, model, hm, feats, tags, dev), 50):8.1f} us")
    # one empty launch cost
    z = torch.empty(1, device=dev)
    print(f"{'torch z.zero_() launch':34s} {t(lambda: z.zero_(), 300):8.1f} us")


if __name__ == "__main__":
    main()
