"""A/B of library builds on the MPN forward alone (GPU box).

usage: python tools/mpn_ab.py [--workload c3] [--iters 30] default v1 v2 ...
  "default" = the in-tree libpemp.so, any other name = build_ab/libpemp_<name>.so (tools/build_variant.sh).
Each build runs in its own process: the workload's graph is built once, then the MPN forward runs --iters times
with the library's event profiler on every kernel; prints one line per build (per-kernel average us, forward
ms) and the largest logit difference against the first build listed (edge / node / class, last recorded step).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def child(args):
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from pemp_amd import _lib
    wl = bench.WORKLOADS[args.workload]
    dev = torch.device("cuda", 0)
    gc = bench.pcfg.inference_gc_config(wl["graph"], 5, False)
    hm, feats, tags = bench.make_inputs(wl, 0, dev)
    model, _ = bench.make_model(wl, dev)
    out = bench.run_step(wl, gc, model, hm, feats, tags, dev)[0]
    x, ea, ei, types = out[0], out[1], out[2], out[7][:, 2]
    with torch.no_grad():
        for _ in range(3):
            res = model(x, ea, ei, node_types=types)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            model(x, ea, ei, node_types=types)
        torch.cuda.synchronize()
        fwd_ms = (time.perf_counter() - t0) / args.iters * 1e3
        _lib.prof_enable("*")
        for _ in range(args.iters):
            res = model(x, ea, ei, node_types=types)
        torch.cuda.synchronize()
    st = _lib.prof_report()
    _lib.prof_enable(None)
    torch.save({"edge": res[0][-1].cpu(), "node": res[1][-1].cpu(), "class": res[2][-1].cpu()}, args.dump)
    print(json.dumps({"forward_ms": round(fwd_ms, 4), "N": int(x.shape[0]), "E": int(ei.shape[1]),
                      "kernels_us": {k: round(ms / n * 1e3, 2) for k, (n, ms) in sorted(st.items())}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--dump")
    ap.add_argument("variants", nargs="*")
    args = ap.parse_args()
    if args.child:
        return child(args)
    import torch
    os.makedirs(OUT, exist_ok=True)
    first = None
    for v in args.variants:
        env = dict(os.environ)
        if v != "default":
            env["PEMP_LIB"] = os.path.join(ROOT, "build_ab", f"libpemp_{v}.so")
        dump = os.path.join(OUT, f"mpnab_{args.workload}_{v}.pt")
        res = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--workload", args.workload,
                              "--iters", str(args.iters), "--dump", dump], env=env, capture_output=True, text=True,
                             timeout=300)
        if res.returncode != 0:
            print(v, "FAILED", res.stderr[-1500:], flush=True)
            sys.exit(1)
        rec = json.loads(res.stdout.strip().splitlines()[-1])
        d = torch.load(dump, weights_only=True)
        if first is None:
            first = d
            diff = {}
        else:
            diff = {k: float((d[k] - first[k]).abs().max()) for k in d}
        print(v, json.dumps({**rec, "max_abs_diff_vs_first": diff}), flush=True)


if __name__ == "__main__":
    main()
