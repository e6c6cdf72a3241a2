"""Diagnostic: determinism of the MPN forward on the symmetric-prepare test graph (fast path twice, sorting path
twice), per output max |diff| between runs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_gpu_mpn import make_model, run, DEV  # noqa: E402
from pemp_amd import config as pcfg  # noqa: E402
from pemp_amd.mpn import model as mm  # noqa: E402

for variant in ("max", "attn"):
    g = torch.Generator().manual_seed(11)
    N = 700
    m = torch.rand(N, N, generator=g) < 0.02
    m[:, 3] = True
    m[np.arange(0, N, 7), np.arange(0, N, 7)] = True
    m[650:] = False
    m[:, 650:] = False
    m = m | m.T
    ei = m.nonzero().T.contiguous()
    cfg = pcfg.published_mpn_config(17, 3, variant)
    model, _ = make_model(cfg, 3.75, "f16x3")
    types = torch.randint(0, 17, (N,), generator=g)
    x = torch.randn(N, 128, generator=g)
    ea = torch.randn(ei.shape[1], 19, generator=g)
    eid = ei.to(DEV)
    outs = {}
    for name in ("fast1", "fast2", "slow1", "slow2"):
        mm._SYM_OFF = name.startswith("slow")
        if not mm._SYM_OFF:
            eid._pemp_sym = eid._version
        o = run(model, x.to(DEV), ea.to(DEV), eid, types.to(DEV))
        outs[name] = [t.cpu() for t in o[0] + o[1] + o[2]]
    for a, b in (("fast1", "fast2"), ("slow1", "slow2"), ("fast1", "slow1")):
        d = [float((p - q).abs().max()) for p, q in zip(outs[a], outs[b])]
        print(variant, a, b, "E", ei.shape[1], "max diffs", ["%.3g" % v for v in d], flush=True)
    mm._SYM_OFF = False
