"""Debug helper (GPU box): one test_detection_edges case through the library in PEMP_LIB (or the in-tree one),
printing the first differences against the oracle per image."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import pemp_amd
from oracle import restate
from pemp_amd import config as pcfg, synthetic as syn
from tests.test_gpu_graph import _edge_maps, run_gc

H, W, pool = (int(a) for a in sys.argv[1:4])
B, J = 3, 17
hm = _edge_maps(B, J, H, W, H * W + pool)
feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25))
tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
gc = pcfg.inference_gc_config("fully", pool, False)
out = run_gc(gc, J, hm, feats, tags, None)
ref = restate.construct_graph(hm, feats, tags, None, gc, J)
det, sc, bi = out[7].cpu(), out[11].cpu(), out[12].cpu()
rdet, rsc, rbi = ref[7], ref[11], ref[12]
print("counts got", torch.bincount(bi, minlength=B).tolist(), "ref", torch.bincount(rbi, minlength=B).tolist())
for b in range(B):
    g = det[bi == b]; r = rdet[rbi == b]
    gs = sc[bi == b]; rs = rsc[rbi == b]
    n = min(len(g), len(r))
    bad = [i for i in range(n) if not torch.equal(g[i], r[i]) or gs[i] != rs[i]]
    print("image", b, "n", len(g), len(r), "first bad", bad[:5])
    for i in bad[:5]:
        print("   ", i, g[i].tolist(), float(gs[i]), "ref", r[i].tolist(), float(rs[i]))
