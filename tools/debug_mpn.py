"""Stage-by-stage check of pemp_mpn_forward against a CPU recomputation (debug tool, GPU box).

Reads the workspace slices (same carve order as csrc/mpn.hip mpn_carve) after a forward and
prints the max error of each stage: node/edge embedding, Q0, e' (sorted order), aggregation,
node update, logits.
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pemp_amd  # noqa: E402
from oracle import restate  # noqa: E402
from pemp_amd import config as pcfg, synthetic as syn  # noqa: E402
from tests import golden_util as gu  # noqa: E402


def carve(ws, T, N, E):
    off = 0
    out = {}

    def take(name, n, dt):
        nonlocal off
        off = (off + 255) // 256 * 256
        sz = n * (4 if dt in (torch.int32, torch.float32) else 8)
        out[name] = ws[off:off + sz].view(dt)
        off += sz

    K = T * N
    take("err", 64, torch.int32); take("cnt", K + 1, torch.int32)
    take("seg", K + 1, torch.int32); take("wg_start", 19, torch.int32)
    for n in ("perm", "s_src", "s_dst", "s_orig"):
        take(n, E, torch.int32)
    take("X", N * 128, torch.float32); take("NT", N * (128 + 64 * T), torch.float32)
    take("agg", N * T * 64, torch.float32)
    for n in ("Q0", "EA", "EB"):
        take(n, E * 64, torch.float32)
    return out


def main(variant="add", steps=1, gname="gc_small_fully"):
    dev = torch.device("cuda:0")
    meta, a = gu.load(gname)
    J = meta["J"]
    hm, feats, tags, masks = gu.gc_inputs(meta, a)
    g = restate.construct_graph(hm, feats, tags, masks, gu.gc_config(meta), J)
    x, ea, ei, types = g[0], g[1], g[2], g[7][:, 2]
    cfg = pcfg.published_mpn_config(J, steps, variant)
    model = pemp_amd.get_mpn_model(cfg)
    sd = syn.closed_form_state_dict(model, 0.5)
    model.load_state_dict(sd)
    model.eval().to(dev)
    with torch.no_grad():
        pe, pn, pc, _ = model(x.to(dev), ea.to(dev), ei.to(dev), node_types=types.to(dev))
    torch.cuda.synchronize()
    T, N, E = model.num_types, x.shape[0], ei.shape[1]
    w = {k: v.cpu() for k, v in carve(model._ws.buf, T, N, E).items()}
    print(f"variant={variant} steps={steps} N={N} E={E} T={T} err={w['err'][0].item()}")
    print("wg_start", w["wg_start"][:T + 1].tolist(), "seg[-1]", w["seg"][T * N].item())
    s_orig = w["s_orig"].long()
    print("perm is permutation:", torch.equal(torch.sort(s_orig).values, torch.arange(E)))
    src_t = types if T > 1 else torch.zeros_like(types)
    key = src_t[ei[0]] * N + ei[1]
    print("sorted keys monotone:", bool((key[s_orig][1:] >= key[s_orig][:-1]).all()))
    print("s_src ok:", torch.equal(w["s_src"].long(), ei[0][s_orig]), "s_dst ok:", torch.equal(w["s_dst"].long(), ei[1][s_orig]))

    x0 = restate._mlp(sd, "node_embedding", x, cfg.NODE_EMB.OUTPUT_SIZES, True)
    e0 = restate._mlp(sd, "edge_embedding", ea, cfg.EDGE_EMB.OUTPUT_SIZES, True)
    X = w["X"].view(N, 128)
    print("node emb err", (X[:, :64] - x0).abs().max().item() if steps == 0 else "(overwritten)",
          " x_init half:", (X[:, :64] - x0).abs().max().item())
    EA = w["EA"].view(E, 64)
    print("edge emb err (EA = e_init sorted)", (EA - e0[s_orig]).abs().max().item())
    p = "mpn_node_cls"
    W1, b1 = sd[f"{p}.mlp_edge.0.weight"], sd[f"{p}.mlp_edge.0.bias"]
    q0 = e0 @ W1[:, 256:320].T + b1
    print("Q0 err", (w["Q0"].view(E, 64) - q0[s_orig]).abs().max().item())
    xx = torch.cat([x0, x0], 1)
    NT = w["NT"].view(N, 128 + 64 * T)
    print("NT A err", (NT[:, :64] - xx @ W1[:, :128].T).abs().max().item(),
          "B err", (NT[:, 64:128] - xx @ W1[:, 128:256].T).abs().max().item())
    if steps == 1:
        ee = torch.cat([e0, e0], 1)
        i, j = ei[1], ei[0]
        h = F.relu(torch.cat([xx[i], xx[j], ee], 1) @ W1.T + b1)
        e1 = F.relu(h @ sd[f"{p}.mlp_edge.2.weight"].T + sd[f"{p}.mlp_edge.2.bias"])
        print("(e' not stored on the last step)")
        if T == 1:
            Wn, bn = sd[f"{p}.mlp_node.0.weight"], sd[f"{p}.mlp_node.0.bias"]
            print("NT P err", (NT[:, 128:192] - (xx @ Wn[:, :128].T + bn)).abs().max().item())
            m = F.relu(torch.cat([xx[i], e1], 1) @ Wn.T + bn)
            agg = restate._scatter(m, i, N, cfg.AGGR)
            print("agg err", (w["agg"].view(N, 64) - agg).abs().max().item())
            print("x_new err", (X[:, 64:] - agg).abs().max().item())
        logit = restate._mlp(sd, "edge_classification", e1, cfg.EDGE_CLASS.OUTPUT_SIZES, False).squeeze()
        print("edge logit err", (pe[-1].cpu() - logit).abs().max().item())
    rpe, rpn, rpc, _ = restate.mpn_forward(sd, cfg, x, ea, ei, types)
    for nm, aa, bb in (("edge", pe[-1], rpe[-1]), ("node", pn[-1], rpn[-1]), ("class", pc[-1], rpc[-1])):
        print(f"final {nm} logits err", (aa.cpu() - bb).abs().max().item())


if __name__ == "__main__":
    for v, s in (("add", 1), ("attn", 1), ("add", 2), ("attn", 3)):
        main(v, s)
        print("-" * 60)
