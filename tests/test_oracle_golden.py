"""The oracle restatement reproduces the reference's own outputs (tests/golden, made by
oracle/gen_golden.py running the reference files). CPU only."""
import numpy as np
import pytest
import torch

from oracle import restate
from tests import golden_util as gu


@pytest.mark.parametrize("name", gu.names("gc_"))
def test_construct_graph_matches_reference(name):
    meta, a = gu.load(name)
    hm, feats, tags, masks = gu.gc_inputs(meta, a)
    out = restate.construct_graph(hm, feats, tags, masks, gu.gc_config(meta), meta["J"])
    x, ea, ei, det, sc, bi, tg = out[0], out[1], out[2], out[7], out[11], out[12], out[14]
    assert all(out[i] is None for i in (3, 4, 5, 6, 8, 9, 10, 13))
    np.testing.assert_array_equal(det.numpy(), a["joint_det"])
    np.testing.assert_array_equal(sc.numpy(), a["joint_scores"])
    np.testing.assert_array_equal(bi.numpy(), a["batch_index"])
    np.testing.assert_array_equal(tg.numpy(), a["joint_tags"])
    assert gu.sha(x) == meta["sha_x"]
    assert gu.sha(ea) == meta["sha_edge_attr"]
    assert gu.sha(ei) == meta["sha_edge_index"]
    assert ei.dtype == torch.int64 and det.dtype == torch.int64


@pytest.mark.parametrize("name", gu.names("mpn_"))
def test_mpn_matches_reference(name):
    meta, a = gu.load(name)
    cfg = gu.mpn_config(meta)
    sd = _state_dict(cfg, meta["salt"], meta.get("attn_gain", 1.0), meta.get("weight_gain", 1.0))
    pe, pn, pc, tag = restate.mpn_forward(sd, cfg, torch.from_numpy(a["x"]), torch.from_numpy(a["edge_attr"]),
                                         torch.from_numpy(a["edge_index"]), torch.from_numpy(a["node_types"]))
    assert len(pe) == int(a["n_edge_preds"]) and len(pn) == int(a["n_node_preds"]) and tag == [None]
    np.testing.assert_allclose(pe[-1].numpy(), a["edge_logits"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(pn[-1].numpy(), a["node_logits"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(pc[-1].numpy(), a["class_logits"], atol=1e-5, rtol=0)


def _state_dict(cfg, salt, attn_gain=1.0, weight_gain=1.0):
    from pemp_amd.mpn.model import NodeClassificationMPNSimple
    from pemp_amd import synthetic as syn
    m = NodeClassificationMPNSimple(cfg)
    return syn.closed_form_state_dict(m, salt, attn_gain, weight_gain)


def test_per_type_attention_golden_distinguishes_rows():
    """The per-type case must not be reproducible with the shared attention row (column 0)."""
    meta, a = gu.load("mpn_attn_pertype_t2")
    cfg = gu.mpn_config(meta)
    assert cfg.AGGR_SUB == "node_edge_attn_per_type"
    sd = _state_dict(cfg, meta["salt"], meta.get("attn_gain", 1.0))
    assert sd["mpn_node_cls.attn_net.0.weight"].shape == (17, 64)
    cfg.AGGR_SUB = "node_edge_attn"
    pe, pn, pc, _ = restate.mpn_forward(sd, cfg, torch.from_numpy(a["x"]), torch.from_numpy(a["edge_attr"]),
                                        torch.from_numpy(a["edge_index"]), torch.from_numpy(a["node_types"]))
    assert np.abs(pc[-1].numpy() - a["class_logits"]).max() > 5e-4      # 5x the logit tolerance


def test_feature_knn_restatement_properties():
    """feature_knn_edge_index (ConstructGraph.py:370-374): symmetric, no self loops, sorted by (src, dst);
    n <= k + 1 gives the fully graph; every node keeps its k nearest by the fp32 fma-chain distance
    (exact f64 check on a draw without near-ties); duplicate feature rows tie by node index."""
    g = torch.Generator().manual_seed(5)
    for n in (0, 1, 2, 51, 52, 130):
        x = torch.randn(n, 24, generator=g)
        ei = restate.feature_knn_edge_index(x)
        if n <= 51:
            assert torch.equal(ei, restate.fully_edge_index(n))
            continue
        s, d = ei
        assert bool((s != d).all())
        key = s * n + d
        assert bool((key[1:] > key[:-1]).all())                      # coalesced order, no duplicates
        adj = torch.zeros(n, n, dtype=torch.bool)
        adj[s, d] = True
        assert torch.equal(adj, adj.t())
        d64 = ((x[:, None, :].double() - x[None, :, :].double()) ** 2).sum(-1)
        d64.fill_diagonal_(float("inf"))
        nearest = torch.argsort(d64, dim=1)[:, :50]
        assert bool(adj.gather(1, nearest).all())                    # each node's 50 nearest are neighbours
        assert int(adj.sum(1).min()) >= 50
    # all rows equal: every distance ties at 0 -> nodes 0..50 for every query, symmetrised
    n = 80
    ei = restate.feature_knn_edge_index(torch.ones(n, 8))
    adj = torch.zeros(n, n, dtype=torch.bool)
    adj[ei[0], ei[1]] = True
    want = torch.zeros(n, n, dtype=torch.bool)
    want[:, :51] = True
    want = want | want.t()
    want.fill_diagonal_(False)
    assert torch.equal(adj, want)
