"""Host-side weight folding (mpn/fold.py) checked on CPU against the oracle's literal restatement:
the dense layers ``node_mlp_kernel`` runs for UPDATE_TYPE hierarch_mlp / hierarch_cnn must compute
HierarchUpdateMlp / HierarchUpdateCnn (layers.py:89-154) exactly (fp64, up to rounding)."""
import pytest
import torch

import pemp_amd
from oracle import restate
from pemp_amd import config as pcfg, synthetic as syn
from pemp_amd.mpn.fold import hierarch_dense_layers


@pytest.mark.parametrize("utype,J", [("hierarch_mlp", 17), ("hierarch_mlp", 14), ("hierarch_cnn", 17)])
def test_hierarch_dense_fold(utype, J):
    cfg = pcfg.published_mpn_config(J, 2, "attn")
    cfg.UPDATE_TYPE = utype
    model = pemp_amd.get_mpn_model(cfg)
    sd = syn.closed_form_state_dict(model, 3.25)
    model.load_state_dict(sd)
    upd = model.mpn_node_cls.update_mlp
    T = model.num_types
    agg = torch.randn(37, T, 64, dtype=torch.float64, generator=torch.Generator().manual_seed(J))
    v = agg.reshape(37, -1)
    layers = hierarch_dense_layers(upd, T)
    assert [W.shape[0] % 16 for W, _ in layers] == [0] * len(layers) and layers[-1][0].shape[0] == 64
    for W, b in layers:
        v = torch.relu(v @ W.T + b)
    sd64 = {k: t.double() for k, t in sd.items()}
    p = "mpn_node_cls.update_mlp"
    ref = restate._hierarch_mlp(sd64, p, agg, J) if utype == "hierarch_mlp" else restate._hierarch_cnn(sd64, p, agg)
    assert torch.allclose(v, ref, rtol=0, atol=1e-12)


def test_hierarch_state_dict_keys():
    cfg = pcfg.published_mpn_config(17, 2, "attn")
    cfg.UPDATE_TYPE = "hierarch_mlp"
    keys = [k for k in pemp_amd.get_mpn_model(cfg).state_dict() if ".update_mlp." in k]
    assert keys[:2] == ["mpn_node_cls.update_mlp.first_layer.0.weight", "mpn_node_cls.update_mlp.first_layer.0.bias"]
    assert len(keys) == 2 * (7 + 6 + 1)


@pytest.mark.parametrize("J", [17, 14])
def test_composed_edge_embedding(J):
    """pemp_mpn_weights.emb_comp_*: Q0 and R0 from the third embedding layer's output through the composed
    matrices equal, in fp64, the literal chain e_init = W4 h3 + b4, Q0 = W1[:, e_init] e_init + b1,
    R0 = Q0 + W1[:, e_cur] e_init of the reference's first edge-MLP layer (layers.py:171-175 on
    NodeClassificationMPNSimple.py:49-56's embedding, BatchNorm folded)."""
    from pemp_amd.mpn.fold import composed_embedding, edge_embedding_layers
    cfg = pcfg.published_mpn_config(J, 3, "attn")
    model = pemp_amd.get_mpn_model(cfg)
    model.load_state_dict(syn.closed_form_state_dict(model, 1.75))
    emb = edge_embedding_layers(model.edge_embedding)
    W1 = model.mpn_node_cls.mlp_edge[0].weight.detach().double()
    b1 = model.mpn_node_cls.mlp_edge[0].bias.detach().double()
    q0, e1 = W1[:, 256:320], W1[:, 320:384]
    (Wq, bq), (Wr, br) = composed_embedding(emb, q0, e1, b1)
    x = torch.randn(53, emb[0][0].shape[1], dtype=torch.float64, generator=torch.Generator().manual_seed(J))
    h = x
    for W, b, relu in emb[:3]:
        h = torch.relu(h @ W.T + b) if relu else h @ W.T + b
    e_init = h @ emb[3][0].T + emb[3][1]
    Q0 = e_init @ q0.T + b1
    R0 = Q0 + e_init @ e1.T
    assert torch.allclose(h @ Wq.T + bq, Q0, rtol=0, atol=1e-12)
    assert torch.allclose(h @ Wr.T + br, R0, rtol=0, atol=1e-12)
    # shapes outside the published embedding compose nothing
    assert composed_embedding(emb[:3], q0, e1, b1) is None
