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
