"""Why does capacity mode not engage? Replays test_capacity_mode_mpn's first steps with the internals printed."""
import torch
import pemp_amd
from pemp_amd import config as pcfg, synthetic as syn
from pemp_amd.graph_constructor import NaiveGraphConstructor
from pemp_amd.mpn import model as mm

DEV = torch.device("cuda:0")
B, J, H, W = 2, 17, 96, 104
gc = pcfg.inference_gc_config("fully", 5, False)
model = pemp_amd.get_mpn_model(pcfg.published_mpn_config(J, 3, "attn"))
model.load_state_dict(syn.closed_form_state_dict(model, 1.25, 1.0, 1.0))
model = model.eval().to(DEV)
feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25)).to(DEV)
orig_fc, orig_take = mm.NodeClassificationMPNSimple._forward_cap, mm.NodeClassificationMPNSimple._take_cap


def fc(self, *a):
    r = orig_fc(self, *a)
    print("  _forward_cap ->", None if r is None else "pending", "n_cap/e_cap", a[3], a[4], flush=True)
    return r


def take(self, x, ea, ei, nt):
    tag = getattr(ei, "_pemp_mpn", None)
    r = orig_take(self, x, ea, ei, nt)
    print("  _take_cap tag", tag is not None, "->", r is not None, flush=True)
    return r


mm.NodeClassificationMPNSimple._forward_cap = fc
mm.NodeClassificationMPNSimple._take_cap = take
pemp_amd.bind_mpn(model)
for seed, persons in ((1, 3), (2, 2), (3, 3)):
    print("seed", seed, "hint", dict(NaiveGraphConstructor._graph_hint), flush=True)
    hm = torch.from_numpy(syn.make_heatmaps(seed, B, J, H, W, persons, margin=4)).to(DEV)
    out = pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=None, joints_gt=None,
                                         factor_list=None, masks=None, device=DEV, testing=True, heatmaps=None,
                                         num_joints=J).construct_graph()
    print("  N", out[0].shape[0], "E", out[2].shape[1], flush=True)
    with torch.no_grad():
        model(out[0], out[1], out[2], node_types=out[7][:, 2])
    torch.cuda.synchronize()
