"""Diagnostic: GPU edge_attr vs a stored golden (full fixture), per column."""
import sys
import numpy as np
import torch
sys.path.insert(0, "/root/repo")
import pemp_amd
from tests import golden_util as gu

name = sys.argv[1] if len(sys.argv) > 1 else "gc_ae_pos_conn_f2"
meta, a = gu.load(name)
hm, feats, tags, masks = gu.gc_inputs(meta, a)
dev = torch.device("cuda:0")
out = pemp_amd.get_graph_constructor(gu.gc_config(meta), scoremaps=hm.to(dev), tagmaps=tags.to(dev),
                                     features=feats.to(dev), joints_gt=None, factor_list=None, masks=None,
                                     device=dev, testing=True, heatmaps=None, num_joints=meta["J"]).construct_graph()
ea = out[1].cpu().numpy()
ref = a["edge_attr"]
print(ea.shape, ref.shape)
bad = np.nonzero(ea != ref)
cols = np.unique(bad[1])
print("mismatch cols", cols, "count", len(bad[0]))
for r, c in list(zip(*bad))[:10]:
    print(r, c, repr(ea[r, c]), repr(ref[r, c]), ea[r, c] - ref[r, c])
