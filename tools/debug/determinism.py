"""Run one golden MPN case R times in this process; report the max error vs the golden and whether the R runs are
bit-identical (a race shows up as run-to-run differences). usage: determinism.py <golden> <precision> [R]"""
import sys

import torch

sys.path.insert(0, ".")
import pemp_amd  # noqa: E402
from pemp_amd import synthetic as syn  # noqa: E402
from tests import golden_util as gu  # noqa: E402

name, prec = sys.argv[1], sys.argv[2]
R = int(sys.argv[3]) if len(sys.argv) > 3 else 10
DEV = torch.device("cuda:0")
meta, a = gu.load(name)
m = pemp_amd.get_mpn_model(gu.mpn_config(meta))
m.load_state_dict(syn.closed_form_state_dict(m, meta["salt"], meta.get("attn_gain", 1.0), meta.get("weight_gain", 1.0)))
m.precision = prec
m = m.eval().to(DEV)
inp = [torch.from_numpy(a[k]).to(DEV) for k in ("x", "edge_attr", "edge_index", "node_types")]
ref = torch.from_numpy(a["edge_logits"])
outs = []
for _ in range(R):
    with torch.no_grad():
        pe, pn, pc, _ = m(inp[0], inp[1], inp[2], node_types=inp[3])
    torch.cuda.synchronize()
    outs.append(torch.cat([pe[-1].flatten(), pn[-1].flatten(), pc[-1].flatten()]).cpu())
errs = [(o[:ref.numel()] - ref).abs().max().item() for o in outs]
same = all(torch.equal(o, outs[0]) for o in outs)
ndiff = max(int((o != outs[0]).sum()) for o in outs)
print(f"{name} {prec}: max err {max(errs):.3g} min err {min(errs):.3g} bit-identical runs: {same} (max differing {ndiff})")
