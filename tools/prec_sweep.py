"""GPU diagnostic: MPN logit error of each precision against the fp64 oracle as the weights grow
toward trained-checkpoint logit magnitudes (every Linear weight x gain). Prints one line per case."""
import sys

import torch

sys.path.insert(0, ".")
import pemp_amd  # noqa: E402
from oracle import restate  # noqa: E402
from pemp_amd import config as pcfg, synthetic as syn  # noqa: E402

DEV = torch.device("cuda:0")
precs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["fp32", "bf16x3"]
hm = torch.from_numpy(syn.make_heatmaps(5, 1, 17, 160, 160, 9))
feats = torch.from_numpy(syn.closed_form((1, 128, 160, 160), 0.25))
g = restate.construct_graph(hm, feats, torch.zeros(1, 17, 160, 160), None, pcfg.inference_gc_config("fully", 5, False), 17)
x, ea, ei, t = g[0], g[1], g[2], g[7][:, 2]
for variant in ("attn", "max"):
    cfg = pcfg.published_mpn_config(17, 3, variant)
    for gain in (1.0, 1.5, 2.0):
        m = pemp_amd.get_mpn_model(cfg)
        sd = syn.closed_form_state_dict(m, 9.5)
        sd = {k: (v * gain if v.dim() == 2 else v) for k, v in sd.items()}
        m.load_state_dict(sd)
        m.eval().to(DEV)
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        r = restate.mpn_forward(sd64, cfg, x.double(), ea.double(), ei, t)
        for prec in precs:
            m.precision = prec
            with torch.no_grad():
                o = m(x.to(DEV), ea.to(DEV), ei.to(DEV), node_types=t.to(DEV))
            torch.cuda.synchronize()
            errs = [float((a[-1].cpu().double() - b[-1]).abs().max()) for a, b in zip(o[:3], r[:3])]
            mags = [float(b[-1].abs().max()) for b in r[:3]]
            print(f"{variant} gain={gain} {prec}: err edge/node/class={errs[0]:.3g}/{errs[1]:.3g}/{errs[2]:.3g} "
                  f"max|logit|={mags[0]:.3g}/{mags[1]:.3g}/{mags[2]:.3g}", flush=True)
