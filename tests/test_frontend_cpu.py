"""The projected test front-end, CPU side: the oracle's explicit fp32 restatement
(oracle/restate.project_frontend) against the reference's own torch ops (ProjectedHeatmaps.materialize:
interpolate / flip / index / average, PoseEstimation.py:329-452, multi_scales_testing.py:144-195).
Tolerance 2e-6 absolute on maps in [0, 1.5): torch's CPU upsample may contract a product into an FMA."""
import numpy as np
import pytest
import torch

from oracle import restate
from pemp_amd.frontend import ProjectedHeatmaps
from pemp_amd import synthetic as syn

COCO_FLIP = [0, 2, 1, 4, 3, 6, 5, 8, 7, 10, 9, 12, 11, 14, 13, 16, 15]


def make_outputs(seed, B, J, sizes, flip):
    outs, flips = [], []
    for k, (h, w) in enumerate(sizes):
        hm = syn.make_heatmaps(seed + k, B, J, h, w, 3, sigma=1.0, margin=2)
        tg = syn.closed_form((B, J, h, w), 0.5 + 0.1 * k)
        outs.append(torch.from_numpy(np.concatenate([hm, tg], 1)))
        if flip:
            hm2 = syn.make_heatmaps(seed + 50 + k, B, J, h, w, 3, sigma=1.0, margin=2)
            tg2 = syn.closed_form((B, J, h, w), 0.7 + 0.1 * k)
            flips.append(torch.from_numpy(np.concatenate([hm2, tg2], 1)))
    return outs, (flips if flip else None)


@pytest.mark.parametrize("sizes,size,flip", [([(40, 40)], (80, 80), True), ([(45, 35)], (80, 96), True),
                                             ([(40, 40), (20, 20)], (80, 80), True), ([(40, 40)], (80, 80), False)])
def test_restatement_matches_torch_ops(sizes, size, flip):
    B, J = 2, 17
    outs, flips = make_outputs(3, B, J, sizes, flip)
    ph = ProjectedHeatmaps(outs, size, J, flips, COCO_FLIP if flip else None)
    ref_s, ref_t = ph.materialize()
    s, t = restate.project_frontend(outs, flips, size, J, COCO_FLIP if flip else None)
    assert s.shape == ref_s.shape and t.shape == ref_t.shape
    assert (s - ref_s).abs().max().item() <= 2e-6
    assert (t - ref_t).abs().max().item() <= 2e-6


def test_projected_heatmaps_validation():
    outs, flips = make_outputs(1, 1, 17, [(20, 20)], True)
    with pytest.raises(ValueError):
        ProjectedHeatmaps(outs, (40, 40), 17, flips, [0] * 17)          # not a permutation
    with pytest.raises(ValueError):
        ProjectedHeatmaps(outs, (40, 40), 17, flips[:0] + [flips[0][:, :, :10]])
    with pytest.raises(ValueError):                                     # neither J nor 2J channels
        ProjectedHeatmaps([o[:, :20] for o in outs], (40, 40), 17)
    with pytest.raises(NotImplementedError):                            # shared tag channel (TAG_PER_JOINT False)
        ProjectedHeatmaps(outs, (40, 40), 17, flips, COCO_FLIP, tag_per_joint=False)
    assert not ProjectedHeatmaps([o[:, :17] for o in outs], (40, 40), 17).has_tags


def test_projected_maps_gather_conv_host():
    """ProjectedMaps(gather=feature_gather): materialize() is the reference's conv + interpolate per scale
    (PoseEstimation.py:341, 426-452); the C-ABI transpose is [Cin, k, k, Cout]; unsupported convs are
    refused loudly."""
    import pytest
    from pemp_amd.frontend import ProjectedMaps
    g = torch.Generator().manual_seed(3)
    raw = [torch.randn(2, 8, 10, 12, generator=g), torch.randn(2, 8, 5, 6, generator=g)]
    conv = torch.nn.Conv2d(8, 16, 3, 1, 1)
    pm = ProjectedMaps(raw, (20, 24), gather=conv)
    assert pm.shape == torch.Size([2, 16, 20, 24])
    with torch.no_grad():
        want = sum(torch.nn.functional.interpolate(conv(m), size=(20, 24), mode="bilinear", align_corners=False)
                   for m in raw) / 2.0
    assert torch.equal(pm.materialize(), want)
    wt, b, k, pad = pm.conv_params()
    assert (k, pad) == (3, 1) and torch.equal(wt, conv.weight.detach().permute(1, 2, 3, 0))
    assert torch.equal(b, conv.bias.detach())
    with pytest.raises(NotImplementedError):
        ProjectedMaps(raw, (20, 24), gather=torch.nn.Conv2d(8, 16, 3, 2, 1))
    with pytest.raises(ValueError):
        ProjectedMaps(raw, (20, 24), gather=torch.nn.Conv2d(4, 16, 3, 1, 1))
