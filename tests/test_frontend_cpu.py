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


def make_stages(seed, B, J, half_sizes, flip):
    """HigherHRNet-shaped per-stage outputs per scale: stage 0 at 1/4 resolution with 2J channels (heatmaps + per-joint
    tags), stage 1 at 1/2 resolution with J heatmap channels."""
    g = torch.Generator().manual_seed(seed)

    def pair(h, w):
        s0 = torch.cat([torch.rand(B, J, h // 2, w // 2, generator=g), torch.randn(B, J, h // 2, w // 2, generator=g)], 1)
        return s0, torch.rand(B, J, h, w, generator=g)

    outs = [pair(h, w) for (h, w) in half_sizes]
    flips = [pair(h, w) for (h, w) in half_sizes] if flip else None
    return outs, flips


def reference_multi_stage(stages, flip_stages, size, J, fi, tag_scale):
    """_get_multi_stage_outputs + aggregate_results_mpn + the scale division (PoseEstimation.py:338-412, 187-229,
    multi_scales_testing.py:144-195) restated with the reference's own torch ops, TEST.PROJECT2IMAGE."""
    up = lambda t, hw: torch.nn.functional.interpolate(t, size=hw, mode="bilinear", align_corners=False)  # noqa: E731
    final, tags_list = None, []
    for k, (s0, s1) in enumerate(stages):
        hw = (s1.size(2), s1.size(3))
        heat, tags = 0, []
        heat += up(s0, hw)[:, :J]
        tags.append(up(s0, hw)[:, J:])
        heat += s1[:, :J]
        heatmaps = [heat / 2]
        if flip_stages is not None:
            f0, f1 = flip_stages[k]
            hf = 0
            o = torch.flip(up(f0, hw), [3])
            hf += o[:, :J][:, fi]
            tags.append(o[:, J:][:, fi])
            hf += torch.flip(f1, [3])[:, :J][:, fi]
            heatmaps.append(hf / 2)
        heatmaps = [up(h, size) for h in heatmaps]
        tags = [up(t, size) for t in tags]
        if k == tag_scale:
            tags_list += [t.unsqueeze(4) for t in tags]
        avg = (heatmaps[0] + heatmaps[1]) / 2.0 if flip_stages is not None else heatmaps[0]
        final = avg if final is None else final + avg
    return final / float(len(stages)), torch.cat(tags_list, dim=4)


@pytest.mark.parametrize("flip", [True, False])
def test_stage_merge_restatement(flip):
    """ProjectedHeatmaps.from_stages' merge (pemp_stage_merge; its oracle restate.stage_merge) + the projection equal
    the reference's multi-stage, multi-scale test path run with its own torch ops: the oracle's fp32 merge within 2e-6
    of the torch ops (FMA contraction in torch's CPU upsample); the torch-op merge fed to the projection equals the
    reference path exactly (the flipped pass merged in the network's orientation, then flipped by the projection)."""
    B, J, fi = 2, 17, COCO_FLIP
    stages, flips = make_stages(4, B, J, [(40, 48), (20, 24)], flip)
    size = (80, 96)
    ref_s, ref_t = reference_multi_stage(stages, flips, size, J, fi, tag_scale=0)
    merged = [ProjectedHeatmaps.merge_stages_reference(a, b, J) for a, b in stages]
    mflip = None if flips is None else [ProjectedHeatmaps.merge_stages_reference(a, b, J) for a, b in flips]
    for (a, b), m in zip(stages + (flips or []), merged + (mflip or [])):
        assert (restate.stage_merge(a, b, J) - m).abs().max().item() <= 2e-6
    ph = ProjectedHeatmaps(merged, size, J, mflip, fi if flip else None)
    s, t = ph.materialize()
    assert torch.equal(s, ref_s) and torch.equal(t, ref_t)


def test_backbone_leg_model_is_higherhrnet_w48():
    """bench.py's backbone leg times tools/hrnet_w48.py: the HigherHRNet-w48 compute graph of model_58_4_4.yaml (63.8 M
    parameters, 2 x 17 heatmap + tag channels at 1/4 resolution, 17 heatmaps and the 48-channel features at 1/2)."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from hrnet_w48 import HigherHRNetW48
    m = HigherHRNetW48(17).eval()
    assert abs(sum(p.numel() for p in m.parameters()) / 1e6 - 63.83) < 0.01
    with torch.no_grad():
        (y0, y1), f = m(torch.zeros(1, 3, 64, 96))
    assert y0.shape == (1, 34, 16, 24) and y1.shape == (1, 17, 32, 48) and f.shape == (1, 48, 32, 48)


def _taps_f32(dst, out_size, in_size):
    """csrc/detect.hip proj_taps in numpy fp32 (one rounding per operation): (i0, i1, l0, l1)."""
    f = np.float32
    scale = f(in_size) / f(out_size)
    src = f(f(scale * f(f(dst) + f(0.5))) - f(0.5))
    src = max(src, f(0.0))
    i0 = int(src)
    i1 = i0 + (1 if i0 < in_size - 1 else 0)
    l1 = min(max(f(src - f(i0)), f(0.0)), f(1.0))
    return i0, i1, f(f(1.0) - l1), l1


def _x2_row(i, P):
    d = i - P
    return d // 2 - 1 if d % 2 == 0 else (d - 1) // 2


@pytest.mark.parametrize("P", [0, 1, 2, 3, 4])
def test_exact_2x_loader_taps(P):
    """proj_x2_first (the projected NMS's register-only loader for an exact 2x upsampling) replaces proj_taps by
    constants: for every interior band (y0 - P >= 1, y0 + SR - 1 + P <= H - 3) of every height, output row i reads
    rows y0 / 2 + x2_row(i) and the next one with weights (0.25, 0.75) for an even y0 - P + i, (0.75, 0.25) for an
    odd one -- exactly what proj_taps computes, so its values are bitwise those of the staged loader."""
    SR = 16
    for h in list(range(9, 80)) + [160, 320, 321, 512]:
        H = 2 * h
        for y0 in range(0, H, SR):
            if not (y0 - P >= 1 and y0 + SR - 1 + P <= H - 3):
                continue
            for i in range(SR + 2 * P):
                Y = y0 - P + i
                i0, i1, l0, l1 = _taps_f32(Y, H, h)
                even = (i - P) % 2 == 0
                assert i0 == y0 // 2 + _x2_row(i, P) and i1 == i0 + 1, (h, y0, i)
                assert (l0, l1) == ((0.25, 0.75) if even else (0.75, 0.25)), (h, y0, i)
