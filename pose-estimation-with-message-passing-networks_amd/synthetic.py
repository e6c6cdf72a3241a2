"""Seeded synthetic inputs for the keypoint-graph hot path.

Heatmaps follow the reference's ``HeatmapGenerator`` (``src/data/utils.py:30-65``): a Gaussian
patch of size 6σ+3 centred at 3σ+1, merged with ``np.maximum``. Each planted joint gets a
distinct amplitude so the detector's top-k has no boundary ties. Features, tags and MLP weights
are closed-form hashes, so fixtures need not store them.
"""
import math

import numpy as np


def gaussian_patch(sigma: float) -> np.ndarray:
    size = 6 * sigma + 3
    x = np.arange(0, size, 1, float)
    y = x[:, np.newaxis]
    x0 = y0 = 3 * sigma + 1
    return np.exp(-((x - x0) ** 2 + (y - y0) ** 2) / (2 * sigma ** 2))


def plant_peaks(hms: np.ndarray, joints: np.ndarray, amps: np.ndarray, sigma: float) -> None:
    """hms [J,H,W]; joints [P,J,2] integer (x,y); amps [P,J]. In-place np.maximum merge."""
    J, H, W = hms.shape
    g = gaussian_patch(sigma)
    r = int(3 * sigma + 1)
    for p in range(joints.shape[0]):
        for j in range(J):
            x, y = int(joints[p, j, 0]), int(joints[p, j, 1])
            x0, y0 = x - r, y - r
            x1, y1 = x0 + g.shape[1], y0 + g.shape[0]
            cx0, cy0 = max(0, x0), max(0, y0)
            cx1, cy1 = min(W, x1), min(H, y1)
            if cx0 >= cx1 or cy0 >= cy1:
                continue
            patch = g[cy0 - y0:cy1 - y0, cx0 - x0:cx1 - x0] * amps[p, j]
            np.maximum(hms[j, cy0:cy1, cx0:cx1], patch.astype(np.float32), out=hms[j, cy0:cy1, cx0:cx1])


def make_heatmaps(seed: int, B: int, J: int, H: int, W: int, persons: int, sigma: float = 2.0,
                  variant: str = "clean", margin: int = 8) -> np.ndarray:
    """[B,J,H,W] float32. variant: clean | noisy (+U[0,0.05) background) | realistic (½-res + bilinear ×2)."""
    rng = np.random.default_rng(seed)
    out = np.zeros((B, J, H, W), np.float32)
    for b in range(B):
        if variant == "realistic":
            h2, w2 = H // 2, W // 2
            hm = np.zeros((J, h2, w2), np.float32)
            joints = np.stack([rng.integers(margin // 2, w2 - margin // 2, (persons, J)),
                               rng.integers(margin // 2, h2 - margin // 2, (persons, J))], -1)
            amps = rng.permutation(np.linspace(0.15, 1.0, persons * J, endpoint=False)).reshape(persons, J)
            plant_peaks(hm, joints, amps, sigma / 2)
            out[b] = bilinear_up2(hm, H, W)
        else:
            joints = np.stack([rng.integers(margin, W - margin, (persons, J)),
                               rng.integers(margin, H - margin, (persons, J))], -1)
            amps = 0.15 + 0.85 * rng.permutation(persons * J).reshape(persons, J) / max(1, persons * J)
            amps = amps + rng.uniform(0, 0.5 / max(1, persons * J), amps.shape)
            plant_peaks(out[b], joints, amps.astype(np.float64), sigma)
            if variant == "noisy":
                out[b] += rng.uniform(0.0, 0.05, (J, H, W)).astype(np.float32)
    return out


def bilinear_up2(hm: np.ndarray, H: int, W: int) -> np.ndarray:
    """Bilinear resize, align_corners=False (as ``interpolate`` in PoseEstimation.py:422-431)."""
    J, h, w = hm.shape

    def coords(n_out, n_in):
        s = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
        s = np.clip(s, 0, None)
        i0 = np.minimum(np.floor(s).astype(np.int64), n_in - 1)
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, (s - i0).astype(np.float32)

    y0, y1, fy = coords(H, h)
    x0, x1, fx = coords(W, w)
    top = hm[:, y0][:, :, x0] * (1 - fx) + hm[:, y0][:, :, x1] * fx
    bot = hm[:, y1][:, :, x0] * (1 - fx) + hm[:, y1][:, :, x1] * fx
    return (top * (1 - fy)[None, :, None] + bot * fy[None, :, None]).astype(np.float32)


def closed_form(shape, salt: float) -> np.ndarray:
    """Deterministic hash in [-1, 1): frac(sin(dot(idx, k) + salt) * 43758.5453) * 2 - 1."""
    idx = np.indices(shape, dtype=np.float64)
    ks = [12.9898, 78.233, 37.719, 4.581, 91.17, 23.11][:len(shape)]
    acc = np.full(shape, salt, np.float64)
    for d, k in enumerate(ks):
        acc += idx[d] * k
    v = np.sin(acc) * 43758.5453
    return ((v - np.floor(v)) * 2.0 - 1.0).astype(np.float32)


def closed_form_state_dict(module_or_sd, salt: float = 0.0, attn_gain: float = 1.0, weight_gain: float = 1.0):
    """Deterministic weights for every tensor of a state_dict (BN stats kept non-trivial).
    `attn_gain` scales the attention net so its softmax is far from uniform (a fixture then tells
    which attention row was used). `weight_gain` scales every Linear weight: 2.0 gives the logit
    magnitudes of a trained checkpoint (|logit| up to ~20-55 on a C2-shaped graph, vs ~0.1 at 1.0)."""
    import torch
    sd = module_or_sd.state_dict() if hasattr(module_or_sd, "state_dict") else module_or_sd
    out = {}
    for n, (k, v) in enumerate(sd.items()):
        if v.dtype in (torch.int64, torch.int32):
            out[k] = v.clone()
            continue
        h = torch.from_numpy(closed_form(tuple(v.shape), salt + 1.7 * n))
        if k.endswith("running_var"):
            t = 0.6 + 0.4 * (h + 1.0)
        elif k.endswith("running_mean"):
            t = 0.1 * h
        elif k.endswith(".weight") and v.dim() == 1:   # BN gamma
            t = 0.8 + 0.2 * h
        elif v.dim() == 2:
            t = h * (1.6 / math.sqrt(v.shape[1])) * weight_gain
        else:
            t = 0.05 * h
        if ".attn_net." in k:
            t = t * attn_gain
        out[k] = t.to(v.dtype)
    return out
