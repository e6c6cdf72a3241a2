"""Fixture helpers shared by CPU and GPU parity tests."""
import hashlib
import json
import os

import numpy as np
import torch

import pemp_amd.config as pcfg
from pemp_amd import synthetic as syn

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FEATURE_SALT, TAG_SALT = 0.25, 0.75   # must match oracle/gen_golden.py


def names(prefix):
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith(prefix) and f.endswith(".npz"))


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return meta, {k: z[k] for k in z.files if k != "meta"}


def sha(t: torch.Tensor) -> str:
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def gc_inputs(meta, arrays):
    B, J, H, W = meta["B"], meta["J"], meta["H"], meta["W"]
    hm = torch.from_numpy(arrays["scoremaps"])
    feats = torch.from_numpy(syn.closed_form((B, meta["C"], H, W), FEATURE_SALT))
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, meta["F"]), TAG_SALT))
    masks = torch.from_numpy(arrays["masks"]) if "masks" in arrays else None
    return hm, feats, tags, masks


def gc_config(meta):
    g = pcfg.inference_gc_config(meta["graph"], meta["pool"], meta["mask_crowds"])
    g.DETECT_THRESHOLD = meta["thr"]
    if "features" in meta:
        g.EDGE_FEATURES_TO_USE = list(meta["features"])
    return g


def mpn_config(meta):
    c = pcfg.published_mpn_config(meta["J"], meta["steps"], meta["variant"])
    if meta.get("aggr_sub") is not None:
        c.AGGR_SUB = meta["aggr_sub"]
        c.AGGR = meta["aggr"]
    if meta.get("update_mlp"):
        c.USE_NODE_UPDATE_MLP = True
    if meta.get("edge_in"):
        c.EDGE_INPUT_DIM = meta["edge_in"]
    if meta.get("update_type"):
        c.UPDATE_TYPE = meta["update_type"]
    if meta.get("edge_mlp"):
        c.EDGE_MLP = meta["edge_mlp"]
    if meta.get("late_fusion"):
        c.LATE_FUSION_POS = True
        c.EDGE_EMB.BN = True
    if meta.get("node_summary"):
        c.NODE_TYPE_SUMMARY = meta["node_summary"]
    return c
