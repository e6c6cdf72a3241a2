"""Drop-in ``NodeClassificationMPNSimple`` (``NodeClassificationMPNSimple.py:23-97``).

The module tree mirrors the reference's so that ``state_dict`` keys (and their order) are
identical and reference checkpoints load unchanged:
``mpn_node_cls.{mlp_edge,mlp_node,update_mlp,attn_net}``, ``edge_embedding``, ``node_embedding``,
``edge_classification``, ``node_classification``, ``classification``. The parameters are plain
containers; ``forward`` folds them once per parameter version (eval-mode BatchNorm into the next
Linear) and runs the whole network in ``pemp_mpn_forward`` (libpemp.so). Inference only.
"""
import ctypes
import itertools
import os
import warnings

import numpy as np
import torch
import torch.nn as nn

from .. import _lib
from .fold import F16RangeError, fold_weights
from .edge_type import TypeAwareEdgeUpdate
from .hierarch import HierarchUpdateCnn, HierarchUpdateMlp

_VALIDATE = os.environ.get("PEMP_VALIDATE", "0") not in ("", "0")   # read once at import
# PEMP_DEBUG_SYNC=1 (the library's synchronising debug mode) also reads the contract flags of every call
_DEBUG_SYNC = os.environ.get("PEMP_DEBUG_SYNC", "0") not in ("", "0")
_FULLY_OFF = os.environ.get("PEMP_NO_FULLY_PREPARE", "0") not in ("", "0")   # force the sorting prepare
_SYM_OFF = os.environ.get("PEMP_NO_SYM_PREPARE", "0") not in ("", "0")       # (for symmetric graphs too)
_KNN_OFF = os.environ.get("PEMP_NO_KNN_PREPARE", "0") not in ("", "0")      # knn graphs: the symmetric prepare
_EDGE_LIMIT = (1 << 23) - 1    # pemp_mpn_forward: E < 2^23 and T N < 2^23 per call (32-bit byte offsets)

AGGR_CODES = {"attn": 0, "add": 1, "sum": 1, "mean": 2, "max": 3}
PRECISIONS = {"fp32": 0, "bf16x3": 1, "f16x3": 2}


def default_precision(aggr_code):
    """Arithmetic of the per-edge GEMMs and the node table. ``PEMP_PRECISION`` (fp32 | bf16x3 | f16x3)
    overrides. The default is f16x3 for every aggregation: f16 hi / scaled-lo split operands on the f16
    MFMA, ~2^-22 relative error per product, which holds the 1e-4 logit bar at trained-checkpoint
    magnitudes (|logit| ~ 50, tests/test_gpu_mpn.py::test_trained_scale) where bf16x3 (~2^-16) does
    not, at the MFMA cost of bf16x3 (exact fp32 MFMA takes ~5x the matrix time). bf16x3 stays an
    opt-in for small-magnitude models."""
    env = os.environ.get("PEMP_PRECISION", "")
    if env:
        if env not in PRECISIONS:
            raise ValueError(f"PEMP_PRECISION={env!r}: expected one of {sorted(PRECISIONS)}")
        return env
    return "f16x3"
TYPE_LUTS = {"left_right": [0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8],
             "per_body_part": [0, 0, 0, 0, 0, 1, 1, 2, 3, 2, 3, 4, 5, 4, 5, 4, 5]}


def _rows(logits, n):
    """[logits[r].view(L, 1).squeeze() for r in range(n)] (the per-step logit lists of NodeClassificationMPNSimple.py:
    81-97) for a [>= n, L] buffer: one unbind instead of three tensor ops per row (host time of the serving loop)."""
    L = logits.shape[1]
    if L != 1:   # squeeze of [L, 1] keeps [L]: the unbound row is the same view
        return list((logits if logits.shape[0] == n else logits[:n]).unbind(0))
    return [logits[r].view(L, 1).squeeze() for r in range(n)]


def _make_mlp(input_dim, hidden_dims, bn=False, end_with_relu=False):
    """Layer indices as ``layers.py:8-29``: Linear, then (ReLU, [BN]) between Linears."""
    mods = [nn.Linear(input_dim, hidden_dims[0])]
    last = len(hidden_dims) - 1
    if last > 0:
        mods.append(nn.ReLU(inplace=True))
        if bn:
            mods.append(nn.BatchNorm1d(hidden_dims[0]))
    for i in range(1, last + 1):
        mods.append(nn.Linear(hidden_dims[i - 1], hidden_dims[i]))
        if i != last:
            mods.append(nn.ReLU(inplace=True))
            if bn:
                mods.append(nn.BatchNorm1d(hidden_dims[i]))
    if end_with_relu:
        mods.append(nn.ReLU(inplace=True))
        if bn:
            mods.append(nn.BatchNorm1d(hidden_dims[-1]))
    return nn.Sequential(*mods)


class LateFusionEdgeMLP(nn.Module):
    """``NodeClassificationMPNSimple.py:7-21`` (LATE_FUSION_POS): separate MLPs on [dx, dy] and on the
    17 connection columns, then out(ReLU(cat)). Parameters only; folded block-diagonally by fold.py."""

    def __init__(self, config):
        super().__init__()
        single = [size // 2 for size in config.EDGE_EMB.OUTPUT_SIZES[:-1]]
        self.pos_mlp = _make_mlp(2, single, bn=config.EDGE_EMB.BN, end_with_relu=config.EDGE_EMB.END_WITH_RELU)
        self.edge_mlp = _make_mlp(17, single, bn=config.EDGE_EMB.BN, end_with_relu=config.EDGE_EMB.END_WITH_RELU)
        self.out = nn.Linear(single[-1] * 2, config.EDGE_EMB.OUTPUT_SIZES[-1])


class TypeAwareNodeUpdate(nn.Module):
    """``layers.py:260-274``: 17 Linear+ReLU message MLPs selected by the source node type."""

    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.mlp = nn.ModuleList([nn.Sequential(nn.Linear(input_dim, output_dim), nn.ReLU(inplace=True))
                                  for _ in range(17)])
        self.output_dim = output_dim


class TypeAwareMPNLayer(nn.Module):
    """``layers.py:157-258`` (edge MLP agnostic; update ``mlp``, ``hierarch_mlp`` or ``hierarch_cnn``)."""

    def __init__(self, node_dim, edge_dim, edge_hidden, aggr, skip=False, edge_mlp="agnostic", num_types=17,
                 aggr_sub=None, update_type="mlp"):
        super().__init__()
        if edge_mlp not in ("agnostic", "per_type"):
            raise NotImplementedError(f"EDGE_MLP={edge_mlp}")
        if update_type not in ("mlp", "hierarch_mlp", "hierarch_cnn"):
            raise NotImplementedError(f"UPDATE_TYPE={update_type}")
        if update_type == "hierarch_cnn" and num_types != 17:
            raise NotImplementedError("UPDATE_TYPE=hierarch_cnn indexes types up to 16 (layers.py:148)")
        nf = 2 if skip else 1
        self.aggr, self.aggr_sub, self.num_types, self.skip = aggr, aggr_sub, num_types, skip
        self.edge_mlp = edge_mlp
        if edge_mlp == "agnostic":
            self.mlp_edge = nn.Sequential(nn.Linear(node_dim * 2 * nf + edge_dim * nf, edge_hidden),
                                          nn.ReLU(inplace=True), nn.Linear(edge_hidden, edge_dim), nn.ReLU(inplace=True))
        else:   # layers.py:177-179 (edge_dim * node_factor, as the reference writes it)
            self.mlp_edge = TypeAwareEdgeUpdate(node_dim * nf, edge_dim * nf, edge_hidden, num_types)
        self.mlp_node = TypeAwareNodeUpdate(node_dim * nf + edge_dim, node_dim)
        self.update_type = update_type
        if update_type == "mlp":
            self.update_mlp = nn.Sequential(nn.Linear(node_dim * num_types, node_dim), nn.ReLU(inplace=True))
        elif update_type == "hierarch_mlp":
            self.update_mlp = HierarchUpdateMlp(node_dim, num_types)
        else:
            self.update_mlp = HierarchUpdateCnn(node_dim)
        if aggr_sub == "node_edge_attn":
            self.attn_net = nn.Sequential(nn.Linear(edge_dim, 1))
        elif aggr_sub == "node_edge_attn_per_type":
            # one attention row per source type (layers.py:199-201, 245-246): always 17 outputs
            self.attn_net = nn.Sequential(nn.Linear(edge_dim, 17))
        else:
            self.attn_net = None


class MPLayer(nn.Module):
    """``layers.py:32-86`` (edge MLP agnostic)."""

    def __init__(self, node_dim, edge_dim, edge_hidden, aggr, use_node_update_mlp, skip=False, edge_mlp="agnostic"):
        super().__init__()
        if edge_mlp == "per_type":   # the reference omits TypeAwareEdgeUpdate's num_joints here (layers.py:52-53)
            raise NotImplementedError("EDGE_MLP=per_type with AGGR_TYPE agnostic: the reference's MPLayer "
                                      "raises TypeError constructing it")
        if edge_mlp != "agnostic":
            raise NotImplementedError(f"EDGE_MLP={edge_mlp}")
        nf = 2 if skip else 1
        self.aggr, self.skip = aggr, skip
        self.mlp_edge = nn.Sequential(nn.Linear(node_dim * 2 * nf + edge_dim * nf, edge_hidden), nn.ReLU(inplace=True),
                                      nn.Linear(edge_hidden, edge_dim), nn.ReLU(inplace=True))
        self.mlp_node = nn.Sequential(nn.Linear(node_dim * nf + edge_dim, node_dim), nn.ReLU(inplace=True))
        self.update_mlp = (nn.Sequential(nn.Linear(node_dim, node_dim), nn.ReLU()) if use_node_update_mlp else None)


class NodeClassificationMPNSimple(nn.Module):
    """``NodeClassificationMPNSimple.py:23-97``."""

    def __init__(self, config):
        super().__init__()
        self.use_skip_connections = config.SKIP
        self.node_summary = config.NODE_TYPE_SUMMARY
        for k, v in (("NODE_FEATURE_DIM", 64), ("EDGE_FEATURE_DIM", 64), ("EDGE_FEATURE_HIDDEN", 64)):
            if config[k] != v:
                raise NotImplementedError(f"{k}={config[k]}: the HIP kernels are built for width 64")
        if config.AGGR_TYPE == "agnostic":
            self.mpn_node_cls = MPLayer(64, 64, 64, aggr=config.AGGR, skip=config.SKIP,
                                        use_node_update_mlp=config.USE_NODE_UPDATE_MLP, edge_mlp=config.EDGE_MLP)
            self.num_types = 1
        elif config.AGGR_TYPE == "per_type":
            self.num_types = {"per_body_part": 6, "not": config.NUM_JOINTS, "left_right": 9}[self.node_summary]
            self.mpn_node_cls = TypeAwareMPNLayer(64, 64, 64, aggr=config.AGGR, skip=config.SKIP,
                                                  edge_mlp=config.EDGE_MLP, num_types=self.num_types,
                                                  aggr_sub=config.AGGR_SUB, update_type=config.UPDATE_TYPE)
        else:
            raise NotImplementedError(f"AGGR_TYPE={config.AGGR_TYPE}")
        if config.get("LATE_FUSION_POS", False):
            if config.EDGE_INPUT_DIM != 19:   # LateFusionEdgeMLP slices [dx, dy | 17 one-hot columns]
                raise NotImplementedError(f"LATE_FUSION_POS needs EDGE_INPUT_DIM 19 (got {config.EDGE_INPUT_DIM})")
            self.edge_embedding = LateFusionEdgeMLP(config)
        else:
            self.edge_embedding = _make_mlp(config.EDGE_INPUT_DIM, config.EDGE_EMB.OUTPUT_SIZES, bn=config.EDGE_EMB.BN,
                                            end_with_relu=config.EDGE_EMB.END_WITH_RELU)
        self.node_embedding = _make_mlp(config.NODE_INPUT_DIM, config.NODE_EMB.OUTPUT_SIZES, bn=config.NODE_EMB.BN,
                                        end_with_relu=config.NODE_EMB.END_WITH_RELU)
        self.edge_classification = _make_mlp(64, config.EDGE_CLASS.OUTPUT_SIZES, bn=config.BN)
        self.node_classification = _make_mlp(64, config.NODE_CLASS.OUTPUT_SIZES, bn=config.BN)
        self.classification = _make_mlp(64, config.CLASS.OUTPUT_SIZES, bn=config.BN)
        self.edge_steps = config.STEPS
        self.node_steps = config.NODE_STEPS
        self.aux_loss_steps = config.AUX_LOSS_STEPS
        self.num_joints = config.CLASS.OUTPUT_SIZES[-1]
        if self.node_steps != 0:
            raise NotImplementedError("NODE_STEPS > 0 (the reference calls the layer without node_types)")
        if config.AGGR_TYPE == "per_type":
            aggr = "attn" if config.AGGR_SUB in ("node_edge_attn", "node_edge_attn_per_type") else config.AGGR
        else:
            aggr = config.AGGR
        if aggr not in AGGR_CODES:
            raise NotImplementedError(f"AGGR={aggr}")
        self.aggr_code = AGGR_CODES[aggr]
        self.precision = default_precision(self.aggr_code)   # "fp32" | "bf16x3" | "f16x3", settable
        self._folded = None
        self._folded_key = None
        self._tensors = None
        self._ws = _lib.Workspace()
        self._desc_key = None
        self._cap_ok = True   # pemp_step_fully_cap may queue this model's forward (cleared when the library refuses it)
        # one libpemp call addresses r, Q0 and the aggregates with 32-bit byte offsets (pemp_mpn_forward: E, T N
        # < 2^23); larger calls are cut into node blocks no edge crosses (image blocks for construct_graph output)
        self._edge_limit = _EDGE_LIMIT
        self._node_rows_limit = _EDGE_LIMIT

    # --------------------------------------------------------------------------------------
    def _apply(self, fn, *args, **kwargs):
        # .to()/.cuda()/.float() move or re-create tensors: drop the folded cache and tensor list
        self._tensors = None
        self._folded = None
        return super()._apply(fn, *args, **kwargs)

    def _load_from_state_dict(self, *args, **kwargs):
        self._tensors = None            # load_state_dict(assign=True) may swap tensor objects
        return super()._load_from_state_dict(*args, **kwargs)

    def _weights(self, device):
        # The fold is cached against the version counters of every parameter/buffer (in-place
        # updates such as load_state_dict bump them); the flat tensor list itself is cached
        # because walking the module tree costs ~0.3 ms per call.
        if self._tensors is None:
            self._tensors = list(self.parameters()) + list(self.buffers())
        key = (device, self.precision, [t._version for t in self._tensors])
        if self._folded is None or self._folded_key != key:
            try:
                self._folded = fold_weights(self, device, self.precision)
            except F16RangeError as exc:      # folded weights outside the f16 split range: exact fp32
                warnings.warn(f"{exc}; this model runs in precision 'fp32'")
                self.precision = "fp32"
                key = (device, self.precision, key[2])
                self._folded = fold_weights(self, device, self.precision)
            self._folded_key = key
        return self._folded

    def _forward_blocks(self, x, edge_attr, edge_index, node_types, kwargs):
        """A call over the library's size limit: the nodes are cut into contiguous blocks that no edge crosses
        (each image of a construct_graph batch is such a block; node ids are image-major, ConstructGraph.py:206-231),
        packed greedily under the limit, and each block runs as its own forward; the logits go back to their
        edges and nodes. Graphs are per-image independent, so the result is the whole call's up to the rounding
        order of the edge passes' work split."""
        dev = x.device
        N, E = x.shape[0], edge_index.shape[1]
        ei = edge_index.long()
        lo = torch.minimum(ei[0], ei[1])
        blocks = node_blocks(ei, N, self._edge_limit, self._node_rows_limit // self.num_types)
        n_rec = sum(1 for i in range(self.edge_steps) if i >= self.edge_steps - self.aux_loss_steps - 1)
        edge_logits = torch.empty(max(n_rec, 1), E, dtype=torch.float32, device=dev)
        node_logits = torch.empty(n_rec + 1, N, dtype=torch.float32, device=dev)
        class_logits = torch.empty(n_rec + 1, N, self.num_joints, dtype=torch.float32, device=dev)
        sub_kw = {k: v for k, v in kwargs.items() if k == "validate"}
        for n0, n1 in blocks:
            ids = torch.nonzero((lo >= n0) & (lo < n1)).flatten()
            pe, pn, pc, _ = self.forward(x[n0:n1], edge_attr[ids], ei[:, ids] - n0, node_types=node_types[n0:n1],
                                         **sub_kw)
            for r in range(n_rec):
                edge_logits[r, ids] = pe[r].reshape(-1)
            for r in range(n_rec + 1):
                node_logits[r, n0:n1] = pn[r].reshape(-1)
                class_logits[r, n0:n1] = pc[r]
        preds_edge = _rows(edge_logits, n_rec)
        preds_node = _rows(node_logits, n_rec + 1)
        preds_class = list(class_logits.unbind(0))
        return preds_edge, preds_node, preds_class, [None]

    def forward(self, x, edge_attr, edge_index, **kwargs):
        if self.training:
            raise NotImplementedError("pemp_amd MPN is inference-only: call .eval() (BatchNorm uses running stats)")
        if x.device.type != "cuda":
            raise RuntimeError("pemp_amd MPN runs on the HIP device only (no CPU fallback)")
        L = _lib.lib()
        dev = x.device
        node_types = kwargs["node_types"]
        N, E = x.shape[0], edge_index.shape[1]
        if E > self._edge_limit or self.num_types * N > self._node_rows_limit:
            return self._forward_blocks(x, edge_attr, edge_index, node_types, kwargs)
        if self.node_summary != "not":
            node_types = torch.tensor(TYPE_LUTS[self.node_summary], device=dev)[node_types]
        else:
            done = self._take_cap(x, edge_attr, edge_index, node_types)
            if done is not None:      # queued by construct_graph ahead of the counts (capacity mode)
                return done
        fully = _fully_graph(edge_index, node_types, N) if self.node_summary == "not" else None
        knn = _knn_graph(edge_index, N) if fully is None else None
        sym = fully is None and knn is None and _sym_graph(edge_index)
        x = _as(x, torch.float32)
        edge_attr = _as(edge_attr, torch.float32)
        edge_index = _as(edge_index, torch.int64)
        if node_types.dtype != torch.int64:
            node_types = node_types.long()
        if node_types.dim() != 1 or (N > 0 and node_types.stride(0) < 1):
            node_types = node_types.reshape(-1).contiguous()
        t_stride = node_types.stride(0) if N > 0 else 1       # joint_det[:, 2] is read in place
        if self.precision not in PRECISIONS:
            raise ValueError(f"precision={self.precision!r}: expected one of {sorted(PRECISIONS)}")
        fw = self._weights(dev)                               # may fall back to fp32 (weight range)
        A = edge_attr.shape[1] if edge_attr.dim() == 2 else 1
        dkey = (A, x.shape[1], self.precision, t_stride)
        if self._desc_key != dkey:
            steps, aux = self.edge_steps, self.aux_loss_steps
            self._n_rec = sum(1 for i in range(steps) if i >= steps - aux - 1)
            self._desc = _lib.PempMpnDesc(self.num_types, self.num_joints, steps, aux, self.aggr_code, 64, A,
                                          x.shape[1], PRECISIONS[self.precision], t_stride, 0)
            self._desc_ref = ctypes.byref(self._desc)
            self._desc_key = dkey
        desc, n_rec = self._desc_ref, self._n_rec
        ws = self._ws.get(L.pemp_mpn_workspace_size(desc, N, E), dev)
        st = _lib.stream(dev)
        # the three logit arrays share one allocation (one caching-allocator call per forward instead of
        # three); each segment starts on a 256-byte boundary
        ne, nn_ = max(n_rec, 1) * E, (n_rec + 1) * N
        nc = nn_ * self.num_joints
        a1 = (ne + 63) // 64 * 64
        a2 = a1 + (nn_ + 63) // 64 * 64
        buf = torch.empty(a2 + nc, dtype=torch.float32, device=dev)
        edge_logits = buf[:ne].view(max(n_rec, 1), E)
        node_logits = buf[a1:a1 + nn_].view(n_rec + 1, N)
        class_logits = buf[a2:a2 + nc].view(n_rec + 1, N, self.num_joints)
        if fully is not None:       # the graph constructor's fully graph: closed-form edge order
            noff, offs, B = fully
            _lib.check(L.pemp_mpn_forward_fully(desc, fw.struct_ref, x.data_ptr(), edge_attr.data_ptr(),
                                                edge_index.data_ptr(), node_types.data_ptr(), N, E, noff.data_ptr(),
                                                offs, B, edge_logits.data_ptr(), node_logits.data_ptr(),
                                                class_logits.data_ptr(), ws.data_ptr(), ws.numel(), st))
        elif knn is not None:       # the constructor's knn graph: order from its build's bit rows
            kws, offs, noff, nh = knn
            base = kws.data_ptr()
            _lib.check(L.pemp_mpn_forward_knn(desc, fw.struct_ref, x.data_ptr(), edge_attr.data_ptr(),
                                              edge_index.data_ptr(), node_types.data_ptr(), N, E, base + offs[0],
                                              base + offs[1], noff.data_ptr(), nh.ctypes.data, base + offs[2],
                                              len(nh) - 1, edge_logits.data_ptr(), node_logits.data_ptr(),
                                              class_logits.data_ptr(), ws.data_ptr(), ws.numel(), st))
        elif sym:                   # a to_undirected graph of the constructor: order from its rows
            _lib.check(L.pemp_mpn_forward_sym(desc, fw.struct_ref, x.data_ptr(), edge_attr.data_ptr(),
                                              edge_index.data_ptr(), node_types.data_ptr(), N, E,
                                              edge_logits.data_ptr(), node_logits.data_ptr(),
                                              class_logits.data_ptr(), ws.data_ptr(), ws.numel(), st))
        else:
            _lib.check(L.pemp_mpn_forward(desc, fw.struct_ref, x.data_ptr(), edge_attr.data_ptr(),
                                          edge_index.data_ptr(), node_types.data_ptr(), N, E, edge_logits.data_ptr(),
                                          node_logits.data_ptr(), class_logits.data_ptr(), ws.data_ptr(), ws.numel(),
                                          st))
        if kwargs.get("validate", _VALIDATE or (_DEBUG_SYNC and (sym or fully is not None or knn is not None))):
            _lib.check(L.pemp_mpn_status(desc, N, E, _lib.ptr(ws), _lib.stream(dev)))
        # list lengths and .squeeze() semantics of NodeClassificationMPNSimple.py:81-97
        preds_edge = _rows(edge_logits, n_rec)
        preds_node = _rows(node_logits, n_rec + 1)
        preds_class = list(class_logits.unbind(0))
        return preds_edge, preds_node, preds_class, [None]


    # ---- capacity mode (graph_constructor.bind_mpn): the forward queued before the detection counts are known ----
    def _forward_cap(self, x, edge_attr, joint_det, n_cap, e_cap, n_det, det_cap, node_off, B, counts_in_off=False):
        """Queue pemp_mpn_forward_fully_cap on the capacity buffers of pemp_fully_graph_build_cap (x [n_cap, C],
        edge_attr [e_cap, A], joint_det [n_cap, 3], node_off [B + 1]) with the detection's device counts n_det.
        Returns the pending result (logit buffer + the key it was computed under) or None when this model / batch
        takes the exact forward (training, type summaries, unfused node MLPs, a detection capacity past the
        closed-form limit, over-size capacities)."""
        launch = self._prepare_cap(x, edge_attr, joint_det, n_cap, e_cap, n_det, det_cap, node_off, B, counts_in_off)
        return None if launch is None else launch()

    def _prepare_cap(self, x, edge_attr, joint_det, n_cap, e_cap, n_det, det_cap, node_off, B, counts_in_off=False):
        """_forward_cap in two halves: the host preparation (weights, descriptor, workspace, logit buffer) now,
        and the returned launch() that queues the call and returns the pending result (or None); None when this
        model / batch takes the exact forward. The graph constructor prepares before its first launch and calls
        launch() right after the graph build's, so nothing but the call itself separates the two on the GPU."""
        if self.training or self.node_summary != "not" or _FULLY_OFF or x.device.type != "cuda":
            return None
        if e_cap > self._edge_limit or self.num_types * n_cap > self._node_rows_limit:
            return None
        L = _lib.lib()
        dev = x.device
        node_types = joint_det[:, 2]
        fw = self._weights(dev)
        A = edge_attr.shape[1]
        dkey = (A, x.shape[1], self.precision, 3)
        if self._desc_key != dkey:
            steps, aux = self.edge_steps, self.aux_loss_steps
            self._n_rec = sum(1 for i in range(steps) if i >= steps - aux - 1)
            self._desc = _lib.PempMpnDesc(self.num_types, self.num_joints, steps, aux, self.aggr_code, 64, A,
                                          x.shape[1], PRECISIONS[self.precision], 3, 0)
            self._desc_ref = ctypes.byref(self._desc)
            self._desc_key = dkey
        desc, n_rec = self._desc_ref, self._n_rec
        if counts_in_off:   # node_off [B + 4]: the build wrote the batch's (N, E, overflow) after the offsets
            if getattr(self, "_desc_cnt_key", None) != dkey:
                d = self._desc
                self._desc_cnt = _lib.PempMpnDesc(d.num_types, d.num_joints, d.steps, d.aux_loss_steps, d.aggr,
                                                  d.hidden, d.edge_attr_dim, d.node_in_dim, d.precision,
                                                  d.types_stride, _lib.MPN_COUNTS_IN_OFFSETS)
                self._desc_cnt_ref = ctypes.byref(self._desc_cnt)
                self._desc_cnt_key = dkey
            desc = self._desc_cnt_ref
        ws = self._ws.get(L.pemp_mpn_workspace_size(desc, n_cap, e_cap), dev)
        ne, nn_ = max(n_rec, 1) * e_cap, (n_rec + 1) * n_cap
        a1 = (ne + 63) // 64 * 64
        a2 = a1 + (nn_ + 63) // 64 * 64
        buf = torch.empty(a2 + nn_ * self.num_joints, dtype=torch.float32, device=dev)
        bp = buf.data_ptr()
        args = (desc, fw.struct_ref, x.data_ptr(), edge_attr.data_ptr(), node_types.data_ptr(), n_cap, e_cap,
                n_det.data_ptr(), det_cap, node_off.data_ptr(), B, bp, bp + 4 * a1, bp + 4 * a2, ws.data_ptr(),
                ws.numel(), _lib.stream(dev))
        result = dict(buf=buf, a1=a1, a2=a2, n_rec=n_rec, key=(dev, self.precision, self._folded_key))

        def launch():
            rc = L.pemp_mpn_forward_fully_cap(*args)
            if rc == _lib.ERR_UNSUPPORTED:
                return None           # the exact forward runs instead
            _lib.check(rc)
            return result
        return launch

    def _cap_info(self, C, A, n_cap, e_cap, dev):
        """The forward's part of a pemp_step_fully_cap plan (graph_constructor's batch-step entry): (descriptor with
        PEMP_MPN_COUNTS_IN_OFFSETS, folded weights, workspace, key of the weights it was planned under), or None when
        this model / capacity takes the exact forward (the conditions of _prepare_cap)."""
        if self.training or self.node_summary != "not" or _FULLY_OFF or dev.type != "cuda":
            return None
        if e_cap > self._edge_limit or self.num_types * n_cap > self._node_rows_limit:
            return None
        fw = self._weights(dev)
        dkey = (A, C, self.precision, 3)
        if getattr(self, "_desc_cnt_key", None) != dkey:
            steps, aux = self.edge_steps, self.aux_loss_steps
            self._n_rec = sum(1 for i in range(steps) if i >= steps - aux - 1)
            self._desc_cnt = _lib.PempMpnDesc(self.num_types, self.num_joints, steps, aux, self.aggr_code, 64, A, C,
                                              PRECISIONS[self.precision], 3, _lib.MPN_COUNTS_IN_OFFSETS)
            self._desc_cnt_ref = ctypes.byref(self._desc_cnt)
            self._desc_cnt_key = dkey
        L = _lib.lib()
        ws = self._ws.get(L.pemp_mpn_workspace_size(self._desc_cnt_ref, n_cap, e_cap), dev)
        return self._desc_cnt, fw, ws, (dev, self.precision, self._folded_key)

    def _attach_cap(self, pending, x, edge_attr, edge_index, joint_det, N, E):
        """Tag construct_graph's output with the queued result (the capacity batch fit: N, E are its counts)."""
        edge_index._pemp_mpn = (self, pending, N, E, x.data_ptr(), x._version, edge_attr.data_ptr(),
                                edge_attr._version, edge_index._version, joint_det.data_ptr(), joint_det._version)

    def _take_cap(self, x, edge_attr, edge_index, node_types):
        """The queued result of this exact graph, as forward returns it (once), or None (no tag, another model, an
        input or weight changed since it was queued, already taken)."""
        tag = getattr(edge_index, "_pemp_mpn", None)
        if tag is None:
            return None
        mdl, pending, N, E, xp, xv, ep, ev, iv, jp, jv = tag
        if (mdl is not self or x.data_ptr() != xp or x._version != xv or edge_attr.data_ptr() != ep
                or edge_attr._version != ev or edge_index._version != iv or x.shape[0] != N
                or edge_index.shape[1] != E or node_types.data_ptr() != jp + 16 or node_types.stride(0) != 3
                or node_types._version != jv):
            return None
        self._weights(x.device)
        if pending["key"] != (x.device, self.precision, self._folded_key):
            return None
        edge_index._pemp_mpn = None                            # one use: a repeated call computes
        buf, a1, a2, n_rec, J = pending["buf"], pending["a1"], pending["a2"], pending["n_rec"], self.num_joints
        edge_logits = buf[:max(n_rec, 1) * E].view(max(n_rec, 1), E)
        node_logits = buf[a1:a1 + (n_rec + 1) * N].view(n_rec + 1, N)
        class_logits = buf[a2:a2 + (n_rec + 1) * N * J].view(n_rec + 1, N, J)
        preds_edge = _rows(edge_logits, n_rec)
        preds_node = _rows(node_logits, n_rec + 1)
        preds_class = list(class_logits.unbind(0))
        return preds_edge, preds_node, preds_class, [None]


def node_blocks(edge_index, N, edge_limit, node_limit):
    """[(n0, n1), ...]: contiguous node blocks covering [0, N) such that no edge joins two blocks, each holding at
    most edge_limit edges and node_limit nodes (greedy: every block ends at the last admissible cut). Raises
    NotImplementedError when one indivisible block is over a limit."""
    E = edge_index.shape[1]
    lo, hi = torch.minimum(edge_index[0], edge_index[1]), torch.maximum(edge_index[0], edge_index[1])
    if E and (int(lo.min()) < 0 or int(hi.max()) >= N):
        raise ValueError(f"edge_index holds node ids outside [0, {N})")
    diff = torch.zeros(N + 1, dtype=torch.int64, device=edge_index.device)
    diff.index_add_(0, lo, torch.ones_like(lo))
    diff.index_add_(0, hi, -torch.ones_like(hi))
    cover = diff.cumsum(0)[:N].cpu().numpy()                           # edges spanning the cut after node p
    cum_e = torch.bincount(lo, minlength=N).cumsum(0).cpu().numpy()    # edges inside nodes [0, p]
    cuts = np.nonzero(cover == 0)[0] + 1                               # admissible block ends; N among them
    blocks, n0, e0 = [], 0, 0
    while n0 < N:
        k = min(int(np.searchsorted(cum_e[cuts - 1], e0 + edge_limit, "right")),
                int(np.searchsorted(cuts, n0 + node_limit, "right"))) - 1
        if k < 0:
            raise NotImplementedError(f"pemp_amd MPN: a connected block of the graph exceeds one call's limit "
                                      f"({edge_limit} edges, {node_limit} nodes)")
        n1 = int(cuts[k])
        blocks.append((n0, n1))
        n0, e0 = n1, int(cum_e[n1 - 1])
        cuts = cuts[k + 1:]
    return blocks


def _fully_graph(edge_index, node_types, N):
    """(node_off, host offsets, B) when edge_index is the untouched fully graph of the graph
    constructor (graph_constructor._tag_fully) and node_types is its joint_det[:, 2], else None."""
    meta = getattr(edge_index, "_pemp_fully", None)
    if meta is None or _FULLY_OFF:
        return None
    noff, counts, jdet, jver, ever = meta
    if (edge_index._version != ever or jdet._version != jver or node_types.dtype != torch.int64
            or node_types.data_ptr() != jdet.data_ptr() + 16 or node_types.stride(0) != 3
            or node_types.shape[0] != N or jdet.shape[0] != N or len(counts) > 64):
        return None
    B = len(counts)
    return noff, (ctypes.c_int64 * (B + 1))(*itertools.accumulate(counts, initial=0)), B


def _knn_graph(edge_index, N):
    """(workspace, offsets, node_off, host offsets) when edge_index is the untouched knn graph of the graph
    constructor (graph_constructor._tag_knn) over these N nodes, else None. A hint like _tag_sym's."""
    meta = getattr(edge_index, "_pemp_knn", None)
    if meta is None or _KNN_OFF or _SYM_OFF:
        return None
    kws, offs, noff, nh, ever = meta
    if edge_index._version != ever or int(nh[-1]) != N:
        return None
    return kws, offs, noff, nh


def _sym_graph(edge_index):
    """True when edge_index is an untouched (src, dst)-sorted symmetric graph of the graph constructor
    (graph_constructor._tag_sym). A hint only: see _tag_sym for the edits it cannot see."""
    ever = getattr(edge_index, "_pemp_sym", None)
    return ever is not None and not _SYM_OFF and edge_index._version == ever


def _as(t, dtype):
    if t.dtype != dtype:
        t = t.to(dtype)
    return t if t.is_contiguous() else t.contiguous()


def get_mpn_model(config, **kwargs):
    """``src/Models/MessagePassingNetwork/__init__.py:27-73`` — the hot-path model only."""
    if config.NAME == "NodeClassificationMPN":
        return NodeClassificationMPNSimple(config)
    raise NotImplementedError(f"MPN NAME={config.NAME}: only NodeClassificationMPN is on the accelerated path")
