"""Drop-in ``NaiveGraphConstructor`` (``src/graph_constructor/ConstructGraph.py:9-249``), inference path.

Same constructor signature, same ``construct_graph()`` 15-tuple, same dtypes (int64 indices) and
node/edge order as the reference; computed by ``libpemp.so`` (``pemp_detect``,
``pemp_pack_nodes``, ``pemp_fully_graph_build`` / ``pemp_knn_graph_*`` / ``pemp_score_graph``,
``pemp_edge_features``). GRAPH_TYPE fully, knn, feature_knn and score_based (``ConstructGraph.py:272-283``).
Host synchronisation: one count read-back after detection (the reference syncs at every
``nonzero``), plus one more for knn graphs.
"""
import ctypes
import os
import threading

import numpy as np
import torch

from . import _lib
from .frontend import ProjectedHeatmaps, ProjectedMaps

_SCORE_BASED_K = 75        # ConstructGraph.py:280 (score_based_graph roots)
_EF_MODES = {
    frozenset(["position", "connection_type"]): 0,
    frozenset(["connection_type"]): 1,
    frozenset(["nothing"]): 2,
    frozenset(["position"]): 3,
    frozenset(["position", "angle", "connection_type"]): 4,
    frozenset(["position", "connection_type", "ae_normed"]): 5,   # associative-embedding modes,
    frozenset(["ae"]): 6,                                         # ConstructGraph.py:337-357
    frozenset(["ae_normed"]): 7,
    frozenset(["ae_tracking_1"]): 8,
}
_EF_TAG_MODES = (5, 6, 7, 8)


def _tag_fully(edge_index, node_off, counts, joint_det):
    """Mark edge_index as this batch's fully graph (per-image node offsets on the device, counts on
    the host) so that the MPN can take pemp_mpn_forward_fully; the versions detect in-place edits."""
    edge_index._pemp_fully = (node_off, tuple(counts), joint_det, joint_det._version, edge_index._version)


def _tag_sym(edge_index):
    """Mark edge_index as a (src, dst)-sorted symmetric graph without duplicates (PyG to_undirected's output:
    knn, feature_knn, score_based), so that the MPN can take pemp_mpn_forward_sym; the version detects in-place
    edits. The tag is only a hint: writes the version counter does not see (through .data, raw pointers from
    ctypes / DLPack / another library) keep it, and such an edited list then breaks the contract of
    pemp_mpn_forward_sym. The library flags a broken contract in its workspace; the MPN reads that flag whenever
    it validates (validate=True, PEMP_VALIDATE=1) and also under PEMP_DEBUG_SYNC=1."""
    edge_index._pemp_sym = edge_index._version


def _tag_knn(edge_index, ws, offs, node_off, node_off_h):
    """Hand the knn build's bit rows to the MPN (pemp_mpn_forward_knn): ws is that call's own workspace (kept
    alive by the tag, never reused by a later build), offs the byte offsets of its rows / row starts / edge
    counts (pemp_knn_rows_layout); the version detects in-place edits of edge_index."""
    edge_index._pemp_knn = (ws, offs, node_off, node_off_h, edge_index._version)


# the capacity graph build hands the capacity-mode MPN the batch's (N, E, overflow) (PEMP_BUILD_WRITE_COUNTS), so the
# forward starts without a counting launch of its own; PEMP_NO_BUILD_COUNTS=1 restores that launch (A/B runs)
_BUILD_COUNTS = not os.environ.get("PEMP_NO_BUILD_COUNTS")
# a repeated fully-graph batch shape goes through the batch-step entry (pemp_step_fully_cap: one C call, one output
# buffer; c2 0.17 -> 0.13 ms per step, profiles/r06_step_entry.md); PEMP_STEP_ENTRY=0 restores the three calls and
# the per-output allocations (A/B runs)
_STEP_ENTRY = _BUILD_COUNTS and os.environ.get("PEMP_STEP_ENTRY", "1") not in ("", "0")


class _StepPlan:
    """A pemp_step_plan (include/pemp.h) for one batch shape, capacity set and forward, with the workspaces it names
    kept alive; outputs() cuts one call's output buffer into construct_graph's tensors."""

    def __init__(self, L, B, J, H, W, pool, use_thr, topk, thr, cap, det_ws, C, F, A, mode, norm, n_cap, e_cap, mi,
                 proj):
        p = _lib.PempStepPlan(B=B, J=J, H=H, W=W, pool_kernel=pool, use_threshold=int(use_thr), topk=topk,
                              det_cap=cap, projected=int(proj), threshold=thr, det_workspace=det_ws.data_ptr(),
                              det_workspace_bytes=det_ws.numel(), C=C, F=F, A=A, mode=mode, norm_factor=norm,
                              n_cap=n_cap, e_cap=e_cap)
        self.mi = mi                                     # (desc, folded weights, workspace, key): kept alive here
        if mi is not None:
            p.desc = ctypes.pointer(mi[0])
            p.weights = ctypes.pointer(mi[1].struct)
            p.mpn_workspace = mi[2].data_ptr()
            p.mpn_workspace_bytes = mi[2].numel()
        if not L.pemp_step_layout(ctypes.byref(p)):
            raise ValueError(L.pemp_last_error().decode())
        self.struct, self.ref, self.det_ws = p, ctypes.byref(p), det_ws
        self.B, self.cap, self.C, self.F, self.A = B, cap, C, F, A
        self.off = [p.off[i] for i in range(_lib.STEP_NOUT)]

    def detections(self, flat):
        """(det_xyt [B, cap, 3], det_scores [B, cap], n_det [B]) of the call that wrote flat."""
        o, B, cap = self.off, self.B, self.cap
        i64, f32, i32 = flat.view(torch.int64), flat.view(torch.float32), flat.view(torch.int32)
        return (i64.as_strided((B, cap, 3), (3 * cap, 3, 1), o[_lib.STEP_DET] // 8),
                f32.as_strided((B, cap), (cap, 1), o[_lib.STEP_DSC] // 4),
                i32.as_strided((B,), (1,), o[_lib.STEP_NDET] // 4))

    def outputs(self, flat, counts_l, cap, tags, mpn, mi):
        """construct_graph's 15-tuple from the call's buffer when the batch fit the capacities (else None); with a
        forward, its queued logits are attached to edge_index for the model call to take."""
        p = self.struct
        N = sum(counts_l)
        E = sum(c * (c - 1) for c in counts_l if c > 1)
        if (max(counts_l) if counts_l else 0) > cap or N > p.n_cap or E > p.e_cap:
            return None
        o, C, F, A = self.off, self.C, self.F, self.A
        i64, f32 = flat.view(torch.int64), flat.view(torch.float32)
        x = f32.as_strided((N, C), (C, 1), o[_lib.STEP_X] // 4)
        joint_det = i64.as_strided((N, 3), (3, 1), o[_lib.STEP_JDET] // 8)
        joint_scores = f32.as_strided((N,), (1,), o[_lib.STEP_JSC] // 4)
        batch_index = i64.as_strided((N,), (1,), o[_lib.STEP_BIDX] // 8)
        joint_tags = None
        if tags is not None:   # [N, F] as the reference's tagmaps[b, type, y, x] rows: [N, *tags.shape[4:]] or [N]
            joint_tags = f32.as_strided((N, F), (F, 1), o[_lib.STEP_JTAGS] // 4).view(
                (N,) + tuple(tags.shape[4:]) if tags.dim() > 4 else (N,))
        edge_index = i64.as_strided((2, E), (E, 1), o[_lib.STEP_EIDX] // 8)
        edge_attr = f32.as_strided((E, A), (A, 1), o[_lib.STEP_EATTR] // 4)
        node_off = i64.as_strided((self.B + 4,), (1,), o[_lib.STEP_NOFF] // 8)
        _tag_fully(edge_index, node_off, counts_l, joint_det)
        if mpn is not None:
            res = dict(buf=f32[o[_lib.STEP_LOGITS] // 4:], a1=p.nlog_off, a2=p.clog_off, n_rec=p.n_rec, key=mi[3])
            mpn._attach_cap(res, x, edge_attr, edge_index, joint_det, N, E)
        return (x, edge_attr, edge_index, None, None, None, None, joint_det, None, None, None, joint_scores,
                batch_index, None, joint_tags)


def get_graph_constructor(config, **kwargs):
    """``src/graph_constructor/__init__.py:4-5``."""
    return NaiveGraphConstructor(config=config, **kwargs)


class PendingGraph:
    """construct_graph_start's handle: result() waits for the detection counts and returns the 15-tuple (once
    computed, the same tuple on every call)."""

    def __init__(self, gc, gen, dev, counts_ent):
        self._gc, self._gen, self._dev, self._counts = gc, gen, dev, counts_ent
        self._out, self._done = None, False

    def _step(self):
        try:
            next(self._gen)
        except StopIteration as stop:
            self._finish(stop.value)
        except BaseException:
            self._fail()
            raise

    def _finish(self, out):
        self._out, self._done = out, True
        NaiveGraphConstructor._host_counts_give(self._dev, self._counts)   # every count was read
        self._gen = None

    def _fail(self):
        self._done = True
        self._gen = None
        torch.cuda.current_stream(self._dev).synchronize()   # queued kernels may still store counts into it
        NaiveGraphConstructor._host_counts_give(self._dev, self._counts)

    def result(self):
        if not self._done:
            try:
                next(self._gen)
                raise RuntimeError("pemp_amd: construct_graph did not finish")   # (the generator yields once)
            except StopIteration as stop:
                self._finish(stop.value)
            except BaseException:
                if not self._done:
                    self._fail()
                raise
        if self._out is None:
            raise RuntimeError("pemp_amd: construct_graph failed")
        return self._out


class NaiveGraphConstructor:
    # Shared between instances, threads and streams (reentrant calls). Device scratch is per
    # (device, stream) (_lib.Workspace); each call takes its own mapped host count buffer from a pool and
    # returns it when the counts are read; the capacity hints are only read / raised under _mu (a stale
    # hint costs a re-build, never a wrong result).
    _ws_detect = _lib.Workspace()
    _ws_knn = _lib.Workspace()
    _mu = threading.Lock()
    _cap = 512   # detections per image kept between calls (grows on overflow)
    _graph_hint = {}   # (shape key) -> (node, edge) capacities of the fully-graph capacity build
    _host_counts_free = {}   # device index -> free (capacity, address, int32 view) mapped host buffers
    _bound_mpn = None        # capacity mode: the MPN queued right behind the capacity graph build (bind_mpn)

    @classmethod
    def bind_mpn(cls, model):
        """Capacity mode for the MPN (None unbinds): when construct_graph takes the capacity graph build
        (pemp_fully_graph_build_cap, a repeated fully-graph batch shape), it also queues `model`'s forward on
        those buffers (pemp_mpn_forward_fully_cap) before it reads the detection counts back, and tags its
        output so that model(x, edge_attr, edge_index, node_types=joint_det[:, 2]) on that output returns the
        queued logits instead of launching again. Any other call of the model -- another graph, an input or
        weight edited in between, a batch that overflowed the capacities -- runs the exact forward."""
        cls._bound_mpn = model

    @classmethod
    def _host_counts_take(cls, L, dev, B):
        """A (capacity, address, int32 view) mapped host buffer of >= B words that pemp_detect stores the
        per-image counts into, owned by the calling construct_graph until _host_counts_give."""
        with cls._mu:
            free = cls._host_counts_free.setdefault(dev.index, [])
            for i, ent in enumerate(free):
                if ent[0] >= B:
                    return free.pop(i)
        cap = max(B, 64)
        addr = L.pemp_host_alloc(4 * cap)
        if not addr:
            raise RuntimeError(f"libpemp: {L.pemp_last_error().decode()}")
        return (cap, addr, np.ctypeslib.as_array((ctypes.c_int32 * cap).from_address(addr)))

    @classmethod
    def _host_counts_give(cls, dev, ent):
        with cls._mu:
            cls._host_counts_free.setdefault(dev.index, []).append(ent)

    @staticmethod
    def _wait_counts(counts, dev):
        """Spin until the device has stored every image's count (pemp_detect's n_det_host): the host
        learns the counts while the emit and graph kernels still run. A stream sync bounds the wait."""
        spins = 0
        while counts.min() < 0:
            spins += 1
            if spins > 200000:
                torch.cuda.current_stream(dev).synchronize()
                if counts.min() < 0:
                    raise RuntimeError("pemp_detect: the device did not publish the detection counts")
        return counts.tolist()

    def __init__(self, scoremaps, tagmaps, features, joints_gt, factor_list, masks, device, config, testing,
                 heatmaps, num_joints):
        if joints_gt is not None:
            raise NotImplementedError("training-time label construction (joints_gt) is out of scope: "
                                      "ConstructGraph.py:114-176 runs only with ground truth")
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("pemp_amd NaiveGraphConstructor runs on the HIP device only (no CPU fallback)")
        self.scoremaps = scoremaps.to(self.device)
        self.tagmaps = tagmaps.to(self.device) if tagmaps is not None else None
        self.features = features.to(self.device)
        self.masks = masks.to(self.device) if masks is not None else None
        self.joints_gt = None
        self.factor_list = factor_list
        self.batch_size = scoremaps.shape[0]
        self.num_joints = num_joints
        self.mask_crowds = config.MASK_CROWDS
        self.detect_threshold = config.DETECT_THRESHOLD if config.DETECT_THRESHOLD <= 1.5 else None
        self.hybrid_k = config.HYBRID_K
        self.mpn_graph_type = config.GRAPH_TYPE
        self.normalize_node_distance = config.NORM_NODE_DISTANCE
        self.edge_features_to_use = config.EDGE_FEATURES_TO_USE
        self.pool_kernel_size = config.POOL_KERNEL_SIZE
        self.testing = testing
        if getattr(config, "USE_GT", False) or getattr(config, "IMAGE_CENTRIC_SAMPLING", False):
            raise NotImplementedError("USE_GT / IMAGE_CENTRIC_SAMPLING need ground truth (training only)")

    # ------------------------------------------------------------------------------------
    def construct_graph(self):
        """ConstructGraph.py:46-68 (inference): the 15-tuple. = construct_graph_start().result()."""
        return self.construct_graph_start().result()

    def construct_graph_start(self):
        """The launch half of construct_graph (no reference counterpart): queues the detection and, with a capacity
        hint, the graph build and the bound MPN, then returns a PendingGraph without waiting for the detection
        counts. Its result() waits for them and returns construct_graph's 15-tuple. A caller with several batches
        in flight (a server, bench.py) queues the next batch before it collects the previous one, so the host's
        count wait overlaps its other work. A pending graph must be collected (result()) before another batch is
        started on the same stream twice over (the library's scratch is per device and stream)."""
        L = _lib.lib()
        st = _lib.stream(self.device)
        sm = self.scoremaps
        if isinstance(sm, ProjectedHeatmaps):   # the test front-end evaluated inside the detection
            self._proj = sm
            self._proj_c = sm.c_struct()
        else:
            self._proj = None
            if sm.dtype != torch.float32:
                sm = sm.float()
            sm = sm.contiguous()
        B, J, H, W = sm.shape
        if J != self.num_joints:
            raise ValueError(f"scoremaps have {J} types, num_joints={self.num_joints}")
        if self.mask_crowds:
            if self.masks is None:
                raise TypeError("MASK_CROWDS is set but masks is None")   # reference: masks[batch] on None
            masks = self.masks.float().contiguous()
        else:
            masks = None
        use_thr = self.detect_threshold is not None
        topk = self.hybrid_k if use_thr else 20
        thr = float(self.detect_threshold) if use_thr else 0.0
        dev = sm.device

        # ---- detection (pemp_detect): one read-back of the per-image counts ----
        counts_ent = self._host_counts_take(L, dev, B)
        gen = self._construct(L, st, sm, masks, B, J, H, W, use_thr, topk, thr, dev, counts_ent[2][:B])
        pending = PendingGraph(self, gen, dev, counts_ent)
        pending._step()                             # up to the count wait: everything is queued
        return pending

    def _construct(self, L, st, sm, masks, B, J, H, W, use_thr, topk, thr, dev, counts_h):
        # host-side preparation of the graph stage, before the first launch: with a capacity hint the detection,
        # the graph build and the MPN are then queued back to back (no host gap between them on the GPU), and in a
        # loop this preparation overlaps the previous batch's GPU work
        feats = self.features
        projected = isinstance(feats, ProjectedMaps)
        if projected:      # x sampled from the projected maps after the graph build (pemp_gather_projected)
            if feats.size != (H, W):
                raise ValueError(f"ProjectedMaps size {feats.size} != scoremap size {(H, W)}")
            pmaps = [m.float().contiguous() for m in feats.maps]
            C = feats.shape[1]
            pconv = feats.conv_params() if feats.gather is not None else None
            feats = None
        else:
            if feats.dtype != torch.float32:
                feats = feats.float()
            feats = feats.contiguous()
            C = feats.shape[1]
        tags = self.tagmaps
        proj_tags = None
        if isinstance(tags, ProjectedHeatmaps):   # sampled at the detections after the build
            if not tags.has_tags:
                raise ValueError(f"ProjectedHeatmaps has {tags.outputs[0].shape[1]} channels: no tag channels")
            proj_tags, tags = tags, None
            F = proj_tags.tag_dims
        elif tags is not None:
            tags = tags.float().contiguous()
            F = 1 if tags.dim() == 4 else int(np.prod(tags.shape[4:]))
        else:
            F = 1
        mode = _EF_MODES.get(frozenset(self.edge_features_to_use))
        if mode is None:
            raise NotImplementedError(f"EDGE_FEATURES_TO_USE={self.edge_features_to_use}")
        if mode in _EF_TAG_MODES and tags is None and proj_tags is None:
            raise TypeError(f"EDGE_FEATURES_TO_USE={self.edge_features_to_use} needs tagmaps")
        A = {0: J + 2, 1: J, 2: 1, 3: 2, 4: J + 3, 5: J + 3, 6: 1, 7: 1, 8: 1}[mode]
        norm = float(max(W, H)) if self.normalize_node_distance else 1.0

        # (projected tags feeding the edge features: the generic path, which samples them before the features)
        fully = self.mpn_graph_type == "fully" and B <= 1024 and not (proj_tags is not None and mode in _EF_TAG_MODES)
        gkey = (B, J, H, W, C, F, A, dev)
        with NaiveGraphConstructor._mu:
            hint = NaiveGraphConstructor._graph_hint.get(gkey) if fully else None
            cap = NaiveGraphConstructor._cap
        built = None
        pending = None
        launch_mpn = None
        step = hint is not None and _STEP_ENTRY and not projected
        if step:
            # the batch-step entry: detection + capacity build + the bound MPN in one call, outputs in one buffer
            n_cap, e_cap = hint
            mpn = NaiveGraphConstructor._bound_mpn
            mi = None
            if mpn is not None and J == getattr(mpn, "num_types", None) and getattr(mpn, "_cap_ok", True):
                mi = mpn._cap_info(C, A, n_cap, e_cap, dev)
            plan = self._step_plan(L, dev, st, B, J, H, W, use_thr, topk, thr, cap, C, F if tags is not None else 0,
                                   A, mode, norm, n_cap, e_cap, mi, self._proj is not None)
            flat = torch.empty(plan.struct.bytes, dtype=torch.uint8, device=dev)
            counts_h.fill(-1)
            rc = L.pemp_step_fully_cap(plan.ref, self._detect_src(sm), _lib.ptr(masks), _lib.ptr(feats), _lib.ptr(tags),
                                       flat.data_ptr(), counts_h.ctypes.data, st)
            if rc == _lib.ERR_UNSUPPORTED and mi is not None:
                mpn._cap_ok = False     # the forward's conditions refused this model: the exact forward from now on
                mi = None
            else:
                _lib.check(rc)
            yield None                                       # (construct_graph_start returns here)
            counts_l = self._wait_counts(counts_h, dev)
            out = plan.outputs(flat, counts_l, cap, tags, mpn if mi is not None else None, mi)
            if out is not None:
                self._update_hint(gkey, counts_l)
                if proj_tags is not None:   # sampled at the detections (pemp_gather_projected_tags)
                    out = out[:14] + (self._gather_proj_tags(L, st, proj_tags, J, H, W, out[7], out[12],
                                                             out[0].shape[0], dev),)
                return out
            # a capacity was exceeded: the exact path below on the step's detections
            ws = plan.det_ws
            det, dsc, n_det = plan.detections(flat)
            hint = None
        else:
            ws = self._ws_detect.get(L.pemp_detect_workspace_size(B, J, H, W, topk), dev)
            det = torch.empty(B, cap, 3, dtype=torch.int64, device=dev)
            dsc = torch.empty(B, cap, dtype=torch.float32, device=dev)
            n_det = torch.empty(B, dtype=torch.int32, device=dev)
        if hint is not None:
            n_cap, e_cap = hint
            bufs = (torch.empty(n_cap, C, dtype=torch.float32, device=dev),
                    torch.empty(n_cap, 3, dtype=torch.int64, device=dev),
                    torch.empty(n_cap, dtype=torch.float32, device=dev),
                    torch.empty(n_cap, dtype=torch.int64, device=dev),
                    torch.empty(n_cap, F, dtype=torch.float32, device=dev) if tags is not None else None,
                    torch.empty(2 * e_cap, dtype=torch.int64, device=dev),
                    torch.empty(e_cap, A, dtype=torch.float32, device=dev),
                    # node offsets (MPN fast path), then the batch's (N, E, overflow) for the capacity-mode MPN
                    torch.empty(B + 4, dtype=torch.int64, device=dev))
            build_args = (_lib.ptr(n_det), B, _lib.ptr(det), _lib.ptr(dsc), cap, _lib.ptr(feats), C, _lib.ptr(tags), F,
                          J, H, W, n_cap, e_cap, norm, mode | (_lib.BUILD_WRITE_COUNTS if _BUILD_COUNTS else 0),
                          *[_lib.ptr(t) for t in bufs], st)
            mpn = NaiveGraphConstructor._bound_mpn
            if mpn is not None and not projected and J == getattr(mpn, "num_types", None):
                pending_mpn = mpn
                launch_mpn = mpn._prepare_cap(bufs[0], bufs[6], bufs[1], n_cap, e_cap, n_det, cap, bufs[7], B,
                                              counts_in_off=_BUILD_COUNTS)
        if step:
            pass                                             # (queued, and the counts read, above)
        elif hint is not None:
            # capacity mode: the graph build (and the bound MPN) queued before the counts are read, so the GPU
            # builds the graph while the host waits for them (pemp_fully_graph_build_cap)
            self._detect_launch(L, st, sm, masks, B, J, H, W, use_thr, topk, thr, ws, det, dsc, n_det, cap, counts_h)
            _lib.check(L.pemp_fully_graph_build_cap(*build_args))
            if launch_mpn is not None:
                pending = launch_mpn()
            yield None                                       # (construct_graph_start returns here)
            counts_l = self._wait_counts(counts_h, dev)
            built = bufs
        else:
            self._detect_launch(L, st, sm, masks, B, J, H, W, use_thr, topk, thr, ws, det, dsc, n_det, cap, counts_h)
            yield None
            counts_l = self._wait_counts(counts_h, dev)      # the one host read-back of the batch
        mx = max(counts_l) if counts_l else 0
        cap_used = cap                                      # the detections the capacity build read
        if mx > cap:
            cap = mx
            with NaiveGraphConstructor._mu:
                NaiveGraphConstructor._cap = max(NaiveGraphConstructor._cap, cap)
            det = torch.empty(B, cap, 3, dtype=torch.int64, device=dev)
            dsc = torch.empty(B, cap, dtype=torch.float32, device=dev)
            _lib.check(self._detect(L)(self._detect_src(sm), _lib.ptr(masks), B, J, H, W, self.pool_kernel_size, thr,
                                       int(use_thr), topk, 2, _lib.ptr(ws), ws.numel(), _lib.ptr(det), _lib.ptr(dsc),
                                       _lib.ptr(n_det), cap, None, st))
        N = sum(counts_l)
        E_fully = sum(c * (c - 1) for c in counts_l if c > 1)
        if fully:
            self._update_hint(gkey, counts_l)
        if built is not None and mx <= cap_used and N <= built[0].shape[0] and E_fully <= built[6].shape[0]:
            # the capacity build fit: the outputs are leading (contiguous) slices of its buffers
            x, joint_det, joint_scores, batch_index = built[0][:N], built[1][:N], built[2][:N], built[3][:N]
            joint_tags = built[4][:N] if tags is not None else None
            edge_index = built[5][:2 * E_fully].view(2, E_fully)
            edge_attr = built[6][:E_fully]
            if projected:
                self._gather_projected(L, st, pmaps, pconv, H, W, joint_det, batch_index, x)
            if tags is not None:
                joint_tags = joint_tags.view((N,) + tuple(tags.shape[4:])) if tags.dim() > 4 else joint_tags.view(N)
            if proj_tags is not None:
                joint_tags = self._gather_proj_tags(L, st, proj_tags, J, H, W, joint_det, batch_index, N, dev)
            _tag_fully(edge_index, built[7], counts_l, joint_det)
            if pending is not None:
                pending_mpn._attach_cap(pending, x, edge_attr, edge_index, joint_det, N, E_fully)
            return (x, edge_attr, edge_index, None, None, None, None, joint_det, None, None, None, joint_scores,
                    batch_index, None, joint_tags)
        x = torch.empty(N, C, dtype=torch.float32, device=dev)
        joint_det = torch.empty(N, 3, dtype=torch.int64, device=dev)
        joint_scores = torch.empty(N, dtype=torch.float32, device=dev)
        batch_index = torch.empty(N, dtype=torch.int64, device=dev)
        joint_tags = torch.empty(N, F, dtype=torch.float32, device=dev) if tags is not None else None

        if fully:
            # one launch: offsets + nodes + edge_index + edge_attr (pemp_fully_graph_build)
            E = sum(c * (c - 1) for c in counts_l if c > 1)
            edge_index = torch.empty(2, E, dtype=torch.int64, device=dev)
            edge_attr = torch.empty(E, A, dtype=torch.float32, device=dev)
            node_off = torch.empty(B + 1, dtype=torch.int64, device=dev)
            _lib.check(L.pemp_fully_graph_build(
                _lib.ptr(n_det), B, _lib.ptr(det), _lib.ptr(dsc), cap, _lib.ptr(feats), C, _lib.ptr(tags), F, J, H, W,
                N, E, norm, mode, _lib.ptr(x), _lib.ptr(joint_det), _lib.ptr(joint_scores), _lib.ptr(batch_index),
                _lib.ptr(joint_tags), _lib.ptr(edge_index), _lib.ptr(edge_attr), _lib.ptr(node_off), st))
            if N > 0:
                _tag_fully(edge_index, node_off, counts_l, joint_det)
        else:
            node_off_h = np.zeros(B + 1, np.int64)
            node_off_h[1:] = np.cumsum(np.asarray(counts_l, np.int64))
            # batch offsets are recomputed on the device from n_det (no host->device upload)
            offs = torch.empty(2, B + 1, dtype=torch.int64, device=dev)
            node_off, fully_off = offs[0], offs[1]
            _lib.check(L.pemp_graph_offsets(_lib.ptr(n_det), B, _lib.ptr(node_off),
                                            _lib.ptr(fully_off) if self.mpn_graph_type == "fully" else None, st))
            _lib.check(L.pemp_pack_nodes(_lib.ptr(feats), C, _lib.ptr(tags), F, B, J, H, W, _lib.ptr(det),
                                         _lib.ptr(dsc), cap, _lib.ptr(node_off), N, _lib.ptr(x), _lib.ptr(joint_det),
                                         _lib.ptr(joint_scores), _lib.ptr(batch_index), _lib.ptr(joint_tags), st))
            if proj_tags is not None:   # before the edge features, which may read them
                joint_tags = self._gather_proj_tags(L, st, proj_tags, J, H, W, joint_det, batch_index, N, dev)
            if self.mpn_graph_type in ("knn", "feature_knn"):   # edge features written by the knn emit itself
                if self.mpn_graph_type == "feature_knn" and projected:   # the graph ranks by x: sample it first
                    self._gather_projected(L, st, pmaps, pconv, H, W, joint_det, batch_index, x)
                    projected = False
                edge_index, edge_attr = self._knn_edges(L, st, joint_det, joint_tags, F, joint_scores, node_off,
                                                        node_off_h, B, J, A, norm, mode, dev,
                                                        x if self.mpn_graph_type == "feature_knn" else None)
                _tag_sym(edge_index)
            else:
                edge_index = self._edges(L, st, joint_det, joint_scores, node_off, fully_off, node_off_h, B, dev)
                if self.mpn_graph_type == "score_based":
                    _tag_sym(edge_index)
                E = edge_index.shape[1]
                edge_attr = torch.empty(E, A, dtype=torch.float32, device=dev)
                _lib.check(L.pemp_edge_features(_lib.ptr(joint_det), _lib.ptr(joint_tags), F, _lib.ptr(joint_scores),
                                                _lib.ptr(edge_index), E, J, norm, mode,
                                                _lib.ptr(edge_attr), st))
        if projected:
            self._gather_projected(L, st, pmaps, pconv, H, W, joint_det, batch_index, x)
        if tags is not None:
            joint_tags = joint_tags.view((N,) + tuple(tags.shape[4:])) if tags.dim() > 4 else joint_tags.view(N)
        if proj_tags is not None and fully:
            joint_tags = self._gather_proj_tags(L, st, proj_tags, J, H, W, joint_det, batch_index, N, dev)
        return (x, edge_attr, edge_index, None, None, None, None, joint_det, None, None, None, joint_scores,
                batch_index, None, joint_tags)

    @staticmethod
    def _update_hint(gkey, counts_l):
        """Capacities for the next batch of this shape: 25 % headroom over this one (grow-only)."""
        N = sum(counts_l)
        E = sum(c * (c - 1) for c in counts_l if c > 1)
        n_hint = (N + N // 4 + 16, E + E // 4 + 256)
        with NaiveGraphConstructor._mu:
            old = NaiveGraphConstructor._graph_hint.get(gkey)
            NaiveGraphConstructor._graph_hint[gkey] = n_hint if old is None else (
                max(old[0], n_hint[0]), max(old[1], n_hint[1]))

    def _detect_launch(self, L, st, sm, masks, B, J, H, W, use_thr, topk, thr, ws, det, dsc, n_det, cap, counts_h):
        counts_h.fill(-1)
        _lib.check(self._detect(L)(self._detect_src(sm), _lib.ptr(masks), B, J, H, W, self.pool_kernel_size, thr,
                                   int(use_thr), topk, 3, _lib.ptr(ws), ws.numel(), _lib.ptr(det), _lib.ptr(dsc),
                                   _lib.ptr(n_det), cap, counts_h.ctypes.data, st))

    _plans = {}   # (device, stream, batch shape, capacities, forward) -> _StepPlan (under _mu)

    def _step_plan(self, L, dev, st, B, J, H, W, use_thr, topk, thr, cap, C, F, A, mode, norm, n_cap, e_cap, mi,
                   proj):
        """The pemp_step_fully_cap plan of this call's arguments (cached per device, stream and shape)."""
        fkey = None if mi is None else (id(mi[1]), mi[2].data_ptr(), mi[2].numel(), ctypes.addressof(mi[0]))
        key = (dev.index, st, B, J, H, W, self.pool_kernel_size, use_thr, topk, thr, cap, C, F, A, mode, norm, n_cap,
               e_cap, fkey, proj)
        with NaiveGraphConstructor._mu:
            plan = NaiveGraphConstructor._plans.get(key)
        if plan is None:
            ws = self._ws_detect.get(L.pemp_detect_workspace_size(B, J, H, W, topk), dev)
            plan = _StepPlan(L, B, J, H, W, self.pool_kernel_size, use_thr, topk, thr, cap, ws, C, F, A, mode, norm,
                             n_cap, e_cap, mi, proj)
            with NaiveGraphConstructor._mu:
                if len(NaiveGraphConstructor._plans) >= 64:
                    NaiveGraphConstructor._plans.clear()
                NaiveGraphConstructor._plans[key] = plan
        return plan

    def _detect(self, L):
        return L.pemp_detect_projected if self._proj is not None else L.pemp_detect

    def _detect_src(self, sm):
        return ctypes.addressof(self._proj_c) if self._proj is not None else _lib.ptr(sm)

    def _gather_proj_tags(self, L, st, pt, J, H, W, joint_det, batch_index, N, dev):
        """joint_tags [N, F] from the projected tag channels (pemp_gather_projected_tags); the reference's
        tagmaps there are [B, J, H, W, F] (torch.cat(tags_list, dim=4)), so F = 1 stays [N, 1]."""
        F = pt.tag_dims
        jt = torch.empty(N, F, dtype=torch.float32, device=dev)
        c = pt.c_struct()
        _lib.check(L.pemp_gather_projected_tags(ctypes.addressof(c), pt.tag_scale, J, H, W, _lib.ptr(joint_det),
                                                _lib.ptr(batch_index), N, _lib.ptr(jt), st))
        return jt

    def _gather_projected(self, L, st, pmaps, pconv, H, W, joint_det, batch_index, x):
        S = len(pmaps)
        ptrs = (ctypes.c_void_p * S)(*[m.data_ptr() for m in pmaps])
        hs = (ctypes.c_int32 * S)(*[m.shape[2] for m in pmaps])
        ws = (ctypes.c_int32 * S)(*[m.shape[3] for m in pmaps])
        vp = ctypes.c_void_p
        if pconv is not None:   # feature_gather conv at the taps (pemp_gather_projected_conv)
            wt, b, k, pad = pconv
            _lib.check(L.pemp_gather_projected_conv(ctypes.cast(ptrs, vp), ctypes.cast(hs, vp), ctypes.cast(ws, vp), S,
                                                    pmaps[0].shape[1], _lib.ptr(wt), _lib.ptr(b), x.shape[1], k, pad,
                                                    H, W, self.features.divisor, _lib.ptr(joint_det),
                                                    _lib.ptr(batch_index), x.shape[0], _lib.ptr(x), st))
            return
        _lib.check(L.pemp_gather_projected(ctypes.cast(ptrs, vp), ctypes.cast(hs, vp), ctypes.cast(ws, vp), S,
                                           x.shape[1], H, W, self.features.divisor,
                                           _lib.ptr(joint_det), _lib.ptr(batch_index), x.shape[0], _lib.ptr(x), st))

    def _edges(self, L, st, joint_det, joint_scores, node_off, fully_off, node_off_h, B, dev):
        counts = np.diff(node_off_h)
        if self.mpn_graph_type == "fully":
            per = counts * np.maximum(counts - 1, 0)
        elif self.mpn_graph_type == "score_based":
            k = _SCORE_BASED_K
            if counts.size and counts.min() < k:   # the reference's joint_scores.topk(k) raises
                raise RuntimeError(f"score_based graph: selected index k={k} out of range for "
                                   f"{int(counts.min())} detections")
            per = k * (2 * counts - k - 1)
        else:
            raise NotImplementedError(f"GRAPH_TYPE={self.mpn_graph_type}")
        E = int(per.sum())
        edge_index = torch.empty(2, E, dtype=torch.int64, device=dev)
        if self.mpn_graph_type == "fully":
            _lib.check(L.pemp_fully_graph(_lib.ptr(node_off), _lib.ptr(fully_off), B, E, _lib.ptr(edge_index), st))
        elif self.mpn_graph_type == "score_based":
            nh = np.ascontiguousarray(node_off_h)
            nh_p = nh.ctypes.data_as(ctypes.c_void_p)
            ws = self._ws_knn.get(L.pemp_score_graph_workspace_size(nh_p, B, _SCORE_BASED_K), dev)
            _lib.check(L.pemp_score_graph(_lib.ptr(joint_scores), _lib.ptr(node_off), nh_p, B, _SCORE_BASED_K, E,
                                          _lib.ptr(ws), ws.numel(), _lib.ptr(edge_index), st))
        return edge_index

    _KNN_K = 50   # ConstructGraph.py:365 (knn_graph(k=50))

    def _knn_edges(self, L, st, joint_det, joint_tags, F, joint_scores, node_off, node_off_h, B, J, A, norm, mode,
                   dev, x=None):
        """knn_mpn_graph (ConstructGraph.py:363-368) + the edge features in one queued call
        (pemp_knn_graph_build): buffers sized by the closed-form edge bound, the total back through
        mapped memory while the emit still runs; edge_index / edge_attr are the leading contiguous
        [2, E] / [E, A] blocks of those buffers. With x: feature_knn_mpn_graph (ConstructGraph.py:370-374),
        the same graph over the node features x [N, C] (pemp_feature_knn_graph_build)."""
        k = self._KNN_K
        nh = np.ascontiguousarray(node_off_h)
        nh_p = nh.ctypes.data_as(ctypes.c_void_p)
        n = np.diff(nh)
        size = (L.pemp_feature_knn_workspace_size if x is not None else L.pemp_knn_workspace_size)(nh_p, B)
        # batches the MPN's knn prepare takes: a workspace of the call's own, whose bit rows go with edge_index
        rows = None
        if 1 <= B <= 64 and 0 < nh[B] <= 4096 and int(n.max()) <= 512:
            rows = (ctypes.c_size_t * 3)()
            _lib.check(L.pemp_knn_rows_layout(nh_p, B, int(x is not None), rows))
            ws = torch.empty(max(int(size), 256), dtype=torch.uint8, device=dev)
        else:
            ws = self._ws_knn.get(size, dev)
        e_cap = int(np.minimum(n * np.maximum(n - 1, 0), 2 * k * n).sum())
        buf = torch.empty(2 * max(e_cap, 1), dtype=torch.int64, device=dev)
        ea = torch.empty(max(e_cap, 1) * A, dtype=torch.float32, device=dev)
        ent = self._host_counts_take(L, dev, 1)
        try:
            word = ent[2][:1]
            word.fill(-1)
            args = (_lib.ptr(joint_det), _lib.ptr(node_off), nh_p, B, k, _lib.ptr(ws), ws.numel(), e_cap,
                    _lib.ptr(buf), ent[1], _lib.ptr(joint_tags), F, _lib.ptr(joint_scores), J, norm, mode,
                    _lib.ptr(ea), st)
            if x is not None:
                _lib.check(L.pemp_feature_knn_graph_build(_lib.ptr(x), x.shape[1], *args))
            else:
                _lib.check(L.pemp_knn_graph_build(*args))
            E = self._wait_counts(word, dev)[0]
        except BaseException:
            torch.cuda.current_stream(dev).synchronize()
            self._host_counts_give(dev, ent)
            raise
        self._host_counts_give(dev, ent)
        if E > e_cap:
            raise RuntimeError(f"pemp_knn_graph_build: {E} edges > bound {e_cap}")
        edge_index = buf[:2 * E].view(2, E)
        if rows is not None:
            _tag_knn(edge_index, ws, tuple(rows), node_off, nh)
        return edge_index, ea[:E * A].view(E, A)
