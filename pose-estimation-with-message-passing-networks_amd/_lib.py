"""ctypes binding of ``csrc/libpemp.so`` (C-ABI declared in ``include/pemp.h``).

The product path has no CPU fallback: ``lib()`` raises if the library is missing, was built for
another ABI, or no gfx950 device is present.
"""
import ctypes
import threading
import os

LIB_PATH = os.environ.get("PEMP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc",
                                                     "libpemp.so")
ABI_VERSION = 20

ERR_INVALID_ARG, ERR_HIP, ERR_WORKSPACE, ERR_UNSUPPORTED = -1, -2, -3, -4
BUILD_WRITE_COUNTS = 0x100          # pemp.h PEMP_BUILD_WRITE_COUNTS
MPN_PREPARED, MPN_COUNTS_IN_OFFSETS = 1, 2   # pemp.h PEMP_MPN_* desc flags

c_i32, c_i64, c_f32, c_sz, c_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p


class PempLayer(ctypes.Structure):
    _fields_ = [("w", c_p), ("b", c_p), ("in_dim", c_i32), ("out_dim", c_i32), ("relu", c_i32), ("pad_", c_i32)]


class PempMlp(ctypes.Structure):
    _fields_ = [("layer", PempLayer * 4), ("n_layers", c_i32), ("pad_", c_i32)]


class PempMpnWeights(ctypes.Structure):
    _fields_ = [("node_emb", PempMlp), ("edge_emb", PempMlp),
                ("pre_w", c_p), ("pre_b", c_p), ("q0_w", c_p), ("q0_b", c_p), ("e1_w", c_p),
                ("e2_w", c_p), ("e2_b", c_p), ("msg_w", c_p), ("attn_w", c_p), ("upd_w", c_p), ("upd_b", c_p),
                ("edge_head", PempMlp), ("node_head", PempMlp), ("class_head", PempMlp),
                ("attn_b", c_f32), ("pad_", c_i32),
                ("e1_bf", c_p), ("e2_bf", c_p), ("msg_bf", c_p), ("head_bf", c_p), ("emb_bf", c_p),
                ("upd_bf", c_p), ("pre_bf", c_p), ("node_img", c_p), ("attn_bv", c_p),
                ("upd_mlp", PempMlp),
                ("ept_l1_w", c_p), ("ept_l1_b", c_p), ("ept_l2_w", c_p), ("ept_l2_b", c_p), ("ept_o1_w", c_p),
                ("ept_o2_w", c_p), ("edge_img", c_p), ("emb_comp_bf", c_p), ("emb_comp_b", c_p)]


class PempProjMaps(ctypes.Structure):
    _fields_ = [("num_scales", c_i32), ("channels", c_i32), ("maps", c_p * 4), ("flip_maps", c_p * 4),
                ("h", c_i32 * 4), ("w", c_i32 * 4), ("flip_index", c_p), ("divisor", c_f32)]


class PempMpnDesc(ctypes.Structure):
    _fields_ = [("num_types", c_i32), ("num_joints", c_i32), ("steps", c_i32), ("aux_loss_steps", c_i32),
                ("aggr", c_i32), ("hidden", c_i32), ("edge_attr_dim", c_i32), ("node_in_dim", c_i32),
                ("precision", c_i32), ("types_stride", c_i32), ("flags", c_i32)]


STEP_DET, STEP_DSC, STEP_NDET, STEP_X, STEP_JDET, STEP_JSC, STEP_BIDX, STEP_JTAGS, STEP_EIDX, STEP_EATTR, STEP_NOFF, \
    STEP_LOGITS, STEP_NOUT = range(13)


class PempStepPlan(ctypes.Structure):
    _fields_ = [("B", c_i32), ("J", c_i32), ("H", c_i32), ("W", c_i32), ("pool_kernel", c_i32), ("use_threshold", c_i32),
                ("topk", c_i32), ("det_cap", c_i32), ("projected", c_i32), ("threshold", c_f32), ("det_workspace", c_p),
                ("det_workspace_bytes", c_sz), ("C", c_i32), ("F", c_i32), ("A", c_i32), ("mode", c_i32),
                ("norm_factor", c_f32), ("n_cap", c_i64), ("e_cap", c_i64), ("desc", ctypes.POINTER(PempMpnDesc)),
                ("weights", ctypes.POINTER(PempMpnWeights)), ("mpn_workspace", c_p), ("mpn_workspace_bytes", c_sz),
                ("n_rec", c_i32), ("elog_n", c_i64), ("nlog_off", c_i64), ("clog_off", c_i64),
                ("off", c_sz * STEP_NOUT), ("bytes", c_sz)]


# name -> (restype, argtypes); every symbol of include/pemp.h
SIGNATURES = {
    "pemp_abi_version": (c_i32, []),
    "pemp_last_error": (ctypes.c_char_p, []),
    "pemp_device_check": (c_i32, []),
    "pemp_detect_workspace_size": (c_sz, [c_i32, c_i32, c_i32, c_i32, c_i32]),
    "pemp_detect": (c_i32, [c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_i32, c_f32, c_i32, c_i32, c_i32, c_p, c_sz,
                            c_p, c_p, c_p, c_i32, c_p, c_p]),
    "pemp_host_alloc": (c_p, [c_sz]),
    "pemp_host_free": (c_i32, [c_p]),
    "pemp_pack_nodes": (c_i32, [c_p, c_i32, c_p, c_i32, c_i32, c_i32, c_i32, c_i32, c_p, c_p, c_i32, c_p, c_i64,
                                c_p, c_p, c_p, c_p, c_p, c_p]),
    "pemp_graph_offsets": (c_i32, [c_p, c_i32, c_p, c_p, c_p]),
    "pemp_fully_graph_build": (c_i32, [c_p, c_i32, c_p, c_p, c_i32, c_p, c_i32, c_p, c_i32, c_i32, c_i32, c_i32,
                                       c_i64, c_i64, c_f32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "pemp_fully_graph_build_cap": (c_i32, [c_p, c_i32, c_p, c_p, c_i32, c_p, c_i32, c_p, c_i32, c_i32, c_i32, c_i32,
                                           c_i64, c_i64, c_f32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "pemp_fully_graph": (c_i32, [c_p, c_p, c_i32, c_i64, c_p, c_p]),
    "pemp_knn_workspace_size": (c_sz, [c_p, c_i32]),
    "pemp_knn_graph_count": (c_i32, [c_p, c_p, c_p, c_i32, c_i32, c_p, c_sz, c_p, c_p]),
    "pemp_knn_graph_emit": (c_i32, [c_p, c_p, c_i32, c_p, c_i64, c_p, c_sz, c_p, c_p]),
    "pemp_knn_graph_build": (c_i32, [c_p, c_p, c_p, c_i32, c_i32, c_p, c_sz, c_i64, c_p, c_p, c_p, c_i32, c_p,
                                     c_i32, c_f32, c_i32, c_p, c_p]),
    "pemp_feature_knn_workspace_size": (c_sz, [c_p, c_i32]),
    "pemp_knn_rows_layout": (c_i32, [c_p, c_i32, c_i32, c_p]),
    "pemp_feature_knn_graph_build": (c_i32, [c_p, c_i32, c_p, c_p, c_p, c_i32, c_i32, c_p, c_sz, c_i64, c_p, c_p,
                                             c_p, c_i32, c_p, c_i32, c_f32, c_i32, c_p, c_p]),
    "pemp_score_graph_workspace_size": (c_sz, [c_p, c_i32, c_i32]),
    "pemp_score_graph": (c_i32, [c_p, c_p, c_p, c_i32, c_i32, c_i64, c_p, c_sz, c_p, c_p]),
    "pemp_gather_projected": (c_i32, [c_p, c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_f32, c_p, c_p, c_i64, c_p, c_p]),
    "pemp_gather_projected_conv": (c_i32, [c_p, c_p, c_p, c_i32, c_i32, c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_i32,
                                           c_f32, c_p, c_p, c_i64, c_p, c_p]),
    "pemp_detect_projected": (c_i32, [c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_i32, c_f32, c_i32, c_i32, c_i32, c_p,
                                      c_sz, c_p, c_p, c_p, c_i32, c_p, c_p]),
    "pemp_gather_projected_tags": (c_i32, [c_p, c_i32, c_i32, c_i32, c_i32, c_p, c_p, c_i64, c_p, c_p]),
    "pemp_project_maps": (c_i32, [c_p, c_i32, c_i32, c_i32, c_i32, c_i32, c_p, c_p, c_p]),
    "pemp_stage_merge": (c_i32, [c_p, c_i32, c_i32, c_i32, c_p, c_i32, c_i32, c_i32, c_i32, c_i32, c_p, c_p]),
    "pemp_edge_features": (c_i32, [c_p, c_p, c_i32, c_p, c_p, c_i64, c_i32, c_f32, c_i32, c_p, c_p]),
    "pemp_mpn_workspace_size": (c_sz, [ctypes.POINTER(PempMpnDesc), c_i64, c_i64]),
    "pemp_mpn_forward": (c_i32, [ctypes.POINTER(PempMpnDesc), ctypes.POINTER(PempMpnWeights), c_p, c_p, c_p, c_p,
                                 c_i64, c_i64, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "pemp_mpn_forward_fully": (c_i32, [ctypes.POINTER(PempMpnDesc), ctypes.POINTER(PempMpnWeights), c_p, c_p, c_p,
                                       c_p, c_i64, c_i64, c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "pemp_mpn_forward_fully_cap": (c_i32, [ctypes.POINTER(PempMpnDesc), ctypes.POINTER(PempMpnWeights), c_p, c_p,
                                           c_p, c_i64, c_i64, c_p, c_i32, c_p, c_i32, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "pemp_mpn_graph_stats": (c_i32, [c_p]),
    "pemp_edge_cus_policy": (c_i32, [c_i32, c_i64, c_i32]),
    "pemp_abi_struct_size": (c_sz, [c_i32]),
    "pemp_mpn_forward_sym": (c_i32, [ctypes.POINTER(PempMpnDesc), ctypes.POINTER(PempMpnWeights), c_p, c_p, c_p,
                                     c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "pemp_mpn_forward_knn": (c_i32, [ctypes.POINTER(PempMpnDesc), ctypes.POINTER(PempMpnWeights), c_p, c_p, c_p,
                                     c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_sz,
                                     c_p]),
    "pemp_mpn_prepare": (c_i32, [ctypes.POINTER(PempMpnDesc), c_p, c_p, c_i64, c_i64, c_p, c_sz, c_p]),
    "pemp_mpn_edge_image_floats": (c_sz, [ctypes.POINTER(PempMpnDesc), ctypes.POINTER(PempMpnWeights)]),
    "pemp_mpn_edge_image": (c_i32, [ctypes.POINTER(PempMpnDesc), ctypes.POINTER(PempMpnWeights), c_p, c_sz, c_p]),
    "pemp_mpn_node_image_floats": (c_sz, [ctypes.POINTER(PempMpnWeights)]),
    "pemp_mpn_node_image": (c_i32, [ctypes.POINTER(PempMpnWeights), c_p, c_sz, c_p]),
    "pemp_mpn_status": (c_i32, [ctypes.POINTER(PempMpnDesc), c_i64, c_i64, c_p, c_p]),
    "pemp_pose_edge_weights": (c_i32, [c_p, c_i64, c_p, c_p, c_f32, c_i32, c_p, c_i32, c_i64, c_i32, c_p, c_p, c_p,
                                       c_p]),
    "pemp_pose_cluster": (c_i32, [c_i32, c_p, c_p, c_i64, c_p, c_p, c_i32, c_i32, c_p, c_p]),
    "pemp_pose_persons": (c_i32, [c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i32, c_i32, c_i64, c_p, c_p, c_p]),
    "pemp_pose_greedy": (c_i32, [c_i32, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i32, c_p, c_i64, c_p, c_p]),
    "pemp_pose_fill_mean": (c_i32, [c_p, c_i32, c_i32]),
    "pemp_pose_refine_workspace_size": (c_sz, [c_i32, c_i32, c_i32, c_i32, c_i32]),
    "pemp_pose_refine": (c_i32, [c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_p, c_i32, c_p, c_sz, c_p]),
    "pemp_pose_adjust": (c_i32, [c_p, c_i32, c_i32, c_i32, c_p, c_i32, c_p]),
    "pemp_pack_to_host": (c_i32, [c_i32, c_p, c_p, c_p, c_sz, c_p, c_p, c_p]),
    "pemp_pose_finish_plan": (c_i32, [c_i32, c_p, c_p, c_p, c_p, c_i32, c_p]),
    "pemp_pose_finish_batch": (c_i32, [c_p, c_p, c_i32, c_i32, c_i32, c_i32, c_i32, c_p, c_i32, c_p, c_p, c_i32,
                                       c_i32, c_p, c_i32, c_p, c_sz, c_p]),
    "pemp_step_layout": (c_sz, [ctypes.POINTER(PempStepPlan)]),
    "pemp_step_fully_cap": (c_i32, [ctypes.POINTER(PempStepPlan), c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "pemp_prof_enable": (c_i32, [ctypes.c_char_p]),
    "pemp_prof_report": (c_i32, [ctypes.c_char_p, c_sz]),
}

_LIB = None


def load_cdll(path: str = LIB_PATH):
    """Load and declare the library WITHOUT touching the GPU (used by the CPU symbol test)."""
    if not os.path.exists(path):
        raise RuntimeError(f"pemp_amd: {path} is missing - build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    if L.pemp_abi_version() != ABI_VERSION:
        raise RuntimeError(f"pemp_amd: libpemp ABI {L.pemp_abi_version()} != {ABI_VERSION}")
    return L


def lib():
    """The HIP library, ready for compute. Raises if no gfx950 HIP device is usable."""
    global _LIB
    if _LIB is None:
        import torch  # torch's HIP runtime must be loaded first: libpemp binds to it by SONAME
        if not torch.cuda.is_available():
            raise RuntimeError("pemp_amd: no HIP device available - the HIP path has no CPU fallback")
        L = load_cdll()
        torch.cuda.init()
        check(L.pemp_device_check(), L)
        _LIB = L
    return _LIB


def check(rc: int, L=None):
    if rc == 0:
        return
    msg = (L or _LIB).pemp_last_error().decode(errors="replace")
    if rc == ERR_INVALID_ARG:
        raise ValueError(msg)
    if rc == ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(f"libpemp error {rc}: {msg}")


def ptr(t):
    # ctypes converts a Python int for a c_void_p argument; None is NULL
    return None if t is None else t.data_ptr()


def stream(device=None):
    """Raw hipStream_t of the current stream of `device` (a torch.device, an index or None for the
    current device) -- the launch stream of every libpemp call."""
    import torch
    if device is None:
        idx = torch.cuda.current_device()
    else:
        idx = device if isinstance(device, int) else device.index
        if idx is None:
            idx = torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)


class Workspace:
    """Grow-only device scratch owned by the caller side (one per use site), one buffer per (device,
    stream): calls queued on different streams never share scratch, calls on one stream are ordered by
    it (a buffer replaced on a stream goes back to torch's stream-aware allocator). Thread-safe."""

    def __init__(self):
        self._bufs = {}
        self._mu = threading.Lock()

    def get(self, nbytes: int, device):
        import torch
        nbytes = max(int(nbytes), 256)
        idx = device.index if device.index is not None else torch.cuda.current_device()
        key = (idx, stream(idx))
        with self._mu:
            buf = self._bufs.get(key)
            if buf is None or buf.numel() < nbytes:
                with torch.cuda.device(idx):
                    buf = torch.empty(nbytes + (nbytes >> 3), dtype=torch.uint8, device=device)
                self._bufs[key] = buf
            return buf


def prof_enable(filt):
    lib().pemp_prof_enable(None if filt is None else filt.encode())


def prof_report():
    """{label: (launches, total_ms)} for the kernels recorded since the last report (syncs)."""
    L = lib()
    buf = ctypes.create_string_buffer(1 << 16)
    L.pemp_prof_report(buf, len(buf))
    out = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split()
        out[name] = (int(cnt), float(ms))
    return out
