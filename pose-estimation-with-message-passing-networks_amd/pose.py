"""Pose grouping after the MPN: MPN edge/node/class probabilities -> persons.

Mirrors, with the same argument meaning and return values:
  * ``pred_to_person`` (``src/Utils/Utils.py:499-514``; ``cc_method`` "GAEC" or "threshold") with the
    GAEC path of ``cluster_graph`` (``src/Utils/correlation_clustering/correlation_clustering_utils.py:21-64,
    99-151, 187-245``) and ``graph_cluster_to_persons`` (``Utils.py:672-743``);
  * ``pred_to_ann``'s grouping prefix (``Utils.py:1445-1459``: detector-score check, node threshold +
    ``subgraph``, the ``None`` returns), batched over every image of a ``construct_graph`` batch:
    ``group_persons``.

Work split (include/pemp.h, ``pemp_pose_*``): the per-edge pass (subgraph test, reverse-edge lookup,
transpose averaging) is one HIP kernel over the whole batch; its output and the node arrays come back in
one stream-ordered copy into pinned memory; greedy additive edge contraction (sequential by nature) and the
person assembly run in C++ in the same library, one image per host thread. No numpy / scipy / Python loop
sits on the path. ``greedy`` (``Utils.py:517-626``) runs on the host after the same edge pass
(``pemp_pose_greedy``). ``MUT`` and ``KL`` are not built (NotImplementedError).
"""
import ctypes
import functools
import os

import numpy as np
import torch

from . import _lib

_METHODS = {"GAEC": 0, "threshold": 1, "greedy": 1}   # greedy: the edge pass keeps raw preds, like threshold


def _method(cc_method):
    if cc_method not in _METHODS:
        raise NotImplementedError(f"cc_method={cc_method!r}: pemp_amd builds GAEC, threshold and greedy")
    return _METHODS[cc_method]


def _host_threads():
    return max(1, min(16, os.cpu_count() or 1))


_NP = {torch.int64: np.int64, torch.int32: np.int32, torch.float32: np.float32, torch.float64: np.float64,
       torch.bool: np.bool_, torch.uint8: np.uint8}


def _to_host_async(tensors, dev):
    """Stream-ordered read-back of device tensors (contiguous; None entries stay None) into one pinned host
    buffer: one pemp_pack_to_host call gathers them into a device staging buffer and one torch copy follows, behind
    the work that produces them on the current stream of `dev`, then an event is recorded. Returns numpy views
    of the host buffer (valid once the event has completed), the event, and the buffer (keep it alive)."""
    L = _lib.lib()
    live = [t for t in tensors if t is not None]
    if len(live) > 16:
        raise ValueError("pemp_amd.pose: at most 16 arrays per read-back")
    offs, total = [], 0
    for t in live:
        offs.append(total)
        total += (t.numel() * t.element_size() + 15) // 16 * 16
    with torch.cuda.device(dev):
        host = torch.empty(max(total, 16), dtype=torch.uint8, pin_memory=True)
        staging = torch.empty(max(total, 16), dtype=torch.uint8, device=dev)
        n = len(live)
        src = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for t in live])
        nb = (ctypes.c_size_t * max(n, 1))(*[t.numel() * t.element_size() for t in live])
        of = (ctypes.c_size_t * max(n, 1))(*offs)
        # the library gathers into the staging buffer; the device-to-host copy goes through torch so that its
        # pinned-memory cache records the copy's event: a job dropped before its copy lands cannot hand the block
        # to a new allocation while the DMA still writes it
        _lib.check(L.pemp_pack_to_host(n, src, nb, of, total, staging.data_ptr(), None, _lib.stream(dev)), L)
        host.copy_(staging, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
    hv = host.numpy()
    out, k = [], 0
    for t in tensors:
        if t is None:
            out.append(None)
            continue
        nbytes = t.numel() * t.element_size()
        out.append(hv[offs[k]:offs[k] + nbytes].view(_NP[t.dtype]).reshape(tuple(t.shape)))
        k += 1
    return out, ev, host


_WORKER = None


def _worker():
    """The library's grouping thread (one, so jobs finish in submission order): it waits for a job's copies and
    runs its host part while the caller's thread queues the next batch. The waits and the C++ calls release
    the GIL (torch event wait, ctypes)."""
    global _WORKER
    if _WORKER is None:
        import concurrent.futures
        _WORKER = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="pemp-grouping")
    return _WORKER


class GroupingJob:
    """The grouping of one batch, started on the GPU (group_persons_start / _start): the edge pass and the copies
    of everything the host part reads are queued on the current stream, nothing waited for. The host part
    (GAEC / threshold components and the person assembly, C++, one image per thread) runs after the copies (an
    event, not a stream sync: work queued after the job keeps running): on the library's grouping thread as soon
    as they land (background=True), or in ``result()``. ``result()`` returns it (and raises its errors)."""

    def __init__(self, state, finish, background=False):
        self._state, self._finish, self._out, self._fut = state, finish, None, None
        if background:
            self._fut = _worker().submit(finish, **state)
            self._state = None

    def result(self):
        if self._fut is not None:
            self._out = self._fut.result()
            self._fut = None
        elif self._state is not None:
            self._out = self._finish(**self._state)
            self._state = None
        return self._out


def _start(joint_det, joint_scores, edge_index, pred, node_off_d, B, th, use_th, class_pred, cc_method, num_joints,
           score_for_poses=None, allow_single=False, timings=None, extra=()):
    """GPU part of the shared path. node_off_d: device int64 [B+1] (computed on the device from batch_index, so
    that nothing here waits for the GPU); extra: more device tensors to bring to the host with the same copies."""
    import time
    t0 = time.perf_counter()
    L = _lib.lib()
    method = _method(cc_method)
    dev = edge_index.device
    if dev.type != "cuda":
        raise ValueError("pemp_amd.pose: expects device tensors (the HIP path has no CPU fallback)")
    N = joint_det.shape[0]
    if joint_det.shape != (N, 3) or joint_scores.shape != (N,):
        raise ValueError(f"pemp_amd.pose: joint_det {tuple(joint_det.shape)} / joint_scores "
                         f"{tuple(joint_scores.shape)} do not match {N} nodes")
    ei = edge_index.to(torch.int64).contiguous()
    E = ei.shape[1]
    pr = pred.reshape(-1).to(torch.float32).contiguous()
    if pr.numel() != E:
        raise ValueError(f"pemp_amd.pose: pred has {pr.numel()} values for {E} edges")
    sc = joint_scores.to(torch.float32).contiguous()
    w = torch.empty(E, dtype=torch.float32, device=dev)
    flags = torch.empty(B + 1, dtype=torch.int32, device=dev)
    row_start = torch.empty(N + 1, dtype=torch.int64, device=dev)
    _lib.check(L.pemp_pose_edge_weights(_lib.ptr(ei), E, _lib.ptr(pr), _lib.ptr(sc), float(th), int(use_th),
                                        _lib.ptr(node_off_d), B, N, method, _lib.ptr(row_start), _lib.ptr(w),
                                        _lib.ptr(flags), _lib.stream(dev)))
    cls = class_pred.to(torch.float32).contiguous() if class_pred is not None else None
    if cls is not None and cls.shape != (N, num_joints):
        raise ValueError(f"pemp_amd.pose: class_pred {tuple(cls.shape)} != ({N}, {num_joints})")
    ps = score_for_poses.to(torch.float32).contiguous() if score_for_poses is not None else None
    if timings is not None:
        torch.cuda.current_stream(dev).synchronize()
        t1 = time.perf_counter()
        timings["edge_pass"] = timings.get("edge_pass", 0.0) + t1 - t0
        t0 = t1
    host, ev, buf = _to_host_async([ei, w, flags, joint_det.to(torch.int64).contiguous(), sc, cls, ps, node_off_d]
                                   + [None if t is None else t.contiguous() for t in extra], dev)
    return dict(host=host, ev=ev, buf=buf, B=B, N=N, E=E, cc_method=cc_method, num_joints=num_joints,
                allow_single=allow_single, timings=timings, t0=t0)


def _cp(a):
    return None if a is None else a.ctypes.data


def _finish(host, ev, buf, B, N, E, cc_method, num_joints, allow_single, timings, t0):
    """Host part of the shared path. Returns (persons list, mutants, labels, flags, node_off, extra host tensors)."""
    import time
    ev.synchronize()
    if timings is not None:
        t1 = time.perf_counter()
        timings["to_host"] = timings.get("to_host", 0.0) + t1 - t0
        t0 = t1
    L = _lib.lib()
    method = _method(cc_method)
    h_ei, h_w, h_flags, h_det, h_sc, h_cls, h_ps, h_off = host[:8]
    extra = host[8:]
    node_off = h_off
    if h_flags[B] & 4:
        raise ValueError("pemp_amd.pose: edge_index holds a node index outside [0, N)")
    if cc_method == "greedy":
        if h_flags[B] & 1:
            raise ValueError("pemp_amd.pose: edge_index is not sorted by (src, dst) without duplicates")
        cap = max(N, 1)
        taken = np.empty(N, dtype=np.int32)
        persons = np.empty((cap, num_joints, 3), dtype=np.float64)
        counts = np.empty(B, dtype=np.int32)
        _lib.check(L.pemp_pose_greedy(B, node_off.ctypes.data, _cp(h_ei), E, _cp(h_w), _cp(h_det), _cp(h_sc),
                                      _cp(h_cls), num_joints, taken.ctypes.data, cap, persons.ctypes.data,
                                      counts.ctypes.data), L)
        starts = np.concatenate([[0], np.cumsum(counts)])
        per_image = [persons[starts[b]:starts[b + 1]].copy() for b in range(B)]
        return per_image, np.zeros(B, dtype=bool), taken, h_flags.copy(), node_off.copy(), extra
    labels = np.empty(N, dtype=np.int32)
    n_comp = np.empty(B, dtype=np.int32)
    _lib.check(L.pemp_pose_cluster(B, node_off.ctypes.data, _cp(h_ei), E, _cp(h_w), _cp(h_flags), method,
                                   _host_threads(), labels.ctypes.data, n_comp.ctypes.data), L)
    if timings is not None:
        t1 = time.perf_counter()
        timings["cluster"] = timings.get("cluster", 0.0) + t1 - t0
        t0 = t1
    cap = max(N, 1)
    persons = np.empty((cap, num_joints, 3), dtype=np.float64)
    counts = np.empty(B, dtype=np.int32)
    mutants = np.empty(B, dtype=np.int32)
    _lib.check(L.pemp_pose_persons(B, node_off.ctypes.data, labels.ctypes.data, n_comp.ctypes.data,
                                   _cp(h_det), _cp(h_sc), _cp(h_ps), _cp(h_cls), num_joints, int(allow_single), cap,
                                   persons.ctypes.data, counts.ctypes.data, mutants.ctypes.data), L)
    if timings is not None:
        timings["persons"] = timings.get("persons", 0.0) + time.perf_counter() - t0
    starts = np.concatenate([[0], np.cumsum(counts)])
    per_image = [persons[starts[b]:starts[b + 1]].copy() for b in range(B)]
    return per_image, mutants.astype(bool), labels, h_flags.copy(), node_off.copy(), extra


def _run(joint_det, joint_scores, edge_index, pred, node_off, th, use_th, class_pred, cc_method, num_joints,
         score_for_poses=None, allow_single=False, timings=None):
    """Shared path, synchronous. node_off: host int64 [B+1]. Returns (persons list, mutants, labels, flags)."""
    off_d = torch.from_numpy(np.ascontiguousarray(node_off, dtype=np.int64)).to(edge_index.device)
    st = _start(joint_det, joint_scores, edge_index, pred, off_d, len(node_off) - 1, th, use_th, class_pred, cc_method,
                num_joints, score_for_poses, allow_single, timings)
    return _finish(**st)[:4]


def pred_to_person(joint_det, joint_scores, edge_index, pred, class_pred, cc_method, num_joints,
                   score_for_poses=None, allow_single_joint_persons=False):
    """``Utils.py:499-514`` for one image's (already thresholded) graph.

    Returns ``(persons, mutant_detected, person_labels)``: persons float64 ``[P, num_joints, 3]`` (x, y,
    score), or an empty ``np.array([])`` when no person is formed, as ``np.array(persons)`` gives there;
    person_labels int32 ``[N]`` component ids in scipy ``connected_components`` order."""
    node_off = np.array([0, joint_det.shape[0]], dtype=np.int64)
    per_image, mutants, labels, _ = _run(joint_det, joint_scores, edge_index, pred, node_off, 0.0, False,
                                         class_pred, cc_method, num_joints, score_for_poses,
                                         allow_single_joint_persons)
    persons = per_image[0] if len(per_image[0]) else np.array([])
    return persons, bool(mutants[0]), labels


def group_persons(joint_det, joint_scores, edge_index, pred, th, class_pred=None, cc_method="GAEC",
                  num_joints=17, batch_index=None, score_map_scores=None, num_images=None, _timings=None):
    """``pred_to_ann``'s grouping prefix (``Utils.py:1447-1459``) for every image of a batch.

    joint_det [ΣN,3] int64, joint_scores [ΣN] (the node probabilities, ``preds_nodes`` in ``valid.py:109``),
    edge_index [2,ΣE] int64 sorted by (src, dst) (``construct_graph``'s output), pred [ΣE] edge
    probabilities, class_pred [ΣN,J] class probabilities or None, batch_index [ΣN] int64 (None: one image),
    score_map_scores [ΣN] detector scores (None: skip that check), num_images the batch size (required
    with batch_index: trailing images without detections have no batch_index entry). Returns one entry
    per image: persons float64 [P, J, 3], or None where ``pred_to_ann`` returns None (no detector score >
    0.1, no edge surviving the node threshold, no person)."""
    return group_persons_start(joint_det, joint_scores, edge_index, pred, th, class_pred, cc_method, num_joints,
                               batch_index, score_map_scores, num_images, _timings, background=False).result()


def group_persons_start(joint_det, joint_scores, edge_index, pred, th, class_pred=None, cc_method="GAEC",
                        num_joints=17, batch_index=None, score_map_scores=None, num_images=None, _timings=None,
                        background=True):
    """group_persons in two halves for pipelined callers: this queues the GPU part (edge pass, copies to pinned
    host memory) on the current stream and returns at once; the host part runs on the library's grouping thread
    once the copies land (background=False: in ``.result()``), so the GPU runs the next batch and the caller
    queues it meanwhile; ``.result()`` of the returned job returns the persons. Same arguments and result as
    group_persons."""
    N = joint_det.shape[0]
    dev = edge_index.device
    if batch_index is None:
        if num_images not in (None, 1):
            raise ValueError("pemp_amd.pose: num_images > 1 needs batch_index")
        B = 1
        off_d = torch.tensor([0, N], dtype=torch.int64, device=dev)
        bi = None
    else:
        if num_images is None:
            raise ValueError("pemp_amd.pose: group_persons(batch_index=...) needs num_images (the batch size)")
        B = int(num_images)
        bi = batch_index.to(torch.int64).contiguous()
        off_d = torch.searchsorted(bi, torch.arange(B + 1, device=dev, dtype=torch.int64))
    extra = [bi if bi is not None else None,
             (score_map_scores > 0.1) if score_map_scores is not None else None]
    st = _start(joint_det, joint_scores, edge_index, pred, off_d, B, th, True, class_pred, cc_method, num_joints,
                timings=_timings, extra=extra)

    def finish(**kw):
        per_image, _, _, flags, node_off, (h_bi, h_ok) = _finish(**kw)
        if h_bi is not None:
            b_np = h_bi
            if len(b_np) and np.any(b_np[1:] < b_np[:-1]):
                raise ValueError("pemp_amd.pose: batch_index must be non-decreasing (construct_graph order)")
            if len(b_np) and (b_np[0] < 0 or b_np[-1] >= B):
                raise ValueError(f"pemp_amd.pose: batch_index outside [0, {B})")
        ok_det = None
        if h_ok is not None:
            ok_det = np.array([h_ok[node_off[b]:node_off[b + 1]].any() for b in range(B)])
        out = []
        for b, persons in enumerate(per_image):
            if (ok_det is not None and not ok_det[b]) or not (flags[b] & 2) or len(persons) == 0:
                out.append(None)
            else:
                out.append(persons)
        return out

    return GroupingJob(st, finish, background=background)


# ----------------------------------------------------------------------------------------------------
# Finishing (pred_to_ann, Utils.py:1460-1478): filter, fill_mean, refine, adjust
# ----------------------------------------------------------------------------------------------------
def _kp_array(keypoints):
    kp = np.ascontiguousarray(keypoints, dtype=np.float64)
    if kp.ndim != 3 or kp.shape[2] != 3:
        raise ValueError(f"pemp_amd.pose: keypoints must be [P, J, 3], got {kp.shape}")
    return kp


def fill_mean(persons):
    """``Utils.py:1468-1470`` in place on a float64 [P, J, 3] array (host C++)."""
    L = _lib.load_cdll() if _lib._LIB is None else _lib._LIB
    kp = _kp_array(persons)
    _lib.check(L.pemp_pose_fill_mean(kp.ctypes.data, kp.shape[0], kp.shape[1]), L)
    if kp is not persons:
        persons[...] = kp
    return persons


def _check_coords(kp, H, W, name):
    """Detected joints (score > 0) must index inside the [H, W] map: the reference indexes numpy arrays at
    int(x), int(y) there (IndexError past the end; a negative index would wrap around, which pemp rejects
    as well)."""
    # int(v) truncates toward zero: int(v) in [0, n) <=> -1 < v < n, and NaN / inf fail both compares (their int64
    # cast is out of range too); one pass over the coordinates instead of masked copies and casts
    x, y = kp[:, :, 0], kp[:, :, 1]
    if kp.size and kp[:, :, :2].min() > -1 and x.max() < W and y.max() < H:
        return   # every joint inside, detected or not (a NaN fails the compares and takes the full test)
    with np.errstate(invalid="ignore"):
        ok = (x > -1) & (x < W) & (y > -1) & (y < H)
    if not ok[kp[:, :, 2] > 0].all():
        raise IndexError(f"pemp_amd.pose.{name}: a detected keypoint lies outside the {H}x{W} map")


def _maps(t, name, ndim):
    if not (isinstance(t, torch.Tensor) and t.device.type == "cuda"):
        raise ValueError(f"pemp_amd.pose: {name} must be a device tensor (no CPU fallback)")
    t = t.to(torch.float32).contiguous()
    if t.dim() not in ndim:
        raise ValueError(f"pemp_amd.pose: {name} has shape {tuple(t.shape)}")
    return t


def refine(scoremaps, tag, keypoints):
    """``Utils.py:1026-1104``: scoremaps [J,H,W], tag [J,H,W] or [J,H,W,F] (F = 1, 2) device tensors,
    keypoints float64 [P, J, 3] (numpy). Updates keypoints in place and returns it, like the reference."""
    L = _lib.lib()
    s = _maps(scoremaps, "scoremaps", (3,))
    tg = _maps(tag, "tag", (3, 4))
    if tg.dim() == 3:
        tg = tg[..., None]
    J, H, W = s.shape
    F = tg.shape[3]
    if tuple(tg.shape[:3]) != (J, H, W):
        raise ValueError(f"pemp_amd.pose: tag {tuple(tg.shape)} does not match scoremaps {tuple(s.shape)}")
    kp = _kp_array(keypoints)
    if kp.shape[1] != J:
        raise ValueError(f"pemp_amd.pose: keypoints have {kp.shape[1]} joints, scoremaps {J}")
    P = kp.shape[0]
    if P == 0:
        return keypoints
    _check_coords(kp, H, W, "refine")
    d_kp = torch.from_numpy(kp).to(s.device)
    ws = torch.empty(L.pemp_pose_refine_workspace_size(P, J, H, W, F), dtype=torch.uint8, device=s.device)
    _lib.check(L.pemp_pose_refine(s.data_ptr(), tg.data_ptr(), J, H, W, F, d_kp.data_ptr(), P, ws.data_ptr(),
                                  ws.numel(), _lib.stream(s.device)))
    keypoints[...] = d_kp.cpu().numpy()
    return keypoints


def adjust(ans, det):
    """``Utils.py:917-936``: ans float64 [P, J, 3] (numpy, updated in place and returned), det [J,H,W]
    device tensor."""
    L = _lib.lib()
    d = _maps(det, "det", (3,))
    kp = _kp_array(ans)
    J, H, W = d.shape
    if kp.shape[0] == 0:
        return ans
    if kp.shape[1] != J:
        raise ValueError(f"pemp_amd.pose: keypoints have {kp.shape[1]} joints, det {J}")
    _check_coords(kp, H, W, "adjust")
    d_kp = torch.from_numpy(kp).to(d.device)
    _lib.check(L.pemp_pose_adjust(d.data_ptr(), J, H, W, d_kp.data_ptr(), kp.shape[0], _lib.stream(d.device)))
    ans[...] = d_kp.cpu().numpy()
    return ans


def finish_persons(persons, scoremaps, tags, adjustment, with_refine, with_filter=False, fill_mean_=True):
    """The middle of ``pred_to_ann`` (``Utils.py:1460-1478``) for one image's grouped persons: the
    optional max-score filter (> 0.25), fill_mean, refine (only when the first person has a score), adjust.
    Returns the float64 [P, J, 3] array, or None where the reference returns None (all filtered out)."""
    if persons is None:
        return None
    if with_filter:
        keep = persons[:, :, 2].max(axis=1) > 0.25
        persons = persons[keep]
        if persons.shape[0] == 0:
            return None
    persons = np.ascontiguousarray(persons, dtype=np.float64)
    if fill_mean_:
        fill_mean(persons)
    if with_refine and persons[0, :, 2].sum() != 0:
        refine(scoremaps, tags, persons)
    if adjustment:
        adjust(persons, scoremaps)
    return persons


class FinishJob:
    """A batch's finishing queued on the GPU (finish_batch_start): ``result()`` waits for its one read-back (an
    event) and returns the per-image keypoint arrays, as finish_batch does."""

    def __init__(self, out, fill=None):
        self._out, self._fill = out, fill

    def result(self):
        if self._fill is not None:
            ev, back, live, starts = self._fill
            ev.synchronize()
            res = back.numpy()
            for k, b in enumerate(live):
                self._out[b][...] = res[starts[k]:starts[k + 1]]
            self._fill = None
        return self._out


def finish_batch(per_image, scoremaps, tags, adjustment=True, with_refine=False, with_filter=False,
                 fill_mean_=True, stream=None):
    """finish_persons over a batch; see finish_batch_start (this waits for the result)."""
    return finish_batch_start(per_image, scoremaps, tags, adjustment, with_refine, with_filter, fill_mean_,
                              stream).result()


def finish_batch_start(per_image, scoremaps, tags, adjustment=True, with_refine=False, with_filter=False,
                       fill_mean_=True, stream=None):
    """finish_persons over a batch (``pred_to_ann``, ``Utils.py:1460-1478``, once per image): per_image as
    group_persons returns it, scoremaps [B, J, H, W] / tags [B, J, H, W(, F)] device tensors. The filter runs
    per image on the host and fill_mean in one host call over every image's persons (both per person, as the
    reference's per-image loop); then the keypoints and the batch plan (person -> image, refine chunks,
    pemp_pose_finish_plan) go up in one pinned copy, one pemp_pose_finish_batch call queues the refine and
    adjust kernels of all images on `stream` (default: the current stream), and one copy back plus one event
    wait replace the two synchronisations per image of finish_persons. Same results as finish_persons image
    by image; the arrays of per_image are updated in place, as finish_persons does."""
    out = [None if p is None else p for p in per_image]
    for b, persons in enumerate(out):
        if persons is None:
            continue
        if with_filter:
            keep = persons[:, :, 2].max(axis=1) > 0.25
            persons = persons[keep]
            if persons.shape[0] == 0:
                out[b] = None
                continue
        out[b] = np.ascontiguousarray(persons, dtype=np.float64)
    live = [b for b, kp in enumerate(out) if kp is not None and kp.shape[0] > 0]
    if not live:
        return FinishJob(out)
    starts = np.cumsum([0] + [out[b].shape[0] for b in live])
    J0 = out[live[0]].shape[1]
    for b in live:
        if out[b].ndim != 3 or out[b].shape[1:] != (J0, 3):
            raise ValueError(f"pemp_amd.pose: keypoints must be [P, {J0}, 3], got {out[b].shape}")
    kp_all = np.concatenate([out[b] for b in live])
    if fill_mean_:
        fill_mean(kp_all)
        for k, b in enumerate(live):
            out[b][...] = kp_all[starts[k]:starts[k + 1]]
    # (refine only where the image's first person has a score, Utils.py:1471)
    do_ref = (kp_all[starts[:-1], :, 2].sum(axis=1) != 0) if with_refine else np.zeros(len(live), dtype=bool)
    if not (adjustment or do_ref.any()):
        return FinishJob(out)
    L = _lib.lib()
    dev = scoremaps.device
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    d = _maps(scoremaps, "scoremaps", (4,))
    B, J, H, W = d.shape
    if len(out) != B:
        raise ValueError(f"pemp_amd.pose: {len(out)} images of persons for {B} scoremaps")
    if J0 != J:
        raise ValueError(f"pemp_amd.pose: keypoints have {J0} joints, maps {J}")
    tg = None
    if do_ref.any():
        tg = _maps(tags, "tags", (4, 5))
        if tg.dim() == 4:
            tg = tg[..., None]
        if tuple(tg.shape[:4]) != (B, J, H, W):
            raise ValueError(f"pemp_amd.pose: tags {tuple(tg.shape)} do not match scoremaps {tuple(d.shape)}")
    F = tg.shape[4] if tg is not None else 1
    _check_coords(kp_all, H, W, "refine" if with_refine else "adjust")
    P = int(starts[-1])
    counts = np.zeros(B, dtype=np.int32)
    ref = np.zeros(B, dtype=np.uint8)
    counts[live] = np.diff(starts)
    ref[live] = do_ref
    # one pinned buffer: the upload (keypoints | pimg [P] i32 | chunks [3P] i32 | ref [B] u8), then the keypoints'
    # read-back at an 8-byte boundary
    o1 = kp_all.nbytes
    o2 = o1 + 4 * P
    o3 = o2 + 12 * P
    ob = (o3 + B + 7) // 8 * 8
    pin = torch.empty(ob + o1, dtype=torch.uint8, pin_memory=True)
    host = pin[:o3 + B]
    hv = host.numpy()
    hv[:o1] = kp_all.reshape(-1).view(np.uint8)
    hv[o3:] = ref
    plan = np.zeros(2, dtype=np.int32)
    _lib.check(L.pemp_pose_finish_plan(B, counts.ctypes.data, ref.ctypes.data, hv[o1:].ctypes.data,
                                       hv[o2:].ctypes.data, P, plan.ctypes.data), L)
    with torch.cuda.stream(st):
        dbuf = host.to(dev, non_blocking=True)
        base = dbuf.data_ptr()
        ws = None
        if plan[0] > 0:
            ws = torch.empty(L.pemp_pose_refine_workspace_size(P, J, H, W, F), dtype=torch.uint8, device=dev)
        _lib.check(L.pemp_pose_finish_batch(d.data_ptr(), tg.data_ptr() if tg is not None else None, B, J, H, W, F,
                                            base, P, base + o1, base + o2, int(plan[0]), int(plan[1]), base + o3,
                                            int(adjustment), ws.data_ptr() if ws is not None else None,
                                            ws.numel() if ws is not None else 0, _lib.stream(dev)), L)
        back = pin[ob:].view(torch.float64).view(kp_all.shape)
        back.copy_(dbuf[:o1].view(torch.float64).view(kp_all.shape), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(st)
    return FinishJob(out, (ev, back, live, starts))


# ----------------------------------------------------------------------------------------------------
# Back to original image coordinates (pred_to_ann, Utils.py:1479; valid.py:175): reverse_affine_map
# ----------------------------------------------------------------------------------------------------
# Host numpy, like the reference: a few hundred points per image. The 2 x 3 affine of three point pairs
# is cv2.getAffineTransform's (OpenCV is not in this image): the 6 x 6 system of the three
# correspondences solved in float64 (LU with partial pivoting, as cv::getAffineTransform's DECOMP_LU);
# equal to OpenCV's up to the last bits of that solve (parity pinned against the reference's own
# functions with this solve, tests/golden/affine_*.npz; the solve itself unpinned).
def affine_from_points(src, dst):
    """[2, 3] float64 M with dst_i = M [src_i; 1] for the three (float32) point pairs."""
    s = np.asarray(src, dtype=np.float32).astype(np.float64)
    d = np.asarray(dst, dtype=np.float32).astype(np.float64)
    a = np.zeros((6, 6))
    a[0::2, 0:2] = s
    a[0::2, 2] = 1.0
    a[1::2, 3:5] = s
    a[1::2, 5] = 1.0
    return np.linalg.solve(a, d.reshape(6)).reshape(2, 3)


def multi_scale_size(img_h, img_w, input_size, current_scale, min_scale):
    """transformations.py:216-238: ((w, h) of the resized input, centre, scale / 200) -- the input side
    rounded up to multiples of 64, the short side set by min_scale."""
    center = np.array([int(img_w / 2.0 + 0.5), int(img_h / 2.0 + 0.5)])
    side = int((min_scale * input_size + 63) // 64 * 64)
    if img_w < img_h:
        short, long_in, long_ = img_w, img_h, "h"
    else:
        short, long_in, long_ = img_h, img_w, "w"
    s_res = int(side * current_scale / min_scale)
    l_res = int(int((side / short * long_in + 63) // 64 * 64) * current_scale / min_scale)
    if long_ == "h":
        size, scale = (s_res, l_res), np.array([img_w / 200.0, l_res / s_res * img_w / 200.0])
    else:
        size, scale = (l_res, s_res), np.array([l_res / s_res * img_h / 200.0, img_h / 200.0])
    return size, center, scale


def crop_affine(center, scale, output_size, inv=False):
    """transformations.py:170-213 at rotation 0: the map of the box of width 200 * scale[0] centred at
    `center` onto an output_size (w, h) image, from three float32 point pairs (centre, top-centre and
    the point a quarter turn from it)."""
    scale = np.asarray(scale) if isinstance(scale, (np.ndarray, list)) else np.array([scale, scale])
    half_src = (scale * 200.0)[0] * -0.5
    ow, oh = output_size
    src = np.zeros((3, 2), np.float32)
    dst = np.zeros((3, 2), np.float32)
    src[0] = center
    src[1] = center + np.array([0.0 - half_src * 0.0, half_src])   # rotation 0: (0 cos - y sin, 0 sin + y cos)
    dst[0] = [ow * 0.5, oh * 0.5]
    dst[1] = np.array([ow * 0.5, oh * 0.5]) + np.array([0, ow * -0.5], np.float32)
    for p in (src, dst):
        v = p[0] - p[1]
        p[2] = p[1] + np.array([-v[1], v[0]], np.float32)
    return affine_from_points(dst, src) if inv else affine_from_points(src, dst)


def box_transform(center, scale, res):
    """transformations.py:142-167 at rotation 0: the 3 x 3 float64 map of the box (200 * scale) around
    `center` onto a res = (h, w) grid."""
    h = 200 * np.asarray(scale)
    t = np.zeros((3, 3))
    t[0, 0] = float(res[1]) / h[1]
    t[1, 1] = float(res[0]) / h[0]
    t[0, 2] = res[1] * (-float(center[0]) / h[0] + .5)
    t[1, 2] = res[0] * (-float(center[1]) / h[1] + .5)
    t[2, 2] = 1
    return t


def apply_affine(points, mat):
    """transformations.py:131-135: [..., 2] points through a [2, 3] matrix (homogeneous, float64)."""
    p = np.array(points)
    flat = p.reshape(-1, 2)
    return np.dot(np.concatenate((flat, flat[:, 0:1] * 0 + 1), axis=1), mat.T).reshape(p.shape)


def reverse_affine_map(keypoints, img_size_orig, input_size, scaling_type, min_scale=1.0):
    """``reverse_affine_map`` (src/Utils/transformations.py:7-77): keypoints [P, J, >=2] in network output
    space -> original image coordinates, in place (returned), for scaling_type "short" (heatmaps at half
    the input size), "short_with_resize" (PROJECT2IMAGE), "long" and "long_with_multiscale" (x4 output
    stride, 512 input). img_size_orig = (width, height). Raises NotImplementedError otherwise, as the
    reference ("short_mine" needs a helper missing from the reference itself)."""
    w0, h0 = img_size_orig[0], img_size_orig[1]
    if scaling_type not in ("short", "short_with_resize", "long", "long_with_multiscale"):
        raise NotImplementedError(f"reverse_affine_map: scaling_type={scaling_type!r}")
    mat = _reverse_matrix(w0, h0, input_size, scaling_type, min_scale)
    pts = keypoints[:, :, :2] * 4 if scaling_type in ("long", "long_with_multiscale") else keypoints[:, :, :2]
    keypoints[:, :, :2] = apply_affine(pts, mat)
    return keypoints


@functools.lru_cache(maxsize=256)
def _reverse_matrix(w0, h0, input_size, scaling_type, min_scale):
    """The [2, 3] map of reverse_affine_map for one image size (the same matrix for every image of that size, so it
    is solved once: the 6 x 6 solve was most of the call's time)."""
    if scaling_type in ("short", "short_with_resize"):
        size, center, scale = multi_scale_size(h0, w0, input_size, 1.0, min_scale)
        out = (int(size[0] / 2), int(size[1] / 2)) if scaling_type == "short" else (int(size[0]), int(size[1]))
        mat = crop_affine(center, scale, out, inv=True)
    else:
        if input_size != 512:
            raise AssertionError("reverse_affine_map: 'long' scaling needs input_size 512")
        s = max(h0, w0) / 200
        res = (512, 512) if scaling_type == "long" else (1024, 1024)
        mat = np.linalg.pinv(box_transform(np.array((w0 / 2, h0 / 2)), np.array([s, s]), res))[:2]
    mat.setflags(write=False)
    return mat
