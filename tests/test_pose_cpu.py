"""Pose grouping, CPU side.

* the oracle (oracle/pose.py) against the golden vectors made by the reference's own functions;
* the library's HOST entry points (pemp_pose_cluster: GAEC / threshold components; pemp_pose_persons:
  graph_cluster_to_persons) against the oracle and the golden vectors. These two are plain C++ (no HIP
  call), so they run here; the GPU edge pass that feeds them is restated below in numpy as test input
  only and is checked against the real kernel by tests/test_gpu_pose.py.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import pose as opose
from pemp_amd import _lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("pose_") and f.endswith(".npz"))
REFINE = [c for c in CASES if c.startswith("pose_refine")]
GROUP = [c for c in CASES if not c.startswith("pose_refine")]


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def edge_pass(ei, pred, scores, th, use_th, node_off, method):
    """numpy statement of pemp_pose_edge_weights (test input only)."""
    E = ei.shape[1]
    B = len(node_off) - 1
    w = np.full(E, np.nan, np.float32)
    flags = np.zeros(B + 1, np.int32)
    keep = np.ones(E, bool) if not use_th else (scores[ei[0]] > th) & (scores[ei[1]] > th)
    img = np.searchsorted(node_off, ei[0], side="right") - 1
    pos = {(int(s), int(d)): i for i, (s, d) in enumerate(ei.T)}
    for e in np.nonzero(keep)[0]:
        s, d = int(ei[0, e]), int(ei[1, e])
        flags[img[e]] |= 2
        if s > d and pred[e] != 0:
            flags[img[e]] |= 1
        if method == 1:
            w[e] = pred[e]
        elif s < d:
            r = pos.get((d, s))
            w[e] = np.float32(pred[e] + (pred[r] if r is not None else np.float32(0)))
    return w, flags


def host_group(det, scores, ei, pred, cls, J, node_off, th, use_th, method, pose_scores=None, allow_single=False):
    L = _lib.load_cdll()
    w, flags = edge_pass(ei, pred, scores, th, use_th, node_off, method)
    B, N = len(node_off) - 1, len(det)
    labels = np.empty(N, np.int32)
    ncomp = np.empty(B, np.int32)
    ei = np.ascontiguousarray(ei, np.int64)
    rc = L.pemp_pose_cluster(B, node_off.ctypes.data, ei.ctypes.data, ei.shape[1], w.ctypes.data, flags.ctypes.data,
                             method, 4, labels.ctypes.data, ncomp.ctypes.data)
    _lib.check(rc, L)
    cap = max(N, 1)
    persons = np.empty((cap, J, 3))
    counts = np.empty(B, np.int32)
    mut = np.empty(B, np.int32)
    det = np.ascontiguousarray(det, np.int64)
    scores = np.ascontiguousarray(scores, np.float32)
    cls_p = None if cls is None else np.ascontiguousarray(cls, np.float32).ctypes.data
    ps_p = None if pose_scores is None else np.ascontiguousarray(pose_scores, np.float32).ctypes.data
    rc = L.pemp_pose_persons(B, node_off.ctypes.data, labels.ctypes.data, ncomp.ctypes.data, det.ctypes.data,
                             scores.ctypes.data, ps_p, cls_p, J, int(allow_single), cap, persons.ctypes.data,
                             counts.ctypes.data, mut.ctypes.data)
    _lib.check(rc, L)
    st = np.concatenate([[0], np.cumsum(counts)])
    return [persons[st[b]:st[b + 1]] for b in range(B)], labels, flags, mut


def method_of(g):
    return {"GAEC": 0, "threshold": 1}[str(g["method"])]


@pytest.mark.parametrize("name", GROUP)
def test_oracle_matches_reference_fixture(name):
    g = load(name)
    cls = g["class_probs"] if g["has_class"] else None
    got = opose.pred_to_ann_persons(g["joint_det"], g["joint_scores"], g["edge_index"], g["pred"], g["th"], cls,
                                    str(g["method"]), int(g["num_joints"]), g["joint_scores"])
    assert (got is None) == bool(g["none"])
    if got is not None:
        np.testing.assert_array_equal(got, g["persons"])


@pytest.mark.parametrize("name", GROUP)
def test_host_grouping_matches_reference_fixture(name):
    g = load(name)
    J = int(g["num_joints"])
    cls = g["class_probs"] if g["has_class"] else None
    N = len(g["joint_det"])
    off = np.array([0, N], np.int64)
    persons, _, flags, _ = host_group(g["joint_det"], g["joint_scores"], g["edge_index"], g["pred"], cls, J, off,
                                      float(g["th"]), True, method_of(g))
    if g["none"]:
        assert not (flags[0] & 2) or len(persons[0]) == 0
    else:
        np.testing.assert_array_equal(persons[0], g["persons"])
    # graph_cluster_to_persons with single-joint persons and pose scores, on the unthresholded graph's
    # GAEC solution restricted to the thresholded subgraph (as the generator built it)
    ei_s, p_s = opose.subgraph(g["joint_scores"] > g["th"], g["edge_index"], g["pred"])
    persons, labels, _, mut = host_group(g["joint_det"], g["joint_scores"], ei_s, p_s, cls, J, off, 0.0, False, 0,
                                         pose_scores=g["pose_scores"], allow_single=True)
    np.testing.assert_array_equal(persons[0].reshape(-1, J, 3), g["single_persons"])
    np.testing.assert_array_equal(labels, g["single_labels"])
    assert bool(mut[0]) == bool(g["single_mutant"])


def test_host_grouping_batched_equals_per_image():
    gs = [load(n) for n in GROUP if str(load(n)["method"]) == "GAEC" and int(load(n)["num_joints"]) == 17]
    dets, scs, eis, prs, clss, offs = [], [], [], [], [], [0]
    for g in gs:
        n = len(g["joint_det"])
        dets.append(g["joint_det"])
        scs.append(g["joint_scores"])
        eis.append(g["edge_index"] + offs[-1])
        prs.append(g["pred"])
        clss.append(g["class_probs"] if g["has_class"] else np.eye(17, dtype=np.float32)[g["joint_det"][:, 2]])
        offs.append(offs[-1] + n)
    off = np.array(offs, np.int64)
    persons, _, _, _ = host_group(np.concatenate(dets), np.concatenate(scs), np.concatenate(eis, 1),
                                  np.concatenate(prs), np.concatenate(clss), 17, off, 0.1, True, 0)
    for b, g in enumerate(gs):
        cls = g["class_probs"] if g["has_class"] else np.eye(17, dtype=np.float32)[g["joint_det"][:, 2]]
        ref = opose.pred_to_ann_persons(g["joint_det"], g["joint_scores"], g["edge_index"], g["pred"],
                                        np.float32(0.1), cls, "GAEC", 17)
        np.testing.assert_array_equal(persons[b], ref if ref is not None else np.zeros((0, 17, 3)))


@pytest.mark.parametrize("dense", [True, False])
@pytest.mark.parametrize("seed", range(12))
def test_gaec_matches_oracle_random_with_ties(seed, dense, monkeypatch):
    """C++ GAEC == the libstdc++-heap restatement, incl. weight ties (quantised weights) and repeated
    contractions; labels compared exactly. Both adjacency forms (dense rows and std::map)."""
    monkeypatch.setenv("PEMP_GAEC_DENSE_MAX", "4096" if dense else "0")
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(2, 70)) if seed < 10 else 220
    dens = rng.uniform(0.1, 1.0)
    up = np.triu(rng.random((n, n)) < dens, 1)
    s, d = np.nonzero(up | up.T)
    ei = np.stack([s, d]).astype(np.int64)
    q = [0, 4, 16][seed % 3]
    pred = rng.random(ei.shape[1]).astype(np.float32)
    if q:
        pred = (np.round(pred * q) / q).astype(np.float32)
    det = np.stack([rng.integers(0, 640, n), rng.integers(0, 640, n), rng.integers(0, 17, n)], 1)
    scores = rng.random(n).astype(np.float32)
    off = np.array([0, n], np.int64)
    _, labels, _, _ = host_group(det, scores, ei, pred, None, 17, off, 0.0, False, 0)
    if ei.shape[1]:
        sol = opose.cluster_gaec(n, ei, pred)
    else:
        sol = np.eye(n, dtype=np.int64)
    _, _, ref_labels = opose.graph_cluster_to_persons(det, scores, np.stack(np.nonzero(sol)), None, 17)
    np.testing.assert_array_equal(labels, ref_labels)


@pytest.mark.parametrize("n,persons,quant", [(153, 9, 0), (60, 4, 0), (231, 13, 0), (90, 5, 64), (40, 3, 8)])
def test_gaec_fast_path_equals_full_heap(n, persons, quant, monkeypatch):
    """The non-negative-heap GAEC (gaec_fast) against the full libstdc++-heap GAEC (PEMP_GAEC_EXACT) on
    person-structured fully graphs (bench.py's synthetic probabilities), batched; quantised probabilities make
    equal weights, where the fast path hands over to the full heap. Labels must be identical, and equal to the
    oracle's restatement of andres' GAEC."""
    rng = np.random.default_rng(n + quant)
    B = 3
    dets, scs, eis, prs, offs = [], [], [], [], [0]
    for b in range(B):
        s, d = np.nonzero(~np.eye(n, dtype=bool))
        same = (s % persons) == (d % persons)
        p = (1 / (1 + np.exp(-(np.where(same, 2.5, -2.5) + 1.5 * rng.standard_normal(s.size))))).astype(np.float32)
        if quant:
            p = (np.round(p * quant) / quant).astype(np.float32)
        dets.append(np.stack([rng.integers(0, 640, n), rng.integers(0, 640, n), np.arange(n) % 17], 1))
        scs.append(rng.uniform(0.2, 1.0, n).astype(np.float32))
        eis.append(np.stack([s, d]).astype(np.int64) + offs[-1])
        prs.append(p)
        offs.append(offs[-1] + n)
    args = (np.concatenate(dets), np.concatenate(scs), np.concatenate(eis, 1), np.concatenate(prs), None, 17,
            np.array(offs, np.int64), 0.0, False, 0)
    _, fast, _, _ = host_group(*args)
    monkeypatch.setenv("PEMP_GAEC_EXACT", "1")
    _, full, _, _ = host_group(*args)
    np.testing.assert_array_equal(fast, full)
    for b in range(B):
        sl = slice(offs[b], offs[b + 1])
        ei = eis[b] - offs[b]
        sol = opose.cluster_gaec(n, ei, prs[b])
        _, _, ref = opose.graph_cluster_to_persons(dets[b], scs[b], np.stack(np.nonzero(sol)), None, 17)
        np.testing.assert_array_equal(fast[sl], ref)


def test_unsorted_edge_index_is_refused():
    L = _lib.load_cdll()
    flags = np.array([2, 1], np.int32)   # image 0 keeps edges; flags[B] bit 0: unsorted
    off = np.array([0, 3], np.int64)
    ei = np.array([[0, 1], [1, 0]], np.int64)
    w = np.zeros(2, np.float32)
    labels = np.empty(3, np.int32)
    nc = np.empty(1, np.int32)
    rc = L.pemp_pose_cluster(1, off.ctypes.data, ei.ctypes.data, 2, w.ctypes.data, flags.ctypes.data, 0, 1,
                             labels.ctypes.data, nc.ctypes.data)
    with pytest.raises(ValueError, match="sorted"):
        _lib.check(rc, L)


@pytest.mark.parametrize("name", REFINE)
def test_oracle_refine_adjust_fixture(name):
    g = load(name)
    filled = opose.fill_mean(g["keypoints"].copy())
    np.testing.assert_array_equal(filled, g["filled"])
    refined = opose.refine(g["scoremaps"], g["tag"], filled.copy())
    np.testing.assert_array_equal(refined, g["refined"])
    np.testing.assert_array_equal(opose.adjust(refined.copy(), g["scoremaps"]), g["adjusted"])


@pytest.mark.parametrize("name", REFINE)
def test_host_fill_mean_fixture(name):
    from pemp_amd import pose as ppose
    g = load(name)
    kp = g["keypoints"].copy()
    ppose.fill_mean(kp)
    np.testing.assert_array_equal(kp, g["filled"])


GREEDY = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("greedy_") and f.endswith(".npz"))


@pytest.mark.parametrize("name", GREEDY)
def test_greedy_oracle_and_host_fixture(name):
    """greedy_person_construction: oracle and pemp_pose_greedy (host C++) against the reference's own
    function's output (pred_to_ann prefix with cc_method "greedy")."""
    g = load(name)
    J = int(g["num_joints"])
    cls = g["class_probs"] if g["has_class"] else None
    ei_s, p_s = opose.subgraph(g["joint_scores"] > g["th"], g["edge_index"], g["pred"])
    persons, taken = opose.greedy_person_construction(g["joint_det"], g["joint_scores"], p_s, cls, ei_s, J)
    np.testing.assert_array_equal(taken, g["taken"])
    if not g["none"]:
        np.testing.assert_array_equal(persons, g["persons"])
    # host C++ on the edge pass (method 1: surviving preds, NaN elsewhere)
    L = _lib.load_cdll()
    N = len(g["joint_det"])
    off = np.array([0, N], np.int64)
    ei = np.ascontiguousarray(g["edge_index"], np.int64)
    w, _ = edge_pass(ei, g["pred"], g["joint_scores"], g["th"], True, off, 1)
    tk = np.empty(N, np.int32)
    out = np.empty((N, J, 3))
    cnt = np.empty(1, np.int32)
    det = np.ascontiguousarray(g["joint_det"], np.int64)
    sc = np.ascontiguousarray(g["joint_scores"], np.float32)
    cls_p = None if cls is None else np.ascontiguousarray(cls, np.float32).ctypes.data
    _lib.check(L.pemp_pose_greedy(1, off.ctypes.data, ei.ctypes.data, ei.shape[1], w.ctypes.data, det.ctypes.data,
                                  sc.ctypes.data, cls_p, J, tk.ctypes.data, N, out.ctypes.data, cnt.ctypes.data), L)
    np.testing.assert_array_equal(tk, g["taken"])
    np.testing.assert_array_equal(out[:cnt[0]], g["persons"])


def test_pose_product_path_has_no_cpu_fallback():
    """group_persons / pred_to_person / refine need the HIP device: on a host without one they raise instead
    of computing on the CPU (the host C++ parts above are only reachable through the GPU edge pass)."""
    import torch
    from pemp_amd import pose as ppose
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    g = load(GROUP[0])
    T = torch.from_numpy
    with pytest.raises((RuntimeError, ValueError)):
        ppose.group_persons(T(g["joint_det"]), T(g["joint_scores"]), T(g["edge_index"]), T(g["pred"]), 0.1)
    with pytest.raises((RuntimeError, ValueError)):
        ppose.pred_to_person(T(g["joint_det"]), T(g["joint_scores"]), T(g["edge_index"]), T(g["pred"]), None,
                             "GAEC", 17)
    r = load(REFINE[0])
    with pytest.raises((RuntimeError, ValueError)):
        ppose.refine(T(r["scoremaps"]), T(r["tag"]), r["filled"].copy())
    with pytest.raises(NotImplementedError):
        ppose._method("MUT")


def test_reverse_affine_map_golden():
    """pemp_amd.pose.reverse_affine_map against the reference's own transformations.py functions
    (oracle/gen_golden_affine.py; cv2.getAffineTransform stubbed by its 6x6 float64 solve)."""
    from pemp_amd import pose as ppose
    g = np.load(os.path.join(GOLDEN, "affine_maps.npz"))
    for c, spec in enumerate(g["cases"]):
        w, h, size, kind, ms = str(spec).split(",")
        got = ppose.reverse_affine_map(g[f"in_{c}"].copy(), (int(w), int(h)), int(size), kind, float(ms))
        np.testing.assert_array_equal(got, g[f"out_{c}"])
    with pytest.raises(NotImplementedError):
        ppose.reverse_affine_map(np.zeros((1, 17, 3)), (640, 480), 512, "short_mine")


def test_finish_plan_chunks():
    """pemp_pose_finish_plan (host): person -> image map, refine chunks of one image each, covering exactly the
    persons of the refined images, all chunks pc wide but an image's last."""
    from pemp_amd import _lib
    L = _lib.load_cdll() if _lib._LIB is None else _lib._LIB
    counts = np.array([0, 37, 3, 2, 1, 9, 16], dtype=np.int32)
    ref = np.array([1, 1, 1, 0, 1, 1, 0], dtype=np.uint8)
    P = int(counts.sum())
    pimg = np.full(P, -1, dtype=np.int32)
    chunks = np.full(3 * P, -1, dtype=np.int32)
    out2 = np.zeros(2, dtype=np.int32)
    assert L.pemp_pose_finish_plan(len(counts), counts.ctypes.data, ref.ctypes.data, pimg.ctypes.data,
                                   chunks.ctypes.data, P, out2.ctypes.data) == 0
    np.testing.assert_array_equal(pimg, np.repeat(np.arange(len(counts)), counts))
    n, pc = int(out2[0]), int(out2[1])
    assert pc in (2, 4, 6, 8, 10, 12, 16) and pc >= (37 + 2) // 3
    c = chunks[:3 * n].reshape(n, 3)
    starts = np.concatenate([[0], np.cumsum(counts)])
    covered = np.zeros(P, dtype=int)
    for p0, np_, b in c:
        assert ref[b] and 1 <= np_ <= pc and starts[b] <= p0 and p0 + np_ <= starts[b + 1]
        covered[p0:p0 + np_] += 1
    np.testing.assert_array_equal(covered, np.repeat(ref.astype(int), counts))
    assert L.pemp_pose_finish_plan(len(counts), counts.ctypes.data, ref.ctypes.data, pimg.ctypes.data,
                                   chunks.ctypes.data, 3, out2.ctypes.data) != 0   # max_chunks too small


def test_check_coords_matches_int_indexing():
    """pose._check_coords (refine / adjust: every detected joint must index the map at int(x), int(y), Utils.py:1096)
    accepts exactly the keypoints whose truncated coordinates lie in [0, W) x [0, H): borders, values in (-1, 0),
    NaN / inf, undetected joints outside the map."""
    from pemp_amd import pose as pp

    def reference(kp, H, W):   # the masked int casts the check replaces
        live = kp[:, :, 2] > 0
        with np.errstate(invalid="ignore"):
            x = kp[:, :, 0][live].astype(np.int64)
            y = kp[:, :, 1][live].astype(np.int64)
        return not ((x < 0).any() or (x >= W).any() or (y < 0).any() or (y >= H).any())

    rng = np.random.default_rng(5)
    H, W = 48, 64
    specials = [-1.0, -0.999, -0.5, -0.0, 0.0, W - 0.5, W - 1e-9, W, W + 0.5, H - 0.5, H, np.nan, np.inf, -np.inf]
    for trial in range(300):
        kp = np.stack([rng.uniform(-2, W + 2, (3, 5)), rng.uniform(-2, H + 2, (3, 5)),
                       (rng.random((3, 5)) > 0.5).astype(np.float64)], -1)
        if trial % 3 == 0:
            kp[:, :, 0] = rng.uniform(0, W - 1, (3, 5))
            kp[:, :, 1] = rng.uniform(0, H - 1, (3, 5))
        for _ in range(trial % 4):
            kp[rng.integers(3), rng.integers(5), rng.integers(2)] = specials[rng.integers(len(specials))]
        try:
            pp._check_coords(kp, H, W, "test")
            got = True
        except IndexError:
            got = False
        assert got == reference(kp, H, W), kp
