"""GPU parity of pose grouping: pemp_amd.pose (HIP edge pass + native GAEC and person
assembly) against the golden vectors made by the reference's own functions and against the oracle on the
same inputs. Bit-exact: persons are integer positions and copied fp32 scores; labels are integers."""
import numpy as np
import pytest
import torch

import pemp_amd
from oracle import pose as opose, restate
from pemp_amd import _lib, config as pcfg, pose as ppose, synthetic as syn
from tests.test_pose_cpu import GROUP, REFINE, edge_pass, load

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("name", GROUP)
def test_group_persons_golden(name):
    g = load(name)
    cls = dev(g["class_probs"]) if g["has_class"] else None
    out = ppose.group_persons(dev(g["joint_det"]), dev(g["joint_scores"]), dev(g["edge_index"]), dev(g["pred"]),
                              float(g["th"]), cls, str(g["method"]), int(g["num_joints"]),
                              score_map_scores=dev(g["joint_scores"]))
    assert len(out) == 1
    if g["none"]:
        assert out[0] is None
    else:
        np.testing.assert_array_equal(out[0], g["persons"])


@pytest.mark.parametrize("name", GROUP)
def test_pred_to_person_golden(name):
    g = load(name)
    J = int(g["num_joints"])
    cls = dev(g["class_probs"]) if g["has_class"] else None
    ei_s, p_s = opose.subgraph(g["joint_scores"] > g["th"], g["edge_index"], g["pred"])
    persons, mutant, labels = ppose.pred_to_person(dev(g["joint_det"]), dev(g["joint_scores"]), dev(ei_s), dev(p_s),
                                                   cls, "GAEC", J, score_for_poses=dev(g["pose_scores"]),
                                                   allow_single_joint_persons=True)
    np.testing.assert_array_equal(np.asarray(persons).reshape(-1, J, 3), g["single_persons"])
    np.testing.assert_array_equal(labels, g["single_labels"])
    assert mutant == bool(g["single_mutant"])


@pytest.mark.parametrize("method", [0, 1])
def test_edge_pass_kernel_bits(method):
    """pemp_pose_edge_weights == its numpy statement, bit for bit (NaN positions included), on a batch of
    three fixture graphs; flags per image."""
    gs = [load(n) for n in GROUP[:3]]
    eis, prs, scs, offs = [], [], [], [0]
    for g in gs:
        eis.append(g["edge_index"] + offs[-1])
        prs.append(g["pred"])
        scs.append(g["joint_scores"])
        offs.append(offs[-1] + len(g["joint_det"]))
    ei, pr, sc, off = np.concatenate(eis, 1), np.concatenate(prs), np.concatenate(scs), np.array(offs, np.int64)
    E, B = ei.shape[1], len(gs)
    w = torch.empty(E, dtype=torch.float32, device=DEV)
    flags = torch.empty(B + 1, dtype=torch.int32, device=DEV)
    L = _lib.lib()
    d_ei, d_pr, d_sc, d_off = dev(ei), dev(pr), dev(sc), dev(off)
    rs = torch.empty(int(off[-1]) + 1, dtype=torch.int64, device=DEV)
    _lib.check(L.pemp_pose_edge_weights(d_ei.data_ptr(), E, d_pr.data_ptr(), d_sc.data_ptr(), 0.3, 1,
                                        d_off.data_ptr(), B, int(off[-1]), method, rs.data_ptr(), w.data_ptr(),
                                        flags.data_ptr(), _lib.stream(DEV)))
    ref_w, ref_flags = edge_pass(ei, pr, sc, np.float32(0.3), True, off, method)
    np.testing.assert_array_equal(w.cpu().numpy().view(np.int32), ref_w.view(np.int32))
    np.testing.assert_array_equal(flags.cpu().numpy(), ref_flags)
    # an unsorted edge list is flagged and refused by the grouping
    bad = ei[:, ::-1].copy()
    with pytest.raises(ValueError, match="sorted"):
        ppose.group_persons(dev(np.zeros((off[-1], 3), np.int64)), dev(sc), dev(bad), dev(pr), 0.3,
                            batch_index=dev(np.repeat(np.arange(B), np.diff(off))), num_images=B)


def test_group_persons_batched():
    gs = [load(n) for n in GROUP if str(load(n)["method"]) == "GAEC" and int(load(n)["num_joints"]) == 17]
    dets, scs, eis, prs, clss, bis = [], [], [], [], [], []
    base = 0
    for b, g in enumerate(gs):
        n = len(g["joint_det"])
        dets.append(g["joint_det"])
        scs.append(g["joint_scores"])
        eis.append(g["edge_index"] + base)
        prs.append(g["pred"])
        clss.append(g["class_probs"] if g["has_class"] else np.eye(17, dtype=np.float32)[g["joint_det"][:, 2]])
        bis.append(np.full(n, b, np.int64))
        base += n
    out = ppose.group_persons(dev(np.concatenate(dets)), dev(np.concatenate(scs)), dev(np.concatenate(eis, 1)),
                              dev(np.concatenate(prs)), 0.1, dev(np.concatenate(clss)), "GAEC", 17,
                              batch_index=dev(np.concatenate(bis)), num_images=len(gs))
    assert len(out) == len(gs)
    for b, g in enumerate(gs):
        cls = g["class_probs"] if g["has_class"] else np.eye(17, dtype=np.float32)[g["joint_det"][:, 2]]
        ref = opose.pred_to_ann_persons(g["joint_det"], g["joint_scores"], g["edge_index"], g["pred"],
                                        np.float32(0.1), cls, "GAEC", 17)
        if ref is None:
            assert out[b] is None
        else:
            np.testing.assert_array_equal(out[b], ref)


@pytest.mark.parametrize("method,graph,persons", [("GAEC", "fully", 3), ("threshold", "fully", 3),
                                                   ("GAEC", "knn", 5), ("greedy", "knn", 5)])
def test_end_to_end_after_mpn(method, graph, persons):
    """construct_graph -> MPN -> sigmoid/softmax (valid.py:109-111) -> group_persons on the GPU, against
    the oracle's pred_to_ann prefix on the SAME probabilities (copied to the host). The knn case (85
    nodes per image, k = 50) exercises a graph that is not complete."""
    B, J, H, W = 2, 17, 128, 128
    hm = torch.from_numpy(syn.make_heatmaps(5, B, J, H, W, persons=persons))
    feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25))
    gc = pcfg.inference_gc_config(graph, 5, False)
    out = pemp_amd.get_graph_constructor(gc, scoremaps=hm.to(DEV), features=feats.to(DEV), tagmaps=None,
                                         joints_gt=None, factor_list=None, masks=None, device=DEV, testing=True,
                                         heatmaps=None, num_joints=J).construct_graph()
    x, ea, ei, det, sc, bi = out[0], out[1], out[2], out[7], out[11], out[12]
    mcfg = pcfg.published_mpn_config(J, steps=3, variant="attn")
    model = pemp_amd.get_mpn_model(mcfg)
    model.load_state_dict(syn.closed_form_state_dict(model, 0.5))
    model.eval().to(DEV)
    with torch.no_grad():
        pe, pn, pc, _ = model(x, ea, ei, node_types=det[:, 2])
    pe, pn, pc = pe[-1].sigmoid().squeeze(), pn[-1].sigmoid(), pc[-1].softmax(dim=1)
    got = ppose.group_persons(det, pn, ei, pe, 0.1, pc, method, J, batch_index=bi, score_map_scores=sc,
                              num_images=B)
    h = [t.cpu().numpy() for t in (det, pn, ei, pe, pc, bi, sc)]
    for b in range(B):
        nm = h[5] == b
        lo = int(np.nonzero(nm)[0][0])
        em = nm[h[2][0]]
        if method == "greedy":
            ei_s, p_s = opose.subgraph(h[1][nm] > np.float32(0.1), h[2][:, em] - lo, h[3][em])
            ref, _ = opose.greedy_person_construction(h[0][nm], h[1][nm], p_s, h[4][nm], ei_s, J)
            ref = None if ref.ndim == 1 or not (h[6][nm] > 0.1).any() or ei_s.shape[1] == 0 else ref
        else:
            ref = opose.pred_to_ann_persons(h[0][nm], h[1][nm], h[2][:, em] - lo, h[3][em], np.float32(0.1),
                                            h[4][nm], method, J, h[6][nm])
        if ref is None:
            assert got[b] is None
        else:
            np.testing.assert_array_equal(got[b], ref)


@pytest.mark.parametrize("name", REFINE)
def test_refine_adjust_golden(name):
    """pemp_pose_refine / pemp_pose_adjust against the reference's own refine / adjust (bit-exact float64
    keypoints; the per-person float32 mean tag follows numpy's summation order)."""
    g = load(name)
    s, tag = dev(g["scoremaps"]), dev(g["tag"])
    kp = g["filled"].copy()
    out = ppose.refine(s, tag, kp)
    assert out is kp
    np.testing.assert_array_equal(kp, g["refined"])
    ppose.adjust(kp, s)
    np.testing.assert_array_equal(kp, g["adjusted"])


def test_finish_persons_matches_oracle():
    g = load(REFINE[0])
    s, tag = dev(g["scoremaps"]), dev(g["tag"])
    got = ppose.finish_persons(g["keypoints"].copy(), s, tag, adjustment=True, with_refine=True, with_filter=True)
    ref = g["keypoints"].copy()
    ref = ref[ref[:, :, 2].max(axis=1) > 0.25]
    ref = opose.adjust(opose.refine(g["scoremaps"], g["tag"], opose.fill_mean(ref)), g["scoremaps"])
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("F", [1, 2])
@pytest.mark.parametrize("seed", range(12))
def test_refine_rounding_boundaries(F, seed):
    """Tag distances placed within a few ulp of half-integers (where rint(sqrt) flips): the refined
    position of an undetected joint must match numpy (oracle) exactly."""
    rng = np.random.default_rng(seed)
    J, H, W = 2, 8, 128
    m = np.float32(rng.uniform(-1, 1))
    tag = np.full((J, H, W, F), m, np.float32)
    k = rng.integers(0, 4, size=(H, W)).astype(np.float32) + np.float32(0.5)
    ulps = rng.integers(-4, 5, size=(H, W))
    d = np.nextafter(k, np.where(ulps > 0, np.float32(np.inf), np.float32(-np.inf)))
    d = np.where(ulps == 0, k, d).astype(np.float32)
    if F == 2:
        # the two components put ||.|| within a few ulp of the half-integer; the small second component
        # moves the sum by sub-ulp amounts, so the correctly rounded sqrt lands on either side
        if seed % 2:
            tag[1, :, :, 0] = m + d
            tag[1, :, :, 1] = m + (rng.integers(0, 64, size=(H, W)) * np.float32(2.0 ** -12)).astype(np.float32)
        else:
            tag[1, :, :, 0] = m + d * np.float32(0.6)
            tag[1, :, :, 1] = m + d * np.float32(0.8)
    else:
        tag[1, :, :, 0] = m + d
    s = (rng.random((J, H, W)) * 0.01).astype(np.float32)
    kp = np.zeros((1, J, 3))
    kp[0, 0] = (3, 2, 0.9)
    tg = tag if F == 2 else tag[..., 0]
    ref = opose.refine(s, tg, kp.copy())
    got = ppose.refine(dev(s), dev(tg), kp.copy())
    np.testing.assert_array_equal(got, ref)


from tests.test_pose_cpu import GREEDY  # noqa: E402


@pytest.mark.parametrize("name", GREEDY)
def test_greedy_golden(name):
    g = load(name)
    J = int(g["num_joints"])
    cls = dev(g["class_probs"]) if g["has_class"] else None
    out = ppose.group_persons(dev(g["joint_det"]), dev(g["joint_scores"]), dev(g["edge_index"]), dev(g["pred"]),
                              float(g["th"]), cls, "greedy", J, score_map_scores=dev(g["joint_scores"]))
    if g["none"]:
        assert out[0] is None
    else:
        np.testing.assert_array_equal(out[0], g["persons"])
    ei_s, p_s = opose.subgraph(g["joint_scores"] > g["th"], g["edge_index"], g["pred"])
    persons, mutant, taken = ppose.pred_to_person(dev(g["joint_det"]), dev(g["joint_scores"]), dev(ei_s), dev(p_s),
                                                  cls, "greedy", J)
    np.testing.assert_array_equal(taken, g["taken"])
    assert mutant is False


@pytest.mark.parametrize("mode", ["some", "all"])
def test_refine_tag_distance_overflow(mode):
    """|tag - mean| so large that its square overflows (numpy: inf, so s - inf = -inf): those pixels never
    win, and when every pixel overflows the first pixel is the argmax, as np.argmax of all -inf."""
    rng = np.random.default_rng(3)
    J, H, W = 2, 8, 96
    tag = np.zeros((J, H, W), np.float32)
    big = np.float32(3e19)
    if mode == "all":
        tag[1] = big
    else:
        tag[1] = np.where(rng.random((H, W)) < 0.5, big, rng.normal(0, 2, (H, W))).astype(np.float32)
    s = rng.random((J, H, W)).astype(np.float32)
    kp = np.zeros((1, J, 3))
    kp[0, 0] = (5, 4, 0.9)
    with np.errstate(over="ignore"):
        ref = opose.refine(s, tag, kp.copy())
    got = ppose.refine(dev(s), dev(tag), kp.copy())
    np.testing.assert_array_equal(got, ref)


def test_group_persons_empty_cases():
    """pred_to_ann's None returns: an image without detections, an image whose nodes all fall below the node
    threshold, and an image without edges, next to a normal one in the same batch; also an empty batch."""
    g = load(GROUP[0])
    n = len(g["joint_det"])
    det = np.concatenate([g["joint_det"], g["joint_det"][:1], g["joint_det"]])
    sc = np.concatenate([g["joint_scores"], np.float32([0.9]), np.zeros(n, np.float32)])
    ei = np.concatenate([g["edge_index"], g["edge_index"] + n + 1], 1)
    pr = np.concatenate([g["pred"], g["pred"]])
    bi = np.concatenate([np.zeros(n, np.int64), np.full(1, 2, np.int64), np.full(n, 3, np.int64)])
    cls = np.concatenate([g["class_probs"], g["class_probs"][:1], g["class_probs"]])
    # images: 0 normal, 1 no detections, 2 one node / no edges, 3 all nodes below threshold, 4 and 5 no
    # detections (trailing: no batch_index entry, counted only by num_images)
    out = ppose.group_persons(dev(det), dev(sc), dev(ei), dev(pr), float(g["th"]), dev(cls), "GAEC",
                              int(g["num_joints"]), batch_index=dev(bi), num_images=6)
    assert len(out) == 6
    np.testing.assert_array_equal(out[0], g["persons"])
    assert all(o is None for o in out[1:])
    # the normal image last (index 3), after an empty image 0, a one-node image 1 and an empty image 2
    out = ppose.group_persons(dev(np.concatenate([g["joint_det"][:1], g["joint_det"]])),
                              dev(np.concatenate([np.float32([0.9]), g["joint_scores"]])), dev(g["edge_index"] + 1),
                              dev(g["pred"]), float(g["th"]), dev(np.concatenate([g["class_probs"][:1], g["class_probs"]])),
                              "GAEC", int(g["num_joints"]), batch_index=dev(np.array([1] + [3] * n, np.int64)),
                              num_images=4)
    np.testing.assert_array_equal(out[3], g["persons"])
    assert len(out) == 4 and out[0] is None and out[1] is None and out[2] is None
    with pytest.raises(ValueError, match="num_images"):
        ppose.group_persons(dev(det), dev(sc), dev(ei), dev(pr), float(g["th"]), dev(cls), "GAEC",
                            int(g["num_joints"]), batch_index=dev(bi))
    empty = ppose.group_persons(dev(np.zeros((0, 3), np.int64)), dev(np.zeros(0, np.float32)),
                                dev(np.zeros((2, 0), np.int64)), dev(np.zeros(0, np.float32)), 0.1)
    assert empty == [None]


def _refine_case(s, tag):
    kp = np.zeros((1, s.shape[0], 3))
    kp[0, 0] = (5, 4, 0.9)
    with np.errstate(invalid="ignore"):
        ref = opose.refine(s, tag, kp.copy())
    got = ppose.refine(dev(s), dev(tag), kp.copy())
    np.testing.assert_array_equal(got, ref)
    return got


def test_refine_signed_zero_tie():
    """np.argmax treats -0.0 and +0.0 as equal (first index wins): a -0.0 at a low pixel beats a +0.0 held by
    another thread and block far away -- and there the score is not > 0, so the joint is not filled."""
    J, H, W = 2, 64, 128
    m = np.float32(0.25)
    tag = np.full((J, H, W), m + 1, np.float32)
    tag[0] = m
    tag[1, 0, 3] = m                       # k = 0 at the low pixel, k = 1 elsewhere
    s = np.full((J, H, W), 0.5, np.float32)
    s[1, 0, 3] = -0.0                      # s - k = -0.0
    s[1, 60, 100] = 1.0                    # s - k = +0.0
    got = _refine_case(s, tag)
    assert got[0, 1, 2] == 0.0             # not filled: the tie went to the -0.0 pixel


def test_refine_nan_first():
    """A NaN in the scoremap is np.argmax's answer (the first NaN): its value is not > 0, the joint stays
    unfilled even though a clear maximum exists elsewhere."""
    rng = np.random.default_rng(9)
    J, H, W = 2, 32, 96
    tag = np.zeros((J, H, W), np.float32)
    s = rng.random((J, H, W)).astype(np.float32)
    s[1, 20, 50] = 5.0
    s[1, 30, 90] = np.nan
    s[1, 31, 2] = np.nan
    got = _refine_case(s, tag)
    assert got[0, 1, 2] == 0.0


def test_bad_indices_raise():
    """Out-of-range inputs raise instead of faulting: a node index >= N in edge_index, a detected keypoint
    outside the map in refine / adjust."""
    g = load(GROUP[0])
    n = len(g["joint_det"])
    ei = g["edge_index"].copy()
    ei[1, -1] = n + 5
    with pytest.raises(ValueError, match="outside"):
        ppose.group_persons(dev(g["joint_det"]), dev(g["joint_scores"]), dev(ei), dev(g["pred"]), 0.0)
    s = dev(np.ones((2, 8, 16), np.float32))
    for x, y in ((16, 3), (3, 8), (-1, 2)):
        kp = np.zeros((1, 2, 3))
        kp[0, 0] = (x, y, 0.9)
        with pytest.raises(IndexError):
            ppose.refine(s, s, kp)
        with pytest.raises(IndexError):
            ppose.adjust(kp, s)


def test_group_persons_start_pipelined():
    """group_persons_start: the GPU half queued for two batches before either host half runs (as the bench's
    pipelined e2e step does) gives exactly group_persons' persons; finish_batch (fill_mean, refine, adjust with one
    wait, on a side stream) equals finish_persons image by image."""
    B, J, H, W = 3, 17, 96, 96
    results = []
    jobs, refs, maps = [], [], []
    for seed in (41, 42):
        hm = torch.from_numpy(syn.make_heatmaps(seed, B, J, H, W, persons=3)).to(DEV)
        feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25)).to(DEV)
        tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75)).to(DEV)
        gc = pcfg.inference_gc_config("fully", 5, False)
        out = pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                             factor_list=None, masks=None, device=DEV, testing=True, heatmaps=None,
                                             num_joints=J).construct_graph()
        det, ei, bi, sc = out[7], out[2], out[12], out[11]
        node_off = torch.searchsorted(bi, torch.arange(B + 1, device=DEV))
        pid = (torch.arange(det.shape[0], device=DEV) - node_off[bi]) % 3
        pe = torch.sigmoid(torch.where(pid[ei[0]] == pid[ei[1]], 2.5, -2.5))
        pn = torch.full((det.shape[0],), 0.9, device=DEV)
        pc = torch.eye(J, device=DEV)[det[:, 2]]
        args = (det, pn, ei, pe, 0.1, pc, "GAEC", J)
        refs.append(ppose.group_persons(*args, batch_index=bi, score_map_scores=sc, num_images=B))
        jobs.append(ppose.group_persons_start(*args, batch_index=bi, score_map_scores=sc, num_images=B))
        maps.append((hm, tags))
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    for job, ref, (hm, tags) in zip(jobs, refs, maps):
        got = job.result()
        assert len(got) == B and sum(p is not None for p in got) > 0
        for a, b in zip(got, ref):
            assert (a is None) == (b is None)
            if a is not None:
                np.testing.assert_array_equal(a, b)
        fin = ppose.finish_batch(got, hm, tags, adjustment=True, with_refine=True, stream=side)
        for b, p in enumerate(ref):
            one = ppose.finish_persons(None if p is None else p.copy(), hm[b], tags[b], True, True)
            assert (one is None) == (fin[b] is None)
            if one is not None:
                np.testing.assert_array_equal(fin[b], one)


@pytest.mark.parametrize("F", [1, 2])
def test_finish_batch_mixed_images(F):
    """finish_batch (one pemp_pose_finish_batch call: refine chunks per image, never across two; adjust for all)
    equals finish_persons image by image on a batch mixing: no persons, more persons than one 16-wide chunk, an
    image whose first person has no detected joint (adjusted, not refined), a single person; with and without
    the max-score filter; the caller's arrays are updated in place as finish_persons updates them."""
    rng = np.random.default_rng(7 + F)
    B, J, H, W = 6, 17, 64, 80
    hm = torch.from_numpy(rng.random((B, J, H, W), dtype=np.float32)).to(DEV)
    tg = torch.from_numpy(rng.normal(0, 3, (B, J, H, W, F)).astype(np.float32)).to(DEV)
    counts = [0, 37, 3, 2, 1, 9]

    def persons(P):
        kp = np.zeros((P, J, 3))
        kp[:, :, 0] = rng.integers(0, W, (P, J))
        kp[:, :, 1] = rng.integers(0, H, (P, J))
        kp[:, :, 2] = np.where(rng.random((P, J)) < 0.6, rng.random((P, J)) * 0.9 + 0.05, 0.0)
        kp[:, :, :2] *= kp[:, :, 2:3] > 0
        return kp

    for with_filter in (False, True):
        per = [None if c == 0 else persons(c) for c in counts]
        per[3][0, :, 2] = 0.0                         # no refine for image 3 (Utils.py:1472)
        per[3][0, :, :2] = 0.0
        ref = [None if p is None else p.copy() for p in per]
        side = torch.cuda.Stream(DEV)
        side.wait_stream(torch.cuda.current_stream(DEV))
        fin = ppose.finish_batch(per, hm, tg if F == 2 else tg[..., 0], adjustment=True, with_refine=True,
                                 with_filter=with_filter, stream=side)
        for b in range(B):
            one = ppose.finish_persons(ref[b], hm[b], tg[b] if F == 2 else tg[b, ..., 0], True, True,
                                       with_filter=with_filter)
            assert (one is None) == (fin[b] is None)
            if one is not None:
                np.testing.assert_array_equal(fin[b], one)
                if not with_filter:
                    np.testing.assert_array_equal(per[b], one)   # in place, as finish_persons
