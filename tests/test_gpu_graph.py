"""GPU parity of the graph-construction kernels (pemp_detect / pack / fully / knn / edge features)
against the reference's own outputs (tests/golden) and the CPU oracle. Bit-exact: every output of
construct_graph is integer or an exactly-rounded fp32 value."""
import numpy as np
import pytest
import torch

import pemp_amd
from oracle import restate
from pemp_amd import config as pcfg, synthetic as syn
from tests import golden_util as gu

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def run_gc(gc, J, hm, feats, tags, masks):
    return pemp_amd.get_graph_constructor(
        gc, scoremaps=hm.to(DEV), features=feats.to(DEV), tagmaps=None if tags is None else tags.to(DEV),
        joints_gt=None, factor_list=None, masks=None if masks is None else masks.to(DEV), device=DEV,
        testing=True, heatmaps=None, num_joints=J).construct_graph()


@pytest.mark.parametrize("name", gu.names("gc_"))
def test_golden(name):
    meta, a = gu.load(name)
    hm, feats, tags, masks = gu.gc_inputs(meta, a)
    out = run_gc(gu.gc_config(meta), meta["J"], hm, feats, tags, masks)
    x, ea, ei, det, sc, bi, tg = [out[i].cpu() for i in (0, 1, 2, 7, 11, 12, 14)]
    assert all(out[i] is None for i in (3, 4, 5, 6, 8, 9, 10, 13))
    np.testing.assert_array_equal(det.numpy(), a["joint_det"])
    np.testing.assert_array_equal(sc.numpy(), a["joint_scores"])
    np.testing.assert_array_equal(bi.numpy(), a["batch_index"])
    np.testing.assert_array_equal(tg.numpy(), a["joint_tags"])
    assert ei.dtype == torch.int64 and det.dtype == torch.int64 and ea.dtype == torch.float32
    assert gu.sha(ei) == meta["sha_edge_index"]
    assert gu.sha(x) == meta["sha_x"]
    assert gu.sha(ea) == meta["sha_edge_attr"]


CASES = [
    # B, J, H, W, persons, variant, graph, pool, thr, mask
    (8, 17, 640, 640, 9, "clean", "fully", 5, 0.1, False),      # C3 shape
    (8, 17, 640, 640, 9, "clean", "knn", 5, 0.1, False),        # C3 shape, published knn (N ~ 150 > k + 1)
    (1, 14, 640, 640, 36, "clean", "fully", 5, 0.1, False),     # C5 shape (CrowdPose-dense)
    (3, 17, 200, 328, 5, "noisy", "knn", 3, 0.1, True),         # ragged W, masks, knn
    (2, 17, 320, 320, 40, "clean", "knn", 3, 0.1, False),       # knn with n > 512 (global-memory path)
    (2, 17, 96, 136, 1, "realistic", "fully", 5, 0.1, False),   # bilinear plateaus (4 equal maxima)
    (2, 17, 64, 64, 2, "noisy", "fully", 3, 2.0, False),        # DETECT_THRESHOLD > 1.5 branch
    (1, 17, 33, 17, 1, "clean", "fully", 7, 0.1, False),        # tiny, odd sizes
    (8, 17, 640, 640, 9, "clean", "score_based", 5, 0.1, False),  # C3 shape, score_based (k = 75 roots)
    (1, 14, 640, 640, 36, "clean", "score_based", 5, 0.1, False), # C5 shape, score_based
    (8, 17, 640, 640, 9, "clean", "feature_knn", 5, 0.1, False),  # C3 shape, feature_knn (N ~ 150 > k + 1)
    (2, 17, 320, 320, 40, "clean", "feature_knn", 3, 0.1, False), # feature_knn with n > 512 (global path)
    (1, 17, 64, 64, 1, "clean", "feature_knn", 5, 0.1, False),    # n <= k + 1: every pair
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}x{c[3]}-{c[5]}-{c[6]}" for c in CASES])
def test_vs_oracle(case):
    B, J, H, W, persons, variant, graph, pool, thr, mask = case
    hm = torch.from_numpy(syn.make_heatmaps(100 + H, B, J, H, W, persons, variant=variant, margin=4))
    feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25))
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 2), 0.75))
    masks = torch.from_numpy((np.random.default_rng(H).random((B, H, W)) > 0.1).astype(np.float32)) if mask else None
    gc = pcfg.inference_gc_config(graph, pool, mask)
    gc.DETECT_THRESHOLD = thr
    out = run_gc(gc, J, hm, feats, tags, masks)
    ref = restate.construct_graph(hm, feats, tags, masks, gc, J)
    for i in (7, 11, 12, 14, 2, 0, 1):
        assert torch.equal(out[i].cpu(), ref[i]), f"output {i}"


def _edge_maps(B, J, H, W, seed):
    """Heatmaps for the detection edge cases: image 0 planted peaks plus a plateau of equal positive maxima
    touching the left border, image 1 negative everywhere but a few values (planes with fewer than top-k
    non-negative pixels: their top-k takes negatives), image 2 zero but for isolated values on the right and
    bottom borders."""
    rng = np.random.default_rng(seed)
    hm = np.zeros((B, J, H, W), np.float32)
    hm[0] = syn.make_heatmaps(seed, 1, J, H, W, 2, margin=2)[0]
    hm[0, :, 1:7, 0:9] = 0.5
    if B > 1:
        hm[1] = -rng.random((J, H, W)).astype(np.float32) - 0.01
        hm[1, :2, H // 2, W // 3] = 0.0
        hm[1, 1, 1, 1] = 0.7
    if B > 2:
        hm[2][:, H - 1, rng.integers(0, W, 3)] = 0.3 + rng.random((J, 3)).astype(np.float32)
        hm[2][:, rng.integers(0, H, 3), W - 1] = 0.2 + rng.random((J, 3)).astype(np.float32)
    return torch.from_numpy(hm)


@pytest.mark.parametrize("H,W,pool,mask", [(50, 1000, 9, False), (37, 8, 1, False), (64, 248, 3, True),
                                           (16, 252, 5, False), (70, 500, 7, True), (33, 17, 5, False)])
def test_detection_edges(H, W, pool, mask):
    """Detection on shapes and values at the edges of both stage-1 layouts (4 columns per lane when W % 4 == 0,
    1 otherwise): strips that end past the plane, single-strip planes narrower than a wave, bands cut by H,
    every pool radius, negative planes, plateaus of equal maxima, maxima on every border, masks."""
    B, J = 3, 17
    hm = _edge_maps(B, J, H, W, H * W + pool)
    feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25))
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
    masks = torch.from_numpy((np.random.default_rng(W).random((B, H, W)) > 0.2).astype(np.float32)) if mask else None
    gc = pcfg.inference_gc_config("fully", pool, mask)
    out = run_gc(gc, J, hm, feats, tags, masks)
    ref = restate.construct_graph(hm, feats, tags, masks, gc, J)
    assert ref[7].shape[0] > 0
    for i in (7, 11, 12, 14, 2):
        assert torch.equal(out[i].cpu(), ref[i]), f"output {i}"


def test_detection_large_plane():
    """A plane of more units than the fused select + emit stage takes (1280 x 1296: 80 bands x 22 strips > 1024)
    goes through the two-kernel selection and emission; noisy background, masks off."""
    B, J, H, W = 1, 17, 1280, 1296
    hm = torch.from_numpy(syn.make_heatmaps(7, B, J, H, W, 9, variant="noisy", margin=4))
    feats = torch.from_numpy(syn.closed_form((B, 16, H, W), 0.25))
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
    gc = pcfg.inference_gc_config("fully", 5, False)
    out = run_gc(gc, J, hm, feats, tags, None)
    ref = restate.construct_graph(hm, feats, tags, None, gc, J)
    assert ref[7].shape[0] > J
    for i in (7, 11, 12, 14, 2, 0):
        assert torch.equal(out[i].cpu(), ref[i]), f"output {i}"


def test_empty_image_and_overflow_growth():
    """An all-zero image yields no detections (N=0 rows) and a crowded one grows the capacity."""
    J, H, W = 17, 64, 64
    hm = torch.zeros(2, J, H, W)
    crowd = torch.from_numpy(syn.make_heatmaps(5, 1, J, H, W, persons=1, variant="noisy"))
    crowd[0, :, ::8, ::8] = 0.5 + torch.rand(J, 8, 8)          # many isolated maxima >= thr
    hm[1] = crowd[0]
    feats = torch.from_numpy(syn.closed_form((2, 128, H, W), 0.25))
    gc = pcfg.inference_gc_config("fully", 3, False)
    out = run_gc(gc, J, hm, feats, None, None)
    ref = restate.construct_graph(hm, feats, torch.zeros(2, J, H, W), None, gc, J)
    assert (out[12].cpu() == 0).sum() == 0
    for i in (7, 11, 12, 2, 1):
        assert torch.equal(out[i].cpu(), ref[i])
    assert out[14] is None


def test_capacity_build_fit_and_overflow():
    """Repeated batches of one shape take the capacity build (pemp_fully_graph_build_cap, launched
    before the count read-back); a batch larger than the capacities falls back to the exact build.
    Every call must equal the oracle bit for bit."""
    B, J, H, W = 2, 17, 96, 96
    gc = pcfg.inference_gc_config("fully", 5, False)
    feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25))
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
    # persons: first call sets the capacities, then smaller (fits), equal, then larger (overflow)
    for seed, persons in ((1, 3), (2, 2), (3, 3), (4, 6), (5, 1)):
        hm = torch.from_numpy(syn.make_heatmaps(seed, B, J, H, W, persons, margin=4))
        out = run_gc(gc, J, hm, feats, tags, None)
        ref = restate.construct_graph(hm, feats, tags, None, gc, J)
        for i in (0, 1, 2, 7, 11, 12, 14):
            assert out[i].is_contiguous()
            assert torch.equal(out[i].cpu(), ref[i]), (seed, i)


def test_score_based_needs_k_detections():
    """score_based_graph takes topk(k=75) of the scores: the reference raises for fewer detections."""
    J, H, W = 17, 64, 64
    hm = torch.from_numpy(syn.make_heatmaps(3, 1, J, H, W, persons=2))
    feats = torch.from_numpy(syn.closed_form((1, 128, H, W), 0.25))
    gc = pcfg.inference_gc_config("score_based", 5, False)
    with pytest.raises(RuntimeError, match="out of range"):
        run_gc(gc, J, hm, feats, None, None)
    with pytest.raises(RuntimeError, match="out of range"):
        restate.construct_graph(hm, feats, torch.zeros(1, J, H, W), None, gc, J)


@pytest.mark.parametrize("graph_type,scales", [("fully", [(80, 80)]), ("knn", [(80, 80), (40, 40)]),
                                               ("fully", [(53, 67), (160, 160), (27, 33)])])
def test_projected_features(graph_type, scales):
    """features=ProjectedMaps: x sampled at the detections from low-resolution maps
    equals the reference's materialised bilinear projection (interpolate, align_corners=False, summed
    over scales / their count) gathered at the same detections. Tolerance 2e-6 absolute (fp32 bilinear
    weights; torch's CPU kernel may contract the products into FMAs); every other output bit-exact."""
    from pemp_amd.frontend import ProjectedMaps
    B, J, H, W = 2, 17, 160, 160
    hm = torch.from_numpy(syn.make_heatmaps(31, B, J, H, W, 4, margin=4))
    maps = [torch.from_numpy(syn.closed_form((B, 128, h, w), 0.25 + 0.1 * k)) for k, (h, w) in enumerate(scales)]
    pm = ProjectedMaps(maps, (H, W))
    dense = pm.materialize()                                   # torch CPU, the reference's tensors
    gc = pcfg.inference_gc_config(graph_type, 5, False)
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
    for _ in range(2):                                          # second call takes the capacity build
        out = run_gc(gc, J, hm, pm, tags, None)
        ref = restate.construct_graph(hm, dense, tags, None, gc, J)
        for i in (1, 2, 7, 11, 12, 14):
            assert torch.equal(out[i].cpu(), ref[i]), i
        assert out[0].shape == ref[0].shape
        assert (out[0].cpu() - ref[0]).abs().max().item() <= 2e-6


def test_feature_knn_projected_and_duplicates():
    """feature_knn (ConstructGraph.py:370-374) ranks by x, so with features=ProjectedMaps the product
    samples x before the graph build; the graph must equal the oracle's feature_knn over that same x.
    Duplicate feature rows (equal distances at the 51st boundary) resolve by node index."""
    from pemp_amd.frontend import ProjectedMaps
    B, J, H, W = 2, 17, 160, 160
    hm = torch.from_numpy(syn.make_heatmaps(33, B, J, H, W, 5, margin=4))
    pm = ProjectedMaps([torch.from_numpy(syn.closed_form((B, 128, 80, 80), 0.35))], (H, W))
    gc = pcfg.inference_gc_config("feature_knn", 5, False)
    out = run_gc(gc, J, hm, pm, None, None)
    x, ei, bi = out[0].cpu(), out[2].cpu(), out[12].cpu()
    parts, off = [], 0
    for b in range(B):
        n = int((bi == b).sum())
        parts.append(restate.feature_knn_edge_index(x[off:off + n]) + off)
        off += n
    assert torch.equal(ei, torch.cat(parts, 1))
    # constant features: every distance ties at 0 -> the 51 lowest indices of each image, symmetrised
    feats = torch.ones(B, 16, H, W)
    out = run_gc(gc, J, hm, feats, None, None)
    ref = restate.construct_graph(hm, feats, torch.zeros(B, J, H, W), None, gc, J)
    for i in (0, 1, 2, 7, 12):
        assert torch.equal(out[i].cpu(), ref[i]), i


@pytest.mark.parametrize("graph", ["fully", "knn"])
def test_reentrant_two_streams(graph):
    """construct_graph is reentrant. Two constructors with different inputs and shapes are
    interleaved on two streams (the second call of each queued while the first's kernels may still
    run), then run again from two host threads at once; every output stays bit-exact with the oracle."""
    import threading
    J = 17
    jobs = []
    for k, (B, H, W, persons) in enumerate(((2, 128, 128, 4), (3, 96, 160, 6))):
        hm = torch.from_numpy(syn.make_heatmaps(70 + k, B, J, H, W, persons, margin=4))
        feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25 + 0.1 * k))
        tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
        gc = pcfg.inference_gc_config(graph, 5, False)
        ref = restate.construct_graph(hm, feats, tags, None, gc, J)
        jobs.append((gc, hm.to(DEV), feats.to(DEV), tags.to(DEV), ref))
    streams = [torch.cuda.Stream(DEV) for _ in jobs]

    def call(j):
        gc, hm, feats, tags, _ = jobs[j]
        with torch.cuda.stream(streams[j]):
            out = run_gc(gc, J, hm, feats, tags, None)
            streams[j].synchronize()
        return out

    def check(j, out):
        for i in (0, 1, 2, 7, 11, 12, 14):
            assert torch.equal(out[i].cpu(), jobs[j][4][i]), (j, i)

    outs = [call(0), call(1), call(0), call(1)]          # interleaved, capacity builds on the repeats
    for n, out in enumerate(outs):
        check(n % 2, out)
    results, errors = [None] * 4, []

    def worker(slot):
        try:
            results[slot] = call(slot % 2)
        except Exception as e:        # noqa: BLE001 -- reported below
            errors.append(e)
    threads = [threading.Thread(target=worker, args=(s,)) for s in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors
    for s, out in enumerate(results):
        check(s % 2, out)


@pytest.mark.parametrize("graph", ["fully", "knn"])
def test_construct_graph_start_pipelined(graph):
    """construct_graph_start / PendingGraph.result (batches in flight): step i + 1 is started on the other stream
    before step i is collected, with the bound MPN queued in capacity mode; every graph equals the oracle bit for
    bit and every step's logits equal a plain construct_graph + forward of the same batch. result() is idempotent."""
    J = 17
    cfg = pcfg.published_mpn_config(J, 3, "attn")
    model = pemp_amd.get_mpn_model(cfg)
    model.load_state_dict(syn.closed_form_state_dict(model, 0.5))
    model.eval().to(DEV)
    gc = pcfg.inference_gc_config(graph, 5, False)
    batches = []
    for k in range(3):
        B, H, W = 2 + k % 2, 96, 128
        hm = torch.from_numpy(syn.make_heatmaps(90 + k, B, J, H, W, 5, margin=4))
        feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.3 + 0.05 * k))
        tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
        batches.append((hm.to(DEV), feats.to(DEV), tags.to(DEV), restate.construct_graph(hm, feats, tags, None, gc, J)))
    streams = [torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)]

    def make(b):
        hm, feats, tags, _ = batches[b]
        return pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                              factor_list=None, masks=None, device=DEV, testing=True, heatmaps=None,
                                              num_joints=J)

    with torch.no_grad():
        refs = []
        for b in range(len(batches)):   # plain calls (also warm the capacity hints)
            out = make(b).construct_graph()
            refs.append([t[-1].cpu() for t in model(out[0], out[1], out[2], node_types=out[7][:, 2])[:3]])
        pemp_amd.bind_mpn(model)
        try:
            for rnd in range(2):
                order = list(range(len(batches))) * 2
                pend = None
                got = []
                for i in range(len(order) + 1):
                    nxt = None
                    if i < len(order):
                        with torch.cuda.stream(streams[i % 2]):
                            nxt = (make(order[i]).construct_graph_start(), streams[i % 2], order[i])
                    if pend is not None:
                        with torch.cuda.stream(pend[1]):
                            out = pend[0].result()
                            assert pend[0].result() is out
                            lg = model(out[0], out[1], out[2], node_types=out[7][:, 2])
                            got.append((pend[2], out, [t[-1] for t in lg[:3]]))
                    pend = nxt
                torch.cuda.synchronize()
                for b, out, lg in got:
                    ref = batches[b][3]
                    for j in (0, 1, 2, 7, 11, 12, 14):
                        assert torch.equal(out[j].cpu(), ref[j]), (graph, b, j)
                    for a_, r_ in zip(lg, refs[b]):
                        assert torch.equal(a_.cpu(), r_), (graph, b)
        finally:
            pemp_amd.bind_mpn(None)


@pytest.mark.parametrize("graph,persons", [("knn", 5), ("knn", 40)])
@pytest.mark.parametrize("features", [["position", "angle", "connection_type"], ["ae_normed"],
                                      ["position", "connection_type", "ae_normed"]])
def test_knn_edge_feature_modes(graph, persons, features):
    """The knn build writes edge_attr itself (LDS path, n <= 512) or through the device-total features
    kernel (n > 512): every EDGE_FEATURES_TO_USE mode, tags with F = 2, bit-exact with the oracle --
    except the angle column: theta = |acos(a_x * rsqrt(a_x^2 + a_y^2))| (ConstructGraph.py:319-321) goes
    through the device acosf, within 2 ulp of torch CPU's (vectorised SLEEF u10 / libm) acos, which
    itself differs between its vector and tail paths: parity at the last ulp is unpinned there."""
    B, J, H, W = 2, 17, 192, 192
    hm = torch.from_numpy(syn.make_heatmaps(11 + persons, B, J, H, W, persons, margin=4))
    feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25))
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 2), 0.75))
    gc = pcfg.inference_gc_config(graph, 3, False)
    gc.EDGE_FEATURES_TO_USE = features
    out = run_gc(gc, J, hm, feats, tags, None)
    ref = restate.construct_graph(hm, feats, tags, None, gc, J)
    for i in (0, 2, 7, 11, 12, 14):
        assert torch.equal(out[i].cpu(), ref[i]), i
    ea, ra = out[1].cpu(), ref[1]
    if "angle" in features:
        np.testing.assert_array_max_ulp(ea[:, 2].numpy(), ra[:, 2].numpy(), maxulp=2)
        ea, ra = torch.cat([ea[:, :2], ea[:, 3:]], 1), torch.cat([ra[:, :2], ra[:, 3:]], 1)
    assert torch.equal(ea, ra)


@pytest.mark.parametrize("sizes,size,flip", [([(80, 80)], (160, 160), True), ([(90, 70)], (160, 176), True),
                                             ([(80, 80), (40, 40)], (160, 160), True), ([(80, 80)], (160, 160), False)])
def test_projected_maps_materialize(sizes, size, flip):
    """pemp_project_maps (the values the projected detection samples) against the oracle's fp32
    restatement: bit-exact scoremaps and tags."""
    from pemp_amd.frontend import ProjectedHeatmaps
    from tests.test_frontend_cpu import COCO_FLIP, make_outputs
    B, J = 2, 17
    outs, flips = make_outputs(7, B, J, sizes, flip)
    fi = COCO_FLIP if flip else None
    ph = ProjectedHeatmaps([o.to(DEV) for o in outs], size, J, None if flips is None else [o.to(DEV) for o in flips],
                           fi)
    s, t = ph.project()
    rs, rt = restate.project_frontend(outs, flips, size, J, fi)
    bad = (s.cpu() != rs).nonzero()
    assert bad.shape[0] == 0, (bad[:5].tolist(), s.cpu()[tuple(bad[0])].item(), rs[tuple(bad[0])].item())
    assert torch.equal(t.cpu(), rt)


@pytest.mark.parametrize("graph,sizes,size,flip,features", [
    ("fully", [(80, 80)], (160, 160), True, ["position", "connection_type"]),
    ("fully", [(90, 70)], (160, 176), True, ["position", "connection_type", "ae_normed"]),
    ("knn", [(80, 80), (40, 40)], (160, 160), True, ["position", "connection_type"]),
    ("fully", [(80, 80)], (160, 160), False, ["ae"]),
])
def test_projected_frontend(graph, sizes, size, flip, features):
    """scoremaps = tagmaps = ProjectedHeatmaps: detection evaluates the flip-averaged,
    upsampled (align_corners=False) and scale-averaged heatmaps inside its NMS loads and the tags are
    sampled at the detections. Bit-exact with the oracle run on the maps its fp32 restatement
    materialises (oracle/restate.project_frontend; that restatement is within 2e-6 of the reference's
    torch ops, tests/test_frontend_cpu.py). Twice: the second call takes the capacity build."""
    from pemp_amd.frontend import ProjectedHeatmaps
    from tests.test_frontend_cpu import COCO_FLIP, make_outputs
    B, J = 2, 17
    outs, flips = make_outputs(7, B, J, sizes, flip)
    fi = COCO_FLIP if flip else None
    ph = ProjectedHeatmaps([o.to(DEV) for o in outs], size, J, None if flips is None else [o.to(DEV) for o in flips],
                           fi)
    s, t = restate.project_frontend(outs, flips, size, J, fi)
    feats = torch.from_numpy(syn.closed_form((B, 128) + tuple(size), 0.25))
    gc = pcfg.inference_gc_config(graph, 5, False)
    gc.EDGE_FEATURES_TO_USE = features
    ref = restate.construct_graph(s, feats, t, None, gc, J)
    for _ in range(2):
        out = pemp_amd.get_graph_constructor(gc, scoremaps=ph, features=feats.to(DEV), tagmaps=ph, joints_gt=None,
                                             factor_list=None, masks=None, device=DEV, testing=True, heatmaps=None,
                                             num_joints=J).construct_graph()
        assert ref[7].shape[0] > 2 * J       # detections found
        for i in (7, 11, 12, 14, 2, 0, 1):
            assert torch.equal(out[i].cpu(), ref[i]), i


@pytest.mark.parametrize("ksize,pad,scales", [(3, 1, [(80, 80)]), (1, 0, [(53, 67), (40, 40)]), (3, 1, [(27, 33), (160, 160)])])
def test_projected_features_gather_conv(ksize, pad, scales):
    """features=ProjectedMaps(raw, gather=feature_gather) (PoseEstimation.py:64-66, 341,
    426-452): the Conv2d evaluated at the bilinear taps of each detection only equals the reference's own
    torch ops (conv over the whole map, interpolate, sum over scales / count) gathered at the detections.
    Floating point with a different summation order: |dx| <= 2e-5 * max(1, max|x|); every other output
    bit-exact."""
    from pemp_amd.frontend import ProjectedMaps
    B, J, H, W = 2, 17, 160, 160
    hm = torch.from_numpy(syn.make_heatmaps(37, B, J, H, W, 4, margin=2))
    g = torch.Generator().manual_seed(5)
    raw = [torch.randn(B, 32, h, w, generator=g) for (h, w) in scales]
    conv = torch.nn.Conv2d(32, 128, ksize, 1, pad, bias=True)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.1)
        conv.bias.copy_(torch.randn(128, generator=g))
    pm = ProjectedMaps(raw, (H, W), gather=conv)
    dense = pm.materialize()
    gc = pcfg.inference_gc_config("fully", 5, False)
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
    pmd = pm.to(DEV)
    for _ in range(2):
        out = run_gc(gc, J, hm, pmd, tags, None)
        ref = restate.construct_graph(hm, dense, tags, None, gc, J)
        for i in (1, 2, 7, 11, 12, 14):
            assert torch.equal(out[i].cpu(), ref[i]), i
        assert out[0].shape == ref[0].shape
        tol = 2e-5 * max(1.0, ref[0].abs().max().item())
        assert (out[0].cpu() - ref[0]).abs().max().item() <= tol


CROWD_FLIP = [1, 0, 3, 2, 5, 4, 7, 6, 9, 8, 11, 10, 12, 13]   # FLIP_CONFIG['CROWDPOSE'] (multi_scales_testing.py:383)


@pytest.mark.parametrize("graph,H,W", [("fully", 160, 160), ("knn", 160, 192)])
def test_projected_frontend_three_scales_c5(graph, H, W):
    """The C5 multi-scale front-end exactly as bench.py's c5ms builds it: CrowdPose J = 14, scale
    factors {2, 1, 0.5} in the reference's descending order (PoseEstimation.py:193), network outputs at half the
    scaled input (H s / 2), flipped passes re-indexed by FLIP_CONFIG['CROWDPOSE'], tags kept from the 1.0 scale
    (tag_scale = 1, aggregate_results_mpn's scale_factor == 1 branch, multi_scales_testing.py:147-157), features
    projected from three ProjectedMaps scales. construct_graph bit-exact with the oracle on its fp32 restatement of
    the same projection; pemp_project_maps bit-exact with that restatement; the second call takes the capacity
    build."""
    from pemp_amd.frontend import ProjectedHeatmaps, ProjectedMaps
    B, J = 2, 14
    scales = [2.0, 1.0, 0.5]
    outs, flips, fmaps = [], [], []
    for k, sc in enumerate(scales):
        h, w = int(H * sc / 2), int(W * sc / 2)
        hm = syn.make_heatmaps(90 + k, B, J, h, w, 4, sigma=1.0, margin=2)
        tg = syn.closed_form((B, J, h, w), 0.5 + 0.1 * k)
        outs.append(torch.from_numpy(np.concatenate([hm, tg], 1)))
        hm2 = syn.make_heatmaps(140 + k, B, J, h, w, 4, sigma=1.0, margin=2)
        tg2 = syn.closed_form((B, J, h, w), 0.7 + 0.1 * k)
        flips.append(torch.from_numpy(np.concatenate([hm2, tg2], 1)))
        fmaps.append(torch.from_numpy(syn.closed_form((B, 128, h, w), 0.25 + 0.1 * k)))
    tag_scale = scales.index(1.0)
    ph = ProjectedHeatmaps([o.to(DEV) for o in outs], (H, W), J, [o.to(DEV) for o in flips], CROWD_FLIP,
                           tag_scale=tag_scale)
    s, t = restate.project_frontend(outs, flips, (H, W), J, CROWD_FLIP, tag_scale=tag_scale)
    ps, pt = ph.project()
    assert torch.equal(ps.cpu(), s) and torch.equal(pt.cpu(), t)
    pm = ProjectedMaps(fmaps, (H, W))
    dense_f = pm.materialize()
    gc = pcfg.inference_gc_config(graph, 5, False)
    ref = restate.construct_graph(s, dense_f, t, None, gc, J)
    assert ref[7].shape[0] > 4 * J
    for _ in range(2):
        out = pemp_amd.get_graph_constructor(gc, scoremaps=ph, features=pm.to(DEV), tagmaps=ph, joints_gt=None,
                                             factor_list=None, masks=None, device=DEV, testing=True, heatmaps=None,
                                             num_joints=J).construct_graph()
        for i in (1, 2, 7, 11, 12, 14):
            assert torch.equal(out[i].cpu(), ref[i]), i
        assert out[14].shape[1] == 2                               # F = 2: the flipped pass's tags too
        assert (out[0].cpu() - ref[0]).abs().max().item() <= 2e-6


@pytest.mark.parametrize("flip,half_sizes,size", [(True, [(80, 80), (40, 40)], (160, 160)),
                                                  (False, [(90, 70)], (180, 140))])
def test_projected_frontend_from_stages(flip, half_sizes, size):
    """ProjectedHeatmaps.from_stages: HigherHRNet's per-stage outputs (1/4-res heatmaps + tags, 1/2-res heatmaps)
    merged by pemp_stage_merge (_get_multi_stage_outputs, PoseEstimation.py:338-412) bit-exact with the oracle's
    restate.stage_merge; construct_graph on the result bit-exact with the oracle on the projection of those maps."""
    from pemp_amd.frontend import ProjectedHeatmaps
    from tests.test_frontend_cpu import COCO_FLIP, make_stages
    B, J = 2, 17
    stages, flips = make_stages(12, B, J, half_sizes, flip)
    # plant peaks in stage 1 so that detections exist (the random maps alone hold few maxima above 0.1)
    for k, (h, w) in enumerate(half_sizes):
        peaks = torch.from_numpy(syn.make_heatmaps(60 + k, B, J, h, w, 4, sigma=1.0, margin=2))
        stages[k] = (stages[k][0] * 0.05, torch.maximum(stages[k][1] * 0.05, peaks))
        if flips is not None:
            flips[k] = (flips[k][0] * 0.05, torch.maximum(flips[k][1] * 0.05, torch.flip(peaks, [3])))
    fi = COCO_FLIP if flip else None
    dev_stages = [(a.to(DEV), b.to(DEV)) for a, b in stages]
    dev_flips = None if flips is None else [(a.to(DEV), b.to(DEV)) for a, b in flips]
    ph = ProjectedHeatmaps.from_stages(dev_stages, size, J, dev_flips, fi)
    merged = [restate.stage_merge(a, b, J) for a, b in stages]
    mflip = None if flips is None else [restate.stage_merge(a, b, J) for a, b in flips]
    for got, want in zip(ph.outputs + (ph.flip_outputs or []), merged + (mflip or [])):
        assert torch.equal(got.cpu(), want)
    s, t = restate.project_frontend(merged, mflip, size, J, fi)
    feats = torch.from_numpy(syn.closed_form((B, 128) + tuple(size), 0.25))
    gc = pcfg.inference_gc_config("fully", 5, False)
    ref = restate.construct_graph(s, feats, t, None, gc, J)
    assert ref[7].shape[0] > 2 * J
    out = pemp_amd.get_graph_constructor(gc, scoremaps=ph, features=feats.to(DEV), tagmaps=ph, joints_gt=None,
                                         factor_list=None, masks=None, device=DEV, testing=True, heatmaps=None,
                                         num_joints=J).construct_graph()
    for i in (7, 11, 12, 14, 2, 0, 1):
        assert torch.equal(out[i].cpu(), ref[i]), i


QUAD_SCRIPT = r"""
import json, sys, numpy as np, torch
from oracle import restate
from pemp_amd import config as pcfg, synthetic as syn
from tests.test_gpu_graph import _edge_maps, run_gc
bad = []
for H, W, pool in [(50, 1000, 9), (37, 8, 1), (16, 252, 5), (33, 17, 5), (64, 640, 5), (40, 516, 3)]:
    B, J = 3, 17
    hm = _edge_maps(B, J, H, W, H * W + pool)
    feats = torch.from_numpy(syn.closed_form((B, 16, H, W), 0.25))
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
    gc = pcfg.inference_gc_config("fully", pool, False)
    out = run_gc(gc, J, hm, feats, tags, None)
    ref = restate.construct_graph(hm, feats, tags, None, gc, J)
    for i in (7, 11, 12, 14, 2):
        if not torch.equal(out[i].cpu(), ref[i]):
            bad.append([H, W, pool, i])
print(json.dumps({"bad": bad}))
"""


def test_detection_quad_nms_variant(tmp_path):
    """The split dense NMS (nms_quad_kernel, 4 columns per lane, opt-in PEMP_NMS_QUAD=1; the library reads the switch
    once per process, so it runs in a child) gives the oracle's detections bit for bit on the edge-case maps: W not a
    multiple of 4 (the clamped loader), blocks past the plane's right edge, planes narrower than a wave, every pool
    radius, negative planes with fewer than top-k non-negative pixels, plateaus, border maxima."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "quad.py"
    script.write_text(QUAD_SCRIPT)
    env = dict(os.environ, PEMP_NMS_QUAD="1", PYTHONPATH=root)
    r = subprocess.run([sys.executable, str(script)], env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["bad"] == []
