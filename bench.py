#!/usr/bin/env python3
"""Hot-path throughput on MI355X: heatmaps -> keypoint graph -> MPN logits.

One step = ``get_graph_constructor(...).construct_graph()`` + ``NodeClassificationMPNSimple``
forward over one batch of synthetic 640x640 COCO-shaped inputs already resident in HBM (the
frozen backbone is out of scope). Steps are issued round-robin on ``--streams`` HIP streams (default
2: one batch's detection overlaps the previous batch's MPN, as a server with two requests in flight
would run; every step still does the whole path on its own batch); ``value_serial_steps`` is the same
K steps on one stream. Multi-GPU: one process per GPU (torchrun), each rank owns its
own images (weak scaling, no data-path collective); barrier + max-over-ranks timing.

Prints ONE JSON line (rank 0). Extra fields: isolated-MPN edge-updates/s, live roofline of the
dominant kernel (hipEvents on the launch stream), and the CPU oracle baseline (rank 0, N=1).
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import pemp_amd  # noqa: E402
from pemp_amd import _lib, config as pcfg, dist as pdist, synthetic as syn  # noqa: E402

METRIC = "images/sec (640px, HRNet-w48) + MPN edge-updates/sec at 1/2/4/8 MI355X"
WORKLOADS = {
    # BASELINE.json configs[2] (C3): COCO-val-shaped batch of 8 at 640px, 3 MPN iterations
    "c3": dict(B=8, J=17, H=640, W=640, persons=9, steps=3, graph="fully", variant="attn"),
    # configs[1] (C2): one 640px image, ~150 detections, dense graph, 3 iterations
    "c2": dict(B=1, J=17, H=640, W=640, persons=9, steps=3, graph="fully", variant="attn"),
    # configs[4] (C5): CrowdPose-dense, ~500 detections / ~250k directed edges per image
    "c5": dict(B=1, J=14, H=640, W=640, persons=36, steps=3, graph="fully", variant="attn"),
    # configs[1] at its stated arithmetic: every per-edge GEMM in exact fp32 MFMA
    "c2fp32": dict(B=1, J=17, H=640, W=640, persons=9, steps=3, graph="fully", variant="attn", precision="fp32"),
    # C3 with the secondary graph type: k = 50 nearest neighbours, symmetrised
    "c3knn": dict(B=8, J=17, H=640, W=640, persons=9, steps=3, graph="knn", variant="attn"),
    # the published model on C3 (experiments/hybrid_class_agnostic_end2end/model_58_4_4.yaml:97,155):
    # GRAPH_TYPE knn, STEPS 10
    "c3knn10": dict(B=8, J=17, H=640, W=640, persons=9, steps=10, graph="knn", variant="attn"),
    # configs[4] (C5) as stated: multi-scale x3 ({2.0, 1.0, 0.5}, multi_scales_testing.py:144-195) with flip test;
    # the timed step starts from the network outputs of every scale (heatmaps + tags, and the gathered feature
    # maps) and projects them on demand (ProjectedHeatmaps / ProjectedMaps) inside construct_graph
    "c5ms": dict(B=1, J=14, H=640, W=640, persons=36, steps=3, graph="fully", variant="attn", scales=(2.0, 1.0, 0.5)),
}
FLIP_INDEX = {17: [0, 2, 1, 4, 3, 6, 5, 8, 7, 10, 9, 12, 11, 14, 13, 16, 15],   # COCO FLIP_CONFIG
              14: [1, 0, 3, 2, 5, 4, 7, 6, 9, 8, 11, 10, 12, 13]}               # CrowdPose
PREC_CODE = {"fp32": 0, "bf16x3": 1, "f16x3": 2}   # PEMP_PREC_* (include/pemp.h)
FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: dense f32 MFMA (= f32 vector) peak
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
BF16_MFMA_PEAK_TFLOPS = 2500.0     # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
REF_EDGE_FLOP = 82048              # the reference's FLOP per edge-update (before the node/edge split)
GEMM64 = 2 * 64 * 64                            # one 64x64 GEMM per edge
EDGE_HEAD_FLOP = 2 * (64 * 64 + 64 * 32 + 32)   # fused edge-classification head
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")   # tools/gpu_profile.sh + tools/pmc_json.py
MFMA_FILE = os.path.join(ROOT, "profiles", "mfma_latest.json")  # tools/mfma_util.py --json over an SQ pass
PREC_NOTE = {
    "f16x3": "f16x3: f16 MFMA on hi/lo split operands (22 bits each), fp32 accumulate; fp32-level logits",
    "bf16x3": "bf16x3: bf16 MFMA on hi/lo split operands, fp32 accumulate (opt-in, ~2^-16 per product)",
    "fp32": "fp32 MFMA (v_mfma_f32_16x16x4_f32)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)   # (a 20-step region is 5 ms at c3: one host hiccup moved it 10 %+)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=30.0, help="bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-backbone", action="store_true",
                    help="skip the backbone leg (a random-weight HigherHRNet-w48 forward on the batch's 640 px images, "
                         "torch / MIOpen bf16 channels-last, tools/hrnet_w48.py; its first call compiles MIOpen "
                         "kernels for ~7 s)")
    ap.add_argument("--profile-steps", action="store_true",
                    help="for rocprofv3 per-shape traces: the warmup and the K steps strictly serial on one stream "
                         "(round-robin on --streams S streams when given), nothing else (no schedule probe, roofline, "
                         "isolated MPN, e2e, grouping or CPU legs)")
    ap.add_argument("--streams", type=int, default=0,
                    help="batches in flight: step i runs on HIP stream i %% S (serving-style overlap of one "
                         "batch's detection with the previous batch's MPN); 1 = strictly serial steps; 0 (default) "
                         "= the faster of 2 and 1, chosen by timing both schedules outside the timed region")
    return ap.parse_args()


def setup_dist(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != n_gpus:   # checked before anything touches the GPU
        raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                         f"(torchrun --nproc-per-node {n_gpus}) or let bench.py spawn them (WORLD_SIZE unset)")
    return pdist.init_from_env("nccl")


def spawn_ranks(n_gpus):
    """`python bench.py --gpus N` without a launcher: start N rank processes of this same command (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment) before anything here touches the GPU, wait
    for all of them and return the worst exit code. Rank 0 prints the JSON line; the timing contract (barrier,
    synchronize, max over ranks) is inside the ranks."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    try:
        for r in range(n_gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n_gpus),
                       LOCAL_WORLD_SIZE=str(n_gpus), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                       MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
        codes = [p.wait() for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


barrier = pdist.barrier
max_over_ranks = pdist.max_over_ranks
sum_over_ranks = pdist.sum_over_ranks


def make_inputs(wl, rank, dev):
    """(scoremaps, features, tagmaps) as construct_graph takes them. Single-scale workloads: image-size tensors.
    Multi-scale ("scales"): the network outputs of every scale and of the flipped pass ([B, 2J, 320 s, 320 s]:
    heatmaps whose planted peaks sit at the same image positions at every scale, then per-joint tags) and the
    gathered feature maps ([B, 128, 320 s, 320 s]), wrapped as ProjectedHeatmaps / ProjectedMaps."""
    B, J, H, W = wl["B"], wl["J"], wl["H"], wl["W"]
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    if not wl.get("scales"):
        hm = torch.from_numpy(syn.make_heatmaps(1000 + rank, B, J, H, W, wl["persons"])).to(dev)
        feats = torch.rand(B, 128, H, W, generator=g, device=dev) * 2 - 1
        tags = torch.rand(B, J, H, W, 1, generator=g, device=dev)
        return hm, feats, tags
    scales = wl["scales"]
    top = max(scales)
    h0, w0 = int(H * top / 2), int(W * top / 2)
    base = torch.from_numpy(syn.make_heatmaps(1000 + rank, B, J, h0, w0, wl["persons"])).to(dev)
    fi = FLIP_INDEX[J]
    outs, flips, fmaps = [], [], []
    for s in scales:
        k = int(round(top / s))
        heat = base if k == 1 else torch.nn.functional.avg_pool2d(base, k)
        h, w = heat.shape[-2:]
        outs.append(torch.cat([heat, torch.rand(B, J, h, w, generator=g, device=dev)], 1))
        flips.append(torch.cat([torch.flip(heat, [3])[:, fi], torch.rand(B, J, h, w, generator=g, device=dev)], 1))
        fmaps.append(torch.rand(B, 128, h, w, generator=g, device=dev) * 2 - 1)
    ph = pemp_amd.ProjectedHeatmaps(outs, (H, W), J, flips, fi, tag_scale=list(scales).index(1.0))
    return ph, pemp_amd.ProjectedMaps(fmaps, (H, W)), ph


def dense_maps(hm, tags):
    """Image-size (scoremaps, tagmaps) for the legs that read whole maps (refine): the workload's own tensors,
    or, multi-scale, the library's projection of them (pemp_project_maps)."""
    if isinstance(hm, torch.Tensor):
        return hm, tags
    return hm.project()


def make_model(wl, dev):
    cfg = pcfg.published_mpn_config(wl["J"], wl["steps"], wl["variant"])
    model = pemp_amd.get_mpn_model(cfg)
    model.load_state_dict(syn.closed_form_state_dict(model, 0.5))
    if wl.get("precision"):
        model.precision = wl["precision"]
    return model.eval().to(dev), cfg


def run_step(wl, gc, model, hm, feats, tags, dev):
    out = pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                         factor_list=None, masks=None, device=dev, testing=True, heatmaps=None,
                                         num_joints=wl["J"]).construct_graph()
    pe, pn, pc, _ = model(out[0], out[1], out[2], node_types=out[7][:, 2])
    return out, pe, pn, pc


def run_steps(n, streams, S, wl, gc, model, hm, feats, tags, dev):
    """n whole steps, step i on streams[i % S]. S > 1: pipelined as a server with S requests in flight -- step i + 1
    is queued (construct_graph_start: detection, capacity graph build, MPN) before step i is collected
    (PendingGraph.result: the count wait, the output views, the model call returning the queued logits), so the
    host's count wait overlaps the next step's launches; each stream then has at most one step pending. S == 1:
    run_step one after the other."""
    if S == 1 or os.environ.get("PEMP_BENCH_NO_PIPELINE"):   # (the latter: round 5's loop, for A/B runs)
        for i in range(n):
            with torch.cuda.stream(streams[i % S]):
                run_step(wl, gc, model, hm, feats, tags, dev)
        return
    pend = None
    for i in range(n + 1):
        nxt = None
        if i < n:
            st = streams[i % S]
            with torch.cuda.stream(st):
                nxt = (pemp_amd.get_graph_constructor(
                    gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None, factor_list=None, masks=None,
                    device=dev, testing=True, heatmaps=None, num_joints=wl["J"]).construct_graph_start(), st)
        if pend is not None:
            with torch.cuda.stream(pend[1]):
                out = pend[0].result()
                model(out[0], out[1], out[2], node_types=out[7][:, 2])
        pend = nxt


_BENCH_MAPS = None
_LAST_GROUPING = None
ROOF_REPEAT = 8   # back-to-back launches per event pair in the roofline phase


def edge_pass_cost(head, upd):
    """Executed FLOP and algorithmic HBM bytes per edge of one edge pass (mpn.hip edge_step_kernel).
    A middle pass (no head) computes e' = ReLU(W2 h + b2) from h = ReLU(r + A[dst] + B[src]), the
    message W_t e', the update block U_t m (upd), the next r = Q0 + W1_e e', and the attention dot;
    it reads r and Q0 (2 x 256 B) and writes the next r (256 B) plus 2 int32 indices. The last pass
    (head) drops the next r and Q0 and runs the fused edge head, writing a 4 B logit. Per launch, both also
    write one 256 B aggregate row per non-empty (target, source type) segment (seg_rows_bytes)."""
    gemms = 2 + (1 if upd else 0) + (0 if head else 1)
    flop = gemms * GEMM64 + 2 * 64 + (EDGE_HEAD_FLOP if head else 0)
    byts = (256 + 8 + 4) if head else (2 * 256 + 256 + 8)
    return flop, byts


def pmc_traffic(kernel_prefix, workload, E):
    """HBM bytes per dispatch of the kernel from the committed PMC passes (profiles/pmc_latest.json,
    tools/pmc_json.py), for a pass over the same workload and edge count; None when no pass covers it."""
    try:
        runs = json.load(open(PMC_FILE))["runs"]
    except (OSError, ValueError, KeyError):
        return None
    for run in runs:
        if run.get("workload") == workload and run.get("edges") == E:
            hits = [v for k, v in run["kernels"].items() if k.startswith(kernel_prefix)]
            return hits[0]["bytes"] if len(hits) == 1 else None
    return None


def mfma_busy(kernel_prefix, workload):
    """MFMA utilisation of the kernel (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), the
    median over its dispatches) from the committed SQ pass of the same workload (profiles/mfma_latest.json,
    tools/mfma_util.py; the formula reads 0.86 on the dense-MFMA microbench tools/ubench/mfma_peak.hip)."""
    try:
        runs = json.load(open(MFMA_FILE))["runs"]
    except (OSError, ValueError, KeyError):
        return None
    for run in runs:
        if run.get("workload") == workload:
            hits = [v for k, v in run["kernels"].items() if kernel_prefix in k]
            return hits[0] if len(hits) == 1 else None
    return None


def graph_stats():
    """The capacity-mode forward's HIP-graph counters since the library loaded (pemp_mpn_graph_stats)."""
    import ctypes
    out = (ctypes.c_uint64 * 3)()
    _lib.check(_lib.lib().pemp_mpn_graph_stats(out))
    return {"captures": out[0], "launches": out[1], "refused": out[2]}


def seg_rows_bytes(ei, types):
    """Aggregate-row bytes one edge pass writes: 64 fp32 per non-empty (target, source type) segment."""
    T = int(types.max().item()) + 1 if types.numel() else 1
    return 256 * int(torch.unique(ei[1] * T + types[ei[0]]).numel())


def roofline_for(label, stats, E, wl, precision, upd, workload, agg_bytes=0):
    """Roofline of the dominant kernel from its measured average launch time.

    edge_step*: executed FLOP and ALGORITHMIC HBM bytes per edge from edge_pass_cost (node-table
    gathers are L2-resident and not counted). fp32: bound = fp32 MFMA peak. f16x3 / bf16x3: the MFMA
    work is 3 16-bit products per fp32 product (f16 and bf16 MFMA run at the same dense rate), so the
    compute floor is 3 x FLOP / bf16 dense peak; the bound reported is whichever floor (compute, HBM)
    is larger. `traffic` = measured HBM bytes per
    launch (PMC FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_latest.json)."""
    if label not in stats:
        return None
    n, ms = stats[label]
    avg_s = ms / n / 1e3
    B, J, H, W = wl["B"], wl["J"], wl["H"], wl["W"]
    if label.startswith("edge_step"):
        head = label == "edge_step_head"
        f1, b1 = edge_pass_cost(head, upd)
        flop, byts = E * f1, E * b1 + agg_bytes
        gbs = byts / avg_s / 1e9
        traffic = pmc_traffic("pemp::edge_step_kernel<0," + ("1" if head else "0"), workload, E)
        mb = mfma_busy("edge_step_kernel<0, " + ("1" if head else "0") + ", " + str(PREC_CODE[precision]), workload)
        common = {"kernel": label, "avg_launch_us": round(avg_s * 1e6, 2), "launches": n, "traffic": traffic,
                  "mfma_busy": mb["mfma_busy"] if mb else None,
                  # the same over the SIMDs of the CUs the pass occupies (4 x min(256, workgroups): 192 CUs under
                  # the CU reservation), when the SQ pass recorded it
                  "mfma_busy_used_simds": mb.get("mfma_busy_used") if mb else None,
                  "mfma_busy_cus": mb.get("cus_used") if mb else None,
                  "mfma_busy_source": f"profiles/mfma_latest.json ({workload}): SQ_VALU_MFMA_BUSY_CYCLES / "
                                      f"(1024 SIMDs x GRBM_GUI_ACTIVE / 8); _used_simds: over 4 x cus SIMDs"
                                      if mb is not None else None,
                  "traffic_source": f"profiles/pmc_latest.json ({workload}, E={E})" if traffic else None,
                  "algorithmic": f"{f1} FLOP and {b1} B HBM x E={E} edges + {agg_bytes} B of aggregate rows "
                                 f"per launch",
                  "tflops_executed": round(flop / avg_s / 1e12, 2), "hbm_GBs_algorithmic": round(gbs, 1),
                  "ref_equiv_tflops": round(E * REF_EDGE_FLOP / avg_s / 1e12, 2), "precision": precision}
        if precision == "fp32":
            ach = flop / avg_s / 1e12
            return {**common, "bound": "mfma", "achieved": round(ach, 3), "peak": FP32_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4)}
        t_mfma = 3 * flop / (BF16_MFMA_PEAK_TFLOPS * 1e12)
        t_hbm = byts / (HBM_PEAK_GBS * 1e9)
        if t_mfma >= t_hbm:
            ach = 3 * flop / avg_s / 1e12
            return {**common, "bound": "mfma", "achieved": round(ach, 3), "peak": BF16_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4)}
        return {**common, "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4)}
    if label == "detect_nms":
        byts = B * J * H * W * 4
        ach = byts / avg_s / 1e9
        traffic = pmc_traffic("pemp::nms_strips_kernel", workload, E)
        return {"kernel": label, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": f"profiles/pmc_latest.json ({workload}, E={E})" if traffic else None,
                "avg_launch_us": round(avg_s * 1e6, 2), "launches": n,
                "algorithmic": f"{byts} B per launch (heatmap read once)"}
    return {"kernel": label, "avg_launch_us": round(avg_s * 1e6, 2), "launches": n}


def cpu_baseline(wl, gc, model, hm, feats, tags, budget_s):
    """The oracle restatement (torch CPU fp32, oracle/restate.py) timed per stage on image 0 of the same workload,
    with torch.set_num_threads(os.cpu_count()) as SURVEY 8(d) / BASELINE.md prescribe (`value`), and again with
    16 threads (the GPU box's CPU share per GPU; `threads_16`). The stages run interleaved, one of each per round
    (3 warm-up rounds), so host noise hits them alike; each stage's figure is the least of the medians of three
    blocks of rounds (min-of-medians), so that a noisy block on a shared host does not decide it."""
    from oracle import restate
    mcfg = pcfg.published_mpn_config(wl["J"], wl["steps"], wl["variant"])
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    thr = gc.DETECT_THRESHOLD if gc.DETECT_THRESHOLD <= 1.5 else None
    holder = {}
    if isinstance(hm, torch.Tensor):
        holder["maps"] = hm[0:1].cpu(), feats[0:1].cpu(), tags[0:1].cpu()
        front_stage = ()
    else:
        # multi-scale: the reference's own torch ops project image 0's per-scale outputs to the image size on
        # the CPU (PoseEstimation.py:329-452, multi_scales_testing.py:144-195) before construct_graph reads them
        ph_cpu = pemp_amd.ProjectedHeatmaps([o[0:1].cpu() for o in hm.outputs], hm.size, wl["J"],
                                            [o[0:1].cpu() for o in hm.flip_outputs], hm.flip_index.tolist(),
                                            tag_scale=hm.tag_scale)
        pm_cpu = pemp_amd.ProjectedMaps([m[0:1].cpu() for m in feats.maps], feats.size)

        def frontend():
            s_, t_ = ph_cpu.materialize()
            holder["maps"] = s_, pm_cpu.materialize(), t_

        frontend()
        front_stage = (("frontend", frontend),)

    def detect():
        h = holder["maps"][0]
        holder["det"] = restate.joint_det_from_scoremap(h[0], wl["J"], threshold=thr, pool_kernel=gc.POOL_KERNEL_SIZE,
                                                        hybrid_k=gc.HYBRID_K)

    def graph():
        holder["g"] = restate.construct_graph(*holder["maps"][:2], holder["maps"][2], None, gc, wl["J"])

    def mpn():
        g = holder["g"]
        restate.mpn_forward(sd, mcfg, g[0], g[1], g[2], g[7][:, 2])

    # detect runs right after construct_graph (which contains it), on the same warm heatmap, as inside it
    stage_fns = front_stage + (("construct_graph", graph), ("detect", detect), ("mpn_forward", mpn))

    def timed(threads, budget):
        torch.set_num_threads(threads)
        times = {name: [] for name, _ in stage_fns}
        spent, rounds, warm = 0.0, 0, 3
        for r in range(3 + 15):
            for name, fn in stage_fns:
                t0 = time.perf_counter()
                fn()
                dt = time.perf_counter() - t0
                spent += dt
                if r >= warm:
                    times[name].append(dt)
            if r == 0 and spent > budget / 6:
                warm = 1                     # slow rounds (oversubscribed host): one warm-up round only
            rounds += r >= warm
            print(f"[bench] cpu_baseline {threads} threads: round {r + 1}, {spent:.1f} s", file=sys.stderr, flush=True)
            if rounds >= (6 if warm == 3 else 1) and spent > budget:
                break
        stages = {}
        for name, ts in times.items():
            k = max(1, len(ts) // 3)
            blocks = [ts[i:i + k] for i in range(0, 3 * k, k)]
            stages[name] = round(min(float(np.median(b)) for b in blocks) * 1e3, 3)
        per_image_ms = stages.get("frontend", 0.0) + stages["construct_graph"] + stages["mpn_forward"]
        return {"value": round(1e3 / per_image_ms, 3), "cores": threads, "stage_ms": stages, "rounds": rounds}

    cores = usable_cpus()
    main_run = timed(cores, 0.65 * budget_s)
    share = timed(min(16, cores), 0.35 * budget_s) if cores != min(16, cores) else None
    return {"value": main_run["value"], "unit": "images/s", "cores": cores, "kind": "port",
            "stage_ms": main_run["stage_ms"], "rounds": main_run["rounds"], "threads_16": share,
            "sample": f"image 0 of the {wl['B']}-image workload; detect / construct_graph / mpn_forward interleaved, "
                      f"3 warm-up rounds, then {main_run['rounds']} rounds; per stage the least median of 3 blocks "
                      f"(oracle/restate.py, torch CPU fp32, torch.set_num_threads(every CPU this process may use: "
                      f"os.cpu_count() {os.cpu_count()} limited by affinity and cgroup quota = {cores})); "
                      f"value = 1 / ({'frontend + ' if front_stage else ''}construct_graph + mpn_forward)",
            "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_model": _cpu_model()}


def usable_cpus():
    """CPUs this process can actually run on: os.cpu_count() limited by its affinity mask, OMP_NUM_THREADS and a
    cgroup CPU quota (cgroup v2 cpu.max / v1 cfs_quota_us). On the GPU box os.cpu_count() is the whole machine's 256
    threads while the process's share is 16: torch with 256 threads there thrashes (the MPN leg measured
    108 s instead of 0.05 s), which times the contention, not the host."""
    n = min(os.cpu_count() or 1, len(os.sched_getaffinity(0)))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():   # the host's declared share (16 per GPU on the box)
        n = min(n, max(1, int(os.environ["OMP_NUM_THREADS"])))
    for path, per in (("/sys/fs/cgroup/cpu.max", None), ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us",
                                                         "/sys/fs/cgroup/cpu/cpu.cfs_period_us")):
        try:
            txt = open(path).read().split()
            quota = txt[0]
            period = txt[1] if per is None else open(per).read().strip()
            if quota not in ("max", "-1"):
                n = min(n, max(1, int(int(quota) // int(period))))
            break
        except (OSError, ValueError, IndexError):
            continue
    return n


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def frontend_projection(wl, gc, model, hm, tags, dev, out):
    """SURVEY 8f row 1, informational: the reference projects the gathered features of every image to
    the image size (interpolate bilinear, PoseEstimation.py:426-452) before construct_graph reads N
    rows of it. Times that dense projection (torch on the GPU, [B, 128, H/2, W/2] -> [B, 128, H, W])
    against pemp_gather_projected sampling only the detections (features=ProjectedMaps)."""
    B, H, W = wl["B"], wl["H"], wl["W"]
    low = torch.randn(B, 128, H // 2, W // 2, device=dev)
    reps = 5
    torch.nn.functional.interpolate(low, size=(H, W), mode="bilinear", align_corners=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        torch.nn.functional.interpolate(low, size=(H, W), mode="bilinear", align_corners=False)
    torch.cuda.synchronize()
    dense_ms = (time.perf_counter() - t0) / reps * 1e3
    pm = pemp_amd.ProjectedMaps([low], (H, W))
    _lib.prof_enable("gather_projected")
    for _ in range(reps):
        pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=pm, tagmaps=tags, joints_gt=None, factor_list=None,
                                       masks=None, device=dev, testing=True, heatmaps=None,
                                       num_joints=wl["J"]).construct_graph()
    torch.cuda.synchronize()
    st = _lib.prof_report()
    _lib.prof_enable(None)
    n, ms = st.get("gather_projected", (1, float("nan")))
    # with the model's feature_gather Conv2d(32, 128, 3, 1, 1) in front (PoseEstimation.py:64-66, 341): the
    # reference convolves the whole half-resolution backbone feature map, then projects it
    raw = torch.randn(B, 32, H // 2, W // 2, device=dev)
    conv = torch.nn.Conv2d(32, 128, 3, 1, 1, bias=True).to(dev).eval()
    with torch.no_grad():
        for it in range(reps + 1):
            if it == 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            torch.nn.functional.interpolate(conv(raw), size=(H, W), mode="bilinear", align_corners=False)
        torch.cuda.synchronize()
    dense_conv_ms = (time.perf_counter() - t0) / reps * 1e3
    pmc = pemp_amd.ProjectedMaps([raw], (H, W), gather=conv)
    _lib.prof_enable("gather_projected_conv")
    for _ in range(reps):
        pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=pmc, tagmaps=tags, joints_gt=None, factor_list=None,
                                       masks=None, device=dev, testing=True, heatmaps=None,
                                       num_joints=wl["J"]).construct_graph()
    torch.cuda.synchronize()
    st = _lib.prof_report()
    _lib.prof_enable(None)
    nc, msc = st.get("gather_projected_conv", (1, float("nan")))
    return {"dense_interpolate_ms": round(dense_ms, 3), "on_demand_gather_us": round(ms / n * 1e3, 2),
            "dense_bytes_written": B * 128 * H * W * 4, "nodes": int(out[0].shape[0]),
            "feature_gather_conv": {"dense_conv_then_interpolate_ms": round(dense_conv_ms, 3),
                                    "on_demand_conv_gather_us": round(msc / nc * 1e3, 2),
                                    "conv": "Conv2d(32, 128, 3, 1, 1) on [B, 32, H/2, W/2]"}}


def frontend_heatmaps(wl, gc, feats, dev, reps=5):
    """SURVEY 8f row 1, informational: the test front-end (flip test + project2image, single scale:
    PoseEstimation.py:329-452, multi_scales_testing.py:144-195) in front of construct_graph. With: the
    reference's own torch ops materialise [B, J, H, W] heatmaps and [B, J, H, W, 2] tags from the
    half-resolution network outputs of both passes (interpolate, flip, index, average), then
    construct_graph reads them. Without: ProjectedHeatmaps -- the NMS loads sample the low-resolution
    outputs directly (pemp_detect_projected) and the tags are sampled at the detections."""
    from pemp_amd.frontend import ProjectedHeatmaps
    B, J, H, W = wl["B"], wl["J"], wl["H"], wl["W"]
    h, w = H // 2, W // 2
    fi = [0, 2, 1, 4, 3, 6, 5, 8, 7, 10, 9, 12, 11, 14, 13, 16, 15] if J == 17 else list(range(J))   # COCO flip
    hm = torch.from_numpy(syn.make_heatmaps(2000, B, J, h, w, wl["persons"], sigma=1.0, margin=4)).to(dev)
    hm2 = torch.flip(hm, [3])[:, fi]      # the flipped pass sees the mirrored image with left / right swapped
    g = torch.Generator(device=dev).manual_seed(99)
    outs = torch.cat([hm, torch.rand(B, J, h, w, generator=g, device=dev)], 1)
    flips = torch.cat([hm2, torch.rand(B, J, h, w, generator=g, device=dev)], 1)
    ph = ProjectedHeatmaps([outs], (H, W), J, [flips], fi)

    def graph(scoremaps, tagmaps):
        return pemp_amd.get_graph_constructor(gc, scoremaps=scoremaps, features=feats, tagmaps=tagmaps, joints_gt=None,
                                              factor_list=None, masks=None, device=dev, testing=True, heatmaps=None,
                                              num_joints=J).construct_graph()

    def dense():
        s, t = ph.materialize()
        return graph(s, t)

    # detection alone (the front-end's consumer): the plateau-duplicated peaks of bilinear x2 give ~600 detections
    # per image, so a whole construct_graph here is dominated by its fully graph build, not by the front-end
    gcobj = pemp_amd.get_graph_constructor(gc, scoremaps=ph, features=feats, tagmaps=ph, joints_gt=None,
                                           factor_list=None, masks=None, device=dev, testing=True, heatmaps=None,
                                           num_joints=J)
    L, st = _lib.lib(), _lib.stream(dev)
    use_thr = gcobj.detect_threshold is not None
    topk = gcobj.hybrid_k if use_thr else 20
    thr = float(gcobj.detect_threshold) if use_thr else 0.0
    ws = torch.empty(L.pemp_detect_workspace_size(B, J, H, W, topk), dtype=torch.uint8, device=dev)
    cap = 64 * J
    det = torch.empty(B, cap, 3, dtype=torch.int64, device=dev)
    dsc = torch.empty(B, cap, dtype=torch.float32, device=dev)
    n_det = torch.empty(B, dtype=torch.int32, device=dev)
    pc = ph.c_struct()

    def detect(fn, src):
        _lib.check(fn(src, None, B, J, H, W, gcobj.pool_kernel_size, thr, int(use_thr), topk, 3, _lib.ptr(ws),
                      ws.numel(), _lib.ptr(det), _lib.ptr(dsc), _lib.ptr(n_det), cap, None, st))

    def dense_detect():
        s, _ = ph.materialize()
        detect(L.pemp_detect, _lib.ptr(s))

    res = {}
    for name, fn in (("reference_ops_then_detect_ms", dense_detect),
                     ("projected_detect_ms", lambda: detect(L.pemp_detect_projected, ctypes.addressof(pc)))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4 * reps):
            fn()
        torch.cuda.synchronize()
        res[name] = round((time.perf_counter() - t0) / (4 * reps) * 1e3, 3)
    for name, fn in (("reference_ops_then_construct_graph_ms", dense),
                     ("projected_construct_graph_ms", lambda: graph(ph, ph))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            out = fn()
        torch.cuda.synchronize()
        res[name] = round((time.perf_counter() - t0) / reps * 1e3, 3)
        res["nodes"] = int(out[0].shape[0])
    s_dense, _ = ph.materialize()
    torch.cuda.synchronize()
    _lib.prof_enable("*")
    for _ in range(reps):
        detect(L.pemp_detect, _lib.ptr(s_dense))
        detect(L.pemp_detect_projected, ctypes.addressof(pc))
    torch.cuda.synchronize()
    prof = _lib.prof_report()
    _lib.prof_enable(None)
    for k in ("detect_nms", "detect_nms_projected"):
        n, ms = prof.get(k, (1, float("nan")))
        res[k + "_us"] = round(ms / n * 1e3, 2)
    res["inputs"] = f"2 passes x [{B}, {2 * J}, {h}, {w}] fp32 -> [{B}, {J}, {H}, {W}] scoremaps + [{B}, {J}, {H}, {W}, 2] tags"
    res["dense_bytes_written_by_reference_ops"] = B * J * H * W * 4 * 3
    return res


E2E_NODE_TH = 0.1     # node-probability threshold of the grouping (pred_to_ann th; bench's grouping leg uses the same)


E2E_DEPTH = int(os.environ.get("PEMP_E2E_DEPTH", "2"))   # batches whose grouping is in flight (e2e leg)
E2E_EARLY = os.environ.get("PEMP_E2E_EARLY", "0") not in ("", "0")   # (A/B) launches before the older host parts


def e2e_pipeline(wl, gc, model, hm, feats, tags, dev, steps, warmup, world):
    """The post-backbone step valid.py runs per image (valid.py:101-123), for a whole batch: the test front-end's
    maps (ProjectedHeatmaps for the multi-scale workload) -> construct_graph -> MPN -> sigmoid / softmax
    (valid.py:109-111) -> pred_to_ann (Utils.py:1445-1490): group_persons (GPU edge pass + host GAEC), fill_mean,
    refine and adjust (TEST.WITH_REFINE / TEST.ADJUST of experiments/hybrid_class_agnostic_end2end/
    model_58_4_4.yaml:170-172), reverse_affine_map. The MPN runs in every step; its closed-form weights form
    no person, so the edge / node probabilities the grouping reads are person_structured_probs of the same graph
    (the class probabilities are the MPN's softmax). Pipelined: batch k+1's GPU part (graph, MPN, edge pass,
    copies) is queued before batch k's host part (GAEC, persons) runs and queues its finishing (refine / adjust on
    a side stream), whose keypoints are collected (reverse_affine_map) after batch k+1's grouping, as a server with
    batches in flight would; `serial_*` runs the same steps one after the other."""
    from pemp_amd import pose as ppose
    J, B, H, W = wl["J"], wl["B"], wl["H"], wl["W"]
    maps, tag_maps = dense_maps(hm, tags)
    # the closed-form MPN weights give unstructured probabilities that form no person, so the grouping input is
    # the pose_grouping leg's person-structured edge / node probabilities for the same graph
    out0 = pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                          factor_list=None, masks=None, device=dev, testing=True, heatmaps=None,
                                          num_joints=J).construct_graph()
    syn_probs = person_structured_probs(wl, out0)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    stage = {}

    def clock(name, t0):
        t1 = time.perf_counter()
        stage[name] = stage.get(name, 0.0) + t1 - t0
        return t1

    def gpu_start():
        """batch k+1's launches (detection, capacity graph build, MPN): construct_graph_start, no count wait"""
        t0 = time.perf_counter()
        p = pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                           factor_list=None, masks=None, device=dev, testing=True, heatmaps=None,
                                           num_joints=J).construct_graph_start()
        clock("construct_graph_start", t0)
        return p

    def gpu_part(p=None):
        p = gpu_start() if p is None else p
        t0 = time.perf_counter()
        out = p.result()
        t0 = clock("construct_graph", t0)
        with torch.no_grad():
            pe, pn, pc, _ = model(out[0], out[1], out[2], node_types=out[7][:, 2])
            pe_p, pn_p, pc_p = pe[-1].sigmoid(), pn[-1].sigmoid(), pc[-1].softmax(dim=1)
            if syn_probs:   # same shapes, person-structured (see pose_grouping); the MPN's class softmax is kept
                pe_p, pn_p = syn_probs[0], syn_probs[1]
        t0 = clock("mpn_queue", t0)
        job = ppose.group_persons_start(out[7], pn_p, out[2], pe_p, E2E_NODE_TH, pc_p, "GAEC", J, batch_index=out[12],
                                        score_map_scores=out[11], num_images=B)
        clock("grouping_queue", t0)
        return job

    def host_part(job):
        """grouping (host GAEC) and the finishing queued on the side stream (not waited for)"""
        t0 = time.perf_counter()
        per_image = job.result()
        t0 = clock("grouping_host", t0)
        fin = ppose.finish_batch_start(per_image, maps, tag_maps, adjustment=True, with_refine=True, stream=side)
        clock("finish_queue", t0)
        return fin

    def collect(fin):
        t0 = time.perf_counter()
        done = fin.result()
        t0 = clock("finish_wait", t0)
        res = [None if p is None else ppose.reverse_affine_map(p.copy(), (W, H), W, "short_with_resize") for p in done]
        clock("reverse_affine_map", t0)
        return sum(0 if r is None else len(r) for r in res)

    def run(n, pipelined):
        persons = 0
        if pipelined:
            # three batches in flight: batch k+1's GPU part is queued, then batch k's grouping runs on the host and
            # its finishing is queued on the side stream, then batch k-1's finished keypoints are collected.
            # (Round 6 measured the other order -- batch k+1's graph collected only after batch k's host stages, its
            # count wait overlapped with them -- at 5.6k vs 8.4k images/s at c3: the count wait then became a wait
            # for batch k's GAEC on the grouping thread, which the old order gives that time to finish;
            # profiles/r06_pipelined_steps.md.)
            # E2E_DEPTH batches' groupings in flight: batch k's host part runs once batch k + E2E_DEPTH is queued,
            # so its GPU edge pass, read-back and GAEC (on the grouping thread) have that many iterations to finish
            # (depth 1: the host part waited ~0.2 ms per batch for the GAEC, ~0.13 ms for the finishing,
            # profiles/r06_e2e_depth.md)
            # E2E_EARLY: batch k+1's launches go out first and its count wait comes after the older batches' host
            # parts and collection, which it then overlaps
            from collections import deque
            jobs, fins = deque(), deque()
            for _ in range(n):
                if E2E_EARLY:
                    p = gpu_start()
                    if len(jobs) >= E2E_DEPTH:
                        fins.append(host_part(jobs.popleft()))
                    if len(fins) > 1:
                        persons += collect(fins.popleft())
                    jobs.append(gpu_part(p))
                    continue
                jobs.append(gpu_part())
                if len(jobs) > E2E_DEPTH:
                    fins.append(host_part(jobs.popleft()))
                if len(fins) > 1:
                    persons += collect(fins.popleft())
            while jobs:
                fins.append(host_part(jobs.popleft()))
            while fins:
                persons += collect(fins.popleft())
        else:
            for _ in range(n):
                persons += collect(host_part(gpu_part()))
        return persons

    rec = {}
    for pipelined in (True, False):
        run(max(2, warmup), pipelined)
        stage.clear()
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        persons = run(steps, pipelined)
        torch.cuda.synchronize()
        barrier(world)
        dt = max_over_ranks(time.perf_counter() - t0, world, dev)
        key = "" if pipelined else "serial_"
        rec[key + "images_per_sec"] = round(B * steps * world / dt, 2)
        rec[key + "ms_per_batch"] = round(dt / steps * 1e3, 3)
        if pipelined:
            rec["stage_host_ms_per_batch"] = {k: round(v / steps * 1e3, 3) for k, v in stage.items()}
            rec["persons_per_batch"] = round(persons / steps, 2)
    rec["node_threshold"] = E2E_NODE_TH
    rec["finishing"] = "fill_mean + refine + adjust (model_58_4_4.yaml TEST) + reverse_affine_map short_with_resize"
    return rec


def backbone_leg(wl, dev, steps, step_s, world):
    """SURVEY 8(d) C3's backbone term: a random-weight HigherHRNet-w48 (tools/hrnet_w48.py, the compute graph of
    model_58_4_4.yaml) on B x 3 x 640 x 640 images, bf16 channels-last on torch / MIOpen (the backbone stays on
    PyTorch-ROCm, out of this path's scope), timed like the step; `with_path_images_per_sec` composes it serially
    with the measured post-backbone step (this leg's ms per batch + ms_per_step)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from hrnet_w48 import HigherHRNetW48
    dt_name = os.environ.get("PEMP_BB_DTYPE", "bf16")
    dtype = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[dt_name]
    layout = os.environ.get("PEMP_BB_LAYOUT", "nhwc")   # (measured: 19.6 ms per batch vs 25.2 NCHW, bf16)
    fmt = torch.channels_last if layout == "nhwc" else torch.contiguous_format
    torch.backends.cudnn.benchmark = True
    torch.manual_seed(0)
    net = HigherHRNetW48(wl["J"]).eval().to(dev, dtype=dtype, memory_format=fmt)
    img = torch.randn(wl["B"], 3, 640, 640, device=dev, dtype=dtype).contiguous(memory_format=fmt)
    with torch.no_grad():
        for i in range(3):                     # MIOpen finds / compiles its kernels here
            t0 = time.perf_counter()
            net(img)
            torch.cuda.synchronize()
            print(f"backbone warm-up {i}: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
        barrier(world)
        t0 = time.perf_counter()
        for _ in range(steps):
            net(img)
        torch.cuda.synchronize()
        dt = max_over_ranks((time.perf_counter() - t0) / steps, world, dev)
    flop = 154.3e9   # HigherHRNet-w48 at 640 px: 154.3 GFLOP per image (the architecture's published figure)
    return {"model": "HigherHRNet-w48 (random weights, tools/hrnet_w48.py)", "input": [wl["B"], 3, 640, 640],
            "dtype": f"{dt_name}, {layout}", "ms_per_batch": round(dt * 1e3, 3),
            "images_per_sec": round(wl["B"] * world / dt, 1),
            "tflops": round(flop * wl["B"] / dt / 1e12, 1),
            "with_path_images_per_sec": round(wl["B"] * world / (dt + step_s), 1)}


def person_structured_probs(wl, out):
    """Edge and node probabilities shaped like a trained network's for construct_graph output `out`: node i of
    an image belongs to person (local index mod persons_per_image); edge probabilities sigmoid(+-2.5 + N(0, 1.5))
    for same / different persons, drawn per direction; node probabilities sigmoid(2 + N(0, 1)), except one node in
    six at sigmoid(-4 + N(0, 1)) (below the grouping's 0.1 node threshold): those joints are missing from their
    persons, as occluded joints are, so the finishing's refine has joints to search."""
    det, ei, bi = out[7], out[2], out[12]
    N, E = det.shape[0], ei.shape[1]
    node_off = torch.searchsorted(bi, torch.arange(wl["B"] + 1, device=bi.device))
    pid = (torch.arange(N, device=bi.device) - node_off[bi]) % wl["persons"]
    gen = torch.Generator(device=bi.device).manual_seed(7)
    with torch.no_grad():
        same = pid[ei[0]] == pid[ei[1]]
        pe_p = torch.sigmoid(torch.where(same, 2.5, -2.5) + 1.5 * torch.randn(E, generator=gen, device=bi.device))
        low = torch.rand(N, generator=gen, device=bi.device) < 1.0 / 6.0
        pn_p = torch.sigmoid(torch.where(low, -4.0, 2.0) + torch.randn(N, generator=gen, device=bi.device))
    return pe_p, pn_p


def pose_grouping(wl, out, pe, pn, pc, cpu_ref):
    """SURVEY 8f row 2, informational: the pred_to_ann grouping prefix (node threshold 0.1, GAEC,
    graph_cluster_to_persons; Utils.py:1445-1459) for the whole step's batch, after the MPN and the
    sigmoid / softmax of valid.py:109-111. GPU edge pass + native host GAEC (pemp_amd.pose), against
    the oracle restatement (oracle/pose.py, numpy + pure-Python GAEC, one image at a time, 1 core)."""
    from pemp_amd import pose as ppose
    det, sc, ei, bi = out[7], out[11], out[2], out[12]
    # The closed-form MPN weights give unstructured probabilities (no person would form), so the grouping
    # input is synthetic and person-structured like a trained network's output: node i of an image
    # belongs to person (local index mod persons_per_image); edge probabilities sigmoid(+-2.5 + N(0, 1.5))
    # for same / different persons, drawn per direction; node probabilities sigmoid(2 + N(0, 1)); class
    # probabilities are the MPN's own softmax.
    pe_p, pn_p = person_structured_probs(wl, out)
    with torch.no_grad():
        pc_p = pc[-1].softmax(dim=1)
    args = (det, pn_p, ei, pe_p, 0.1, pc_p, "GAEC", wl["J"])
    ppose.group_persons(*args, batch_index=bi, score_map_scores=sc, num_images=wl["B"])
    reps = 5
    torch.cuda.synchronize()
    _lib.prof_enable("pose_edge_weights")
    t0 = time.perf_counter()
    for _ in range(reps):
        res = ppose.group_persons(*args, batch_index=bi, score_map_scores=sc, num_images=wl["B"])
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    global _LAST_GROUPING
    _LAST_GROUPING = res
    st = _lib.prof_report()
    _lib.prof_enable(None)
    tm = {}
    for _ in range(reps):
        ppose.group_persons(*args, batch_index=bi, score_map_scores=sc, num_images=wl["B"], _timings=tm)
    n, ms = st.get("pose_edge_weights", (1, float("nan")))
    rec = {"ms_per_batch": round(gpu_ms, 3), "edge_pass_us": round(ms / n * 1e3, 2),
           "stage_ms": {k: round(v / reps * 1e3, 3) for k, v in tm.items()},
           "persons": int(sum(0 if r is None else len(r) for r in res)), "images": wl["B"],
           "method": "GAEC", "node_threshold": 0.1}
    if cpu_ref:
        from oracle import pose as opose
        h = [t.cpu().numpy() for t in (det, pn_p, ei, pe_p, pc_p, bi, sc)]
        t0 = time.perf_counter()
        for b in range(wl["B"]):
            nm = h[5] == b
            lo = int(np.nonzero(nm)[0][0])
            em = nm[h[2][0]]
            opose.pred_to_ann_persons(h[0][nm], h[1][nm], h[2][:, em] - lo, h[3][em], np.float32(0.1), h[4][nm],
                                      "GAEC", wl["J"], h[6][nm])
        rec["cpu_oracle_ms_per_batch"] = round((time.perf_counter() - t0) * 1e3, 1)
    rec["refine"] = pose_refine(wl, res, cpu_ref)
    return rec


def pose_refine(wl, persons, cpu_ref):
    """SURVEY 8f row 3, informational: refine (Utils.py:1026-1104) of image 0's grouped persons on its
    full-size [J, H, W] scoremaps and [J, H, W, 1] tag maps (the pred_to_ann order: fill_mean, refine,
    adjust). GPU kernels vs the oracle restatement (numpy, the reference's own ops)."""
    from pemp_amd import pose as ppose
    hm, tags = _BENCH_MAPS
    kp0 = next((p for p in persons if p is not None), None)
    if kp0 is None:
        return None
    kp0 = ppose.fill_mean(np.ascontiguousarray(kp0, dtype=np.float64).copy())
    s, tg = hm[0], tags[0]
    J, H, W = s.shape
    P = kp0.shape[0]
    ppose.refine(s, tg, kp0.copy())
    reps = 5
    torch.cuda.synchronize()
    _lib.prof_enable("pose_refine")
    t0 = time.perf_counter()
    for _ in range(reps):
        ppose.refine(s, tg, kp0.copy())
    ms = (time.perf_counter() - t0) / reps * 1e3
    st = _lib.prof_report()
    _lib.prof_enable(None)
    n, kms = st.get("pose_refine", (1, float("nan")))
    F = tg.shape[-1] if tg.dim() == 4 else 1
    byts = J * H * W * (4 + 4 * F)
    rec = {"persons": P, "map": [J, H, W, F], "ms_per_image": round(ms, 3), "kernels_us": round(kms / n * 1e3, 2),
           "algorithmic_bytes": byts, "hbm_GBs_algorithmic": round(byts / (kms / n * 1e-3) / 1e9, 1)}
    if cpu_ref:
        from oracle import pose as opose
        sh, th = s.cpu().numpy(), tg.cpu().numpy()
        t0 = time.perf_counter()
        opose.refine(sh, th, kp0.copy())
        rec["cpu_oracle_ms_per_image"] = round((time.perf_counter() - t0) * 1e3, 1)
    return rec


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    rank, world, dev = setup_dist(args.gpus)
    wl = WORKLOADS[args.workload]
    gc = pcfg.inference_gc_config(wl["graph"], 5, False)
    hm, feats, tags = make_inputs(wl, rank, dev)
    model, _ = make_model(wl, dev)
    if wl["graph"] == "fully" and not os.environ.get("PEMP_NO_CAP_MPN"):
        pemp_amd.bind_mpn(model)   # capacity mode: the MPN queued behind the graph build, ahead of the counts
    _lib.lib()

    if args.profile_steps:
        # (--streams S > 1: the steps round-robin on S streams, as the timed region runs them)
        ps = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(max(args.streams, 1) - 1)]
        for i in range(max(args.warmup, len(ps))):
            with torch.cuda.stream(ps[i % len(ps)]):
                run_step(wl, gc, model, hm, feats, tags, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            with torch.cuda.stream(ps[i % len(ps)]):
                run_step(wl, gc, model, hm, feats, tags, dev)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if rank == 0:
            print(json.dumps({"profile_steps": args.steps, "workload": args.workload,
                              "ms_per_step": round(dt / args.steps * 1e3, 3), "graph_stats": graph_stats()}),
                  flush=True)
        return

    # batches in flight: each stream has its own library scratch (construct_graph and the MPN are
    # reentrant per (device, stream)); inputs are read-only and resident before the timed region
    S = max(1, args.streams) if args.streams > 0 else 2
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    torch.cuda.synchronize()
    for w in range(S):    # per-stream scratch and side streams allocated outside the timed region
        with torch.cuda.stream(streams[w]):
            run_step(wl, gc, model, hm, feats, tags, dev)
    torch.cuda.synchronize()
    schedule_probe = None
    if args.streams == 0:
        # two batches in flight overlap one batch's detection with the other's MPN, but on some boxes the
        # interleaving of the two queues serialises worse than one stream: time both schedules here (outside
        # the timed region, every rank the same choice) and run the faster one
        # (each trial runs >= 20 ms of steps: a batch-1 step of ~0.2 ms over the warmup count alone left the two
        # schedules inside the host's noise; the count comes from a calibration run, the same on every rank)
        def probe_run(S_try, n):
            barrier(world)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run_steps(n, streams, S_try, wl, gc, model, hm, feats, tags, dev)
            torch.cuda.synchronize()
            return max_over_ranks(time.perf_counter() - t0, world, dev)
        n_probe = max(args.warmup, 4)
        n_probe = max(n_probe, min(400, math.ceil(n_probe * 0.02 / max(probe_run(1, n_probe), 1e-6))))
        probe = {}
        for S_try in (2, 1, 2, 1):
            per_step = probe_run(S_try, n_probe) / n_probe
            probe[S_try] = min(probe.get(S_try, per_step), per_step)
        S = 2 if probe[2] < probe[1] else 1
        schedule_probe = {f"streams_{k}_ms_per_step": round(v * 1e3, 3) for k, v in probe.items()}
        schedule_probe["steps_per_trial"] = n_probe

    # warmup (also finds the dominant kernel with the profiler on for every kernel)
    dominant = dominant_overall = None
    for w in range(max(args.warmup, 1)):
        if w == max(args.warmup, 1) - 1 and not args.no_roofline:
            _lib.prof_enable("*")
        out, pe, pn, pc = run_step(wl, gc, model, hm, feats, tags, dev)
    torch.cuda.synchronize()
    N, E = int(out[0].shape[0]), int(out[2].shape[1])
    if not args.no_roofline:
        stats = _lib.prof_report()
        _lib.prof_enable(None)
        totals = {k: v[1] for k, v in stats.items()}
        # the roofline kernel: the largest total time among the kernels with an algorithmic-bytes model (edge
        # passes, NMS); at batch 1 the node kernels' launch latency can total more (reported beside it)
        modelled = {k: v for k, v in totals.items() if k.startswith("edge_step") or k == "detect_nms"}
        pool = modelled or totals
        dominant = max(pool, key=pool.get) if pool else None
        dominant_overall = max(totals, key=totals.get) if totals else None
        breakdown = {k: round(v[1] / v[0] * 1e3, 2) for k, v in stats.items()}

    # timed region (value): the path alone, no profiler events; step i on stream i % S (run_steps)
    run_steps(args.warmup, streams, S, wl, gc, model, hm, feats, tags, dev)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps, streams, S, wl, gc, model, hm, feats, tags, dev)
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    dt_max = max_over_ranks(dt, world, dev)
    imgs = wl["B"] * args.steps * world
    value = imgs / dt_max
    # the same K steps strictly serial on one stream (reported beside value)
    value_serial = None
    if S > 1:
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run_step(wl, gc, model, hm, feats, tags, dev)
        torch.cuda.synchronize()
        barrier(world)
        value_serial = imgs / max_over_ranks(time.perf_counter() - t0, world, dev)
    E_all = sum_over_ranks(E, world, dev)

    # roofline: the same K steps again with HIP events recorded on the launch stream of the dominant
    # kernel (the library's profiler), kept out of `value` because the event records add host work to
    # the step. The edge passes are idempotent: each is launched ROOF_REPEAT times back to back inside
    # one event pair, so the per-launch average carries no event-record overhead
    stats_timed = {}
    if dominant:
        _lib.prof_enable(f"{dominant}@{ROOF_REPEAT}" if dominant.startswith("edge_step") else dominant)
        barrier(world)
        torch.cuda.synchronize()
        for _ in range(args.steps):
            run_step(wl, gc, model, hm, feats, tags, dev)
        torch.cuda.synchronize()
        barrier(world)
        stats_timed = _lib.prof_report()
        _lib.prof_enable(None)

    # isolated MPN (same graphs): edge-updates/s
    x, ea, ei, types = out[0], out[1], out[2], out[7][:, 2]
    with torch.no_grad():
        for _ in range(2):
            model(x, ea, ei, node_types=types)
    barrier(world)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    with torch.no_grad():
        for _ in range(args.steps):
            model(x, ea, ei, node_types=types)
    torch.cuda.synchronize()
    barrier(world)
    dt_mpn = max_over_ranks(time.perf_counter() - t1, world, dev)
    mpn_eups = E_all * wl["steps"] * args.steps / dt_mpn

    e2e = e2e_pipeline(wl, gc, model, hm, feats, tags, dev, args.steps, args.warmup, world) \
        if not args.no_roofline else None
    # (single-scale workloads: the front-end legs beside the step; a multi-scale workload runs them inside it)
    single = not wl.get("scales")
    front = frontend_projection(wl, gc, model, hm, tags, dev, out) if single and not args.no_roofline else None
    front_hm = frontend_heatmaps(wl, gc, feats, dev) if single and not args.no_roofline else None

    global _BENCH_MAPS
    _BENCH_MAPS = dense_maps(hm, tags)
    grouping = pose_grouping(wl, out, pe, pn, pc, rank == 0 and world == 1 and not args.no_cpu_baseline) \
        if not args.no_roofline else None
    if grouping is not None and world > 1:
        # the one data collective of the sharded path -- every rank's grouped poses to all ranks
        try:
            start, _ = pdist.image_block(wl["B"] * world, rank, world)
            barrier(world)
            t2 = time.perf_counter()
            ids, poses = pdist.gather_poses(_LAST_GROUPING, list(range(start, start + wl["B"])), wl["J"], world, dev,
                                            total_images=wl["B"] * world)
            grouping["pose_all_gather_ms"] = round((time.perf_counter() - t2) * 1e3, 3)
            grouping["gathered_images"] = len(ids)
        except Exception as exc:  # informational field only: never lose the bench line over it
            grouping["pose_all_gather_error"] = repr(exc)[:200]

    upd = wl["variant"] in ("attn", "mean")      # update block pre-applied in the edge pass (mpn.hip UPD)
    roof = roofline_for(dominant, stats_timed, E, wl, model.precision, upd, args.workload,
                        seg_rows_bytes(out[2], out[7][:, 2])) if dominant else None
    if roof is not None and dominant_overall != dominant:
        roof["largest_total_time_kernel"] = dominant_overall
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(wl, gc, model, hm, feats, tags, args.cpu_seconds)
    bb = None
    if not args.no_backbone and not args.no_roofline:
        try:   # (an informational leg: never lose the bench line over it)
            bb = backbone_leg(wl, dev, args.steps, dt_max / args.steps, world)
        except Exception as exc:
            bb = {"error": repr(exc)[:200]}

    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": model.precision,
            "data": "synthetic (seeded planted-Gaussian heatmaps, random features; closed-form MPN weights)",
            "config": {"workload": f"{args.workload}: {wl['B']}x{wl['J']}x{wl['H']}x{wl['W']} heatmaps/GPU -> "
                                   f"{wl['graph']} graph -> MPN TypeAware-attn T={wl['steps']}",
                       "images_per_gpu": wl["B"], "global_batch": wl["B"] * world, "persons_per_image": wl["persons"],
                       "nodes_per_gpu": N, "edges_per_gpu": E, "parallelism": f"image-sharded x{world}",
                       "batches_in_flight": S,
                       "mpn_edge_gemms": PREC_NOTE[model.precision],
                       "detection_and_node_math": "fp32"},
            "value_serial_steps": round(value_serial if value_serial else value, 2) if (value_serial or S == 1) else None,
            "schedule_probe": schedule_probe,
            # the whole post-backbone step of valid.py (grouping and finishing included), pipelined over batches
            "e2e_images_per_sec": e2e["images_per_sec"] if e2e else None,
            "e2e": e2e,
            "mpn_edge_updates_per_sec": round(mpn_eups, 1),
            "mpn_ms_per_step": round(dt_mpn / args.steps * 1e3, 3),
            "pipeline_edge_updates_per_sec": round(E_all * wl["steps"] * args.steps / dt_max, 1),
            "roofline": roof,
            "kernel_avg_us": breakdown if not args.no_roofline else None,
            "cpu_baseline": cpu,
            "frontend_projection": front,
            "frontend_heatmaps": front_hm,
            "pose_grouping": grouping,
            # the one collective of the sharded path (RCCL all_gather of every rank's grouped poses)
            "pose_all_gather_ms": grouping.get("pose_all_gather_ms") if grouping else None,
            "capacity_graphs": graph_stats(),
            "backbone": bb,
        }
        if cpu:
            rec["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
