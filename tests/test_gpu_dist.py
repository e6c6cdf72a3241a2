"""Multi-process coverage of the image-sharded path on the GPU: two ranks share cuda:0 and run
the HIP path (construct_graph, the MPN, pose grouping) on their image blocks, with the collectives over gloo
(`PEMP_DIST_BACKEND=gloo PEMP_SHARE_DEVICE=1`, the one-GPU rehearsal of `pemp_amd.dist`; RCCL itself needs one
GPU per rank). Checked against one process running the whole batch: the graph shards re-assemble bit for bit,
the shards' logits agree with the whole batch's within the logit bar (the edge-pass work split depends on the
graph it is given, so segments are cut into pieces at other places), and both ranks receive the same
batch-ordered poses from `gather_poses`, each rank's block being exactly what it grouped itself.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, J, H, W, PERSONS = 4, 17, 96, 96, 3
TOL = 1e-4


def _inputs(dev):
    from pemp_amd import synthetic as syn
    hm = torch.from_numpy(syn.make_heatmaps(23, B, J, H, W, PERSONS)).to(dev)
    feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25)).to(dev)
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75)).to(dev)
    return hm, feats, tags


def _path(hm, feats, tags, dev):
    """construct_graph + MPN + grouping on a block of images (the HIP path)."""
    import pemp_amd
    from pemp_amd import config as pcfg, pose as ppose, synthetic as syn
    gc = pcfg.inference_gc_config("fully", 5, False)
    out = pemp_amd.get_graph_constructor(gc, scoremaps=hm, features=feats, tagmaps=tags, joints_gt=None,
                                         factor_list=None, masks=None, device=dev, testing=True, heatmaps=None,
                                         num_joints=J).construct_graph()
    cfg = pcfg.published_mpn_config(J, 3, "attn")
    model = pemp_amd.get_mpn_model(cfg)
    model.load_state_dict(syn.closed_form_state_dict(model, 1.5))
    model.eval().to(dev)
    with torch.no_grad():
        pe, pn, pc, _ = model(out[0], out[1], out[2], node_types=out[7][:, 2])
    torch.cuda.synchronize()
    # person-structured probabilities (the closed-form weights form no persons; as bench.py's grouping leg):
    # node i of an image belongs to person (local index mod PERSONS)
    det, ei, bi = out[7], out[2], out[12]
    node_off = torch.searchsorted(bi, torch.arange(hm.shape[0] + 1, device=dev))
    pid = (torch.arange(det.shape[0], device=dev) - node_off[bi]) % PERSONS
    pe_p = torch.sigmoid(torch.where(pid[ei[0]] == pid[ei[1]], 2.5, -2.5))
    pn_p = torch.full((det.shape[0],), 0.9, device=dev)
    per_image = ppose.group_persons(det, pn_p, ei, pe_p, 0.1, pc[-1].softmax(dim=1), "GAEC", J, batch_index=bi,
                                    score_map_scores=out[11], num_images=hm.shape[0])
    graph = {k: out[i].cpu() for k, i in (("x", 0), ("ea", 1), ("ei", 2), ("det", 7), ("bi", 12))}
    logits = {"edge": pe[-1].cpu(), "node": pn[-1].cpu(), "class": pc[-1].cpu()}
    return graph, logits, per_image


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PEMP_DIST_BACKEND="gloo", PEMP_SHARE_DEVICE="1")
    from pemp_amd import dist as pdist
    r, w, dev = pdist.init_from_env("nccl")
    assert (r, w) == (rank, world) and dev == torch.device("cuda", 0)
    hm, feats, tags = _inputs(dev)
    s, e = pdist.image_block(B, r, w)
    graph, logits, per_image = _path(hm[s:e], feats[s:e], tags[s:e], dev)
    ids, poses = pdist.gather_poses(per_image, list(range(s, e)), J, w, dev, total_images=B)
    torch.save({"graph": graph, "logits": logits, "start": s, "ids": ids,
                "local": [None if p is None else torch.from_numpy(np.asarray(p)) for p in per_image],
                "poses": [None if p is None else torch.from_numpy(np.asarray(p)) for p in poses]},
               os.path.join(out_dir, f"r{r}.pt"))
    torch.distributed.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _same(a, b):
    return (a is None and b is None) or (a is not None and b is not None and torch.equal(a, b))


@pytest.mark.timeout(600)
def test_two_ranks_share_gpu_hip_path(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    parts = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    dev = torch.device("cuda", 0)
    full_graph, full_logits, _ = _path(*_inputs(dev), dev)
    # graph: node blocks in rank order, edge indices offset by the earlier shards' nodes
    off = np.cumsum([0] + [p["graph"]["x"].shape[0] for p in parts])
    assert torch.equal(torch.cat([p["graph"]["x"] for p in parts]), full_graph["x"])
    assert torch.equal(torch.cat([p["graph"]["det"] for p in parts]), full_graph["det"])
    assert torch.equal(torch.cat([p["graph"]["ea"] for p in parts]), full_graph["ea"])
    assert torch.equal(torch.cat([p["graph"]["ei"] + int(off[i]) for i, p in enumerate(parts)], 1), full_graph["ei"])
    assert torch.equal(torch.cat([p["graph"]["bi"] + p["start"] for p in parts]), full_graph["bi"])
    for k in ("edge", "node", "class"):
        got = torch.cat([p["logits"][k] for p in parts])
        assert got.shape == full_logits[k].shape
        assert (got - full_logits[k]).abs().max().item() < TOL, k
    # gather_poses: every rank holds the whole batch in image order; rank r's block is what it grouped
    assert parts[0]["ids"] == parts[1]["ids"] == list(range(B))
    assert sum(0 if q is None else q.shape[0] for q in parts[0]["poses"]) > 0   # persons were formed
    for a, b in zip(parts[0]["poses"], parts[1]["poses"]):
        assert _same(a, b)
    for p in parts:
        s = p["start"]
        for k, loc in enumerate(p["local"]):
            assert _same(parts[0]["poses"][s + k], loc)


@pytest.mark.timeout(420)
def test_bench_spawns_ranks():
    """`python bench.py --gpus 2` with no launcher starts its two rank processes itself (bench.spawn_ranks) and
    prints one line for the 2-rank job: n_gpus 2, the global batch of both image blocks, and the timed pose
    all-gather. One-GPU rehearsal: both ranks on cuda:0, collectives over gloo."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PEMP_SHARE_DEVICE="1", PEMP_DIST_BACKEND="gloo")
    res = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--no-cpu-baseline", "--no-backbone", "--streams", "1"], cwd=root, env=env,
                         capture_output=True, text=True, timeout=400)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 16 and rec["config"]["images_per_gpu"] == 8
    assert rec["pose_all_gather_ms"] is not None and rec["pose_grouping"]["gathered_images"] == 16
    assert rec["value"] > 0
