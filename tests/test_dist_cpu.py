"""Multi-process (gloo, world_size 2, CPU) coverage of the image-sharded path.

Each rank takes its contiguous image block, builds the graph of its images with the CPU oracle
(the HIP path needs a GPU; the sharding logic is the same), and the test checks that the shards
re-assemble to the single-process result: sharding over images is exact and needs no data-path
collective. The benchmark's timing reductions (max of time, sum of work) are checked too.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import restate
from pemp_amd import config as pcfg, dist as pdist, synthetic as syn

B, J, H, W, PERSONS = 5, 17, 64, 64, 3


def _inputs():
    hm = torch.from_numpy(syn.make_heatmaps(11, B, J, H, W, PERSONS))
    feats = torch.from_numpy(syn.closed_form((B, 128, H, W), 0.25))
    tags = torch.from_numpy(syn.closed_form((B, J, H, W, 1), 0.75))
    return hm, feats, tags


def _graph(hm, feats, tags):
    return restate.construct_graph(hm, feats, tags, None, pcfg.inference_gc_config("fully", 5, False), J)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, dev = pdist.init_from_env("gloo")
    assert (r, w) == (rank, world)
    hm, feats, tags = _inputs()
    s, e = pdist.image_block(B, r, w)
    g = _graph(hm[s:e], feats[s:e], tags[s:e])
    pdist.barrier(w)
    t_max = pdist.max_over_ranks(float(r + 1), w, dev)
    n_sum = pdist.sum_over_ranks(float(g[0].shape[0]), w, dev)
    torch.save({"x": g[0], "ea": g[1], "ei": g[2], "det": g[7], "bi": g[12], "start": s, "t_max": t_max,
                "n_sum": n_sum}, os.path.join(out_dir, f"r{r}.pt"))
    torch.distributed.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_image_block_partition():
    for total in (0, 1, 7, 8, 64):
        for world in (1, 2, 3, 8):
            blocks = [pdist.image_block(total, r, world) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == total
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.timeout(300)
def test_gloo_world2_shards_reassemble(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    parts = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    full = _graph(*_inputs())
    # nodes: concatenation in rank order; edges: per-shard indices offset by the earlier shards
    x = torch.cat([p["x"] for p in parts])
    det = torch.cat([p["det"] for p in parts])
    off = np.cumsum([0] + [p["x"].shape[0] for p in parts])
    ei = torch.cat([p["ei"] + int(off[i]) for i, p in enumerate(parts)], 1)
    bi = torch.cat([p["bi"] + p["start"] for p in parts])
    assert torch.equal(x, full[0]) and torch.equal(det, full[7])
    assert torch.equal(ei, full[2]) and torch.equal(torch.cat([p["ea"] for p in parts]), full[1])
    assert torch.equal(bi, full[12])
    assert all(p["t_max"] == world for p in parts)
    assert all(p["n_sum"] == full[0].shape[0] for p in parts)


def _poses_for(img, crowded=False):
    """Deterministic per-image pose arrays (None for some images, varying person counts; ``crowded``: image 3
    holds more persons than MAX_NUM_PEOPLE, the record capacity)."""
    rng = np.random.default_rng(img)
    n = int(rng.integers(0, 5)) if not (crowded and img == 3) else pdist.MAX_NUM_PEOPLE + 7
    if n == 0:
        return None
    kp = rng.integers(0, 640, size=(n, J, 3)).astype(np.float64) + 0.25
    kp[:, :, 2] = rng.random((n, J)).astype(np.float32)
    kp[0, 0, 2] = 0.001
    return kp


def _pose_worker(rank, world, port, out_dir, total, crowded):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, w, dev = pdist.init_from_env("gloo")
    s, e = pdist.image_block(total, r, w)
    # count every collective gather_poses issues (one all_gather, nothing to agree a size first)
    calls = []
    for name in ("all_gather_into_tensor", "all_gather", "all_reduce", "broadcast", "all_to_all_single"):
        orig = getattr(torch.distributed, name)
        setattr(torch.distributed, name, (lambda f, n: (lambda *a, **k: (calls.append(n), f(*a, **k))[1]))(orig, name))
    ids, poses = pdist.gather_poses([_poses_for(i, crowded) for i in range(s, e)], [1000 + i for i in range(s, e)],
                                    J, w, dev, total_images=total)
    np.savez(os.path.join(out_dir, f"p{r}.npz"), ids=np.array(ids), calls=np.array(calls),
             counts=np.array([-1 if p is None else len(p) for p in poses]),
             flat=np.concatenate([p.reshape(-1) for p in poses if p is not None] or [np.zeros(0)]))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("total,crowded", [(5, False), (4, False), (5, True)])
def test_gloo_world2_gather_poses(tmp_path, total, crowded):
    """The §8(e) pose all-gather: every rank ends with every image's poses, in global order, exact, through
    exactly one all_gather of fixed [MAX_NUM_PEOPLE x J x 3] records (a second one only for an image with
    more persons than that: the crowded case)."""
    world = 2
    mp.start_processes(_pose_worker, args=(world, _free_port(), str(tmp_path), total, crowded), nprocs=world,
                       join=True, start_method="spawn")
    ref = [_poses_for(i, crowded) for i in range(total)]
    for r in range(world):
        z = np.load(tmp_path / f"p{r}.npz")
        assert z["calls"].tolist() == ["all_gather_into_tensor"] * (2 if crowded else 1)
        assert z["ids"].tolist() == [1000 + i for i in range(total)]
        assert z["counts"].tolist() == [-1 if p is None else len(p) for p in ref]
        flat = np.concatenate([p.reshape(-1) for p in ref if p is not None] or [np.zeros(0)])
        np.testing.assert_array_equal(z["flat"], flat)
