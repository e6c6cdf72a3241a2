"""Image sharding over ranks (one process per GPU) — the multi-GPU contract of SURVEY §8(e).

Images are independent units (the reference loops over them: ``ConstructGraph.py:58``,
``valid.py:95``), so a batch is split into contiguous image blocks per rank and every rank runs
the whole path on its block with no data-path collective. The collectives are the timing
reductions of the benchmark (max of elapsed time, sum of work), the barrier around it, and after
pose grouping the one pose all-gather of §8(e) (``gather_poses``).
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend="nccl"):
    """(rank, world, device) from the torchrun environment; initialises the process group when
    WORLD_SIZE > 1 (rendezvous on 127.0.0.1 unless MASTER_ADDR is set).

    Rehearsal knobs (one-GPU boxes; never the production setting): PEMP_DIST_BACKEND=gloo runs the
    collectives over gloo on host copies while every rank still computes on its GPU, and
    PEMP_SHARE_DEVICE=1 puts every rank on cuda:0 (RCCL refuses two ranks on one device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = backend == "nccl"
    backend = os.environ.get("PEMP_DIST_BACKEND", backend) if gpu else backend
    if gpu:
        shared = os.environ.get("PEMP_SHARE_DEVICE", "0") == "1"
        dev = torch.device("cuda", local if world > 1 and not shared else 0)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world, dev


def _coll_dev(dev):
    """Where collective buffers live: the rank's device under RCCL, host memory under gloo."""
    return torch.device("cpu") if dist.is_initialized() and dist.get_backend() == "gloo" else dev


def image_block(total, rank, world):
    """Contiguous [start, stop) image range of ``rank``: sizes differ by at most one."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def barrier(world):
    if world > 1:
        dist.barrier()


def _reduce(v, world, dev, op):
    if world == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=_coll_dev(dev))
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(v, world, dev):
    return _reduce(v, world, dev, dist.ReduceOp.MAX)


def sum_over_ranks(v, world, dev):
    return _reduce(v, world, dev, dist.ReduceOp.SUM)


def gather_poses(per_image, image_ids, num_joints, world, dev):
    """after each rank has grouped its own image block, one all_gather hands every rank the
    poses of the whole batch, in global image order (rank order of the contiguous blocks).

    per_image: this rank's list of float64 [P, J, 3] arrays or None (``pred_to_ann``'s "no poses");
    image_ids: this rank's int image ids, same length. Returns (ids, poses) over all ranks. Records are
    fixed-size ([cap, J, 3] f64 + person count + image id, cap = the largest P over all ranks, found by one
    MAX all-reduce), blocks padded to the largest block; float64 keeps every value exact."""
    n_local = len(per_image)
    if len(image_ids) != n_local:
        raise ValueError("gather_poses: per_image and image_ids differ in length")
    if world == 1:
        return list(image_ids), list(per_image)
    p_local = max([0] + [0 if p is None else int(p.shape[0]) for p in per_image])
    dev = _coll_dev(dev)
    t = torch.tensor([p_local, n_local], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    cap, n_max = max(1, int(t[0])), max(1, int(t[1]))
    rec = torch.zeros(n_max, cap, num_joints, 3, dtype=torch.float64)
    meta = torch.full((n_max, 3), -1, dtype=torch.int64)   # (image id, person count or -1 for None, valid)
    meta[:, 2] = 0
    for k, (p, iid) in enumerate(zip(per_image, image_ids)):
        meta[k, 0] = int(iid)
        meta[k, 2] = 1
        if p is not None:
            rec[k, :p.shape[0]] = torch.from_numpy(p)
            meta[k, 1] = p.shape[0]
    rec, meta = rec.to(dev), meta.to(dev)
    all_rec = torch.empty((world * n_max,) + tuple(rec.shape[1:]), dtype=rec.dtype, device=dev)
    all_meta = torch.empty((world * n_max, 3), dtype=meta.dtype, device=dev)
    dist.all_gather_into_tensor(all_rec, rec)
    dist.all_gather_into_tensor(all_meta, meta)
    all_rec = all_rec.cpu().numpy().reshape((world, n_max) + tuple(rec.shape[1:]))
    all_meta = all_meta.cpu().numpy().reshape(world, n_max, 3)
    ids, poses = [], []
    for r in range(world):
        for k in range(n_max):
            iid, cnt, valid = all_meta[r, k]
            if not valid:
                continue
            ids.append(int(iid))
            poses.append(None if cnt < 0 else all_rec[r, k, :cnt].copy())
    return ids, poses
