"""Image sharding over ranks (one process per GPU) — the multi-GPU contract of SURVEY §8(e).

Images are independent units (the reference loops over them: ``ConstructGraph.py:58``,
``valid.py:95``), so a batch is split into contiguous image blocks per rank and every rank runs
the whole path on its block with no data-path collective. The collectives are the timing
reductions of the benchmark (max of elapsed time, sum of work), the barrier around it, and after
pose grouping the one pose all-gather of §8(e) (``gather_poses``).
"""
import os

import numpy as np
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


# DATASET.MAX_NUM_PEOPLE (/root/reference/src/config/default_config.py:175): the fixed person capacity of one
# image's pose record, so that every rank knows the record size without a collective of its own
MAX_NUM_PEOPLE = 30
_META = 4   # record header: image id, person count (-1: None), valid flag, spare (all exact in float64)


def _pack_records(per_image, image_ids, n_max, cap, num_joints, skip=0):
    """[n_max, _META + cap*J*3] float64: per image the header and persons skip .. skip+cap-1 of its poses."""
    stride = cap * num_joints * 3
    rec = torch.zeros(n_max, _META + stride, dtype=torch.float64)
    rec[:, 1] = -1
    for k, (p, iid) in enumerate(zip(per_image, image_ids)):
        rec[k, 0] = int(iid)
        rec[k, 2] = 1
        if p is not None:
            rec[k, 1] = p.shape[0]
            part = p[skip:skip + cap]
            if part.shape[0]:
                rec[k, _META:_META + part.size] = torch.from_numpy(np.ascontiguousarray(part, dtype=np.float64)).reshape(-1)
    return rec


def _all_gather_records(rec, world, dev):
    out = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=dev)
    dist.all_gather_into_tensor(out, rec.to(dev))
    return out.cpu().numpy().reshape(world, rec.shape[0], rec.shape[1])


def gather_poses(per_image, image_ids, num_joints, world, dev, total_images=None, max_people=MAX_NUM_PEOPLE):
    """after each rank has grouped its own image block, ONE all_gather hands every rank the
    poses of the whole batch, in global image order (rank order of the contiguous blocks).

    per_image: this rank's list of float64 [P, J, 3] arrays or None (``pred_to_ann``'s "no poses");
    image_ids: this rank's int image ids, same length. Returns (ids, poses) over all ranks.

    Each image is one fixed-size float64 record packed into a single tensor: header (image id, person count,
    valid) + [max_people, J, 3] poses, max_people = DATASET.MAX_NUM_PEOPLE = 30. Every rank derives the block
    size from ``total_images`` (the ``image_block`` partition: ceil(total / world) records per rank, shorter
    blocks padded with invalid records); without it every rank must hold the same number of images. So the
    common case is exactly one collective, no size agreement first. An image with more than max_people
    persons (the grouping caps nothing) is still exact: every rank sees the counts after the first gather and
    the rare overflow persons travel in one more all_gather of the same form. float64 keeps every value exact."""
    n_local = len(per_image)
    if len(image_ids) != n_local:
        raise ValueError("gather_poses: per_image and image_ids differ in length")
    if world == 1:
        return list(image_ids), list(per_image)
    n_max = max(1, -(-int(total_images) // world)) if total_images is not None else max(1, n_local)
    if n_local > n_max:
        raise ValueError(f"gather_poses: {n_local} images on this rank, block size {n_max}")
    cap = max(1, int(max_people))
    dev = _coll_dev(dev)
    allr = _all_gather_records(_pack_records(per_image, image_ids, n_max, cap, num_joints), world, dev)
    counts = allr[:, :, 1].astype(np.int64)
    over = int(max(0, counts.max() - cap))
    extra = None
    if over:   # (all ranks take this branch together: they all hold the same counts)
        extra = _all_gather_records(_pack_records(per_image, image_ids, n_max, over, num_joints, skip=cap),
                                    world, dev)
    ids, poses = [], []
    for r in range(world):
        for k in range(n_max):
            if not allr[r, k, 2]:
                continue
            ids.append(int(allr[r, k, 0]))
            cnt = int(counts[r, k])
            if cnt < 0:
                poses.append(None)
                continue
            p = allr[r, k, _META:].reshape(cap, num_joints, 3)[:min(cnt, cap)]
            if cnt > cap:
                p = np.concatenate([p, extra[r, k, _META:].reshape(over, num_joints, 3)[:cnt - cap]])
            poses.append(p.copy())
    return ids, poses
