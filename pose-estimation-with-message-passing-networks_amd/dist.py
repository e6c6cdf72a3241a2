"""Image sharding over ranks (one process per GPU) — the multi-GPU contract of SURVEY §8(e).

Images are independent units (the reference loops over them: ``ConstructGraph.py:58``,
``valid.py:95``), so a batch is split into contiguous image blocks per rank and every rank runs
the whole path on its block with no data-path collective. The only collectives are the timing
reductions of the benchmark (max of elapsed time, sum of work) and the barrier around it.
"""
import os

import torch
import torch.distributed as dist


def init_from_env(backend="nccl"):
    """(rank, world, device) from the torchrun environment; initialises the process group when
    WORLD_SIZE > 1 (rendezvous on 127.0.0.1 unless MASTER_ADDR is set)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        dev = torch.device("cuda", local if world > 1 else 0)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world, dev


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
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(v, world, dev):
    return _reduce(v, world, dev, dist.ReduceOp.MAX)


def sum_over_ranks(v, world, dev):
    return _reduce(v, world, dev, dist.ReduceOp.SUM)
