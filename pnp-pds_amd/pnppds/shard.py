"""Multi-GPU: one process per GPU, each running the solver on a contiguous shard of images.

Every image's PnP-PDS state (x, y, s, x_obs, metrics) is independent and every reduction
in test_iter (l2 norm, l1 threshold, c_n, PSNR) is per image, so the batch
is split into contiguous shards with no collective on the data path.  torch.distributed
(RCCL over xGMI on the GPU box, gloo in the CPU tests) is used only
  * to gather the per-shard results on rank 0 after the run (off the timed path), and
  * for the max-over-ranks wall time of the benchmark.

The reference runs its images one after another in one process (main.py:36-69); a batch
split over G ranks gives per-image results bit-identical to G = 1 (tests/test_shard.py,
tests/test_gpu_iter.py::test_batch_equals_single_images), for every precision: under
precision='converge' each image switches on its own c_n (ABI 8), so a gloo world-2 sharded
converge solve equals world 1 bit for bit (tests/test_gpu_converge.py).
"""
from __future__ import annotations

import numpy as np


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) slice of n items owned by `rank`: ceil(n / world) per rank, the
    last ranks possibly short or empty."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    per = -(-n // world)
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def dist_info() -> tuple[int, int]:
    """(rank, world) of the default process group, (0, 1) without one."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def max_over_ranks(value: float, device=None) -> float:
    """Max of a float over the ranks (the benchmark's job time).  `device`: the tensor
    device the backend needs ("cuda:k" for nccl/RCCL, None/"cpu" for gloo)."""
    import torch
    import torch.distributed as dist
    rank, world = dist_info()
    if world == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def test_iter_sharded(x_0, x_obsrv, x_true, *args, runner=None, gather="rank0", **kwargs):
    """Batched test_iter ([B, C, H, W] arrays) over the ranks of the default process group:
    each rank solves images shard_bounds(B, world, rank) on its own GPU.  x_obsrv / x_true
    may be shared (C, H, W) arrays, broadcast to every image as in test_iter_batch.

    gather="rank0" (default): rank 0 returns the whole batch's results, the other ranks
    **None** (one gather to one host, so the results are not replicated on every rank).
    Peak host memory on rank 0: gather_object pickles every shard, so rank 0 holds the
    world's pickled shards plus the concatenated result, about 2-3x the batch's result bytes
    (cfg5, 512 x RGB 1024^2: x and s are 13 GB, so up to ~40 GB on rank 0).  For batches of
    that size use gather="none" and write each shard from its own rank.  gather="none": every rank returns
    (its shard's results, (lo, hi)) and nothing crosses ranks.  `runner` defaults to
    pnppds.iteration.test_iter_batch (the device solver); tests substitute the CPU oracle
    to check the sharding alone."""
    if gather not in ("rank0", "none"):
        raise ValueError(f"gather must be 'rank0' or 'none', not {gather!r}")
    if runner is None:
        from .iteration import test_iter_batch as runner
    rank, world = dist_info()
    x0 = np.asarray(x_0)
    B = x0.shape[0]
    lo, hi = shard_bounds(B, world, rank)
    sl = slice(lo, hi)
    xo = np.broadcast_to(np.asarray(x_obsrv), x0.shape)
    xt = None if x_true is None else np.broadcast_to(np.asarray(x_true), x0.shape)[sl]
    parts = tuple(runner(x0[sl], xo[sl], xt, *args, **kwargs)) if hi > lo else None
    if gather == "none":
        return parts, (lo, hi)
    if world == 1:
        return parts
    import torch.distributed as dist
    allp = [None] * world if rank == 0 else None
    dist.gather_object(parts, allp, dst=0)
    if rank != 0:
        return None
    allp = [p for p in allp if p is not None]
    out = []
    for k in range(len(allp[0])):
        if isinstance(allp[0][k], np.ndarray):
            out.append(np.concatenate([p[k] for p in allp], axis=0))
        else:
            out.append(max(p[k] for p in allp))
    return tuple(out)
