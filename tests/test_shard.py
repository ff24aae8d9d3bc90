"""Multi-process sharding on CPU: gloo, world_size 2 and 3, 127.0.0.1.

The device solver cannot run here, so the shards are solved by the CPU oracle through the
same pnppds.shard.test_iter_sharded entry the GPU ranks use; the property checked is the
one the multi-GPU path relies on: splitting the batch over ranks gives the same per-image
results as one process, and the job time is the max over ranks.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import pnp_oracle as O
from pnppds import shard
from pnppds.weights import random_weights

B, C, H, W, ITERS = 3, 3, 16, 16, 2


def _inputs():
    rng = np.random.default_rng(7)
    xt = rng.uniform(0, 1, (B, C, H, W)).astype(np.float32)
    xo = xt + 0.01 * rng.standard_normal(xt.shape)
    return xt, xo


def oracle_batch_runner(x0, xo, xt, method, iters):
    """test_iter_batch stand-in: the oracle per image, stacked like the device results."""
    den = O.OracleDenoiser(random_weights(C, depth=4, seed=3, scale=0.9))
    phi, adj = O.observation_operators("Id")
    res = [O.test_iter(x0[b].astype(np.float64), xo[b].astype(np.float64), xt[b], phi, adj, 0.99, 0.99, 0.95,
                       0.95, 1.0, 2, 2, 0.1, 0.01, 0.1, 300, den, iters, method, C, 0.8) for b in range(len(x0))]
    return (np.stack([r[0] for r in res]).astype(np.float32), np.stack([r[1] for r in res]),
            np.stack([r[2] for r in res]), np.stack([r[3] for r in res]), max(r[5] for r in res))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, method):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        xt, xo = _inputs()
        res = shard.test_iter_sharded(xo, xo, xt, method, ITERS, runner=oracle_batch_runner)
        local, (lo, hi) = shard.test_iter_sharded(xo, xo, xt, method, ITERS, runner=oracle_batch_runner,
                                                  gather="none")
        tmax = shard.max_over_ranks(float(rank + 1))
        if rank == 0:
            x, s, c, p, t = res
            np.savez(os.path.join(out_dir, "gathered.npz"), x=x, s=s, c=c, p=p)
        else:
            assert res is None                    # results are gathered on rank 0 only
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), lo=lo, hi=hi, tmax=tmax,
                 x=local[0] if local is not None else np.zeros((0, C, H, W), np.float32))
    finally:
        dist.destroy_process_group()


def test_shard_bounds_cover_batch():
    for n in (0, 1, 5, 256, 257):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
    assert shard.shard_bounds(256, 8, 3) == (96, 128)   # 256 images over 8 GPUs: 32 each
    with pytest.raises(ValueError):
        shard.shard_bounds(4, 2, 2)


@pytest.mark.parametrize("world,method", [(2, "B-Proposed"), (3, "A-Proposed")])
def test_sharded_equals_single_process(world, method):
    xt, xo = _inputs()
    ref = oracle_batch_runner(xo, xo, xt, method, ITERS)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, method), nprocs=world, join=True)
        got = np.load(os.path.join(d, "gathered.npz"))
        np.testing.assert_array_equal(got["x"], ref[0])
        np.testing.assert_array_equal(got["s"], ref[1])
        np.testing.assert_array_equal(got["c"], ref[2])
        np.testing.assert_array_equal(got["p"], ref[3])
        for r in range(world):
            loc = np.load(os.path.join(d, f"r{r}.npz"))
            lo, hi = int(loc["lo"]), int(loc["hi"])
            assert (lo, hi) == shard.shard_bounds(B, world, r)
            np.testing.assert_array_equal(loc["x"], ref[0][lo:hi])   # gather="none": the local shard only
            assert float(loc["tmax"]) == float(world)   # max over ranks of rank+1


def test_shared_observation_is_broadcast():
    """A shared (C, H, W) x_obsrv / x_true is broadcast to every image before slicing (as in
    test_iter_batch), not sliced along the channel axis."""
    xt, xo = _inputs()
    seen = []

    def runner(x0, xo_, xt_, *a, **k):
        seen.append((xo_.shape, xt_.shape))
        return (x0,)
    out = shard.test_iter_sharded(xo, xo[0], xt[1], runner=runner)
    assert seen == [((B, C, H, W), (B, C, H, W))]
    np.testing.assert_array_equal(out[0], xo)
