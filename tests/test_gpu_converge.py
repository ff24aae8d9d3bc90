"""precision='converge' is per image.

PNP_PREC_CONVERGE switches an image to split activations once its OWN c_n (iteration.py:187)
falls below the threshold; while only some images of a batch have switched, each denoiser pass
runs the batch as runs of consecutive images of one precision (capi.hip run_denoiser).  So an
image's bits must not depend on its batch or on the shard it lands in (per-image
outputs on G GPUs bit-identical to G = 1):

* a batch whose images switch at different iterations equals each image solved alone (x, s, c,
  PSNR bit for bit), and each image's switch iteration is the one it has alone;
* a gloo world-2 sharded converge solve (pnppds.shard.test_iter_sharded, both ranks on
  cuda:0) equals the world-1 solve bit for bit.
"""
import os
import socket
import tempfile

import numpy as np
import pytest

from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu

B, C, N, ITERS = 5, 3, 64, 48
ARCH = "DnCNN_nobn_nch_3_nlev_0.01"
# ours-A on blur_1, the metric's parameters (main.py / param_memo.py defaults)
ARGS = (0.99, 0.99, 1.0, 0.95, 1.0, 15, 15, 0.1, 0.01, 0.0, 300, ARCH, ITERS, "A-Proposed", 3, 0.8)


def _batch():
    """Five 64x64 RGB images whose c_n cross 3e-3 at different iterations: smooth and textured
    contents alternate, and the observations carry different noise (the l2-ball radius is the
    solve's sigma = 0.01 for all), so the switched images form non-contiguous runs."""
    from pnppds.operators import load_blur_kernel
    rng = np.random.default_rng(66)
    yy, xx = np.meshgrid(np.linspace(0, 1, N), np.linspace(0, 1, N), indexing="ij")
    xt = np.empty((B, C, N, N), np.float32)
    for b in range(B):
        f = rng.uniform(1, 3 if b % 2 else 9, (C, 2))
        for c in range(C):
            xt[b, c] = 0.5 + 0.3 * np.sin(2 * np.pi * f[c, 0] * xx) * np.cos(2 * np.pi * f[c, 1] * yy)
    np.clip(xt, 0, 1, out=xt)
    h = load_blur_kernel("blur_1")
    noise = (0.004, 0.03, 0.008, 0.02, 0.012)
    xo = np.stack([O.blur(xt[b].astype(np.float64), h) + noise[b] * rng.standard_normal((C, N, N))
                   for b in range(B)]).astype(np.float32)
    return xt, xo


def _solve(xt, xo, ctx=None):
    from pnppds import operators as ops
    from pnppds.iteration import last_precision_switches, test_iter_batch
    phi, adj = ops.get_observation_operators("blur", "blur_1", 0.8)
    x, s, c, p, _, _ = test_iter_batch(xo, xo, xt, phi, adj, *ARGS, precision="converge", ctx=ctx)
    return x, s, c, p, last_precision_switches(len(xt), ctx)


def test_converge_batch_equals_single_images():
    from pnppds.iteration import last_precision_switch
    xt, xo = _batch()
    xb, sb, cb, pb, swb = _solve(xt, xo)
    print("per-image switch iterations:", swb.tolist(), "batch-wide:", last_precision_switch())
    sw_on = swb[swb >= 0]
    assert len(set(sw_on.tolist())) >= 2, ("the batch should switch at different iterations", swb)
    assert (sw_on >= 2).all() and (sw_on < ITERS).all(), swb
    assert last_precision_switch() == (swb.max() if (swb >= 0).all() else -1)
    for b in range(B):
        # the rule, per image: split from two iterations after its own c_n < 3e-3 (r06 run: images
        # switch at different iterations or not at all within 48 iterations)
        if swb[b] >= 0:
            assert swb[b] == np.nonzero(cb[b] < 3e-3)[0][0] + 2, (b, swb[b], cb[b][:12])
        else:
            assert (cb[b][:ITERS - 2] >= 3e-3).all(), (b, cb[b])
        x1, s1, c1, p1, sw1 = _solve(xt[b:b + 1], xo[b:b + 1])
        assert sw1[0] == swb[b], (b, sw1, swb)
        np.testing.assert_array_equal(x1[0], xb[b])
        np.testing.assert_array_equal(s1[0], sb[b])
        np.testing.assert_array_equal(c1[0], cb[b])
        np.testing.assert_array_equal(p1[0], pb[b])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PNPPDS_DEVICE="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pnppds import shard
        from pnppds import operators as ops
        from pnppds._device import get_ctx
        # both ranks share one device here: per-layer launches, so neither runs a persistent
        # grid beside the other's (the multi-GPU bench gives each rank its own device)
        get_ctx().set_body_layers(1)
        xt, xo = _batch()
        phi, adj = ops.get_observation_operators("blur", "blur_1", 0.8)
        res = shard.test_iter_sharded(xo, xo, xt, phi, adj, *ARGS, precision="converge")
        lo, hi = shard.shard_bounds(B, world, rank)
        np.save(os.path.join(out_dir, f"sw{rank}.npy"), get_ctx().get_precision_switches(hi - lo))
        if rank == 0:
            x, s, c, p = res[:4]
            np.savez(os.path.join(out_dir, "gathered.npz"), x=x, s=s, c=c, p=p)
    finally:
        dist.destroy_process_group()


def test_converge_sharded_world2_equals_world1():
    import torch.multiprocessing as mp
    xt, xo = _batch()
    xb, sb, cb, pb, swb = _solve(xt, xo)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = np.load(os.path.join(d, "gathered.npz"))
        np.testing.assert_array_equal(got["x"], xb)
        np.testing.assert_array_equal(got["s"], sb)
        np.testing.assert_array_equal(got["c"], cb)
        np.testing.assert_array_equal(got["p"], pb)
        sw = np.concatenate([np.load(os.path.join(d, f"sw{r}.npy")) for r in range(2)])
        np.testing.assert_array_equal(sw, swb)
