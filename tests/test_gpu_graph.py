"""hipGraph replay of the iteration launches (PNP_TUNE_GRAPH) gives the same bits as direct
launches: x, s and every recorded metric (c_n, PSNR, SSIM), for ours-A/B/C, odd and even
iteration counts, iterations split over several pnp_solver_iterate calls, metrics capacity
shorter than the run, and a rebuild after a setter changes the state."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu


def _setup(case, B):
    from pnppds import _lib
    from pnppds import operators as ops
    from pnppds.iteration import make_params, resolve_method
    from pnppds.weights import resolve_weights
    g = load_golden(f"iter_{case}.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    ctx = _lib.Context(0)
    m = resolve_method(str(g["method"]))
    ctx.set_precision("auto")
    ctx.set_denoiser(resolve_weights(str(g["arch"]), int(ch)))
    phi, _ = ops.get_observation_operators(str(g["deg_op"]), "blur_1", r)
    phi.configure(ctx, g["x_0"].shape[-2], g["x_0"].shape[-1])
    prm = make_params(g1, g2, as_, an, lam, int(m1), int(m2), gadmm, sig, sp, palpha, r, True, True)
    rng = np.random.default_rng(1)
    chw = (lambda a: a[None]) if g["x_0"].ndim == 2 else (lambda a: a)   # gray: the reference's (H, W)
    x0 = np.stack([chw(g["x_0"])] * B) + 0.01 * rng.standard_normal((B,) + chw(g["x_0"]).shape)
    xo = np.stack([chw(g["x_obs"])] * B).astype(np.float32)
    xt = np.stack([chw(g["x_true"])] * B).astype(np.float32)
    return ctx, m, prm, x0.astype(np.float32), xo, xt


@pytest.mark.parametrize("case,B,iters", [("A_blur", 1, 7), ("A_rs", 2, 6), ("B_blur", 1, 5), ("C_rs", 2, 5)])
def test_graph_equals_direct_launches(case, B, iters):
    ctx, m, prm, x0, xo, xt = _setup(case, B)
    ctx.set_graph(0)
    ref = ctx.run(m, prm, x0, xo, xt, iters)
    ctx.set_graph(1)
    got = ctx.run(m, prm, x0, xo, xt, iters)
    for a, b in zip(ref[:5], got[:5]):
        np.testing.assert_array_equal(a, b)
    assert np.isfinite(got[3]).all() and np.isfinite(got[4]).all()   # every PSNR / SSIM row written


def test_graph_split_iterate_and_short_capacity():
    """Iterations in several calls (odd counts: plain steps realign the x ping-pong), a metrics
    capacity shorter than the run (the counter runs past it), and a setter between calls (the
    graph is recaptured)."""
    ctx, m, prm, x0, xo, xt = _setup("A_blur", 1)
    B, Cc, H, W = x0.shape
    out = {}
    for mode in (0, 1):
        ctx.set_graph(mode)
        ctx.solver_setup(m, prm, B, Cc, H, W, 6)
        ctx.solver_load(x0, xo, xt)
        ctx.solver_iterate(3)
        ctx.solver_iterate(4)
        ctx.set_denoise_chunk(1)                      # bumps the state generation
        ctx.solver_iterate(2)
        out[mode] = ctx.solver_fetch()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)
    assert np.isfinite(out[1][2]).all()               # c rows 0..5 written, rows past 6 dropped


def test_graph_mode_rejects_bad_values(gpu_ctx):
    from pnppds._lib import PnpError
    with pytest.raises(PnpError):
        gpu_ctx.set_graph(2)


def test_denoise_passes_same_bits():
    """The denoiser's images-per-pass split (auto: the HBM budget, evenly split; forced: 3 -> passes
    of 3, 3, 1; 1) leaves every image's result unchanged: x, s and all metric rows."""
    ctx, m, prm, x0, xo, xt = _setup("A_blur", 7)
    ref = ctx.run(m, prm, x0, xo, xt, 4)
    for chunk in (3, 1):
        ctx.set_denoise_chunk(chunk)
        got = ctx.run(m, prm, x0, xo, xt, 4)
        for a, b in zip(ref[:5], got[:5]):
            np.testing.assert_array_equal(a, b)


def test_op_denoise_between_graph_replays_fp32():
    """pnp_op_denoise at fp32 on another image size between two graph-replayed
    solver_iterate calls (ours-C, fp32 operands) must not disturb the solver's fp32 activation
    borders: the single op has its own scratch pair, so the replay gives the direct bits."""
    import torch
    ctx, m, prm, x0, xo, xt = _setup("C_rs", 1)
    B, Cc, H, W = x0.shape
    xs = torch.rand(2, Cc, H + 24, W + 8, device="cuda")
    ys = torch.empty_like(xs)
    out = {}
    for mode in (0, 1):
        ctx.set_graph(mode)
        ctx.solver_setup(m, prm, B, Cc, H, W, 8)
        ctx.solver_load(x0, xo, xt)
        ctx.solver_iterate(4)
        ctx.op_denoise(xs.data_ptr(), ys.data_ptr(), 2, Cc, H + 24, W + 8)
        ctx.solver_iterate(4)
        out[mode] = ctx.solver_fetch()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


def test_op_l1_ball_side_stream_fresh_context():
    """on a fresh context pnp_op_proj_l1_ball on a caller stream zeroes its own
    histogram scratch on that stream (not on the context's stream), so the first call is right."""
    import torch
    from oracle import pnp_oracle as O
    from pnppds import _lib
    rng = np.random.default_rng(5)
    v = rng.standard_normal((3, 3 * 64 * 64)).astype(np.float32) * 0.1
    want = np.stack([O.proj_l1_ball(v[b].astype(np.float64), 0.95, 0.1, 0.8) for b in range(3)])
    s = torch.cuda.Stream()
    for _ in range(3):
        ctx = _lib.Context(0)
        dv = torch.from_numpy(v).cuda()
        do = torch.empty_like(dv)
        torch.cuda.synchronize()
        ctx.op_proj_l1_ball(dv.data_ptr(), do.data_ptr(), 3, v.shape[1], 0.95, 0.1, 0.8, stream=s.cuda_stream)
        s.synchronize()
        np.testing.assert_allclose(do.cpu().numpy(), want, atol=2e-6)
        ctx.close()


@pytest.mark.parametrize("case", ["A_blur", "A_gray", "B_blur"])
def test_single_image_stack_equals_per_layer(case):
    """B = 1 (the reference's call pattern): the auto choice for a single image, all body
    layers in one persistent launch (conv_stack16x2, two layers per hand-off; conv_stack16, one),
    against one launch per layer, through the
    solver: x, s and every metric, same bits; and with graph replay on (captured steps fall
    back to per-layer launches, the plain ones keep the persistent launch)."""
    ctx, m, prm, x0, xo, xt = _setup(case, 1)
    ctx.set_precision("fp16")
    ctx.set_body_layers(1)
    ref = ctx.run(m, prm, x0, xo, xt, 7)
    for mode, graph in ((0, 0), (3, 0), (4, 0), (0, 1)):
        ctx.set_body_layers(mode)
        ctx.set_graph(graph)
        got = ctx.run(m, prm, x0, xo, xt, 7)
        for a, b in zip(ref[:5], got[:5]):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("case", ["A_blur", "B_blur"])
def test_dual_state_between_iterates(case):
    """ours-A / ours-B on the blur operator run K3 inside the next K1's halo fill, so between
    iterations the dual buffer holds v and 1 - f.  Reading the state (pnp_solver_state) applies
    the pending l2-ball step in place; the run then continues from the finalized dual, with
    graph replay on and off (the captured pending-dual K1 is recaptured), to the same bits as an
    uninterrupted run: the finalized y is the y the fused fill computes."""
    import torch
    ctx, m, prm, x0, xo, xt = _setup(case, 2)
    B, Cc, H, W = x0.shape
    ref = ctx.run(m, prm, x0, xo, xt, 9)
    for graph in (0, 1):
        ctx.set_graph(graph)
        ctx.solver_setup(m, prm, B, Cc, H, W, 9)
        ctx.solver_load(x0, xo, xt)
        ctx.solver_iterate(4)
        _, dy, _ = ctx.solver_state()
        ctx.synchronize()
        y4 = torch.empty(B * Cc * H * W, dtype=torch.float32, device="cuda")
        ctx.device_copy(y4.data_ptr(), dy, y4.numel() * 4)
        ctx.synchronize()
        assert torch.isfinite(y4).all()
        ctx.solver_iterate(5)
        got = ctx.solver_fetch()
        for a, b in zip(ref[:5], got[:5]):
            np.testing.assert_array_equal(a, b)


def _dev_array(ctx, ptr, shape):
    import torch
    n = int(np.prod(shape))
    t = torch.empty(n, dtype=torch.float32, device="cuda")
    ctx.device_copy(t.data_ptr(), ptr, n * 4)
    ctx.synchronize()
    return t.cpu().numpy().reshape(shape).astype(np.float64)


@pytest.mark.parametrize("case", ["A_blur", "B_blur"])
def test_dual_state_values_after_even_and_odd_counts(case):
    """The dual pnp_solver_state returns is the reference's y (iteration.py:51-52 / 57-58),
    recomputed on the host in fp64 from the device's own iterates: after 4 iterations (dual in
    buffer y) and after 5 (dual in y2).  y_k = v - g2 P_l2(v / g2), v = y_{k-1} + g2 (Phi(2x_k -
    x_{k-1}) [+ 2 s_k - s_{k-1}])."""
    from pnppds.operators import load_blur_kernel
    ctx, m, prm, x0, xo, xt = _setup(case, 2)
    B, Cc, H, W = x0.shape
    h = load_blur_kernel("blur_1")
    ctx.solver_setup(m, prm, B, Cc, H, W, 9)
    ctx.solver_load(x0, xo, xt)
    ctx.solver_iterate(3)

    def state():
        dx, dy, ds = ctx.solver_state()
        return _dev_array(ctx, dx, x0.shape), _dev_array(ctx, dy, x0.shape), _dev_array(ctx, ds, x0.shape)

    xp, yp, sp_ = state()
    for _ in (4, 5):
        ctx.solver_iterate(1)
        xn, yn, sn = state()
        n = Cc * H * W
        r = prm.r if case.startswith("B") else 1.0
        eps = np.sqrt(n * (1 - prm.sp_nl)) * r * prm.alpha_n * prm.gaussian_nl
        for b in range(B):
            v = yp[b] + prm.gamma2 * (O.blur(2 * xn[b] - xp[b], h) + (2 * sn[b] - sp_[b] if case.startswith("B") else 0))
            want = v - prm.gamma2 * O.proj_l2_ball(v / prm.gamma2, prm.alpha_n, prm.gaussian_nl, prm.sp_nl,
                                                   xo[b].astype(np.float64), r)
            assert np.isfinite(eps)
            np.testing.assert_allclose(yn[b], want, atol=2e-5 * max(1.0, np.abs(want).max()))
        xp, yp, sp_ = xn, yn, sn


def test_destroy_releases_device_memory():
    """pnp_destroy frees every buffer of the context (the fused-dual y2 / omf were
    left out of the release list): three create / solve / destroy rounds of ours-A blur at
    B = 64 RGB 256^2 (50 MB per state array) leave the device's free memory where it was."""
    import torch
    from pnppds import _lib
    from pnppds.iteration import make_params, resolve_method
    from pnppds.operators import load_blur_kernel
    from pnppds.weights import resolve_weights
    B, Cc, H, W = 64, 3, 256, 256
    x0 = np.full((B, Cc, H, W), 0.5, np.float32)
    prm = make_params(0.99, 0.99, 1.0, 0.95, 1.0, 15, 15, 0.1, 0.01, 0.0, 300, 0.8, True, True)
    torch.cuda.synchronize()
    free0 = None
    for k in range(3):
        ctx = _lib.Context(0)
        ctx.set_denoiser(resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3))
        ctx.set_operator(_lib.OP_BLUR, h=load_blur_kernel("blur_1"))
        ctx.solver_setup(resolve_method("ours-A"), prm, B, Cc, H, W, 2)
        ctx.solver_load(x0, x0, x0)
        ctx.solver_iterate(2)
        ctx.solver_fetch()
        ctx.close()
        torch.cuda.synchronize()
        free = torch.cuda.mem_get_info()[0]
        if free0 is None:
            free0 = free                     # after the first round: runtime / code objects loaded
        assert free0 - free < 32 << 20, (k, (free0 - free) >> 20)
