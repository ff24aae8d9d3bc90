"""GPU parity of the operator / prox kernels (through the C-ABI) vs golden vectors and the oracle."""
import numpy as np
import pytest

from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(torch, t, ctx):
    torch.cuda.synchronize()
    ctx.synchronize()
    return t.cpu().numpy()


@pytest.mark.parametrize("tag", ["rgb64", "gray64", "gray256", "rgb48x80"])
def test_blur_phi_adj(gpu_ctx, torch_cuda, golden_ops, tag):
    from pnppds import _lib
    g = golden_ops
    x = g[f"x_{tag}"]
    x4 = x.reshape((1, 1) + x.shape) if x.ndim == 2 else x[None]
    _, C, H, W = x4.shape
    gpu_ctx.set_operator(_lib.OP_BLUR, h=g["h"])
    dx = dev(torch_cuda, x4)
    for adj, key in ((False, "phi"), (True, "adj")):
        dy = torch_cuda.empty_like(dx)
        gpu_ctx.op_phi(dx.data_ptr(), dy.data_ptr(), 1, C, H, W, adj=adj)
        out = host(torch_cuda, dy, gpu_ctx).reshape(x.shape)
        np.testing.assert_allclose(out, g[f"{key}_blur_{tag}"], atol=2e-6, rtol=0)


@pytest.mark.parametrize("tag,r,key", [("rgb64", 0.8, "rs8"), ("rgb64", 0.5, "rs5"), ("gray64", 0.8, "rs8")])
def test_random_sampling(gpu_ctx, torch_cuda, golden_ops, tag, r, key):
    from pnppds import _lib
    from pnppds.operators import sampling_keep_mask
    g = golden_ops
    x = g[f"x_{tag}"]
    x4 = x.reshape((1, 1) + x.shape) if x.ndim == 2 else x[None]
    _, C, H, W = x4.shape
    gpu_ctx.set_operator(_lib.OP_RANDOM_SAMPLING, mask=sampling_keep_mask(H, W, r))
    dx = dev(torch_cuda, x4)
    dy = torch_cuda.empty_like(dx)
    gpu_ctx.op_phi(dx.data_ptr(), dy.data_ptr(), 1, C, H, W)
    out = host(torch_cuda, dy, gpu_ctx).reshape(x.shape)
    np.testing.assert_array_equal(out, g[f"phi_{key}_{tag}"].astype(np.float32))


@pytest.mark.parametrize("shape,kernel", [((2, 3, 37, 53), "blur_1"), ((1, 1, 6, 7), "blur_1"),
                                          ((1, 3, 8, 9), "blur_1"), ((2, 1, 40, 24), "dense5")])
def test_blur_phi_adj_shapes(gpu_ctx, torch_cuda, shape, kernel):
    """pnp_op_phi / pnp_op_adj_phi (the register-blocked k0 kernel, and the modulo-wrapped
    stencil for images smaller than the taps' radius) against the FFT oracle: odd widths,
    images smaller than the 19x19 kernel (np.pad 'wrap' repeats them), a dense 5x5 kernel."""
    from pnppds import _lib
    from pnppds.operators import load_blur_kernel
    rng = np.random.default_rng(7)
    h = load_blur_kernel("blur_1") if kernel == "blur_1" else rng.random((5, 5)) / 12.5
    x = rng.random(shape).astype(np.float32)
    gpu_ctx.set_operator(_lib.OP_BLUR, h=h)
    dx = dev(torch_cuda, x)
    B, C, H, W = shape
    for adj, ref in ((False, O.blur), (True, O.adj_blur)):
        dy = torch_cuda.empty_like(dx)
        gpu_ctx.op_phi(dx.data_ptr(), dy.data_ptr(), B, C, H, W, adj=adj)
        out = host(torch_cuda, dy, gpu_ctx)
        np.testing.assert_allclose(out, ref(x, h), atol=3e-6, rtol=0)


def test_blur_adjointness_full_size(gpu_ctx, torch_cuda):
    """<Φx, z> == <x, Φᵀz> at the metric's image size (size-independent property)."""
    from pnppds import _lib
    from pnppds.operators import load_blur_kernel
    rng = np.random.default_rng(1)
    B, C, H, W = 4, 3, 256, 256
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    z = rng.standard_normal((B, C, H, W)).astype(np.float32)
    gpu_ctx.set_operator(_lib.OP_BLUR, h=load_blur_kernel("blur_1"))
    dx, dz = dev(torch_cuda, x), dev(torch_cuda, z)
    px, pz = torch_cuda.empty_like(dx), torch_cuda.empty_like(dz)
    gpu_ctx.op_phi(dx.data_ptr(), px.data_ptr(), B, C, H, W)
    gpu_ctx.op_phi(dz.data_ptr(), pz.data_ptr(), B, C, H, W, adj=True)
    a = float((host(torch_cuda, px, gpu_ctx).astype(np.float64) * z).sum())
    b = float((x.astype(np.float64) * host(torch_cuda, pz, gpu_ctx)).sum())
    assert abs(a - b) <= 1e-5 * np.sqrt(x.size), (a, b)
    # and against the FFT oracle on one image
    np.testing.assert_allclose(host(torch_cuda, px, gpu_ctx)[1], O.blur(x[1], load_blur_kernel("blur_1")),
                               atol=3e-6)


def test_l2_ball(gpu_ctx, torch_cuda, golden_ops):
    g = golden_ops
    v, x0 = g["prox_v"], g["prox_x0"]
    n = v.size
    for nl, a in ((0.01, 0.95), (10.0, 1.0)):
        dx, d0 = dev(torch_cuda, (x0 + v).reshape(1, -1)), dev(torch_cuda, x0.reshape(1, -1))
        out = torch_cuda.empty_like(dx)
        gpu_ctx.op_proj_l2_ball(dx.data_ptr(), d0.data_ptr(), out.data_ptr(), 1, n, a, nl, 0.1, 0.8)
        np.testing.assert_allclose(host(torch_cuda, out, gpu_ctx).reshape(v.shape), g[f"l2_{nl}_{a}"], atol=2e-7)


@pytest.mark.parametrize("sp", [0.0, 0.01, 0.1, 0.5])
def test_l1_ball_golden(gpu_ctx, torch_cuda, golden_ops, sp):
    g = golden_ops
    v = g["prox_v"]
    dx = dev(torch_cuda, v.reshape(1, -1))
    out = torch_cuda.empty_like(dx)
    gpu_ctx.op_proj_l1_ball(dx.data_ptr(), out.data_ptr(), 1, v.size, 0.95, sp, 0.8)
    np.testing.assert_allclose(host(torch_cuda, out, gpu_ctx).reshape(v.shape), g[f"l1_{sp}"], atol=1e-6)


def test_l1_ball_inside(gpu_ctx, torch_cuda, golden_ops):
    g = golden_ops
    v = (g["prox_v"] * 1e-4)
    dx = dev(torch_cuda, v.reshape(1, -1))
    out = torch_cuda.empty_like(dx)
    gpu_ctx.op_proj_l1_ball(dx.data_ptr(), out.data_ptr(), 1, v.size, 0.95, 0.1, 1.0)
    np.testing.assert_allclose(host(torch_cuda, out, gpu_ctx).reshape(v.shape), g["l1_inside"], atol=1e-10)


@pytest.mark.parametrize("shape,dist", [((3, 256, 256), "normal"), ((3, 256, 256), "sparse"),
                                         ((3, 1024, 1024), "normal"), ((1, 37, 53), "ties")])
def test_l1_ball_vs_oracle_batched(gpu_ctx, torch_cuda, shape, dist):
    """Batched projection at full image sizes, heavy-tailed / tied data; checks ||s||_1 == eta too."""
    rng = np.random.default_rng(7)
    B = 3
    if dist == "normal":
        v = rng.standard_normal((B,) + shape) * 0.05
    elif dist == "sparse":
        v = rng.standard_normal((B,) + shape) * 1e-3
        m = rng.random((B,) + shape) < 0.05
        v[m] = rng.choice([-1.0, 1.0], m.sum()) * rng.uniform(0.2, 1.0, m.sum())
    else:
        v = rng.choice([-0.5, -0.25, 0.0, 0.25, 0.5], size=(B,) + shape)
    v = v.astype(np.float32)
    n = int(np.prod(shape))
    dx = dev(torch_cuda, v.reshape(B, -1))
    out = torch_cuda.empty_like(dx)
    gpu_ctx.op_proj_l1_ball(dx.data_ptr(), out.data_ptr(), B, n, 0.95, 0.1, 0.8)
    got = host(torch_cuda, out, gpu_ctx).reshape(v.shape)
    eta = 0.95 * n * 0.1 * 0.8 * 0.5
    for b in range(B):
        ref = O.proj_l1_ball(v[b].astype(np.float64), 0.95, 0.1, 0.8)
        np.testing.assert_allclose(got[b], ref, atol=2e-6 * max(1.0, np.abs(v).max()))
        if np.abs(v[b]).sum() > eta:
            assert abs(np.abs(got[b].astype(np.float64)).sum() - eta) <= 1e-4 * eta


def test_l1_ball_deterministic(gpu_ctx, torch_cuda):
    """The threshold search is order-independent (exact integer bin sums): repeated batched
    launches and one-image launches give the same bits (the property sharding relies on)."""
    rng = np.random.default_rng(21)
    B, n = 8, 3 * 128 * 128
    v = (rng.standard_normal((B, n)) * 0.05).astype(np.float32)
    dx = dev(torch_cuda, v)
    outs = []
    for _ in range(4):
        out = torch_cuda.empty_like(dx)
        gpu_ctx.op_proj_l1_ball(dx.data_ptr(), out.data_ptr(), B, n, 0.95, 0.1, 0.8)
        outs.append(host(torch_cuda, out, gpu_ctx))
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])
    for b in (0, B - 1):
        one = torch_cuda.empty_like(dx[b:b + 1])
        gpu_ctx.op_proj_l1_ball(dx[b:b + 1].data_ptr(), one.data_ptr(), 1, n, 0.95, 0.1, 0.8)
        np.testing.assert_array_equal(host(torch_cuda, one, gpu_ctx)[0], outs[0][b])


@pytest.mark.parametrize("kind", ["exponents", "ties"])
def test_l1_ball_exact_bins_edge_cases(gpu_ctx, torch_cuda, kind):
    """The exact-bin radix select on data that exercises its edge paths: magnitudes spread
    over 140 binary exponents including subnormals (the e == 0 significand branch and bins
    at exponent boundaries), and many exactly repeated values at / near the threshold.
    Bits batch vs one-image launch; values against the oracle's sort-based projection."""
    rng = np.random.default_rng(5 if kind == "exponents" else 6)
    B, n = 4, 3 * 96 * 96
    if kind == "exponents":
        mag = np.ldexp(rng.uniform(1, 2, (B, n)), rng.integers(-140, 3, (B, n)))
        mag[:, :64] = np.ldexp(rng.integers(1, 1 << 20, (B, 64)).astype(np.float64), -149)   # subnormals
        mag[:, 64:96] = np.ldexp(1.0, rng.integers(-126, 2, (B, 32)))                         # exact powers of 2
    else:
        mag = rng.uniform(0, 0.3, (B, n))
        mag[:, : n // 3] = 0.125                                     # a third of the entries tie
        mag[:, n // 3: n // 3 + 500] = np.nextafter(np.float32(0.125), np.float32(1))
        mag[:, n // 3 + 500: n // 3 + 1000] = np.nextafter(np.float32(0.125), np.float32(0))
    v = (mag * rng.choice([-1.0, 1.0], (B, n))).astype(np.float32)
    assert (np.abs(v[:, :64]) < np.finfo(np.float32).tiny).all() or kind == "ties"
    dx = dev(torch_cuda, v)
    out = torch_cuda.empty_like(dx)
    gpu_ctx.op_proj_l1_ball(dx.data_ptr(), out.data_ptr(), B, n, 0.95, 0.1, 0.8)
    got = host(torch_cuda, out, gpu_ctx)
    eta = 0.95 * n * 0.1 * 0.8 * 0.5
    for b in range(B):
        ref = O.proj_l1_ball(v[b].astype(np.float64), 0.95, 0.1, 0.8)
        np.testing.assert_allclose(got[b], ref, atol=2e-6 * max(1.0, float(np.abs(v[b]).max())))
        if np.abs(v[b].astype(np.float64)).sum() > eta:
            assert abs(np.abs(got[b].astype(np.float64)).sum() - eta) <= 1e-4 * eta
        one = torch_cuda.empty_like(dx[b:b + 1])
        gpu_ctx.op_proj_l1_ball(dx[b:b + 1].data_ptr(), one.data_ptr(), 1, n, 0.95, 0.1, 0.8)
        np.testing.assert_array_equal(host(torch_cuda, one, gpu_ctx)[0], got[b])


def test_l1_ball_rejects_oversized_images(gpu_ctx):
    """Above 2^29 elements per image the bin sums would no longer be exact: rejected."""
    from pnppds._lib import PnpError
    with pytest.raises(PnpError):
        gpu_ctx.op_proj_l1_ball(16, 16, 1, 1 << 29, 0.95, 0.1, 0.8)


def test_prox_gkl(gpu_ctx, torch_cuda, golden_ops):
    g = golden_ops
    v, x0 = g["prox_v"] * 10, np.round(g["prox_x0"] * 300)
    dx, d0 = dev(torch_cuda, v), dev(torch_cuda, x0)
    out = torch_cuda.empty_like(dx)
    gpu_ctx.op_prox_gkl(dx.data_ptr(), d0.data_ptr(), out.data_ptr(), v.size, 0.5, 300.0)
    np.testing.assert_allclose(host(torch_cuda, out, gpu_ctx), g["gkl"], rtol=1e-6, atol=1e-5)


def test_psnr(gpu_ctx, torch_cuda, golden_ops):
    g = golden_ops
    x0, v = g["prox_x0"], g["prox_v"]
    a, b = dev(torch_cuda, x0[None]), dev(torch_cuda, (x0 + v)[None])
    p = gpu_ctx.op_psnr(a.data_ptr(), b.data_ptr(), 1, x0.size)
    assert abs(p[0] - g["psnr"][0]) < 1e-4
