"""The MFMA blur stencils of the fused passes (blur_mf.hip, PNP_TUNE_BLUR_MFMA = 1, the default)
against the packed-fp32 VALU stencils (ops.hip rb_stencil, = 0): whole solver iterations with
fp32 denoiser operands (so a stencil difference is not amplified by fp16 rounding flips), for
ours-A / ours-B / ours-C on the blur operator, the metric's shape and ragged ones (partial
64 x 64 tiles, widths that are not a multiple of 4, grayscale).  The split-fp16 stencil agrees
with the fp32 one to ~1e-6 (tools/blur_mf_emu.py); the reference goldens themselves are checked
on the default path by test_gpu_iter.py / test_gpu_long.py."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _setup(case, B, crop=None, method=None):
    from pnppds import _lib
    from pnppds import operators as ops
    from pnppds.iteration import make_params, resolve_method
    from pnppds.weights import resolve_weights
    g = load_golden(f"iter_{case}.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    ctx = _lib.Context(0)
    m = resolve_method(method or str(g["method"]))
    ctx.set_precision("fp32")
    ctx.set_denoiser(resolve_weights(str(g["arch"]), int(ch)))
    chw = (lambda a: a[None]) if g["x_0"].ndim == 2 else (lambda a: a)
    x0, xo, xt = (chw(g[k]) for k in ("x_0", "x_obs", "x_true"))
    if crop:
        h, w = crop
        x0, xo, xt = (a[..., :h, :w] for a in (x0, xo, xt))
    H, W = x0.shape[-2:]
    phi, _ = ops.get_observation_operators("blur", "blur_1", r)
    phi.configure(ctx, H, W)
    prm = make_params(g1, g2, as_, an, lam, int(m1), int(m2), gadmm, sig, sp, palpha, r, True, True)
    rng = np.random.default_rng(3)
    x0 = np.stack([x0] * B) + 0.01 * rng.standard_normal((B,) + x0.shape)
    xo = np.stack([xo] * B).astype(np.float32)
    xt = np.stack([xt] * B).astype(np.float32)
    return ctx, m, prm, np.clip(x0, 0, 1).astype(np.float32), xo, xt


@pytest.mark.parametrize("case,B,crop,method", [
    ("A_blur", 2, None, None),
    ("B_blur", 2, None, None),
    ("A_blur", 1, (100, 70), None),         # partial tiles, W % 4 == 2: scalar epilogue columns
    ("A_blur", 2, (37, 53), "C-Proposed"),  # ours-C (GKL prox in K2) on the blur operator
    ("B_blur", 1, (64, 66), None),
])
def test_mfma_stencil_matches_valu(case, B, crop, method):
    ctx, m, prm, x0, xo, xt = _setup(case, B, crop, method)
    iters = 4
    ctx.set_blur_mfma(0)
    ref = ctx.run(m, prm, x0, xo, xt, iters)
    ctx.set_blur_mfma(1)
    got = ctx.run(m, prm, x0, xo, xt, iters)
    names = ("x", "s", "c", "psnr", "ssim")
    for name, a, b in zip(names, ref[:5], got[:5]):
        a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
        assert np.isfinite(b).all(), name
        if name == "psnr":
            np.testing.assert_allclose(b, a, atol=1e-4, err_msg=name)
        elif name == "c":
            np.testing.assert_allclose(b, a, rtol=1e-3, atol=1e-9, err_msg=name)
        else:
            np.testing.assert_allclose(b, a, atol=2e-5, err_msg=name)


def test_gray_mfma_stencil_matches_valu():
    """Grayscale (C = 1) at the reference's cfg1 size, ours-A."""
    from pnppds import _lib
    from pnppds import operators as ops
    from pnppds.iteration import make_params, resolve_method
    from pnppds.weights import resolve_weights
    rng = np.random.default_rng(5)
    B, H, W = 2, 256, 256
    xt = rng.random((B, 1, H, W)).astype(np.float32)
    xo = np.clip(xt + 0.01 * rng.standard_normal(xt.shape), 0, 1).astype(np.float32)
    ctx = _lib.Context(0)
    ctx.set_precision("fp32")
    ctx.set_denoiser(resolve_weights("DnCNN_nobn_nch_1_nlev_0.01", 1))
    phi, _ = ops.get_observation_operators("blur", "blur_1", 1.0)
    phi.configure(ctx, H, W)
    prm = make_params(0.5, 0.99 / 0.5, 1.0, 1.0, 1.0, 0, 0, 0.0, 0.01, 0.0, 1.0, 1.0, True, True)
    m = resolve_method("A-Proposed")
    ctx.set_blur_mfma(0)
    ref = ctx.run(m, prm, xo.copy(), xo, xt, 3)
    ctx.set_blur_mfma(1)
    got = ctx.run(m, prm, xo.copy(), xo, xt, 3)
    np.testing.assert_allclose(got[0], ref[0], atol=2e-5)
    np.testing.assert_allclose(got[3], ref[3], atol=1e-4)


def test_blur_mfma_rejects_bad_values(gpu_ctx):
    from pnppds._lib import PnpError
    with pytest.raises(PnpError):
        gpu_ctx.set_blur_mfma(2)
