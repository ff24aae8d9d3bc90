"""GPU SSIM (pnp_op_ssim and the solver's per-iteration record) vs the oracle's restatement of
utils/utils_eval.py:9-12.  PARITY UNPINNED (skimage absent; see tests/test_ssim_oracle.py).
Tolerance 2e-5: float32 map as skimage computes it, the device sums in float64 in a different
order than numpy's pairwise float64 mean."""
import numpy as np
import pytest

from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu
TOL = 2e-5


def _pairs(B, shape, seed, noise=0.08):
    rng = np.random.default_rng(seed)
    a = rng.uniform(0, 1, (B,) + shape).astype(np.float32)
    # smooth structure so the SSIM is far from 0 and 1
    a = (0.5 * a + 0.5 * np.cumsum(a, axis=-1) / np.arange(1, shape[-1] + 1)).astype(np.float32)
    b = (a + noise * rng.standard_normal(a.shape)).astype(np.float32)
    b[0] *= 0.7                                   # different data_range per image
    return a, b


@pytest.mark.parametrize("shape", [(3, 64, 64), (3, 48, 80), (3, 37, 29), (3, 256, 256), (1, 64, 64),
                                   (1, 37, 53), (1, 256, 256)])
def test_op_ssim_matches_oracle(gpu_ctx, shape):
    import torch
    B = 3
    a, b = _pairs(B, shape, 11)
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    got = gpu_ctx.op_ssim(da.data_ptr(), db.data_ptr(), B, *shape)
    for i in range(B):
        want = O.ssim(a[i] if shape[0] > 1 else a[i, 0], b[i] if shape[0] > 1 else b[i, 0])
        assert abs(got[i] - want) < TOL, (shape, i, got[i], want)


def test_op_ssim_identical_is_one(gpu_ctx):
    import torch
    a, _ = _pairs(2, (3, 40, 40), 3)
    da = torch.from_numpy(a).cuda()
    got = gpu_ctx.op_ssim(da.data_ptr(), da.data_ptr(), 2, 3, 40, 40)
    np.testing.assert_allclose(got, 1.0, atol=1e-6)


@pytest.mark.parametrize("case", ["A_blur", "A_gray", "B_blur", "C_rs", "ADMM_B2"])
def test_solver_records_ssim(case):
    """iteration.py:189: ssim_data[i] = eval_ssim(x_true, x_n) every iteration; the last entry
    is checked against the oracle on the returned x."""
    from conftest import load_golden
    from test_gpu_iter import run_case
    g = load_golden(f"iter_{case}.npz")
    x, s, c, psnr, ssim, t = run_case(g)
    assert ssim.shape == psnr.shape and np.all(np.isfinite(ssim))
    assert abs(ssim[-1] - O.ssim(g["x_true"], x)) < TOL
    # and within the x tolerance of the reference's own final iterate
    assert abs(ssim[-1] - O.ssim(g["x_true"], g["x_out"])) < 5e-3


@pytest.mark.parametrize("method,op,B,C,H,W", [("A-Proposed", "blur", 2, 3, 50, 70), ("A-Proposed", "blur", 3, 3, 57, 33),
                                               ("A-Proposed", "blur", 1, 1, 37, 45), ("A-Proposed", "Id", 2, 3, 41, 29),
                                               ("B-Proposed", "blur", 2, 3, 61, 37),
                                               ("C-Proposed", "random_sampling", 2, 3, 45, 58)])
def test_psnr_same_with_and_without_ssim(method, op, B, C, H, W):
    """With SSIM recorded the PSNR's squared-error sum moves from K2's fp64 partials into the SSIM
    pass (fp32 sums over 8 pixels per RGB thread or a whole gray row, then fp64): the recorded
    PSNR must not depend on record_ssim.  Ragged H / W, partial 56 x 32 SSIM tiles,
    gray and RGB, the fused (blur A / B) and plain K2 paths; the iterates themselves are the same
    bits either way, so the two PSNR tracks differ only by summation order."""
    from pnppds import operators as ops
    from pnppds.iteration import test_iter_batch
    from pnppds.operators import load_blur_kernel
    rng = np.random.default_rng(H * W + C)
    xt = rng.uniform(0.1, 0.9, (B, C, H, W)).astype(np.float32)
    xt = (0.5 * xt + 0.5 * np.cumsum(xt, axis=-1) / np.arange(1, W + 1)).astype(np.float32)
    phi, adj = ops.get_observation_operators(op, "blur_1", 0.8)
    pois = method == "C-Proposed"
    phi_o = O.observation_operators(op, load_blur_kernel("blur_1"), 0.8)[0]
    xo = np.stack([np.asarray(phi_o(xt[b].astype(np.float64) if C > 1 else xt[b, 0].astype(np.float64))).reshape(C, H, W)
                   for b in range(B)])
    if pois:
        xo = np.round(xo * 300) / 300.0
    else:
        xo = xo + 0.01 * rng.standard_normal(xo.shape)
    xo = xo.astype(np.float32)
    g1, g2 = (0.00035, 1 / 0.00035) if pois else (0.99, 0.99)
    args = (g1, g2, 1.0, 0.95, 1.0, 15, 15, 0.1, 0.0 if pois else 0.01, 0.1 if method == "B-Proposed" else 0.0, 300,
            f"DnCNN_nobn_nch_{C}_nlev_0.01", 6, method, C, 0.8)
    x1, _, _, p1, s1, _ = test_iter_batch(xo, xo, xt, phi, adj, *args, record_ssim=True)
    x0, _, _, p0, _, _ = test_iter_batch(xo, xo, xt, phi, adj, *args, record_ssim=False)
    np.testing.assert_array_equal(x1, x0)
    assert np.isfinite(s1).all()
    d = np.abs(p1 - p0).max()
    print(f"{method} {op} {B}x{C}x{H}x{W}: max |PSNR(ssim on) - PSNR(ssim off)| = {d:.2e} dB")
    assert d < 1e-7, d          # r06: 1.1e-8 .. 2.7e-8 dB over these six cases
