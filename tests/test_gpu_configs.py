"""The SURVEY.md §8(d) configurations at their full per-GPU sizes (BASELINE.json configs 3-5).

The oracle finishes one image of these sizes in seconds, so each test checks image 0 of the
device batch against the oracle on identical inputs (x_obs from the device observation
pipeline, bit-identical to the reference's numpy stream), and the whole batch through
size-independent properties:
* the last image of the batch gives the same bits alone (what sharding over GPUs relies on);
* the iteration's own invariants: s inside the l1 ball of radius eta (B), finite duals (C).
The x / s bounds are 2-3x what the product measured against the oracle (round 5); the PSNR
bound is north_star's 0.01 dB.
Per-GPU shard sizes: cfg4 = 256 images / 8 GPUs, cfg5 = 512 / 8.
"""
import numpy as np
import pytest

from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu

ARCH = "DnCNN_nobn_nch_3_nlev_0.01"


def _synthetic(B, H, W, seed):
    from bench import synthetic_batch
    return synthetic_batch(B, 3, H, W, seed)


def _observe(xt, deg_op, r, sig, sp, poisson, alpha):
    from pnppds import operators as ops
    from pnppds.noise import make_observation_batch
    phi, adj = ops.get_observation_operators(deg_op, "blur_1", r)
    xobs64, x0 = make_observation_batch(xt, phi, sig, sp, poisson, alpha, float64=True)
    return phi, adj, xobs64, x0


def _oracle_image0(xt, xobs64, deg_op, r, prm, iters, method, poisson=False):
    from pnppds.operators import load_blur_kernel
    from pnppds.weights import resolve_weights
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha = prm
    phi, adj = O.observation_operators(deg_op, load_blur_kernel("blur_1"), r)
    xo = xobs64[0]
    x0_ref = xo / palpha if poisson else np.copy(xo)          # main.py:60-64 (float64)
    return O.test_iter(x0_ref, xo, xt[0], phi, adj, g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha,
                       O.OracleDenoiser(resolve_weights(ARCH, 3)), iters, method, 3, r)


def _run(xt, xobs64, x0, phi, adj, prm, iters, method, r, sl=slice(None)):
    from pnppds.iteration import test_iter_batch
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha = prm
    return test_iter_batch(x0[sl], xobs64[sl], xt[sl], phi, adj, g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp,
                           palpha, ARCH, iters, method, 3, r)


def test_cfg3_ours_b_blur_sparse_batch64():
    """cfg3: batch 64, RGB 256x256, blur + Gaussian 0.01 + salt-and-pepper 0.1, ours-B; image 0
    against the oracle every iteration for 60 iterations."""
    B, H, iters, r = 64, 256, 60, 0.8
    prm = (1.0, 0.49, 0.95, 0.95, 1.0, 15, 15, 0.1, 0.01, 0.1, 300.0)   # param_memo.py:44
    xt = _synthetic(B, H, H, seed=3)
    phi, adj, xobs, x0 = _observe(xt, "blur", r, 0.01, 0.1, False, 300.0)
    x, s, c, psnr, ssim, _ = _run(xt, xobs, x0, phi, adj, prm, iters, "ours-B", r)
    assert np.isfinite(x).all() and np.isfinite(c).all()
    # image 0 vs the oracle on the same observation
    xo, so, co, po, _, _ = _oracle_image0(xt, xobs, "blur", r, prm, iters, "B-Proposed")
    print(f"cfg3: |dPSNR| {np.abs(psnr[0] - po).max():.5f} dB, max|dx| {np.abs(x[0] - xo).max():.2e}, "
          f"max|ds| {np.abs(s[0] - so).max():.2e}")
    np.testing.assert_allclose(psnr[0], po, atol=0.01)
    np.testing.assert_allclose(x[0], xo, atol=2e-3)        # fp16 (auto): measured 9.5e-4 (r05)
    np.testing.assert_allclose(s[0], so, atol=1e-3)        # measured 3.0e-4
    # s stays in the l1 ball of radius eta = alpha_s * N * sp_nl * r * 0.5 (operators.py:94-100)
    eta = 0.95 * x[0].size * 0.1 * r * 0.5
    l1 = np.abs(s.astype(np.float64) - 0.5).reshape(B, -1).sum(1)
    assert (l1 <= eta * (1 + 1e-4)).all(), (l1.max(), eta)
    # the last image alone gives the same bits
    x1, s1, c1, p1, _, _ = _run(xt, xobs, x0, phi, adj, prm, iters, "ours-B", r, sl=slice(B - 1, B))
    np.testing.assert_array_equal(x1[0], x[B - 1])
    np.testing.assert_array_equal(s1[0], s[B - 1])
    np.testing.assert_array_equal(p1[0], psnr[B - 1])


def test_cfg4_ours_c_random_sampling_poisson_512():
    """cfg4: RGB 512x512, random_sampling r=0.8 + Poisson alpha=300, ours-C; one GPU's shard
    of the 8-GPU batch of 256 (32 images); image 0 against the oracle for 50 iterations."""
    B, H, iters, r = 32, 512, 50, 0.8
    prm = (0.00035, 1 / 0.00035, 1.0, 1.0, 1.0, 15, 15, 0.1, 0.0, 0.0, 300.0)   # param_memo.py:92
    xt = _synthetic(B, H, H, seed=4)
    phi, adj, xobs, x0 = _observe(xt, "random_sampling", r, 0.0, 0.0, True, 300.0)
    assert np.array_equal(xobs, np.round(xobs)) and (xobs >= 0).all()      # Poisson counts
    x, s, c, psnr, ssim, _ = _run(xt, xobs, x0, phi, adj, prm, iters, "ours-C", r)
    assert np.isfinite(x).all() and np.isfinite(psnr).all()
    np.testing.assert_array_equal(s, np.float32(0.5))                        # C never touches s
    xo, so, co, po, _, _ = _oracle_image0(xt, xobs, "random_sampling", r, prm, iters, "C-Proposed", poisson=True)
    print(f"cfg4: |dPSNR| {np.abs(psnr[0] - po).max():.5f} dB, max|dx| {np.abs(x[0] - xo).max():.2e}, "
          f"c rel {np.abs(c[0] - co).max() / np.abs(co).min():.2e}")
    np.testing.assert_allclose(psnr[0], po, atol=0.01)
    np.testing.assert_allclose(x[0], xo, atol=1e-5)        # split fp16 (auto): measured 3.5e-6 (r05)
    np.testing.assert_allclose(c[0], co, rtol=1e-4, atol=1e-9)   # measured 9e-6 relative
    x1, s1, c1, p1, _, _ = _run(xt, xobs, x0, phi, adj, prm, iters, "ours-C", r, sl=slice(B - 1, B))
    np.testing.assert_array_equal(x1[0], x[B - 1])
    np.testing.assert_array_equal(p1[0], psnr[B - 1])


def test_cfg5_admm_blur_sparse_1024():
    """cfg5: RGB 1024x1024, blur + Gaussian 0.01 + salt-and-pepper 0.1, ours-B with the ADMM
    inner step (comparisonB-2, m1=35, m2=5, param_memo.py:61-63); one GPU's shard of the
    8-GPU batch of 512 (64 images), one outer iteration.  The oracle's CPU denoiser needs
    ~2 s per 1024^2 pass, so image 0 is compared with m1 = m2 = 2."""
    B, H, r = 64, 1024, 0.8
    prm = (0.99, 0.99, 0.95, 0.95, 1.0, 35, 5, 0.1, 0.01, 0.1, 300.0)
    xt = _synthetic(B, H, H, seed=5)
    phi, adj, xobs, x0 = _observe(xt, "blur", r, 0.01, 0.1, False, 300.0)
    x, s, c, psnr, ssim, _ = _run(xt, xobs, x0, phi, adj, prm, 1, "comparisonB-2", r)
    assert np.isfinite(x).all() and np.isfinite(s).all() and np.isfinite(c).all() and np.isfinite(psnr).all()
    x1, s1, c1, p1, _, _ = _run(xt, xobs, x0, phi, adj, prm, 1, "comparisonB-2", r, sl=slice(B - 1, B))
    np.testing.assert_array_equal(x1[0], x[B - 1])
    np.testing.assert_array_equal(s1[0], s[B - 1])
    # image 0 against the oracle at m1 = m2 = 2
    prm2 = prm[:5] + (2, 2) + prm[7:]
    xb, sb, cb, pb, _, _ = _run(xt, xobs, x0, phi, adj, prm2, 1, "comparisonB-2", r, sl=slice(0, 1))
    xo, so, co, po, _, _ = _oracle_image0(xt, xobs, "blur", r, prm2, 1, "comparisonB-2")
    print(f"cfg5 m1=m2=2: |dPSNR| {np.abs(pb[0] - po).max():.5f} dB, max|dx| {np.abs(xb[0] - xo).max():.2e}, "
          f"max|ds| {np.abs(sb[0] - so).max():.2e}")
    np.testing.assert_allclose(pb[0], po, atol=0.01)
    np.testing.assert_allclose(xb[0], xo, atol=7.5e-4)     # fp16 (auto): measured 2.5e-4 (r05)
    np.testing.assert_allclose(sb[0], so, atol=1.5e-4)     # measured 4.4e-5


def test_cfg5_admm_full_inner_counts_256_crop():
    """cfg5's method at its own inner counts (m1 = 35 denoiser x-steps, m2 = 5 l1 s-steps,
    admm.py:30-44) for one outer iteration on a 256^2 crop, against the oracle."""
    H, r = 256, 0.8
    prm = (0.99, 0.99, 0.95, 0.95, 1.0, 35, 5, 0.1, 0.01, 0.1, 300.0)
    xt = np.ascontiguousarray(_synthetic(1, 1024, 1024, seed=5)[:, :, :H, :H])
    phi, adj, xobs, x0 = _observe(xt, "blur", r, 0.01, 0.1, False, 300.0)
    x, s, c, psnr, _, _ = _run(xt, xobs, x0, phi, adj, prm, 1, "comparisonB-2", r)
    xo, so, co, po, _, _ = _oracle_image0(xt, xobs, "blur", r, prm, 1, "comparisonB-2")
    print(f"cfg5 crop m1=35 m2=5: |dPSNR| {abs(psnr[0, 0] - po[0]):.5f} dB, max|dx| {np.abs(x[0] - xo).max():.2e}, "
          f"max|ds| {np.abs(s[0] - so).max():.2e}")
    np.testing.assert_allclose(psnr[0], po, atol=0.01)
    np.testing.assert_allclose(x[0], xo, atol=7.5e-4)      # fp16 (auto): measured 2.7e-4 (r05)
    np.testing.assert_allclose(s[0], so, atol=2e-4)        # measured 6.4e-5
