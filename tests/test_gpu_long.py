"""GPU parity at the lengths and batch the metric is quoted on.

* 1200 iterations of ours-A on 3x256^2 blur (main.py:136-139 runs blur experiments for 1200
  iterations): every iteration's PSNR within the north-star 0.01 dB of the reference's own
  trajectory (tests/golden/long_A_blur_1200.npz, made by make_golden.py --long from the
  imported reference), for the fp16-operand denoiser (default) and the fp32 one.
* 300 iterations of ours-B (blur + salt-and-pepper) and 300 / 3000 iterations of ours-C
  (random sampling + Poisson; main.py:136-139 runs 3000 for random sampling) at 3x128^2,
  same bound.
* The metric's batch, B = 256 RGB 256^2 blur: images 0, 127 and 255 against the oracle over
  20 iterations, and image 127 alone gives the batch's bits.
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu

PSNR_TOL_DB = 0.01          # north_star: PSNR within 0.01 dB of the reference
AUTO_FP16_MARGIN_DB = 0.005  # where PNP_PREC_AUTO picks plain fp16 operands: half the bound
# c_n = ||x_n - x_prev|| / ||x_prev|| (iteration.py:187).  With fp16 denoiser operands the
# iteration settles into a fixed point of the fp16-rounded map, where successive iterates
# still differ by about one fp16 rounding (2^-11 relative): c_n stalls near 3e-4 while the
# reference's fp32 iteration keeps contracting (to 7e-8 after 1200 iterations).  So c_n is
# compared down to that floor for fp16, and down to 2e-6 for the fp32-operand path.
C_FLOOR = {"fp16": 1e-3, "fp16w2": 1e-3, "fp16x3": 2e-5, "fp32": 2e-6}


# Ill-conditioned trajectories (tools/chaos_probe.py on the fp32 test oracle): ours-B
# at sigma 0.04 moves 0.19 % of its pixels by more than 5e-3 (max 0.025) when x_0 moves by one
# float32 ulp; PnP-FBS at sigma 0.04 is stable against x_0 but its final pixels differ by up to
# 0.0022 between two fp32 convolutions (the oracle's vs the reference's) and by 0.012 under split
# fp16.  Their final iterate is checked by the share of pixels more than 5e-3 off the reference's
# (bounded here), not pixel by pixel; the PSNR trajectory is the criterion.
CHAOTIC = {"B_blur_s004_1200": 0.005, "FBS_blur_s004_1200": 0.001}
FP16_BLUR = ("A-Proposed", "B-Proposed", "comparisonB-2", "A-PnPFBS-DnCNN", "A-RED-DnCNN")
FP16W2_BLUR = ("A-Proposed", "comparisonB-2")


def expected_auto(g):
    """PNP_PREC_AUTO restated (capi.hip auto_precision): the operands a solve of this golden runs."""
    sigma, method = float(g["params"][8]), str(g["method"])
    if str(g["deg_op"]) == "blur":
        if method in FP16_BLUR and sigma <= 0.01 * (1 + 1e-9):
            return "fp16"
        if method in FP16W2_BLUR:
            return "fp16w2"
    return "fp16x3"


def run_long(g, precision=None):
    from pnppds import operators as ops
    from pnppds.iteration import test_iter
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    phi, adj = ops.get_observation_operators(str(g["deg_op"]), "blur_1", r)
    kw = {} if precision is None else {"precision": precision}
    return test_iter(g["x_0"], g["x_obs"], g["x_true"], phi, adj, g1, g2, as_, an, lam, int(m1), int(m2), gadmm,
                     sig, sp, palpha, str(g["arch"]) + ".pth", int(iters), str(g["method"]), int(ch), r, **kw)


@pytest.mark.parametrize("case,precision", [("A_blur_1200", "fp16"), ("A_blur_1200", "fp32"),
                                            ("B_blur_300", "fp16"), ("B_blur_300", "fp32"),
                                            ("A_blur_1200", "fp16w2"),
                                            ("C_rs_300", "auto"), ("C_rs_3000", "auto"),
                                            # split fp16 (three MFMAs per product)
                                            ("A_blur_1200", "fp16x3"), ("C_rs_3000", "fp16x3"),
                                            ("B_blur_300", "fp16x3"),
                                            # the reference's other regimes (main.py:130-139, BASELINE
                                            # config 1): gray 256^2 Id, random sampling x 3000, sigma 0.0025
                                            ("A_gray_id_1200", "auto"), ("A_rs_3000", "auto"),
                                            ("A_blur_s0025_1200", "auto"), ("A_rs_s0025_3000", "auto"),
                                            ("A_gray_id_1200", "fp16x3"), ("A_rs_3000", "fp16x3"),
                                            ("A_blur_s0025_1200", "fp16x3"), ("A_rs_s0025_3000", "fp16x3"),
                                            # comparisonB-2 at config 5's inner counts (m1 = 35, m2 = 5)
                                            ("ADMM_B2_30", "auto"),
                                            # round 4: the fp16 regimes at the lengths they run (VERDICT
                                            # r03 item 1): ours-B blur x 1200, comparisonB-2 x 200 outer,
                                            # ours-A blur sigma 0.0025 at the grid's alpha_n = 1.00
                                            ("B_blur_1200", "auto"), ("ADMM_B2_200", "auto"),
                                            ("A_blur_s0025_a100_1200", "auto"),
                                            ("B_blur_1200", "fp16x3"), ("A_blur_s0025_a100_1200", "fp16x3"),
                                            # the rest of main.py's blur grid (:130,143): sigma 0.005 / 0.02 /
                                            # 0.04 and the smallest ball alpha_n = 0.82 at sigma 0.0025
                                            ("A_blur_s0005_1200", "auto"), ("A_blur_s002_1200", "auto"),
                                            ("A_blur_s004_1200", "auto"), ("A_blur_s0025_a082_1200", "auto"),
                                            # the grid's DnCNN comparison methods on blur (:133,148-152)
                                            ("FBS_blur_1200", "auto"), ("FBS_blur_s0025_1200", "auto"),
                                            ("RED_blur_1200", "auto"), ("RED_blur_s0025_1200", "auto"),
                                            # the grid's higher noise levels for the other methods of the
                                            # blur family (auto: fp16w2 above sigma 0.01)
                                            ("B_blur_s002_1200", "auto"), ("B_blur_s004_1200", "auto"),
                                            ("FBS_blur_s004_1200", "auto"), ("RED_blur_s004_1200", "auto"),
                                            ("ADMM_B2_s004_30", "auto"),
                                            ("A_blur_s004_1200", "fp16x3")])
def test_long_trajectory_psnr(case, precision):
    """Every iteration's PSNR within 0.01 dB of the reference's trajectory.  'auto' is the
    default precision policy (PNP_PREC_AUTO, restated in expected_auto: on blur, fp16 operands up
    to sigma 0.01, fp16w2 above it for ours-A and comparisonB-2; split fp16 elsewhere, where fp16
    ones drift 0.19 dB (ours-C over 3000 iterations) and 0.05-0.11 dB (ours-A random sampling))."""
    g = load_golden(f"long_{case}.npz")
    x, s, c, psnr, ssim, t = run_long(g, precision)
    d = np.abs(psnr - g["psnr"])
    from pnppds._device import get_ctx
    print(f"{case} {precision} ({get_ctx().get_precision()[1]}): max|dPSNR| = {d.max():.5f} dB at iteration {int(d.argmax())}, "
          f"final {psnr[-1]:.4f} vs {g['psnr'][-1]:.4f} dB")
    assert d.max() < PSNR_TOL_DB, (d.max(), int(d.argmax()))
    if case in CHAOTIC:   # a share of pixels may move; the PSNR above is the criterion
        off = np.mean(np.abs(x - g["x_out"].astype(np.float32)) > 5e-3)
        print(f"  pixels off by > 5e-3: {off:.5f}")
        assert off <= CHAOTIC[case], (case, off)
    else:
        np.testing.assert_allclose(x, g["x_out"].astype(np.float32), atol=5e-3)
    from pnppds._device import get_ctx
    prec = get_ctx().get_precision()[1]          # what 'auto' resolved to for this solve
    if precision == "auto":
        assert prec == expected_auto(g), (case, prec)
        if prec in ("fp16", "fp16w2"):
            # the policy runs fp16 activations only with half the bound to spare
            assert d.max() <= AUTO_FP16_MARGIN_DB, (case, d.max())
    np.testing.assert_allclose(c, g["c"], rtol=0.05, atol=C_FLOOR[prec])
    print(f"  c_n final {c[-1]:.3e} vs {g['c'][-1]:.3e}")


def _metric_batch(B=256, C=3, H=256, W=256):
    """Deterministic structured RGB images + blur_1 + 0.01 Gaussian noise (float32)."""
    from pnppds.operators import load_blur_kernel
    yy, xx = np.meshgrid(np.linspace(0, 1, H, dtype=np.float32), np.linspace(0, 1, W, dtype=np.float32),
                         indexing="ij")
    rng = np.random.default_rng(256)
    xt = np.empty((B, C, H, W), np.float32)
    for b in range(B):
        f = rng.uniform(1, 6, (C, 2)).astype(np.float32)
        for c in range(C):
            xt[b, c] = 0.45 + 0.25 * np.sin(2 * np.pi * f[c, 0] * xx + b) * np.cos(2 * np.pi * f[c, 1] * yy) \
                + 0.2 * (xx - 0.5)
    np.clip(xt, 0, 1, out=xt)
    h = load_blur_kernel("blur_1")
    xo = np.stack([O.blur(a.astype(np.float64), h) for a in xt])
    xo += 0.01 * rng.standard_normal(xo.shape)
    return xt, xo.astype(np.float32), h


def test_metric_batch_256_vs_oracle():
    """B = 256 RGB 256^2 blur ours-A (the metric's configuration): images 0, 127, 255 against
    the oracle (fp16-emulating denoiser) every iteration for 20 iterations."""
    from pnppds import operators as ops
    from pnppds.iteration import test_iter_batch
    from pnppds.weights import resolve_weights
    xt, xo, h = _metric_batch()
    iters = 20
    phi, adj = ops.get_observation_operators("blur", "blur_1", 0.8)
    args = (0.99, 0.99, 1.0, 0.95, 1.0, 15, 15, 0.1, 0.01, 0.0, 300, "DnCNN_nobn_nch_3_nlev_0.01", iters,
            "ours-A", 3, 0.8)
    x, s, c, psnr, _, _ = test_iter_batch(xo, xo, xt, phi, adj, *args)
    assert np.isfinite(x).all() and np.isfinite(psnr).all()
    den = O.OracleDenoiser(resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3), emulate_fp16=True)
    p_ref, p_adj = O.observation_operators("blur", h)
    for b in (0, 127, 255):
        xr, _, cr, pr, _, _ = O.test_iter(xo[b].astype(np.float64), xo[b].astype(np.float64), xt[b], p_ref, p_adj,
                                          0.99, 0.99, 1.0, 0.95, 1.0, 15, 15, 0.1, 0.01, 0.0, 300, den, iters,
                                          "A-Proposed", 3, 0.8)
        assert np.abs(psnr[b] - pr).max() < PSNR_TOL_DB, (b, np.abs(psnr[b] - pr).max())
        np.testing.assert_allclose(x[b], xr, atol=2e-3)
        np.testing.assert_allclose(c[b], cr, rtol=0.05, atol=2e-4)
    x1, s1, c1, p1, _, _ = test_iter_batch(xo[127:128], xo[127:128], xt[127:128], phi, adj, *args)
    np.testing.assert_array_equal(x1[0], x[127])
    np.testing.assert_array_equal(p1[0], psnr[127])
