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
# c_n = ||x_n - x_prev|| / ||x_prev|| (iteration.py:187), the reference's convergence output
# (c_evolution, main.py:82; plotted on a log axis by plot.py:26,49).  Checked to C_RTOL relative
# wherever the reference's c is at least the mode's C_MIN:
#  * near-fp32 operands (split fp16 'fp16x3', 'fp32', and 'converge' after its hand-over) follow
#    the reference's c down to its ~7e-8 floor within a few per cent (r05 probe,
#    profiles/r05/converge_probe.txt: <= 1.7 % wherever c_ref >= 1e-6; their own floor is
#    ~1.6e-7, which is why C_MIN is 1e-6);
#  * fp16 activations ('fp16', 'fp16w2') settle on the fp16-rounded map's fixed point, where
#    successive iterates stay about one fp16 rounding apart: c stalls at FP16_C_FLOOR's order
#    (2.3-2.8e-4 on every blur golden, r04 parity.txt) while the reference's keeps contracting.
#    There c is checked to C_RTOL only where c_ref >= 10x that floor, and everywhere to
#    |c - c_ref| <= C_RTOL c_ref + FP16_C_FLOOR (so a worse floor fails).  'converge' exists for the c
#    curve: see test_converge_c_trajectory.
C_RTOL = 0.10
FP16_C_FLOOR = 5e-4
C_MIN = {"fp16": 3e-3, "fp16w2": 3e-3, "fp16x3": 1e-6, "fp32": 1e-6, "fp16a2": 1e-6}   # fp16: ~10x its floor
# x against the reference's final iterate (stored in fp32 since round 6: the fp16 fixture of
# rounds 2-5 capped the check at half an fp16 ulp, 2.4e-4).  Measured max |dx| on the fp32
# fixtures (r06, gpurun_out/r06/f/pytest.log; the bounds are 2-3x the largest of each group):
#  * fp32 operands: 7.8e-7 (ours-A blur x 1200) and 3.6e-6 (ours-B x 300);
#  * split fp16 (fp16x3): 3.6e-7 .. 4.8e-6 on the well-conditioned goldens, ours-B sigma 0.02
#    x 1200 3.6e-5 (its l1-ball support moving), ours-C x 300 1.7e-5;
#  * fp16 / fp16w2 activations: 3.7e-4 .. 8.7e-4 / 3.9e-4 .. 4.2e-4 (ours-B x 300: 1.9e-3);
#  * fp16a2 (converge after its hand-over): 8.6e-5 .. 4.4e-4, ours-A sigma 0.04 1.3e-3.
# Two trajectories are ill-conditioned (a perturbation of the iterate grows over the run): ours-C
# x 3000 (random sampling + Poisson, gamma2 = 1 / gamma1 = 2857) and RED at sigma 0.04.  There
# the fp32 control lands 5.3e-5 / 2.6e-4 from the reference (the device's fp32 summation order
# alone) and split fp16 1.6e-4 / 2.1e-4.  (Before round 6 split fp16 landed 2.2e-3 / 1.2e-3 there
# and had per-case bounds of 4e-3 / 2.5e-3: its weights' low halves were fp16 subnormals; they are
# split at 2^8 times the weights now, common.h kSplitWScale)
X_TOL = {"fp16": 2e-3, "fp16w2": 1e-3, "fp16x3": 1e-4, "fp32": 1e-5, "fp16a2": 3e-3}
X_TOL_CASE = {("B_blur_300", "fp16"): 4e-3,   # 1.9e-3: fp16 activations; its fp32 control is 3.6e-6 (fp32 row)
              # the ill-conditioned pair, each with its fp32 control beside it
              ("C_rs_3000", "fp16x3"): 5e-4, ("C_rs_3000", "fp32"): 1.5e-4,                 # 1.6e-4 / 5.3e-5
              ("RED_blur_s004_1200", "fp16x3"): 6e-4, ("RED_blur_s004_1200", "fp32"): 7e-4}  # 2.1e-4 / 2.6e-4


def check_c(case, c, gc, prec):
    """c (the device's c_n per iteration) against the golden's, per the mode's rule above."""
    gc = np.asarray(gc, np.float64)
    m = gc >= C_MIN[prec]
    rel = np.abs(c[m] - gc[m]) / gc[m]
    print(f"  c_n: max rel err {rel.max() if rel.size else 0:.4f} over {int(m.sum())} iterations with c_ref >= "
          f"{C_MIN[prec]:.0e}; final {c[-1]:.3e} vs {gc[-1]:.3e}")
    assert rel.size == 0 or rel.max() <= C_RTOL, (case, prec, float(rel.max()), int(np.argmax(rel)))
    if prec in ("fp16", "fp16w2") and case not in CHAOTIC:
        # everywhere: the fp16 floor adds to the reference's c at most FP16_C_FLOOR
        err = np.abs(c - gc) - C_RTOL * gc
        assert np.all(err <= FP16_C_FLOOR), (case, prec, int(np.argmax(err)), float(err.max()))


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
                                            # round 5: comparisonB-2 above sigma 0.01 (auto:
                                            # fp16w2) at the 200 outer iterations that qualified fp16
                                            ("ADMM_B2_s002_200", "auto"), ("ADMM_B2_s004_200", "auto"),
                                            ("A_blur_s004_1200", "fp16x3"),
                                            # round 6: fp32 controls of the two
                                            # split-fp16 cases with per-case x bounds
                                            ("C_rs_3000", "fp32"), ("RED_blur_s004_1200", "fp32")])
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
    prec = get_ctx().get_precision()[1]          # what 'auto' resolved to for this solve
    if case not in CHAOTIC:
        dx = np.abs(x - g["x_out"].astype(np.float32)).max()
        print(f"  max|dx| {dx:.2e}")
        assert dx <= X_TOL_CASE.get((case, prec), X_TOL[prec]), (case, prec, float(dx))
    if precision == "auto":
        assert prec == expected_auto(g), (case, prec)
        if prec in ("fp16", "fp16w2"):
            # the policy runs fp16 activations only with half the bound to spare
            assert d.max() <= AUTO_FP16_MARGIN_DB, (case, d.max())
    check_c(case, c, g["c"], prec)


CONVERGE_C = 3e-3   # PNP_PREC_CONVERGE's default threshold (include/pnppds.h PNP_TUNE_CONVERGE_C)


@pytest.mark.parametrize("case", ["A_blur_1200", "B_blur_1200", "ADMM_B2_200", "A_blur_s004_1200",
                                  "FBS_blur_1200", "RED_blur_s0025_1200", "A_blur_s0025_a100_1200"])
def test_converge_c_trajectory(case):
    """precision='converge' (PNP_PREC_CONVERGE): auto's fp16 / fp16w2 operands until the smallest
    c_n of the batch falls below 3e-3, split activations (fp16a2) from two iterations later (the
    host reads c_n one iteration behind the device).  The returned c follows the reference's within 10 % wherever
    the reference's is >= 1e-6 (fp16 alone stalls near 3e-4 there, 1 100+ of 1 200 iterations of
    long_A_blur_1200 unchecked before round 5), PSNR within the bound with auto's margin, x like
    split fp16's; the reported switch iteration is where the rule puts it."""
    from pnppds.iteration import last_precision_switch
    g = load_golden(f"long_{case}.npz")
    x, s, c, psnr, ssim, t = run_long(g, "converge")
    sw = last_precision_switch()
    below = np.nonzero(c < CONVERGE_C)[0]
    assert below.size and sw == below[0] + 2, (case, sw, below[:3])
    d = np.abs(psnr - g["psnr"])
    dx = np.abs(x - g["x_out"].astype(np.float32)).max()
    print(f"{case} converge: switch at {sw}; max|dPSNR| {d.max():.5f} dB at {int(d.argmax())}; max|dx| {dx:.2e}")
    assert d.max() <= AUTO_FP16_MARGIN_DB, (case, d.max())
    assert dx <= X_TOL["fp16a2"], (case, dx)       # after the hand-over: fp16a2 (fp16 weights)
    check_c(case, c, g["c"], "fp16a2")


def test_converge_handover_bits():
    """The hand-over is a plain precision change between iterations: a converge solve that
    switches at iteration k gives the bits of k fp16 iterations followed by fp16a2 ones; with no
    metrics to watch it runs split activations from iteration 0 (switch 0, fp16a2's bits)."""
    from pnppds import operators as ops
    from pnppds._device import get_ctx
    from pnppds.iteration import _resolve_denoiser, make_params, resolve_method
    g = load_golden("long_A_blur_1200.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    phi, adj = ops.get_observation_operators("blur", "blur_1", r)
    ctx = get_ctx()
    _resolve_denoiser(str(g["arch"]) + ".pth", 3).configure(ctx)
    x0, xo, xt = (np.asarray(g[k], np.float32)[None] for k in ("x_0", "x_obs", "x_true"))
    phi.configure(ctx, x0.shape[2], x0.shape[3])
    n = 40

    def solve(plan, record=True, threshold=None):
        ctx.set_precision(plan[0][0])
        if threshold:
            ctx.set_converge_threshold(threshold)
        ctx.solver_setup(resolve_method("A-Proposed"),
                         make_params(g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, r, record, False),
                         1, 3, x0.shape[2], x0.shape[3], n)
        ctx.solver_load(x0, xo, xt)
        for prec, k in plan:
            ctx.set_precision(prec)
            ctx.solver_iterate(k)
        out = ctx.solver_fetch()
        return out, ctx.get_precision_switch()

    try:
        (xc, _, cc, pc, _), sw = solve([("converge", n)], threshold=CONVERGE_C)
        assert 2 <= sw < n, sw
        (xm, _, cm, pm, _), _ = solve([("fp16", sw), ("fp16a2", n - sw)])
        np.testing.assert_array_equal(xc, xm)
        np.testing.assert_array_equal(cc, cm)
        np.testing.assert_array_equal(pc, pm)
        (xn, _, _, _, _), sw0 = solve([("converge", n)], record=False)
        (xs, _, _, _, _), _ = solve([("fp16a2", n)], record=False)
        assert sw0 == 0
        np.testing.assert_array_equal(xn, xs)
    finally:
        ctx.set_converge_threshold(CONVERGE_C)
        ctx.set_precision("auto")


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
        dx = np.abs(x[b] - xr).max()
        rel = np.abs(c[b] - cr) / cr
        print(f"image {b}: max|dPSNR| {np.abs(psnr[b] - pr).max():.5f} dB, max|dx| {dx:.2e}, c rel {rel.max():.4f}")
        assert dx <= X_TOL["fp16"], (b, dx)
        np.testing.assert_allclose(c[b], cr, rtol=0.05, atol=2e-4)
    x1, s1, c1, p1, _, _ = test_iter_batch(xo[127:128], xo[127:128], xt[127:128], phi, adj, *args)
    np.testing.assert_array_equal(x1[0], x[127])
    np.testing.assert_array_equal(p1[0], psnr[127])
