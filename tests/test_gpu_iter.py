"""GPU parity of the whole on-device PnP-PDS loop vs trajectories of the reference's test_iter."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu

CASES = ["A_blur", "A_id", "A_rs", "A_gray", "B_blur", "C_rs", "C_blur", "ADMM_B2"]


def run_case(g):
    from pnppds import operators as ops
    from pnppds.iteration import test_iter
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    phi, adj = ops.get_observation_operators(str(g["deg_op"]), "blur_1", r)
    return test_iter(g["x_0"], g["x_obs"], g["x_true"], phi, adj, g1, g2, as_, an, lam, int(m1), int(m2), gadmm,
                     sig, sp, palpha, str(g["arch"]) + ".pth", int(iters), str(g["method"]), int(ch), r)


@pytest.mark.parametrize("case", CASES)
def test_trajectory_matches_reference(case):
    g = load_golden(f"iter_{case}.npz")
    x, s, c, psnr, ssim, t = run_case(g)
    assert x.shape == g["x_out"].shape and x.dtype == np.float32
    # PSNR within the north-star tolerance (0.01 dB) at every iteration
    from pnppds._device import get_ctx
    print(f"{case} ({get_ctx().get_precision()[1]}): max|dx| {np.abs(x - g['x_out']).max():.2e}, "
          f"max|dPSNR| {np.abs(psnr - g['psnr']).max():.2e} dB")
    np.testing.assert_allclose(psnr, g["psnr"], atol=0.01)
    # r06 measured: fp16 2.5-3.8e-4, split fp16 1.8-3.6e-7 (5e-3 for every precision before)
    np.testing.assert_allclose(x, g["x_out"], atol={"fp16": 1e-3, "fp16w2": 1e-3}.get(get_ctx().get_precision()[1], 1e-6))
    np.testing.assert_allclose(c, g["c"], rtol=0.05, atol=2e-4)
    s_is_zero = case.startswith(("A_", "C_"))          # A / C never touch s: s + 0.5 exactly
    np.testing.assert_allclose(s, g["s_out"], atol=1e-7 if s_is_zero else 5e-3)
    assert t > 0


def test_long_run_psnr_within_001db():
    """3x256x256, ours-A + blur, 120 iterations: every PSNR within 0.01 dB of the reference."""
    from pnppds import operators as ops
    from pnppds.iteration import test_iter
    g = load_golden("long_A_blur_256.npz")
    phi, adj = ops.get_observation_operators("blur", "blur_1", 0.8)
    x, s, c, psnr, ssim, t = test_iter(g["x_obs"], g["x_obs"], g["x_true"], phi, adj, 0.99, 0.99, 1.0, 0.95, 1.0,
                                       15, 15, 0.1, 0.01, 0.0, 300, "DnCNN_nobn_nch_3_nlev_0.01.pth", 120,
                                       "ours-A", 3, 0.8)
    d = np.abs(psnr - g["psnr"])
    print(f"long_A_blur_256: max|dx| {np.abs(x - g['x_out']).max():.2e}, max|dPSNR| {d.max():.2e} dB")
    assert d.max() < 0.01, (d.max(), int(d.argmax()))
    np.testing.assert_allclose(x, g["x_out"], atol=1e-3)          # r06: 4.5e-4 (fp16)


def test_batch_equals_single_images():
    """Images are independent: a batch gives bit-identical results to one-image runs
    (the property the multi-GPU sharding relies on)."""
    from pnppds import operators as ops
    from pnppds.iteration import test_iter_batch
    g = load_golden("iter_B_blur.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    rng = np.random.default_rng(0)
    xt = np.stack([g["x_true"], np.clip(g["x_true"] + 0.05 * rng.standard_normal(g["x_true"].shape), 0, 1),
                   g["x_true"][:, ::-1, :]]).astype(np.float32)
    phi, adj = ops.get_observation_operators("blur", "blur_1", r)
    xo = np.stack([O.blur(a, ops.load_blur_kernel("blur_1")) + 0.01 * rng.standard_normal(a.shape) for a in xt])
    args = (g1, g2, as_, an, lam, int(m1), int(m2), gadmm, sig, sp, palpha, "DnCNN_nobn_nch_3_nlev_0.01", 4,
            "B-Proposed", 3, r)
    xb, sb, cb, pb, _, _ = test_iter_batch(xo, xo, xt, phi, adj, *args)
    for i in range(3):
        x1, s1, c1, p1, _, _ = test_iter_batch(xo[i:i + 1], xo[i:i + 1], xt[i:i + 1], phi, adj, *args)
        np.testing.assert_array_equal(x1[0], xb[i])
        np.testing.assert_array_equal(s1[0], sb[i])
        np.testing.assert_array_equal(p1[0], pb[i])


def test_unknown_method_and_closure_rejected():
    from pnppds import operators as ops
    from pnppds.iteration import test_iter
    x = np.zeros((3, 16, 16))
    phi, adj = ops.get_observation_operators("Id", "blur_1", 0.8)
    with pytest.raises(ValueError):
        test_iter(x, x, x, phi, adj, 1, 1, 1, 1, 1, 1, 1, 0.1, 0.01, 0, 300, "DnCNN_nobn_nch_3_nlev_0.01", 1,
                  "A-Nonexistent", 3, 1)
    with pytest.raises(TypeError):
        test_iter(x, x, x, lambda v: v, lambda v: v, 1, 1, 1, 1, 1, 1, 1, 0.1, 0.01, 0, 300,
                  "DnCNN_nobn_nch_3_nlev_0.01", 1, "A-Proposed", 3, 1)


def test_numpy_api_mirrors_reference(golden_ops):
    """pnppds.operators functions (numpy in / numpy out, device inside) vs golden."""
    from pnppds import operators as ops
    g = golden_ops
    phi, adj = ops.get_observation_operators("blur", "blur_1", 0.8)
    np.testing.assert_allclose(phi(g["x_rgb64"]), g["phi_blur_rgb64"], atol=2e-6)
    np.testing.assert_allclose(adj(g["x_gray64"]), g["adj_blur_gray64"], atol=2e-6)
    v, x0 = g["prox_v"], g["prox_x0"]
    np.testing.assert_allclose(ops.proj_l2_ball(x0 + v, 0.95, 0.01, 0.1, x0, 0.8), g["l2_0.01_0.95"], atol=2e-7)
    np.testing.assert_allclose(ops.proj_l1_ball(v, 0.95, 0.1, 0.8), g["l1_0.1"], atol=1e-6)


@pytest.mark.parametrize("deg_op,method,C,H,W", [("Id", "A-Proposed", 3, 37, 53), ("random_sampling", "C-Proposed", 3, 30, 45),
                                                 ("random_sampling", "B-Proposed", 1, 34, 41),
                                                 ("blur", "B-Proposed", 3, 50, 70)])
def test_ragged_shapes_vs_oracle(deg_op, method, C, H, W):
    """Widths that are not multiples of 4 (the scalar edge paths of the pointwise K1/K2) or of
    the 64-pixel blur tile, every operator, against the oracle on the same observation."""
    from pnppds import operators as ops
    from pnppds.iteration import test_iter
    from pnppds.noise import make_observation
    from pnppds.weights import resolve_weights
    rng = np.random.default_rng(H * W)
    yy, xx = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    xt = np.stack([0.5 + 0.3 * np.sin(5 * xx + c) * np.cos(3 * yy) for c in range(C)]).astype(np.float32)
    xt = np.clip(xt + 0.02 * rng.standard_normal(xt.shape), 0, 1).astype(np.float32)
    if C == 1:
        xt = xt[0]
    poisson = method == "C-Proposed"
    sp = 0.1 if method == "B-Proposed" else 0.0
    sig = 0.0 if poisson else 0.01
    xobs, x0 = make_observation(xt, deg_op, "blur_1", 0.8, sig, sp, poisson, 300.0)
    if method == "C-Proposed":
        g1, g2 = 0.00035, 1 / 0.00035
    elif method == "B-Proposed":
        g1, g2 = 1.0, 0.49
    else:
        g1, g2 = 0.99, 0.99
    arch = "DnCNN_nobn_nch_3_nlev_0.01" if C == 3 else "DnCNN_nobn_nch_1_nlev_0.01"
    args = (g1, g2, 0.95, 0.95, 1.0, 15, 15, 0.1, sig, sp, 300.0)
    phi, adj = ops.get_observation_operators(deg_op, "blur_1", 0.8)
    x, s, c, psnr, _, _ = test_iter(x0, xobs, xt, phi, adj, *args, arch + ".pth", 4, method, C, 0.8)
    p_ref, p_adj = O.observation_operators(deg_op, ops.load_blur_kernel("blur_1"), 0.8)
    xo, so, co, po, _, _ = O.test_iter(np.asarray(x0, np.float64), np.asarray(xobs, np.float64), xt, p_ref, p_adj,
                                       *args, O.OracleDenoiser(resolve_weights(arch, C)), 4, method, C, 0.8)
    np.testing.assert_allclose(psnr, po, atol=0.01)
    np.testing.assert_allclose(x, xo, atol=5e-3)
    np.testing.assert_allclose(s, so, atol=5e-3)


@pytest.mark.parametrize("case", ["A_blur", "A_rs", "B_blur", "C_rs"])
def test_metrics_paths_do_not_change_iterates(case):
    """x_true and metric recording feed only the metrics: with x_true absent (PSNR/SSIM NaN) or
    recording off (all metrics NaN) the iterates are the same bits.  Covers the kernels'
    compile-time no-x_true / no-record instantiations."""
    from pnppds import operators as ops
    from pnppds.iteration import test_iter_batch
    g = load_golden(f"iter_{case}.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    phi, adj = ops.get_observation_operators(str(g["deg_op"]), "blur_1", r)
    arch = str(g["arch"]) + ".pth"
    args = (g1, g2, as_, an, lam, int(m1), int(m2), gadmm, sig, sp, palpha, arch, int(iters), str(g["method"]),
            int(ch), r)
    x0, xo, xt = g["x_0"][None], g["x_obs"][None], g["x_true"][None]
    full = test_iter_batch(x0, xo, xt, phi, adj, *args)
    no_true = test_iter_batch(x0, xo, None, phi, adj, *args)
    no_rec = test_iter_batch(x0, xo, xt, phi, adj, *args, record_metrics=False)
    for other in (no_true, no_rec):
        np.testing.assert_array_equal(other[0], full[0])     # x
        np.testing.assert_array_equal(other[1], full[1])     # s
    np.testing.assert_array_equal(no_true[2], full[2])       # c_n does not use x_true
    assert np.isnan(no_true[3]).all() and np.isfinite(full[3]).all()


def test_profile_modes():
    """pnp_profile_enable: 1 times every launch, 2 only the denoiser's body launches (the bench's
    timed region), 0 none; other values are rejected.  The iterates do not depend on it."""
    from pnppds import operators as ops
    from pnppds._device import get_ctx
    from pnppds.iteration import _resolve_denoiser, make_params, resolve_method
    from pnppds._lib import PnpError
    g = load_golden("iter_A_blur.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    phi, adj = ops.get_observation_operators(str(g["deg_op"]), "blur_1", r)
    ctx = get_ctx()
    den = _resolve_denoiser(str(g["arch"]) + ".pth", int(ch))
    den.configure(ctx)
    x0 = np.asarray(g["x_0"], np.float32)
    to4 = lambda a: np.asarray(a, np.float32).reshape((1,) + x0.shape)   # noqa: E731
    B, C, H, W = to4(x0).shape
    phi.configure(ctx, H, W)
    prm = make_params(g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, r, True, False)
    xs = []
    for mode in (0, 1, 2):
        ctx.solver_setup(resolve_method(str(g["method"])), prm, B, C, H, W, 4)
        ctx.solver_load(to4(x0), to4(g["x_obs"]), to4(g["x_true"]))
        ctx.profile_enable(mode)
        ctx.solver_iterate(4)
        names = set(ctx.profile_read())
        ctx.profile_enable(0)
        xs.append(ctx.solver_fetch()[0])
        if mode == 0:
            assert not names
        elif mode == 1:
            assert any(n.startswith("k2") for n in names) and any(n.startswith("conv") for n in names)
        else:
            assert names and all(n.startswith(("conv_body", "conv32_body", "conv_stack")) for n in names), names
    np.testing.assert_array_equal(xs[1], xs[0])
    np.testing.assert_array_equal(xs[2], xs[0])
    with pytest.raises(PnpError):
        ctx.profile_enable(3)
