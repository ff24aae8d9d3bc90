"""Pin the oracle (CPU restatement) against golden vectors from the imported reference."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import pnp_oracle as O
from pnppds.weights import DenoiserWeights, WEIGHTS_DIR

import os


def test_blur_and_adjoint(golden_ops):
    g = golden_ops
    h = g["h"]
    for tag in ("rgb64", "gray64", "gray256", "rgb48x80"):
        x = g[f"x_{tag}"]
        np.testing.assert_allclose(O.blur(x, h), g[f"phi_blur_{tag}"], atol=1e-12, rtol=0)
        np.testing.assert_allclose(O.adj_blur(x, h), g[f"adj_blur_{tag}"], atol=1e-12, rtol=0)


def test_random_sampling(golden_ops):
    g = golden_ops
    for tag in ("rgb64", "gray64"):
        for r, key in ((0.8, "rs8"), (0.5, "rs5")):
            x = g[f"x_{tag}"]
            np.testing.assert_array_equal(O.random_sampling(x, r), g[f"phi_{key}_{tag}"])
            np.testing.assert_array_equal(O.random_sampling(x, r), g[f"adj_{key}_{tag}"])


def test_mask_count():
    m = O.sampling_mask(256, 256, 0.8)
    assert m.sum() == 256 * 256 - round(256 * 256 * 0.2)


def test_proxes(golden_ops):
    g = golden_ops
    v, x0 = g["prox_v"], g["prox_x0"]
    for nl, a in ((0.01, 0.95), (10.0, 1.0)):
        np.testing.assert_allclose(O.proj_l2_ball(x0 + v, a, nl, 0.1, x0, 0.8), g[f"l2_{nl}_{a}"], atol=1e-14)
    for sp in (0.0, 0.01, 0.1, 0.5):
        np.testing.assert_allclose(O.proj_l1_ball(v, 0.95, sp, 0.8), g[f"l1_{sp}"], atol=1e-14)
    np.testing.assert_allclose(O.proj_l1_ball(v * 1e-4, 0.95, 0.1, 1), g["l1_inside"], atol=1e-18)
    np.testing.assert_allclose(O.prox_gkl(v * 10, 0.5, 300.0, np.round(x0 * 300)), g["gkl"], atol=1e-12)
    assert abs(O.psnr(x0, x0 + v) - g["psnr"][0]) < 1e-12


@pytest.mark.parametrize("name", ["DnCNN_nobn_nch_3_nlev_0.01", "DnCNN_nobn_nch_1_nlev_0.01",
                                  "dncnn_color_blind", "dncnn_15"])
def test_denoiser(golden_denoiser, name):
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    d = O.OracleDenoiser(w)
    xin, ref = golden_denoiser[f"in_{name}"], golden_denoiser[f"out_{name}"]
    out = d.denoise(xin)
    # torch-CPU conv2d in both: bit-exact up to oneDNN's thread-blocking (tiny)
    np.testing.assert_allclose(out, ref, atol=2e-6, rtol=0)


def test_denoiser_fp16_emulation_within_tolerance(golden_denoiser):
    """fp16 operands / fp32 accumulation (the device numerics) stay close to fp32."""
    name = "DnCNN_nobn_nch_3_nlev_0.01"
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    out = O.OracleDenoiser(w, emulate_fp16=True).denoise(golden_denoiser[f"in_{name}"])
    err = np.abs(out - golden_denoiser[f"out_{name}"]).max()
    assert err < 5e-3, err


@pytest.mark.parametrize("case", ["A_blur", "A_id", "A_rs", "A_gray", "B_blur", "C_rs", "C_blur", "ADMM_B2"])
def test_test_iter_trajectory(case):
    g = load_golden(f"iter_{case}.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, str(g["arch"]) + ".npz"))
    h = load_golden("ops.npz")["h"]
    phi, adj = O.observation_operators(str(g["deg_op"]), h, r)
    x, s, c, ps, _ss, _t = O.test_iter(g["x_0"], g["x_obs"], g["x_true"], phi, adj, g1, g2, as_, an, lam,
                                       int(m1), int(m2), gadmm, sig, sp, palpha, O.OracleDenoiser(w),
                                       int(iters), str(g["method"]), int(ch), r)
    np.testing.assert_allclose(x, g["x_out"], atol=2e-5)
    np.testing.assert_allclose(s, g["s_out"], atol=2e-5)
    np.testing.assert_allclose(c, g["c"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(ps, g["psnr"], atol=1e-4)


CMP_CASES = ["A_pnpfbs", "A_pdstv", "A_fbstv", "A_red", "A_unstable", "B3_htv", "C_admm", "C_red", "C_unstable"]


@pytest.mark.parametrize("case", CMP_CASES)
def test_comparison_method_trajectory(case):
    """Comparison methods (iteration.py:71-180) restated vs the reference's own trajectories."""
    g = load_golden(f"iter_cmp_{case}.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, str(g["arch"]) + ".npz"))
    h = load_golden("ops.npz")["h"]
    phi, adj = O.observation_operators(str(g["deg_op"]), h, r)
    x, s, c, ps, _ss, _t = O.test_iter(g["x_0"], g["x_obs"], g["x_true"], phi, adj, g1, g2, as_, an, lam,
                                       int(m1), int(m2), gadmm, sig, sp, palpha, O.OracleDenoiser(w),
                                       int(iters), str(g["method"]), int(ch), r)
    np.testing.assert_allclose(x, g["x_out"], atol=2e-5)
    np.testing.assert_allclose(s, g["s_out"], atol=2e-5)
    np.testing.assert_allclose(c, g["c"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(ps, g["psnr"], atol=1e-4)


def test_method_alias_and_unknown():
    x = np.zeros((1, 8, 8))
    phi, adj = O.observation_operators("Id")
    with pytest.raises(ValueError):
        O.test_iter(x, x, x, phi, adj, 1, 1, 1, 1, 1, 1, 1, 0.1, 0.01, 0, 300, None, 1, "nope", 1, 1)
