"""GPU trajectories of the comparison methods (iteration.py:71-180) vs the reference's own
(tests/golden/iter_cmp_*.npz), and of comparisonB-4 / -5 vs the oracle (the reference raises
UnboundLocalError for those two, see pnppds/iteration.py).

Tolerances: methods with the fp16-operand denoiser as in test_gpu_iter (PSNR 0.01 dB,
x 5e-3); the TV methods (no denoiser, fp32 state vs the reference's fp64) x 1e-4."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu
CASES = ["A_pnpfbs", "A_pdstv", "A_fbstv", "A_red", "A_unstable", "B3_htv", "C_admm", "C_red", "C_unstable"]
TV = ("A_pdstv", "A_fbstv", "B3_htv")


def run(g, method=None, iters=None):
    from pnppds import operators as ops
    from pnppds.iteration import test_iter
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, it, ch, r = g["params"]
    phi, adj = ops.get_observation_operators(str(g["deg_op"]), "blur_1", r)
    return test_iter(g["x_0"], g["x_obs"], g["x_true"], phi, adj, g1, g2, as_, an, lam, int(m1), int(m2), gadmm,
                     sig, sp, palpha, str(g["arch"]) + ".pth", int(iters or it), method or str(g["method"]), int(ch),
                     r)


@pytest.mark.parametrize("case", CASES)
def test_trajectory_matches_reference(case):
    g = load_golden(f"iter_cmp_{case}.npz")
    x, s, c, psnr, ssim, t = run(g)
    assert x.shape == g["x_out"].shape and np.all(np.isfinite(ssim))
    tv = case in TV
    np.testing.assert_allclose(psnr, g["psnr"], atol=2e-3 if tv else 0.01)
    np.testing.assert_allclose(x, g["x_out"], atol=1e-4 if tv else 5e-3)
    np.testing.assert_allclose(c, g["c"], rtol=0.01 if tv else 0.05, atol=2e-4)
    np.testing.assert_allclose(s, g["s_out"], atol=1e-4 if tv else 5e-3)


@pytest.mark.parametrize("method", ["comparisonB-4", "comparisonB-5"])
def test_unreachable_reference_methods_vs_oracle(method):
    from pnppds.operators import load_blur_kernel
    from pnppds.weights import resolve_weights
    g = load_golden("iter_B_blur.npz")
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, it, ch, r = g["params"]
    g = dict(g)
    g["params"] = np.array([0.5, g2, as_, an, 1.0, m1, m2, gadmm, sig, sp, palpha, 4, ch, 1.0])
    x, s, c, psnr, ssim, t = run(g, method, 4)
    phi, adj = O.observation_operators("blur", load_blur_kernel("blur_1"), 1.0)
    den = O.OracleDenoiser(resolve_weights(str(g["arch"]), 3))
    xo, so, co, po, _, _ = O.test_iter(g["x_0"], g["x_obs"], g["x_true"], phi, adj, 0.5, g2, as_, an, 1.0, int(m1),
                                       int(m2), gadmm, sig, sp, palpha, den, 4, method, 3, 1.0)
    np.testing.assert_allclose(psnr, po, atol=0.01)
    np.testing.assert_allclose(x, xo, atol=5e-3)
    np.testing.assert_allclose(s, so, atol=5e-3)


def test_bm3d_methods_raise():
    with pytest.raises(ValueError, match="bm3d"):
        run(load_golden("iter_cmp_A_pdstv.npz"), "A-PnPPDS-BM3D", 1)
