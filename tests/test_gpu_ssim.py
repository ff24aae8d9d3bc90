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
