"""CPU checks of the oracle's SSIM (utils/utils_eval.py:9-12 -> skimage 0.22 structural_similarity).

PARITY UNPINNED: scikit-image is not installed here and the reference's golden outputs hold no
SSIM values, so the restatement is checked against an independent direct-window computation of
the published formula (Wang et al. 2004 with skimage's defaults) and against its invariants.
"""
import numpy as np
import pytest

from oracle import pnp_oracle as O


def _direct_ssim_2d(a, b, R):
    """Direct per-window statistics (float64), window 7x7, sample covariance, crop 3."""
    H, W = a.shape
    C1, C2 = (0.01 * R) ** 2, (0.03 * R) ** 2
    vals = []
    for i in range(3, H - 3):
        for j in range(3, W - 3):
            x = a[i - 3:i + 4, j - 3:j + 4].astype(np.float64).ravel()
            y = b[i - 3:i + 4, j - 3:j + 4].astype(np.float64).ravel()
            ux, uy = x.mean(), y.mean()
            vx, vy = x.var(ddof=1), y.var(ddof=1)
            vxy = ((x - ux) * (y - uy)).sum() / (x.size - 1)
            vals.append((2 * ux * uy + C1) * (2 * vxy + C2) / ((ux * ux + uy * uy + C1) * (vx + vy + C2)))
    return float(np.mean(vals))


def _direct_ssim_1d(a, b, R):
    C1, C2 = (0.01 * R) ** 2, (0.03 * R) ** 2
    vals = []
    for j in range(3, a.size - 3):
        x, y = a[j - 3:j + 4].astype(np.float64), b[j - 3:j + 4].astype(np.float64)
        ux, uy = x.mean(), y.mean()
        vx, vy = x.var(ddof=1), y.var(ddof=1)
        vxy = ((x - ux) * (y - uy)).sum() / 6
        vals.append((2 * ux * uy + C1) * (2 * vxy + C2) / ((ux * ux + uy * uy + C1) * (vx + vy + C2)))
    return float(np.mean(vals))


def _pair(shape, seed):
    rng = np.random.default_rng(seed)
    a = rng.uniform(0, 1, shape).astype(np.float32)
    b = np.clip(a + 0.08 * rng.standard_normal(shape), 0, 1).astype(np.float32)
    return a, b


def test_rgb_matches_direct_windows():
    a, b = _pair((3, 20, 23), 0)
    R = float(b.max() - b.min())
    want = np.mean([_direct_ssim_2d(a[c], b[c], R) for c in range(3)])
    assert abs(O.ssim(a, b) - want) < 2e-5


def test_gray_is_mean_of_row_ssims():
    """channel_axis=0 on an (H, W) array: skimage iterates over rows."""
    a, b = _pair((9, 31), 1)
    R = float(b.max() - b.min())
    want = np.mean([_direct_ssim_1d(a[i], b[i], R) for i in range(9)])
    assert abs(O.ssim(a, b) - want) < 2e-5


def test_identity_and_range():
    a, b = _pair((3, 32, 32), 2)
    assert O.ssim(a, a) == pytest.approx(1.0, abs=1e-6)
    v = O.ssim(a, b)
    assert -1.0 <= v < 1.0
    # data_range comes from the second argument only (utils_eval.py:10)
    Rb = float(b.max() - b.min())
    want = np.mean([O._ssim_single(a[c], b[c], np.float32(Rb)) for c in range(3)])
    assert O.ssim(a, b) == pytest.approx(want, abs=1e-7)
