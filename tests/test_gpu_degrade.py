"""GPU observation pipeline (pnp_degrade) vs x_obs of the reference's own
utils_noise.py (tests/golden) and vs the oracle restatement on further shapes.

Tolerances: Id / random_sampling observations are bit-identical in float32 (the solver's
state) and within 4 float64 ulps in float64 (the polar method's log is the device's, not
glibc's).  Poisson counts and salt-and-pepper pixels are exact integers.  Blur observations
differ from the golden by the golden's own float32 FFT (numpy 2, see test_oracle_noise.py)
and from the float64-FFT oracle by < 1e-12."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import pnp_oracle as O

pytestmark = pytest.mark.gpu
CASES = ["A_blur", "A_id", "A_rs", "A_gray", "B_blur", "C_rs", "C_blur", "ADMM_B2"]


def _device_obs(x_true, deg, r, sig, sp, pois, alpha, B=1):
    from pnppds.noise import make_observation_batch
    from pnppds.operators import get_observation_operators
    x = np.asarray(x_true, np.float32)
    x4 = x.reshape((1, 1) + x.shape) if x.ndim == 2 else x[None]
    x4 = np.repeat(x4, B, axis=0)
    phi, _ = get_observation_operators(deg, "blur_1", r)
    o64, x0 = make_observation_batch(x4, phi, sig, sp, pois, alpha, float64=True)
    o32, _ = make_observation_batch(x4, phi, sig, sp, pois, alpha)
    return o64.reshape((B,) + x.shape), o32.reshape((B,) + x.shape), x0.reshape((B,) + x.shape)


def _check(o64, o32, x0, want, want_x0, blur, pois, alpha):
    if pois:
        np.testing.assert_array_equal(o64, want)                       # integer counts, exact
        np.testing.assert_array_equal(x0, (want / alpha).astype(np.float32))
    elif blur:
        np.testing.assert_allclose(o64, want, atol=5e-8, rtol=0)
        np.testing.assert_array_equal(o64 == 0, want == 0)
        np.testing.assert_array_equal(o64 == 1, want == 1)
    else:
        np.testing.assert_allclose(o64, want, rtol=4 * np.finfo(np.float64).eps, atol=1e-300)
        np.testing.assert_array_equal(o32, want.astype(np.float32))
        np.testing.assert_array_equal(x0, want_x0.astype(np.float32))


@pytest.mark.parametrize("case", CASES)
def test_matches_reference_noise(case):
    g = load_golden(f"iter_{case}.npz")
    g1, g2, as_, an, lam, m1, m2, gad, sig, sp, pa, it, ch, r = g["params"]
    deg, pois = str(g["deg_op"]), str(g["method"]).startswith("C")
    o64, o32, x0 = _device_obs(g["x_true"], deg, r, sig, sp, pois, pa, B=2)
    for b in range(2):                                  # every image gets the reseeded noise field
        _check(o64[b], o32[b], x0[b], g["x_obs"], g["x_0"], deg == "blur", pois, pa)


def _img(shape, seed, lo=0.0, hi=1.0):
    rng = np.random.default_rng(seed)
    return rng.uniform(lo, hi, shape).astype(np.float32)


@pytest.mark.parametrize("shape,deg,sig,sp,pois", [
    ((64, 64), "random_sampling", 0.02, 0.1, False),      # gray RS: S&P target is the mask
    ((3, 48, 80), "Id", 0.01, 0.05, False),                # randint(0, 48): masked rejection draws
    ((3, 40, 40), "Id", 0.0, 0.0, True),                   # Poisson, lam across both regimes
    ((3, 64, 64), "random_sampling", 0.0, 0.2, True),      # Poisson then S&P
    ((3, 33, 47), "blur", 0.01, 0.1, False),               # blur on an odd, non-square image
    ((256, 256), "Id", 0.01, 0.1, False),                  # full-size gray
])
def test_matches_oracle(shape, deg, sig, sp, pois):
    from pnppds.operators import load_blur_kernel
    x = _img(shape, 5)
    if pois:
        x[..., : shape[-2] // 2, :] *= 0.02                # dark half: lam < 10 (multiplication method)
    want, want_x0 = O.make_observation(x, deg, load_blur_kernel("blur_1"), 0.8, sig, sp, pois, 300.0)
    o64, o32, x0 = _device_obs(x, deg, 0.8, sig, sp, pois, 300.0)
    if deg == "blur":
        np.testing.assert_allclose(o64[0], want, atol=1e-12, rtol=0)
    else:
        _check(o64[0], o32[0], x0[0], want, want_x0, False, pois, 300.0)


def test_full_size_batch_blur_poisson_sp():
    """3x256x256, blur + Poisson + S&P, batch 4 (the C-method input path at the metric's size)."""
    from pnppds.operators import load_blur_kernel
    xs = np.stack([_img((3, 256, 256), s) for s in range(4)])
    from pnppds.noise import make_observation_batch
    from pnppds.operators import get_observation_operators
    phi, _ = get_observation_operators("blur", "blur_1", 0.8)
    o64, x0 = make_observation_batch(xs, phi, 0.0, 0.05, True, 300.0, float64=True)
    for b in (0, 3):
        want, _ = O.make_observation(xs[b], "blur", load_blur_kernel("blur_1"), 0.8, 0.0, 0.05, True, 300.0)
        np.testing.assert_array_equal(o64[b], want)


def test_errors_mirror_numpy():
    from pnppds import _lib
    from pnppds.noise import make_observation_batch
    from pnppds.operators import get_observation_operators
    phi, _ = get_observation_operators("Id", "blur_1", 0.8)
    with pytest.raises(_lib.PnpError, match="lam < 0"):           # numpy: ValueError lam < 0
        make_observation_batch(-_img((1, 3, 16, 16), 1), phi, 0.0, 0.0, True, 300.0)
    with pytest.raises(_lib.PnpError, match="IndexError"):        # S&P columns drawn in [0, H), H > W
        make_observation_batch(_img((1, 3, 80, 48), 1), phi, 0.0, 0.1, False, 300.0)
