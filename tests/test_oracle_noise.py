"""CPU checks of the oracle's observation pipeline (main.py:49-64, utils/utils_noise.py)
against x_obs / x_0 that the reference's own noise functions produced (tests/golden)."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import pnp_oracle as O



@pytest.mark.parametrize("case", ["A_blur", "A_id", "A_rs", "A_gray", "B_blur", "C_rs", "C_blur", "ADMM_B2"])
def test_observation_pipeline_matches_reference(case):
    """main.py:49-64 restated (oracle.make_observation) vs x_obs / x_0 produced by the
    reference's own utils_noise.py.  Id / random_sampling: bit-identical.  Blur: the golden's
    FFT ran in float32 (numpy 2 keeps single precision in np.fft; the reference pins numpy
    1.25, which promotes), so only the blur's rounding differs."""
    from pnppds.operators import load_blur_kernel
    g = load_golden(f"iter_{case}.npz")
    g1, g2, as_, an, lam, m1, m2, gad, sig, sp, pa, it, ch, r = g["params"]
    pois = str(g["method"]).startswith("C")
    obs, x0 = O.make_observation(g["x_true"], str(g["deg_op"]), load_blur_kernel("blur_1"), r, sig, sp, pois, pa)
    assert obs.dtype == g["x_obs"].dtype and obs.shape == g["x_obs"].shape
    if str(g["deg_op"]) == "blur" and not pois:
        np.testing.assert_allclose(obs, g["x_obs"], atol=5e-8, rtol=0)
        np.testing.assert_array_equal(obs == 0, g["x_obs"] == 0)
        np.testing.assert_array_equal(obs == 1, g["x_obs"] == 1)      # salt & pepper pixels
    else:
        np.testing.assert_array_equal(obs, g["x_obs"])
        np.testing.assert_array_equal(x0, g["x_0"])
