"""pnppds — MI355X-native PnP-PDS inner loop (drop-in for yodai49/PnP-PDS's solver path).

Public surface mirrors the reference:
  iteration.test_iter            (iteration.py:10)       -> pnppds.test_iter / test_iter_batch
  operators.get_observation_operators, proj_l2_ball, proj_l1_ball, prox_GKL (operators.py)
  models.denoiser.Denoiser       (models/denoiser.py:9)  -> pnppds.Denoiser
All compute runs in libpnppds.so (HIP, gfx950); see include/pnppds.h for the C ABI.
"""
from .weights import DenoiserWeights, resolve_weights, random_weights  # noqa: F401


def __getattr__(name):
    # Lazy: importing the package must not need the GPU library (CPU tests, build()).
    if name in ("test_iter", "test_iter_batch"):
        from . import iteration
        return getattr(iteration, name)
    if name in ("get_observation_operators", "proj_l2_ball", "proj_l1_ball", "prox_GKL"):
        from . import operators
        return getattr(operators, name)
    if name == "Denoiser":
        from .denoiser import Denoiser
        return Denoiser
    raise AttributeError(name)
