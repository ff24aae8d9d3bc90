"""Observation pipeline of main.py:49-64 (utils/utils_noise.py) on the device.

``make_observation`` is the reference's degradation sequence for one image ((C,H,W) RGB or
(H,W) gray) and ``make_observation_batch`` the same for a [B,C,H,W] batch:

    img_obsrv = phi(img_true)
    img_obsrv = add_gaussian_noise(img_obsrv, gaussian_nl, Id or phi)   # utils_noise.py:35-38
    img_obsrv = apply_poisson_noise(img_obsrv, poisson_alpha)           # if poisson_noise
    img_obsrv = add_salt_and_pepper_noise(img_obsrv, sp_nl, Id or phi)  # utils_noise.py:3-33
    x_0 = img_obsrv (/ poisson_alpha)

The noise is numpy's legacy ``np.random.seed(1234)`` stream, regenerated on the device
(libpnppds ``pnp_degrade``), so x_obs carries the reference's bit pattern: every image of a
batch gets the noise field the reference would give it, as main.py reseeds per image.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._device import get_ctx
from .operators import ObservationOperator, get_observation_operators

SEED = 1234   # utils_noise.py:6,36,41


def _params(gaussian_nl, sp_nl, poisson_noise, poisson_alpha, seed=SEED):
    return _lib.pnp_degrade_params(float(gaussian_nl), float(sp_nl), float(poisson_alpha),
                                   1 if poisson_noise else 0, int(seed))


def make_observation_batch(x_true, phi: ObservationOperator, gaussian_nl=0.01, sp_nl=0.0, poisson_noise=False,
                           poisson_alpha=300.0, ctx=None, float64=False, device_out=False):
    """x_true: [B,C,H,W] float32 (numpy or a device torch tensor).  Returns (x_obs, x_0):
    float32 arrays (the solver's state) or, with float64=True, x_obs in float64 as the
    reference hands it to test_iter.  device_out=True returns torch tensors on the device."""
    import torch
    if not isinstance(phi, ObservationOperator) or phi.adjoint:
        raise TypeError("phi must be the forward operator from pnppds.operators.get_observation_operators")
    ctx = ctx or get_ctx()
    dev = f"cuda:{ctx.device}"
    xt = x_true if isinstance(x_true, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x_true, np.float32))
    xt = xt.to(dev, torch.float32).contiguous()
    if xt.dim() != 4:
        raise ValueError("x_true must be [B, C, H, W]")
    B, C, H, W = xt.shape
    phi.configure(ctx, H, W)
    xobs = torch.empty((B, C, H, W), dtype=torch.float64 if float64 else torch.float32, device=dev)
    x0 = torch.empty((B, C, H, W), dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)
    ctx.degrade(_params(gaussian_nl, sp_nl, poisson_noise, poisson_alpha), xt.data_ptr(), B, C, H, W,
                xobs=None if float64 else xobs.data_ptr(), x0=x0.data_ptr(),
                xobs64=xobs.data_ptr() if float64 else None)
    if device_out:
        return xobs, x0
    return xobs.cpu().numpy(), x0.cpu().numpy()


def make_observation(img_true, deg_op="blur", path_kernel="blur_1", r=0.8, gaussian_nl=0.01, sp_nl=0.0,
                     poisson_noise=False, poisson_alpha=300.0):
    """main.py:49-64 for one image: returns (img_obsrv, x_0) with the reference's dtypes
    (float64; int64 counts under Poisson noise; x_0 float64)."""
    x = np.asarray(img_true, np.float32)
    x4 = x.reshape((1, 1) + x.shape) if x.ndim == 2 else x[None]
    phi, _ = get_observation_operators(deg_op, path_kernel, r)
    obs, _ = make_observation_batch(x4, phi, gaussian_nl, sp_nl, poisson_noise, poisson_alpha, float64=True)
    obs = obs.reshape(x.shape)
    if poisson_noise:
        obs = obs.astype(np.int64)                     # np.random.poisson returns int64
        return obs, obs / poisson_alpha
    return obs, np.copy(obs)
