"""Observation operators and proximal operators — device-backed mirror of operators.py.

Same names, signatures and return dtypes as the reference (operators.py:7-137 for the
hot-path subset).  Every call executes on the MI355X through libpnppds.so; numpy arrays
are staged through device memory.  ``get_observation_operators`` returns callables that
also carry their description (``kind``, ``h``, ``r``) so that ``test_iter`` can run the
whole loop on the device instead of calling the closures.
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib
from ._device import from_device, get_ctx, to_device

_WEIGHTS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "weights")


def load_blur_kernel(path_kernel: str) -> np.ndarray:
    """blur_models/*.mat ('blur' variable, operators.py:77-78).  Falls back to the npy copy
    shipped in pnp-pds_amd/weights when the .mat is not present (e.g. on the GPU box)."""
    if path_kernel and os.path.exists(path_kernel) and path_kernel.endswith(".mat"):
        import scipy.io
        return np.asarray(scipy.io.loadmat(path_kernel)["blur"], np.float64)
    stem = os.path.splitext(os.path.basename(path_kernel or "blur_1"))[0] or "blur_1"
    npy = os.path.join(_WEIGHTS, stem + ".npy")
    if not os.path.exists(npy):
        raise FileNotFoundError(f"blur kernel {path_kernel!r} not found (looked for {npy})")
    return np.load(npy, allow_pickle=False)


def sampling_keep_mask(H: int, W: int, r: float) -> np.ndarray:
    """operators.py:40-58: drop round(H*W*(1-r)) pixels chosen by RandomState(1234)."""
    cnt = round(H * W * (1 - r))
    q = np.random.RandomState(seed=1234).permutation(H * W)[:cnt]
    m = np.ones(H * W, np.uint8)
    m[q] = 0
    return m.reshape(H, W)


class ObservationOperator:
    """Φ or Φᵀ of operators.py:60-79, executed on the device."""

    def __init__(self, kind: str, h: np.ndarray | None, r: float, adjoint: bool):
        if kind not in ("blur", "random_sampling", "Id"):
            raise ValueError(f"unknown operator {kind!r}")
        self.kind, self.h, self.r, self.adjoint = kind, h, r, adjoint

    @property
    def code(self) -> int:
        return {"Id": _lib.OP_ID, "blur": _lib.OP_BLUR, "random_sampling": _lib.OP_RANDOM_SAMPLING}[self.kind]

    def configure(self, ctx, H: int, W: int):
        if self.kind == "blur":
            ctx.set_operator(_lib.OP_BLUR, h=self.h, key=("blur", self.h.tobytes()))
        elif self.kind == "random_sampling":
            ctx.set_operator(_lib.OP_RANDOM_SAMPLING, mask=sampling_keep_mask(H, W, self.r),
                             key=("rs", H, W, self.r))
        else:
            ctx.set_operator(_lib.OP_ID, key=("id",))

    def __call__(self, x):
        if self.kind == "Id":                  # operators.py:66-67: returns x itself
            return x
        x = np.asarray(x)
        shp = x.shape
        x4 = x.reshape((1, 1) + shp) if x.ndim == 2 else x.reshape((1,) + shp)
        _, Cc, H, W = x4.shape
        ctx = get_ctx()
        self.configure(ctx, H, W)
        dx = to_device(x4)
        dy = to_device(np.empty_like(x4, dtype=np.float32))
        ctx.op_phi(dx.data_ptr(), dy.data_ptr(), 1, Cc, H, W, adj=self.adjoint)
        return from_device(dy, ctx).astype(np.float64).reshape(shp)

    def __repr__(self):
        return f"ObservationOperator({self.kind!r}, adjoint={self.adjoint}, r={self.r})"


def get_observation_operators(operator, path_kernel, r):
    """operators.py:60-79 — returns (phi, adj_phi)."""
    h = load_blur_kernel(path_kernel) if operator == "blur" else None
    return ObservationOperator(operator, h, r, False), ObservationOperator(operator, h, r, True)


def _batched(x):
    x = np.asarray(x)
    return x.reshape(1, -1), x.shape


def proj_l2_ball(x, alpha_n, gaussian_nl, sp_nl, x_0, r=1):
    """operators.py:102-108 on the device."""
    xb, shp = _batched(x)
    ctx = get_ctx()
    dx, d0 = to_device(xb), to_device(np.broadcast_to(np.asarray(x_0), shp).reshape(1, -1))
    out = to_device(np.empty_like(xb, dtype=np.float32))
    ctx.op_proj_l2_ball(dx.data_ptr(), d0.data_ptr(), out.data_ptr(), 1, xb.size, alpha_n, gaussian_nl, sp_nl, r)
    return from_device(out, ctx).astype(np.float64).reshape(shp)


def proj_l1_ball(x, alpha_s, sp_nl, r=1):
    """operators.py:94-100 on the device (radix-select threshold, see ops.hip)."""
    xb, shp = _batched(x)
    ctx = get_ctx()
    dx = to_device(xb)
    out = to_device(np.empty_like(xb, dtype=np.float32))
    ctx.op_proj_l1_ball(dx.data_ptr(), out.data_ptr(), 1, xb.size, alpha_s, sp_nl, r)
    return from_device(out, ctx).astype(np.float64).reshape(shp)


def prox_GKL(x, gamma, alpha, x_0):
    """operators.py:114-115 on the device."""
    xb, shp = _batched(x)
    ctx = get_ctx()
    dx, d0 = to_device(xb), to_device(np.broadcast_to(np.asarray(x_0), shp).reshape(1, -1))
    out = to_device(np.empty_like(xb, dtype=np.float32))
    ctx.op_prox_gkl(dx.data_ptr(), d0.data_ptr(), out.data_ptr(), xb.size, gamma, alpha)
    return from_device(out, ctx).astype(np.float64).reshape(shp)


def denoise(x, path_prox, ch):
    """operators.py:81-83."""
    from .denoiser import Denoiser
    return Denoiser(path_prox, ch).denoise(x)


def grad_x_l2(x, s, phi, adj_phi, x_0):
    """operators.py:88-89."""
    return 2 * adj_phi(phi(x) + s - x_0)


def grad_s_l2(x, s, phi, x_0):
    """operators.py:91-92."""
    return phi(x) + s - x_0
