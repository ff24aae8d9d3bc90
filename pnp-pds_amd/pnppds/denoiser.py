"""Denoiser — device-backed mirror of models/denoiser.py.

``Denoiser(file_name, ch).denoise(x)`` as in the reference (denoiser.py:9-16): x is (C,H,W)
for RGB or (H,W) for gray, float; output float32 of the same shape, clamped to [0,1] on the
way in and out (denoiser.py:40,42).  Weights come from the converted npz matching the
reference checkpoint name (pnppds.weights.resolve_weights); the forward runs as MFMA
implicit-GEMM kernels in libpnppds.so.
"""
from __future__ import annotations

import numpy as np

from ._device import from_device, get_ctx, to_device
from .weights import DenoiserWeights, resolve_weights


class Denoiser:
    def __init__(self, file_name, ch=3, weights: DenoiserWeights | None = None, precision="auto"):
        self.weights = weights if weights is not None else resolve_weights(file_name, ch)
        self.ch = ch
        # 'auto' (default): split fp16 for a single denoiser call (the reference's fp32 to ~2e-7);
        # 'fp16', 'fp16w2', 'fp16x3' or 'fp32' (Context.set_precision)
        self.precision = precision
        self.key = ("den", self.weights.name, file_name, id(weights) if weights is not None else 0)
        self.cost = 0

    def configure(self, ctx):
        ctx.set_denoiser(self.weights, key=self.key)

    def denoise_batch(self, x: np.ndarray) -> np.ndarray:
        """x: [B, C, H, W] -> [B, C, H, W] float32."""
        x = np.asarray(x)
        B, Cc, H, W = x.shape
        ctx = get_ctx()
        self.configure(ctx)
        prev = ctx.precision               # this call's precision only: the shared context keeps its own
        ctx.set_precision(self.precision)
        try:
            dx = to_device(x)
            dy = to_device(np.empty(x.shape, np.float32))
            ctx.op_denoise(dx.data_ptr(), dy.data_ptr(), B, Cc, H, W)
            ctx.op_status()
            return from_device(dy, ctx)
        finally:
            if prev != ctx.precision:
                ctx.set_precision(prev)

    def denoise(self, x):
        x = np.asarray(x)
        if x.ndim == 2:
            return self.denoise_batch(x[None, None])[0, 0]
        return self.denoise_batch(x[None])[0]
