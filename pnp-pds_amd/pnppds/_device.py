"""Device-memory plumbing for the numpy-facing API (torch-ROCm tensors as buffers only).

All arithmetic happens in libpnppds.so; torch is used here purely to allocate HBM and
copy host<->device, on the same HIP runtime the library uses.
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib

_ctx = None


def current_device() -> int:
    return int(os.environ.get("LOCAL_RANK", "0")) if os.environ.get("PNPPDS_DEVICE") is None \
        else int(os.environ["PNPPDS_DEVICE"])


def get_ctx():
    global _ctx
    if _ctx is None:
        _ctx = _lib.get_context(current_device())
    return _ctx


def to_device(a: np.ndarray):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
    return t.to(f"cuda:{get_ctx().device}")


def from_device(t, ctx=None) -> np.ndarray:
    import torch
    torch.cuda.synchronize(t.device)
    (ctx or get_ctx()).synchronize()
    return t.cpu().numpy()
