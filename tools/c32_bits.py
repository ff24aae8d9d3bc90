"""Denoiser output of the fp32-operand path for a fixed batch (A/B bit-identity helper, profiling only)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pnp-pds_amd"))
from pnppds import _lib  # noqa: E402
from pnppds.weights import resolve_weights  # noqa: E402

ctx = _lib.Context(0)
ctx.set_precision("fp32")
ctx.set_denoiser(resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3))
rng = np.random.default_rng(5)
x = rng.random((4, 3, 96, 80)).astype(np.float32)
dx = torch.from_numpy(x).cuda()
dy = torch.empty_like(dx)
ctx.op_denoise(dx.data_ptr(), dy.data_ptr(), *x.shape)
torch.cuda.synchronize()
ctx.synchronize()
np.savez(sys.argv[1], y=dy.cpu().numpy())
