"""Diagnostic: the clock conv_body_x8 runs at (separate clock from cycles).  From
the X8_CLOCK build: per workgroup, shader-clock cycles (s_memtime) and 100 MHz ticks
(s_memrealtime) over the launch -> effective clock; for the metric's batch (256 x RGB 256^2,
two body layers per launch) with the real weights on structured inputs, and with random
weights on uniform-random inputs (more bit toggling per MFMA).
    PNP_LIB_PATH=abl_libs/x8_clock.so python tools/x8_clock.py"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pnp-pds_amd")]
import torch  # noqa: E402
from pnppds import _lib  # noqa: E402
from pnppds.weights import random_weights, resolve_weights  # noqa: E402
import bench  # noqa: E402

ctx = _lib.Context(0)
ctx.set_precision("fp16")
ctx.set_body_layers(2)
B = 256
xs = torch.from_numpy(bench.synthetic_batch(B, 3, 256, 256, seed=9)).cuda()
xr = torch.rand(B, 3, 256, 256, device="cuda")
y = torch.empty_like(xs)
for label, w, x in (("real weights, structured images", resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3), xs),
                    ("random weights, uniform inputs", random_weights(3, depth=20, seed=1, scale=1.0), xr)):
    ctx.set_denoiser(w)
    for _ in range(3):
        ctx.op_denoise(x.data_ptr(), y.data_ptr(), B, 3, 256, 256)
    ctx.synchronize()
    ctx.op_denoise(x.data_ptr(), y.data_ptr(), B, 3, 256, 256)
    ctx.synchronize()
    buf = (C.c_ulonglong * 2048)()
    assert ctx.lib.pnp_diag_x8_clock(buf, C.c_size_t(2048)) == 0
    a = np.frombuffer(buf, np.uint64).reshape(1024, 2)[:256].astype(np.float64)   # the last launch (layers 17-18)
    ghz = a[:, 0] / (a[:, 1] * 10.0)
    print(f"{label}: conv_body_x8 effective clock median {np.median(ghz):.3f} GHz (min {ghz.min():.3f}, max "
          f"{ghz.max():.3f}); launch {np.median(a[:, 1]) / 1e5:.3f} ms by the real-time clock (median workgroup)",
          flush=True)
