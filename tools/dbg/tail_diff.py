"""Debug: locate denoiser output errors vs the fp16-emulating oracle (pattern by tile position)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "pnp-pds_amd")]
import torch
from pnppds import _lib
from pnppds.weights import DenoiserWeights, WEIGHTS_DIR
from oracle import pnp_oracle as O
w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, "DnCNN_nobn_nch_3_nlev_0.01.npz"))
ctx = _lib.Context(0)
ctx.set_denoiser(w)
rng = np.random.default_rng(0)
for (B, H, W) in [(1, 64, 64), (1, 8, 32), (2, 16, 64)]:
    x = rng.uniform(0, 1, (B, 3, H, W)).astype(np.float32)
    dx = torch.from_numpy(x).cuda(); dy = torch.empty_like(dx)
    ctx.op_denoise(dx.data_ptr(), dy.data_ptr(), B, 3, H, W); ctx.synchronize(); torch.cuda.synchronize()
    out = dy.cpu().numpy()
    emu = O.OracleDenoiser(w, emulate_fp16=True).forward_batch(x)
    d = np.abs(out - emu)
    print(B, H, W, "max", d.max())
    bad = np.argwhere(d > 3e-3)
    if len(bad):
        print(" nbad", len(bad), "first", bad[:8].tolist())
        print(" by channel", np.bincount(bad[:, 1], minlength=3), "row%8", np.bincount(bad[:, 2] % 8, minlength=8),
              "col%32", np.bincount(bad[:, 3] % 32, minlength=32))
