"""Diagnostic (profiling only): where conv_body_f2's waves spend a step, from the s_memtime
stamps of a -DF2_STAMPS build (abl_libs/<name>.so via PNP_LIB_PATH).

    SRCF=conv bash tools/build_ab.sh f2_stamps -DF2_STAMPS
    PNP_LIB_PATH=$PWD/abl_libs/f2_stamps.so python tools/f2_stamps.py [--batch 256]

Per wave role (layer l = waves 0-1, layer l+1 = waves 2-3): mean cycles per step of setup,
MFMA stream, last group's epilogue, DMA wait and barrier wait, over the last launch's
workgroups.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pnp-pds_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from pnppds import _lib
    from pnppds.weights import resolve_weights
    from bench import synthetic_batch
    ctx = _lib.Context(0)
    ctx.set_denoiser(resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3))
    ctx.set_body_layers(2)
    B, C, H, W = a.batch, 3, 256, 256
    x = torch.from_numpy(synthetic_batch(B, C, H, W, seed=1)).cuda()
    y = torch.empty_like(x)
    for _ in range(a.reps):
        ctx.op_denoise(x.data_ptr(), y.data_ptr(), B, C, H, W)
    ctx.synchronize()
    n = 1024 * 4 * 8
    buf = (ctypes.c_ulonglong * n)()
    fn = ctx.lib.pnp_diag_f2_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    assert fn(buf, n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 4, 8).astype(np.float64)
    used = st[:, :, 5].sum(axis=1) > 0
    st = st[used]
    names = ["setup", "stream", "last epilogue", "DMA wait", "barrier wait"]
    for role, waves in (("layer l  ", [0, 1]), ("layer l+1", [2, 3])):
        s = st[:, waves, :].reshape(-1, 8)
        steps = s[:, 5]
        per = s[:, :5] / steps[:, None]
        tot = per.sum(axis=1).mean()
        print(f"{role}: {tot:8.0f} cycles/step  " +
              "  ".join(f"{nm} {per[:, i].mean():7.0f} ({100 * per[:, i].mean() / tot:4.1f}%)"
                        for i, nm in enumerate(names)))
    print(f"workgroups {used.sum()}, steps per workgroup {st[:, 0, 5].mean():.1f}")


if __name__ == "__main__":
    main()
