"""Profiling driver: the denoiser alone (pnp_op_denoise) on a batch of RGB images.

    rocprofv3 --kernel-trace --stats -- python3 tools/prof_denoise.py [--batch 64] [--reps 3]
    rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... -- python3 tools/prof_denoise.py
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pnp-pds_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--height", type=int, default=0, help="image height (0 = --size)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--random", action="store_true", help="uniform-random input instead of structured images")
    ap.add_argument("--ablate", type=int, default=0,
                    help="profiling build only (PNP_LIB_PATH=.../lib_prof/libpnppds.so): 1 DMA, 2 stores, 4 MFMA skipped")
    ap.add_argument("--precision", default="fp16", choices=["fp16", "fp32", "fp16w2", "fp16x3", "fp16a2"])
    ap.add_argument("--body-layers", type=int, default=0)
    ap.add_argument("--fuse-ends", type=int, default=1, help="0: separate head / tail launches")
    a = ap.parse_args()
    import torch
    from pnppds import _lib
    from pnppds.weights import resolve_weights
    ctx = _lib.Context(0)
    ctx.set_denoiser(resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3))
    ctx.set_denoise_chunk(a.chunk)
    ctx.set_precision(a.precision)
    if a.ablate:
        ctx.set_ablate(a.ablate)
    if a.body_layers:
        ctx.set_body_layers(a.body_layers)
    ctx.set_fuse_ends(a.fuse_ends)
    B, C, H, W = a.batch, 3, a.height or a.size, a.size
    if a.random:
        x = torch.rand((B, C, H, W), device="cuda:0")
    else:                                   # the bench's structured synthetic images (denoiser input range)
        sys.path.insert(0, REPO)
        from bench import synthetic_batch
        x = torch.from_numpy(synthetic_batch(B, C, H, W, seed=1)).cuda()
    y = torch.empty_like(x)
    for _ in range(a.reps):
        ctx.op_denoise(x.data_ptr(), y.data_ptr(), B, C, H, W)
    ctx.synchronize()
    torch.cuda.synchronize()
    print("done", float(y.mean()))


if __name__ == "__main__":
    main()
