"""A/B timing of denoiser body variants in one process (profiling only).

    python3 tools/ab_body.py --variants 0,2 [--batch 256] [--rounds 5]

Runs pnp_op_denoise on the bench's image batch, alternating the variants round by round,
and prints the median HIP-event time per conv kernel for each variant.
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pnp-pds_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--ablates", default="", help="raw PNP_TUNE_ABLATE codes instead of variants (profiling)")
    ap.add_argument("--chunks", default="", help="denoiser images per pass instead of variants (totals per pass)")
    a = ap.parse_args()
    import torch
    from bench import synthetic_batch
    from pnppds import _lib
    from pnppds.weights import resolve_weights
    ctx = _lib.Context(0)
    ctx.set_denoiser(resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3))
    B, C, H, W = a.batch, 3, a.size, a.size
    x = torch.from_numpy(synthetic_batch(B, C, H, W, seed=1)).cuda()
    y = torch.empty_like(x)
    vs = [int(v) for v in (a.chunks or a.ablates or a.variants).split(",")]
    setv = ctx.set_denoise_chunk if a.chunks else ctx.set_ablate if a.ablates else ctx.set_body_variant
    res = {v: {} for v in vs}
    for v in vs:                                   # warm-up
        setv(v)
        ctx.op_denoise(x.data_ptr(), y.data_ptr(), B, C, H, W)
    ctx.synchronize()
    for _ in range(a.rounds):
        for v in vs:
            setv(v)
            ctx.profile_enable(True)
            ctx.op_denoise(x.data_ptr(), y.data_ptr(), B, C, H, W)
            ctx.synchronize()
            for k, (ms, n) in ctx.profile_read().items():
                res[v].setdefault(k, []).append(ms * n if a.chunks else ms)
            ctx.profile_enable(False)
    for v in vs:
        print(f"variant {v}: " + "  ".join(f"{k} {statistics.median(t):.4f}" for k, t in sorted(res[v].items())),
              flush=True)


if __name__ == "__main__":
    main()
