"""Benchmark: PnP-PDS iterations/s on batch=256 RGB 256x256 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--size S]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

A "step" is one PnP-PDS iteration (iteration.py:48-52, ours-A with the blur operator,
blur_1.mat, sigma=0.01, real DnCNN_nobn_nch_3_nlev_0.01 weights) over a batch of 256
synthetic RGB 256x256 images per GPU, inputs resident in HBM.  Images are independent, so
ranks process disjoint shards with no data-path collective (weak scaling: 256 images per
GPU).  ``value`` = image-iterations/s over the whole job (sum over ranks / max rank time).

Also reported: ``roofline`` of the dominant kernel (conv_body: 288 FLOP/B, below the
2500/8 = 312 FLOP/B ridge, so HBM-bound: algorithmic bytes / HIP-event duration vs 8 TB/s,
with the MFMA fraction alongside and ``traffic`` = PMC-measured bytes per launch from this
round's committed profile), HBM fractions of the fused
prox/operator kernels, PSNR delta vs the CPU oracle on image 0, and ``cpu_baseline``: the
oracle restatement of the reference's test_iter timed on this host (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "pnp-pds_amd"))
sys.path.insert(0, REPO)

METRIC = "PDS iters/sec, batch=256 RGB 256×256, 1/2/4/8 GPU; PSNR Δ vs ref"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP16_PEAK_TFLOPS = 2500.0      # dense fp16/bf16 MFMA (spec, no sparsity)
ARCH = "DnCNN_nobn_nch_3_nlev_0.01"
GAMMA1 = GAMMA2 = 0.99         # main.py:144-147 / ideas/param_memo.py:7
ALPHA_N = 0.95
SIGMA = 0.01


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synthetic_batch(B, C, H, W, seed):
    """Structured synthetic images in [0,1] (gradients, sinusoids, rectangles), float32."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.linspace(0, 1, H, dtype=np.float32), np.linspace(0, 1, W, dtype=np.float32),
                         indexing="ij")
    out = np.empty((B, C, H, W), np.float32)
    for b in range(B):
        f = rng.uniform(1, 6, (C, 2)).astype(np.float32)
        ph = rng.uniform(0, 6.28, C).astype(np.float32)
        for c in range(C):
            img = 0.45 + 0.25 * np.sin(2 * np.pi * f[c, 0] * xx + ph[c]) * np.cos(2 * np.pi * f[c, 1] * yy) \
                + 0.2 * (xx - 0.5)
            for _ in range(3):
                y0, x0 = rng.integers(0, H - H // 4), rng.integers(0, W - W // 4)
                img[y0:y0 + rng.integers(4, H // 4), x0:x0 + rng.integers(4, W // 4)] += rng.uniform(-0.3, 0.3)
            out[b, c] = np.clip(img, 0, 1)
    return out


def images_per_launch(B, H, W, chunk):
    """Mirror of capi.hip denoise_chunk(): images per conv launch."""
    if chunk > 0:
        return min(chunk, B)
    per_img = 2.0 * (H + 2) * (W + 2) * 64 * 2
    return max(1, min(int(8e9 // per_img), B))


def conv_flops_per_launch(m, H, W):
    """Algorithmic FLOPs of one 64->64 3x3 conv launch over m images."""
    return 2.0 * 64 * 64 * 9 * m * H * W


def conv_bytes_per_launch(m, H, W):
    """Algorithmic HBM bytes of one 64->64 conv launch over m images: read and write the
    fp16 64-channel activations once (the zero border, halo re-reads and weights are not
    algorithmic)."""
    return 2 * m * H * W * 64 * 2


TRAFFIC_JSON = "profiles/r01/bench/traffic.json"


def measured_traffic(kernel, B):
    """HBM bytes per launch from this round's committed PMC passes of this bench command
    (tools/profile_bench.sh + tools/traffic_from_pmc.py), or None."""
    try:
        with open(os.path.join(REPO, TRAFFIC_JSON)) as f:
            t = json.load(f)
        return t["kernels"][kernel]["bytes"] if B == 256 else None
    except (OSError, KeyError, ValueError):
        return None


def prox_bytes(B, C, H, W):
    """Algorithmic HBM bytes per launch of the fused ours-A passes."""
    n = B * C * H * W
    npx = B * H * W
    return {
        "k1_primal_pre": 4 * n * 3 + 8 * npx,      # read x, y; write u32; write u16 (8 B/pixel)
        "k2_dual": 4 * n * 6,                      # read x+, x, y, xobs, xtrue; write v
        "k3_dual": 4 * n * 3,                      # read v, xobs; write y
    }


def cpu_baseline(x_true, x_obs, h, budget_s, max_iter):
    """Oracle restatement of test_iter (numpy FFT + torch-CPU conv, all host cores) on image 0."""
    import torch
    from oracle import pnp_oracle as O
    from pnppds.weights import resolve_weights
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1))
    den = O.OracleDenoiser(resolve_weights(ARCH, 3))
    phi, adj = O.observation_operators("blur", h)
    xo = x_obs.astype(np.float64)
    O.test_iter(xo, xo, x_true, phi, adj, GAMMA1, GAMMA2, 1.0, ALPHA_N, 1.0, 15, 15, 0.1, SIGMA, 0.0, 300, den, 1,
                "A-Proposed", 3, 0.8)                                            # warm-up
    t = time.perf_counter()                                                      # size the sample
    O.test_iter(xo, xo, x_true, phi, adj, GAMMA1, GAMMA2, 1.0, ALPHA_N, 1.0, 15, 15, 0.1, SIGMA, 0.0, 300, den, 2,
                "A-Proposed", 3, 0.8)
    per = (time.perf_counter() - t) / 2
    n_total = int(min(max_iter, max(2, budget_s / per)))
    t = time.perf_counter()
    res = O.test_iter(xo, xo, x_true, phi, adj, GAMMA1, GAMMA2, 1.0, ALPHA_N, 1.0, 15, 15, 0.1, SIGMA, 0.0, 300,
                      den, n_total, "A-Proposed", 3, 0.8)
    el = time.perf_counter() - t
    return n_total / el, n_total, res[3], torch.get_num_threads()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile", type=int, default=1, help="HIP-event per-kernel timing in the timed region")
    ap.add_argument("--chunk", type=int, default=0, help="images per denoiser pass (0 = auto)")
    ap.add_argument("--chunk-sweep", type=str, default="", help="e.g. 4,8,16,256: time each (stderr)")
    ap.add_argument("--variant", type=int, default=0, help="body layers per launch: 0 = one (default), 1 = two fused")
    ap.add_argument("--variant-sweep", type=str, default="", help="e.g. 0,1: interleaved A/B (stderr)")
    ap.add_argument("--op", default="blur", choices=["blur", "Id", "random_sampling"],
                    help="degradation operator (the metric's is blur; the others time the elementwise K1/K2)")
    ap.add_argument("--ablate", type=int, default=0, help="profiling only (results wrong): 1 DMA, 2 stores, 4 MFMA")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # Rehearsal of the N-rank path on fewer GPUs (never used by the driver): PNP_BENCH_REHEARSAL=1
    # maps ranks onto the visible devices round-robin and does the barrier / max over gloo.
    rehearsal = os.environ.get("PNP_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local %= torch.cuda.device_count()
    backend = "gloo" if rehearsal else "nccl"
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend, init_method="env://")
    from pnppds import _lib
    from pnppds.iteration import make_params
    from pnppds.operators import load_blur_kernel
    from pnppds.shard import max_over_ranks
    from pnppds.weights import resolve_weights

    B, C, H, W = args.batch, 3, args.size, args.size
    K, Wm = args.steps, args.warmup
    ctx = _lib.Context(local)
    ctx.set_denoiser(resolve_weights(ARCH, 3))
    h = load_blur_kernel("blur_1")
    if args.op == "blur":
        ctx.set_operator(_lib.OP_BLUR, h=h)
    elif args.op == "Id":
        ctx.set_operator(_lib.OP_ID)
    else:
        from pnppds.operators import sampling_keep_mask
        ctx.set_operator(_lib.OP_RANDOM_SAMPLING, mask=sampling_keep_mask(H, W, 0.8))

    # ---- synthetic inputs, degraded on the device exactly as main.py:49-64 does ---------------
    t0 = time.perf_counter()
    x_true = synthetic_batch(B, C, H, W, seed=1000 * rank + 1)
    d_true = torch.from_numpy(x_true).cuda(local)
    d_obs = torch.empty_like(d_true)
    ctx.degrade(_lib.pnp_degrade_params(SIGMA, 0.0, 300.0, 0, 1234), d_true.data_ptr(), B, C, H, W,
                xobs=d_obs.data_ptr())           # blur_1 + 0.01 * np.random.seed(1234) randn
    torch.cuda.synchronize()
    log(f"[rank {rank}] inputs ready in {time.perf_counter() - t0:.1f}s")

    cap = Wm + K
    prm = make_params(GAMMA1, GAMMA2, 1.0, ALPHA_N, 1.0, 15, 15, 0.1, SIGMA, 0.0, 300, 0.8, True)
    ctx.set_denoise_chunk(args.chunk)
    ctx.solver_setup(_lib.METHOD_A, prm, B, C, H, W, cap)
    ctx.solver_load_device(d_obs.data_ptr(), d_obs.data_ptr(), d_true.data_ptr())   # x_0 = x_obs (main.py:62)
    ctx.solver_iterate(Wm)
    ctx.synchronize()
    torch.cuda.synchronize()
    for ch in [int(v) for v in args.chunk_sweep.split(",") if v]:
        ctx.set_denoise_chunk(ch)
        ctx.solver_iterate(1)
        ctx.synchronize()
        ts = time.perf_counter()
        ctx.solver_iterate(3)
        ctx.synchronize()
        log(f"[sweep] chunk={ch}: {(time.perf_counter() - ts) / 3 * 1e3:.2f} ms/iter")
    vs = [int(v) for v in args.variant_sweep.split(",") if v]
    if vs:
        res = {v: [] for v in vs}
        for _ in range(3):                     # interleaved rounds in one process
            for v in vs:
                ctx.set_body_variant(v)
                ctx.solver_iterate(1)
                ctx.synchronize()
                ts = time.perf_counter()
                ctx.solver_iterate(2)
                ctx.synchronize()
                res[v].append((time.perf_counter() - ts) / 2 * 1e3)
        for v in vs:
            log(f"[variant] {v}: ms/iter median {sorted(res[v])[1]:.2f} min {min(res[v]):.2f}")
    ctx.set_body_variant(args.variant)
    if args.ablate:
        ctx.set_ablate(args.ablate)
    if args.chunk_sweep or vs:                 # restart the trajectory after the sweep
        ctx.set_denoise_chunk(args.chunk)
        ctx.solver_load_device(d_obs.data_ptr(), d_obs.data_ptr(), d_true.data_ptr())
        ctx.solver_iterate(Wm)
        ctx.synchronize()

    # ---- timed region ------------------------------------------------------------------------
    if args.profile:
        ctx.profile_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    ctx.solver_iterate(K)
    ctx.synchronize()
    torch.cuda.synchronize()
    t_el = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
        t_el = max_over_ranks(t_el, device=None if rehearsal else f"cuda:{local}")   # job time = slowest rank
    prof = ctx.profile_read() if args.profile else {}
    x_out, s_out, c_hist, psnr_hist, ssim_hist = ctx.solver_fetch()

    value = B * world * K / t_el
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "image-iterations/s",
            "n_gpus": world, "steps": K, "warmup": Wm,
            "ms_per_step": round(1e3 * t_el / K, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp16-mfma/fp32-acc+state",
            "data": "synthetic structured RGB images, x_obs = blur_1(x_true) + 0.01 randn of np.random.seed(1234) "
                    "(main.py:49-64, generated on device); real "
                    "DnCNN_nobn_nch_3_nlev_0.01 weights",
            "config": {"workload": f"ours-A (A-Proposed) blur, batch={B}/GPU RGB {H}x{W}", "global_batch": B * world,
                       "image": f"{C}x{H}x{W}", "deg_op": "blur_1" if args.op == "blur" else args.op,
                       "method": "ours-A",
                       "parallelism": f"dp{world} (independent image shards, no collective)"},
            "batch_iters_per_s": round(K / t_el, 3),
        }
        if prof:
            kt = {k: round(v[0], 4) for k, v in prof.items()}
            line["kernel_ms"] = kt
            fused = "conv_body2" in prof          # two 64->64 layers per launch (intermediate in LDS)
            kname = "conv_body2" if fused else "conv_body"
            body_ms = prof[kname][0]
            m = images_per_launch(B, H, W, args.chunk)
            nl = 2 if fused else 1
            fl = nl * conv_flops_per_launch(m, H, W)
            by = conv_bytes_per_launch(m, H, W)    # read + write the fp16 activations once per launch
            gbs = by / (body_ms * 1e-3) / 1e9
            tfl = fl / (body_ms * 1e-3) / 1e12
            # per launch: 288 FLOP/B (one layer, below the 312 FLOP/B ridge: HBM roof) or 576 FLOP/B
            # (two fused layers, above it: MFMA roof)
            if fused:
                line["roofline"] = {"kernel": "conv_body2 (two fused 64->64 3x3 layers, fp16 MFMA)", "bound": "mfma",
                                    "achieved": round(tfl, 1), "peak": FP16_PEAK_TFLOPS, "unit": "TFLOP/s",
                                    "frac": round(tfl / FP16_PEAK_TFLOPS, 4),
                                    "traffic": measured_traffic(kname, B), "bytes_per_launch": by,
                                    "flops_per_launch": fl, "hbm_gbs": round(gbs, 1),
                                    "hbm_frac": round(gbs / HBM_PEAK_GBS, 4), "traffic_source": TRAFFIC_JSON}
            else:
                line["roofline"] = {"kernel": "conv_body (64->64 3x3 implicit GEMM, fp16 MFMA)", "bound": "hbm",
                                    "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": measured_traffic(kname, B),
                                    "bytes_per_launch": by, "flops_per_launch": fl,
                                    "mfma_tflops": round(tfl, 1), "mfma_frac": round(tfl / FP16_PEAK_TFLOPS, 4),
                                    "traffic_source": TRAFFIC_JSON}
            pb = prox_bytes(B, C, H, W)
            line["prox_hbm"] = {k: {"GB/s": round(pb[k] / (prof[k][0] * 1e-3) / 1e9, 1),
                                    "frac": round(pb[k] / (prof[k][0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                                for k in pb if k in prof}
        line["psnr_img0_db"] = [round(float(psnr_hist[0, 0]), 4), round(float(psnr_hist[0, cap - 1]), 4)]
        line["ssim_img0"] = [round(float(ssim_hist[0, 0]), 5), round(float(ssim_hist[0, cap - 1]), 5)]
        if world == 1 and not args.no_cpu_baseline and args.op == "blur":
            rate, n_cpu, ps_cpu, thr = cpu_baseline(x_true[0], d_obs[0].cpu().numpy(), h, args.cpu_budget, cap)
            line["cpu_baseline"] = {"value": round(rate, 3), "unit": "image-iterations/s", "cores": thr,
                                    "kind": "port",
                                    "sample": f"oracle test_iter (numpy FFT blur + torch-CPU conv), image 0, "
                                              f"{n_cpu} iterations after 1 warm-up"}
            line["psnr_delta_db_vs_oracle"] = round(float(np.max(np.abs(ps_cpu - psnr_hist[0, :n_cpu]))), 5)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
