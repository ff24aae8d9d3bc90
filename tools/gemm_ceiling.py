"""Sustained fp16 MFMA rate of a library GEMM (torch.matmul -> hipBLASLt) on this box: the
practical ceiling the denoiser's conv kernels are compared against in DESIGN.md (the dense
2.5 PFLOP/s figure assumes the peak clock, which a long MFMA-bound run does not hold)."""
import json
import sys
import time

import torch


def rate(m, n, k, iters):
    a = torch.randn(m, k, device="cuda", dtype=torch.float16)
    b = torch.randn(k, n, device="cuda", dtype=torch.float16)
    for _ in range(3):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.matmul(a, b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return 2.0 * m * n * k / (ms * 1e-3) / 1e12, ms


def main():
    out = {}
    for (m, n, k, it) in [(8192, 8192, 8192, 50), (16384, 16384, 8192, 20), (4096, 65536, 576, 200)]:
        t0 = time.time()
        tf, ms = rate(m, n, k, it)
        out[f"{m}x{n}x{k}"] = {"tflops": round(tf, 1), "ms": round(ms, 3), "wall_s": round(time.time() - t0, 1)}
        print(json.dumps(out), flush=True)
    json.dump(out, sys.stdout)


if __name__ == "__main__":
    main()
