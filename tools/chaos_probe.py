"""How well-conditioned is a golden's trajectory?  The fp32 test oracle (torch-CPU conv stack)
run from the golden's x_0 and from x_0 moved by one float32 ulp at every pixel (random signs,
seed 0): max |dx| between the two final iterates and the max |dPSNR| over the run, beside the
same numbers against the reference's golden.  A trajectory whose own fp32 solves move pixels
by 1e-2 .. 1e-1 from a one-ulp start cannot be checked pixel-wise; its PSNR is the criterion
(tests/test_gpu_long.py CHAOTIC).  CPU only (profiling aid, round 4).

    python tools/chaos_probe.py CASE [CASE ...]        (CASE: a long_*.npz golden's name)
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pnp-pds_amd"), os.path.join(REPO, "tests")]
from oracle import pnp_oracle as O  # noqa: E402
from pnppds.operators import load_blur_kernel  # noqa: E402
from pnppds.weights import resolve_weights  # noqa: E402
from conftest import load_golden  # noqa: E402

torch.set_num_threads(int(os.environ.get("THREADS", "4")))


def run(g, x0):
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    phi, adj = O.observation_operators(str(g["deg_op"]), load_blur_kernel("blur_1"), r)
    den = O.OracleDenoiser(resolve_weights(str(g["arch"]), int(ch)))
    res = O.test_iter(x0, g["x_obs"].astype(np.float64), g["x_true"], phi, adj, g1, g2, as_, an, lam, int(m1),
                      int(m2), gadmm, sig, sp, palpha, den, int(iters), str(g["method"]), int(ch), r)
    return np.asarray(res[0], np.float32), np.asarray(res[3])


for case in sys.argv[1:]:
    g = load_golden(f"long_{case}.npz")
    x0 = g["x_0"].astype(np.float32)
    sign = np.where(np.random.default_rng(0).random(x0.shape) < 0.5, -np.inf, np.inf).astype(np.float32)
    x0p = np.nextafter(x0, sign)
    xa, pa = run(g, x0.astype(np.float64))
    xb, pb = run(g, x0p.astype(np.float64))
    ref = g["x_out"].astype(np.float32)
    print(f"{case}: one-ulp start: max|dx| {np.abs(xa - xb).max():.4f}, pixels > 5e-3 {np.mean(np.abs(xa - xb) > 5e-3):.5f}, "
          f"max|dPSNR| {np.abs(pa - pb).max():.5f} | oracle vs golden: max|dx| {np.abs(xa - ref).max():.4f}, "
          f"pixels > 5e-3 {np.mean(np.abs(xa - ref) > 5e-3):.5f}, max|dPSNR| {np.abs(pa - g['psnr']).max():.5f}",
          flush=True)
