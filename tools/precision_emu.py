"""Which rounding moves BASELINE config 1 (1 x gray 256^2, Id, sigma 0.01, ours-A)?  The oracle's
test_iter with the denoiser's operands rounded as a device precision would round them (CPU,
torch conv2d in fp32 on the rounded operands; profiling aid, round 3).

    python tools/precision_emu.py {fp32,fp16,a,w,w2,s3,s3u} ITERS [THREADS]

  fp16  activations and weights fp16 (PNP_PREC_FP16)      a / w   only activations / weights
  w2    fp16 activations, weights hi + lo (PNP_PREC_FP16W2)
  s3u   activations and weights hi + lo, products hi*hi + hi*lo + lo*hi (PNP_PREC_FP16X3)
  s3    the same with the lo halves scaled by 2^11 (an alternative not built)
The input is bench.py's synthetic cfg1 image (seed 1) with the observation of main.py:49-64;
prints PSNR at iterations 0, 1, 2, 5, 10, 22 and the last (the bench compares 23 iterations).
Results: profiles/r03/precision_emu_cfg1.txt.
"""
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pnp-pds_amd")]
from oracle import pnp_oracle as O  # noqa: E402
from pnppds.weights import resolve_weights  # noqa: E402
import bench  # noqa: E402

mode, n = sys.argv[1], int(sys.argv[2])
torch.set_num_threads(int(sys.argv[3]) if len(sys.argv) > 3 else 4)


def round_sum16(w):
    """fp16 weights with each (cout, cin) 3x3 filter's rounding errors summed to ~0: taps are
    moved to their other fp16 neighbour, cheapest first, while that shrinks |sum of errors|."""
    w = w.numpy().astype(np.float32)
    o, i = w.shape[:2]
    f = w.reshape(o * i, -1).astype(np.float64)
    r = f.astype(np.float16).astype(np.float64)
    up = np.nextafter(r.astype(np.float16), np.float16(np.inf)).astype(np.float64)
    dn = np.nextafter(r.astype(np.float16), np.float16(-np.inf)).astype(np.float64)
    alt = np.where(r > f, dn, up)
    alt = np.where(r == f, r, alt)
    cost = np.abs(alt - f) - np.abs(r - f)
    out = r.copy()
    for k in range(f.shape[0]):
        S = (out[k] - f[k]).sum()
        used = np.zeros(f.shape[1], bool)
        while True:
            d = alt[k] - out[k]
            cand = (~used) & (np.abs(S + d) < np.abs(S) - 1e-30)
            if not cand.any():
                break
            j = np.argmin(np.where(cand, cost[k], np.inf))
            S += d[j]
            out[k, j] = alt[k, j]
            used[j] = True
    return torch.from_numpy(out.reshape(w.shape).astype(np.float32))


def split(t, scale):
    hi = t.half().float()
    return hi, ((t - hi) * scale).half().float() / scale


class Emu(O.OracleDenoiser):
    @torch.no_grad()
    def forward_batch(self, x):
        xin = torch.from_numpy(np.ascontiguousarray(x, np.float32)).clamp(0, 1)
        h = xin
        for i, (w, b) in enumerate(zip(self.tw, self.tb)):
            if mode == "fp32":
                h = F.conv2d(h, w, b, padding=1)
            elif mode == "fp16":
                h = F.conv2d(h.half().float(), w.half().float(), b, padding=1)
            elif mode == "a":
                h = F.conv2d(h.half().float(), w, b, padding=1)
            elif mode == "w":
                h = F.conv2d(h, w.half().float(), b, padding=1)
            elif mode in ("ws", "fs"):
                if not hasattr(self, "_ws"):
                    self._ws = [round_sum16(t) for t in self.tw]
                hin = h if mode == "ws" else h.half().float()
                h = F.conv2d(hin, self._ws[i], b, padding=1)
            elif mode == "w2":
                wh, wl = split(w, 1.0)
                h = F.conv2d(h.half().float(), wh + wl, b, padding=1)
            else:                                   # s3 / s3u
                sc = 2048.0 if mode == "s3" else 1.0
                ah, al = split(h, sc)
                wh, wl = split(w, sc)
                h = F.conv2d(ah, wh, b, padding=1) + (F.conv2d(ah, wl, None, padding=1) + F.conv2d(al, wh, None, padding=1))
            if i < len(self.tw) - 1:
                h = F.leaky_relu(h, 0.01)
        return (h + xin).clamp(0, 1).numpy()


xt = bench.synthetic_batch(1, 1, 256, 256, seed=1)[0][0]
obs, x0 = O.make_observation(xt, "Id", None, 0.8, 0.01, 0.0, False, 300.0)
phi, adj = O.observation_operators("Id")
den = Emu(resolve_weights("DnCNN_nobn_nch_1_nlev_0.01", 1))
t = time.time()
res = O.test_iter(x0.astype(np.float32).astype(np.float64), obs.astype(np.float32).astype(np.float64), xt, phi, adj,
                  0.99, 0.99, 1.0, 0.95, 1.0, 15, 15, 0.1, 0.01, 0.0, 300.0, den, n, "A-Proposed", 1, 0.8)
idx = [i for i in (0, 1, 2, 5, 10, 22, n - 1) if i < n]
print(mode, f"{time.time() - t:.0f}s", {i: round(float(res[3][i]), 5) for i in idx}, flush=True)
if len(sys.argv) > 4:                      # save the PSNR track for max-over-iterations comparisons
    np.save(sys.argv[4], np.asarray(res[3]))
