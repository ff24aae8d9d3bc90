"""Would a row-Winograd F(2,3) body keep the fp16 policy's parity margin?  (VERDICT r03 item 4a;
profiling aid, CPU only.)  Runs a long golden's trajectory through the oracle's test_iter with the
denoiser emulated at the device's rounding points, and prints max |dPSNR| against the golden
(the imported reference's own trajectory).

    python tools/winograd_emu.py MODE GOLDEN [THREADS] [ITERS]

  fp16   the product's numerics (PNP_PREC_FP16): fp16 activations, fp16 weights from
         fp16_filter_round, fp32 accumulation with the bias, act_h2 (the activation on the
         fp16-rounded value in packed fp16)
  wino   the same with every 64->64 body layer as F(2,3) along x: for output pixel pairs
         (2p, 2p+1) and each tap row, inputs d0..d3 = x[2p-1 .. 2p+2] (fp16) transformed as
         D = (d0-d2, d1+d2, d2-d1, d1-d3) rounded to fp16 (one v_pk_add/sub_f16), weights
         G = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2) rounded to fp16 from fp32, M_k = sum D_k G_k
         in fp32 (the MFMA), y0 = m0+m1+m2, y1 = m1-m2-m3 in fp32: 4 products per 2 outputs
         instead of 6, i.e. 2/3 of the body's MFMAs.  Head and tail stay direct.
  winoc  wino with the transformed weights' rounding errors compensated per filter row (the
         fp16_filter_round idea applied to the 3 G_k taps of each (c_out, c_in, component))
"""
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pnp-pds_amd"), os.path.join(REPO, "tests")]
from oracle import pnp_oracle as O  # noqa: E402
from pnppds.weights import resolve_weights  # noqa: E402

mode, case = sys.argv[1], sys.argv[2]
torch.set_num_threads(int(sys.argv[3]) if len(sys.argv) > 3 else 4)
H16 = torch.float16


def act_h2(h, act):
    """bias included, fp32 -> fp16 -> activation in fp16 (conv.hip act_h2)."""
    a = h.to(H16)
    if act == 0:
        a = torch.maximum(a, (a * torch.tensor(0.01, dtype=H16)))
    else:
        a = torch.clamp_min(a, 0)
    return a.float()


def round_rows3(g):
    """fp16 values of [..., 3] weight rows with each row's rounding-error sum compensated."""
    sh = g.shape
    w = g.reshape(-1, 3).numpy().astype(np.float32)
    pad = np.zeros((w.shape[0], 9), np.float32)
    pad[:, :3] = w
    r = O.fp16_filter_round(pad.reshape(-1, 1, 3, 3)).reshape(-1, 9)[:, :3]
    return torch.from_numpy(np.ascontiguousarray(r)).reshape(sh)


class Emu(O.OracleDenoiser):
    def __init__(self, w):
        super().__init__(w, emulate_fp16=True)      # self.tw: the fp16 weights (fp16_filter_round)
        self.G = []
        for i, t in enumerate(self.w.weights):
            g = torch.from_numpy(np.ascontiguousarray(t, np.float32))   # [co, ci, ky, kx] fp32
            g0, g1, g2 = g[..., 0], g[..., 1], g[..., 2]
            G = torch.stack([g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2])   # [4, co, ci, ky]
            if mode == "winoc":
                G = round_rows3(G)
            else:
                G = G.to(H16).float()
            self.G.append(G)

    def wino_layer(self, a, i):
        """a: [B, ci, H, W] fp16-valued fp32 activations (W even), layer i (64 -> 64)."""
        B, ci, H, W = a.shape
        ap = F.pad(a, (1, 1, 0, 0))                      # x = -1 and W (zero padding)
        d = [ap[..., k::2][..., :W // 2] for k in range(4)]   # d_k[p] = x[2p - 1 + k]
        D = [(d[0] - d[2]), (d[1] + d[2]), (d[2] - d[1]), (d[1] - d[3])]
        D = [t.to(H16).float() for t in D]
        m = [F.conv2d(D[k], self.G[i][k][..., None], None, padding=(1, 0)) for k in range(4)]
        y0 = m[0] + m[1] + m[2]
        y1 = m[1] - m[2] - m[3]
        out = torch.stack([y0, y1], -1).reshape(B, -1, H, W)
        return out + self.tb[i][None, :, None, None]

    @torch.no_grad()
    def forward_batch(self, x):
        xin = torch.from_numpy(np.ascontiguousarray(x, np.float32))
        if self.w.clamp_io:
            xin = xin.clamp(0, 1)
        h = xin.to(H16).float()
        n = len(self.tw)
        for i in range(n):
            if mode != "fp16" and 0 < i < n - 1:
                z = self.wino_layer(h, i)
            else:
                z = F.conv2d(h, self.tw[i], self.tb[i], padding=1)
            if i < n - 1:
                h = act_h2(z, self.w.act)
            else:
                h = z
        out = h + xin if self.w.residual > 0 else xin - h
        if self.w.clamp_io:
            out = out.clamp(0, 1)
        return out.numpy()


from conftest import load_golden  # noqa: E402
g = load_golden(f"long_{case}.npz")
g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
iters = int(sys.argv[4]) if len(sys.argv) > 4 else int(iters)
ch = int(ch)
h = np.load(os.path.join(REPO, "pnp-pds_amd", "weights", "blur_1.npy"))
phi, adj = O.observation_operators(str(g["deg_op"]), h, r)
den = Emu(resolve_weights(str(g["arch"]), ch))
t = time.time()
res = O.test_iter(np.asarray(g["x_0"], np.float64), np.asarray(g["x_obs"], np.float64), g["x_true"], phi, adj, g1, g2,
                  as_, an, lam, int(m1), int(m2), gadmm, sig, sp, palpha, den, iters, str(g["method"]), ch, r)
d = np.abs(res[3] - g["psnr"][:iters])
print(f"{case} {mode}: max|dPSNR| {d.max():.5f} @ {int(d.argmax())} over {iters} iterations "
      f"(final {res[3][-1]:.4f} vs {g['psnr'][iters - 1]:.4f}; {time.time() - t:.0f}s)", flush=True)
