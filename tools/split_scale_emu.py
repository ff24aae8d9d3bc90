"""Where does split fp16 (PNP_PREC_FP16X3) lose precision on ours-C x 3000?

    python tools/split_scale_emu.py MODE [THREADS] [CASE]      (CPU; CASE default C_rs_3000)

The oracle's test_iter on a long golden's inputs with the denoiser's products formed as the
device forms them, every conv in torch-CPU fp32 on the rounded operands:
  fp32   the reference's arithmetic;
  s3u    the product's split: a_hi w_hi + a_hi w_lo + a_lo w_hi with x_lo = fp16(x - fp16(x))
         (fp16 subnormals kept: |x_lo| <= 2^-11 |x| is subnormal below |x| = 2^-3, so small
         weights and activations keep fewer bits);
  s3w    the same with every layer's weights scaled by 2^8 before the split (unscaled after
         the sum: exact), so weight lo halves stay normal above |w| = 2^-11;
  s3     weights and activations scaled by 2^8 (the ideal ~22-bit split).
Prints max |x - x_golden| and max |dPSNR| against the golden (the imported reference's own
trajectory, fp32 x_out since round 6).
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
from pnppds.operators import load_blur_kernel  # noqa: E402
from pnppds.weights import resolve_weights  # noqa: E402

MODE = sys.argv[1]
torch.set_num_threads(int(sys.argv[2]) if len(sys.argv) > 2 else 4)
CASE = sys.argv[3] if len(sys.argv) > 3 else "C_rs_3000"
S = 256.0


def split(t, scale):
    ts = t * scale
    hi = ts.half().float()
    return hi / scale, (ts - hi).half().float() / scale


class SplitEmu(O.OracleDenoiser):
    @torch.no_grad()
    def forward_batch(self, x):
        xin = torch.from_numpy(np.ascontiguousarray(x, np.float32))
        if self.w.clamp_io:
            xin = xin.clamp(0, 1)
        h = xin
        n = len(self.tw)
        for i in range(n):
            w, b = self.tw[i], self.tb[i]
            if MODE == "fp32":
                h = F.conv2d(h, w, b, padding=1)
            else:
                ah, al = split(h, S if MODE == "s3" else 1.0)
                wh, wl = split(w, S if MODE in ("s3", "s3w") else 1.0)
                h = F.conv2d(ah, wh, b, padding=1) + (F.conv2d(ah, wl, None, padding=1) + F.conv2d(al, wh, None, padding=1))
            if i < n - 1:
                h = F.leaky_relu(h, O.LEAKY_SLOPE) if self.w.act == 0 else F.relu(h)
        out = h + xin if self.w.residual > 0 else xin - h
        return (out.clamp(0, 1) if self.w.clamp_io else out).numpy()


def main():
    with np.load(os.path.join(REPO, "tests", "golden", f"long_{CASE}.npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    phi, adj = O.observation_operators(str(g["deg_op"]), load_blur_kernel("blur_1"), r)
    den = SplitEmu(resolve_weights(str(g["arch"]), int(ch)))
    t = time.time()
    res = O.test_iter(np.asarray(g["x_0"], np.float64), np.asarray(g["x_obs"], np.float64), g["x_true"], phi, adj,
                      g1, g2, as_, an, lam, int(m1), int(m2), gadmm, sig, sp, palpha, den, int(iters), str(g["method"]),
                      int(ch), r)
    dx = np.abs(np.asarray(res[0], np.float64) - g["x_out"]).max()
    dp = np.abs(np.asarray(res[3]) - g["psnr"]).max()
    print(f"{CASE} {MODE}: max|dx| {dx:.2e}, max|dPSNR| {dp:.5f} dB ({time.time() - t:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
