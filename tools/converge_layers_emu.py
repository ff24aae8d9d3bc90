"""Which denoiser layers need split (hi + lo) activations for PNP_PREC_CONVERGE's c_n to follow
the reference's?  ("find which layers actually need split activations to keep
c within 10 % wherever c >= 1e-6", CPU only.)

    python tools/converge_layers_emu.py ITERS [THREADS] > profiles/r06/converge_layers_emu.txt

The oracle's test_iter (ours-A, blur_1, sigma 0.01, 3 x 128^2 synthetic image) with the denoiser's
operands rounded as the device rounds them:
  * reference: every conv in fp32 (torch-CPU; the reference's own arithmetic);
  * each mode runs PNP_PREC_CONVERGE's schedule: fp16 operands (PNP_PREC_FP16: fp16 input
    activations of every conv, fp16_filter_round weights) until c_n < 3e-3, then from two
    iterations later the layers in the mode's set with split activations (PNP_PREC_FP16A2:
    activations kept at fp32 -- the device's hi + lo pair carries ~21 bits --, body weights at
    their fp16 values, head / tail weights exact) and the others still fp16.
Printed per mode: the switch iteration, max relative c_n error over the iterations where the
reference's c_n >= 1e-6 (the converge tests' rule, tests/test_gpu_long.py C_MIN), the final c_n,
and max |dPSNR| against the reference.
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
from pnppds.operators import load_blur_kernel  # noqa: E402
from pnppds.weights import resolve_weights  # noqa: E402
import bench  # noqa: E402

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 800
torch.set_num_threads(int(sys.argv[2]) if len(sys.argv) > 2 else 8)
CONV_C = 3e-3


class LayerEmu(O.OracleDenoiser):
    """split = None: fp32 reference; otherwise the set of conv indices (0 = head .. 19 = tail) that
    run split activations once `self.switched`; before the switch every conv runs fp16."""

    def __init__(self, weights, split):
        super().__init__(weights)
        self.split = split
        self.switched = False
        self.w16 = [torch.from_numpy(O.fp16_filter_round(t.numpy())) for t in self.tw]

    @torch.no_grad()
    def forward_batch(self, x):
        xin = torch.from_numpy(np.ascontiguousarray(x, np.float32)).clamp(0, 1)
        h = xin
        n = len(self.tw)
        for i in range(n):
            if self.split is None:
                w = self.tw[i]
            elif self.switched and i in self.split:
                w = self.w16[i] if 0 < i < n - 1 else self.tw[i]      # fp16a2: fp16 body weights
            else:
                h = h.half().float()                                   # fp16 activations
                w = self.w16[i]
            h = F.conv2d(h, w, self.tb[i], padding=1)
            if i < n - 1:
                h = F.leaky_relu(h, O.LEAKY_SLOPE) if self.w.act == 0 else F.relu(h)
        out = h + xin if self.w.residual > 0 else xin - h
        return out.clamp(0, 1).numpy() if self.w.clamp_io else out.numpy()


def run(split, xt, obs, x0, phi, adj, weights):
    """One solve; c_n is recomputed from consecutive denoiser outputs (ours-A: x_n is the denoiser's
    output, iteration.py:187), which the switch rule reads two iterations behind, as the device."""
    den = LayerEmu(weights, split)
    c, state = [], {"i": 0, "prev": np.asarray(x0, np.float64), "sw": None}
    orig = den.denoise

    def denoise(x):
        i = state["i"]
        if split is not None and not den.switched and i >= 2 and c[i - 2] < CONV_C:
            den.switched = True
            state["sw"] = i
        out = orig(x)
        prev = state["prev"]
        c.append(float(np.linalg.norm(np.asarray(out, np.float64) - prev) / np.linalg.norm(prev)))
        state["prev"] = np.asarray(out, np.float64)
        state["i"] = i + 1
        return out

    den.denoise = denoise
    res = O.test_iter(x0, obs, xt, phi, adj, 0.99, 0.99, 1.0, 0.95, 1.0, 15, 15, 0.1, 0.01, 0.0, 300.0, den, ITERS,
                      "A-Proposed", 3, 0.8)
    cc = np.asarray(c)
    big = cc > 1e-4                          # the switch rule's range: the recomputed c_n is the solver's
    assert np.allclose(np.asarray(res[2])[big], cc[big], rtol=1e-4, atol=0), "c_n bookkeeping"
    return np.asarray(res[2]), np.asarray(res[3]), state["sw"]


def main():
    h = load_blur_kernel("blur_1")
    xt = bench.synthetic_images(0, 1, 3, 128, 128, seed=7)[0].astype(np.float64)
    obs, x0 = O.make_observation(xt, "blur", h, 0.8, 0.01, 0.0, False, 300.0)
    obs, x0 = np.asarray(obs, np.float64), np.asarray(x0, np.float64)
    phi, adj = O.observation_operators("blur", h)
    weights = resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3)
    n = weights.depth
    t = time.time()
    c_ref, p_ref, _ = run(None, xt, obs, x0, phi, adj, weights)
    print(f"reference (fp32): {ITERS} iterations in {time.time() - t:.0f}s; c_n {c_ref[0]:.3e} -> {c_ref[-1]:.3e}; "
          f"iterations with c_ref >= 1e-6: {int((c_ref >= 1e-6).sum())}", flush=True)
    modes = {
        "fp16 (no switch)": set(),
        "all 20 convs split (fp16a2)": set(range(n)),
        "body only (1-18)": set(range(1, n - 1)),
        "last 10 convs (10-19)": set(range(10, n)),
        "first 10 convs (0-9)": set(range(10)),
        "last 4 convs (16-19)": set(range(n - 4, n)),
        "every other conv (0, 2, .., 18)": set(range(0, n, 2)),
        "all but the last 2 (0-17)": set(range(n - 2)),
        "head only (0)": {0},
        "tail only (19)": {n - 1},
        "head and tail (0, 19)": {0, n - 1},
    }
    if len(sys.argv) > 3:                       # a subset of the modes, by name prefix
        modes = {k: v for k, v in modes.items() if any(k.startswith(p) for p in sys.argv[3].split(","))}
    m = c_ref >= 1e-6
    for name, sp in modes.items():
        t = time.time()
        c, p, sw = run(sp, xt, obs, x0, phi, adj, weights)
        rel = np.abs(c[m] - c_ref[m]) / c_ref[m]
        print(f"{name:34s} switch {sw}: max rel c err {rel.max():.4f} (c_ref >= 1e-6), final c {c[-1]:.3e} "
              f"(ref {c_ref[-1]:.3e}), max|dPSNR| {np.abs(p - p_ref).max():.5f} dB  [{time.time() - t:.0f}s]",
              flush=True)


if __name__ == "__main__":
    main()
