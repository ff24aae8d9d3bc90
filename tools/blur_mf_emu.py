"""CPU emulation of the split-fp16 MFMA blur stencil (the round-3 experiment blur_mf.hip, in git
history at commit "Experiment: blur stencils of K1/K2 as row-Toeplitz MFMAs"), analysis only.

Operands split into fp16 halves after power-of-two scaling (taps: max |w| < 2^15; data: the
block's max |v| < 2^15), products hi*hi + lo*hi + hi*lo (exact in fp32), fp32 accumulation in tap
order; compared with the float64 periodic convolution.  Prints the absolute and max-relative
error for unit-range, small (dual-like) and large inputs, with and without the data scaling.

    python tools/blur_mf_emu.py
"""
import numpy as np


def split(v):
    hi = v.astype(np.float16)
    lo = (v - hi.astype(np.float64)).astype(np.float16)
    return hi.astype(np.float64), lo.astype(np.float64)


def main():
    h = np.load("pnp-pds_amd/weights/blur_1.npy").astype(np.float32).astype(np.float64)
    nz = h[h != 0]
    rng = np.random.default_rng(0)
    for name, x in [("unit", rng.random((64, 64))), ("small", rng.standard_normal((64, 64)) * 1e-3),
                    ("large", rng.standard_normal((64, 64)) * 30)]:
        x = x.astype(np.float32).astype(np.float64)
        c = 9
        exact = sum(h[i, j] * np.roll(np.roll(x, -(i - c), 0), -(j - c), 1)
                    for i in range(19) for j in range(19) if h[i, j] != 0)
        for scaled in (False, True):
            ed = 15 - np.frexp(np.abs(x).max())[1] if scaled else 0
            eh = 15 - np.frexp(np.abs(nz).max())[1]
            xh, xl = split(x * 2.0 ** ed)
            hh, hl = split(h * 2.0 ** eh)
            out = np.zeros_like(x, dtype=np.float32)
            for i in range(19):
                for j in range(19):
                    if h[i, j] == 0:
                        continue
                    sh = lambda a: np.roll(np.roll(a, -(i - c), 0), -(j - c), 1)
                    out = (out + (hh[i, j] * sh(xh) + hl[i, j] * sh(xh) + hh[i, j] * sh(xl)).astype(np.float32)
                           ).astype(np.float32)
            got = out.astype(np.float64) * 2.0 ** (-ed - eh)
            err = np.abs(got - exact).max()
            print(f"{name:6s} data scaling {'on ' if scaled else 'off'}: max abs err {err:.3e}, "
                  f"relative to max |out| {err / np.abs(exact).max():.3e}")


if __name__ == "__main__":
    main()
