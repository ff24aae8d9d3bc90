"""Probe (GPU): c_n fidelity of a precision hand-over inside one solve.

Runs a long golden with the fast precision for the first K iterations and a second precision for
the rest (pnp_set_precision between pnp_solver_iterate calls), then compares the returned c_n
with the reference's over every iteration where the golden's c >= 1e-6, and the PSNR.

  python tools/converge_probe.py A_blur_1200 fp16 fp16x3 0 3 5 8 12 16
  python tools/converge_probe.py A_blur_1200 auto converge 3000 1000     (thresholds in 1e-6)
"""
import os
import sys
import time

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (REPO, os.path.join(REPO, "pnp-pds_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

from conftest import load_golden  # noqa: E402


def run_switch(g, fast, slow, K):
    from pnppds import operators as ops
    from pnppds._device import get_ctx
    from pnppds.iteration import _resolve_denoiser, make_params, resolve_method
    g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, iters, ch, r = g["params"]
    iters, ch = int(iters), int(ch)
    phi, adj = ops.get_observation_operators(str(g["deg_op"]), "blur_1", r)
    ctx = get_ctx()
    den = _resolve_denoiser(str(g["arch"]) + ".pth", ch)
    den.configure(ctx)
    x0 = np.asarray(g["x_0"], np.float32)
    shp = x0.shape
    to4 = (lambda a: np.asarray(a, np.float32).reshape((1, 1) + shp)) if x0.ndim == 2 else \
        (lambda a: np.asarray(a, np.float32).reshape((1,) + shp))
    B, C, H, W = to4(x0).shape
    phi.configure(ctx, H, W)
    prm = make_params(g1, g2, as_, an, lam, m1, m2, gadmm, sig, sp, palpha, r, True, False)
    m = resolve_method(str(g["method"]))
    ctx.set_precision(fast)
    if slow == "converge":                   # the library's own hand-over at c_n < K * 1e-6
        ctx.set_precision("converge")
        ctx.set_converge_threshold(K * 1e-6)
    ctx.solver_setup(m, prm, B, C, H, W, iters)
    ctx.solver_load(to4(x0), to4(g["x_obs"]), to4(g["x_true"]))
    t0 = time.time()
    if slow == "converge":
        ctx.solver_iterate(iters)
        x, s, c, p, _ = ctx.solver_fetch()
        run_switch.switch_it = ctx.get_precision_switch()
        return x, c[0], p[0], time.time() - t0
    if K > 0:
        ctx.solver_iterate(min(K, iters))
    if K < iters:
        ctx.set_precision(slow)
        ctx.solver_iterate(iters - K)
    x, s, c, p, _ = ctx.solver_fetch()
    return x, c[0], p[0], time.time() - t0


def main():
    case, fast, slow = sys.argv[1:4]
    Ks = [int(k) for k in sys.argv[4:]] or [0]
    g = load_golden(f"long_{case}.npz")
    gc = np.asarray(g["c"]).ravel()
    mask = gc >= 1e-6
    for K in Ks:
        x, c, p, t = run_switch(g, fast, slow, K)
        rel = np.abs(c - gc) / gc
        worst = int(np.argmax(np.where(mask, rel, 0)))
        dp = np.abs(p - g["psnr"])
        dx = np.abs(x.ravel() - np.asarray(g["x_out"], np.float32).ravel()).max()
        if slow == "converge":
            print(f"  threshold {K * 1e-6:.1e}: switched at iteration {run_switch.switch_it}", flush=True)
            K = max(run_switch.switch_it, 0)
        after = rel[K + 1:][mask[K + 1:]] if K + 1 < len(gc) else np.zeros(1)
        print(f"{case} {fast}->{slow} K={K:4d}: c rel err (c_ref>=1e-6) max {rel[mask].max():.3f} at it {worst} "
              f"(after K: max {after.max() if after.size else 0:.3f}, median {np.median(after) if after.size else 0:.4f}); "
              f"final c {c[-1]:.2e} vs {gc[-1]:.2e}; max|dPSNR| {dp.max():.5f} dB; max|dx| {dx:.2e}; {t:.1f} s",
              flush=True)


if __name__ == "__main__":
    main()
