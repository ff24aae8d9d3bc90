"""Diagnostic: |dPSNR| along the long golden trajectories for fp16 / fp32 denoiser operands."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "pnp-pds_amd")
sys.path.insert(0, ".")
from conftest import load_golden
from test_gpu_long import run_long

for case in [a for a in sys.argv[1:] if "," not in a] or ["C_rs_300", "A_blur_1200", "B_blur_300"]:
    g = load_golden(f"long_{case}.npz")
    for prec in (sys.argv[-1].split(",") if "," in sys.argv[-1] else ("fp16", "fp16w2", "fp32")):
        x, s, c, psnr, ssim, t = run_long(g, prec)
        d = np.abs(psnr - g["psnr"])
        idx = sorted({min(i, len(d) - 1) for i in (0, 9, 49, 99, 199, len(d) // 2, len(d) - 1)})
        print(f"{case} {prec}: max|dPSNR| {d.max():.5f} @ {int(d.argmax())}; at {idx}: {np.round(d[idx], 5).tolist()}; "
              f"max|dx| {np.abs(x - g['x_out'].astype(np.float32)).max():.4f}; c_n end {c[-1]:.2e} vs {g['c'][-1]:.2e}",
              flush=True)
