"""test_iter — device-resident mirror of iteration.test_iter (iteration.py:10-196).

Same positional signature and return tuple as the reference:
    x_n, s_n + 0.5, c[max_iter], psnr[max_iter], ssim[max_iter], average_time
The whole loop (primal prox step through the MFMA denoiser, dual ascent with Φ/Φᵀ,
over-relaxation, l2-ball / l1-ball / GKL proxes, c_n and PSNR) runs on the MI355X via
``pnp_run``; nothing is computed on the host.

Differences from the reference, by design:
  * method names: README's 'ours-A/B/C' are accepted as aliases of 'A/B/C-Proposed'
    (the reference only recognises the latter, iteration.py:48-63, and crashes on the
    README names at :183-185); unknown methods raise ValueError.
  * ``phi``/``adj_phi`` must come from pnppds.operators.get_observation_operators (opaque
    Python closures cannot run on the device; there is no host fallback).
  * state is fp32 on the device (the reference mixes fp32 x and fp64 y); the denoiser's
    operands follow ``precision='auto'`` (the library's per-solve policy, PNP_PREC_AUTO in
    include/pnppds.h): fp16 with fp32 accumulation for ours-A / ours-B / comparisonB-2 on the blur operator,
    split fp16 (fp16x3, near-fp32) for everything else.  Tolerances: DESIGN.md §Parity.
  * ``ssim`` is computed on the device every iteration (utils_eval.eval_ssim restated;
    skimage is absent here, so its parity is unpinned).
  * comparisonB-4 / comparisonB-5 run with the DnCNN denoiser their text uses; the
    reference raises UnboundLocalError for them (denoiser_J is only built for names
    containing 'Proposed' or 'DnCNN', iteration.py:40-41).
  * the BM3D methods (A-PnPPDS-BM3D, A-PnPFBS-BM3D, comparisonB-1, C-PnPPDS-BM3D) need the
    bm3d package and are not available: they raise ValueError.
  * ``average_time`` is wall-clock seconds per iteration (the reference reports
    process_time, iteration.py:43,193-194).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._device import get_ctx
from .denoiser import Denoiser
from .operators import ObservationOperator
from .weights import DenoiserWeights

METHODS = {
    "A-Proposed": _lib.METHOD_A, "ours-A": _lib.METHOD_A,
    "B-Proposed": _lib.METHOD_B, "ours-B": _lib.METHOD_B,
    "C-Proposed": _lib.METHOD_C, "ours-C": _lib.METHOD_C,
    "comparisonB-2": _lib.METHOD_ADMM_B2,
    # comparison methods (iteration.py:71-180)
    "A-PnPFBS-DnCNN": _lib.METHOD_A_PNPFBS, "A-PDS-TV": _lib.METHOD_A_PDS_TV, "A-FBS-TV": _lib.METHOD_A_FBS_TV,
    "A-RED-DnCNN": _lib.METHOD_A_RED, "comparisonB-3": _lib.METHOD_B_HTV, "comparisonB-4": _lib.METHOD_B_RED,
    "comparisonB-5": _lib.METHOD_B_PNPFBS, "C-PnPADMM-DnCNN": _lib.METHOD_C_PNPADMM,
    "C-RED-DnCNN": _lib.METHOD_C_RED,
    # the KAIR DnCNN (path_prox = dncnn_color_blind / dncnn_15) in the A / C loops (iteration.py:104-110,174-180)
    "A-PnPPDS-unstable-DnCNN": _lib.METHOD_A, "C-PnP-unstable-DnCNN": _lib.METHOD_C,
}


def make_params(gamma1, gamma2, alpha_s, alpha_n, myLambda, m1, m2, gammaInADMMStep1, gaussian_nl, sp_nl,
                poisson_alpha, r, record_metrics=True, record_ssim=True) -> _lib.pnp_params:
    return _lib.pnp_params(float(gamma1), float(gamma2), float(alpha_s), float(alpha_n), float(myLambda),
                           int(m1), int(m2), float(gammaInADMMStep1), float(gaussian_nl), float(sp_nl),
                           float(poisson_alpha), float(r), 1 if record_metrics else 0,
                           1 if (record_metrics and record_ssim) else 0)


BM3D_METHODS = ("A-PnPPDS-BM3D", "A-PnPFBS-BM3D", "comparisonB-1", "C-PnPPDS-BM3D")

# Denoiser operand precision.  'auto' (the default) leaves the choice to the library, per solve
# (include/pnppds.h PNP_PREC_AUTO, capi.hip auto_precision), from the reference's own long
# trajectories (tests/test_gpu_long.py): on the blur operator fp16 operands (fp16w2
# above sigma 0.01 for ours-A / comparisonB-2) for ours-A / ours-B / comparisonB-2 / PnP-FBS / RED,
# every iteration's PSNR within 0.0035 dB of the reference; split fp16 (fp16x3: activations and
# weights as fp16 hi + lo pairs, three MFMAs per product, near-fp32) everywhere else.
# Under fp16 / fp16w2 operands x and PSNR follow the reference but the returned c (c_n,
# iteration.py:187) does not below ~3e-4: the fp16 activations' rounding leaves successive
# iterates ~3e-4 apart where the reference's keep contracting (to ~7e-8 after 1200 iterations).
# 'converge' keeps auto's operands, per image, while the image's own c_n is above 3e-3 and runs
# split activations after that (fp16a2 on the blur family, fp16x3 elsewhere), so c follows the
# reference's curve (checked to 10 % wherever it is >= 1e-6) and an image's results do not
# depend on its batch or shard; last_precision_switch() / last_precision_switches() report when.
def resolve_precision(precision) -> str:
    if precision not in _lib.PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(_lib.PRECISIONS)}, not {precision!r}")
    return precision


def last_precision_switch(ctx=None) -> int:
    """After a precision='converge' solve: the first iteration from which every image ran split
    activations (-1: some image never switched)."""
    return (ctx or get_ctx()).get_precision_switch()


def last_precision_switches(batch: int, ctx=None) -> np.ndarray:
    """After a precision='converge' solve of ``batch`` images: each image's switch iteration."""
    return (ctx or get_ctx()).get_precision_switches(batch)


def resolve_method(method: str) -> int:
    if method in BM3D_METHODS:
        raise ValueError(f"{method} needs the bm3d package (iteration.py:74-85,119-126,158-162); not available")
    if method not in METHODS:
        raise ValueError(f"Unknown method: {method!r} (device path supports {sorted(METHODS)})")
    return METHODS[method]


def _resolve_denoiser(path_prox, ch) -> Denoiser:
    if isinstance(path_prox, Denoiser):
        return path_prox
    if isinstance(path_prox, DenoiserWeights):
        return Denoiser(path_prox.name, ch, weights=path_prox)
    return Denoiser(path_prox, ch)


def _check_ops(phi, adj_phi):
    if not isinstance(phi, ObservationOperator) or not isinstance(adj_phi, ObservationOperator):
        raise TypeError("phi/adj_phi must come from pnppds.operators.get_observation_operators "
                        "(the device solver needs the operator's description, not a closure)")
    if phi.kind != adj_phi.kind or adj_phi.adjoint is phi.adjoint:
        raise ValueError("adj_phi must be the adjoint of phi")


def test_iter_batch(x_0, x_obsrv, x_true, phi, adj_phi, gamma1, gamma2, alpha_s, alpha_n, myLambda, m1, m2,
                    gammaInADMMStep1, gaussian_nl, sp_nl, poisson_alpha, path_prox, max_iter,
                    method="A-Proposed", ch=3, r=1, record_metrics=True, record_ssim=True, ctx=None,
                    precision="auto"):
    """Batched test_iter over B independent images: arrays are [B, C, H, W].
    Returns (x[B,C,H,W] f32, s+0.5 [B,C,H,W] f32, c[B,max_iter], psnr[B,max_iter], ssim[B,max_iter],
    avg_time).  ssim is computed on the device each iteration (iteration.py:189) when record_ssim;
    C == 1 batches are scored as the reference's (H, W) grayscale arrays.  precision: the
    denoiser's MFMA operands, 'fp16', 'fp16w2' (split weights, two MFMAs per product), 'fp32'
    (the reference's, about 10x slower), 'fp16x3' (split fp16: hi + lo activations and weights,
    three MFMAs per product, near-fp32) or 'auto' (default: the library's per-solve policy,
    fp16 for ours-A/B and comparisonB-2 on blur, fp16x3 otherwise: c_n floors near 3e-4 under
    fp16) or 'converge' (per image, auto until its c_n < 3e-3, then split activations: the
    reference's c_n curve)."""
    m = resolve_method(method)
    _check_ops(phi, adj_phi)
    x0 = np.asarray(x_0)
    if x0.ndim != 4:
        raise ValueError("test_iter_batch expects [B, C, H, W] arrays")
    B, Cc, H, W = x0.shape
    if Cc != ch:
        raise ValueError(f"ch={ch} but images have {Cc} channels")
    ctx = ctx or get_ctx()
    ctx.set_precision(resolve_precision(precision))
    if m not in _lib.TV_METHODS:                       # the TV methods use no denoiser
        den = _resolve_denoiser(path_prox, ch)
        den.configure(ctx)
    phi.configure(ctx, H, W)
    prm = make_params(gamma1, gamma2, alpha_s, alpha_n, myLambda, m1, m2, gammaInADMMStep1, gaussian_nl, sp_nl,
                      poisson_alpha, r, record_metrics, record_ssim)
    xt = None if x_true is None else np.broadcast_to(np.asarray(x_true, np.float32), x0.shape)
    xo = np.broadcast_to(np.asarray(x_obsrv, np.float32), x0.shape)
    x, s, c, psnr, ssim, t = ctx.run(m, prm, x0, xo, xt, int(max_iter))
    return x, s, c, psnr, ssim, t


def test_iter(x_0, x_obsrv, x_true, phi, adj_phi, gamma1, gamma2, alpha_s, alpha_n, myLambda, m1, m2,
              gammaInADMMStep1, gaussian_nl, sp_nl, poisson_alpha, path_prox, max_iter, method="A-Proposed",
              ch=3, r=1, *, precision="auto"):
    """iteration.py:10 signature; x_0 etc. are (C,H,W) (RGB) or (H,W) (gray).  Keyword-only
    extension: precision ('auto' default, 'fp16', 'fp16w2', 'fp16x3', 'fp32', 'converge'; see
    test_iter_batch and the precision notes above resolve_precision)."""
    x0 = np.asarray(x_0)
    shp = x0.shape
    to4 = (lambda a: np.asarray(a).reshape((1, 1) + shp)) if x0.ndim == 2 else \
        (lambda a: np.asarray(a).reshape((1,) + shp))
    x, s, c, psnr, ssim, t = test_iter_batch(to4(x0), to4(x_obsrv), None if x_true is None else to4(x_true),
                                             phi, adj_phi, gamma1, gamma2, alpha_s, alpha_n, myLambda, m1, m2,
                                             gammaInADMMStep1, gaussian_nl, sp_nl, poisson_alpha, path_prox,
                                             max_iter, method, ch, r, precision=precision)
    return x.reshape(shp), s.reshape(shp).astype(np.float64), c[0], psnr[0], ssim[0], t
