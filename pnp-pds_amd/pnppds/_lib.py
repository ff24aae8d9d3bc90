"""ctypes binding of libpnppds.so (include/pnppds.h).

There is no CPU fallback: if the library is missing or no gfx950 device is present,
every compute call raises.  The library is built in-tree by ``make -C pnp-pds_amd``
(``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PNP_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "lib", "libpnppds.so")   # override: profiling A/B only

PNP_OK = 0
ERRORS = {-1: "PNP_E_ARG", -2: "PNP_E_UNSUPPORTED", -3: "PNP_E_HIP", -4: "PNP_E_OOM", -5: "PNP_E_STATE", -6: "PNP_E_INTERNAL"}

METHOD_A, METHOD_B, METHOD_C, METHOD_ADMM_B2 = 0, 1, 2, 3
(METHOD_A_PNPFBS, METHOD_A_PDS_TV, METHOD_A_FBS_TV, METHOD_A_RED, METHOD_B_HTV, METHOD_B_RED, METHOD_B_PNPFBS,
 METHOD_C_PNPADMM, METHOD_C_RED) = range(4, 13)
TV_METHODS = (METHOD_A_PDS_TV, METHOD_A_FBS_TV, METHOD_B_HTV)   # no denoiser
OP_ID, OP_BLUR, OP_RANDOM_SAMPLING = 0, 1, 2
PREC_FP16, PREC_FP32, PREC_FP16W2, PREC_FP16X3, PREC_AUTO, PREC_CONVERGE, PREC_FP16A2 = 0, 1, 2, 3, 4, 5, 6
PRECISIONS = {"fp16": PREC_FP16, "fp32": PREC_FP32, "fp16w2": PREC_FP16W2, "fp16x3": PREC_FP16X3, "auto": PREC_AUTO,
              "converge": PREC_CONVERGE, "fp16a2": PREC_FP16A2}
PRECISION_NAMES = {v: k for k, v in PRECISIONS.items()}
TUNE_DENOISE_CHUNK = 1
TUNE_BODY_LAYERS = 2
TUNE_GRAPH = 3
TUNE_CONVERGE_C = 4      # PNP_PREC_CONVERGE's c_n threshold, units of 1e-6 (ABI 7)
TUNE_FUSE_ENDS = 5       # head / tail inside the first / last two-layer launch (ABI 7)
TUNE_ABLATE_K2 = 98      # profiling build only: k2_blur_rb ablation legs (ops.hip ABL bits)
TUNE_ABLATE = 99         # profiling build only (make PROFILING=1, lib_prof/): not in include/pnppds.h


class PnpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class pnp_params(C.Structure):
    _fields_ = [("gamma1", C.c_double), ("gamma2", C.c_double), ("alpha_s", C.c_double),
                ("alpha_n", C.c_double), ("my_lambda", C.c_double), ("m1", C.c_int32), ("m2", C.c_int32),
                ("gamma_in_admm_step1", C.c_double), ("gaussian_nl", C.c_double), ("sp_nl", C.c_double),
                ("poisson_alpha", C.c_double), ("r", C.c_double), ("record_metrics", C.c_int32),
                ("record_ssim", C.c_int32)]


ABI_VERSION = 8   # include/pnppds.h PNP_ABI_VERSION
class pnp_degrade_params(C.Structure):
    _fields_ = [("gaussian_nl", C.c_double), ("sp_nl", C.c_double), ("poisson_alpha", C.c_double),
                ("poisson_noise", C.c_int32), ("seed", C.c_uint32)]


_lib = None
_lock = threading.Lock()

_P = C.c_void_p
_F = C.POINTER(C.c_float)
_D = C.POINTER(C.c_double)
_SIGS = {
    "pnp_abi_version": ([], C.c_int),
    "pnp_build_id": ([], C.c_char_p),
    "pnp_device_count": ([C.POINTER(C.c_int)], C.c_int),
    "pnp_create": ([C.c_int, C.POINTER(_P)], C.c_int),
    "pnp_destroy": ([_P], C.c_int),
    "pnp_last_error": ([_P], C.c_char_p),
    "pnp_synchronize": ([_P], C.c_int),
    "pnp_set_denoiser": ([_P, C.c_int, C.c_int, C.c_int, _F, C.c_size_t, C.c_int, C.c_int, C.c_int], C.c_int),
    "pnp_set_precision": ([_P, C.c_int], C.c_int),
    "pnp_get_precision": ([_P, C.POINTER(C.c_int), C.POINTER(C.c_int)], C.c_int),
    "pnp_get_precision_switch": ([_P, C.POINTER(C.c_int)], C.c_int),
    "pnp_get_precision_switches": ([_P, C.POINTER(C.c_int), C.c_int], C.c_int),
    "pnp_device_copy": ([_P, _P, _P, C.c_size_t, _P], C.c_int),
    "pnp_set_tuning": ([_P, C.c_int, C.c_int], C.c_int),
    "pnp_set_operator": ([_P, C.c_int, _D, C.c_int, C.c_int, C.POINTER(C.c_uint8), C.c_int, C.c_int], C.c_int),
    "pnp_run": ([_P, C.c_int, C.POINTER(pnp_params), C.c_int, C.c_int, C.c_int, C.c_int, _F, _F, _F, C.c_int,
                 _F, _F, _D, _D, _D, _D], C.c_int),
    "pnp_solver_setup": ([_P, C.c_int, C.POINTER(pnp_params), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int],
                         C.c_int),
    "pnp_solver_load": ([_P, _F, _F, _F], C.c_int),
    "pnp_solver_load_device": ([_P, _P, _P, _P], C.c_int),
    "pnp_solver_iterate": ([_P, C.c_int], C.c_int),
    "pnp_solver_fetch": ([_P, _F, _F, _D, _D, _D], C.c_int),
    "pnp_solver_iterations_done": ([_P, C.POINTER(C.c_int)], C.c_int),
    "pnp_solver_state": ([_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P)], C.c_int),
    "pnp_profile_enable": ([_P, C.c_int], C.c_int),
    "pnp_profile_read": ([_P, C.c_int, C.POINTER(C.c_char_p), _D, C.POINTER(C.c_int), C.POINTER(C.c_int)],
                         C.c_int),
    "pnp_op_phi": ([_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P], C.c_int),
    "pnp_op_adj_phi": ([_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P], C.c_int),
    "pnp_op_proj_l2_ball": ([_P, _P, _P, _P, C.c_int, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double,
                             _P], C.c_int),
    "pnp_op_proj_l1_ball": ([_P, _P, _P, C.c_int, C.c_int64, C.c_double, C.c_double, C.c_double, _P], C.c_int),
    "pnp_op_prox_gkl": ([_P, _P, _P, _P, C.c_int64, C.c_double, C.c_double, _P], C.c_int),
    "pnp_op_denoise": ([_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P], C.c_int),
    "pnp_op_status": ([_P, _P], C.c_int),
    "pnp_fp16_filter_round": ([_F, C.c_size_t, _F], C.c_int),
    "pnp_auto_precision": ([C.c_int, C.c_int, C.c_double], C.c_int),
    "pnp_op_psnr": ([_P, _P, _P, C.c_int, C.c_int64, _D, _P], C.c_int),
    "pnp_degrade": ([_P, C.POINTER(pnp_degrade_params), C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P],
                    C.c_int),
    "pnp_op_ssim": ([_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _D, _P], C.c_int),
}


_PKG = os.path.dirname(_HERE)


def source_hash() -> str | None:
    """The build id libpnppds.so must carry: SHA-256 prefix of the sources listed in the
    Makefile's SRC and HDR (sorted, concatenated), as the Makefile computes it.  None if the
    sources are not in the tree."""
    import hashlib
    try:
        with open(os.path.join(_PKG, "Makefile")) as f:
            mk = f.read()
    except OSError:
        return None
    files = []
    for line in mk.splitlines():
        key, _, val = line.partition("=")
        if key.strip() in ("SRC", "HDR") and not line.startswith((" ", "\t")):
            files += val.split()
    h = hashlib.sha256()
    for rel in sorted(set(files)):
        try:
            with open(os.path.join(_PKG, rel), "rb") as f:
                h.update(f.read())
        except OSError:
            return None
    return h.hexdigest()[:16]


def build_id() -> str:
    return load_library().pnp_build_id().decode()


def load_library(path: str = LIB_PATH):
    """Load libpnppds.so (raises if absent — there is no fallback path — or if it was built
    from other sources than the tree's: a stale prebuilt library must not pass for this one)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise RuntimeError(f"libpnppds.so not found at {path}; run `make -C pnp-pds_amd` "
                                   "(or __graft_entry__.build())")
            try:   # torch ships its own HIP runtime under the same soname: load it first so the
                import torch  # noqa: F401  process has one runtime (ours would shadow torch's)
            except ImportError:
                pass
            lib = C.CDLL(path)
            for name, (args, res) in _SIGS.items():
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = res
            if lib.pnp_abi_version() != ABI_VERSION:
                raise RuntimeError("libpnppds ABI mismatch")
            want, got = source_hash(), lib.pnp_build_id().decode()
            if want is not None and got != want and path == os.path.join(_PKG, "lib", "libpnppds.so"):
                raise RuntimeError(f"{path} was built from other sources (build id {got}, tree {want}); "
                                   "rebuild with `make -C pnp-pds_amd`")
            _lib = lib
    return _lib


def _fptr(a):
    return a.ctypes.data_as(_F) if a is not None else None


def _dptr(a):
    return a.ctypes.data_as(_D) if a is not None else None


def device_count() -> int:
    lib = load_library()
    n = C.c_int(0)
    rc = lib.pnp_device_count(C.byref(n))
    if rc != PNP_OK:
        return 0
    return n.value


OP_KINDS = {"Id": OP_ID, "blur": OP_BLUR, "random_sampling": OP_RANDOM_SAMPLING}


def auto_precision(method: int, op_kind, gaussian_nl: float) -> str:
    """What precision='auto' (PNP_PREC_AUTO) resolves to for a solve of ``method`` (a METHOD_*
    code) on ``op_kind`` (OP_* code or 'Id' / 'blur' / 'random_sampling') at noise level
    ``gaussian_nl``: 'fp16', 'fp16w2' or 'fp16x3' (pnp_auto_precision; no device needed)."""
    op = OP_KINDS[op_kind] if isinstance(op_kind, str) else int(op_kind)
    rc = load_library().pnp_auto_precision(int(method), op, float(gaussian_nl))
    if rc < 0:
        raise PnpError(rc, f"unknown method {method} or operator {op_kind}")
    return PRECISION_NAMES[rc]


def as_f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class Context:
    """One device context (one GPU).  Not thread-safe; one per host thread / rank."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        self.device = device
        h = _P()
        rc = self.lib.pnp_create(device, C.byref(h))
        if rc != PNP_OK:
            raise PnpError(rc, self.lib.pnp_last_error(None).decode())
        self.h = h
        self._denoiser_key = None
        self._operator_key = None
        self.precision = PREC_AUTO            # the library's default (pnp_set_precision)

    # -- plumbing --
    def _check(self, rc):
        if rc != PNP_OK:
            raise PnpError(rc, self.lib.pnp_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.pnp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        self._check(self.lib.pnp_synchronize(self.h))

    # -- configuration --
    def set_denoiser(self, weights, key=None):
        """weights: pnppds.weights.DenoiserWeights."""
        if key is not None and key == self._denoiser_key:
            return
        flat = as_f32(weights.flat())
        self._check(self.lib.pnp_set_denoiser(self.h, weights.channels, weights.depth, weights.width,
                                              _fptr(flat), flat.size, weights.act, weights.residual,
                                              weights.clamp_io))
        self._denoiser_key = key

    def set_precision(self, precision):
        """Denoiser operands: 'auto' (default: the library's per-solve policy, auto_precision()
        below; include/pnppds.h PNP_PREC_AUTO), 'fp16' (fp32
        accumulation), 'fp16w2' (fp16 activations, weights as fp16 hi + lo pairs: two MFMAs per
        product), 'fp16x3' (activations and weights as hi + lo pairs: three MFMAs per product,
        near-fp32), 'fp32' (the reference's own precision, models/denoiser.py:37; about a
        tenth of the fp16 throughput) or 'converge' (per image: auto's operands while the image's
        own c_n is above 3e-3, then split activations -- fp16a2 on the blur family, where auto runs
        fp16 / fp16w2, fp16x3 elsewhere: c_n then follows the reference's curve, which fp16
        activations stop following below ~3e-4; get_precision_switches() says when each image
        switched)."""
        code = PRECISIONS[precision] if isinstance(precision, str) else int(precision)
        self._check(self.lib.pnp_set_precision(self.h, code))
        self.precision = code

    def get_precision(self):
        """(requested, effective) precision names; effective = what the next solver step uses."""
        r, e = C.c_int(), C.c_int()
        self._check(self.lib.pnp_get_precision(self.h, C.byref(r), C.byref(e)))
        return PRECISION_NAMES[r.value], PRECISION_NAMES[e.value]

    def get_precision_switch(self) -> int:
        """precision='converge': the first iteration of the current solve from which every image
        ran split activations (fp16a2 on the blur family, fp16x3 elsewhere), or -1 while some
        image has not switched (pnp_get_precision_switch; for one image, its switch)."""
        it = C.c_int()
        self._check(self.lib.pnp_get_precision_switch(self.h, C.byref(it)))
        return it.value

    def get_precision_switches(self, batch: int) -> np.ndarray:
        """precision='converge': per image of the current solve (``batch`` = its B), the first
        iteration it ran split activations, -1 if not yet (pnp_get_precision_switches)."""
        out = np.full(int(batch), -1, np.int32)
        self._check(self.lib.pnp_get_precision_switches(self.h, out.ctypes.data_as(C.POINTER(C.c_int)),
                                                        int(batch)))
        return out

    def set_converge_threshold(self, c: float):
        """precision='converge': an image switches to split activations once its own c_n is below
        c (default 3e-3; set in units of 1e-6, PNP_TUNE_CONVERGE_C)."""
        self._check(self.lib.pnp_set_tuning(self.h, TUNE_CONVERGE_C, max(1, int(round(c * 1e6)))))

    def set_denoise_chunk(self, images: int):
        """Images per denoiser pass (0 = auto).  Performance only."""
        self._check(self.lib.pnp_set_tuning(self.h, TUNE_DENOISE_CHUNK, int(images)))

    def set_graph(self, mode: int):
        """Iteration launches replayed from a hipGraph: 1 = on, 0 = off (default).  Same results
        either way (methods A/B/C; the others always launch directly)."""
        self._check(self.lib.pnp_set_tuning(self.h, TUNE_GRAPH, int(mode)))

    def set_body_layers(self, n: int):
        """64->64 denoiser layers per launch: 0 = auto (default: all in one persistent launch for
        batches with at most 2 tiles per CU, fused pairs when the batch has a 32-column strip per
        CU), 1, 2, 3 (all, two layers per tile hand-off) or 4 (all, one per hand-off).  Same bits
        either way."""
        self._check(self.lib.pnp_set_tuning(self.h, TUNE_BODY_LAYERS, int(n)))

    def set_fuse_ends(self, on: int):
        """1 (default): with the two-layer launches (FP16, even body depth) the head runs inside
        the first one and the tail inside the last; 0: separate head / tail launches.  Same bits."""
        self._check(self.lib.pnp_set_tuning(self.h, TUNE_FUSE_ENDS, int(on)))

    def set_ablate(self, bits: int):
        """Profiling build only (make PROFILING=1, PNP_LIB_PATH=.../lib_prof/libpnppds.so;
        results wrong): skip parts of the one-layer body kernel (1 = halo DMA, 2 = stores,
        4 = MFMA K-loop).  The product library rejects the key (PNP_E_UNSUPPORTED)."""
        self._check(self.lib.pnp_set_tuning(self.h, TUNE_ABLATE, int(bits)))

    def set_ablate_k2(self, bits: int):
        """Profiling build only (results wrong): blur K2 (k2_blur_rb, ours-A, batched) with phases
        removed: 1 stencil, 2 fp64 partials, 4 epilogue stores, 8 halo fill, 16 epilogue loads
        (and the combinations 3, 6, 7, 9, 20).  Process-wide."""
        self._check(self.lib.pnp_set_tuning(self.h, TUNE_ABLATE_K2, int(bits)))

    def set_operator(self, kind: int, h=None, mask=None, key=None):
        if key is not None and key == self._operator_key:
            return
        hh = np.ascontiguousarray(h, np.float64) if h is not None else None
        mm = np.ascontiguousarray(mask, np.uint8) if mask is not None else None
        self._check(self.lib.pnp_set_operator(
            self.h, kind, hh.ctypes.data_as(_D) if hh is not None else None,
            hh.shape[0] if hh is not None else 0, hh.shape[1] if hh is not None else 0,
            mm.ctypes.data_as(C.POINTER(C.c_uint8)) if mm is not None else None,
            mm.shape[0] if mm is not None else 0, mm.shape[1] if mm is not None else 0))
        self._operator_key = key

    # -- whole solver --
    def run(self, method, params: pnp_params, x0, xobs, xtrue, max_iter, want_s=True):
        x0, xobs = as_f32(x0), as_f32(xobs)
        xtrue = as_f32(xtrue) if xtrue is not None else None
        B, Cc, H, W = x0.shape
        x_out = np.empty_like(x0)
        s_out = np.empty_like(x0) if want_s else None
        c_out = np.empty((B, max_iter), np.float64)
        p_out = np.empty((B, max_iter), np.float64)
        m_out = np.empty((B, max_iter), np.float64)
        t = C.c_double(0)
        self._check(self.lib.pnp_run(self.h, method, C.byref(params), B, Cc, H, W, _fptr(x0), _fptr(xobs),
                                     _fptr(xtrue), max_iter, _fptr(x_out), _fptr(s_out), _dptr(c_out),
                                     _dptr(p_out), _dptr(m_out), C.byref(t)))
        return x_out, s_out, c_out, p_out, m_out, t.value

    def solver_setup(self, method, params, B, Cc, H, W, cap):
        self._check(self.lib.pnp_solver_setup(self.h, method, C.byref(params), B, Cc, H, W, cap))
        self._shape = (B, Cc, H, W)
        self._cap = cap

    def solver_load(self, x0, xobs, xtrue=None):
        x0, xobs = as_f32(x0), as_f32(xobs)
        xtrue = as_f32(xtrue) if xtrue is not None else None
        self._check(self.lib.pnp_solver_load(self.h, _fptr(x0), _fptr(xobs), _fptr(xtrue)))

    def solver_load_device(self, d_x0: int, d_xobs: int, d_xtrue: int | None):
        self._check(self.lib.pnp_solver_load_device(self.h, _P(d_x0), _P(d_xobs),
                                                    _P(d_xtrue) if d_xtrue else None))

    def solver_iterate(self, n):
        self._check(self.lib.pnp_solver_iterate(self.h, n))

    def solver_fetch(self):
        B, Cc, H, W = self._shape
        x = np.empty((B, Cc, H, W), np.float32)
        s = np.empty((B, Cc, H, W), np.float32)
        c = np.empty((B, max(self._cap, 0)), np.float64)
        p = np.empty((B, max(self._cap, 0)), np.float64)
        m = np.empty((B, max(self._cap, 0)), np.float64)
        self._check(self.lib.pnp_solver_fetch(self.h, _fptr(x), _fptr(s), _dptr(c), _dptr(p), _dptr(m)))
        return x, s, c, p, m

    def solver_state(self):
        """Device pointers (x, y, s) of the solver's current state; y is the dual as the reference
        holds it (a pending l2-ball step is applied first)."""
        x, y, sv = _P(), _P(), _P()
        self._check(self.lib.pnp_solver_state(self.h, C.byref(x), C.byref(y), C.byref(sv)))
        return x.value, y.value, sv.value

    def profile_enable(self, on=True):
        """on: False / 0 off, True / 1 every launch, 2 only the denoiser's body launches."""
        self._check(self.lib.pnp_profile_enable(self.h, int(on)))

    def profile_read(self):
        cap = 64
        names = (C.c_char_p * cap)()
        avg = (C.c_double * cap)()
        calls = (C.c_int * cap)()
        n = C.c_int(0)
        self._check(self.lib.pnp_profile_read(self.h, cap, names, avg, calls, C.byref(n)))
        return {names[i].decode(): (avg[i], calls[i]) for i in range(n.value)}

    # -- single operators on device pointers (ints from e.g. torch.Tensor.data_ptr()) --
    def op_phi(self, x, y, B, Cc, H, W, adj=False, stream=None):
        fn = self.lib.pnp_op_adj_phi if adj else self.lib.pnp_op_phi
        self._check(fn(self.h, _P(x), _P(y), B, Cc, H, W, _P(stream) if stream else None))

    def op_proj_l2_ball(self, x, x0, out, B, n, alpha_n, gaussian_nl, sp_nl, r=1.0, stream=None):
        self._check(self.lib.pnp_op_proj_l2_ball(self.h, _P(x), _P(x0), _P(out), B, n, alpha_n, gaussian_nl,
                                                 sp_nl, r, _P(stream) if stream else None))

    def op_proj_l1_ball(self, x, out, B, n, alpha_s, sp_nl, r=1.0, stream=None):
        self._check(self.lib.pnp_op_proj_l1_ball(self.h, _P(x), _P(out), B, n, alpha_s, sp_nl, r,
                                                 _P(stream) if stream else None))

    def op_prox_gkl(self, x, x0, out, count, gamma, alpha, stream=None):
        self._check(self.lib.pnp_op_prox_gkl(self.h, _P(x), _P(x0), _P(out), count, gamma, alpha,
                                             _P(stream) if stream else None))

    def op_denoise(self, x, out, B, Cc, H, W, stream=None):
        self._check(self.lib.pnp_op_denoise(self.h, _P(x), _P(out), B, Cc, H, W, _P(stream) if stream else None))

    def op_status(self, stream=None):
        """Synchronize the single ops' stream and raise if a persistent denoiser launch failed."""
        self._check(self.lib.pnp_op_status(self.h, _P(stream) if stream else None))

    def device_copy(self, dst, src, nbytes, stream=None):
        """dst = src (device pointers): the float4 streaming copy bench.py measures."""
        self._check(self.lib.pnp_device_copy(self.h, _P(dst), _P(src), nbytes, _P(stream) if stream else None))

    def op_psnr(self, xt, x, B, n, stream=None):
        out = np.empty(B, np.float64)
        self._check(self.lib.pnp_op_psnr(self.h, _P(xt), _P(x), B, n, _dptr(out), _P(stream) if stream else None))
        return out

    def degrade(self, params: "pnp_degrade_params", xt, B, Cc, H, W, xobs=None, x0=None, xobs64=None,
                stream=None):
        """main.py:49-64 on device pointers (ints); synchronous."""
        self._check(self.lib.pnp_degrade(self.h, C.byref(params), B, Cc, H, W, _P(xt), _P(xobs) if xobs else None,
                                         _P(x0) if x0 else None, _P(xobs64) if xobs64 else None,
                                         _P(stream) if stream else None))

    def op_ssim(self, xt, x, B, Cc, H, W, stream=None):
        """utils_eval.eval_ssim per image (Cc == 1: the reference's (H, W) grayscale arrays)."""
        out = np.empty(B, np.float64)
        self._check(self.lib.pnp_op_ssim(self.h, _P(xt), _P(x), B, Cc, H, W, _dptr(out),
                                         _P(stream) if stream else None))
        return out


_contexts: dict = {}


def get_context(device: int = 0) -> Context:
    """Process-wide cached context per device."""
    ctx = _contexts.get(device)
    if ctx is None:
        ctx = Context(device)
        _contexts[device] = ctx
    return ctx
