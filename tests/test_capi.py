"""C-ABI: the library builds, loads and exports every symbol include/pnppds.h declares.
CPU-only (no compute calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "pnppds.h")
LIB = os.path.join(REPO, "pnp-pds_amd", "lib", "libpnppds.so")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(pnp_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(REPO, "pnp-pds_amd"), "-j8"], check=True,
                       capture_output=True)
    return ctypes.CDLL(LIB)


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("pnp_create", "pnp_run", "pnp_set_denoiser", "pnp_set_operator", "pnp_op_denoise",
              "pnp_op_proj_l1_ball", "pnp_op_proj_l2_ball", "pnp_op_prox_gkl", "pnp_solver_iterate", "pnp_op_ssim"):
        assert s in syms
    assert len(syms) >= 25


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_no_unresolved_library_symbols(lib):
    """Every kernel the library launches is defined in it (an uninstantiated kernel template
    shows up as an undefined pnp:: symbol and only fails at load on the GPU box)."""
    out = subprocess.run(["nm", "-D", "--undefined-only", LIB], capture_output=True, text=True, check=True).stdout
    bad = [ln.split()[-1] for ln in out.splitlines() if "pnp" in ln]
    assert not bad, bad


def test_exports_are_plain_c(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    for s in declared_symbols():
        assert s in exported, s           # unmangled extern "C"


def test_abi_version_and_errors_without_gpu(lib):
    from pnppds import _lib
    assert lib.pnp_abi_version() == _lib.ABI_VERSION == 8
    lib.pnp_last_error.restype = ctypes.c_char_p
    h = ctypes.c_void_p()
    rc = lib.pnp_create(0, ctypes.byref(h))
    if rc != 0:      # no GPU here: must fail loudly with a message, never fall back
        assert rc in (-2, -3)
        assert lib.pnp_last_error(None)
        assert not h.value


def test_null_context_is_rejected(lib):
    assert lib.pnp_solver_iterate(None, 1) == -1
    assert lib.pnp_synchronize(None) == -1
    it = ctypes.c_int(5)
    assert lib.pnp_get_precision_switch(None, ctypes.byref(it)) == -1 and it.value == 5
    assert lib.pnp_get_precision_switches(None, ctypes.byref(it), 1) == -1 and it.value == 5
    assert lib.pnp_set_precision(None, 5) == -1


def test_precision_enum_matches_python():
    """The Python names of pnp_precision / the tuning keys are the header's values (ABI 7 added
    PNP_PREC_CONVERGE, PNP_PREC_FP16A2 and PNP_TUNE_CONVERGE_C)."""
    from pnppds import _lib
    src = open(HEADER).read()
    vals = {k: int(v) for k, v in re.findall(r"(PNP_(?:PREC|TUNE)_\w+)\s*=\s*(\d+)", src)}
    assert {k[len("PNP_PREC_"):].lower(): v for k, v in vals.items() if k.startswith("PNP_PREC_")} == \
        {("fp16" if k == "fp16" else k): v for k, v in _lib.PRECISIONS.items()}
    assert vals["PNP_TUNE_CONVERGE_C"] == _lib.TUNE_CONVERGE_C and vals["PNP_TUNE_GRAPH"] == _lib.TUNE_GRAPH


def test_params_struct_layout():
    from pnppds import _lib
    # 5 doubles, 2 int32, 5 doubles, 2 int32 as in pnppds.h
    assert ctypes.sizeof(_lib.pnp_params) == 8 * 5 + 4 * 2 + 8 * 5 + 8
    assert _lib.pnp_params.m1.offset == 40 and _lib.pnp_params.gamma_in_admm_step1.offset == 48
    assert _lib.pnp_params.record_metrics.offset == 88 and _lib.pnp_params.record_ssim.offset == 92


def test_product_does_not_import_oracle():
    """The shipped package never references the test oracle."""
    pkg = os.path.join(REPO, "pnp-pds_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h")):
                txt = open(os.path.join(root, f)).read()
                assert "pnp_oracle" not in txt and "import oracle" not in txt, f


def test_fp16_filter_round_matches_oracle(lib):
    """The fp16 weight values the device uses (capi.hip fp16_filter_round, host code) equal the
    oracle's restatement bit for bit, for every layer of the shipped denoisers plus edge values
    (exact fp16 weights, zeros, subnormals, ties); each filter's rounding-error sum is never
    larger than round-to-nearest's and every value stays within one fp16 ulp."""
    import numpy as np
    from oracle.pnp_oracle import fp16_filter_round
    from pnppds.weights import resolve_weights
    fn = lib.pnp_fp16_filter_round
    fn.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_size_t, ctypes.POINTER(ctypes.c_float)]
    rng = np.random.default_rng(3)
    edge = np.concatenate([np.zeros(9), np.full(9, 0.5), rng.standard_normal(9) * 1e-6,
                           np.float16(0.1) + np.array([0.5, -0.5, 0.25, 0, 1, -1, 0.5, 0.5, -0.5]) *
                           float(np.spacing(np.float16(0.1))),
                           rng.standard_normal(9 * 64) * 0.05]).astype(np.float32).reshape(-1, 1, 3, 3)
    layers = [edge]
    for arch, ch in (("DnCNN_nobn_nch_3_nlev_0.01", 3), ("DnCNN_nobn_nch_1_nlev_0.01", 1), ("dncnn_15", 1)):
        layers += list(resolve_weights(arch, ch).weights)
    for w in layers:
        w = np.ascontiguousarray(w, np.float32)
        out = np.empty_like(w)
        assert fn(w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), w.size // 9,
                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))) == 0
        ref = fp16_filter_round(w)
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), w.shape
        assert np.array_equal(out.astype(np.float16).astype(np.float32), out)          # fp16 values
        f = w.reshape(-1, 9).astype(np.float64)
        rn = w.astype(np.float16).astype(np.float64).reshape(-1, 9)
        e = np.abs((out.reshape(-1, 9) - f).sum(1))
        assert np.all(e <= np.abs((rn - f).sum(1)))
        ulp = np.spacing(np.abs(w.reshape(-1, 9)).astype(np.float16)).astype(np.float64)
        assert np.all(np.abs(out.reshape(-1, 9) - f) <= ulp * (1 + 1e-9) + 6e-8)


def test_auto_precision_policy(lib):
    """PNP_PREC_AUTO (capi.hip auto_precision, exported as pnp_auto_precision) against the
    policy test_gpu_long.py asserts on the device: every long golden's method, operator and
    sigma, plus the sigma threshold's edges, the non-denoiser operators and bad arguments."""
    from conftest import load_golden
    from pnppds import _lib
    from pnppds.iteration import resolve_method
    from test_gpu_long import expected_auto
    golden_dir = os.path.join(REPO, "tests", "golden")
    names = sorted(f[len("long_"):-len(".npz")] for f in os.listdir(golden_dir) if f.startswith("long_"))
    checked = 0
    for name in names:
        g = load_golden(f"long_{name}.npz")
        if "method" not in g:                # long_A_blur_256: the trajectory-only fixture
            continue
        checked += 1
        got = _lib.auto_precision(resolve_method(str(g["method"])), str(g["deg_op"]), float(g["params"][8]))
        assert got == expected_auto(g), (name, got)
    assert checked >= 25
    A, B, C = _lib.METHOD_A, _lib.METHOD_B, _lib.METHOD_C
    for m, op, sig, want in [(A, "blur", 0.01, "fp16"), (A, "blur", 0.0100001, "fp16w2"), (A, "blur", 0.0, "fp16"),
                             (B, "blur", 0.01, "fp16"), (B, "blur", 0.02, "fp16x3"),
                             (_lib.METHOD_ADMM_B2, "blur", 0.04, "fp16w2"), (_lib.METHOD_A_RED, "blur", 0.04, "fp16x3"),
                             (_lib.METHOD_A_PNPFBS, "blur", 0.005, "fp16"), (C, "blur", 0.0, "fp16x3"),
                             (A, "Id", 0.01, "fp16x3"), (A, "random_sampling", 0.01, "fp16x3"),
                             (_lib.METHOD_B_RED, "blur", 0.01, "fp16x3"), (_lib.METHOD_C_RED, "blur", 0.0, "fp16x3")]:
        assert _lib.auto_precision(m, op, sig) == want, (m, op, sig)
    fn = lib.pnp_auto_precision
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double]
    assert fn(13, 1, 0.01) == -1 and fn(-1, 1, 0.01) == -1 and fn(0, 3, 0.01) == -1
