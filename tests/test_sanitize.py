"""Host runtime under AddressSanitizer + UBSan: `make -C pnp-pds_amd sanitize`
builds every translation unit with the sanitizers on its host side only and links the C-ABI
exercise tests/sanitize/capi_args.cpp (argument validation of every entry point, the no-device
error path of pnp_create, the host-side fp16 weight rounding with aliasing and edge values).
CPU only; the first build takes about a minute, later runs reuse build_asan/."""
import os
import subprocess

from conftest import REPO

PKG = os.path.join(REPO, "pnp-pds_amd")


def test_capi_host_paths_under_asan_ubsan():
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.run(["make", "-C", PKG, "-j", jobs, "sanitize"], check=True, capture_output=True, timeout=1200)
    exe = os.path.join(PKG, "build_asan", "capi_args")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    report = r.stdout + r.stderr
    assert "AddressSanitizer" not in report and "runtime error:" not in report, report[-4000:]
    assert r.returncode == 0 and "capi_args ok" in r.stdout, report[-4000:]
