"""Static check of the persistent small-batch denoiser's cross-workgroup hand-off in the BUILT
code object (CPU only: disassembles pnp-pds_amd/lib/libpnppds.so).

common.h tile_publish / tile_wait use relaxed agent-scope atomics; the tile data's visibility
across CUs and XCDs rests on every hand-off access bypassing the non-coherent caches (sc1) and
on the publishing waves draining their stores before the workgroup barrier that precedes the
flag store (small batches).  The compiler is not told about that contract, so
this test pins it on the ISA it emitted, for every stack kernel (conv_stack16, conv_stack16x2,
conv_stack_s3; both activations):
  * every store of the kernel's tile data (buffer_store) carries sc1;
  * every halo LDS-DMA load (buffer_load ... lds) and every progress-word poll (global_load_dword)
    carries sc1;
  * every flag store (global_store_dword: tile_publish, the error word) is preceded, since the
    last data store in program order, by an s_waitcnt vmcnt(0) and then an s_barrier.
"""
import os
import re
import subprocess

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "pnp-pds_amd", "lib", "libpnppds.so")
LLVM = "/opt/rocm/lib/llvm/bin"
STACK_KERNELS = ("conv_stack16_kernel", "conv_stack16x2_kernel", "conv_stack_s3_kernel")


@pytest.fixture(scope="module")
def disasm(tmp_path_factory):
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("ROCm LLVM tools not found")
    d = tmp_path_factory.mktemp("isa")
    fat = d / "fatbin.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, str(d / "lib.so")],
                   check=True, capture_output=True)
    data = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs = [m.start() for m in re.finditer(re.escape(magic), data)] + [len(data)]
    funcs = {}
    for k in range(len(offs) - 1):                 # one bundle per translation unit
        part = d / f"b{k}.bin"
        part.write_bytes(data[offs[k]:offs[k + 1]])
        co = d / f"b{k}.co"
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode != 0 or not co.exists() or co.stat().st_size == 0:
            continue
        out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(co)], check=True, capture_output=True,
                             text=True).stdout
        name = None
        for line in out.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
            if m:
                name = m.group(1)
                funcs[name] = []
            elif name and line.startswith("\t"):
                funcs[name].append(line.split("//")[0].strip())
    return funcs


def _stack_funcs(disasm):
    f = {n: body for n, body in disasm.items() if any(k in n for k in STACK_KERNELS)}
    assert len(f) >= 6, sorted(f)                 # 3 kernels x 2 activations
    return f


def test_stack_kernels_hand_off_with_sc1(disasm):
    for name, body in _stack_funcs(disasm).items():
        stores = [i for i in body if i.startswith("buffer_store")]
        assert stores, name
        assert all(re.search(r"\bsc1\b", i) for i in stores), (name, [i for i in stores if "sc1" not in i][:3])
        dma = [i for i in body if i.startswith("buffer_load") and re.search(r"\blds\b", i)]
        assert dma, name
        assert all(re.search(r"\bsc1\b", i) for i in dma), name
        polls = [i for i in body if re.match(r"global_load_dword\s", i)]
        assert polls, name
        assert all(re.search(r"\bsc1\b", i) for i in polls), name


def test_flag_stores_follow_drain_and_barrier(disasm):
    for name, body in _stack_funcs(disasm).items():
        flags = 0
        pending, drained = False, False
        for ins in body:
            op = ins.split()[0] if ins else ""
            if op.startswith("buffer_store"):
                pending, drained = True, False
            elif op == "s_waitcnt" and "vmcnt(0)" in ins and pending:
                drained = True
            elif op == "s_barrier" and drained:
                pending, drained = False, False
            elif op.startswith("global_store_dword"):
                flags += 1
                assert re.search(r"\bsc1\b", ins), (name, ins)
                assert not pending, (name, "flag store without vmcnt(0) + s_barrier after the tile stores")
        assert flags >= 2, (name, flags)          # the progress word and the error word
