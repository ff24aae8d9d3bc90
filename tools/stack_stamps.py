"""Diagnostic: per-phase time of the persistent denoiser at B = 1 from the STACK_STAMPS build
(s_memrealtime, 100 MHz).  PNP_LIB_PATH=abl_libs/stk_stamps.so python tools/stack_stamps.py [3|4]
(3: conv_stack16x2, two layers per hand-off; 4: conv_stack16, one)"""
import ctypes as C, os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pnp-pds_amd")]
import torch
from pnppds import _lib
from pnppds.weights import resolve_weights
ctx = _lib.Context(0)
w = resolve_weights("DnCNN_nobn_nch_3_nlev_0.01", 3)
ctx.set_denoiser(w)
ctx.set_precision("fp16")
MODE = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ctx.set_body_layers(MODE)
NL = 9 if MODE == 3 else 18
x = torch.rand(1, 3, 256, 256, device="cuda")
y = torch.empty_like(x)
for _ in range(5):
    ctx.op_denoise(x.data_ptr(), y.data_ptr(), 1, 3, 256, 256)
torch.cuda.synchronize()
n = 512 * 24 * 6
buf = (C.c_ulonglong * n)()
assert ctx.lib.pnp_diag_stack_stamps(buf, C.c_size_t(n)) == 0
a = np.frombuffer(buf, np.uint64).reshape(512, 24, 6).astype(np.int64)[:256, :NL]
t0 = a[:, 0, 0].min()
ns = lambda v: v * 10.0   # 100 MHz
names = ["wait", "halo DMA", "K-loop", "epilogue+drain", "publish"] if MODE == 4 else \
    ["wait", "halo DMA", "layer l (+ LDS)", "layer l+1 K-loop", "epilogue+drain+publish"]
for i, nm in enumerate(names):
    d = ns(a[:, 1:, i + 1] - a[:, 1:, i])
    print(f"{nm:16s} median {np.median(d):7.0f} ns  p90 {np.percentile(d, 90):7.0f}")
lay = ns(a[:, 1:, 0] - a[:, :-1, 0])
print(f"hand-off period     median {np.median(lay):7.0f} ns  p90 {np.percentile(lay, 90):7.0f}")
print(f"whole stack      {ns(a[:, NL - 1, 5].max() - t0) / 1e3:.1f} us from the first WG's start")
st = ns(a[:, 0, 0] - t0)
print(f"WG start skew    median {np.median(st):7.0f} ns  max {st.max():7.0f}")
