"""GPU parity of the MFMA denoiser vs the reference's outputs and the fp16-emulating oracle."""
import os

import numpy as np
import pytest

from oracle import pnp_oracle as O
from pnppds.weights import DenoiserWeights, WEIGHTS_DIR, random_weights

pytestmark = pytest.mark.gpu

# fp16 operands / fp32 accumulation vs the reference's fp32 conv (fp16 passes
# the 0.01 dB target).  Against the oracle that rounds the same operands to fp16 the only
# difference is accumulation order: tight.
TOL_VS_FP32 = 6e-3
TOL_VS_FP16_EMU = 2.5e-3   # fp16 rounding-boundary flips propagate through 17-20 layers


def run_denoise(ctx, w, x):
    import torch
    ctx.set_denoiser(w)
    B, C, H, W = x.shape
    dx = torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()
    dy = torch.empty_like(dx)
    ctx.op_denoise(dx.data_ptr(), dy.data_ptr(), B, C, H, W)
    torch.cuda.synchronize()
    ctx.synchronize()
    return dy.cpu().numpy()


@pytest.mark.parametrize("name", ["DnCNN_nobn_nch_3_nlev_0.01", "DnCNN_nobn_nch_1_nlev_0.01",
                                  "dncnn_color_blind", "dncnn_15"])
def test_denoiser_golden(gpu_ctx, golden_denoiser, name):
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    xin = golden_denoiser[f"in_{name}"]
    x4 = xin.reshape((1, 1) + xin.shape) if xin.ndim == 2 else xin[None]
    out = run_denoise(gpu_ctx, w, x4).reshape(xin.shape)
    ref = golden_denoiser[f"out_{name}"]
    scale = max(1.0, float(np.abs(ref).max()))
    assert np.abs(out - ref).max() <= TOL_VS_FP32 * scale
    emu = O.OracleDenoiser(w, emulate_fp16=True).forward_batch(x4).reshape(xin.shape)
    assert np.abs(out - emu).max() <= TOL_VS_FP16_EMU * scale


@pytest.mark.parametrize("B,C,H,W", [(3, 3, 50, 70), (2, 1, 33, 31), (1, 3, 8, 32), (5, 3, 64, 96)])
def test_denoiser_ragged_batched(gpu_ctx, B, C, H, W):
    """Partial tiles (H % 8, W % 32 != 0), tiny images, several images per launch."""
    rng = np.random.default_rng(B * 100 + H)
    w = random_weights(C, depth=6, seed=H, scale=0.9)
    x = rng.uniform(-0.1, 1.1, (B, C, H, W)).astype(np.float32)
    out = run_denoise(gpu_ctx, w, x)
    emu = O.OracleDenoiser(w, emulate_fp16=True).forward_batch(x)
    np.testing.assert_allclose(out, emu, atol=TOL_VS_FP16_EMU)
    # images are independent: each one alone gives the same bits
    one = run_denoise(gpu_ctx, w, x[B - 1:B])
    np.testing.assert_array_equal(one[0], out[B - 1])


# fp32 operands (PNP_PREC_FP32, v_mfma_f32_32x32x2_f32: exact fp32 FMA chains) vs the
# reference's fp32 conv: only the summation order differs.
TOL_FP32 = 1e-5


@pytest.mark.parametrize("name", ["DnCNN_nobn_nch_3_nlev_0.01", "DnCNN_nobn_nch_1_nlev_0.01",
                                  "dncnn_color_blind", "dncnn_15"])
def test_denoiser_fp32_golden(gpu_ctx, golden_denoiser, name):
    """The fp32-operand path against the reference's own denoiser outputs (denoiser.npz,
    made by the imported reference) and the fp32 oracle."""
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    xin = golden_denoiser[f"in_{name}"]
    x4 = xin.reshape((1, 1) + xin.shape) if xin.ndim == 2 else xin[None]
    gpu_ctx.set_precision("fp32")
    try:
        out = run_denoise(gpu_ctx, w, x4).reshape(xin.shape)
    finally:
        gpu_ctx.set_precision("fp16")
    ref = golden_denoiser[f"out_{name}"]
    scale = max(1.0, float(np.abs(ref).max()))
    err = float(np.abs(out - ref).max())
    print(f"{name}: fp32 path max|d| vs reference = {err:.2e}")
    assert err <= TOL_FP32 * scale
    o32 = O.OracleDenoiser(w).forward_batch(x4).reshape(xin.shape)
    assert np.abs(out - o32).max() <= TOL_FP32 * scale


@pytest.mark.parametrize("name", ["DnCNN_nobn_nch_3_nlev_0.01", "dncnn_15"])
@pytest.mark.parametrize("B,C,H,W", [(3, 3, 50, 70), (2, 3, 256, 256), (1, 3, 8, 32)])
def test_denoiser_fp16w2(gpu_ctx, name, B, C, H, W):
    """Split weights (PNP_PREC_FP16W2): against the oracle emulating the same numerics (fp16
    activations, fp16 hi + lo weights) to the fp16-activation tolerance, closer to the fp32
    reference than the plain fp16 path, batch vs single bits."""
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    if w.channels != C:
        C = w.channels
    rng = np.random.default_rng(B * 7 + H)
    x = rng.uniform(0, 1, (B, C, H, W)).astype(np.float32)
    gpu_ctx.set_precision("fp16w2")
    try:
        out = run_denoise(gpu_ctx, w, x)
        one = run_denoise(gpu_ctx, w, x[B - 1:B])
    finally:
        gpu_ctx.set_precision("fp16")
    emu = O.OracleDenoiser(w, emulate_fp16="w2").forward_batch(x)
    np.testing.assert_allclose(out, emu, atol=TOL_VS_FP16_EMU)
    np.testing.assert_array_equal(one[0], out[B - 1])
    ref = O.OracleDenoiser(w).forward_batch(x)
    e16 = np.abs(O.OracleDenoiser(w, emulate_fp16=True).forward_batch(x) - ref).mean()
    assert np.abs(out - ref).mean() < e16          # on average nearer fp32 than fp16 weights


# split fp16 (PNP_PREC_FP16X3, conv_s3.hip): activations and weights as fp16 hi + lo pairs,
# three MFMAs per product.  ~21 significant bits on both operands (the lo halves of small
# values are fp16 subnormals), so it sits between the fp32 path and fp16w2.
TOL_X3 = 5e-5


@pytest.mark.parametrize("name", ["DnCNN_nobn_nch_3_nlev_0.01", "DnCNN_nobn_nch_1_nlev_0.01",
                                  "dncnn_color_blind", "dncnn_15"])
def test_denoiser_fp16x3_golden(gpu_ctx, golden_denoiser, name):
    """The split-fp16 path against the reference's own denoiser outputs and the fp32 oracle."""
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    xin = golden_denoiser[f"in_{name}"]
    x4 = xin.reshape((1, 1) + xin.shape) if xin.ndim == 2 else xin[None]
    gpu_ctx.set_precision("fp16x3")
    try:
        out = run_denoise(gpu_ctx, w, x4).reshape(xin.shape)
    finally:
        gpu_ctx.set_precision("fp16")
    ref = golden_denoiser[f"out_{name}"]
    scale = max(1.0, float(np.abs(ref).max()))
    err = float(np.abs(out - ref).max())
    e16 = float(np.abs(O.OracleDenoiser(w, emulate_fp16=True).forward_batch(x4).reshape(xin.shape) - ref).max())
    print(f"{name}: fp16x3 path max|d| vs reference = {err:.2e} (fp16 operands: {e16:.2e})")
    assert err <= TOL_X3 * scale
    o32 = O.OracleDenoiser(w).forward_batch(x4).reshape(xin.shape)
    assert np.abs(out - o32).max() <= TOL_X3 * scale


@pytest.mark.parametrize("B,C,H,W", [(3, 3, 50, 70), (2, 1, 33, 31), (1, 3, 8, 16), (1, 1, 5, 7), (2, 3, 256, 256),
                                     (4, 3, 41, 100)])
def test_denoiser_fp16x3_ragged_batched(gpu_ctx, B, C, H, W):
    """Split fp16: partial 8 x 16 tiles, tiny images, several images per launch, against the
    fp32 oracle; each image alone gives the batch's bits."""
    rng = np.random.default_rng(B * 100 + H + 9)
    w = random_weights(C, depth=6, seed=H + 1, scale=0.9)
    x = rng.uniform(-0.1, 1.1, (B, C, H, W)).astype(np.float32)
    gpu_ctx.set_precision("fp16x3")
    try:
        out = run_denoise(gpu_ctx, w, x)
        one = run_denoise(gpu_ctx, w, x[B - 1:B])
    finally:
        gpu_ctx.set_precision("fp16")
    ref = O.OracleDenoiser(w).forward_batch(x)
    print(f"fp16x3 {B}x{C}x{H}x{W}: max|d| vs fp32 oracle = {np.abs(out - ref).max():.2e}")
    np.testing.assert_allclose(out, ref, atol=TOL_X3)
    np.testing.assert_array_equal(one[0], out[B - 1])


@pytest.mark.parametrize("B,C,H,W", [(3, 3, 50, 70), (2, 1, 33, 31), (1, 3, 8, 16), (1, 1, 5, 7), (2, 3, 256, 256),
                                     (4, 3, 41, 100)])
def test_denoiser_fp16a2_ragged_batched(gpu_ctx, B, C, H, W):
    """fp16a2 (PNP_PREC_FP16A2, the converge mode's second phase): split activations, fp16 body
    weights, two MFMAs per product, two M-subtiles per wave.  Against the oracle emulating it (fp16
    body weights, fp32 activations) at split fp16's tolerance, nearer that than fp32; partial 8 x 16
    tiles, tiny images; each image alone gives the batch's bits."""
    rng = np.random.default_rng(B * 100 + H + 11)
    w = random_weights(C, depth=6, seed=H + 3, scale=0.9)
    x = rng.uniform(-0.1, 1.1, (B, C, H, W)).astype(np.float32)
    gpu_ctx.set_precision("fp16a2")
    try:
        out = run_denoise(gpu_ctx, w, x)
        one = run_denoise(gpu_ctx, w, x[B - 1:B])
    finally:
        gpu_ctx.set_precision("fp16")
    emu = O.OracleDenoiser(w, emulate_fp16="a2").forward_batch(x)
    ref = O.OracleDenoiser(w).forward_batch(x)
    print(f"fp16a2 {B}x{C}x{H}x{W}: max|d| vs its emulation {np.abs(out - emu).max():.2e}, vs fp32 "
          f"{np.abs(out - ref).max():.2e}")
    np.testing.assert_allclose(out, emu, atol=TOL_X3)
    np.testing.assert_array_equal(one[0], out[B - 1])


@pytest.mark.parametrize("name", ["DnCNN_nobn_nch_3_nlev_0.01", "dncnn_color_blind"])
def test_denoiser_fp16a2_golden(gpu_ctx, golden_denoiser, name):
    """fp16a2 against the reference's own denoiser outputs: within the fp16 path's bound, and closer
    than fp16 operands."""
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    xin = golden_denoiser[f"in_{name}"]
    x4 = xin.reshape((1, 1) + xin.shape) if xin.ndim == 2 else xin[None]
    gpu_ctx.set_precision("fp16a2")
    try:
        out = run_denoise(gpu_ctx, w, x4).reshape(xin.shape)
    finally:
        gpu_ctx.set_precision("fp16")
    ref = golden_denoiser[f"out_{name}"]
    err = float(np.abs(out - ref).max())
    e16 = float(np.abs(O.OracleDenoiser(w, emulate_fp16=True).forward_batch(x4).reshape(xin.shape) - ref).max())
    emu = O.OracleDenoiser(w, emulate_fp16="a2").forward_batch(x4).reshape(xin.shape)
    print(f"{name}: fp16a2 max|d| vs reference {err:.2e} (fp16 operands {e16:.2e}), vs its emulation "
          f"{np.abs(out - emu).max():.2e}")
    assert err < e16
    assert np.abs(out - emu).max() <= TOL_X3 * max(1.0, float(np.abs(ref).max()))


@pytest.mark.parametrize("B,C,H,W", [(3, 3, 50, 70), (2, 1, 33, 31), (1, 3, 8, 32), (2, 3, 256, 256)])
def test_denoiser_fp32_ragged_batched(gpu_ctx, B, C, H, W):
    """fp32 path: partial tiles, tiny images, several images per launch; batch vs single bits."""
    rng = np.random.default_rng(B * 100 + H + 7)
    w = random_weights(C, depth=6, seed=H, scale=0.9)
    x = rng.uniform(-0.1, 1.1, (B, C, H, W)).astype(np.float32)
    gpu_ctx.set_precision("fp32")
    try:
        out = run_denoise(gpu_ctx, w, x)
        one = run_denoise(gpu_ctx, w, x[B - 1:B])
    finally:
        gpu_ctx.set_precision("fp16")
    ref = O.OracleDenoiser(w).forward_batch(x)
    np.testing.assert_allclose(out, ref, atol=TOL_FP32)
    np.testing.assert_array_equal(one[0], out[B - 1])


@pytest.mark.parametrize("name,B,C,H,W", [("DnCNN_nobn_nch_3_nlev_0.01", 3, 3, 50, 70),
                                          ("DnCNN_nobn_nch_3_nlev_0.01", 2, 3, 256, 256),
                                          ("dncnn_15", 2, 1, 37, 45), ("DnCNN_nobn_nch_1_nlev_0.01", 1, 1, 8, 32),
                                          ("dncnn_color_blind", 1, 3, 9, 33), ("DnCNN_nobn_nch_3_nlev_0.01", 1, 3, 64, 96),
                                          # more strips than CUs: workgroups chain strips of different
                                          # images / columns into one row stream (2-3 strips each)
                                          ("DnCNN_nobn_nch_3_nlev_0.01", 90, 3, 20, 70), ("dncnn_15", 300, 1, 9, 33)])
def test_body_two_layers_per_launch_bit_identical(gpu_ctx, name, B, C, H, W):
    """conv_body_f2 (two 64->64 layers per launch, the intermediate in LDS) runs each output's
    MFMA K-sequence and the intermediate's fp16 rounding exactly as two conv_body_v3 launches:
    same bits, for ragged shapes (H % 8, W % 32 != 0, images narrower than a strip), odd
    layer counts (dncnn_15: 15 body layers), both activations, and batches with more strips
    than CUs (each workgroup chains several strips)."""
    rng = np.random.default_rng(11)
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    x = rng.uniform(0, 1, (B, C, H, W)).astype(np.float32)
    gpu_ctx.set_body_layers(1)
    try:
        single = run_denoise(gpu_ctx, w, x)
        gpu_ctx.set_body_layers(2)
        fused = run_denoise(gpu_ctx, w, x)
    finally:
        gpu_ctx.set_body_layers(0)
    np.testing.assert_array_equal(fused, single)


@pytest.mark.parametrize("depth,act,residual,clamp,B,C,H,W",
                         [(20, 0, +1, 1, 2, 3, 256, 256), (20, 0, +1, 1, 3, 3, 50, 70), (6, 1, -1, 0, 2, 1, 37, 45),
                          (6, 0, +1, 1, 1, 1, 8, 32), (4, 1, -1, 0, 1, 3, 9, 33), (20, 1, +1, 0, 90, 3, 20, 70),
                          (6, 0, -1, 1, 300, 1, 9, 33), (8, 0, +1, 1, 5, 3, 64, 96),
                          (6, 0, +1, 1, 40, 3, 5, 40)])      # H + 1 < 24: strips padded to 24 rows (a step looks ahead at most one strip)
def test_head_tail_inside_pair_launches_bit_identical(gpu_ctx, depth, act, residual, clamp, B, C, H, W):
    """conv_body_x8_kernel's HEAD / TAIL modes (the head inside the first two-layer launch, the
    tail inside the last: PNP_TUNE_FUSE_ENDS) give the separate conv_head / conv_tail launches'
    bits: both activations, both residual signs, clamp on / off, ragged shapes, images narrower
    than a strip, several strips per workgroup."""
    rng = np.random.default_rng(depth * 7 + B)
    w = random_weights(C, depth=depth, seed=B + H, scale=0.9)
    w.act, w.residual, w.clamp_io = act, residual, clamp
    x = rng.uniform(-0.1, 1.1, (B, C, H, W)).astype(np.float32)
    if clamp:
        x = np.clip(x, 0, 1)
    try:
        gpu_ctx.set_body_layers(2)
        gpu_ctx.set_fuse_ends(0)
        apart = run_denoise(gpu_ctx, w, x)
        gpu_ctx.set_fuse_ends(1)
        fused = run_denoise(gpu_ctx, w, x)
        fused2 = run_denoise(gpu_ctx, w, x)
    finally:
        gpu_ctx.set_body_layers(0)
        gpu_ctx.set_fuse_ends(1)
    np.testing.assert_array_equal(fused, apart)
    np.testing.assert_array_equal(fused2, apart)
    emu = O.OracleDenoiser(w, emulate_fp16=True).forward_batch(x[:1])
    np.testing.assert_allclose(fused[:1], emu, atol=TOL_VS_FP16_EMU)


@pytest.mark.parametrize("name,B,C,H,W", [("DnCNN_nobn_nch_3_nlev_0.01", 1, 3, 256, 256),     # 256 tiles: 1 per CU
                                          ("DnCNN_nobn_nch_1_nlev_0.01", 2, 1, 256, 256),     # 512: 2 per workgroup
                                          ("DnCNN_nobn_nch_3_nlev_0.01", 3, 3, 256, 256),     # 768: 3 per workgroup
                                          ("dncnn_15", 2, 1, 37, 45),                         # odd layer count
                                          ("dncnn_color_blind", 1, 3, 9, 33),                 # ReLU, tiny image
                                          ("DnCNN_nobn_nch_3_nlev_0.01", 3, 3, 50, 70)])      # ragged tiles
@pytest.mark.parametrize("mode", [3, 4])
def test_body_all_layers_one_launch_bit_identical(gpu_ctx, name, B, C, H, W, mode):
    """Every body layer in one persistent launch, tiles handed between workgroups through
    per-tile progress words: conv_stack16x2 (mode 3: two layers per hand-off, the intermediate
    in LDS; odd layer counts fall back to one) and conv_stack16 (mode 4: one layer per hand-off)
    give the one-layer launches' bits."""
    rng = np.random.default_rng(12)
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    x = rng.uniform(0, 1, (B, C, H, W)).astype(np.float32)
    try:
        gpu_ctx.set_body_layers(1)
        single = run_denoise(gpu_ctx, w, x)
        gpu_ctx.set_body_layers(mode)
        stack = run_denoise(gpu_ctx, w, x)
        stack2 = run_denoise(gpu_ctx, w, x)          # a second launch: the next epoch of the progress words
    finally:
        gpu_ctx.set_body_layers(0)
    np.testing.assert_array_equal(stack, single)
    np.testing.assert_array_equal(stack2, single)


def test_denoiser_full_size_rgb(gpu_ctx):
    """256x256 RGB, real weights, batch 2 — the metric's image shape."""
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, "DnCNN_nobn_nch_3_nlev_0.01.npz"))
    rng = np.random.default_rng(3)
    yy, xx = np.meshgrid(np.linspace(0, 1, 256), np.linspace(0, 1, 256), indexing="ij")
    clean = np.stack([0.5 + 0.3 * np.sin(6 * xx + c) * np.cos(4 * yy) for c in range(3)])
    x = np.stack([clean + 0.01 * rng.standard_normal(clean.shape) for _ in range(2)]).astype(np.float32)
    out = run_denoise(gpu_ctx, w, x)
    ref = O.OracleDenoiser(w).forward_batch(x)
    assert np.abs(out - ref).max() < TOL_VS_FP32
    # the denoiser denoises: closer to the clean image than its input
    assert np.mean((out[0] - clean) ** 2) < np.mean((x[0] - clean) ** 2)


@pytest.mark.parametrize("name,B,C,H,W", [("DnCNN_nobn_nch_1_nlev_0.01", 1, 1, 256, 256),     # 512 tiles: 2 per WG
                                          ("DnCNN_nobn_nch_3_nlev_0.01", 1, 3, 64, 96),
                                          ("dncnn_15", 2, 1, 37, 45),                         # odd layer count
                                          ("dncnn_color_blind", 1, 3, 9, 33),                 # ReLU, tiny image
                                          ("DnCNN_nobn_nch_3_nlev_0.01", 3, 3, 256, 256)])    # 1536 tiles: 6 per WG
@pytest.mark.parametrize("prec", ["fp16x3", "fp16a2"])
def test_fp16x3_all_layers_one_launch_bit_identical(gpu_ctx, name, B, C, H, W, prec):
    """conv_stack_s3 (every split-fp16 body layer in one persistent launch) gives the bits of
    one conv_s3 launch per layer, with (fp16x3) and without (fp16a2) the w_lo term."""
    rng = np.random.default_rng(13)
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, name + ".npz"))
    x = rng.uniform(0, 1, (B, C, H, W)).astype(np.float32)
    gpu_ctx.set_precision(prec)
    try:
        gpu_ctx.set_body_layers(1)
        single = run_denoise(gpu_ctx, w, x)
        gpu_ctx.set_body_layers(3)
        stack = run_denoise(gpu_ctx, w, x)
        stack2 = run_denoise(gpu_ctx, w, x)
    finally:
        gpu_ctx.set_body_layers(0)
        gpu_ctx.set_precision("fp16")
    np.testing.assert_array_equal(stack, single)
    np.testing.assert_array_equal(stack2, single)


@pytest.mark.parametrize("prec", ["fp16", "fp16x3"])
def test_op_denoise_side_stream_equals_context_stream(gpu_ctx, prec):
    """A single denoise on the context's stream (NULL) may take the persistent all-layers
    kernel at a small batch; on a caller's stream it takes the per-layer launches (only the
    context's stream runs persistent grids, so two of them never compete for CUs).  Both give
    the same bits, and pnp_op_status reports success on both streams."""
    import torch
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, "DnCNN_nobn_nch_3_nlev_0.01.npz"))
    rng = np.random.default_rng(11)
    x = rng.uniform(0, 1, (1, 3, 64, 96)).astype(np.float32)
    gpu_ctx.set_denoiser(w)
    prev = gpu_ctx.precision
    gpu_ctx.set_precision(prec)
    try:
        dx = torch.from_numpy(x).cuda()
        d0, d1 = torch.empty_like(dx), torch.empty_like(dx)
        gpu_ctx.op_denoise(dx.data_ptr(), d0.data_ptr(), 1, 3, 64, 96)        # the context's stream
        gpu_ctx.op_status()
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        gpu_ctx.op_denoise(dx.data_ptr(), d1.data_ptr(), 1, 3, 64, 96, stream=s.cuda_stream)
        gpu_ctx.op_status(stream=s.cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d0.cpu().numpy(), d1.cpu().numpy())
    finally:
        gpu_ctx.set_precision(prev)


def test_fused_ends_with_denoiser_passes_same_bits(gpu_ctx):
    """The batch split into denoiser passes (PNP_TUNE_DENOISE_CHUNK 3 -> passes of 3, 3, 1) with
    the head / tail inside the two-layer launches: every image as in one pass, and as with
    separate head / tail launches."""
    w = DenoiserWeights.load_npz(os.path.join(WEIGHTS_DIR, "DnCNN_nobn_nch_3_nlev_0.01.npz"))
    x = np.random.default_rng(31).uniform(0, 1, (7, 3, 40, 72)).astype(np.float32)
    try:
        gpu_ctx.set_body_layers(2)
        whole = run_denoise(gpu_ctx, w, x)
        gpu_ctx.set_denoise_chunk(3)
        passes = run_denoise(gpu_ctx, w, x)
        gpu_ctx.set_fuse_ends(0)
        apart = run_denoise(gpu_ctx, w, x)
    finally:
        gpu_ctx.set_denoise_chunk(0)
        gpu_ctx.set_fuse_ends(1)
        gpu_ctx.set_body_layers(0)
    np.testing.assert_array_equal(passes, whole)
    np.testing.assert_array_equal(apart, whole)
