// Denoiser forward on MFMA: implicit-GEMM 3x3 convolutions for gfx950.
//
// Reference: models/basic_models.py:25-38 (simple_CNN.forward: in_conv + LeakyReLU,
// 18 x [conv + LeakyReLU], out_conv + x_in) and models/denoiser.py:34-46 (clamp in/out);
// KAIR variant models/network_dncnn.py:42-77 (ReLU, x - n, no clamps).
//
// GEMM view per layer: D[cout][pixel] = sum_k W[cout][k] * X[k][pixel], k = (tap, cin).
// A operand = host-packed weights (MFMA fragment order), B operand = activations from an
// LDS halo tile, fp16 operands, fp32 accumulation (v_mfma_f32_32x32x16_f16 for the
// 64-channel layers, v_mfma_f32_16x16x32_f16 for the 64 -> C tail).
//
// Hidden activations are fp16 NHWC64 images with a zero border of s.pad = 2 pixels (each
// pixel one 128-B line).
//
//   conv_head      C -> 64, from the fp32 NCHW input u32 (fp16 conversion in the halo fill)
//   conv_body_v3   64 -> 64, one layer per launch
//   conv_tail      64 -> C + residual + clamp, fp32 NCHW out
// (conv32.hip holds the fp32-operand path, PNP_PREC_FP32.)
#include "kernels.h"

namespace pnp {

__device__ __forceinline__ void decode_tile(int t, const ConvShape& s, int& b, int& ty0, int& tx0) {
  const int per_img = s.tiles_x * s.tiles_y;
  b = t / per_img;
  const int r = t - b * per_img;
  const int ty = r / s.tiles_x;
  ty0 = ty * kTileH;
  tx0 = (r - ty * s.tiles_x) * kTileW;
}

// Epilogue of the head: bias + activation, fp16, two 16-B stores per M-tile into the
// padded NHWC64 output.  Lane (col, h) owns channels 32m+16h .. +15.
__device__ __forceinline__ void store_act64(half_t* __restrict__ out, const ConvShape& s, int b, int y,
                                            int x, int h, const floatx16& acc0, const floatx16& acc1,
                                            const float (&bias)[2][16], int act) {
  if (y >= s.H || x >= s.W) return;
  half_t* o = out + (((size_t)b * s.Hp + y + s.pad) * s.Wp + x + s.pad) * kWidth + 16 * h;
  half8_t v0, v1, v2, v3;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    v0[r] = (half_t)act_fn(acc0[r] + bias[0][r], act);
    v1[r] = (half_t)act_fn(acc0[r + 8] + bias[0][r + 8], act);
    v2[r] = (half_t)act_fn(acc1[r] + bias[1][r], act);
    v3[r] = (half_t)act_fn(acc1[r + 8] + bias[1][r + 8], act);
  }
  *reinterpret_cast<half8_t*>(o) = v0;
  *reinterpret_cast<half8_t*>(o + 8) = v1;
  *reinterpret_cast<half8_t*>(o + 32) = v2;
  *reinterpret_cast<half8_t*>(o + 40) = v3;
}


// XCD-aware tile order for a persistent grid: workgroup b runs on XCD b % 8, so logical
// block (b % 8) * (G / 8) + b / 8 gives each XCD a contiguous run of G / 8 tiles per round
// (neighbouring tiles, whose halos overlap, share one L2).  Identity when G % 8 != 0.
__device__ __forceinline__ int xcd_block(int b, int G) {
  return (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3);
}

// bias + activation of 8 accumulator rows -> 8 fp16 (packed adds/muls; LeakyReLU(x) = max(x, 0.01x),
// ReLU(x) = max(x, 0): bit-identical to act_fn, half the VALU of the select form)
typedef float f2v_t __attribute__((ext_vector_type(2)));
template <int ACT>
__device__ __forceinline__ half8_t bias_act8(const floatx16& a, int off, const float* bl) {
  half8_t o;
#pragma unroll
  for (int r = 0; r < 8; r += 2) {
    f2v_t v = f2v_t{a[off + r], a[off + r + 1]} + f2v_t{bl[r], bl[r + 1]};
    if (ACT == 0) {
      const f2v_t t = v * 0.01f;
      v = f2v_t{fmaxf(v.x, t.x), fmaxf(v.y, t.y)};
    } else {
      v = f2v_t{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f)};
    }
    o[r] = (half_t)v.x;
    o[r + 1] = (half_t)v.y;
  }
  return o;
}

// bias + activation of NV accumulator rows a[off + NV q ..] into o[NV q ..], scalar fp32 (beside
// MFMAs packed fp32 VALU costs extra issue cycles: MI355X_MICROARCH.md); same values as bias_act8
template <int ACT, int NV>
__device__ __forceinline__ void bias_act_s(half8_t& o, int q, const floatx16& a, int off, const float* bl) {
#pragma unroll
  for (int r = 0; r < NV; ++r) {
    const float v = a[off + NV * q + r] + bl[NV * q + r];
    o[NV * q + r] = (half_t)(ACT == 0 ? fmaxf(v, v * 0.01f) : fmaxf(v, 0.f));
  }
}

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));

// Epilogue of the fp16 body layers (conv_body_x8 / conv_body_v3 / conv_stack16; round 3).  The
// bias is the C operand of a tile's first MFMA, so the accumulator already holds conv + bias;
// the activation runs on the fp16-rounded pair in packed fp16: LeakyReLU(h) = max(h, h * 0.01h),
// ReLU(h) = max(h, 0).  Three single-pass VALU ops per pair (v_cvt_pk_f16_f32, v_pk_mul_f16,
// v_pk_max_f16) instead of five with fp32 packed ops (bias add, 0.01x, two maxes, cvt).  The
// kernels run at the chip's power limit, where fewer VALU instructions per MFMA return as clock:
// conv_body_x8 2.316 -> 2.215 ms per launch at the metric (A/B, r03).  ReLU is bit-identical to
// rounding after the fp32 activation; LeakyReLU's negative branch multiplies by fp16(0.01) =
// 0.0100021 in fp16 (≤ 1 fp16 ulp from fp16(0.01 v)), the same in all three kernels, so they
// stay bit-identical to each other (tests/test_gpu_graph.py, test_gpu_denoiser.py).
typedef _Float16 h2v_t __attribute__((ext_vector_type(2)));
template <int ACT>
__device__ __forceinline__ h2v_t act_h2(f2v_t v) {
  const h2v_t h = __builtin_convertvector(v, h2v_t);
  return ACT == 0 ? __builtin_elementwise_max(h, h * (h2v_t){(_Float16)0.01f, (_Float16)0.01f})
                  : __builtin_elementwise_max(h, (h2v_t){(_Float16)0.f, (_Float16)0.f});
}
// 8 accumulator rows a[off .. off + 7] (bias included) -> 8 x fp16
template <int ACT>
__device__ __forceinline__ half8_t act8_h(const floatx16& a, int off) {
  half8_t o;
#pragma unroll
  for (int r = 0; r < 8; r += 2) {
    const h2v_t hv = act_h2<ACT>(f2v_t{a[off + r], a[off + r + 1]});
    o[r] = hv.x;
    o[r + 1] = hv.y;
  }
  return o;
}
__device__ __forceinline__ floatx16 bias16(const float* bl) {     // C operand: rows = bl[0 .. 15]
  floatx16 c;
#pragma unroll
  for (int r = 0; r < 16; ++r) c[r] = bl[r];
  return c;
}

// ------------------------------------------------------------------------------------
// LDS-DMA halo staging (buffer_load_dword... lds).  The 10 x 34 halo of an 8 x 32 tile
// is 340 pixels = 43 slots of 8 pixels (1 KiB); lane l of a slot loads 16-B chunk
// (l&7) ^ swz(pc) of pixel 8g + l/8 into the lane-linear destination, so the LDS image is
// the XOR-swizzled layout of halo_off() (common.h).  The tile base is in SGPRs and the
// per-lane offsets of a wave's slots are tile-invariant (computed once per launch).
// ------------------------------------------------------------------------------------
constexpr int kDmaSlots = (kHaloPix + 7) / 8;                 // 43
constexpr int kV3Halo = kHaloPix * 128;                        // 43520: slot 42 is issued by half a wave

template <int NW>
__device__ __forceinline__ int dma_count(int wave) {           // slots issued by `wave`
  return (kDmaSlots - wave + NW - 1) / NW;
}

// UNIFORM: every wave issues kSlots (the extra slots re-read pixel 339 into padding past
// the halo), so the issue has no control flow and the compiler's own vmcnt accounting for
// loads issued before it stays exact; the buffer must then hold NW * kSlots KiB.
template <int NW, bool UNIFORM = false, int SWZ = 0>
struct RingDma {                                               // one wave's share of a halo DMA
  static constexpr int kSlots = (kDmaSlots + NW - 1) / NW;     // NW=8: 6 (waves >= 3: 5); NW=4: 11 (wave 3: 10)
  unsigned off[kSlots];
  __device__ __forceinline__ void init(const ConvShape& s, int wave) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < kSlots; ++j) {
      const int p = 8 * (NW * j + wave) + (lane >> 3);
      const int pl = min(p, kHaloPix - 1);
      const int pr = pl / kHaloW, pc = pl - pr * kHaloW;
      const int c = (lane & 7) ^ (SWZ ? (pc & 6) : ((pc >> 1) & 7));
      off[j] = (unsigned)(((pr * s.Wp + pc) * kWidth + c * 8) * 2);
    }
  }
  // one slot of the DMA of tile t (issue() = every slot), for spreading the slots over a K-loop
  __device__ __forceinline__ static __amdgpu_buffer_rsrc_t rsrc(const half_t* __restrict__ in, const ConvShape& s,
                                                                int t) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const half_t* base = in + (((size_t)b * s.Hp + ty0 + s.pad - 1) * s.Wp + tx0 + s.pad - 1) * kWidth;
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
  }
  __device__ __forceinline__ void issue_slot(unsigned char* hl, __amdgpu_buffer_rsrc_t rs, int j, int wave) const {
    const int g = NW * j + wave;
    if (UNIFORM || g < kDmaSlots - 1 || (g == kDmaSlots - 1 && (threadIdx.x & 63) < 32))
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(hl + g * 1024), 16,
                                               off[j], 0, 0, 0);
  }
  template <int CPOL = 0>
  __device__ __forceinline__ void issue(unsigned char* hl, const half_t* __restrict__ in, const ConvShape& s, int t,
                                        int wave) const {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    // halo origin: image pixel (ty0 - 1, tx0 - 1) = padded (ty0 + pad - 1, tx0 + pad - 1)
    const half_t* base = in + (((size_t)b * s.Hp + ty0 + s.pad - 1) * s.Wp + tx0 + s.pad - 1) * kWidth;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < kSlots; ++j) {
      const int g = NW * j + wave;
      if (UNIFORM || g < kDmaSlots - 1 || (g == kDmaSlots - 1 && lane < 32))   // slot 42: pixels 336..339
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(hl + g * 1024), 16,
                                                 off[j], 0, 0, CPOL);
    }
  }
};

// ------------------------------------------------------------------------------------
// Body layer (one per launch): weights in registers + 3-deep halo ring.
// 8 waves; wave w owns output channels 32m..32m+31 (m = w&1) of tile rows 2(w>>1) and
// 2(w>>1)+1, and keeps its 36 A-fragments (the whole K extent of its M-tile, 144 VGPRs) in
// registers for the launch, so the K-loop reads only 2 activation fragments per 2 MFMAs
// from LDS and the LDS holds three halo buffers: the DMA runs two tiles ahead.  Outputs go
// through a wave-private 4 KiB staging area (64-B half pixels, read back 16 pixels x 64 B
// per instruction) and are stored during the next tile's K-loop (range-checked buffer
// stores), so the only workgroup barrier per tile is the ring hand-over, after a counted
// vmcnt that waits for the next tile's DMA only.
// LDS: 3 x 42.5 KiB halo + 8 x 4 KiB staging + bias = 163584 B.
// (Round-1 alternatives measured slower and removed: weights in LDS with 4 or 8 waves,
// warp-specialised DMA waves, one wave per SIMD holding the whole layer, a channel-plane
// halo, the head computed into the first layer's LDS halo (1.82 ms vs 0.51 + 1.22 ms),
// DMA slots spread over the K-loop, full 128-B line stores through a shared staging tile,
// non-temporal stores, 16x16x32 MFMAs, a row Winograd F(2,3) form, two layers per launch
// with a 2-D intermediate tile, a staggered epilogue)
// ------------------------------------------------------------------------------------
constexpr int kV3Stage = 3 * kV3Halo;
constexpr int kV3Bias = kV3Stage + 8 * 4096;
constexpr int kV3Lds = kV3Bias + 256;                           // 163584 B

// ABL: bits 1/2/4 = profiling ablation, compile-time, instantiated only in the PNP_PROFILING
//      build (make PROFILING=1; results wrong): skip the halo DMA / the stores / the MFMAs.
// ACT: 0 = LeakyReLU(0.01) (simple_CNN), 1 = ReLU (KAIR DnCNN).
template <int ABL, int ACT>
__global__ __launch_bounds__(512, 2) void conv_body_v3_kernel(const half_t* __restrict__ in,
                                                               half_t* __restrict__ out,
                                                               const uint4* __restrict__ wpk,
                                                               const float* __restrict__ bias,
                                                               ConvShape s) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* bias_l = reinterpret_cast<float*>(smem + kV3Bias);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = wave & 1, rp = wave >> 1;    // M-tile, row pair
  const int h = lane >> 5, col = lane & 31;
  unsigned char* stg = smem + kV3Stage + wave * 4096;
  if (tid < kWidth) bias_l[tid] = bias[tid];

  half8_t wA[kBodyKSteps];                    // this wave's weights, resident for the launch
#pragma unroll
  for (int ks = 0; ks < kBodyKSteps; ++ks)
    wA[ks] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wpk) +
                                               ((ks * 2 + m) * 64 + lane) * 16);

  auto buf = [&](int i) { return smem + i * kV3Halo; };
  RingDma<8> dma;
  dma.init(s, wave);
  auto issue_dma = [&](int tt, int bi) {      // clamped: always the same instruction count
    dma.issue(buf(bi), in, s, tt < s.tiles ? tt : s.tiles - 1, wave);
  };
  const int ndma = dma_count<8>(wave);

  int t = xcd_block(blockIdx.x, gridDim.x);
  if (t < s.tiles) {
    issue_dma(t, 0);
    issue_dma(t + gridDim.x, 1);
    if (ndma == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // tile t landed
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  }
  __syncthreads();
  // Deferred stores of the previous tile: 16 pixels x 64 B (this wave's channel half) each.
  __amdgpu_buffer_rsrc_t rs[2];
  rs[0] = rs[1] = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000);   // first tile: dropped
  auto stage_read = [&](int j) {
    const int pix = 16 * j + (lane >> 2), c = lane & 3;
    return *reinterpret_cast<const v4i_t*>(stg + pix * 64 + 16 * (c ^ ((pix >> 1) & 3)));
  };
  auto stage_store = [&](int j, const v4i_t& v) {
    const int pix = 16 * j + (lane >> 2), c = lane & 3;
    if constexpr ((ABL & 2) == 0) __builtin_amdgcn_raw_buffer_store_b128(v, rs[j >> 1], (pix & 31) * 128 + 64 * m + 16 * c, 0, 0);
  };
  floatx16 acc0 = {}, acc1 = {};
  auto epilogue = [&](int eb, int ety0, int etx0) {   // activation -> fp16 -> staging (wave-private)
    const int sw = (col >> 1) & 3;    // ds_write_b128 banks repeat every 128 B: 8 lanes distinct
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int pix = n * 32 + col;
      const floatx16& a = n == 0 ? acc0 : acc1;
      *reinterpret_cast<half8_t*>(stg + pix * 64 + 16 * ((2 * h) ^ sw)) = act8_h<ACT>(a, 0);
      *reinterpret_cast<half8_t*>(stg + pix * 64 + 16 * ((2 * h + 1) ^ sw)) = act8_h<ACT>(a, 8);
    }
    const int ncols = min(kTileW, s.W - etx0);
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int y = ety0 + 2 * rp + n;
      half_t* row = out + (((size_t)eb * s.Hp + y + s.pad) * s.Wp + etx0 + s.pad) * kWidth;
      rs[n] = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
    }
  };
  int cur = 0;
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const int nxt2 = cur >= 1 ? cur - 1 : 2;  // (cur + 2) % 3
    if constexpr ((ABL & 1) == 0) issue_dma(t + 2 * gridDim.x, nxt2);
    const unsigned char* hl = buf(cur);
    auto ldB = [&](int ks, int n) {
      const int tap = ks >> 2, sub = ks & 3;
      return *reinterpret_cast<const half8_t*>(
          hl + halo_off(2 * rp + n + tap / 3, col + tap % 3, 2 * sub + h));
    };
    const floatx16 cb = *reinterpret_cast<const floatx16*>(bias_l + 32 * m + 16 * h);   // first MFMA's C
    half8_t fb[2][2];
    v4i_t sv;
#pragma unroll
    for (int k = 0; k < 1; ++k) { fb[k][0] = ldB(k, 0); fb[k][1] = ldB(k, 1); }
    if constexpr ((ABL & 4) != 0) {           // profiling: memory path only
#pragma unroll
      for (int j = 0; j < 4; ++j) stage_store(j, stage_read(j));
    } else
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks) {
      const int r = ks & 1;
      if ((ks & 7) == 2) {                    // previous tile's stores, one per 8 K-steps
        __builtin_amdgcn_sched_barrier(0);
        sv = stage_read(ks >> 3);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (ks + 1 < kBodyKSteps) {
        fb[r ^ 1][0] = ldB(ks + 1, 0);
        fb[r ^ 1][1] = ldB(ks + 1, 1);
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[r][0], ks == 0 ? cb : acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[r][1], ks == 0 ? cb : acc1, 0, 0, 0);
      if ((ks & 7) == 4) {
        __builtin_amdgcn_sched_barrier(0);
        stage_store(ks >> 3, sv);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    epilogue(b, ty0, tx0);
    // tile t+1 landed: only the DMA of t+2 (ndma ops) and this tile's 4 stores are younger
    if (ndma == 6) asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) stage_store(j, stage_read(j));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
}


#define PNP_V3_INST(A, F)                                                                                  \
  template __global__ void conv_body_v3_kernel<A, F>(const half_t* __restrict__, half_t* __restrict__,    \
                                                     const uint4* __restrict__, const float* __restrict__, \
                                                     ConvShape);
PNP_V3_INST(0, 0)
PNP_V3_INST(0, 1)
#ifdef PNP_PROFILING
PNP_V3_INST(1, 0)
PNP_V3_INST(2, 0)
PNP_V3_INST(3, 0)
PNP_V3_INST(4, 0)
PNP_V3_INST(6, 0)
#endif
#undef PNP_V3_INST

// ------------------------------------------------------------------------------------
// Two body layers per launch, streamed down 32-pixel-wide column strips (conv_body_f2).
// Layers l and l+1 of basic_models.py:29-33: the intermediate activation never leaves the
// CU.  A workgroup walks one strip (image b, columns x0 .. x0+31, all rows) in steps of 8
// rows; per step j
//   * waves 0-1 (layer l, one 32-channel M-tile each) compute intermediate rows 8j .. 8j+7
//     over columns x0-1 .. x0+32 (8 row N-tiles of 32 + one N-tile of the 16 halo pixels:
//     the only recompute is the strip's 2-column halo) from an 18-row input ring, and write them
//     (fp16, zero outside the image = the next layer's padding) into an 18-row LDS ring;
//   * waves 2-3 (layer l+1) compute output rows 8j-9 .. 8j-2 from intermediate rows computed
//     in earlier steps and store them to HBM;
//   * LDS-DMA brings input rows 8j+9 .. 8j+16 (the next step's) into ring rows no wave reads
//     in this step (16 buffer_load ... lds per wave, no registers);
//   * one workgroup barrier.
// The two layers run side by side on different SIMDs (one wave per SIMD; each wave keeps its
// layer's 36 A-fragments, 144 VGPRs, for the launch), so the HBM traffic per layer pair is
// one read (x 36/32 for the strip halo) and one write instead of two of each.
// Both rings are chunk-planar: plane c (c = 0..7) holds channels 8c .. 8c+7 of every ring
// pixel, 16 B per pixel, so a B fragment (16 pixels of one chunk per ds_read_b128 lane group)
// is 256 contiguous bytes (conflict-free without a swizzle) and the 36 fragment reads of an
// N-tile are one address register per tap row + immediate offsets (chunk plane, tap column).
// The K order per output and the fp16 rounding of the intermediate are those of conv_body_v3
// twice, so the result is bit-identical to two one-layer launches.
// LDS: input ring 18 x 36 px + intermediate ring 18 x 34 px, 128 B per pixel = 161280 B.
// ------------------------------------------------------------------------------------
constexpr int kF2Ring = 18;                                    // rows per ring
struct SGeom { int b, x0; };
constexpr int kF2InW = kTileW + 4, kF2MidW = kTileW + 2;       // 36, 34 pixels per ring row
// Chunk planes padded to multiples of 256 B: the 16x16x32 B fragments (conv_body_x8) read
// two planes per ds_read_b128 lane group, which then hit disjoint banks (unpadded: 2-way
// conflicts on every read); the two rings then fill the LDS exactly.
constexpr int kF2InPlane = (kF2Ring * kF2InW * 16 + 255) / 256 * 256;     // 10496 B per chunk plane
constexpr int kF2MidPlane = (kF2Ring * kF2MidW * 16 + 255) / 256 * 256;   // 9984
constexpr int kF2Mid = 8 * kF2InPlane;                         // 83968: intermediate ring offset
constexpr int kF2Lds = kF2Mid + 8 * kF2MidPlane;               // 163840 B: all of it

__device__ __forceinline__ int f2_slot(int row) { return (row + 1 + 18 * 64) % kF2Ring; }   // row >= -1 - 18*64


// ------------------------------------------------------------------------------------
// conv_body_x8: conv_body_f8's schedule on v_mfma_f32_16x16x32_f16 (MI355X_MICROARCH.md:
// under the chip's power limit this shape delivers ~1.12-1.15x the FLOP/s of 32x32x16 at
// equal cycles per FLOP).  K-step ks (18 of 32) = tap ks >> 1, channel half ks & 1; an
// N-subtile is 16 pixels; a wave's 32-channel M-tile is two 16-row A-subtiles sharing each
// B fragment.  A row r of subtile q is channel 8 (r >> 2) + 4 q + (r & 3) of the M-tile, so
// lane l ends with the 8 consecutive channels of chunk 4M + (l >> 4) of pixel l & 15: one
// 16-B store per lane and subtile.  The strip halo is exactly one N-subtile (16 pixels).
// Weights: pack_body_weights16, [18 ks][2 M-tiles][2 subtiles][64 lanes][8 x f16].
// ------------------------------------------------------------------------------------
constexpr int kX8KSteps = 18;
constexpr int kX8HeadFrag = 8192;     // HEAD mode: the head's fragments in the (quad-sized) input ring's LDS
constexpr int kX8HeadBias = kX8HeadFrag + kHeadWBytes;   // HEAD mode: the head's 64 biases after them
// Non-temporal output stores (A/B at the metric, r03, ms per launch): the head's 0.446 -> 0.439
// (kept); conv_body_x8 2.248 -> 2.267 and the tail unchanged (not kept).
constexpr int kNtX8 = 0, kNtTail = 0;                          // buffer-store cache policy (2 = nt)
constexpr bool kNtHead = true;
#ifdef X8_CLOCK
__device__ unsigned long long x8_clock[1024][2];   // per workgroup: shader-clock cycles, 100 MHz ticks
#endif

// Schedule choices measured by A/B builds in round 3 (the alternatives are in git
// history before round 4): fragment addresses as opaque VGPRs; groups of 3 N-subtiles with
// fragment prefetch depth 1; the strip-halo N-subtile's two A-subtiles split over the two
// halves' waves (306 MFMAs per SIMD and step each instead of 324 / 288); static s_setprio 1 for
// layer l+1's waves (2.182 -> 2.164 ms); layer l's zero-padding select skipped on interior
// steps; the step barrier without the store drain (lds_barrier).
// QL: the A-subtiles (bit q) computed for the last N-subtile (the strip halo's split).
template <int NT, int PLANE, class Side, int D = 2, int QL = 3>
__device__ __forceinline__ void x8_kloop(const half8_t (&wA)[kX8KSteps][2], const unsigned char* ring,
                                         const int (&ad)[NT][3], floatx4 (&acc)[NT][2], Side&& side,
                                         const floatx4 (&c0)[2]) {
  // One VGPR per (N-subtile, tap row), opaque to the compiler: otherwise it splits ad into the
  // lane part and the wave-uniform ring-row part and re-adds them (v_add_u32 SGPR + VGPR) for
  // every fragment read instead of folding the K-step's constant into the ds_read offset.
  int av[NT][3];
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      av[n][dy] = (int)(size_t)ring + ad[n][dy];          // LDS byte address
      asm volatile("" : "+v"(av[n][dy]));
    }
  typedef const __attribute__((address_space(3))) half8_t* lds_h8p;
  auto ldB = [&](int ks, int n) {
    const int tap = ks >> 1, hs = ks & 1, dy = tap / 3, dx = tap - 3 * dy;
    return *(lds_h8p)(size_t)(unsigned)(av[n][dy] + (4 * hs * PLANE + 16 * dx));
  };
  half8_t fb[D + 1][NT];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int n = 0; n < NT; ++n) fb[d][n] = ldB(d, n);
#pragma unroll
  for (int ks = 0; ks < kX8KSteps; ++ks) {
    if (ks + D < kX8KSteps) {
#pragma unroll
      for (int n = 0; n < NT; ++n) fb[(ks + D) % (D + 1)][n] = ldB(ks + D, n);
    }
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (n < NT - 1 || ((QL >> q) & 1))
          acc[n][q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wA[ks][q], fb[ks % (D + 1)][n],
                                                             ks == 0 ? c0[q] : acc[n][q], 0, 0, 0);
    side(ks);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// activation of a lane's chunk (acc[0] = channels +0..3, acc[1] = +4..7; bias included) -> 8 x fp16
template <int ACT>
__device__ __forceinline__ half8_t x8_act(const floatx4 (&a)[2]) {
  half8_t o;
#pragma unroll
  for (int r = 0; r < 8; r += 2) {
    const h2v_t hv = act_h2<ACT>(f2v_t{a[r >> 2][r & 3], a[r >> 2][(r & 3) + 1]});
    o[r] = hv.x;
    o[r + 1] = hv.y;
  }
  return o;
}

// MODE kX8Head: layer l is the head (C -> 64, conv_head_kernel's PREC 0 arithmetic: its packed
// weights, in LDS here, three v_mfma_f32_32x32x16_f16 per output from a zero accumulator over the
// fp16-rounded input quads, bias_act8) computed into the intermediate ring from the fp32 input,
// which every thread stages as fp16 quads (18 rows x 36 pixels x 8 B) one step ahead instead of the
// 64-channel DMA ring; layer l + 1 is the first body layer.  Every wave runs both: a quarter of
// the head's N-tiles and two of L0's output rows (the two waves of a SIMD in opposite orders).
// MODE kX8Tail: layer l is the last body layer and layer l + 1 the tail (conv_tail_kernel's
// arithmetic: 64 -> C on v_mfma_f32_16x16x32_f16 from a zero accumulator, + bias, +/- the fp32
// residual, clamp), storing x+ in fp32 NCHW; every wave runs a quarter of layer l's N-subtiles and
// one tail output row (its fragments streamed from L2).  Both give the bits of the separate head /
// tail launches around a plain pair, without the head's 2.15 GB write and the tail's 2.15 GB read
// at the metric.
template <int ACT, int MODE = kX8Pair>
__global__ __launch_bounds__(512, 1) void conv_body_x8_kernel(const half_t* __restrict__ in,
                                                               half_t* __restrict__ out,
                                                               const uint4* __restrict__ w1,
                                                               const float* __restrict__ b1,
                                                               const uint4* __restrict__ w2,
                                                               const float* __restrict__ b2, ConvShape s,
                                                               int strips_x, int nstrips, int srows, X8Ends ends) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ring = smem;
  unsigned char* mid = smem + kF2Mid;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int layer = wave >> 2, m = wave & 1, half = (wave >> 1) & 1;
  const int g = lane >> 4, px = lane & 15;               // chunk-in-M-tile, pixel of an N-subtile
  // HEAD: every wave runs L0 (M-tile m) and a share of the head, whose fragments sit in LDS;
  // TAIL: every wave runs L(n-1) and a share of the tail, whose fragments stream from L2
  const uint4* wsrc = MODE == kX8Head ? w2 : MODE == kX8Tail ? w1 : layer ? w2 : w1;
  half8_t wA[kX8KSteps][2];
#pragma unroll
  for (int ks = 0; ks < kX8KSteps; ++ks)
#pragma unroll
    for (int q = 0; q < 2; ++q)
      wA[ks][q] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wsrc) +
                                                    (((ks * 2 + m) * 2 + q) * 64 + lane) * 16);
  float bl[8];
  float tbl[MODE == kX8Tail ? kMaxC : 1];
  if (MODE == kX8Tail) {
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) tbl[c % (MODE == kX8Tail ? kMaxC : 1)] = c < ends.C ? ends.tb[c] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 8; ++r)
    bl[r] = (MODE == kX8Head ? b2 : MODE == kX8Tail ? b1 : layer ? b2 : b1)[32 * m + 8 * g + r];
  const floatx4 c0[2] = {floatx4{bl[0], bl[1], bl[2], bl[3]}, floatx4{bl[4], bl[5], bl[6], bl[7]}};   // first MFMA's C
  // The launch-constant registers are consumed here once, so the compiler's wait for their loads
  // sits before the step loop: its waitcnt pass does not read the inline-asm s_waitcnt below, and
  // otherwise put an s_waitcnt vmcnt(0) before the first MFMA of every step, which also waited
  // for that step's HEAD staging loads and the previous part's output stores (r06).
#pragma unroll
  for (int ks = 0; ks < kX8KSteps; ++ks) asm volatile("" ::"v"(wA[ks][0]), "v"(wA[ks][1]));
  asm volatile("" ::"v"(c0[0]), "v"(c0[1]));
  if (MODE == kX8Tail) {
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) asm volatile("" ::"v"(tbl[c % (MODE == kX8Tail ? kMaxC : 1)]));
  }
#ifdef X8_CLOCK   // diagnostic build (tools/x8_clock.py): shader clock vs the 100 MHz real-time clock
  unsigned long long c0_, r0_;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0_), "=s"(r0_)::"memory");
#endif
  const unsigned img_bytes = (unsigned)(s.Hp * s.Wp) * 128u;

  // strip k's row r is stream row k S + r; S = H + 1 (one zero separator row between strips,
  // the next strip's top halo and this one's bottom halo), so a step's 8 rows may straddle two
  // strips: masks and geometry are per row (round 5; strips were 8 ceil((H+1)/8) rows, an idle
  // layer-l step per strip at H = 256: 1 % of the launch)
  const int S = srows;
  // (An XCD-aware strip order, an image's neighbouring strips on CUs sharing one L2, measured
  // the same: 2.109 vs 2.108 ms, r03.)  HEAD takes it: its fp32 NCHW input rows are 144 B per
  // strip and channel over three 128-B lines, so strips on different XCDs fetched each line
  // about three times (0.55 GB per launch for 0.20 GB of input; 0.20 GB with this order, the
  // same time: 1.366-1.372 vs 1.359-1.366 ms, r06).
  const int bx = MODE == kX8Head ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const int K = (nstrips - bx + (int)gridDim.x - 1) / (int)gridDim.x;
  const int Jend = (K * S + 7) / 8;                      // the last step (layer l+1 only)
  auto geom = [&](int k) {
    const int st = min(bx + k * (int)gridDim.x, nstrips - 1);
    const int b = st / strips_x;
    return SGeom{b, (st - b * strips_x) * kTileW};
  };
  int kJ = 0;                                            // the strip of row 8 J
  int gpb, gpx, gcb, gcx, gnb, gnx;
  {
    const SGeom g0 = geom(0), g1 = geom(1);
    gpb = gcb = g0.b;
    gpx = gcx = g0.x0;
    gnb = g1.b;
    gnx = g1.x0;
  }
  auto pick = [&](int k) {
    const int pb = gpb, pxx = gpx, cb = gcb, cx = gcx, nb = gnb, nx = gnx;
    return SGeom{k > kJ ? nb : (k < kJ ? pb : cb), k > kJ ? nx : (k < kJ ? pxx : cx)};
  };
  auto locate = [&](int R, int kJ, int& k, int& r) {
    k = kJ;
    r = R - kJ * S;
    if (r < 0) { --k; r += S; } else if (r >= S) { ++k; r -= S; }
  };
  int J = 0;                                             // the step (rows 8 J .. 8 J + 7 of layer l)
  // layer-l row 8 J + p (p may vary by lane): whether it is an image row, and its strip's x0
  auto rowgeom = [&](int p, int& x0r) {
    int k, r;
    locate(8 * J + p, kJ, k, r);
    x0r = pick(k).x0;
    return k < K && r < s.H;
  };
  __amdgpu_buffer_rsrc_t dsrc;
  unsigned dvo;
  unsigned char* ddst;
  auto dma_at = [&](int R, int kJ) {
    int k, r;
    locate(R, kJ, k, r);
    const bool valid = R >= 0 && k < K;
    const SGeom G = pick(k);
    dsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(in + (size_t)G.b * s.Hp * s.Wp * kWidth), (short)0,
                                             valid ? (int)img_bytes : 0, 0x00020000);
    dvo = (unsigned)(((r + s.pad) * s.Wp + G.x0 + lane) * 128);
    ddst = ring + f2_slot(R) * (kF2InW * 16);
  };
  auto dma_plane = [&](int c) {
    if (lane < kF2InW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dsrc, (__attribute__((address_space(3))) void*)(ddst + c * kF2InPlane),
                                               16, dvo + 16 * c, 0, 0, 0);   // (nt: 2.17 -> 2.52 ms, r03)
  };
  // HEAD: the input ring holds fp16 quads of the fp32 input (channels >= C and pixels outside the
  // image 0, as conv_head_kernel's quad()): stream row R, pixel p (column x0 - 2 + p) at
  // ring + (f2_slot(R) * kF2InW + p) * 8 (5 184 B of the ring's LDS; the head's fragments follow
  // at hfr).  stage_load(.., k, q): the thread loads quad q of nrows rows from R0 into slot k
  // (q < nrows * 36); stage_store(k) writes it.  One buffer resource for the pass's whole input
  // (the host keeps it under 2 GB): a per-lane resource (the image and the inside test vary by
  // lane where a step straddles two strips) made every load a waterfall loop.
  unsigned char* hfr = ring + kX8HeadFrag;
  float sv[1][kMaxC];
  int sslot[1] = {-1};
  const unsigned plane = (unsigned)(s.H * s.W);
  const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(
      (void*)ends.u32, (short)0, MODE == kX8Head ? (int)((unsigned)s.B * ends.C * plane * 4u) : 0, 0x00020000);
  auto stage_load = [&](int R0, int nrows, int kJ_, int k, int q) {
    sslot[k] = -1;
    if (q >= nrows * kF2InW) return;
    const int R = R0 + q / kF2InW, p = q - (q / kF2InW) * kF2InW;
    int kk, r;
    locate(R, kJ_, kk, r);
    const SGeom G = pick(kk);
    const int x = G.x0 - 2 + p;
    const bool inside = R >= 0 && kk < K && r < s.H && x >= 0 && x < s.W;
    const unsigned o = inside ? ((unsigned)G.b * ends.C * plane + (unsigned)(r * s.W + x)) * 4u : 0x80000000u;
#pragma unroll
    for (int ch = 0; ch < kMaxC; ++ch)
      sv[k][ch] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                ru, o + (unsigned)min(ch, ends.C - 1) * plane * 4u, 0, 0));
    sslot[k] = (f2_slot(R) * kF2InW + p) * 8;
    if (!inside) sslot[k] |= 1 << 30;                      // zero quad
  };
  auto stage_store = [&](int k) {
    if (sslot[k] < 0) return;
    const bool zero = (sslot[k] >> 30) & 1;
    _Float16 h4[4];
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) h4[ch] = (ch < ends.C && !zero) ? (_Float16)sv[k][ch] : (_Float16)0;
    *reinterpret_cast<uint2*>(ring + (sslot[k] & ~(1 << 30))) =
        make_uint2((uint32_t)__builtin_bit_cast(uint16_t, h4[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, h4[1]) << 16),
                   (uint32_t)__builtin_bit_cast(uint16_t, h4[2]) | ((uint32_t)__builtin_bit_cast(uint16_t, h4[3]) << 16));
  };
  if (MODE == kX8Head) {
    stage_load(-1, 10, 0, 0, tid);                         // rows -1 .. 8 of the first strip: 360 quads
    stage_store(0);
    for (int i = tid; i < kHeadKSteps * 2 * 64; i += 512)  // conv_head's packed fragments, [ks][m][lane]
      *reinterpret_cast<uint4*>(hfr + 16 * i) = reinterpret_cast<const uint4*>(ends.hw)[i];
    if (tid < kWidth) reinterpret_cast<float*>(ring + kX8HeadBias)[tid] = ends.hb[tid];
  } else {
    for (int r = wave; r < 10; r += 8) {
      dma_at(r - 1, 0);
#pragma unroll 1
      for (int c = 0; c < 8; ++c) dma_plane(c);
    }
  }
  for (int q = tid; q < 8 * kF2MidW; q += 512) {
    const int c = q / kF2MidW, p = q - c * kF2MidW;
    *reinterpret_cast<v4i_t*>(mid + c * kF2MidPlane + p * 16) = v4i_t{0, 0, 0, 0};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (MODE == kX8Pair && layer == 1) __builtin_amdgcn_s_setprio(1);   // layer l+1's waves (4-7, the second-dispatched half)

  for (J = 0; J <= Jend; ++J) {
    auto side = [&](int ks) {                            // this wave's DMA row of the next step
      if constexpr (MODE == kX8Head) return;             // (HEAD: layer l's waves stage the quads)
      if (ks == 0) dma_at(8 * J + 9 + wave, kJ);
      if ((ks & 1) == 0 && (ks >> 1) < 8) dma_plane(ks >> 1);
    };
    auto noside = [](int) {};
    if constexpr (MODE == kX8Head) {
      // every wave: a share of the head's N-tiles (intermediate rows 8J .. 8J+7), then two of L0's
      // output rows (8J-9 + 2 qr, + 1); quads of the next step's input rows staged around them
      // (an LDS-DMA staging of fp32 rows two steps ahead measured slower, r06: 1.54 vs 1.50 ms)
      const int qr = wave >> 1;                            // quarter: 0 .. 3
      if (J < Jend) stage_load(8 * J + 9, 8, kJ, 0, tid);
      else sslot[0] = -1;
      const int hh = lane >> 5, col = lane & 31;
      auto head_part = [&]() {
        if (J < Jend) {
          // channels 32m + 16h .. (per step: short-lived).  From LDS: a global load here would
          // put an s_waitcnt vmcnt(0) in every head epilogue, which also waits for this wave's
          // staging loads and output stores of the step (r06: the head's serial latency).
          float hbl[16];
          typedef const __attribute__((address_space(3))) floatx4* lds_f4p;
#pragma unroll
          for (int r = 0; r < 16; r += 4) {
            const floatx4 bq = *(lds_f4p)(size_t)(unsigned)(size_t)(ring + kX8HeadBias + 4 * (32 * m + 16 * hh + r));
            hbl[r] = bq[0]; hbl[r + 1] = bq[1]; hbl[r + 2] = bq[2]; hbl[r + 3] = bq[3];
          }
          // ring-row byte offsets of input row 8J - 1 + q and mid-ring row 8J + q (q may vary by lane)
          const int sl0 = f2_slot(8 * J - 1);
          auto rin = [&](int q) { const int t = sl0 + q; return (t >= kF2Ring ? t - kF2Ring : t) * (kF2InW * 8); };
          auto rmid = [&](int q) { const int t = sl0 + 1 + q; return (t >= kF2Ring ? t - kF2Ring : t) * (kF2MidW * 16); };
          typedef const __attribute__((address_space(3))) half8_t* lds_h8p;
          // N-tile u < 8: intermediate row u, columns x0 .. x0+31 (pixel column 1 + col); u == 8: the
          // strip halo, lane col < 16 -> row col >> 1, column x0 - 1 or x0 + 32.  NT tiles' MFMA
          // chains interleaved.
          auto htiles = [&](auto ntc, int ua, int ub, int uc) {
            constexpr int NT = decltype(ntc)::value;
            int uu[NT], prow[NT], pcol[NT];
            floatx16 acc[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              uu[n] = n == 0 ? ua : n == 1 ? ub : uc;
              prow[n] = uu[n] < 8 ? uu[n] : (col & 15) >> 1;
              pcol[n] = uu[n] < 8 ? 1 + col : ((col & 1) ? kF2MidW - 1 : 0);
              acc[n] = floatx16{};
            }
#pragma unroll
            for (int ks = 0; ks < kHeadKSteps; ++ks) {
              const int t0 = 4 * ks + 2 * hh;             // this lane's two taps (k = 8hh .. 8hh+7)
              const half8_t ha = *(lds_h8p)(size_t)(unsigned)(size_t)(hfr + ((ks * 2 + m) * 64 + lane) * 16);
#pragma unroll
              for (int n = 0; n < NT; ++n) {
                // taps past 8 (k >= 36) meet zero weights: read tap 8's (finite) quad there instead
                // of branching around the read (0 x finite adds nothing: the separate head's bits)
                const int ta = min(t0, 8), tb = min(t0 + 1, 8);
                const uint2 q0 = *reinterpret_cast<const uint2*>(ring + rin(prow[n] + ta / 3) + (pcol[n] + ta % 3) * 8);
                const uint2 q1 = *reinterpret_cast<const uint2*>(ring + rin(prow[n] + tb / 3) + (pcol[n] + tb % 3) * 8);
                const uint4 q = make_uint4(q0.x, q0.y, q1.x, q1.y);
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, *reinterpret_cast<const half8_t*>(&q), acc[n], 0, 0, 0);
              }
            }
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              half8_t v0 = bias_act8<ACT>(acc[n], 0, hbl), v1 = bias_act8<ACT>(acc[n], 8, hbl + 8);
              int x0r;
              const bool rin_img = rowgeom(prow[n], x0r);
              const int x = x0r - 1 + pcol[n];
              if (!(rin_img && x >= 0 && x < s.W)) v0 = v1 = half8_t{};   // the next layer's zero padding
              if (uu[n] < 8 || col < 16) {
                unsigned char* dst = mid + rmid(prow[n]) + pcol[n] * 16;
                *reinterpret_cast<half8_t*>(dst + (4 * m + 2 * hh) * kF2MidPlane) = v0;
                *reinterpret_cast<half8_t*>(dst + (4 * m + 2 * hh + 1) * kF2MidPlane) = v1;
              }
            }
          };
          using I1 = std::integral_constant<int, 1>;
          htiles(I1{}, 2 * qr, 0, 0);
          htiles(I1{}, 2 * qr + 1, 0, 0);
          if (qr == 0) htiles(I1{}, 8, 0, 0);
        } else {
          for (int q = lane; q < 4 * kF2MidW * 2; q += 64) {
            const int c = q / (2 * kF2MidW), p = q - c * (2 * kF2MidW), rr = p / kF2MidW, pc = p - rr * kF2MidW;
            *reinterpret_cast<v4i_t*>(mid + (4 * m + c) * kF2MidPlane +
                                      (f2_slot(8 * J + 2 * qr + rr) * kF2MidW + pc) * 16) = v4i_t{0, 0, 0, 0};
          }
        }
      };
      auto l0_part = [&]() {
        if (J == 0) return;
        // L0 on output rows 8J-9 + 2 qr + t, t = 0, 1: N-subtiles v = 0..3 (row v >> 1, column half v & 1)
        int sl = f2_slot(8 * J - 10 + 2 * qr);
        int rowoff[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rowoff[q] = sl * (kF2MidW * 16);
          sl = sl == kF2Ring - 1 ? 0 : sl + 1;
        }
        const int lb = g * kF2MidPlane + px * 16;
        auto rowrs = [&](int t) {
          const int R = 8 * J - 9 + 2 * qr + t;
          int k, r;
          locate(R, kJ, k, r);
          const bool ok = R >= 0 && k < K && r < s.H;
          const SGeom G = pick(k);
          half_t* row = out + (((size_t)G.b * s.Hp + r + s.pad) * s.Wp + G.x0 + s.pad) * kWidth;
          return __builtin_amdgcn_make_buffer_rsrc(ok ? (void*)row : (void*)out, (short)0,
                                                   ok ? min(kTileW, s.W - G.x0) * 128 : 0, 0x00020000);
        };
        auto group = [&](int v0, int v1) {
          int ad[2][3];
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const int v = n ? v1 : v0;
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) ad[n][dy] = lb + rowoff[(v >> 1) + dy] + 16 * 16 * (v & 1);
          }
          floatx4 acc[2][2];
          x8_kloop<2, kF2MidPlane, decltype(noside)&, 2>(wA, mid, ad, acc, noside, c0);
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const int v = n ? v1 : v0;
            const half8_t o = x8_act<ACT>(acc[n]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, o), rowrs(v >> 1),
                                                   (unsigned)((16 * (v & 1) + px) * 128 + 64 * m + 16 * g), 0,
                                                   kNtX8);
          }
        };
        group(0, 1);
        group(2, 3);
      };
      // the two waves of a SIMD (w, w + 4) run the parts in opposite orders: one's L0 MFMA stream
      // covers the other's head-tile latency
      if (layer == 0) {
        head_part();
        l0_part();
      } else {
        l0_part();
        head_part();
      }
      stage_store(0);
    } else if (layer == 0 || MODE == kX8Tail) {
      // (TAIL: every wave runs a quarter of L(n-1)'s N-subtiles here, then one output row of the
      // tail below)
      const int x0 = gcx, qr = wave >> 1;
      auto lpart = [&]() {
      if (J < Jend) {
        int sl = f2_slot(8 * J - 1);
        int rowoff[10];
#pragma unroll
        for (int q = 0; q < 10; ++q) {
          rowoff[q] = sl * (kF2InW * 16);
          sl = sl == kF2Ring - 1 ? 0 : sl + 1;
        }
        // rows and columns of u < 16 inside (one strip: its rows r0 .. r0+7 < H < S)
        const bool all_in = 8 * J - kJ * S + 8 <= s.H && x0 + kTileW <= s.W;
        // N-subtile u < 16: row u >> 1, columns 1 + 16 (u & 1) .. +15; u == 16: the strip halo
        // (columns 0 and 33 of the 8 rows: pixel px -> row px >> 1, column px & 1 ? 33 : 0)
        // QL (qlc): the A-subtiles computed for the group's last N-subtile (the strip halo's
        // q = 0 on half 0's wave, q = 1 on half 1's; each writes its 4 channels, 8 B)
        auto group = [&](auto ntc, auto qlc, int u0, int u1, int u2, bool first) {
          constexpr int NT = decltype(ntc)::value, QL = decltype(qlc)::value;
          constexpr int DP = NT >= 3 ? 1 : 2;   // fragment prefetch depth (registers)
          int ad[NT][3], prow[NT], pcol[NT], uu[NT];
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            const int u = n == 0 ? u0 : n == 1 ? u1 : u2;
            uu[n] = u;
            prow[n] = u < 16 ? u >> 1 : px >> 1;
            pcol[n] = u < 16 ? 1 + 16 * (u & 1) + px : ((px & 1) ? kF2MidW - 1 : 0);
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
              int ro = rowoff[0];
#pragma unroll
              for (int q = 1; q < 10; ++q) ro = prow[n] + dy == q ? rowoff[q] : ro;
              ad[n][dy] = g * kF2InPlane + ro + pcol[n] * 16;
            }
          }
          floatx4 acc[NT][2];
          if (first) x8_kloop<NT, kF2InPlane, decltype(side)&, DP, QL>(wA, ring, ad, acc, side, c0);
          else x8_kloop<NT, kF2InPlane, decltype(noside)&, DP, QL>(wA, ring, ad, acc, noside, c0);
          auto epi = [&](bool masked) {
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              int x0r;
              const bool rin_img = rowgeom(prow[n], x0r);
              const int x = x0r - 1 + pcol[n];
              const bool inside = rin_img && x >= 0 && x < s.W;
              if (n == NT - 1 && QL != 3) {              // one A-subtile: channels 8g + 4q .. +3
                constexpr int q = QL == 1 ? 0 : 1;
                const h2v_t h0 = act_h2<ACT>(f2v_t{acc[n][q][0], acc[n][q][1]});
                const h2v_t h1 = act_h2<ACT>(f2v_t{acc[n][q][2], acc[n][q][3]});
                half4_t v = half4_t{h0.x, h0.y, h1.x, h1.y};
                if (!inside) v = half4_t{};
                *reinterpret_cast<half4_t*>(mid + (4 * m + g) * kF2MidPlane +
                                            (f2_slot(8 * J + prow[n]) * kF2MidW + pcol[n]) * 16 + 8 * q) = v;
                continue;
              }
              half8_t v = x8_act<ACT>(acc[n]);
              if ((masked || uu[n] == 16) && !inside) v = half8_t{};   // the next layer's zero padding
              *reinterpret_cast<half8_t*>(mid + (4 * m + g) * kF2MidPlane +
                                          (f2_slot(8 * J + prow[n]) * kF2MidW + pcol[n]) * 16) = v;
            }
          };
          if (__builtin_amdgcn_readfirstlane((int)all_in)) epi(false);
          else epi(true);
        };
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        if constexpr (MODE == kX8Tail) {                // 4 N-subtiles (+ one halo A-subtile: quarters 0, 1)
          if (qr == 0) {
            group(I3{}, I3{}, 0, 1, 2, true);
            group(I2{}, I1{}, 3, 16, 16, false);
          } else if (qr == 1) {
            group(I3{}, I3{}, 4, 5, 6, true);
            group(I2{}, I2{}, 7, 16, 16, false);
          } else if (qr == 2) {
            group(I3{}, I3{}, 8, 9, 10, true);
            group(I1{}, I3{}, 11, 11, 11, false);
          } else {
            group(I3{}, I3{}, 12, 13, 14, true);
            group(I1{}, I3{}, 15, 15, 15, false);
          }
        } else if (half == 0) {                          // 8 N-subtiles + one A-subtile of the halo each
          group(I3{}, I3{}, 0, 1, 2, true);
          group(I3{}, I3{}, 3, 4, 5, false);
          group(I3{}, I1{}, 6, 7, 16, false);
        } else {
          group(I3{}, I3{}, 8, 9, 10, true);
          group(I3{}, I3{}, 11, 12, 13, false);
          group(I3{}, I2{}, 14, 15, 16, false);
        }
      } else {
#pragma unroll 1
        for (int ks = 0; ks < kX8KSteps; ++ks) side(ks);
        constexpr int ZR = MODE == kX8Tail ? 2 : 4;       // rows this wave zero-fills
        const int zr0 = MODE == kX8Tail ? 2 * qr : 4 * half;
        for (int q = lane; q < 4 * kF2MidW * ZR; q += 64) {
          const int c = q / (ZR * kF2MidW), p = q - c * (ZR * kF2MidW), rr = p / kF2MidW, pc = p - rr * kF2MidW;
          *reinterpret_cast<v4i_t*>(mid + (4 * m + c) * kF2MidPlane +
                                    (f2_slot(8 * J + zr0 + rr) * kF2MidW + pc) * 16) = v4i_t{0, 0, 0, 0};
        }
      }
      };
      auto tpart = [&]() {
        if (MODE == kX8Tail && J > 0) {
          // the tail on output row 8J-9 + wave, columns 16 i + px (N-subtiles i = 0, 1): 64 -> C
          // (A rows = output channels, c >= C zero), conv_tail's K order; its fragments stream from
          // L2 (no registers or LDS left for them beside L(n-1)'s), 6 K-steps ahead
          const int R = 8 * J - 9 + wave;
          int sl = f2_slot(R - 1);
          int rowoff[3];
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            rowoff[q] = sl * (kF2MidW * 16);
            sl = sl == kF2Ring - 1 ? 0 : sl + 1;
          }
          const int lb = g * kF2MidPlane + px * 16;
          int av[2][3];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
              av[i][dy] = (int)(size_t)mid + lb + rowoff[dy] + 16 * 16 * i;
              asm volatile("" : "+v"(av[i][dy]));
            }
          unsigned tw_off = (unsigned)lane * 16u;
          asm volatile("" : "+v"(tw_off));                // per step: not hoisted out of the loop
          const __amdgpu_buffer_rsrc_t trs =
              __builtin_amdgcn_make_buffer_rsrc((void*)ends.tw, (short)0, kX8KSteps * 64 * 16, 0x00020000);
          constexpr int TP = 6;
          half8_t ta[TP + 1];
          auto ldA = [&](int ks) {
            return __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(trs, tw_off + ks * 1024u, 0, 0));
          };
#pragma unroll
          for (int ks = 0; ks < TP; ++ks) ta[ks] = ldA(ks);
          // the residual input (lanes 0..15: pixel px of N-subtile i)
          const unsigned plane = (unsigned)(s.H * s.W);
          int k, r;
          locate(R, kJ, k, r);
          const SGeom G = pick(k);
          float xi[2][kMaxC];
          unsigned toff[2];
          const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(ends.u32 + (size_t)G.b * ends.C * plane), (short)0, (int)(ends.C * plane * 4u), 0x00020000);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int x = G.x0 + 16 * i + px;
            const bool ok = R >= 0 && k < K && r < s.H && x < s.W && lane < 16;
            toff[i] = ok ? (unsigned)(r * s.W + x) * 4u : 0x80000000u;     // out of range: dropped
#pragma unroll
            for (int c = 0; c < kMaxC; ++c)
              xi[i][c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                        ro, toff[i] + (unsigned)min(c, ends.C - 1) * plane * 4u, 0, 0));
          }
          typedef const __attribute__((address_space(3))) half8_t* lds_h8p;
          floatx4 acc[2] = {};
#pragma unroll
          for (int ks = 0; ks < kX8KSteps; ++ks) {
            if (ks + TP < kX8KSteps) ta[(ks + TP) % (TP + 1)] = ldA(ks + TP);
            const int tap = ks >> 1, hs = ks & 1, dy = tap / 3, dx = tap - 3 * dy;
            half8_t fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fb[i] = *(lds_h8p)(size_t)(unsigned)(av[i][dy] + (4 * hs * kF2MidPlane + 16 * dx));
#pragma unroll
            for (int i = 0; i < 2; ++i)
              acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ta[ks % (TP + 1)], fb[i], acc[i], 0, 0, 0);
          }
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int c = 0; c < kMaxC; ++c) {
              const float nc = acc[i][c] + tbl[c];
              float o = ends.residual_sign > 0 ? nc + xi[i][c] : xi[i][c] - nc;
              if (ends.clamp_out) o = fminf(fmaxf(o, 0.f), 1.f);
              __builtin_amdgcn_raw_buffer_store_b32(
                  __builtin_bit_cast(int, o),
                  __builtin_amdgcn_make_buffer_rsrc((void*)(ends.xout + ((size_t)G.b * ends.C + (c < ends.C ? c : 0)) * plane),
                                                    (short)0, c < ends.C ? (int)(plane * 4u) : 0, 0x00020000),
                  toff[i], 0, kNtTail);
            }
        }
      };
      // TAIL: the two waves of a SIMD (w, w + 4) run the parts in opposite orders, so one's MFMA
      // stream covers the other's latencies (the tail's L2 fragment loads)
      if (MODE != kX8Tail || layer == 0) {
        lpart();
        tpart();
      } else {
        tpart();
        lpart();
      }
      // (TAIL: leaving the tail's 8 output stores in flight here, vmcnt(8) on the waves that run
      // it last, measured no faster, r06)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (J > 0) {
        // output rows 8J-9 + 4 half + t, t = 0..3: N-subtiles (t, column half), two per group
        int sl = f2_slot(8 * J - 10 + 4 * half);
        int rowoff[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          rowoff[q] = sl * (kF2MidW * 16);
          sl = sl == kF2Ring - 1 ? 0 : sl + 1;
        }
        const int lb = g * kF2MidPlane + px * 16;
        auto rowrs = [&](int t) {                      // output row t's store descriptor
          const int R = 8 * J - 9 + 4 * half + t;
          int k, r;
          locate(R, kJ, k, r);
          const bool ok = R >= 0 && k < K && r < s.H;
          const SGeom G = pick(k);
          half_t* row = out + (((size_t)G.b * s.Hp + r + s.pad) * s.Wp + G.x0 + s.pad) * kWidth;
          return __builtin_amdgcn_make_buffer_rsrc(ok ? (void*)row : (void*)out, (short)0,
                                                   ok ? min(kTileW, s.W - G.x0) * 128 : 0, 0x00020000);
        };
        // N-subtile v = 0..7: output row t = v >> 1, columns 16 (v & 1) .. +15
        auto group = [&](auto ntc, int v0, int v1, int v2, bool first) {
          constexpr int NT = decltype(ntc)::value;
          constexpr int DP = NT >= 3 ? 1 : 2;
          int ad[NT][3], vv[NT];
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            vv[n] = n == 0 ? v0 : n == 1 ? v1 : v2;
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) ad[n][dy] = lb + rowoff[(vv[n] >> 1) + dy] + 16 * 16 * (vv[n] & 1);
          }
          floatx4 acc[NT][2];
          if (first) x8_kloop<NT, kF2MidPlane, decltype(side)&, DP>(wA, mid, ad, acc, side, c0);
          else x8_kloop<NT, kF2MidPlane, decltype(noside)&, DP>(wA, mid, ad, acc, noside, c0);
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            const half8_t v = x8_act<ACT>(acc[n]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), rowrs(vv[n] >> 1),
                                                   (unsigned)((16 * (vv[n] & 1) + px) * 128 + 64 * m + 16 * g), 0,
                                                   kNtX8);
          }
        };
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        group(I3{}, 0, 1, 2, true);
        group(I3{}, 3, 4, 5, false);
        group(I2{}, 6, 7, 7, false);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // the DMAs (older than the 8 stores) landed
      } else {
#pragma unroll 1
        for (int ks = 0; ks < kX8KSteps; ++ks) side(ks);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    lds_barrier();     // the layer-l+1 stores stay in flight (vmcnt above, per role)
    if (8 * (J + 1) >= (kJ + 1) * S) {                  // the next step starts in the next strip
      ++kJ;
      gpb = gcb;
      gpx = gcx;
      gcb = gnb;
      gcx = gnx;
      const SGeom gg = geom(kJ + 1);
      gnb = gg.b;
      gnx = gg.x0;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef X8_CLOCK
  unsigned long long c1_, r1_;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1_), "=s"(r1_)::"memory");
  if (tid == 0 && blockIdx.x < 1024) {
    x8_clock[blockIdx.x][0] = c1_ - c0_;
    x8_clock[blockIdx.x][1] = r1_ - r0_;
  }
#endif
}

#define PNP_X8_INST(A, M)                                                                                      \
  template __global__ void conv_body_x8_kernel<A, M>(const half_t* __restrict__, half_t* __restrict__,        \
                                                     const uint4* __restrict__, const float* __restrict__,   \
                                                     const uint4* __restrict__, const float* __restrict__,   \
                                                     ConvShape, int, int, int, X8Ends);
PNP_X8_INST(0, kX8Pair)
PNP_X8_INST(1, kX8Pair)
PNP_X8_INST(0, kX8Head)
PNP_X8_INST(1, kX8Head)
PNP_X8_INST(0, kX8Tail)
PNP_X8_INST(1, kX8Tail)
#undef PNP_X8_INST

// ------------------------------------------------------------------------------------
// Body layer with split weights (PNP_PREC_FP16W2): W = W_hi + W_lo, both fp16 (W_lo =
// fp16(W - W_hi), subnormals kept: the f16 MFMA inputs do not flush them, probed in
// tools/probes/mfma_f16_denorm.hip), fp16 activations, fp32 accumulation: every product is
// a * W_hi + a * W_lo in the same accumulator, so the weights carry ~22 significant bits.
// Why: with fp16-rounded weights the Poisson method's slow primal steps integrate the
// rounded network's deterministic error (0.19 dB after 3000 iterations of ours-C), while
// fp16 activations alone stay within 0.001 dB (profiles/r02/precision_drift.txt).
// Twice the MFMAs of conv_body_v3.  The hi halves stay in registers (144 VGPRs, as in v3);
// the lo halves of both M-tiles (72 KiB) sit in LDS for the launch, one A-fragment read per
// K-step; with them the halo ring is 2 deep (2 x 44 KiB: tile t+1's DMA runs during tile t)
// and the LDS is exactly 160 KiB.  4 waves, one per SIMD: wave w owns channels
// 32m..32m+31 (m = w & 1) of tile rows 4(w>>1) .. +3 (four N-tiles, 64 accumulators); per
// K-step 4 B fragments + 1 lo A fragment, 8 MFMAs.  The epilogue stores 2 x 16 B per lane
// and N-tile straight from registers.
constexpr int kW2Halo = 44 * 1024;
constexpr int kW2Lo = 2 * kW2Halo;
constexpr int kW2Lds = kW2Lo + kBodyWBytes;                    // 163840 B

template <int ACT>
__global__ __launch_bounds__(256, 1) void conv_body_w2_kernel(const half_t* __restrict__ in,
                                                               half_t* __restrict__ out,
                                                               const uint4* __restrict__ wpk,
                                                               const uint4* __restrict__ wpk_lo,
                                                               const float* __restrict__ bias,
                                                               ConvShape s) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = wave & 1, rq = wave >> 1;    // M-tile, row quad
  const int h = lane >> 5, col = lane & 31;
  unsigned char* wlo = smem + kW2Lo;
  for (int i = tid; i < kBodyWBytes / 16; i += 256) reinterpret_cast<uint4*>(wlo)[i] = wpk_lo[i];
  float bl[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) bl[r] = bias[32 * m + 16 * h + r];
  half8_t wA[kBodyKSteps];                    // hi halves, resident for the launch
#pragma unroll
  for (int ks = 0; ks < kBodyKSteps; ++ks)
    wA[ks] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wpk) +
                                               ((ks * 2 + m) * 64 + lane) * 16);
  auto buf = [&](int i) { return smem + i * kW2Halo; };
  RingDma<4, true> dma;
  dma.init(s, wave);
  auto issue_dma = [&](int tt, int bi) {      // clamped: always the same instruction count
    dma.issue(buf(bi), in, s, tt < s.tiles ? tt : s.tiles - 1, wave);
  };
  int t = xcd_block(blockIdx.x, gridDim.x);
  if (t < s.tiles) {
    issue_dma(t, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // tile t (and the lo weights) landed
  }
  __syncthreads();
  int cur = 0;
  // (r06) One wave per SIMD, so nothing overlapped the burst of DMA slots before a tile's K-loop
  // or the epilogue after it: tile t+1's slots now issue one per K-step (1 .. kSlots) and tile
  // t-1's epilogue (bias, activation, 2 stores per N-tile) runs at K-steps kSlots+1 .. +4; a
  // workgroup's first tile stores its empty predecessor through zero-size buffer resources, so
  // every tile issues its slots and then 8 stores and the vmcnt(8) below stays exact.  The
  // accumulators of the previous tile live on (64 more registers: AGPRs at one wave per SIMD).
  constexpr int kW2Slots = RingDma<4, true>::kSlots;
  static_assert(kW2Slots + 4 < kBodyKSteps, "slots and stores fit in the K-loop");
  floatx16 pacc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) pacc[n] = floatx16{};
  int pb = 0, pty0 = 0, ptx0 = 0;
  bool pv = false;
  auto store_n = [&](int n) {
    const int y = pty0 + 4 * rq + n;
    const half8_t v0 = bias_act8<ACT>(pacc[n], 0, bl), v1 = bias_act8<ACT>(pacc[n], 8, bl + 8);
    half_t* row = out + (((size_t)pb * s.Hp + y + s.pad) * s.Wp + ptx0 + s.pad) * kWidth;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        row, (short)0, (pv && y < s.H) ? min(kTileW, s.W - ptx0) * 128 : 0, 0x00020000);
    const unsigned off = (unsigned)(col * 128 + 64 * m + 32 * h);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v0), rs, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v1), rs, off + 16, 0, 0);
  };
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const int tn = t + gridDim.x;             // buffer cur ^ 1 was last read by tile t - 1
    const __amdgpu_buffer_rsrc_t drs = RingDma<4, true>::rsrc(in, s, tn < s.tiles ? tn : s.tiles - 1);
    unsigned char* dbuf = buf(cur ^ 1);
    const unsigned char* hl = buf(cur);
    auto ldB = [&](int ks, int n) {
      const int tap = ks >> 2, sub = ks & 3;
      return *reinterpret_cast<const half8_t*>(hl + halo_off(4 * rq + n + tap / 3, col + tap % 3, 2 * sub + h));
    };
    auto ldL = [&](int ks) {
      return *reinterpret_cast<const half8_t*>(wlo + ((ks * 2 + m) * 64 + lane) * 16);
    };
    floatx16 acc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = floatx16{};
    half8_t fb[4], fl = ldL(0);
#pragma unroll
    for (int n = 0; n < 4; ++n) fb[n] = ldB(0, n);
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks) {
      const half8_t lo = fl;
      if (ks + 1 < kBodyKSteps) fl = ldL(ks + 1);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[n], acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(lo, fb[n], acc[n], 0, 0, 0);
        if (ks + 1 < kBodyKSteps) fb[n] = ldB(ks + 1, n);
      }
      if (ks >= 1 && ks <= kW2Slots) dma.issue_slot(dbuf, drs, ks - 1, wave);          // tile t+1's halo
      if (ks > kW2Slots && ks <= kW2Slots + 4) store_n(ks - kW2Slots - 1);             // tile t-1's rows
    }
    // epilogue (deferred): lane (col, h) holds channels 32m + 16h .. +15 of pixel (row 4rq + n, column col)
#pragma unroll
    for (int n = 0; n < 4; ++n) pacc[n] = acc[n];
    pb = b;
    pty0 = ty0;
    ptx0 = tx0;
    pv = true;
    // tile t+1 landed: only tile t-1's 8 stores are younger than its DMA
    asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur ^= 1;
  }
  if (pv) {                                   // the last tile's rows
#pragma unroll
    for (int n = 0; n < 4; ++n) store_n(n);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
}

template __global__ void conv_body_w2_kernel<0>(const half_t* __restrict__, half_t* __restrict__,
                                                const uint4* __restrict__, const uint4* __restrict__,
                                                const float* __restrict__, ConvShape);
template __global__ void conv_body_w2_kernel<1>(const half_t* __restrict__, half_t* __restrict__,
                                                const uint4* __restrict__, const uint4* __restrict__,
                                                const float* __restrict__, ConvShape);

// ------------------------------------------------------------------------------------
// conv_stack16: every 64 -> 64 body layer of a small batch in ONE launch (fp16 operands).
// The reference denoises one image per call (main.py:36,69), where each per-layer launch of
// conv_body_v3 (one 8 x 32 tile per CU at 256^2) spends ~11 us for ~2 us of MFMA work: wave
// launch, weights into registers, halo DMA, drain.  Here a workgroup keeps its tiles for all
// layers; layer l + 1 of a tile starts once the 3 x 3 neighbourhood of tiles has published
// layer l (tile_wait / tile_publish, common.h: relaxed agent-scope stores and polls of a
// per-tile progress word, epoch-tagged per launch so the words are never reset; ordering by
// the sc1-only contract stated there), and the next layer's
// weights load into the registers right after a layer's last tile is published, in flight
// while the neighbourhood catches up.  The handed-off activations never sit stale in a cache:
// the epilogue stores and the halo's LDS-DMA loads are device-scope (sc1), so neither side
// needs an L2 write-back or invalidate fence (MI355X_MICROARCH.md, inter-workgroup
// visibility: the sc1 form).  Measured at B = 1 RGB 256^2 (cfg2 iteration, ms): agent-scope
// release / acquire fences with plain DMA 0.29 (per-layer launches: 0.24); sc1 loads through
// registers 0.235; sc1 LDS-DMA 0.207.  One wave per SIMD (4 waves): wave w
// owns channels 32 (w & 1) .. +31 of tile rows 4 (w >> 1) .. +3, i.e. conv_body_w2's tiling
// on conv_body_v3's fragments (pack_body_weights), so every output is the same MFMA chain and
// the same fp16 rounding as the per-layer launches: bit-identical (test_gpu_graph.py).  Two
// 44 KiB halo buffers alternate over a workgroup's tiles.  The grid is at most one workgroup
// per CU (all resident: the waits only ever point at lower layers, so no cycle) and the host
// uses it only when the batch has at most 2 tiles per CU.
// ------------------------------------------------------------------------------------
constexpr int kStkLds = 2 * kW2Halo;                           // 90112 B
#ifdef STACK_STAMPS   // diagnostic build (tools/stack_stamps.py): s_memrealtime per phase, first tile of WG < 512
__device__ unsigned long long stack_stamps[512][24][6];
#define STK_STAMP(L, I)                                                                                     \
  do {                                                                                                      \
    if (k == 0 && blockIdx.x < 512 && (L) < 24) {                                                           \
      unsigned long long t_;                                                                                \
      __builtin_amdgcn_sched_barrier(0);                                                                    \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                        \
      __builtin_amdgcn_sched_barrier(0);                                                                    \
      if (tid == 0) stack_stamps[blockIdx.x][(L)][(I)] = t_;                                                \
    }                                                                                                       \
  } while (0)
#else
#define STK_STAMP(L, I) do {} while (0)
#endif
constexpr int kCpolDevice = 16;                                // sc1: device-scope load / store

template <int ACT>
__global__ __launch_bounds__(256, 1) void conv_stack16_kernel(half_t* __restrict__ actA, half_t* __restrict__ actB,
                                                               const uint4* __restrict__ wpk,
                                                               const float* __restrict__ bias, int nbody,
                                                               ConvShape s, int* __restrict__ done, int epoch,
                                                               int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = wave & 1, rq = wave >> 1;
  const int h = lane >> 5, col = lane & 31;
  auto buf = [&](int i) { return smem + i * kW2Halo; };
  RingDma<4, true> dma;
  dma.init(s, wave);
  const int G = gridDim.x;
  const int K = (s.tiles - (int)blockIdx.x + G - 1) / G;      // this workgroup's tiles (grid <= tiles)

  half8_t w[kBodyKSteps];
  float bl[16];
  auto load_w = [&](int l) {
    const unsigned char* src = reinterpret_cast<const unsigned char*>(wpk) + (size_t)l * kBodyWBytes;
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks)
      w[ks] = *reinterpret_cast<const half8_t*>(src + ((ks * 2 + m) * 64 + lane) * 16);
#pragma unroll
    for (int r = 0; r < 16; ++r) bl[r] = bias[l * kWidth + 32 * m + 16 * h + r];
  };
  load_w(0);
  for (int l = 0; l < nbody; ++l) {
    const half_t* in = (l & 1) ? actB : actA;
    half_t* out = (l & 1) ? actA : actB;
    for (int k = 0; k < K; ++k) {
      const int t = (int)blockIdx.x + k * G;
      int b, ty0, tx0;
      decode_tile(t, s, b, ty0, tx0);
      STK_STAMP(l, 0);
      if (l > 0) {                            // the 3 x 3 neighbourhood has published layer l - 1
        if (wave == 0) {
          const int ny = ty0 / kTileH + lane / 3 - 1, nx = tx0 / kTileW + lane % 3 - 1;
          const bool want = lane < 9 && ny >= 0 && ny < s.tiles_y && nx >= 0 && nx < s.tiles_x;
          tile_wait(done, want ? (b * s.tiles_y + ny) * s.tiles_x + nx : 0, want, epoch + l, err);
        }
        __syncthreads();
      }
      STK_STAMP(l, 1);
      dma.template issue<kCpolDevice>(buf(k & 1), in, s, t, wave);   // device scope: never a stale line
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      STK_STAMP(l, 2);
      const unsigned char* hl = buf(k & 1);
      auto ldB = [&](int ks, int n) {
        const int tap = ks >> 2, sub = ks & 3;
        return *reinterpret_cast<const half8_t*>(hl + halo_off(4 * rq + n + tap / 3, col + tap % 3, 2 * sub + h));
      };
      floatx16 acc[4];
      half8_t fb[2][4];
#pragma unroll
      for (int n = 0; n < 4; ++n) fb[0][n] = ldB(0, n);
#pragma unroll
      for (int ks = 0; ks < kBodyKSteps; ++ks) {
        const int r = ks & 1;
        if (ks + 1 < kBodyKSteps) {
#pragma unroll
          for (int n = 0; n < 4; ++n) fb[r ^ 1][n] = ldB(ks + 1, n);
        }
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[ks], fb[r][n], ks == 0 ? bias16(bl) : acc[n], 0, 0, 0);
      }
      STK_STAMP(l, 3);
      // lane (col, h) holds channels 32m + 16h .. +15 of pixel (row 4rq + n, column col)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int y = ty0 + 4 * rq + n;
        const half8_t v0 = act8_h<ACT>(acc[n], 0), v1 = act8_h<ACT>(acc[n], 8);
        half_t* row = out + (((size_t)b * s.Hp + y + s.pad) * s.Wp + tx0 + s.pad) * kWidth;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? min(kTileW, s.W - tx0) * 128 : 0, 0x00020000);
        const unsigned off = (unsigned)(col * 128 + 64 * m + 32 * h);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v0), rs, off, 0, kCpolDevice);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v1), rs, off + 16, 0, kCpolDevice);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores done (device scope)
      __syncthreads();
      STK_STAMP(l, 4);
      if (tid == 0) tile_publish(done + t, epoch + l + 1);
      STK_STAMP(l, 5);
    }
    // the next layer's weights: in flight while the neighbourhood catches up
    if (l + 1 < nbody) load_w(l + 1);
  }
}

template __global__ void conv_stack16_kernel<0>(half_t* __restrict__, half_t* __restrict__, const uint4* __restrict__,
                                                const float* __restrict__, int, ConvShape, int* __restrict__, int,
                                                int* __restrict__);
template __global__ void conv_stack16_kernel<1>(half_t* __restrict__, half_t* __restrict__, const uint4* __restrict__,
                                                const float* __restrict__, int, ConvShape, int* __restrict__, int,
                                                int* __restrict__);

// ------------------------------------------------------------------------------------
// conv_stack16x2: conv_stack16 with TWO body layers per hand-off (small batches, round 3).
// Per layer the persistent chain costs a neighbour wait, the halo DMA and the device-scope
// store round trip besides its ~2 us of MFMA work (9.1 us per layer at B = 1 RGB 256^2,
// profiles/r03/stack_stamps.txt); here a tile computes layers l and l+1 from one 12 x 36 input
// halo (2 pixels of border: the activation images' zero border is 2 pixels wide), the 10 x 34
// intermediate of layer l staying in LDS, so the chain has half as many links.  Layer l costs
// 11 N-tiles instead of 8 (the intermediate's border: 10 rows of 32 columns + one N-tile of its
// 20 edge pixels, columns 0 and 33).  Wave w (one per SIMD): M-tile m = w & 1; layer l rows
// 0..4 + the edge N-tile (w >> 1 == 0) or rows 5..9, in groups of at most 3 N-tiles; layer l+1
// as conv_stack16 (rows 4 (w >> 1) .. +3).  Same MFMA chains and fp16 roundings as the
// per-layer launches (the intermediate is zero outside the image = the next layer's padding),
// so the results are bit-identical (tests/test_gpu_graph.py).  The pairs ping-pong A -> B -> A:
// after an odd number of pairs the output is in actB (launch_conv_stack16x2 returns which).
// ------------------------------------------------------------------------------------
constexpr int kX2InW = kTileW + 4, kX2InH = kTileH + 4;        // 36 x 12 input halo
constexpr int kX2InPix = kX2InW * kX2InH;                      // 432 = 54 DMA slots of 8 pixels
constexpr int kX2Slots = kX2InPix / 8;
constexpr int kX2SlotsW = (kX2Slots + 3) / 4;                  // 14 per wave (the last 2 re-read slot 53)
constexpr int kX2In = 4 * kX2SlotsW * 1024;                    // 57344 B per input buffer
constexpr int kX2Mid = 2 * kX2In;                              // intermediate (10 x 34, halo_off layout)
constexpr int kX2Lds = kX2Mid + kV3Halo;                       // 158208 B
static_assert(kX2Lds <= 163840, "conv_stack16x2 LDS");
// HEAD: the head layer (C -> 64) computed into the first pair's input halo (round 4, VERDICT r03
// item 6): its 12 x 36 outputs need the fp32 input on 14 x 38 pixels, staged as 4 fp16 channels
constexpr int kX2HeadW = kX2InW + 2, kX2HeadPix = kX2HeadW * (kX2InH + 2);   // 38 x 14 = 532
constexpr int kX2LdsHead = kX2Lds + kX2HeadPix * 8;            // 162464 B
static_assert(kX2LdsHead <= 163840, "conv_stack16x2 LDS with the head stage");

__device__ __forceinline__ int x2_in_off(int pr, int pc, int chunk) {          // 12 x 36 input halo
  return (pr * kX2InW + pc) * 128 + 16 * (chunk ^ ((pc >> 1) & 7));
}

// HEAD: pair 0's input halo is the head layer of conv_head_kernel (PREC 0) computed in place from
// the fp32 NCHW input u32 (C channels): the same packed weights hw, the same three
// v_mfma_f32_32x32x16_f16 per output in the same K order from a zero accumulator, the same fp16
// input rounding and bias_act8 epilogue, zero outside the image (the activation images' border),
// so the bits are those of the head launch plus the DMA it replaces.
template <int ACT, bool HEAD>
__global__ __launch_bounds__(256, 1) void conv_stack16x2_kernel(half_t* __restrict__ actA, half_t* __restrict__ actB,
                                                                 const uint4* __restrict__ wpk,
                                                                 const float* __restrict__ bias, int npairs,
                                                                 ConvShape s, int* __restrict__ done, int epoch,
                                                                 int* __restrict__ err, const float* __restrict__ u32,
                                                                 int C, const uint4* __restrict__ hw,
                                                                 const float* __restrict__ hb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = wave & 1, rq = wave >> 1;
  const int h = lane >> 5, col = lane & 31;
  unsigned char* mid = smem + kX2Mid;
  const int G = gridDim.x;
  const int K = (s.tiles - (int)blockIdx.x + G - 1) / G;      // this workgroup's tiles (grid <= tiles)
  // DMA: slot g (8 pixels of the 12 x 36 halo, 1 KiB) -> lane l loads chunk (l & 7) ^ swz(pc) of
  // pixel 8g + l / 8 to the lane-linear destination (the x2_in_off layout)
  unsigned doff[kX2SlotsW];
#pragma unroll
  for (int j = 0; j < kX2SlotsW; ++j) {
    const int g = min(4 * j + wave, kX2Slots - 1);
    const int p = 8 * g + (lane >> 3), pr = p / kX2InW, pc = p - pr * kX2InW;
    const int c = (lane & 7) ^ ((pc >> 1) & 7);
    doff[j] = (unsigned)(((pr * s.Wp + pc) * kWidth + c * 8) * 2);
  }
  auto issue_dma = [&](unsigned char* dst, const half_t* in, int b, int ty0, int tx0) {
    // halo origin: image pixel (ty0 - 2, tx0 - 2) = padded (ty0, tx0); bounded by the image's end
    const size_t o = ((size_t)b * s.Hp + ty0 + s.pad - 2) * s.Wp + tx0 + s.pad - 2;
    const size_t end = ((size_t)b + 1) * s.Hp * s.Wp;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(in + o * kWidth), (short)0, (int)min((size_t)0x7fffffff, (end - o) * 128), 0x00020000);
#pragma unroll
    for (int j = 0; j < kX2SlotsW; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + (4 * j + wave) * 1024),
                                               16, doff[j], 0, 0, kCpolDevice);
  };

  // One layer's weights in registers at a time: layer 2p + 1's are loaded after layer 2p, the next
  // pair's first layer after the publish (in flight while the neighbourhood catches up).
  // (buffer loads: one lane offset + a scalar offset per K-step, instead of a 64-bit address
  // register per K-step that the compiler keeps live across the whole kernel)
  half8_t w[kBodyKSteps];
  float bl[16];
  const unsigned wlane = (unsigned)((m * 64 + lane) * 16);
  auto load_w = [&](int l, int ks0 = 0, int ks1 = kBodyKSteps) {
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const unsigned char*>(wpk) + (size_t)l * kBodyWBytes), (short)0, kBodyWBytes, 0x00020000);
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks)
      if (ks >= ks0 && ks < ks1)
        w[ks] = __builtin_bit_cast(half8_t, __builtin_amdgcn_raw_buffer_load_b128(rw, wlane, ks * 2048, 0));
    if (ks0 == 0)
#pragma unroll
      for (int r = 0; r < 16; ++r) bl[r] = bias[l * kWidth + 32 * m + 16 * h + r];
  };
  load_w(0);
  for (int p = 0; p < npairs; ++p) {
    const half_t* src = (p & 1) ? actB : actA;                 // pairs ping-pong: A -> B -> A ...
    half_t* out = (p & 1) ? actA : actB;
    for (int k = 0; k < K; ++k) {
      const int t = (int)blockIdx.x + k * G;
      int b, ty0, tx0;
      decode_tile(t, s, b, ty0, tx0);
      if (k > 0) load_w(2 * p);               // (more than one tile per workgroup: layer 2p again)
      STK_STAMP(p, 0);
      if (p > 0) {                            // the 3 x 3 neighbourhood has published pair p - 1
        if (wave == 0) {
          const int ny = ty0 / kTileH + lane / 3 - 1, nx = tx0 / kTileW + lane % 3 - 1;
          const bool want = lane < 9 && ny >= 0 && ny < s.tiles_y && nx >= 0 && nx < s.tiles_x;
          tile_wait(done, want ? (b * s.tiles_y + ny) * s.tiles_x + nx : 0, want, epoch + p, err);
        }
        __syncthreads();
      }
      STK_STAMP(p, 1);
      unsigned char* hin = smem + (k & 1) * kX2In;
      if (HEAD && p == 0) {
        // fp32 input rows ty0-3 .. ty0+10, columns tx0-3 .. tx0+34 -> 4 fp16 channels per pixel
        // (channels >= C and pixels outside the image 0, as conv_head_kernel's quad())
        // (buffer loads of the image's C planes: no plain global load besides the progress polls,
        // which tests/test_isa_handoff.py requires to be sc1)
        uint2* hst = reinterpret_cast<uint2*>(smem + kX2Lds);
        const unsigned plane = (unsigned)(s.H * s.W);
        const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(u32 + (size_t)b * C * plane), (short)0, (int)(C * plane * 4u), 0x00020000);
        for (int q = tid; q < kX2HeadPix; q += 256) {
          const int r = q / kX2HeadW, c = q - r * kX2HeadW;
          const int gy = ty0 - 3 + r, gx = tx0 - 3 + c;
          const bool in = gy >= 0 && gy < s.H && gx >= 0 && gx < s.W;
          const unsigned o = in ? (unsigned)(gy * s.W + gx) : 0u;
          _Float16 h4[4];
#pragma unroll
          for (int ch = 0; ch < 4; ++ch) {
            const float v = __builtin_bit_cast(
                float, __builtin_amdgcn_raw_buffer_load_b32(ru, ((unsigned)min(ch, C - 1) * plane + o) * 4u, 0, 0));
            h4[ch] = (ch < C && in) ? (_Float16)v : (_Float16)0;
          }
          hst[q] = make_uint2((uint32_t)__builtin_bit_cast(uint16_t, h4[0]) |
                                  ((uint32_t)__builtin_bit_cast(uint16_t, h4[1]) << 16),
                              (uint32_t)__builtin_bit_cast(uint16_t, h4[2]) |
                                  ((uint32_t)__builtin_bit_cast(uint16_t, h4[3]) << 16));
        }
        half8_t ha[kHeadKSteps];
#pragma unroll
        for (int ks = 0; ks < kHeadKSteps; ++ks)
          ha[ks] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(hw) +
                                                     ((ks * 2 + m) * 64 + lane) * 16);
        float hbl[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) hbl[r] = hb[32 * m + 16 * h + r];
        __syncthreads();
        // the 12 x 36 halo = 432 pixels, N-tiles of 32 (pixel 32 n + col, the last one half used);
        // wave (m, rq): M-tile m of N-tiles rq, rq + 2, ..
        for (int n = rq; n < (kX2InPix + 31) / 32; n += 2) {
          const int pix = 32 * n + col, pl = min(pix, kX2InPix - 1);
          const int pr = pl / kX2InW, pc = pl - pr * kX2InW;
          floatx16 acc = {};
#pragma unroll
          for (int ks = 0; ks < kHeadKSteps; ++ks) {
            const int t0 = 4 * ks + 2 * h;               // this lane's two taps (k = 8h .. 8h+7)
            uint2 q0 = make_uint2(0, 0), q1 = make_uint2(0, 0);
            if (t0 < 9) q0 = hst[(pr + t0 / 3) * kX2HeadW + pc + t0 % 3];
            if (t0 + 1 < 9) q1 = hst[(pr + (t0 + 1) / 3) * kX2HeadW + pc + (t0 + 1) % 3];
            const uint4 q = make_uint4(q0.x, q0.y, q1.x, q1.y);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha[ks], *reinterpret_cast<const half8_t*>(&q), acc, 0, 0, 0);
          }
          const int gy = ty0 - 2 + pr, gx = tx0 - 2 + pc;
          const bool inside = gy >= 0 && gy < s.H && gx >= 0 && gx < s.W;
          half8_t v0 = bias_act8<ACT>(acc, 0, hbl), v1 = bias_act8<ACT>(acc, 8, hbl + 8);
          if (!inside) v0 = v1 = half8_t{};
          if (pix < kX2InPix) {
            *reinterpret_cast<half8_t*>(hin + x2_in_off(pr, pc, 4 * m + 2 * h)) = v0;
            *reinterpret_cast<half8_t*>(hin + x2_in_off(pr, pc, 4 * m + 2 * h + 1)) = v1;
          }
        }
        __syncthreads();
      } else {
        issue_dma(hin, src, b, ty0, tx0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      STK_STAMP(p, 2);
      // ---- layer 2p: the 10 x 34 intermediate into LDS ----
      // N-tile u < 10: intermediate row u, columns 1 .. 32 (lane col -> column col + 1);
      // u == 10: the edge pixels, lane n < 20 -> row n >> 1, column (n & 1) ? 33 : 0
      // Fragment addresses: per (tap column dx, channel quarter sub) a lane offset, opaque so the
      // compiler keeps 12 registers per kind of N-tile instead of hoisting every (N-tile, K-step)
      // address out of the pair / tile loops (that spilled); tap rows and N-tile rows are immediates.
      const int e = min(col, 19);                          // edge N-tile: lane -> row e >> 1, column 0 / 33
      const int epr = e >> 1, epc = (e & 1) ? kHaloW - 1 : 0;
      int cor[3][4], coe[3][4];
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int sub = 0; sub < 4; ++sub) {
          cor[dx][sub] = x2_in_off(0, col + 1 + dx, 2 * sub + h);
          coe[dx][sub] = x2_in_off(epr, epc + dx, 2 * sub + h);
          asm volatile("" : "+v"(cor[dx][sub]), "+v"(coe[dx][sub]));
        }
      auto group = [&](auto ntc, int u0, int u1, int u2, bool last) {
        constexpr int NT = decltype(ntc)::value;
        int pr[NT], pc[NT], uu[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int u = n == 0 ? u0 : n == 1 ? u1 : u2;
          uu[n] = u;
          pr[n] = u < 10 ? u : epr;
          pc[n] = u < 10 ? col + 1 : epc;
        }
        auto ldB = [&](int ks, int n) {
          const int tap = ks >> 2, sub = ks & 3, dy = tap / 3, dx = tap - 3 * dy;
          const int o = uu[n] < 10 ? cor[dx][sub] + (uu[n] + dy) * (kX2InW * 128) : coe[dx][sub] + dy * (kX2InW * 128);
          return *reinterpret_cast<const half8_t*>(hin + o);
        };
        floatx16 acc[NT];
        half8_t fb[2][NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) fb[0][n] = ldB(0, n);
#pragma unroll
        for (int ks = 0; ks < kBodyKSteps; ++ks) {
          const int r = ks & 1;
          if (ks + 1 < kBodyKSteps) {
#pragma unroll
            for (int n = 0; n < NT; ++n) fb[r ^ 1][n] = ldB(ks + 1, n);
          }
#pragma unroll
          for (int n = 0; n < NT; ++n)
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[ks], fb[r][n], ks == 0 ? bias16(bl) : acc[n], 0, 0, 0);
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int y = ty0 - 1 + pr[n], x = tx0 - 1 + pc[n];
          const bool inside = y >= 0 && y < s.H && x >= 0 && x < s.W;
          half8_t v0 = act8_h<ACT>(acc[n], 0), v1 = act8_h<ACT>(acc[n], 8);
          if (!inside) v0 = v1 = half8_t{};                 // the next layer's zero padding
          if (uu[n] < 10 || col < 20) {
            *reinterpret_cast<half8_t*>(mid + halo_off(pr[n], pc[n], 4 * m + 2 * h)) = v0;
            *reinterpret_cast<half8_t*>(mid + halo_off(pr[n], pc[n], 4 * m + 2 * h + 1)) = v1;
          }
        }
      };
      using I2 = std::integral_constant<int, 2>;
      using I3 = std::integral_constant<int, 3>;
      if (rq == 0) {                                      // rows 0..4 + the edge N-tile
        group(I3{}, 0, 1, 2, false);
        group(I3{}, 3, 4, 10, true);
      } else {                                            // rows 5..9
        group(I3{}, 5, 6, 7, false);
        group(I2{}, 8, 9, 9, true);
      }
      __syncthreads();
      STK_STAMP(p, 3);
      load_w(2 * p + 1, 0, kBodyKSteps);   // (part of it during layer 2p's last epilogue spilled, r03)
      // ---- layer 2p + 1: the 8 x 32 tile from the intermediate (conv_stack16's K-loop) ----
      {
        int com[3][4];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int sub = 0; sub < 4; ++sub) {
            com[dx][sub] = halo_off(4 * rq, col + dx, 2 * sub + h);
            asm volatile("" : "+v"(com[dx][sub]));
          }
        auto ldB = [&](int ks, int n) {
          const int tap = ks >> 2, sub = ks & 3, dy = tap / 3, dx = tap - 3 * dy;
          return *reinterpret_cast<const half8_t*>(mid + com[dx][sub] + (n + dy) * (kHaloW * 128));
        };
        floatx16 acc[4];
        half8_t fb[2][4];
#pragma unroll
        for (int n = 0; n < 4; ++n) fb[0][n] = ldB(0, n);
#pragma unroll
        for (int ks = 0; ks < kBodyKSteps; ++ks) {
          const int r = ks & 1;
          if (ks + 1 < kBodyKSteps) {
#pragma unroll
            for (int n = 0; n < 4; ++n) fb[r ^ 1][n] = ldB(ks + 1, n);
          }
#pragma unroll
          for (int n = 0; n < 4; ++n)
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[ks], fb[r][n], ks == 0 ? bias16(bl) : acc[n], 0, 0, 0);
        }
        STK_STAMP(p, 4);
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int y = ty0 + 4 * rq + n;
          const half8_t v0 = act8_h<ACT>(acc[n], 0), v1 = act8_h<ACT>(acc[n], 8);
          half_t* row = out + (((size_t)b * s.Hp + y + s.pad) * s.Wp + tx0 + s.pad) * kWidth;
          const __amdgpu_buffer_rsrc_t rs =
              __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? min(kTileW, s.W - tx0) * 128 : 0, 0x00020000);
          const unsigned off = (unsigned)(col * 128 + 64 * m + 32 * h);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v0), rs, off, 0, kCpolDevice);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v1), rs, off + 16, 0, kCpolDevice);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores done (device scope)
      __syncthreads();
      if (tid == 0) tile_publish(done + t, epoch + p + 1);
      STK_STAMP(p, 5);
    }
    // the next pair's weights: in flight while the neighbourhood catches up
    if (p + 1 < npairs) load_w(2 * p + 2);
  }
}

#define PNP_X2_INST(A, HD)                                                                                   \
  template __global__ void conv_stack16x2_kernel<A, HD>(half_t* __restrict__, half_t* __restrict__,             \
                                                        const uint4* __restrict__, const float* __restrict__, int, \
                                                        ConvShape, int* __restrict__, int, int* __restrict__,    \
                                                        const float* __restrict__, int, const uint4* __restrict__, \
                                                        const float* __restrict__);
PNP_X2_INST(0, false)
PNP_X2_INST(1, false)
PNP_X2_INST(0, true)
PNP_X2_INST(1, true)
#undef PNP_X2_INST

// ------------------------------------------------------------------------------------
// Head layer C -> 64 (basic_models.py:16,27-28).  Input: the fp32 NCHW denoiser input u32
// (the same buffer the tail's residual reads), converted to fp16 (round to nearest even, as
// every fp16 cast here) while the halo is written to LDS as one 8-B quad per pixel (channels
// past C and pixels outside the image 0 = the conv's zero padding).  K = 9 taps x 4
// channels = 36, padded to 48 = 3 K-steps of 16: k = 4*tap + ch.
// ------------------------------------------------------------------------------------
// PREC 1: split weights (W_hi + W_lo, PNP_PREC_FP16W2), two MFMAs per product.  PREC 2
// (PNP_PREC_FP16X3): the input is split as well (x_hi + x_lo fp16), three MFMAs per product
// (x_hi W_hi + x_hi W_lo + x_lo W_hi), and the output is written as hi (out) + lo (out_lo)
// images for conv_s3.hip.  NC = C when it is a compile-time 1 or 3, 0 = runtime C <= kMaxC
// (channel index clamped, extra lanes 0).
template <int PREC, int NC>
__global__ __launch_bounds__(256) void conv_head_kernel(const float* __restrict__ in32, int Crt,
                                                         half_t* __restrict__ out,
                                                         half_t* __restrict__ out_lo,
                                                         const uint4* __restrict__ wpk,
                                                         const uint4* __restrict__ wpk_lo,
                                                         const float* __restrict__ bias,
                                                         ConvShape s, int act) {
  constexpr bool W2 = PREC >= 1, X3 = PREC == 2;
  __shared__ __attribute__((aligned(16))) unsigned char wl[kHeadWBytes];
  __shared__ __attribute__((aligned(16))) unsigned char wll[W2 ? kHeadWBytes : 16];
  __shared__ __attribute__((aligned(16))) uint2 hl[kHaloPix];
  __shared__ __attribute__((aligned(16))) uint2 hlo[X3 ? kHaloPix : 1];
  __shared__ __attribute__((aligned(16))) unsigned char stg_all[4 * 8192];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned char* stg = stg_all + wave * 8192;
  const int h = lane >> 5, col = lane & 31;
  for (int i = tid; i < kHeadWBytes / 16; i += 256) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
  if (W2)
    for (int i = tid; i < kHeadWBytes / 16; i += 256) reinterpret_cast<uint4*>(wll)[i] = wpk_lo[i];
  float bias_r[2][16];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) bias_r[m][r] = bias[32 * m + 16 * h + r];

  // the next tile's halo is loaded into registers while this tile computes (2 pixels per thread)
  constexpr int CM = NC ? NC : kMaxC;
  const int C = NC ? NC : Crt;
  const size_t plane = (size_t)s.H * s.W;
  float pre[2][CM];
  bool pin[2];
  auto load_halo = [&](int tt) {
    int pb_, pty, ptx;
    decode_tile(tt < s.tiles ? tt : s.tiles - 1, s, pb_, pty, ptx);
    const float* base = in32 + (size_t)pb_ * C * plane;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = tid + 256 * k;
      const int pl = p < kHaloPix ? p : kHaloPix - 1;
      const int pr = pl / kHaloW, pc = pl - pr * kHaloW;
      const int gy = pty - 1 + pr, gx = ptx - 1 + pc;
      pin[k] = gy >= 0 && gy < s.H && gx >= 0 && gx < s.W;
      const size_t o = pin[k] ? (size_t)gy * s.W + gx : 0;
#pragma unroll
      for (int c = 0; c < CM; ++c) pre[k][c] = base[(size_t)(NC ? c : min(c, C - 1)) * plane + o];
    }
  };
  auto quad = [&](int k, bool lo) {           // lo: the low halves x - fp16(x)
    _Float16 h[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float v = pre[k][c < CM ? c : 0];
      const _Float16 vh = (_Float16)v;
      h[c] = (c < CM && (NC || c < C) && pin[k]) ? (lo ? (_Float16)(v - (float)vh) : vh) : (_Float16)0;
    }
    return make_uint2((uint32_t)__builtin_bit_cast(uint16_t, h[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[1]) << 16),
                      (uint32_t)__builtin_bit_cast(uint16_t, h[2]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[3]) << 16));
  };
  if (blockIdx.x < s.tiles) load_halo(blockIdx.x);
  for (int t = blockIdx.x; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    // (lds_barrier: the previous tile's stores stay in flight; the halo registers' loads are
    // waited for where they are used)
    lds_barrier();
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (tid + 256 * k < kHaloPix) {
        hl[tid + 256 * k] = quad(k, false);
        if (X3) hlo[tid + 256 * k] = quad(k, true);
      }
    lds_barrier();
    load_halo(t + gridDim.x);
    floatx16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
#pragma unroll
    for (int ks = 0; ks < kHeadKSteps; ++ks) {
      const half8_t a0 = *reinterpret_cast<const half8_t*>(wl + ((ks * 2 + 0) * 64 + lane) * 16);
      const half8_t a1 = *reinterpret_cast<const half8_t*>(wl + ((ks * 2 + 1) * 64 + lane) * 16);
      const int t0 = 4 * ks + 2 * h;          // this lane's two taps (k = 8h .. 8h+7)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        uint2 q0 = make_uint2(0, 0), q1 = make_uint2(0, 0);
        if (t0 < 9) q0 = hl[(2 * wave + n + t0 / 3) * kHaloW + col + t0 % 3];
        if (t0 + 1 < 9) q1 = hl[(2 * wave + n + (t0 + 1) / 3) * kHaloW + col + (t0 + 1) % 3];
        uint4 q = make_uint4(q0.x, q0.y, q1.x, q1.y);
        const half8_t bf = *reinterpret_cast<const half8_t*>(&q);
        if (X3) {                              // x_lo W_hi
          uint2 r0 = make_uint2(0, 0), r1 = make_uint2(0, 0);
          if (t0 < 9) r0 = hlo[(2 * wave + n + t0 / 3) * kHaloW + col + t0 % 3];
          if (t0 + 1 < 9) r1 = hlo[(2 * wave + n + (t0 + 1) / 3) * kHaloW + col + (t0 + 1) % 3];
          uint4 rq = make_uint4(r0.x, r0.y, r1.x, r1.y);
          const half8_t bfl = *reinterpret_cast<const half8_t*>(&rq);
          if (n == 0) {
            acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bfl, acc00, 0, 0, 0);
            acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, bfl, acc10, 0, 0, 0);
          } else {
            acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bfl, acc01, 0, 0, 0);
            acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, bfl, acc11, 0, 0, 0);
          }
        }
        if (n == 0) {
          acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bf, acc00, 0, 0, 0);
          acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, bf, acc10, 0, 0, 0);
        } else {
          acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bf, acc01, 0, 0, 0);
          acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, bf, acc11, 0, 0, 0);
        }
        if (W2) {
          const half8_t l0 = *reinterpret_cast<const half8_t*>(wll + ((ks * 2 + 0) * 64 + lane) * 16);
          const half8_t l1 = *reinterpret_cast<const half8_t*>(wll + ((ks * 2 + 1) * 64 + lane) * 16);
          if (n == 0) {
            acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(l0, bf, acc00, 0, 0, 0);
            acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(l1, bf, acc10, 0, 0, 0);
          } else {
            acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(l0, bf, acc01, 0, 0, 0);
            acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(l1, bf, acc11, 0, 0, 0);
          }
        }
      }
    }
    // epilogue through wave-private LDS staging: 2 rows x 32 pixels x 128 B, 16-B chunks
    // XOR-swizzled by pixel (conflict-free writes), stored back as full 128-B pixel lines
    // (1 KiB contiguous per instruction) instead of 16-B pieces at a 128-B stride.
#pragma unroll
    for (int part = 0; part < (X3 ? 2 : 1); ++part) {   // X3: hi image, then lo image
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const floatx16& a0 = n == 0 ? acc00 : acc01;
        const floatx16& a1 = n == 0 ? acc10 : acc11;
        unsigned char* px = stg + (n * 32 + col) * 128;
        const int sw = col & 7;
        half8_t v[4];
        if (X3) {                               // fp32 bias + activation, then the hi or lo half
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              const floatx16& a = q < 2 ? a0 : a1;
              float f = a[8 * (q & 1) + r] * kSplitWInv + bias_r[q >> 1][8 * (q & 1) + r];   // weights at 2^8
              f = act == 0 ? fmaxf(f, f * 0.01f) : fmaxf(f, 0.f);
              const _Float16 fh = (_Float16)f;
              v[q][r] = part == 0 ? fh : (_Float16)(f - (float)fh);
            }
        } else if (act == 0) {                  // packed bias + activation (bit-identical to act_fn)
          v[0] = bias_act8<0>(a0, 0, bias_r[0]); v[1] = bias_act8<0>(a0, 8, bias_r[0] + 8);
          v[2] = bias_act8<0>(a1, 0, bias_r[1]); v[3] = bias_act8<0>(a1, 8, bias_r[1] + 8);
        } else {
          v[0] = bias_act8<1>(a0, 0, bias_r[0]); v[1] = bias_act8<1>(a0, 8, bias_r[0] + 8);
          v[2] = bias_act8<1>(a1, 0, bias_r[1]); v[3] = bias_act8<1>(a1, 8, bias_r[1] + 8);
        }
        *reinterpret_cast<half8_t*>(px + 16 * ((2 * h) ^ sw)) = v[0];          // channels 16h .. +7
        *reinterpret_cast<half8_t*>(px + 16 * ((2 * h + 1) ^ sw)) = v[1];      // 16h+8 .. +15
        *reinterpret_cast<half8_t*>(px + 16 * ((4 + 2 * h) ^ sw)) = v[2];      // 32+16h .. +7
        *reinterpret_cast<half8_t*>(px + 16 * ((5 + 2 * h) ^ sw)) = v[3];      // 32+16h+8 .. +15
      }
      half_t* dst = part == 0 ? out : out_lo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {             // 8 pixels x 8 chunks per instruction
        const int n = j >> 2, p = 8 * (j & 3) + (lane >> 3), c = lane & 7;
        const uint4 q = *reinterpret_cast<const uint4*>(stg + (n * 32 + p) * 128 + 16 * (c ^ (p & 7)));
        const int y = ty0 + 2 * wave + n, x = tx0 + p;
        if (y < s.H && x < s.W)
        {
          if (kNtHead)
            __builtin_nontemporal_store(__builtin_bit_cast(v4i_t, q),
                                        reinterpret_cast<v4i_t*>(dst + (((size_t)b * s.Hp + y + s.pad) * s.Wp + x + s.pad) *
                                                                           kWidth + 8 * c));
          else
            *reinterpret_cast<uint4*>(dst + (((size_t)b * s.Hp + y + s.pad) * s.Wp + x + s.pad) * kWidth + 8 * c) = q;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Tail layer 64 -> C (basic_models.py:18,35-36) + residual + clamp (denoiser.py:42),
// writing the new primal iterate x+ in fp32 NCHW.  v_mfma_f32_16x16x32_f16 with the C
// output channels as the (padded-to-16) A rows, kept in registers for the launch (72
// VGPRs); each wave covers 4 N-tiles of 16 px (2 tile rows).  The kernel is HBM-bound
// (8.4 MB of fp16 activations in, 2 x 0.8 MB fp32 per RGB 256^2 image), so it runs the
// variant-3 memory pipeline: 3-deep LDS-DMA halo ring (two tiles in flight per CU), the
// residual input x loaded by range-checked buffer loads at tile start (older than the
// DMA, so the compiler's vmcnt for them does not wait on it), outputs moved to a
// row-major lane layout with ds_bpermute (no LDS memory access, so no wait on the pending
// LDS-DMA) so every load/store is one 64-lane row-contiguous fp32 instruction per channel,
// and a counted vmcnt at the tile boundary that waits for the next tile's DMA only.
// ------------------------------------------------------------------------------------
constexpr int kTailHalo = 44 * 1024;                           // 11 uniform DMA slots per wave
constexpr int kTailLds = 3 * kTailHalo;                         // 135168 B

template <bool W2>
__global__ __launch_bounds__(256, 1) void conv_tail_kernel(const half_t* __restrict__ in,
                                                            const float* __restrict__ xin,
                                                            float* __restrict__ xout,
                                                            const uint4* __restrict__ wpk,
                                                            const uint4* __restrict__ wpk_lo,
                                                            const float* __restrict__ bias,
                                                            ConvShape s, int C, int residual_sign,
                                                            int clamp_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q4 = lane >> 4, c16 = lane & 15;
  half8_t wA[kTailKSteps], wL[W2 ? kTailKSteps : 1];
#pragma unroll
  for (int ks = 0; ks < kTailKSteps; ++ks) {
    wA[ks] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wpk) + (ks * 64 + lane) * 16);
    if (W2)
      wL[ks] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wpk_lo) + (ks * 64 + lane) * 16);
  }
  float bias_r[kMaxC];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) bias_r[c] = c < C ? bias[c] : 0.f;
  const unsigned plane = (unsigned)(s.H * s.W);

  auto buf = [&](int i) { return smem + i * kTailHalo; };
  RingDma<4, true> dma;
  dma.init(s, wave);
  auto issue_dma = [&](int tt, int bi) {      // clamped: always the same instruction count
    dma.issue(buf(bi), in, s, tt < s.tiles ? tt : s.tiles - 1, wave);
  };

  int t = blockIdx.x;      // (an XCD-aware tile order measured the same: 0.5599 vs 0.5545-0.5599 ms, r03)
  if (t < s.tiles) {
    issue_dma(t, 0);
    issue_dma(t + gridDim.x, 1);
    asm volatile("s_waitcnt vmcnt(11)" ::: "memory");                 // tile t landed
  }
  __syncthreads();
  int cur = 0;
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    // store layout: lane -> pixel (tile row 2*wave + lane/32, column lane%32)
    const int y = ty0 + 2 * wave + (lane >> 5), x = tx0 + (lane & 31);
    const unsigned off = (y < s.H && x < s.W) ? (unsigned)(y * s.W + x) * 4u : 0x80000000u;   // OOR: dropped
    __amdgpu_buffer_rsrc_t rs[kMaxC];
    float xi[kMaxC];
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {         // always kMaxC loads (c >= C: zero-size descriptor)
      rs[c] = __builtin_amdgcn_make_buffer_rsrc((void*)(xin + ((size_t)b * C + (c < C ? c : 0)) * plane), (short)0,
                                                c < C ? (int)(plane * 4u) : 0, 0x00020000);
      xi[c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs[c], off, 0, 0));
    }
    __builtin_amdgcn_sched_barrier(0);       // residual loads stay older than the DMA
    const int nxt2 = cur >= 1 ? cur - 1 : 2;
    // (r06) tile t+2's 11 slots issue one per K-step (1 .. 11) between MFMAs: one wave per SIMD,
    // so a burst before the K-loop had nothing to hide behind
    const int tn2 = t + 2 * gridDim.x;
    const __amdgpu_buffer_rsrc_t drs = RingDma<4, true>::rsrc(in, s, tn2 < s.tiles ? tn2 : s.tiles - 1);
    unsigned char* dbuf = buf(nxt2);
    static_assert(RingDma<4, true>::kSlots < kTailKSteps, "the slots fit in the K-loop");
    const unsigned char* hl = buf(cur);
    auto ldB = [&](int ks, int n) {
      const int tap = ks >> 1;
      return *reinterpret_cast<const half8_t*>(
          hl + halo_off(2 * wave + (n >> 1) + tap / 3, 16 * (n & 1) + c16 + tap % 3, 4 * (ks & 1) + q4));
    };
    floatx4 acc[4] = {};
    half8_t fb[2][4];
#pragma unroll
    for (int n = 0; n < 4; ++n) fb[0][n] = ldB(0, n);
#pragma unroll
    for (int ks = 0; ks < kTailKSteps; ++ks) {          // step ks+1 read while ks computes
      const int r = ks & 1;
      if (ks + 1 < kTailKSteps) {
#pragma unroll
        for (int n = 0; n < 4; ++n) fb[r ^ 1][n] = ldB(ks + 1, n);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wA[ks], fb[r][n], acc[n], 0, 0, 0);
      if (W2) {
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wL[W2 ? ks : 0], fb[r][n], acc[n], 0, 0, 0);
      }
      if (ks >= 1 && ks <= RingDma<4, true>::kSlots) dma.issue_slot(dbuf, drs, ks - 1, wave);
    }
    // C/D map of 16x16: col = lane & 15 (pixel of N-tile n), row = 4*(lane>>4) + r (channel):
    // lanes 0..15 hold channels 0..3 of N-tile n.  Store-layout lane l wants N-tile l>>4,
    // pixel l&15: four cross-lane permutes per channel, then a per-lane select.
    float net[kMaxC];
    const int src = (lane & 15) << 2;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      float pv[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float e = acc[n][c];   // a copy: bit_cast of an ext-vector element lvalue reads element 0 here
        pv[n] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, e)));
      }
      const int nn = lane >> 4;
      net[c] = nn == 0 ? pv[0] : nn == 1 ? pv[1] : nn == 2 ? pv[2] : pv[3];
    }

#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      const float nc = net[c] + bias_r[c];
      float o = residual_sign > 0 ? nc + xi[c] : xi[c] - nc;
      if (clamp_out) o = fminf(fmaxf(o, 0.f), 1.f);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, o),
                                            __builtin_amdgcn_make_buffer_rsrc(
                                                (void*)(xout + ((size_t)b * C + (c < C ? c : 0)) * plane), (short)0,
                                                c < C ? (int)(plane * 4u) : 0, 0x00020000),
                                            off, 0, kNtTail);
    }
    // tile t+1 landed: younger than its DMA are this tile's 4 loads, DMA of t+2 and 4 stores
    asm volatile("s_waitcnt vmcnt(19) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
}

#define PNP_TAIL_INST(W)                                                                                     \
  template __global__ void conv_tail_kernel<W>(const half_t* __restrict__, const float* __restrict__,         \
                                               float* __restrict__, const uint4* __restrict__,                \
                                               const uint4* __restrict__, const float* __restrict__, ConvShape, \
                                               int, int, int);
PNP_TAIL_INST(false)
PNP_TAIL_INST(true)
#undef PNP_TAIL_INST

// ------------------------------------------------------------------------------------
// Host-side weight packing (fp32 PyTorch layout -> fp16 MFMA fragment order).
// ------------------------------------------------------------------------------------
static inline uint16_t f32_to_f16_bits(float f) {
  _Float16 h = (_Float16)f;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

// W: [64][64][3][3].  out: [36 k-steps][2 M-tiles][64 lanes][8] fp16 bits.
void pack_body_weights(const float* W, uint16_t* out) {
  for (int ks = 0; ks < kBodyKSteps; ++ks) {
    const int tap = ks / 4, sub = ks % 4, ky = tap / 3, kx = tap % 3;
    for (int m = 0; m < 2; ++m)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int co = 32 * m + mfma32_row_to_channel(l & 31);
          const int ci = 16 * sub + 8 * (l >> 5) + j;
          out[((ks * 2 + m) * 64 + l) * 8 + j] = f32_to_f16_bits(W[((co * 64 + ci) * 3 + ky) * 3 + kx]);
        }
  }
}

// W: [64][64][3][3].  out: [18 k-steps][2 M-tiles][2 subtiles][64 lanes][8] fp16 bits for
// v_mfma_f32_16x16x32_f16: lane l holds A[row l & 15][k = 8 (l >> 4) .. +7]; row r of
// subtile q is channel 32 M + 8 (r >> 2) + 4 q + (r & 3); k-step ks = tap ks >> 1, input
// channels 32 (ks & 1) + k.
void pack_body_weights16(const float* W, uint16_t* out) {
  for (int ks = 0; ks < kX8KSteps; ++ks) {
    const int tap = ks >> 1, hs = ks & 1, ky = tap / 3, kx = tap % 3;
    for (int M = 0; M < 2; ++M)
      for (int q = 0; q < 2; ++q)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int r = l & 15;
            const int co = 32 * M + 8 * (r >> 2) + 4 * q + (r & 3);
            const int ci = 32 * hs + 8 * (l >> 4) + j;
            out[(((ks * 2 + M) * 2 + q) * 64 + l) * 8 + j] = f32_to_f16_bits(W[((co * 64 + ci) * 3 + ky) * 3 + kx]);
          }
  }
}

// W: [64][C][3][3].  k = 4*tap + ch, 3 k-steps of 16.
void pack_head_weights(const float* W, int C, uint16_t* out) {
  for (int ks = 0; ks < kHeadKSteps; ++ks)
    for (int m = 0; m < 2; ++m)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int co = 32 * m + mfma32_row_to_channel(l & 31);
          const int k = 16 * ks + 8 * (l >> 5) + j;
          const int tap = k / 4, ch = k % 4;
          float v = 0.f;
          if (tap < 9 && ch < C) v = W[((co * C + ch) * 3 + tap / 3) * 3 + tap % 3];
          out[((ks * 2 + m) * 64 + l) * 8 + j] = f32_to_f16_bits(v);
        }
}

// W: [C][64][3][3].  16x16x32: lane l holds A[row l&15][k = 8(l>>4)+j]; k-step ks covers
// tap ks/2, input channels 32*(ks&1) .. +31.
void pack_tail_weights(const float* W, int C, uint16_t* out) {
  for (int ks = 0; ks < kTailKSteps; ++ks) {
    const int tap = ks / 2, ky = tap / 3, kx = tap % 3;
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) {
        const int co = l & 15;
        const int ci = 32 * (ks & 1) + 8 * (l >> 4) + j;
        float v = 0.f;
        if (co < C) v = W[((co * 64 + ci) * 3 + ky) * 3 + kx];
        out[(ks * 64 + l) * 8 + j] = f32_to_f16_bits(v);
      }
  }
}

// ------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------
ConvShape make_conv_shape(int B, int H, int W) {
  ConvShape s;
  s.B = B; s.H = H; s.W = W;
  s.pad = kActPad;
  s.Hp = H + 2 * kActPad; s.Wp = W + 2 * kActPad;
  s.tiles_x = (W + kTileW - 1) / kTileW;
  s.tiles_y = (H + kTileH - 1) / kTileH;
  s.tiles = B * s.tiles_x * s.tiles_y;
  return s;
}

hipError_t conv_kernels_init() {
  hipError_t e = hipSuccess;
  for (const void* k : {(const void*)conv_body_v3_kernel<0, 0>, (const void*)conv_body_v3_kernel<0, 1>
#ifdef PNP_PROFILING
                        , (const void*)conv_body_v3_kernel<1, 0>, (const void*)conv_body_v3_kernel<2, 0>,
                        (const void*)conv_body_v3_kernel<3, 0>, (const void*)conv_body_v3_kernel<4, 0>,
                        (const void*)conv_body_v3_kernel<6, 0>
#endif
       }) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kV3Lds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_body_x8_kernel<0, kX8Pair>, (const void*)conv_body_x8_kernel<1, kX8Pair>,
                        (const void*)conv_body_x8_kernel<0, kX8Head>, (const void*)conv_body_x8_kernel<1, kX8Head>,
                        (const void*)conv_body_x8_kernel<0, kX8Tail>, (const void*)conv_body_x8_kernel<1, kX8Tail>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kF2Lds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_body_w2_kernel<0>, (const void*)conv_body_w2_kernel<1>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kW2Lds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_stack16_kernel<0>, (const void*)conv_stack16_kernel<1>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kStkLds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_stack16x2_kernel<0, false>, (const void*)conv_stack16x2_kernel<1, false>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kX2Lds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_stack16x2_kernel<0, true>, (const void*)conv_stack16x2_kernel<1, true>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kX2LdsHead);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_tail_kernel<false>, (const void*)conv_tail_kernel<true>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kTailLds);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

void launch_conv_head(const float* in32, int C, half_t* out, const void* w, const void* w_lo, const float* bias,
                      const ConvShape& s, int act, int num_cus, int blocks_per_cu, hipStream_t st, half_t* out_lo) {
  // (grid of 2 / 3 / 4 / 6 blocks per CU at the metric: 0.453 / 0.548 / 0.461 / 0.459 ms, r03)
  const int grid = s.tiles < num_cus * blocks_per_cu ? s.tiles : num_cus * blocks_per_cu;
#define HEAD(PV, NCV)                                                                                            \
  hipLaunchKernelGGL((conv_head_kernel<PV, NCV>), dim3(grid), dim3(256), 0, st, in32, C, out, out_lo,              \
                     (const uint4*)w, (const uint4*)w_lo, bias, s, act)
  if (out_lo) {
    if (C == 3) HEAD(2, 3); else if (C == 1) HEAD(2, 1); else HEAD(2, 0);
  } else if (w_lo) {
    if (C == 3) HEAD(1, 3); else if (C == 1) HEAD(1, 1); else HEAD(1, 0);
  } else {
    if (C == 3) HEAD(0, 3); else if (C == 1) HEAD(0, 1); else HEAD(0, 0);
  }
#undef HEAD
}

// Two body layers per launch: conv_body_x8 (16x16x32 MFMAs, w16_*: pack_body_weights16).
// (The round-2 A/B variants on 32x32x16 fragments, w32_*: conv_body_f2 / conv_body_f8, are in
// git history before round 3; DESIGN.md §3 keeps their measurements.)
void launch_conv_body_f2(const half_t* in, half_t* out, const void* w16_1, const void* w16_2, const void* w32_1,
                         const void* w32_2, const float* b1, const float* b2, const ConvShape& s, int act,
                         int num_cus, hipStream_t st, int mode, const X8Ends* ends) {
  const int strips_x = (s.W + kTileW - 1) / kTileW, nstrips = s.B * strips_x;
  // rows per strip: H + 1 (the separator), at least 24 so that a step's look-ahead rows (up to
  // 8 J + 16) lie at most one strip ahead (locate())
  const int srows = s.H + 1 < 24 ? 24 : s.H + 1;
  const int grid = nstrips < num_cus ? nstrips : num_cus;
  const X8Ends e = ends ? *ends : X8Ends{};
#define F2_LAUNCH(KERN, NT, W1, W2)                                                                              \
  hipLaunchKernelGGL((KERN), dim3(grid), dim3(NT), kF2Lds, st, in, out, (const uint4*)(W1), b1, (const uint4*)(W2), \
                     b2, s, strips_x, nstrips, srows, e)
  if (mode == kX8Head) {
    if (act == 0) F2_LAUNCH((conv_body_x8_kernel<0, kX8Head>), 512, w16_1, w16_2);
    else F2_LAUNCH((conv_body_x8_kernel<1, kX8Head>), 512, w16_1, w16_2);
  } else if (mode == kX8Tail) {
    if (act == 0) F2_LAUNCH((conv_body_x8_kernel<0, kX8Tail>), 512, w16_1, w16_2);
    else F2_LAUNCH((conv_body_x8_kernel<1, kX8Tail>), 512, w16_1, w16_2);
  } else {
    if (act == 0) F2_LAUNCH((conv_body_x8_kernel<0, kX8Pair>), 512, w16_1, w16_2);
    else F2_LAUNCH((conv_body_x8_kernel<1, kX8Pair>), 512, w16_1, w16_2);
  }
#undef F2_LAUNCH
  (void)w32_1; (void)w32_2;
}

void launch_conv_body_w2(const half_t* in, half_t* out, const void* w, const void* w_lo, const float* bias,
                         const ConvShape& s, int act, int num_cus, hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  if (act == 0)
    hipLaunchKernelGGL((conv_body_w2_kernel<0>), dim3(grid), dim3(256), kW2Lds, st, in, out, (const uint4*)w,
                       (const uint4*)w_lo, bias, s);
  else
    hipLaunchKernelGGL((conv_body_w2_kernel<1>), dim3(grid), dim3(256), kW2Lds, st, in, out, (const uint4*)w,
                       (const uint4*)w_lo, bias, s);
}

void launch_conv_body(const half_t* in, half_t* out, const void* w, const float* bias, const ConvShape& s,
                      int act, int num_cus, int ablate, hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
#define V3(A, F) hipLaunchKernelGGL((conv_body_v3_kernel<A, F>), dim3(grid), dim3(512), kV3Lds, st, in, out, \
                                    (const uint4*)w, bias, s)
#ifdef PNP_PROFILING
  switch (act == 0 ? ablate : 0) {            // profiling build only: parts skipped, results wrong
    case 1: V3(1, 0); return;
    case 2: V3(2, 0); return;
    case 3: V3(3, 0); return;
    case 4: V3(4, 0); return;
    case 6: V3(6, 0); return;
    default: break;
  }
#else
  (void)ablate;
#endif
  if (act != 0) V3(0, 1);
  else V3(0, 0);
#undef V3
}

bool stack16_takes_head(int nbody, bool pairs) { return pairs && nbody >= 2 && (nbody & 1) == 0; }

int launch_conv_stack16(half_t* a, half_t* b, const void* w, const float* bias, int nbody, const ConvShape& s,
                        int act, int num_cus, int* done, int epoch, int* err, bool pairs, hipStream_t st,
                        const float* u32, int C, const void* head_w, const float* head_b) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  const uint4* wp = (const uint4*)w;
  if (stack16_takes_head(nbody, pairs)) {           // two layers per hand-off
    const int np = nbody / 2;
    const uint4* hw = (const uint4*)head_w;
    if (u32)                                         // the head computed in pair 0
      (void)persistent_launch(act == 0 ? conv_stack16x2_kernel<0, true> : conv_stack16x2_kernel<1, true>, grid, 256,
                              kX2LdsHead, st, a, b, wp, bias, np, s, done, epoch, err, u32, C, hw, head_b);
    else
      (void)persistent_launch(act == 0 ? conv_stack16x2_kernel<0, false> : conv_stack16x2_kernel<1, false>, grid, 256,
                              kX2Lds, st, a, b, wp, bias, np, s, done, epoch, err, u32, C, hw, head_b);
    return np & 1;
  }
  (void)persistent_launch(act == 0 ? conv_stack16_kernel<0> : conv_stack16_kernel<1>, grid, 256, kStkLds, st, a, b, wp,
                    bias, nbody, s, done, epoch, err);
  return nbody & 1;
}

void launch_conv_tail(const half_t* in, const float* xin, float* xout, const void* w, const void* w_lo,
                      const float* bias, const ConvShape& s, int C, int residual_sign, int clamp_out, int num_cus,
                      hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  if (w_lo)
    hipLaunchKernelGGL(conv_tail_kernel<true>, dim3(grid), dim3(256), kTailLds, st, in, xin, xout,
                       (const uint4*)w, (const uint4*)w_lo, bias, s, C, residual_sign, clamp_out);
  else
    hipLaunchKernelGGL(conv_tail_kernel<false>, dim3(grid), dim3(256), kTailLds, st, in, xin, xout,
                       (const uint4*)w, (const uint4*)nullptr, bias, s, C, residual_sign, clamp_out);
}

}  // namespace pnp

#ifdef STACK_STAMPS
extern "C" int pnp_diag_stack_stamps(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(pnp::stack_stamps), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

#ifdef X8_CLOCK
extern "C" int pnp_diag_x8_clock(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(pnp::x8_clock), n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
