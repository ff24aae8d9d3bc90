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
// pixel one 128-B line): the two-layer fused body kernel reads a 2-pixel halo.
//
//   conv_head      C -> 64, from the padded NHWC4 fp16 input
//   conv_body_v3   64 -> 64, one layer per launch
//   conv_body2     64 -> 64 -> 64, two layers per launch (halves the activation traffic)
//   conv_tail      64 -> C + residual + clamp, fp32 NCHW out
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

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));

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
                                                 off[j], 0, 0, 0);
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
// non-temporal stores; the 16x16x32 form is kept below as variant 3; DESIGN.md.)
// ------------------------------------------------------------------------------------
constexpr int kV3Stage = 3 * kV3Halo;
constexpr int kV3Bias = kV3Stage + 8 * 4096;
constexpr int kV3Lds = kV3Bias + 256;                           // 163584 B

// ABL: bits 1/2/4 = profiling ablation (PNP_TUNE_ABLATE, results wrong), compile-time;
//      bit 8 = stagger: waves 4-7 (the SIMD partners of waves 0-3) run each tile's epilogue
//      at the start of the next tile, after the barrier, so on every SIMD one wave's
//      bias/activation/staging work overlaps its partner's MFMAs (MI355X_MICROARCH.md, "two
//      waves per SIMD", item 9).  Results are bit-identical.
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
  constexpr bool kStagger = (ABL & 8) != 0;
  const bool late = kStagger && wave >= 4;
  if constexpr ((ABL & 16) != 0) {            // static priority for the second-dispatched half
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  floatx16 acc0 = {}, acc1 = {};
  int pb = 0, pty0 = 0, ptx0 = 0;             // previous tile (late waves' deferred epilogue)
  bool have_prev = false;
  auto epilogue = [&](int eb, int ety0, int etx0) {   // bias + activation -> fp16 -> staging (wave-private)
    const float* bl = bias_l + 32 * m + 16 * h;
    const int sw = (col >> 1) & 3;    // ds_write_b128 banks repeat every 128 B: 8 lanes distinct
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int pix = n * 32 + col;
      const floatx16& a = n == 0 ? acc0 : acc1;
      *reinterpret_cast<half8_t*>(stg + pix * 64 + 16 * ((2 * h) ^ sw)) = bias_act8<ACT>(a, 0, bl);
      *reinterpret_cast<half8_t*>(stg + pix * 64 + 16 * ((2 * h + 1) ^ sw)) = bias_act8<ACT>(a, 8, bl + 8);
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
    if (late && have_prev) epilogue(pb, pty0, ptx0);
    const int nxt2 = cur >= 1 ? cur - 1 : 2;  // (cur + 2) % 3
    if constexpr ((ABL & 1) == 0) issue_dma(t + 2 * gridDim.x, nxt2);
    const unsigned char* hl = buf(cur);
    auto ldB = [&](int ks, int n) {
      const int tap = ks >> 2, sub = ks & 3;
      return *reinterpret_cast<const half8_t*>(
          hl + halo_off(2 * rp + n + tap / 3, col + tap % 3, 2 * sub + h));
    };
    acc0 = floatx16{};
    acc1 = floatx16{};
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
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[r][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[r][1], acc1, 0, 0, 0);
      if ((ks & 7) == 4) {
        __builtin_amdgcn_sched_barrier(0);
        stage_store(ks >> 3, sv);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (!late) epilogue(b, ty0, tx0);
    pb = b; pty0 = ty0; ptx0 = tx0;
    have_prev = true;
    // tile t+1 landed: only the DMA of t+2 (ndma ops) and this tile's 4 stores are younger
    if (ndma == 6) asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
  if (late && have_prev) epilogue(pb, pty0, ptx0);
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
PNP_V3_INST(8, 0)
PNP_V3_INST(8, 1)
PNP_V3_INST(16, 0)
PNP_V3_INST(24, 0)
PNP_V3_INST(1, 0)
PNP_V3_INST(2, 0)
PNP_V3_INST(3, 0)
PNP_V3_INST(4, 0)
PNP_V3_INST(6, 0)
#undef PNP_V3_INST

// ------------------------------------------------------------------------------------
// Body layer on v_mfma_f32_16x16x32_f16 (PNP_TUNE_BODY_VARIANT 3).  Same tile, 3-deep
// LDS-DMA ring and resident weights as conv_body_v3; the 16x16x32 form issues in half the
// cycles of 32x32x16 for half the FLOPs and the chip holds a higher clock on it
// (MI355X_MICROARCH.md, DVFS give-back item 7).  Wave w owns channels 32m..32m+31 (m = w&1)
// as two 16-row M-tiles and its two tile rows as four 16-pixel N-tiles; one K-step is one
// tap x 32 input channels (18 steps, 8 MFMAs each, 4 activation fragments from LDS): the
// same LDS bytes per MFMA FLOP as v3.
// Planar halo: 16-B chunk c (channels 8c..8c+7) of halo pixel p at c * 5632 + 16 p (planes
// of 352 pixels, a multiple of 16, so the q = 0..3 lane groups of a ds_read_b128 over 16
// consecutive pixels hit 16 distinct bank slots).  Every B-fragment address is then ONE
// per-lane register (16 col + 5632 q) plus an immediate: no per-tap address registers, no
// spills - a spilled register reloaded inside the K-loop waits on vmcnt(0), i.e. on the
// in-flight halo DMA, and serialises the ring.
// A row R of M-tile i is channel 8(R>>2) + 4i + (R&3) of the wave's 32, so lane group
// q = lane>>4 owns channels 8q..8q+7 of its pixel: the epilogue stores 16 B per lane and
// N-tile straight from registers (16 pixels x 64 B per instruction), no staging.
// LDS: 3 x 45056 B halo + bias = 135424 B.
// Measured (B = 256): 1.28 ms vs 1.21-1.24 for conv_body_v3; PMC at B = 64: clock 1.78 vs
// 1.60 GHz, MFMA busy 48 vs 56 %.  The planar halo took it from 1.94 ms (14 spilled address
// registers reloaded inside the K-loop).  Not kept: B double-buffered (same), stores
// deferred into the next K-loop from registers (1.36 ms), one wave per SIMD holding all
// 64 channels (4 MFMAs per B fragment, 450 registers: 1.45 ms).
// ------------------------------------------------------------------------------------
constexpr int kBody16KSteps = 18;
constexpr int kPlanePix = 352;                                  // >= 340, multiple of 16
constexpr int kPlaneBytes = kPlanePix * 16;                     // 5632
constexpr int kV5Halo = 8 * kPlaneBytes;                        // 45056
constexpr int kV5Slots = kV5Halo / 1024;                        // 44 DMA pieces of 64 x 16 B
constexpr int kV5Bias = 3 * kV5Halo;
constexpr int kV5Lds = kV5Bias + 256;                           // 135424

template <int ACT>
__global__ __launch_bounds__(512, 2) void conv_body_v4_kernel(const half_t* __restrict__ in,
                                                               half_t* __restrict__ out,
                                                               const uint4* __restrict__ wpk,
                                                               const float* __restrict__ bias,
                                                               ConvShape s) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* bias_l = reinterpret_cast<float*>(smem + kV5Bias);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = wave & 1, rp = wave >> 1;    // channel half, row pair
  const int q = lane >> 4, col = lane & 15;
  if (tid < kWidth) bias_l[tid] = bias[tid];

  half8_t wA[kBody16KSteps][2];               // [k-step][M-tile], resident for the launch
#pragma unroll
  for (int ks = 0; ks < kBody16KSteps; ++ks)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      wA[ks][i] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wpk) +
                                                    (((ks * 2 + m) * 2 + i) * 64 + lane) * 16);

  // DMA: piece g (64 lanes x 16 B) of the planar image; wave w issues g = w, w + 8, ...
  constexpr int kSlotsPerWave = (kV5Slots + 7) / 8;             // 6 (waves >= 4: 5)
  const int ndma = (kV5Slots - wave + 7) / 8;
  unsigned doff[kSlotsPerWave];
#pragma unroll
  for (int j = 0; j < kSlotsPerWave; ++j) {
    const int k = 64 * (8 * j + wave) + lane;                   // 16-B unit of the planar image
    const int c = k / kPlanePix, p = min(k - c * kPlanePix, kHaloPix - 1);
    const int pr = p / kHaloW, pc = p - pr * kHaloW;
    doff[j] = (unsigned)(((pr * s.Wp + pc) * kWidth + 8 * min(c, 7)) * 2);
  }
  auto buf = [&](int i) { return smem + i * kV5Halo; };
  auto issue_dma = [&](int tt, int bi) {
    int b, ty0, tx0;
    decode_tile(tt < s.tiles ? tt : s.tiles - 1, s, b, ty0, tx0);
    const half_t* base = in + (((size_t)b * s.Hp + ty0 + s.pad - 1) * s.Wp + tx0 + s.pad - 1) * kWidth;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < kSlotsPerWave; ++j)
      if (j < ndma)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(buf(bi) + (8 * j + wave) * 1024),
                                                 16, doff[j], 0, 0, 0);
  };

  int t = blockIdx.x;
  if (t < s.tiles) {
    issue_dma(t, 0);
    issue_dma(t + gridDim.x, 1);
    if (ndma == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // tile t landed
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  }
  __syncthreads();
  const int lane_off = q * kPlaneBytes + col * 16 + rp * 2 * kHaloW * 16;
  floatx4 acc[4][2];
  int cur = 0;
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const int nxt2 = cur >= 1 ? cur - 1 : 2;  // (cur + 2) % 3
    issue_dma(t + 2 * gridDim.x, nxt2);
    const unsigned char* hl = buf(cur) + lane_off;
    auto ldB = [&](int ks, int n) {           // everything but lane_off is an immediate
      const int tap = ks >> 1, sub = ks & 1;
      const int pr = (n >> 1) + tap / 3, pc = 16 * (n & 1) + tap % 3;
      return *reinterpret_cast<const half8_t*>(hl + 4 * sub * kPlaneBytes + (pr * kHaloW + pc) * 16);
    };
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n][0] = acc[n][1] = floatx4{};
    // rolling ring: fragment n of step ks+1 is read right after the two MFMAs of step ks
    // that use fragment n (sched barriers pin the order, so it reuses n's registers)
    half8_t fb[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) fb[n] = ldB(0, n);
#pragma unroll
    for (int ks = 0; ks < kBody16KSteps; ++ks) {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        acc[n][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wA[ks][0], fb[n], acc[n][0], 0, 0, 0);
        acc[n][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wA[ks][1], fb[n], acc[n][1], 0, 0, 0);
        if (ks + 1 < kBody16KSteps) {
          __builtin_amdgcn_sched_barrier(0);
          fb[n] = ldB(ks + 1, n);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    {                                          // bias + activation -> fp16 -> 16 B per lane and N-tile
      const float* bl = bias_l + 32 * m + 8 * q;
      const int ncols = min(kTileW, s.W - tx0);
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int y = ty0 + 2 * rp + rr;
        half_t* row = out + (((size_t)b * s.Hp + y + s.pad) * s.Wp + tx0 + s.pad) * kWidth;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
#pragma unroll
        for (int nh = 0; nh < 2; ++nh) {
          const int n = 2 * rr + nh;
          half8_t o;
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r2 = 0; r2 < 4; r2 += 2) {
              f2v_t v = f2v_t{acc[n][i][r2], acc[n][i][r2 + 1]} + f2v_t{bl[4 * i + r2], bl[4 * i + r2 + 1]};
              if (ACT == 0) {
                const f2v_t tt = v * 0.01f;
                v = f2v_t{fmaxf(v.x, tt.x), fmaxf(v.y, tt.y)};
              } else {
                v = f2v_t{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f)};
              }
              o[4 * i + r2] = (half_t)v.x;
              o[4 * i + r2 + 1] = (half_t)v.y;
            }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, o), rs,
                                                 (16 * nh + col) * 128 + 64 * m + 16 * q, 0, 0);
        }
      }
    }
    // tile t+1 landed: only the DMA of t+2 (ndma ops) and this tile's 4 stores are younger
    if (ndma == 6) asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
}
template __global__ void conv_body_v4_kernel<0>(const half_t* __restrict__, half_t* __restrict__,
                                                const uint4* __restrict__, const float* __restrict__, ConvShape);
template __global__ void conv_body_v4_kernel<1>(const half_t* __restrict__, half_t* __restrict__,
                                                const uint4* __restrict__, const float* __restrict__, ConvShape);

// ------------------------------------------------------------------------------------
// Body layer as a row-wise Winograd F(2,3) (PNP_TUNE_BODY_VARIANT 4).  Along x, each pair of
// output pixels (2n, 2n+1) of a row is
//   y0 = M0 + M1 + M2,  y1 = M1 - M2 - M3,   M_j = sum_{a, ci} U[a][j] . d'_j(row + a)
// with the input transform d' = (d0 - d2, d1 + d2, d2 - d1, d1 - d3) of halo columns
// 2n .. 2n+3 and the weight transform U = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2) of each
// kernel row (pack_body_weights_wg, fp64 -> fp16).  12 MFMA taps per output pair instead of
// 18: two thirds of the MFMA work of conv_body_v3.  Same tile, 3-deep LDS-DMA ring and
// resident weights as conv_body_v4 (planar halo); wave w owns output channels 16(w&3) ..
// +15 (one 16x16x32 M-tile, all 12 (a, j) x 2 K-halves = 96 VGPRs) of tile rows
// 4(w>>2) .. +3, as 16 x 4 accumulators (one 16-pixel-pair N-tile per row and j).  Each
// halo row of its 6 is read once per K-half (4 x ds_read_b128 for d0..d3), transformed
// with 16 packed fp16 adds, and feeds the 1-3 output rows that use it.
// Planar halo with an ODD plane stride (341 pixels): lane group q = lane>>4 reads chunk
// 4ks+q of pixels 2n+c, so the two chunks of one ds_read_b128 lane group land on opposite
// bank-slot parities and the 16 lanes hit 16 distinct slots.
// Numerics: the fp16 rounding of d' and U replaces that of d and g; fp32 accumulation and
// output transform.  Not bit-identical to variants 0-3 (tested against the oracle within
// the fp16 tolerance).
// LDS: 3 x 44032 B halo + bias = 132352 B.
// Measured (B = 256): 1.37-1.40 ms vs 1.23-1.29 ms for conv_body_v3.  PMC at B = 64: 2/3 of
// v3's MFMA cycles but 2x its vector instructions (192 packed transform adds + the output
// transform per wave and tile), MFMA busy 27 vs 55 %, 45 % of wave cycles stalled on issue.
// A forced 1 MFMA : 2 VALU : 1/2 LDS interleave (sched_group_barrier) changed nothing.
// ------------------------------------------------------------------------------------
// a - b on 8 fp16 as 4 v_pk_add_f16 with the second operand negated (the compiler splits a
// vector fsub into per-half v_sub_f16 + repack: 3 instructions per pair instead of 1)
__device__ __forceinline__ half8_t pk_sub8(const half8_t& a, const half8_t& b) {
  const v4i_t ai = __builtin_bit_cast(v4i_t, a), bi = __builtin_bit_cast(v4i_t, b);
  v4i_t r;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    asm("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r[i]) : "v"(ai[i]), "v"(bi[i]));
  return __builtin_bit_cast(half8_t, r);
}

constexpr int kWgPlanePix = 341;                               // odd, >= 340
constexpr int kWgPlaneBytes = kWgPlanePix * 16;                // 5456
constexpr int kWgPieces = (8 * kWgPlanePix + 63) / 64;         // 43 DMA pieces of 64 x 16 B
constexpr int kWgHalo = kWgPieces * 1024;                      // 44032
constexpr int kWgBias = 3 * kWgHalo;
constexpr int kWgLds = kWgBias + 256;                          // 132352

template <int ACT>
__global__ __launch_bounds__(512, 2) void conv_body_wg_kernel(const half_t* __restrict__ in,
                                                               half_t* __restrict__ out,
                                                               const uint4* __restrict__ wpk,
                                                               const float* __restrict__ bias,
                                                               ConvShape s) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* bias_l = reinterpret_cast<float*>(smem + kWgBias);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mt = wave & 3, rq = wave >> 2;   // M-tile (16 channels), row quad
  const int q = lane >> 4, n = lane & 15;
  if (tid < kWidth) bias_l[tid] = bias[tid];

  half8_t wU[3][4][2];                        // [kernel row a][j][K-half], resident for the launch
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        wU[a][j][ks] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wpk) +
                                                         (((((a * 4 + j) * 2 + ks) * 4 + mt) * 64 + lane) * 16));

  // DMA: piece g (64 lanes x 16 B) of the planar image; wave w issues g = w, w + 8, ...
  constexpr int kSlotsPerWave = (kWgPieces + 7) / 8;            // 6 (waves >= 3: 5)
  const int ndma = (kWgPieces - wave + 7) / 8;
  unsigned doff[kSlotsPerWave];
#pragma unroll
  for (int j = 0; j < kSlotsPerWave; ++j) {
    const int k = 64 * (8 * j + wave) + lane;                   // 16-B unit of the planar image
    const int c = k / kWgPlanePix, p = min(k - c * kWgPlanePix, kHaloPix - 1);
    const int pr = p / kHaloW, pc = p - pr * kHaloW;
    doff[j] = (unsigned)(((pr * s.Wp + pc) * kWidth + 8 * min(c, 7)) * 2);
  }
  auto buf = [&](int i) { return smem + i * kWgHalo; };
  auto issue_dma = [&](int tt, int bi) {
    int b, ty0, tx0;
    decode_tile(tt < s.tiles ? tt : s.tiles - 1, s, b, ty0, tx0);
    const half_t* base = in + (((size_t)b * s.Hp + ty0 + s.pad - 1) * s.Wp + tx0 + s.pad - 1) * kWidth;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < kSlotsPerWave; ++j)
      if (j < ndma)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(buf(bi) + (8 * j + wave) * 1024),
                                                 16, doff[j], 0, 0, 0);
  };

  int t = blockIdx.x;
  if (t < s.tiles) {
    issue_dma(t, 0);
    issue_dma(t + gridDim.x, 1);
    if (ndma == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // tile t landed
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  }
  __syncthreads();
  const int lane_off = q * kWgPlaneBytes + 2 * n * 16 + 4 * rq * kHaloW * 16;
  int cur = 0;
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const int nxt2 = cur >= 1 ? cur - 1 : 2;  // (cur + 2) % 3
    issue_dma(t + 2 * gridDim.x, nxt2);
    const unsigned char* hl = buf(cur) + lane_off;
    auto ldD = [&](int ks, int R, int c) {    // everything but lane_off is an immediate
      return *reinterpret_cast<const half8_t*>(hl + 4 * ks * kWgPlaneBytes + (R * kHaloW + c) * 16);
    };
    floatx4 acc[4][4];                        // [output row][j]
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[r][j] = floatx4{};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int R = 0; R < 6; ++R) {
        const half8_t d0 = ldD(ks, R, 0), d1 = ldD(ks, R, 1), d2 = ldD(ks, R, 2), d3 = ldD(ks, R, 3);
        half8_t B[4];
        B[0] = pk_sub8(d0, d2);
        B[1] = d1 + d2;
        B[2] = pk_sub8(d2, d1);
        B[3] = pk_sub8(d1, d3);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int a = R - r;
          if (a < 0 || a > 2) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wU[a][j][ks], B[j], acc[r][j], 0, 0, 0);
        }
      }
    {                                          // output transform + bias + activation -> 8 B per lane and pixel
      const float* bl = bias_l + 16 * mt + 4 * q;
      const float bv[4] = {bl[0], bl[1], bl[2], bl[3]};
      const int ncols = min(kTileW, s.W - tx0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int y = ty0 + 4 * rq + r;
        half_t* row = out + (((size_t)b * s.Hp + y + s.pad) * s.Wp + tx0 + s.pad) * kWidth;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          half4_t o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float z = v == 0 ? (acc[r][0][i] + acc[r][1][i]) + acc[r][2][i]
                             : (acc[r][1][i] - acc[r][2][i]) - acc[r][3][i];
            z += bv[i];
            z = ACT == 0 ? fmaxf(z, 0.01f * z) : fmaxf(z, 0.f);
            o[i] = (half_t)z;
          }
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i_t, o), rs,
                                                (2 * n + v) * 128 + (16 * mt + 4 * q) * 2, 0, 0);
        }
      }
    }
    // tile t+1 landed: only the DMA of t+2 (ndma ops) and this tile's 8 stores are younger
    if (ndma == 6) asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(13) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
}
template __global__ void conv_body_wg_kernel<0>(const half_t* __restrict__, half_t* __restrict__,
                                                const uint4* __restrict__, const float* __restrict__, ConvShape);
template __global__ void conv_body_wg_kernel<1>(const half_t* __restrict__, half_t* __restrict__,
                                                const uint4* __restrict__, const float* __restrict__, ConvShape);


// ------------------------------------------------------------------------------------
// Two body layers per launch (l+1 and l+2 of basic_models.py:29-33): the intermediate
// activation never leaves LDS, so each pair of layers reads and writes the fp16 image
// once (half the HBM traffic of two one-layer launches) for 25 % more MFMA work.
//
// Tile: 8 x 16 output pixels.  Stage 1 computes layer l+1 on the 10 x 18 region around
// the tile (180 pixels = 6 N-tiles of 32, zero outside the image = layer l+2's padding)
// from the 12 x 20 input halo; stage 2 computes layer l+2 on the 8 x 16 tile (4 N-tiles
// of 2 rows x 16) from that intermediate.
//
// 8 waves, 2 per SIMD.  Waves 0-3 run stage 1 and hold layer l+1's weights for M-tile
// m = w&1 (144 VGPRs); waves 4-7 run stage 2 with layer l+2's weights: every SIMD carries
// one wave of each stage.  The stages are software-pipelined over the CU's tiles: in step
// k stage 1 builds tile k's intermediate while stage 2 finishes tile k-1 from the other
// intermediate buffer, and stage-1 waves stream the 12 x 20 halo of tile k+2 into a 3-deep
// LDS-DMA ring (8 uniform 1-KiB slots per wave).  One workgroup barrier per step.
// Stage-2 outputs go through wave-private staging and are stored during the next step.
// LDS: 3 x 32 KiB input ring + 2 x 22.5 KiB intermediate + 4 x 4 KiB staging + bias.
// ------------------------------------------------------------------------------------
constexpr int kB2TH = 8, kB2TW = 16;                        // output tile
constexpr int kB2IW = kB2TW + 4, kB2IH = kB2TH + 4;         // input halo 12 x 20
constexpr int kB2MW = kB2TW + 2, kB2MH = kB2TH + 2;         // intermediate 10 x 18
constexpr int kB2InPix = kB2IW * kB2IH;                     // 240
constexpr int kB2MidPix = kB2MW * kB2MH;                    // 180
constexpr int kB2InBytes = 32 * 1024;                       // 32 uniform DMA slots (30 used)
constexpr int kB2MidBytes = kB2MidPix * 128;                // 23040
constexpr int kB2Mid = 3 * kB2InBytes;
constexpr int kB2Stage = kB2Mid + 2 * kB2MidBytes;
constexpr int kB2Bias = kB2Stage + 4 * 4096;
constexpr int kB2Lds = kB2Bias + 2 * 64 * 4;                // 161280 B

// XOR-swizzled pixel-major LDS image of width `w` (as halo_off, common.h)
__device__ __forceinline__ int img_off(int pr, int pc, int w, int chunk) {
  return (pr * w + pc) * 128 + 16 * (chunk ^ ((pc >> 1) & 7));
}

__device__ __forceinline__ void decode_tile2(int t, const ConvShape& s, int& b, int& ty0, int& tx0) {
  const int tx = (s.W + kB2TW - 1) / kB2TW, ty = (s.H + kB2TH - 1) / kB2TH;
  const int per_img = tx * ty;
  b = t / per_img;
  const int r = t - b * per_img;
  const int yy = r / tx;
  ty0 = yy * kB2TH;
  tx0 = (r - yy * tx) * kB2TW;
}

// Stage-1 waves' share of the 12 x 20 input-halo DMA of a fused tile: 8 uniform slots each
// (slot g = wave + 4j; slots 30, 31 re-read pixel 239 into padding).  The per-lane offsets
// are recomputed at each issue (a few VALU per slot) rather than held in 8 VGPRs; the
// opaque copy of the lane id keeps the compiler from hoisting (and spilling) them.
__device__ __forceinline__ void b2_halo_dma(unsigned char* hl, const half_t* __restrict__ in, const ConvShape& s,
                                            int t, int wave, int lane) {
  int b, ty0, tx0;
  decode_tile2(t, s, b, ty0, tx0);
  // input halo origin: image (ty0 - 2, tx0 - 2) = padded (ty0 + pad - 2, tx0 + pad - 2)
  const half_t* base = in + (((size_t)b * s.Hp + ty0 + s.pad - 2) * s.Wp + tx0 + s.pad - 2) * kWidth;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
  int ln = lane;
  asm volatile("" : "+v"(ln));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int p = 8 * (4 * j + (wave & 3)) + (ln >> 3);
    const int pl = min(p, kB2InPix - 1);
    const int pr = pl / kB2IW, pc = pl - pr * kB2IW;
    const int c = (ln & 7) ^ ((pc >> 1) & 7);
    const unsigned off = (unsigned)(((pr * s.Wp + pc) * kWidth + c * 8) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(hl + (4 * j + (wave & 3)) * 1024), 16, off, 0, 0, 0);
  }
}

template <int ACT>
__global__ __launch_bounds__(512, 2) void conv_body2_kernel(const half_t* __restrict__ in,
                                                             half_t* __restrict__ out,
                                                             const uint4* __restrict__ w1,
                                                             const float* __restrict__ b1,
                                                             const uint4* __restrict__ w2,
                                                             const float* __restrict__ b2,
                                                             ConvShape s, int tiles) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* bias_l = reinterpret_cast<float*>(smem + kB2Bias);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool st1 = wave < 4;
  const int m = wave & 1, part = (wave >> 1) & 1;
  const int h = lane >> 5, col = lane & 31;
  if (tid < kWidth) bias_l[tid] = b1[tid];
  else if (tid < 2 * kWidth) bias_l[tid] = b2[tid - kWidth];

  half8_t wA[kBodyKSteps];                    // this wave's layer's weights, M-tile m
  {
    const unsigned char* wsrc = reinterpret_cast<const unsigned char*>(st1 ? w1 : w2);
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks)
      wA[ks] = *reinterpret_cast<const half8_t*>(wsrc + ((ks * 2 + m) * 64 + lane) * 16);
  }
  auto inbuf = [&](int i) { return smem + i * kB2InBytes; };
  auto midbuf = [&](int i) { return smem + kB2Mid + i * kB2MidBytes; };

  auto issue_dma = [&](int tt, int bi) {      // stage-1 waves only; clamped tile: fixed op count
    b2_halo_dma(inbuf(bi), in, s, tt < tiles ? tt : tiles - 1, wave, lane);
  };

  const int t0 = blockIdx.x;
  const int nt = t0 < tiles ? (tiles - 1 - t0) / (int)gridDim.x + 1 : 0;   // tiles of this workgroup
  if (st1 && nt > 0) {
    issue_dma(t0, 0);
    issue_dma(t0 + gridDim.x, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                          // tile 0's halo landed
  }
  __syncthreads();

  // stage-2 deferred stores (previous step's tile): 16 pixels x 64 B (channel half m) each
  unsigned char* stg = smem + kB2Stage + (wave & 3) * 4096;
  __amdgpu_buffer_rsrc_t rs[4];
  rs[0] = rs[1] = rs[2] = rs[3] = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000);
  auto stage_read = [&](int j) {              // j = output row (of this wave's 4) ; 16 px x 4 chunks
    const int pix = 16 * j + (lane >> 2), c = lane & 3;
    return *reinterpret_cast<const v4i_t*>(stg + pix * 64 + 16 * (c ^ ((pix >> 1) & 3)));
  };
  auto stage_store = [&](int j, const v4i_t& v) {
    const int pix = 16 * j + (lane >> 2), c = lane & 3;
    __builtin_amdgcn_raw_buffer_store_b128(v, rs[j], (pix & 15) * 128 + 64 * m + 16 * c, 0, 0);
  };

  for (int k = 0; k <= nt; ++k) {
    if (st1) {
      if (k < nt) {
        // ---------------- stage 1: layer l+1 on the 10 x 18 region of tile k ----------------
        int b, ty0, tx0;
        decode_tile2(t0 + k * gridDim.x, s, b, ty0, tx0);
        issue_dma(t0 + (k + 2) * gridDim.x, (k + 2) % 3);
        const unsigned char* hl = inbuf(k % 3);
        unsigned char* mid = midbuf(k & 1);
        const float* bl = bias_l + 32 * m + 16 * h;
#pragma unroll 1
        for (int i = 0; i < 3; ++i) {
          const int n = 32 * (part + 2 * i) + col;           // intermediate pixel (flattened 10 x 18)
          const int nc = min(n, kB2MidPix - 1);
          const int r1 = nc / kB2MW, c1 = nc - r1 * kB2MW;
          auto ldB = [&](int ks) {
            const int tap = ks >> 2, sub = ks & 3;
            return *reinterpret_cast<const half8_t*>(
                hl + img_off(r1 + tap / 3, c1 + tap % 3, kB2IW, 2 * sub + h));
          };
          floatx16 acc = {};
          half8_t fb[4];
          fb[0] = ldB(0); fb[1] = ldB(1); fb[2] = ldB(2);
#pragma unroll
          for (int ks = 0; ks < kBodyKSteps; ++ks) {
            if (ks + 3 < kBodyKSteps) fb[(ks + 3) & 3] = ldB(ks + 3);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[ks & 3], acc, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);               // keep the reads 3 steps ahead
          }
          // bias + act -> fp16 -> intermediate; zero outside the image (layer l+2's padding)
          const int y = ty0 - 1 + r1, x = tx0 - 1 + c1;
          const bool inside = y >= 0 && y < s.H && x >= 0 && x < s.W;
          const half8_t z = {};
          const half8_t lo = inside ? bias_act8<ACT>(acc, 0, bl) : z;
          const half8_t hi = inside ? bias_act8<ACT>(acc, 8, bl + 8) : z;
          if (n < kB2MidPix) {
            const int q = 4 * m + 2 * h;
            *reinterpret_cast<half8_t*>(mid + img_off(r1, c1, kB2MW, q)) = lo;
            *reinterpret_cast<half8_t*>(mid + img_off(r1, c1, kB2MW, q + 1)) = hi;
          }
        }
      }
      // halo of tile k+1 landed: only the 8 DMA ops of tile k+2 are younger
      asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    } else {
      if (k >= 1) {
        // ---------------- stage 2: layer l+2 on tile k-1 ----------------
        int b, ty0, tx0;
        decode_tile2(t0 + (k - 1) * gridDim.x, s, b, ty0, tx0);
        const unsigned char* mid = midbuf((k - 1) & 1);
        const int orow = 4 * part + 2 * 0;          // this wave's output rows 4part .. 4part+3
        auto ldB = [&](int ks, int nn) {            // N-tile nn (0,1): rows orow + 2nn + col/16
          const int tap = ks >> 2, sub = ks & 3;
          const int rr = orow + 2 * nn + (col >> 4), cc = col & 15;
          return *reinterpret_cast<const half8_t*>(
              mid + img_off(rr + tap / 3, cc + tap % 3, kB2MW, 2 * sub + h));
        };
        floatx16 acc0 = {}, acc1 = {};
        half8_t fb[3][2];
        v4i_t sv;
        fb[0][0] = ldB(0, 0); fb[0][1] = ldB(0, 1);
        fb[1][0] = ldB(1, 0); fb[1][1] = ldB(1, 1);
#pragma unroll
        for (int ks = 0; ks < kBodyKSteps; ++ks) {
          if ((ks & 7) == 1 && ks < 32) {           // previous step's stores, one per 8 K-steps
            __builtin_amdgcn_sched_barrier(0);
            sv = stage_read(ks >> 3);
            __builtin_amdgcn_sched_barrier(0);
          }
          if (ks + 2 < kBodyKSteps) { fb[(ks + 2) % 3][0] = ldB(ks + 2, 0); fb[(ks + 2) % 3][1] = ldB(ks + 2, 1); }
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[ks % 3][0], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[ks % 3][1], acc1, 0, 0, 0);
          if ((ks & 7) == 4 && ks < 32) {
            __builtin_amdgcn_sched_barrier(0);
            stage_store(ks >> 3, sv);
            __builtin_amdgcn_sched_barrier(0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        // bias + act -> fp16 -> wave-private staging [64 px][64 B], px = 16 * row + col
        const float* bl = bias_l + kWidth + 32 * m + 16 * h;
#pragma unroll
        for (int nn = 0; nn < 2; ++nn) {
          const floatx16& a = nn == 0 ? acc0 : acc1;
          const int pix = 32 * nn + col;            // rows 2nn + col/16 of this wave, col%16
          const int sw = (pix >> 1) & 3;
          *reinterpret_cast<half8_t*>(stg + pix * 64 + 16 * ((2 * h) ^ sw)) = bias_act8<ACT>(a, 0, bl);
          *reinterpret_cast<half8_t*>(stg + pix * 64 + 16 * ((2 * h + 1) ^ sw)) = bias_act8<ACT>(a, 8, bl + 8);
        }
        const int ncols = min(kB2TW, s.W - tx0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int y = ty0 + orow + j;
          half_t* row = out + (((size_t)b * s.Hp + y + s.pad) * s.Wp + tx0 + s.pad) * kWidth;
          rs[j] = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }
  if (!st1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) stage_store(j, stage_read(j));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
}

// ------------------------------------------------------------------------------------
// Head layer C -> 64 (basic_models.py:16,27-28).  Input: padded NHWC4 fp16 (8 B/pixel).
// K = 9 taps x 4 channels = 36, padded to 48 = 3 K-steps of 16: k = 4*tap + ch.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_head_kernel(const half_t* __restrict__ in4,
                                                         half_t* __restrict__ out,
                                                         const uint4* __restrict__ wpk,
                                                         const float* __restrict__ bias,
                                                         ConvShape s, int act) {
  __shared__ __attribute__((aligned(16))) unsigned char wl[kHeadWBytes];
  __shared__ __attribute__((aligned(16))) uint2 hl[kHaloPix];
  __shared__ __attribute__((aligned(16))) unsigned char stg_all[4 * 8192];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  unsigned char* stg = stg_all + wave * 8192;
  const int h = lane >> 5, col = lane & 31;
  for (int i = tid; i < kHeadWBytes / 16; i += 256) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
  float bias_r[2][16];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) bias_r[m][r] = bias[32 * m + 16 * h + r];

  // the next tile's halo is loaded into registers while this tile computes (2 pixels per thread)
  const int Wp4 = s.W + 2;                    // u16: NHWC4 with a one-pixel zero border
  uint2 pre[2];
  auto load_halo = [&](int tt) {
    int pb_, pty, ptx;
    decode_tile(tt < s.tiles ? tt : s.tiles - 1, s, pb_, pty, ptx);
    const uint2* base = reinterpret_cast<const uint2*>(in4) + ((size_t)pb_ * (s.H + 2) + pty) * Wp4 + ptx;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = tid + 256 * k;
      const int pl = p < kHaloPix ? p : kHaloPix - 1;
      const int pr = pl / kHaloW, pc = pl - pr * kHaloW;
      pre[k] = base[(size_t)pr * Wp4 + pc];
    }
  };
  if (blockIdx.x < s.tiles) load_halo(blockIdx.x);
  for (int t = blockIdx.x; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (tid + 256 * k < kHaloPix) hl[tid + 256 * k] = pre[k];
    __syncthreads();
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
        if (n == 0) {
          acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bf, acc00, 0, 0, 0);
          acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, bf, acc10, 0, 0, 0);
        } else {
          acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bf, acc01, 0, 0, 0);
          acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, bf, acc11, 0, 0, 0);
        }
      }
    }
    // epilogue through wave-private LDS staging: 2 rows x 32 pixels x 128 B, 16-B chunks
    // XOR-swizzled by pixel (conflict-free writes), stored back as full 128-B pixel lines
    // (1 KiB contiguous per instruction) instead of 16-B pieces at a 128-B stride.
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const floatx16& a0 = n == 0 ? acc00 : acc01;
      const floatx16& a1 = n == 0 ? acc10 : acc11;
      unsigned char* px = stg + (n * 32 + col) * 128;
      const int sw = col & 7;
      half8_t v[4];
      if (act == 0) {                         // packed bias + activation (bit-identical to act_fn)
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
#pragma unroll
    for (int j = 0; j < 8; ++j) {             // 8 pixels x 8 chunks per instruction
      const int n = j >> 2, p = 8 * (j & 3) + (lane >> 3), c = lane & 7;
      const uint4 q = *reinterpret_cast<const uint4*>(stg + (n * 32 + p) * 128 + 16 * (c ^ (p & 7)));
      const int y = ty0 + 2 * wave + n, x = tx0 + p;
      if (y < s.H && x < s.W)
        *reinterpret_cast<uint4*>(out + (((size_t)b * s.Hp + y + s.pad) * s.Wp + x + s.pad) * kWidth + 8 * c) = q;
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

__global__ __launch_bounds__(256, 1) void conv_tail_kernel(const half_t* __restrict__ in,
                                                            const float* __restrict__ xin,
                                                            float* __restrict__ xout,
                                                            const uint4* __restrict__ wpk,
                                                            const float* __restrict__ bias,
                                                            ConvShape s, int C, int residual_sign,
                                                            int clamp_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q4 = lane >> 4, c16 = lane & 15;
  half8_t wA[kTailKSteps];
#pragma unroll
  for (int ks = 0; ks < kTailKSteps; ++ks)
    wA[ks] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wpk) + (ks * 64 + lane) * 16);
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

  int t = blockIdx.x;
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
    issue_dma(t + 2 * gridDim.x, nxt2);
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
                                            off, 0, 0);
    }
    // tile t+1 landed: younger than its DMA are this tile's 4 loads, DMA of t+2 and 4 stores
    asm volatile("s_waitcnt vmcnt(19) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
}

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

// conv_body_v4 (16x16x32): [ks 18][m 2][i 2][lane 64][8 x f16]; k-step ks = tap ks/2, input
// channels 32(ks&1) + 8(l>>4) + j; A row R = l&15 of M-tile i = channel 32m + 8(R>>2) + 4i + (R&3).
void pack_body_weights16(const float* W, uint16_t* out) {
  for (int ks = 0; ks < kBody16KSteps; ++ks) {
    const int tap = ks / 2, sub = ks % 2, ky = tap / 3, kx = tap % 3;
    for (int m = 0; m < 2; ++m)
      for (int i = 0; i < 2; ++i)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int R = l & 15;
            const int co = 32 * m + 8 * (R >> 2) + 4 * i + (R & 3);
            const int ci = 32 * sub + 8 * (l >> 4) + j;
            out[((((ks * 2 + m) * 2 + i) * 64 + l) * 8) + j] = f32_to_f16_bits(W[((co * 64 + ci) * 3 + ky) * 3 + kx]);
          }
  }
}

// conv_body_wg order: [kernel row a][j][K-half ks][M-tile mt][lane][8 x f16], lane l holding
// U_j[a] of output channel 16mt + (l&15), input channels 32ks + 8(l>>4) .. +7, where
// U = (g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2) of kernel row a (transformed in fp64, rounded once).
void pack_body_weights_wg(const float* W, uint16_t* out) {
  for (int a = 0; a < 3; ++a)
    for (int j = 0; j < 4; ++j)
      for (int ks = 0; ks < 2; ++ks)
        for (int mt = 0; mt < 4; ++mt)
          for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) {
              const int co = 16 * mt + (l & 15), ci = 32 * ks + 8 * (l >> 4) + e;
              const float* g = W + ((co * 64 + ci) * 3 + a) * 3;
              const double g0 = g[0], g1 = g[1], g2 = g[2];
              const double u = j == 0 ? g0 : j == 1 ? 0.5 * (g0 + g1 + g2) : j == 2 ? 0.5 * (g0 - g1 + g2) : g2;
              out[((((a * 4 + j) * 2 + ks) * 4 + mt) * 64 + l) * 8 + e] = f32_to_f16_bits((float)u);
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
  for (const void* k : {(const void*)conv_body_v3_kernel<0, 0>, (const void*)conv_body_v3_kernel<0, 1>,
                        (const void*)conv_body_v3_kernel<8, 0>, (const void*)conv_body_v3_kernel<8, 1>,
                        (const void*)conv_body_v3_kernel<16, 0>, (const void*)conv_body_v3_kernel<24, 0>,
                        (const void*)conv_body_v3_kernel<1, 0>, (const void*)conv_body_v3_kernel<2, 0>,
                        (const void*)conv_body_v3_kernel<3, 0>, (const void*)conv_body_v3_kernel<4, 0>,
                        (const void*)conv_body_v3_kernel<6, 0>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kV3Lds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_body_v4_kernel<0>, (const void*)conv_body_v4_kernel<1>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kV5Lds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_body_wg_kernel<0>, (const void*)conv_body_wg_kernel<1>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kWgLds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_body2_kernel<0>, (const void*)conv_body2_kernel<1>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kB2Lds);
    if (e != hipSuccess) return e;
  }
  return hipFuncSetAttribute((const void*)conv_tail_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kTailLds);
}

void launch_conv_head(const half_t* in4, half_t* out, const void* w, const float* bias, const ConvShape& s,
                      int act, int num_cus, int blocks_per_cu, hipStream_t st) {
  const int grid = s.tiles < num_cus * blocks_per_cu ? s.tiles : num_cus * blocks_per_cu;
  hipLaunchKernelGGL(conv_head_kernel, dim3(grid), dim3(256), 0, st, in4, out, (const uint4*)w, bias, s, act);
}

void launch_conv_body(const half_t* in, half_t* out, const void* w, const float* bias, const ConvShape& s,
                      int act, int num_cus, int ablate, hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
#define V3(A, F) hipLaunchKernelGGL((conv_body_v3_kernel<A, F>), dim3(grid), dim3(512), kV3Lds, st, in, out, \
                                    (const uint4*)w, bias, s)
  if (ablate == 8) {                          // staggered epilogue (PNP_TUNE_BODY_VARIANT 2)
    if (act != 0) V3(8, 1);
    else V3(8, 0);
    return;
  }
  if (act != 0) {
    V3(0, 1);
    return;
  }
  switch (ablate) {
    case 16: V3(16, 0); break;
    case 24: V3(24, 0); break;
    case 1: V3(1, 0); break;
    case 2: V3(2, 0); break;
    case 3: V3(3, 0); break;
    case 4: V3(4, 0); break;
    case 6: V3(6, 0); break;
    default: V3(0, 0);
  }
#undef V3
}

void launch_conv_body16(const half_t* in, half_t* out, const void* w16, const float* bias, const ConvShape& s,
                        int act, int num_cus, hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  if (act == 0)
    hipLaunchKernelGGL((conv_body_v4_kernel<0>), dim3(grid), dim3(512), kV5Lds, st, in, out, (const uint4*)w16, bias, s);
  else
    hipLaunchKernelGGL((conv_body_v4_kernel<1>), dim3(grid), dim3(512), kV5Lds, st, in, out, (const uint4*)w16, bias, s);
}

void launch_conv_body_wg(const half_t* in, half_t* out, const void* wwg, const float* bias, const ConvShape& s,
                         int act, int num_cus, hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  if (act == 0)
    hipLaunchKernelGGL((conv_body_wg_kernel<0>), dim3(grid), dim3(512), kWgLds, st, in, out, (const uint4*)wwg, bias, s);
  else
    hipLaunchKernelGGL((conv_body_wg_kernel<1>), dim3(grid), dim3(512), kWgLds, st, in, out, (const uint4*)wwg, bias, s);
}

void launch_conv_body2(const half_t* in, half_t* out, const void* w1, const float* b1, const void* w2,
                       const float* b2, const ConvShape& s, int act, int num_cus, hipStream_t st) {
  const int tiles = s.B * ((s.W + kB2TW - 1) / kB2TW) * ((s.H + kB2TH - 1) / kB2TH);
  const int grid = tiles < num_cus ? tiles : num_cus;
  if (act == 0)
    hipLaunchKernelGGL((conv_body2_kernel<0>), dim3(grid), dim3(512), kB2Lds, st, in, out, (const uint4*)w1, b1,
                       (const uint4*)w2, b2, s, tiles);
  else
    hipLaunchKernelGGL((conv_body2_kernel<1>), dim3(grid), dim3(512), kB2Lds, st, in, out, (const uint4*)w1, b1,
                       (const uint4*)w2, b2, s, tiles);
}

void launch_conv_tail(const half_t* in, const float* xin, float* xout, const void* w, const float* bias,
                      const ConvShape& s, int C, int residual_sign, int clamp_out, int num_cus,
                      hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  hipLaunchKernelGGL(conv_tail_kernel, dim3(grid), dim3(256), kTailLds, st, in, xin, xout,
                     (const uint4*)w, bias, s, C, residual_sign, clamp_out);
}

}  // namespace pnp
