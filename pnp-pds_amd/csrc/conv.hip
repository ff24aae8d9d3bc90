// Denoiser forward on MFMA: implicit-GEMM 3x3 convolutions for gfx950.
//
// Reference: models/basic_models.py:25-38 (simple_CNN.forward: in_conv + LeakyReLU,
// 18 x [conv + LeakyReLU], out_conv + x_in) and models/denoiser.py:34-46 (clamp in/out);
// KAIR variant models/network_dncnn.py:42-77 (ReLU, x - n, no clamps).
//
// GEMM view per layer: D[cout][pixel] = sum_k W[cout][k] * X[k][pixel],
// k = (tap, cin).  A operand = packed weights (host-packed in MFMA fragment order,
// staged once per workgroup into LDS), B operand = activations read from an LDS
// halo tile.  fp16 operands, fp32 accumulation (v_mfma_f32_32x32x16_f16 for the
// 64-channel layers, v_mfma_f32_16x16x32_f16 for the 64->C tail).
//
// Workgroup = 4 waves, persistent over 8x32-pixel output tiles; wave w owns output
// rows 2w, 2w+1 (two 32-pixel N-tiles) x all 64 output channels (two 32-row M-tiles)
// = 4 accumulators of 32x32.  Per K-step: 2 weight + 2 activation ds_read_b128 and
// 4 MFMAs.
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

// The 10 x 34 x 64-channel halo tile (padded coords [ty0, ty0+10) x [tx0, tx0+34)) is
// 2720 16-byte chunks: 11 per thread.  Consecutive threads read consecutive 16 B of a
// pixel row (coalesced); 8 lanes write one 128-B pixel of the swizzled LDS image.
constexpr int kHaloChunks = kHaloPix * 8;
constexpr int kHaloPerThread = (kHaloChunks + 255) / 256;

// Issue the global loads of a halo tile into registers (no wait: T14 issue-early).
// Every lane loads unconditionally (surplus lanes re-read the last pixel): a guarded load
// makes hipcc merge the destination through a branch and wait vmcnt right after issue.
__device__ __forceinline__ void halo_load(uint4 (&v)[kHaloPerThread], const half_t* __restrict__ in,
                                          const ConvShape& s, int b, int ty0, int tx0) {
  const half_t* base = in + (((size_t)b * s.Hp + ty0) * s.Wp + tx0) * kWidth;
#pragma unroll
  for (int k = 0; k < kHaloPerThread; ++k) {
    const int q = threadIdx.x + 256 * k;
    const int p = min(q >> 3, kHaloPix - 1), c = q & 7;
    const int pr = p / kHaloW, pc = p - pr * kHaloW;
    v[k] = *reinterpret_cast<const uint4*>(base + ((size_t)pr * s.Wp + pc) * kWidth + c * 8);
  }
}

// Write a loaded halo tile into an LDS image (write-late).
__device__ __forceinline__ void halo_store(unsigned char* hl, const uint4 (&v)[kHaloPerThread]) {
#pragma unroll
  for (int k = 0; k < kHaloPerThread; ++k) {
    const int q = threadIdx.x + 256 * k;
    if (q < kHaloChunks) *reinterpret_cast<uint4*>(hl + halo_chunk_offset(q >> 3, q & 7)) = v[k];
  }
}

__device__ __forceinline__ void stage_halo64(unsigned char* hl, const half_t* __restrict__ in,
                                             const ConvShape& s, int b, int ty0, int tx0) {
  uint4 v[kHaloPerThread];
  halo_load(v, in, s, b, ty0, tx0);
  halo_store(hl, v);
}

// LDS-DMA (global_load_lds_dwordx4) staging of a halo tile: no register destination, so
// the loads stay in flight across the MFMA loop.  One wave-instruction writes 1 KiB of
// LDS = 8 pixels: slot g (g = 4j + wave, 43 slots) covers pixels 8g .. 8g+7.  The LDS
// destination is lane-linear, so the XOR swizzle is applied to the per-lane SOURCE
// address (lane l loads logical chunk (l&7) ^ swz(p) of pixel p into slot l&7).  Slots
// past pixel 339 re-read pixel 339 into the 4-pixel pad (never read back).
constexpr int kDmaSlots = (kHaloPix + 7) / 8;                 // 43
constexpr int kHaloDmaBytes = kDmaSlots * 1024;               // 44032
__device__ __forceinline__ void halo_dma(unsigned char* hl, const half_t* __restrict__ in, const ConvShape& s,
                                         int b, int ty0, int tx0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const half_t* base = in + (((size_t)b * s.Hp + ty0) * s.Wp + tx0) * kWidth;
#pragma unroll
  for (int j = 0; j < (kDmaSlots + 3) / 4; ++j) {
    const int g = 4 * j + wave;
    if (g < kDmaSlots) {
      const int p = 8 * g + (lane >> 3);
      const int c = (lane & 7) ^ ((p >> 1) & 7);
      const int pl = min(p, kHaloPix - 1);
      const int pr = pl / kHaloW, pc = pl - pr * kHaloW;
      const half_t* src = base + ((size_t)pr * s.Wp + pc) * kWidth + c * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(hl + g * 1024), 16, 0, 0);
    }
  }
}

// Epilogue shared by head and body: bias + activation, fp16, two 16-B stores per
// (M-tile) into the padded NHWC64 output.  Lane (col, h) owns channels 32m+16h .. +15.
__device__ __forceinline__ void store_act64(half_t* __restrict__ out, const ConvShape& s, int b, int y,
                                            int x, int h, const floatx16& acc0, const floatx16& acc1,
                                            const float (&bias)[2][16], int act) {
  if (y >= s.H || x >= s.W) return;
  half_t* o = out + (((size_t)b * s.Hp + y + 1) * s.Wp + x + 1) * kWidth + 16 * h;
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

// ------------------------------------------------------------------------------------
// Body layer 64 -> 64 (basic_models.py:16-17,29-33).  LDS: 72 KiB weights + two 42.5 KiB
// halo buffers = 157 KiB -> one workgroup (4 waves) per CU, persistent over tiles.
// Software pipeline per tile: issue the global loads of tile t+1 into registers, run
// tile t's 144 MFMAs/wave from LDS buffer `cur`, store tile t, then write tile t+1 into
// buffer `cur^1`; one barrier per tile.
// ------------------------------------------------------------------------------------
constexpr int kHaloBytes = kHaloPix * 128;

__global__ __launch_bounds__(256, 1) void conv_body_kernel(const half_t* __restrict__ in,
                                                            half_t* __restrict__ out,
                                                            const uint4* __restrict__ wpk,
                                                            const float* __restrict__ bias,
                                                            ConvShape s, int act) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* wl = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, col = lane & 31;

  for (int i = tid; i < kBodyWBytes / 16; i += 256) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
  float bias_r[2][16];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) bias_r[m][r] = bias[32 * m + 16 * h + r];

  int t = blockIdx.x;
  int cur = 0;
  if (t < s.tiles) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    halo_dma(smem + kBodyWBytes, in, s, b, ty0, tx0);
  }
  __syncthreads();                            // drains the DMA (vmcnt(0)) + barrier
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const int tn = t + gridDim.x;
    if (tn < s.tiles) {                       // next tile -> the other buffer, in flight
      int bn, tyn, txn;
      decode_tile(tn, s, bn, tyn, txn);
      halo_dma(smem + kBodyWBytes + (cur ^ 1) * kHaloDmaBytes, in, s, bn, tyn, txn);
    }
    const unsigned char* hl = smem + kBodyWBytes + cur * kHaloDmaBytes;
    const int pw = 2 * wave * kHaloW + col;   // this lane's pixel at tap (0,0), N-tile 0
    auto ldA = [&](int ks, int m) {
      return *reinterpret_cast<const half8_t*>(wl + ((ks * 2 + m) * 64 + lane) * 16);
    };
    auto ldB = [&](int ks, int n) {
      const int tap = ks >> 2, sub = ks & 3;
      const int p = pw + (n + tap / 3) * kHaloW + tap % 3;
      return *reinterpret_cast<const half8_t*>(hl + halo_chunk_offset(p, 2 * sub + h));
    };

    // K loop with the fragments of step ks+1 read from LDS while step ks's MFMAs run.
    floatx16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
    half8_t a0 = ldA(0, 0), a1 = ldA(0, 1), b0 = ldB(0, 0), b1 = ldB(0, 1);
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks) {
      half8_t na0, na1, nb0, nb1;
      if (ks + 1 < kBodyKSteps) {
        na0 = ldA(ks + 1, 0); na1 = ldA(ks + 1, 1);
        nb0 = ldB(ks + 1, 0); nb1 = ldB(ks + 1, 1);
      }
      acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc00, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc10, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc01, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, acc11, 0, 0, 0);
      if (ks + 1 < kBodyKSteps) { a0 = na0; a1 = na1; b0 = nb0; b1 = nb1; }
    }
    store_act64(out, s, b, ty0 + 2 * wave, tx0 + col, h, acc00, acc10, bias_r, act);
    store_act64(out, s, b, ty0 + 2 * wave + 1, tx0 + col, h, acc01, acc11, bias_r, act);
    __syncthreads();                          // next tile landed (vmcnt(0)); buffer cur free
    cur ^= 1;
  }
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
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, col = lane & 31;
  for (int i = tid; i < kHeadWBytes / 16; i += 256) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
  float bias_r[2][16];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) bias_r[m][r] = bias[32 * m + 16 * h + r];

  for (int t = blockIdx.x; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    __syncthreads();
    const uint2* base = reinterpret_cast<const uint2*>(in4) + ((size_t)b * s.Hp + ty0) * s.Wp + tx0;
    for (int p = tid; p < kHaloPix; p += 256) {
      const int pr = p / kHaloW, pc = p - pr * kHaloW;
      hl[p] = base[(size_t)pr * s.Wp + pc];
    }
    __syncthreads();
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
    store_act64(out, s, b, ty0 + 2 * wave, tx0 + col, h, acc00, acc10, bias_r, act);
    store_act64(out, s, b, ty0 + 2 * wave + 1, tx0 + col, h, acc01, acc11, bias_r, act);
  }
}

// ------------------------------------------------------------------------------------
// Tail layer 64 -> C (basic_models.py:18,35-36) + residual + clamp (denoiser.py:42),
// writing the new primal iterate x+ in fp32 NCHW.  v_mfma_f32_16x16x32_f16 with the C
// output channels as the (padded-to-16) A rows; each wave covers 4 N-tiles of 16 px.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_tail_kernel(const half_t* __restrict__ in,
                                                         const float* __restrict__ xin,
                                                         float* __restrict__ xout,
                                                         const uint4* __restrict__ wpk,
                                                         const float* __restrict__ bias,
                                                         ConvShape s, int C, int residual_sign,
                                                         int clamp_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* wl = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q4 = lane >> 4, c16 = lane & 15;
  for (int i = tid; i < kTailWBytes / 16; i += 256) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
  float bias_r[kMaxC];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) bias_r[c] = c < C ? bias[c] : 0.f;
  const size_t plane = (size_t)s.H * s.W;

  unsigned char* hl = smem + kTailWBytes;
  for (int t = blockIdx.x; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    __syncthreads();                      // previous tile's reads of hl are done
    stage_halo64(hl, in, s, b, ty0, tx0);
    __syncthreads();
    auto ldB = [&](int ks, int n) {
      const int tap = ks >> 1;
      const int p = (2 * wave + (n >> 1) + tap / 3) * kHaloW + 16 * (n & 1) + c16 + tap % 3;
      return *reinterpret_cast<const half8_t*>(hl + halo_chunk_offset(p, 4 * (ks & 1) + q4));
    };
    floatx4 acc[4] = {};
    half8_t a = *reinterpret_cast<const half8_t*>(wl + lane * 16);
    half8_t bf[4] = {ldB(0, 0), ldB(0, 1), ldB(0, 2), ldB(0, 3)};
#pragma unroll
    for (int ks = 0; ks < kTailKSteps; ++ks) {          // step ks+1 read while ks computes
      half8_t na, nb[4];
      if (ks + 1 < kTailKSteps) {
        na = *reinterpret_cast<const half8_t*>(wl + ((ks + 1) * 64 + lane) * 16);
#pragma unroll
        for (int n = 0; n < 4; ++n) nb[n] = ldB(ks + 1, n);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bf[n], acc[n], 0, 0, 0);
      if (ks + 1 < kTailKSteps) {
        a = na;
#pragma unroll
        for (int n = 0; n < 4; ++n) bf[n] = nb[n];
      }
    }
    // C/D map of 16x16: col = lane & 15 (pixel), row = 4*(lane>>4) + r (output channel).
    if (q4 == 0) {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int y = ty0 + 2 * wave + (n >> 1), x = tx0 + 16 * (n & 1) + c16;
        if (y < s.H && x < s.W) {
#pragma unroll
          for (int c = 0; c < kMaxC; ++c) {
            if (c < C) {
              const size_t idx = ((size_t)b * C + c) * plane + (size_t)y * s.W + x;
              const float net = acc[n][c] + bias_r[c];
              const float xi = xin[idx];
              float o = residual_sign > 0 ? net + xi : xi - net;
              if (clamp_out) o = fminf(fmaxf(o, 0.f), 1.f);
              xout[idx] = o;
            }
          }
        }
      }
    }
  }
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
  s.B = B; s.H = H; s.W = W; s.Hp = H + 2; s.Wp = W + 2;
  s.tiles_x = (W + kTileW - 1) / kTileW;
  s.tiles_y = (H + kTileH - 1) / kTileH;
  s.tiles = B * s.tiles_x * s.tiles_y;
  return s;
}

constexpr int kBodyLds = kBodyWBytes + 2 * kHaloDmaBytes;   // 161792 B of the 160 KiB
constexpr int kTailLds = kTailWBytes + kHaloBytes;        // 61952 B: two workgroups per CU

hipError_t conv_kernels_init() {
  hipError_t e = hipFuncSetAttribute((const void*)conv_body_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, kBodyLds);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)conv_tail_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             kTailLds);
}

void launch_conv_head(const half_t* in4, half_t* out, const void* w, const float* bias, const ConvShape& s,
                      int act, int num_cus, hipStream_t st) {
  const int grid = s.tiles < num_cus * 4 ? s.tiles : num_cus * 4;
  hipLaunchKernelGGL(conv_head_kernel, dim3(grid), dim3(256), 0, st, in4, out, (const uint4*)w, bias, s, act);
}

void launch_conv_body(const half_t* in, half_t* out, const void* w, const float* bias, const ConvShape& s,
                      int act, int num_cus, hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  hipLaunchKernelGGL(conv_body_kernel, dim3(grid), dim3(256), kBodyLds, st, in, out, (const uint4*)w, bias,
                     s, act);
}

void launch_conv_tail(const half_t* in, const float* xin, float* xout, const void* w, const float* bias,
                      const ConvShape& s, int C, int residual_sign, int clamp_out, int num_cus,
                      hipStream_t st) {
  const int grid = s.tiles < num_cus * 2 ? s.tiles : num_cus * 2;
  hipLaunchKernelGGL(conv_tail_kernel, dim3(grid), dim3(256), kTailLds, st, in, xin, xout,
                     (const uint4*)w, bias, s, C, residual_sign, clamp_out);
}

}  // namespace pnp
