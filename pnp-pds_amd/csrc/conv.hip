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

// Stage the 10 x 34 x 64-channel halo tile (padded coords [ty0, ty0+10) x [tx0, tx0+34))
// into the swizzled LDS image.  2720 16-byte chunks, 11 per thread; consecutive threads
// read consecutive 16 B of a pixel row (coalesced), write 8 lanes per 128-B pixel.
__device__ __forceinline__ void stage_halo64(unsigned char* hl, const half_t* __restrict__ in,
                                             const ConvShape& s, int b, int ty0, int tx0) {
  const half_t* base = in + (((size_t)b * s.Hp + ty0) * s.Wp + tx0) * kWidth;
  constexpr int kChunks = kHaloPix * 8;
  uint4 v[(kChunks + 255) / 256];
#pragma unroll
  for (int k = 0; k < (kChunks + 255) / 256; ++k) {
    const int q = threadIdx.x + 256 * k;
    if (q < kChunks) {
      const int p = q >> 3, c = q & 7;
      const int pr = p / kHaloW, pc = p - pr * kHaloW;
      v[k] = *reinterpret_cast<const uint4*>(base + ((size_t)pr * s.Wp + pc) * kWidth + c * 8);
    }
  }
#pragma unroll
  for (int k = 0; k < (kChunks + 255) / 256; ++k) {
    const int q = threadIdx.x + 256 * k;
    if (q < kChunks) {
      const int p = q >> 3, c = q & 7;
      *reinterpret_cast<uint4*>(hl + halo_chunk_offset(p, c)) = v[k];
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
// Body layer 64 -> 64 (basic_models.py:16-17,29-33).  LDS: 72 KiB weights + 42.5 KiB
// halo tile = 114.5 KiB -> one workgroup (4 waves) per CU, persistent over tiles.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 1) void conv_body_kernel(const half_t* __restrict__ in,
                                                            half_t* __restrict__ out,
                                                            const uint4* __restrict__ wpk,
                                                            const float* __restrict__ bias,
                                                            ConvShape s, int act) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* wl = smem;
  unsigned char* hl = smem + kBodyWBytes;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, col = lane & 31;

  for (int i = tid; i < kBodyWBytes / 16; i += 256) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
  float bias_r[2][16];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) bias_r[m][r] = bias[32 * m + 16 * h + r];

  for (int t = blockIdx.x; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    __syncthreads();                      // previous tile's reads of hl are done
    stage_halo64(hl, in, s, b, ty0, tx0);
    __syncthreads();

    floatx16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
      const int p0 = (2 * wave + ky) * kHaloW + col + kx;
      const int p1 = p0 + kHaloW;
#pragma unroll
      for (int sub = 0; sub < 4; ++sub) {
        const int ks = tap * 4 + sub;
        const half8_t a0 = *reinterpret_cast<const half8_t*>(wl + ((ks * 2 + 0) * 64 + lane) * 16);
        const half8_t a1 = *reinterpret_cast<const half8_t*>(wl + ((ks * 2 + 1) * 64 + lane) * 16);
        const int chunk = 2 * sub + h;
        const half8_t b0 = *reinterpret_cast<const half8_t*>(hl + halo_chunk_offset(p0, chunk));
        const half8_t b1 = *reinterpret_cast<const half8_t*>(hl + halo_chunk_offset(p1, chunk));
        acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc00, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc10, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc01, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, acc11, 0, 0, 0);
      }
    }
    store_act64(out, s, b, ty0 + 2 * wave, tx0 + col, h, acc00, acc10, bias_r, act);
    store_act64(out, s, b, ty0 + 2 * wave + 1, tx0 + col, h, acc01, acc11, bias_r, act);
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
  unsigned char* hl = smem + kTailWBytes;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q4 = lane >> 4, c16 = lane & 15;
  for (int i = tid; i < kTailWBytes / 16; i += 256) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
  float bias_r[kMaxC];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) bias_r[c] = c < C ? bias[c] : 0.f;
  const size_t plane = (size_t)s.H * s.W;

  for (int t = blockIdx.x; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    __syncthreads();
    stage_halo64(hl, in, s, b, ty0, tx0);
    __syncthreads();
    floatx4 acc[4] = {};
#pragma unroll
    for (int ks = 0; ks < kTailKSteps; ++ks) {
      const int tap = ks >> 1, ky = tap / 3, kx = tap % 3;
      const half8_t a = *reinterpret_cast<const half8_t*>(wl + (ks * 64 + lane) * 16);
      const int chunk = 4 * (ks & 1) + q4;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int p = (2 * wave + (n >> 1) + ky) * kHaloW + 16 * (n & 1) + c16 + kx;
        const half8_t bf = *reinterpret_cast<const half8_t*>(hl + halo_chunk_offset(p, chunk));
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bf, acc[n], 0, 0, 0);
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

constexpr int kBodyLds = kBodyWBytes + kHaloPix * 128;
constexpr int kTailLds = kTailWBytes + kHaloPix * 128;

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
