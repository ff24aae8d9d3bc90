// fp32-operand denoiser (PNP_PREC_FP32): the parity fallback of SURVEY.md §7 hard part 2.
//
// Reference: models/denoiser.py:34-46 runs simple_CNN (basic_models.py:25-38) in fp32;
// KAIR DnCNN (network_dncnn.py:42-77) likewise.  The default path (conv.hip) rounds the
// MFMA operands to fp16; this one keeps every operand fp32 on v_mfma_f32_32x32x2_f32,
// which is an exact fp32 FMA chain (MI355X_MICROARCH.md, Matrix cores), at the fp32
// matrix rate (157 TF, 1/16 of fp16).
//
// Activations: fp32 [B][H+2][W+2][64] ("padded NHWC64", 256 B per pixel, one-pixel zero
// border).  Head input: the fp32 NCHW u32 image K1 writes (clamped denoiser input), read
// with bounds checks.  Tail output: x+ in fp32 NCHW, with the residual (+x / x - n) and clamp.
//
// conv32_kernel serves the head and the body; the tail (64 -> C, C <= 4) has its own VALU
// kernel (conv32_tail_kernel below): on the MFMA its C rows padded to 32 wasted 29/32 of the
// work (7.95 ms per launch at the metric, 64 % of a 64 -> 64 layer).
// conv32_kernel tile: 8 output rows x 32 columns, all
// output channels; 4 waves, wave w owns tile rows 2w and 2w+1 (two 32-pixel N-tiles) and
// every 32-channel M-tile.  The 10 x 34 input halo is staged in LDS with a pixel pitch of
// CIN + 1 floats, so the 32 lanes of a ds_read_b32 (32 consecutive pixels, one channel)
// hit 32 distinct banks.  The A fragments (weights, [k-step][M-tile][lane] fp32, 147 KB per
// body layer, L2-resident) are loaded per tap, one tap ahead of the MFMAs that use them.
// GEMM view per tap: K = CIN input channels in steps of 2 (one MFMA K-step).
#include "kernels.h"

namespace pnp {

constexpr int kC32Pitch64 = kWidth + 1;   // LDS floats per halo pixel (64-channel input)
constexpr int kC32Pitch4 = kMaxC + 1;     // (head: C <= 4 channels)
constexpr int kC32Lds = kHaloPix * kC32Pitch64 * 4;   // 88400 B

template <int MODE>   // 0 = head (C -> 64), 1 = body (64 -> 64)
struct C32Traits {
  static constexpr int CIN = MODE == 0 ? kMaxC : kWidth;
  static constexpr int PITCH = CIN + 1;
  static constexpr int CP = CIN / 2;            // MFMA K-steps per tap
  static constexpr int NM = 2;                  // 32-channel M-tiles
  static constexpr int KS = 9 * CP;             // K-steps per layer
};

constexpr int kC32TailQ = kWidth / 4;      // tail: input channel quads
size_t conv32_weight_floats(int mode) {
  return mode == 0 ? (size_t)C32Traits<0>::KS * C32Traits<0>::NM * 64
       : mode == 1 ? (size_t)C32Traits<1>::KS * C32Traits<1>::NM * 64
                   : (size_t)kC32TailQ * 9 * 4 * 4;   // tail: [quad][tap][k][c], c < 4
}

// PyTorch layout W[cout][cin][3][3] -> [ks][m][lane]: lane l holds A[row l&31][k l>>5] of
// M-tile m at k-step ks = tap * CP + cp, i.e. input channel 2cp + (l>>5) of tap ks / CP.  Row i
// is output channel 32m + mfma32_row_to_channel(i) (64-channel outputs: accumulator register r
// of lane-half h = channel 16h + r) or channel i (tail: the C rows are registers 0..C-1 of
// lane-half 0); rows and input channels past the layer's are zero.
void pack_conv32_weights(const float* W, int mode, int cin, int cout, float* out) {
  if (mode == 2) {   // tail (VALU): out[((q * 9 + tap) * 4 + k) * 4 + c] = W[c][4q + k][tap]
    for (int q = 0; q < kC32TailQ; ++q)
      for (int tap = 0; tap < 9; ++tap)
        for (int k = 0; k < 4; ++k)
          for (int c = 0; c < 4; ++c) {
            const int ci = 4 * q + k;
            out[((q * 9 + tap) * 4 + k) * 4 + c] = (c < cout && ci < cin) ? W[((size_t)c * cin + ci) * 9 + tap] : 0.f;
          }
    return;
  }
  const int CP = mode == 0 ? kMaxC / 2 : kWidth / 2, NM = mode == 2 ? 1 : 2;
  for (int ks = 0; ks < 9 * CP; ++ks) {
    const int tap = ks / CP, cp = ks % CP;
    for (int m = 0; m < NM; ++m)
      for (int l = 0; l < 64; ++l) {
        const int i = l & 31, ci = 2 * cp + (l >> 5);
        const int co = mode == 2 ? i : 32 * m + mfma32_row_to_channel(i);
        float v = 0.f;
        if (co < cout && ci < cin) v = W[((size_t)co * cin + ci) * 9 + tap];
        out[((size_t)ks * NM + m) * 64 + l] = v;
      }
  }
}

template <int MODE, int ACT>
__global__ __launch_bounds__(256, 1) void conv32_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        const float* __restrict__ xin,
                                                        const float* __restrict__ wpk,
                                                        const float* __restrict__ bias, ConvShape s, int C,
                                                        int residual_sign, int clamp_out) {
  using T = C32Traits<MODE>;
  extern __shared__ float hl[];            // [kHaloPix][PITCH]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 31, kk = lane >> 5;
  const int Hp = s.H + 2, Wp = s.W + 2;    // fp32 activations: one-pixel border
  float bias_r[T::NM][16];
#pragma unroll
  for (int m = 0; m < T::NM; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) bias_r[m][r] = bias[32 * m + 16 * kk + r];

  auto decode = [&](int t, int& b, int& ty0, int& tx0) {
    const int per_img = s.tiles_x * s.tiles_y;
    b = t / per_img;
    const int r = t - b * per_img, ty = r / s.tiles_x;
    ty0 = ty * kTileH;
    tx0 = (r - ty * s.tiles_x) * kTileW;
  };
  // Body: the next tile's halo is loaded into registers during this tile's last tap (whose
  // next-tap weight registers are free then) and written to LDS after the tile's barrier, so
  // only the LDS writes of the fill stay exposed (one workgroup per CU: nothing else hides it).
  constexpr bool kPrefetch = MODE == 1;    // (without: 12.54 vs 10.61 ms per body layer at the metric, r02)
  constexpr int kPre = (kHaloPix * 16 + 255) / 256;   // float4 per thread
  float4 pre[kPrefetch ? kPre : 1];
  auto load_pre = [&](int tt) {
    int pb, pty, ptx;
    decode(tt, pb, pty, ptx);
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int i = tid + 256 * k;
      const int p = min(i >> 4, kHaloPix - 1), q = i & 15;
      const int pr = p / kHaloW, pc = p - pr * kHaloW;
      const int yp = pty + pr, xp = ptx + pc;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (yp < Hp && xp < Wp) v = *reinterpret_cast<const float4*>(in + (((size_t)pb * Hp + yp) * Wp + xp) * kWidth + 4 * q);
      pre[kPrefetch ? k : 0] = v;
    }
  };
  bool have_pre = false;

  for (int t = blockIdx.x; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode(t, b, ty0, tx0);
    __syncthreads();                       // previous tile's readers are done with the halo
    if (kPrefetch && have_pre) {
#pragma unroll
      for (int k = 0; k < kPre; ++k) {
        const int i = tid + 256 * k;
        if (i < kHaloPix * 16) {
          float* d = hl + (i >> 4) * T::PITCH + 4 * (i & 15);
          const float4 v = pre[kPrefetch ? k : 0];
          d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
      }
    } else if (MODE == 0) {                // gather C channels of the NCHW input, zero outside
      for (int i = tid; i < kHaloPix * kMaxC; i += 256) {
        const int p = i / kMaxC, c = i - p * kMaxC;
        const int pr = p / kHaloW, pc = p - pr * kHaloW;
        const int y = ty0 - 1 + pr, x = tx0 - 1 + pc;
        float v = 0.f;
        if (c < C && y >= 0 && y < s.H && x >= 0 && x < s.W) v = in[(((size_t)b * C + c) * s.H + y) * s.W + x];
        hl[p * T::PITCH + c] = v;
      }
    } else {                               // padded NHWC64: 16 float4 per pixel
      for (int i = tid; i < kHaloPix * 16; i += 256) {
        const int p = i >> 4, q = i & 15;
        const int pr = p / kHaloW, pc = p - pr * kHaloW;
        const int yp = ty0 + pr, xp = tx0 + pc;   // padded coordinates of the halo origin (ty0 - 1, tx0 - 1)
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (yp < Hp && xp < Wp) v = *reinterpret_cast<const float4*>(in + (((size_t)b * Hp + yp) * Wp + xp) * kWidth + 4 * q);
        float* d = hl + p * T::PITCH + 4 * q;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
    }
    __syncthreads();

    floatx16 acc[T::NM][2];
#pragma unroll
    for (int m = 0; m < T::NM; ++m) acc[m][0] = acc[m][1] = floatx16{};
    float wc[T::CP * T::NM], wn[T::CP * T::NM];
#pragma unroll
    for (int j = 0; j < T::CP * T::NM; ++j) wc[j] = wpk[j * 64 + lane];
    auto do_tap = [&](int tap, const float (&w)[T::CP * T::NM]) {
      const int dy = tap / 3, dx = tap - 3 * dy;
      const float* h0 = hl + ((2 * wave + dy) * kHaloW + col + dx) * T::PITCH + kk;
      const float* h1 = h0 + kHaloW * T::PITCH;
      // B values read PD = 2 K-steps ahead, the order pinned by a scheduling barrier per K-step
      // (the compiler's own schedule read them one MFMA ahead: 5.34 vs 5.27 ms per layer at cfg4;
      // PD = 1 / 4: 5.27 / 5.28)
      constexpr int PD = 2;
      float q0[PD + 1], q1[PD + 1];
#pragma unroll
      for (int i = 0; i < PD; ++i) { q0[i] = h0[2 * i]; q1[i] = h1[2 * i]; }
#pragma unroll
      for (int cp = 0; cp < T::CP; ++cp) {
        if (cp + PD < T::CP) {
          q0[(cp + PD) % (PD + 1)] = h0[2 * (cp + PD)];
          q1[(cp + PD) % (PD + 1)] = h1[2 * (cp + PD)];
        }
        const float b0 = q0[cp % (PD + 1)], b1 = q1[cp % (PD + 1)];
#pragma unroll
        for (int m = 0; m < T::NM; ++m) {
          acc[m][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[cp * T::NM + m], b0, acc[m][0], 0, 0, 0);
          acc[m][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[cp * T::NM + m], b1, acc[m][1], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    auto load_w = [&](float (&w)[T::CP * T::NM], int tap) {   // in flight during the tap before
#pragma unroll
      for (int j = 0; j < T::CP * T::NM; ++j) w[j] = wpk[(tap * T::CP * T::NM + j) * 64 + lane];
    };
    // Taps in pairs: the two weight sets swap roles instead of being copied (a copy of 64
    // registers per tap, into AGPRs beside the MFMAs reading them: 5.27 vs 5.02 ms per layer at cfg4)
    for (int tap = 0; tap < 8; tap += 2) {
      load_w(wn, tap + 1);
      do_tap(tap, wc);
      load_w(wc, tap + 2);
      do_tap(tap + 1, wn);
    }
    have_pre = false;
    if (kPrefetch && t + (int)gridDim.x < s.tiles) {
      load_pre(t + gridDim.x);
      have_pre = true;
    }
    do_tap(8, wc);

    // epilogue: lane (col, kk), register r of M-tile m = channel 32m + 16kk + r
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int y = ty0 + 2 * wave + n, x = tx0 + col;
      if (y >= s.H || x >= s.W) continue;
      float* o = out + (((size_t)b * Hp + y + 1) * Wp + x + 1) * kWidth + 16 * kk;
#pragma unroll
      for (int m = 0; m < T::NM; ++m)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 v;
          v.x = act_fn(acc[m][n][4 * q + 0] + bias_r[m][4 * q + 0], ACT);
          v.y = act_fn(acc[m][n][4 * q + 1] + bias_r[m][4 * q + 1], ACT);
          v.z = act_fn(acc[m][n][4 * q + 2] + bias_r[m][4 * q + 2], ACT);
          v.w = act_fn(acc[m][n][4 * q + 3] + bias_r[m][4 * q + 3], ACT);
          *reinterpret_cast<float4*>(o + 32 * m + 4 * q) = v;
        }
    }
  }
}

// Tail 64 -> C (basic_models.py:18,35-36) + residual + clamp, fp32 on the VALU: thread = one
// output pixel of an 8 x 32 tile, all C channels.  The 10 x 34 halo is staged through LDS in
// two halves of 32 channels, as 8 planes of float4 (channels 4q .. 4q+3) per half, so the 32
// lanes of a ds_read_b128 group read 512 contiguous bytes; 43.5 KiB per block (3 blocks per
// CU).  Weights are wave-uniform scalar loads, [quad][tap][k][c]; channel pairs (0,1), (2,3)
// accumulate as packed FMAs.  The sum over (channel, tap) runs in fp32 like the MFMA form,
// in a different order.
constexpr int kC32TailHalf = kC32TailQ / 2;
template <int NC>
__global__ __launch_bounds__(256) void conv32_tail_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                          const float* __restrict__ xin, const float* __restrict__ wv,
                                                          const float* __restrict__ bias, ConvShape s, int Crt,
                                                          int residual_sign, int clamp_out) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  constexpr int CM = NC ? NC : kMaxC;
  constexpr int NP = (CM + 1) / 2;           // packed channel pairs
  const int C = NC ? NC : Crt;
  __shared__ float4 hq[kC32TailHalf * kHaloPix];
  const int tid = threadIdx.x, ty = tid >> 5, tx = tid & 31;
  const int Hp = s.H + 2, Wp = s.W + 2;
  f2v bias2[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p)
    bias2[p] = f2v{2 * p < C ? bias[2 * p] : 0.f, 2 * p + 1 < C ? bias[2 * p + 1] : 0.f};
  for (int t = blockIdx.x; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    {
      const int per_img = s.tiles_x * s.tiles_y;
      b = t / per_img;
      const int r = t - b * per_img, tyy = r / s.tiles_x;
      ty0 = tyy * kTileH;
      tx0 = (r - tyy * s.tiles_x) * kTileW;
    }
    f2v acc[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) acc[p] = f2v{0.f, 0.f};
    for (int h = 0; h < 2; ++h) {
      __syncthreads();                       // the previous half's / tile's readers are done
      for (int i = tid; i < kHaloPix * kC32TailHalf; i += 256) {
        const int p = i >> 3, q = i & 7;
        const int pr = p / kHaloW, pc = p - pr * kHaloW;
        const int yp = ty0 + pr, xp = tx0 + pc;   // padded coordinates of the halo origin (ty0 - 1, tx0 - 1)
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (yp < Hp && xp < Wp)
          v = *reinterpret_cast<const float4*>(in + (((size_t)b * Hp + yp) * Wp + xp) * kWidth + 4 * (8 * h + q));
        hq[q * kHaloPix + p] = v;
      }
      __syncthreads();
      const float4* base = hq + ty * kHaloW + tx;
      for (int q = 0; q < kC32TailHalf; ++q) {
        const float* wq = wv + (size_t)(8 * h + q) * 9 * 16;
#pragma unroll 1
        for (int dy = 0; dy < 3; ++dy)       // one tap row per pass: 48 weight SGPRs live, not 144
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int tap = 3 * dy + dx;
          const float4 v = base[q * kHaloPix + dy * kHaloW + dx];
          const float vk[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int p = 0; p < NP; ++p) {
              const f2v w2 = *reinterpret_cast<const f2v*>(wq + (tap * 4 + k) * 4 + 2 * p);
              acc[p] = __builtin_elementwise_fma(w2, f2v{vk[k], vk[k]}, acc[p]);
            }
        }
      }
    }
    const int y = ty0 + ty, x = tx0 + tx;
    if (y < s.H && x < s.W) {
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        if (c >= C) break;
        const size_t o = (((size_t)b * C + c) * s.H + y) * s.W + x;
        const float net = acc[c >> 1][c & 1] + bias2[c >> 1][c & 1];
        float v = residual_sign > 0 ? net + xin[o] : xin[o] - net;
        if (clamp_out) v = fminf(fmaxf(v, 0.f), 1.f);
        out[o] = v;
      }
    }
  }
}

hipError_t conv32_kernels_init() {
  for (const void* k : {(const void*)conv32_kernel<0, 0>, (const void*)conv32_kernel<0, 1>,
                        (const void*)conv32_kernel<1, 0>, (const void*)conv32_kernel<1, 1>}) {
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kC32Lds);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

size_t act32_bytes(int B, int H, int W) {
  return (size_t)B * (H + 2) * (W + 2) * kWidth * sizeof(float);
}

void launch_conv32(int mode, const float* in, float* out, const float* xin, const float* w, const float* bias,
                   const ConvShape& s, int C, int act, int residual_sign, int clamp_out, int num_cus,
                   hipStream_t st) {
  if (mode == 2) {                                      // tail: 43.5 KB of LDS, 3 workgroups per CU
    const int grid = s.tiles < 3 * num_cus ? s.tiles : 3 * num_cus;
#define C32T(NCV) hipLaunchKernelGGL((conv32_tail_kernel<NCV>), dim3(grid), dim3(256), 0, st, in, out, xin, w, bias, s, C, \
                                     residual_sign, clamp_out)
    if (C == 3) C32T(3); else if (C == 1) C32T(1); else C32T(0);
#undef C32T
    return;
  }
  const int cap = mode == 0 ? 4 * num_cus : num_cus;   // body: 88 KB of LDS, one workgroup per CU
  const int grid = s.tiles < cap ? s.tiles : cap;
  const size_t lds = mode == 0 ? (size_t)kHaloPix * kC32Pitch4 * 4 : (size_t)kC32Lds;
#define C32(M, A) hipLaunchKernelGGL((conv32_kernel<M, A>), dim3(grid), dim3(256), lds, st, in, out, xin, w, bias, s, \
                                     C, residual_sign, clamp_out)
  if (mode == 0) {
    if (act == 0) C32(0, 0); else C32(0, 1);
  } else {
    if (act == 0) C32(1, 0); else C32(1, 1);
  }
#undef C32
}

}  // namespace pnp
