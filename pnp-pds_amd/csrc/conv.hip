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
#include <type_traits>

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
template <int NW = 4>
__device__ __forceinline__ void halo_dma(unsigned char* hl, const half_t* __restrict__ in, const ConvShape& s,
                                         int b, int ty0, int tx0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const half_t* base = in + (((size_t)b * s.Hp + ty0) * s.Wp + tx0) * kWidth;
#pragma unroll
  for (int j = 0; j < (kDmaSlots + NW - 1) / NW; ++j) {
    const int g = NW * j + wave;
    if (g < kDmaSlots) {
      const int p = 8 * g + (lane >> 3);
      const int pl = min(p, kHaloPix - 1);
      const int pr = pl / kHaloW, pc = pl - pr * kHaloW;
      const int c = (lane & 7) ^ ((pc >> 1) & 7);
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

// Coalesced epilogue: bias + activation + fp16 of NT 32-pixel N-tiles held by one wave,
// written into that wave's private LDS staging region (pixel-major, 16-B chunks XOR-
// swizzled by pixel&7: conflict-free ds_write_b128), then read back so that each
// wave-instruction stores 8 whole pixels = 1 KiB contiguous (8 full 128-B lines).
// The scattered direct store (64 separate 16-B pieces per instruction) cost 0.5 ms of a
// 1.45 ms layer at 256x256x256 (ablation).
template <int NT>
__device__ __forceinline__ void epilogue_coalesced(unsigned char* stage, half_t* __restrict__ out,
                                                   const ConvShape& s, int b, const int (&rows)[NT], int tx0,
                                                   const floatx16 (&acc)[2][NT], const float (&bias)[2][16],
                                                   int act) {
  const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int pix = n * 32 + col;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      half8_t lo, hi;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        lo[r] = (half_t)act_fn(acc[m][n][r] + bias[m][r], act);
        hi[r] = (half_t)act_fn(acc[m][n][r + 8] + bias[m][r + 8], act);
      }
      const int q = 4 * m + 2 * h;       // 16-B chunk index of channels 32m+16h .. +7
      *reinterpret_cast<half8_t*>(stage + pix * 128 + 16 * (q ^ (pix & 7))) = lo;
      *reinterpret_cast<half8_t*>(stage + pix * 128 + 16 * ((q + 1) ^ (pix & 7))) = hi;
    }
  }
  // own region only: a wave-level LDS fence suffices before reading back
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // Stores through one buffer descriptor per output row whose record count covers exactly
  // the valid pixels: the hardware range check drops out-of-image lanes, so every wave
  // issues exactly NT*4 store instructions with no branches, and the caller's counted
  // vmcnt(NT*4) waits for the (older) prefetch DMA only, leaving these stores in flight.
  typedef int v4i_t __attribute__((ext_vector_type(4)));
  v4i_t v[NT * 4];
#pragma unroll
  for (int j = 0; j < NT * 4; ++j) {
    const int pix = 8 * j + (lane >> 3), c = lane & 7;
    v[j] = *reinterpret_cast<const v4i_t*>(stage + pix * 128 + 16 * (c ^ (pix & 7)));
  }
  const int ncols = min(kTileW, s.W - tx0);
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int y = __builtin_amdgcn_readfirstlane(rows[n]);          // wave-uniform (T20)
    half_t* row = out + (((size_t)b * s.Hp + y + 1) * s.Wp + tx0 + 1) * kWidth;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = 4 * n + q, pix = 8 * j + (lane >> 3), c = lane & 7;
      __builtin_amdgcn_raw_buffer_store_b128(v[j], rs, (pix & 31) * 128 + c * 16, 0, 0);
    }
  }
}

// Deferred form of the same epilogue: stage + read back now, issue the 4*NT stores later
// (spread over the next tile's MFMA loop, where their issue hides in MFMA gaps).
typedef int v4i_t __attribute__((ext_vector_type(4)));
template <int NT>
struct PendingStores {
  v4i_t v[NT * 4];
  __amdgpu_buffer_rsrc_t rs[NT];
};

template <int NT>
__device__ __forceinline__ void pending_clear(PendingStores<NT>& ps, half_t* out) {
#pragma unroll
  for (int n = 0; n < NT; ++n) ps.rs[n] = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000);
#pragma unroll
  for (int j = 0; j < NT * 4; ++j) ps.v[j] = v4i_t{0, 0, 0, 0};
}

template <int NT>
__device__ __forceinline__ void epilogue_stage(unsigned char* stage, half_t* __restrict__ out, const ConvShape& s,
                                               int b, const int (&rows)[NT], int tx0, const floatx16 (&acc)[2][NT],
                                               const float (&bias)[2][16], int act, PendingStores<NT>& ps) {
  const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int pix = n * 32 + col;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      half8_t lo, hi;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        lo[r] = (half_t)act_fn(acc[m][n][r] + bias[m][r], act);
        hi[r] = (half_t)act_fn(acc[m][n][r + 8] + bias[m][r + 8], act);
      }
      const int q = 4 * m + 2 * h;
      *reinterpret_cast<half8_t*>(stage + pix * 128 + 16 * (q ^ (pix & 7))) = lo;
      *reinterpret_cast<half8_t*>(stage + pix * 128 + 16 * ((q + 1) ^ (pix & 7))) = hi;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int j = 0; j < NT * 4; ++j) {
    const int pix = 8 * j + (lane >> 3), c = lane & 7;
    ps.v[j] = *reinterpret_cast<const v4i_t*>(stage + pix * 128 + 16 * (c ^ (pix & 7)));
  }
  const int ncols = min(kTileW, s.W - tx0);
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int y = __builtin_amdgcn_readfirstlane(rows[n]);
    half_t* row = out + (((size_t)b * s.Hp + y + 1) * s.Wp + tx0 + 1) * kWidth;
    ps.rs[n] = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
  }
}

template <int NT>
__device__ __forceinline__ void pending_store(const PendingStores<NT>& ps, int j) {
  const int lane = threadIdx.x & 63;
  const int pix = 8 * j + (lane >> 3), c = lane & 7;
  __builtin_amdgcn_raw_buffer_store_b128(ps.v[j], ps.rs[j >> 2], (pix & 31) * 128 + c * 16, 0, 0);
}

// End of a pipelined tile: this wave's prefetch DMA (issued before its NSTORES epilogue
// stores) has landed, all of this wave's LDS reads are done, then the workgroup barrier.
template <int NSTORES>
__device__ __forceinline__ void tile_boundary() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORES) : "memory");
  __builtin_amdgcn_s_barrier();
}

// ------------------------------------------------------------------------------------
// Body layer 64 -> 64 (basic_models.py:16-17,29-33).  LDS: 72 KiB weights + two 42.5 KiB
// halo buffers = 157 KiB -> one workgroup (4 waves) per CU, persistent over tiles.
// Software pipeline per tile: issue the global loads of tile t+1 into registers, run
// tile t's 144 MFMAs/wave from LDS buffer `cur`, store tile t, then write tile t+1 into
// buffer `cur^1`; one barrier per tile.
// ------------------------------------------------------------------------------------

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
      if (!(s.ablate & 1)) halo_dma(smem + kBodyWBytes + (cur ^ 1) * kHaloDmaBytes, in, s, bn, tyn, txn);
    }
    const unsigned char* hl = smem + kBodyWBytes + cur * kHaloDmaBytes;
    auto ldA = [&](int ks, int m) {
      return *reinterpret_cast<const half8_t*>(wl + ((ks * 2 + m) * 64 + lane) * 16);
    };
    auto ldB = [&](int ks, int n) {           // this lane's pixel at tap (0,0): (2*wave, col)
      const int tap = ks >> 2, sub = ks & 3;
      return *reinterpret_cast<const half8_t*>(
          hl + halo_off(2 * wave + n + tap / 3, col + tap % 3, 2 * sub + h));
    };

    // K loop over a 3-slot fragment ring: the LDS reads of step ks+2 are issued while
    // step ks's MFMAs run, so each read has at least one full step (4 MFMAs, ~128
    // cycles) to land — at one wave per SIMD nothing else hides LDS latency.
    floatx16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
    half8_t fa[3][2], fb[3][2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      fa[q][0] = ldA(q, 0); fa[q][1] = ldA(q, 1);
      fb[q][0] = ldB(q, 0); fb[q][1] = ldB(q, 1);
    }
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks) {
      const int r = ks % 3;
      if (ks + 2 < kBodyKSteps) {
        const int w = (ks + 2) % 3;
        fa[w][0] = ldA(ks + 2, 0); fa[w][1] = ldA(ks + 2, 1);
        fb[w][0] = ldB(ks + 2, 0); fb[w][1] = ldB(ks + 2, 1);
      }
      // hipcc's scheduler otherwise sinks the reads to just before their consumers
      __builtin_amdgcn_sched_barrier(0);
      acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r][0], fb[r][0], acc00, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r][1], fb[r][0], acc10, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r][0], fb[r][1], acc01, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r][1], fb[r][1], acc11, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!(s.ablate & 2)) {
      // every wave is done reading halo buffer `cur`: reuse it as the store staging area
      // (raw barrier: no vmcnt(0), the next tile's DMA stays in flight)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int rows[2] = {ty0 + 2 * wave, ty0 + 2 * wave + 1};
      const floatx16 acc[2][2] = {{acc00, acc01}, {acc10, acc11}};
      epilogue_coalesced<2>(smem + kBodyWBytes + cur * kHaloDmaBytes + wave * 8192, out, s, b, rows, tx0, acc,
                            bias_r, act);
      tile_boundary<8>();                     // next tile landed; stores stay in flight
    } else {
      if (acc00[0] + acc01[0] + acc10[0] + acc11[0] == -1e30f) out[0] = (half_t)0;   // keeps MFMAs live
      __syncthreads();
    }
    cur ^= 1;
  }
}

// ------------------------------------------------------------------------------------
// Body layer, 8-wave variant: 512 threads = two waves per SIMD, wave w owns output row
// w of the 8x32 tile (one 32-pixel N-tile) x 64 channels (two M-tiles).  Per K-step
// 2 weight + 1 activation ds_read_b128 and 2 MFMAs.  The partner wave on the same SIMD
// issues its MFMAs while this one waits on LDS, runs its epilogue or issues DMA.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(512, 2) void conv_body8_kernel(const half_t* __restrict__ in,
                                                             half_t* __restrict__ out,
                                                             const uint4* __restrict__ wpk,
                                                             const float* __restrict__ bias,
                                                             ConvShape s, int act) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* wl = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, col = lane & 31;

  for (int i = tid; i < kBodyWBytes / 16; i += 512) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
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
    halo_dma<8>(smem + kBodyWBytes, in, s, b, ty0, tx0);
  }
  __syncthreads();
  PendingStores<1> ps;                        // stores of the previous tile (none yet:
  pending_clear(ps, out);                     // zero-record descriptor, dropped by hardware)
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const int tn = t + gridDim.x;
    if (tn < s.tiles) {
      int bn, tyn, txn;
      decode_tile(tn, s, bn, tyn, txn);
      if (!(s.ablate & 1)) halo_dma<8>(smem + kBodyWBytes + (cur ^ 1) * kHaloDmaBytes, in, s, bn, tyn, txn);
    }
    const unsigned char* hl = smem + kBodyWBytes + cur * kHaloDmaBytes;
    auto ldA = [&](int ks, int m) {
      return *reinterpret_cast<const half8_t*>(wl + ((ks * 2 + m) * 64 + lane) * 16);
    };
    auto ldB = [&](int ks) {
      const int tap = ks >> 2, sub = ks & 3;
      return *reinterpret_cast<const half8_t*>(hl + halo_off(wave + tap / 3, col + tap % 3, 2 * sub + h));
    };
    floatx16 acc0 = {}, acc1 = {};
    half8_t fa0 = ldA(0, 0), fa1 = ldA(0, 1), fb = ldB(0);
    if (s.ablate & 4) {                       // profiling: memory path only
#pragma unroll
      for (int j = 0; j < 4; ++j) pending_store(ps, j);
      acc0[0] = (float)fa0[0] + (float)fb[0];
      acc1[0] = (float)fa1[0];
    } else
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks) {
      half8_t na0, na1, nb;
      if (ks + 1 < kBodyKSteps) { na0 = ldA(ks + 1, 0); na1 = ldA(ks + 1, 1); nb = ldB(ks + 1); }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa0, fb, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa1, fb, acc1, 0, 0, 0);
      if (ks + 1 < kBodyKSteps) { fa0 = na0; fa1 = na1; fb = nb; }
      if ((ks & 7) == 4) {                    // previous tile's stores, one per 8 K-steps
        __builtin_amdgcn_sched_barrier(0);
        pending_store(ps, ks >> 3);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // every wave is done reading halo buffer `cur`: reuse it as the staging area
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (!(s.ablate & 2)) {
      const int rows[1] = {ty0 + wave};
      const floatx16 acc[2][1] = {{acc0}, {acc1}};
      epilogue_stage<1>(smem + kBodyWBytes + cur * kHaloDmaBytes + wave * 4096, out, s, b, rows, tx0, acc, bias_r,
                        act, ps);
    } else if (acc0[0] + acc1[0] == -1e30f) {
      out[0] = (half_t)0;                     // keeps every MFMA live (rule 17)
    }
    tile_boundary<4>();                       // DMA of the next tile landed (4 stores younger)
    cur ^= 1;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) pending_store(ps, j);   // last tile's stores
}

// ------------------------------------------------------------------------------------
// Body layer, wave-specialised variant (2): 8 waves = 4 compute + 4 memory waves, one of
// each per SIMD.  Compute waves (0-3) only read LDS and issue MFMAs (2 rows x 64 ch each);
// memory waves (4-7) move bytes: they read the previous tile's staged outputs from LDS,
// issue its coalesced stores and the next tile's LDS-DMA, and wait for that DMA — so a
// store or DMA that stalls at issue never stalls the MFMA stream.  Per tile:
//   compute: MFMA(t) from buf c   | memory: staged(t-1) from buf c^1 -> regs, DMA(t+1) -> c^1, stores(t-1)
//   --- barrier B1 ---
//   compute: stage outputs(t) -> buf c (8 KiB per compute wave)
//   --- barrier B2 ---
// Memory wave i re-fills by DMA only LDS it has itself just read (staging region i = DMA
// slots 8i..8i+7) or that nobody reads (slots 32..42), so no barrier is needed between
// its reads and the DMA.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void dma_slot(unsigned char* hl, const half_t* __restrict__ base, const ConvShape& s,
                                         int g) {
  const int lane = threadIdx.x & 63;
  const int p = 8 * g + (lane >> 3);
  const int pl = min(p, kHaloPix - 1);
  const int pr = pl / kHaloW, pc = pl - pr * kHaloW;
  const int c = (lane & 7) ^ ((pc >> 1) & 7);
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + ((size_t)pr * s.Wp + pc) *
                                                                                       kWidth + c * 8),
                                   (__attribute__((address_space(3))) void*)(hl + g * 1024), 16, 0, 0);
}

// DMA slots owned by memory wave mw: 8mw..8mw+7 and 32+3mw .. min(32+3mw+2, 42).
__device__ __forceinline__ void dma_owned(unsigned char* hl, const half_t* __restrict__ in, const ConvShape& s,
                                          int b, int ty0, int tx0, int mw) {
  const half_t* base = in + (((size_t)b * s.Hp + ty0) * s.Wp + tx0) * kWidth;
#pragma unroll
  for (int k = 0; k < 8; ++k) dma_slot(hl, base, s, 8 * mw + k);
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (32 + 3 * mw + k < kDmaSlots) dma_slot(hl, base, s, 32 + 3 * mw + k);
}

__global__ __launch_bounds__(512, 2) void conv_body_ws_kernel(const half_t* __restrict__ in,
                                                               half_t* __restrict__ out,
                                                               const uint4* __restrict__ wpk,
                                                               const float* __restrict__ bias,
                                                               ConvShape s, int act) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* wl = smem;
  unsigned char* hbuf = smem + kBodyWBytes;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool is_mem = wave >= 4;
  const int cw = wave & 3;                    // compute wave index / memory wave index
  const int h = lane >> 5, col = lane & 31;
  float* bias_l = reinterpret_cast<float*>(smem + kBodyWBytes + 2 * kHaloDmaBytes);   // 256 B, not registers

  for (int i = tid; i < kBodyWBytes / 16; i += 512) reinterpret_cast<uint4*>(wl)[i] = wpk[i];
  if (tid < kWidth) bias_l[tid] = bias[tid];

  int t = blockIdx.x;
  if (is_mem && t < s.tiles) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    dma_owned(hbuf, in, s, b, ty0, tx0, cw);
  }
  __syncthreads();                            // vmcnt(0): first tile landed
  int cur = 0;
  int pb = 0, pty0 = 0, ptx0 = 0;             // previous tile (its outputs are staged)
  bool have_prev = false;
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    floatx16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
    if (is_mem) {
      unsigned char* other = hbuf + (cur ^ 1) * kHaloDmaBytes;
      v4i_t v[8];
      if (have_prev) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int pix = 8 * j + (lane >> 3), c = lane & 7;
          v[j] = *reinterpret_cast<const v4i_t*>(other + cw * 8192 + pix * 128 + 16 * (c ^ (pix & 7)));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // data in registers before the DMA lands
      }
      const int tn = t + gridDim.x;
      if (tn < s.tiles) {
        int bn, tyn, txn;
        decode_tile(tn, s, bn, tyn, txn);
        dma_owned(other, in, s, bn, tyn, txn, cw);
      }
      if (have_prev) {
        const int ncols = min(kTileW, s.W - ptx0);
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int y = pty0 + 2 * cw + n;
          half_t* row = out + (((size_t)pb * s.Hp + y + 1) * s.Wp + ptx0 + 1) * kWidth;
          const __amdgpu_buffer_rsrc_t rs =
              __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int j = 4 * n + q, pix = 8 * j + (lane >> 3), c = lane & 7;
            __builtin_amdgcn_raw_buffer_store_b128(v[j], rs, (pix & 31) * 128 + c * 16, 0, 0);
          }
        }
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");     // the DMA (older than the stores)
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      const unsigned char* hl = hbuf + cur * kHaloDmaBytes;
      auto ldA = [&](int ks, int m) {
        return *reinterpret_cast<const half8_t*>(wl + ((ks * 2 + m) * 64 + lane) * 16);
      };
      auto ldB = [&](int ks, int n) {
        const int tap = ks >> 2, sub = ks & 3;
        return *reinterpret_cast<const half8_t*>(
            hl + halo_off(2 * cw + n + tap / 3, col + tap % 3, 2 * sub + h));
      };
      half8_t fa[2][2], fb[2][2];             // 2-slot ring: step ks+1 read while ks computes
      fa[0][0] = ldA(0, 0); fa[0][1] = ldA(0, 1);
      fb[0][0] = ldB(0, 0); fb[0][1] = ldB(0, 1);
#pragma unroll
      for (int ks = 0; ks < kBodyKSteps; ++ks) {
        const int r = ks & 1;
        if (ks + 1 < kBodyKSteps) {
          const int w = r ^ 1;
          fa[w][0] = ldA(ks + 1, 0); fa[w][1] = ldA(ks + 1, 1);
          fb[w][0] = ldB(ks + 1, 0); fb[w][1] = ldB(ks + 1, 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r][0], fb[r][0], acc00, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r][1], fb[r][0], acc10, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r][0], fb[r][1], acc01, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r][1], fb[r][1], acc11, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();             // B1: buf cur fully read; DMA(t+1) landed
    if (!is_mem) {                            // stage tile t's outputs into buf cur
      unsigned char* stage = hbuf + cur * kHaloDmaBytes + cw * 8192;
      const floatx16 acc[2][2] = {{acc00, acc01}, {acc10, acc11}};
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int pix = n * 32 + col;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const float* bl = bias_l + 32 * m + 16 * h;
          half8_t lo, hi;
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            lo[r] = (half_t)act_fn(acc[m][n][r] + bl[r], act);
            hi[r] = (half_t)act_fn(acc[m][n][r + 8] + bl[r + 8], act);
          }
          const int q = 4 * m + 2 * h;
          *reinterpret_cast<half8_t*>(stage + pix * 128 + 16 * (q ^ (pix & 7))) = lo;
          *reinterpret_cast<half8_t*>(stage + pix * 128 + 16 * ((q + 1) ^ (pix & 7))) = hi;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();             // B2: tile t staged
    pb = b; pty0 = ty0; ptx0 = tx0;
    have_prev = true;
    cur ^= 1;
  }
  if (is_mem && have_prev) {                  // the last tile's outputs
    const unsigned char* other = hbuf + (cur ^ 1) * kHaloDmaBytes;
    const int ncols = min(kTileW, s.W - ptx0);
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int y = pty0 + 2 * cw + n;
      half_t* row = out + (((size_t)pb * s.Hp + y + 1) * s.Wp + ptx0 + 1) * kWidth;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 4 * n + q, pix = 8 * j + (lane >> 3), c = lane & 7;
        const v4i_t v = *reinterpret_cast<const v4i_t*>(other + cw * 8192 + pix * 128 + 16 * (c ^ (pix & 7)));
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (pix & 31) * 128 + c * 16, 0, 0);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Body layer, variant 3: weights in registers + 3-deep halo ring.
// 8 waves; wave w owns output channels 32m..32m+31 (m = w&1) of tile rows 2(w>>1) and
// 2(w>>1)+1, and keeps its 36 A-fragments (the whole K extent of its M-tile, 144 VGPRs) in
// registers for the launch.  The K-loop reads only 2 activation fragments per 2 MFMAs from
// LDS, and the 72 KiB that held the weights in variants 0-2 now holds a third halo buffer:
// the DMA runs two tiles ahead.  Outputs go through a wave-private 4 KiB staging area
// (64-B half pixels, read back 16 pixels x 64 B per instruction) and are stored during the
// next tile's K-loop, so the only workgroup barrier per tile is the ring hand-over.
// LDS: 3 x 42.5 KiB halo + 8 x 4 KiB staging + bias = 163584 B.
// ------------------------------------------------------------------------------------
constexpr int kV3Halo = kHaloPix * 128;  // 43520: the last DMA slot is issued by half a wave
constexpr int kV3Stage = 3 * kV3Halo;
constexpr int kV3Bias = kV3Stage + 8 * 4096;
constexpr int kV3Lds = kV3Bias + 256;                           // 163584 B

template <int NW>
__device__ __forceinline__ int dma_count(int wave) {           // slots issued by `wave`
  return (kDmaSlots - wave + NW - 1) / NW;
}

// Halo DMA through a buffer descriptor: the tile base lives in SGPRs and the per-lane
// byte offsets of this wave's slots are tile-invariant (computed once per launch), so an
// issue costs one VGPR per slot instead of a 64-bit address.
// UNIFORM: every wave issues kSlots (the extra slots re-read pixel 339 into padding past
// the halo), so the issue has no control flow and the compiler's own vmcnt accounting for
// loads issued before it stays exact; the buffer must then hold NW * kSlots KiB.
template <int NW, bool UNIFORM = false>
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
      const int c = (lane & 7) ^ ((pc >> 1) & 7);
      off[j] = (unsigned)(((pr * s.Wp + pc) * kWidth + c * 8) * 2);
    }
  }
  __device__ __forceinline__ void issue(unsigned char* hl, const half_t* __restrict__ in, const ConvShape& s, int t,
                                        int wave) const {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const half_t* base = in + (((size_t)b * s.Hp + ty0) * s.Wp + tx0) * kWidth;
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

// Channel-plane halo image (variant 3 PLANES): chunk c (channels 8c..8c+7) of halo pixel p
// at c*5440 + 16p.  A 16-lane ds_read_b128 group over consecutive pixels is then 256
// contiguous bytes (conflict-free without a swizzle) and every fragment address is one
// per-lane base plus an immediate.  Wave w DMAs plane w: 6 instructions of 64 pixels
// (the last one 20), each lane one 16-B chunk; the 8 waves read the 8 chunks of the same
// 128-B pixel lines together, so the lines are fetched from L2 once.
constexpr int kPlaneBytes = kHaloPix * 16;                     // 5440
struct PlaneDma {
  unsigned off[6];
  __device__ __forceinline__ void init(const ConvShape& s, int wave) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int pl = min(64 * j + lane, kHaloPix - 1);
      const int pr = pl / kHaloW, pc = pl - pr * kHaloW;
      off[j] = (unsigned)(((pr * s.Wp + pc) * kWidth + wave * 8) * 2);
    }
  }
  __device__ __forceinline__ void issue(unsigned char* hl, const half_t* __restrict__ in, const ConvShape& s, int t,
                                        int wave) const {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const half_t* base = in + (((size_t)b * s.Hp + ty0) * s.Wp + tx0) * kWidth;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (j < 5 || lane < kHaloPix - 320)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(hl + wave * kPlaneBytes + 1024 * j), 16, off[j], 0, 0, 0);
  }
};

template <bool PLANES, int NFRAG>
__global__ __launch_bounds__(512, 2) void conv_body_v3_kernel(const half_t* __restrict__ in,
                                                               half_t* __restrict__ out,
                                                               const uint4* __restrict__ wpk,
                                                               const float* __restrict__ bias,
                                                               ConvShape s, int act) {
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
  typename std::conditional<PLANES, PlaneDma, RingDma<8>>::type dma;
  dma.init(s, wave);
  auto issue_dma = [&](int tt, int bi) {      // clamped: always the same instruction count
    dma.issue(buf(bi), in, s, tt < s.tiles ? tt : s.tiles - 1, wave);
  };
  const int ndma = PLANES ? 6 : dma_count<8>(wave);

  int t = blockIdx.x;
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
    __builtin_amdgcn_raw_buffer_store_b128(v, rs[j >> 1], (pix & 31) * 128 + 64 * m + 16 * c, 0, 0);
  };
  int cur = 0;
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const int nxt2 = cur >= 1 ? cur - 1 : 2;  // (cur + 2) % 3
    issue_dma(t + 2 * gridDim.x, nxt2);
    const unsigned char* hl = buf(cur);
    // PLANES: one per-lane base, every tap / chunk offset an instruction immediate
    const unsigned char* pb = hl + h * kPlaneBytes + (2 * rp * kHaloW + col) * 16;
    auto ldB = [&](int ks, int n) {
      const int tap = ks >> 2, sub = ks & 3;
      if (PLANES)
        return *reinterpret_cast<const half8_t*>(pb + 2 * sub * kPlaneBytes +
                                                 ((n + tap / 3) * kHaloW + tap % 3) * 16);
      return *reinterpret_cast<const half8_t*>(
          hl + halo_off(2 * rp + n + tap / 3, col + tap % 3, 2 * sub + h));
    };
    floatx16 acc0 = {}, acc1 = {};
    half8_t fb[NFRAG][2];
    v4i_t sv;
#pragma unroll
    for (int k = 0; k < NFRAG - 1; ++k) { fb[k][0] = ldB(k, 0); fb[k][1] = ldB(k, 1); }
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks) {
      const int r = ks % NFRAG;
      if ((ks & 7) == 2) {                    // previous tile's stores, one per 8 K-steps
        __builtin_amdgcn_sched_barrier(0);
        sv = stage_read(ks >> 3);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (ks + NFRAG - 1 < kBodyKSteps) {
        const int kn = ks + NFRAG - 1;
        fb[kn % NFRAG][0] = ldB(kn, 0);
        fb[kn % NFRAG][1] = ldB(kn, 1);
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[r][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks], fb[r][1], acc1, 0, 0, 0);
      if ((ks & 7) == 4) {
        __builtin_amdgcn_sched_barrier(0);
        stage_store(ks >> 3, sv);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (NFRAG > 2) __builtin_amdgcn_sched_barrier(0);   // keep the reads NFRAG-1 steps ahead
    }
    {                                         // bias + activation -> fp16 -> staging (wave-private)
      const float* bl = bias_l + 32 * m + 16 * h;
      const int sw = (col >> 1) & 3;    // ds_write_b128 banks repeat every 128 B: 8 lanes distinct
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int pix = n * 32 + col;
        const floatx16& a = n == 0 ? acc0 : acc1;
        half8_t lo, hi;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          lo[r] = (half_t)act_fn(a[r] + bl[r], act);
          hi[r] = (half_t)act_fn(a[r + 8] + bl[r + 8], act);
        }
        *reinterpret_cast<half8_t*>(stg + pix * 64 + 16 * ((2 * h) ^ sw)) = lo;
        *reinterpret_cast<half8_t*>(stg + pix * 64 + 16 * ((2 * h + 1) ^ sw)) = hi;
      }
      const int ncols = min(kTileW, s.W - tx0);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int y = ty0 + 2 * rp + n;
        half_t* row = out + (((size_t)b * s.Hp + y + 1) * s.Wp + tx0 + 1) * kWidth;
        rs[n] = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
      }
    }
    // tile t+1 landed: only the DMA of t+2 (ndma ops) and this tile's 4 stores are younger
    if (ndma == 6) asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) stage_store(j, stage_read(j));
}

// ------------------------------------------------------------------------------------
// Body layer, variant 4: one wave per SIMD holding the WHOLE layer's weights.
// 4 waves; wave w computes all 64 output channels of tile rows 2w, 2w+1.  Its 72
// A-fragments (288 registers) stay resident for the launch, so every activation fragment
// read from LDS feeds 2 MFMAs (half the LDS reads of variant 3 per MFMA), and the fragment
// ring runs two K-steps (8 MFMAs) ahead with counted lgkmcnt waits.  Staging is
// wave-private (8 KiB: 64 whole 128-B pixels) and its 8 full-line stores per wave are
// issued during the next tile's K-loop.  Same LDS map as variant 3 (3-deep halo ring).
// ------------------------------------------------------------------------------------
constexpr int kV4Stage = 3 * kV3Halo;
constexpr int kV4Bias = kV4Stage + 4 * 8192;
constexpr int kV4Lds = kV4Bias + 256;                           // 163584 B

__global__ __launch_bounds__(256, 1) void conv_body_v4_kernel(const half_t* __restrict__ in,
                                                               half_t* __restrict__ out,
                                                               const uint4* __restrict__ wpk,
                                                               const float* __restrict__ bias,
                                                               ConvShape s, int act) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* bias_l = reinterpret_cast<float*>(smem + kV4Bias);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, col = lane & 31;
  unsigned char* stg = smem + kV4Stage + wave * 8192;
  if (tid < kWidth) bias_l[tid] = bias[tid];

  half8_t wA[kBodyKSteps][2];                 // the layer's weights, resident for the launch
#pragma unroll
  for (int ks = 0; ks < kBodyKSteps; ++ks)
#pragma unroll
    for (int m = 0; m < 2; ++m)
      wA[ks][m] = *reinterpret_cast<const half8_t*>(reinterpret_cast<const unsigned char*>(wpk) +
                                                    ((ks * 2 + m) * 64 + lane) * 16);

  auto buf = [&](int i) { return smem + i * kV3Halo; };
  RingDma<4> dma;
  dma.init(s, wave);
  auto issue_dma = [&](int tt, int bi) {      // clamped: always the same instruction count
    dma.issue(buf(bi), in, s, tt < s.tiles ? tt : s.tiles - 1, wave);
  };
  const bool full = dma_count<4>(wave) == 11; // waves 0-2 issue 11 slots, wave 3 issues 10

  int t = blockIdx.x;
  if (t < s.tiles) {
    issue_dma(t, 0);
    issue_dma(t + gridDim.x, 1);
    if (full) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");     // tile t landed
    else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  }
  __syncthreads();
  __amdgpu_buffer_rsrc_t rs[2];
  rs[0] = rs[1] = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0, 0x00020000);   // first tile: dropped
  auto stage_read = [&](int j) {              // 8 whole pixels per instruction
    const int pix = 8 * j + (lane >> 3), c = lane & 7;
    return *reinterpret_cast<const v4i_t*>(stg + pix * 128 + 16 * (c ^ (pix & 7)));
  };
  auto stage_store = [&](int j, const v4i_t& v) {
    const int pix = 8 * j + (lane >> 3), c = lane & 7;
    __builtin_amdgcn_raw_buffer_store_b128(v, rs[j >> 2], (pix & 31) * 128 + 16 * c, 0, 0);
  };
  int cur = 0;
  for (; t < s.tiles; t += gridDim.x) {
    int b, ty0, tx0;
    decode_tile(t, s, b, ty0, tx0);
    const int nxt2 = cur >= 1 ? cur - 1 : 2;  // (cur + 2) % 3
    issue_dma(t + 2 * gridDim.x, nxt2);
    const unsigned char* hl = buf(cur);
    auto ldB = [&](int ks, int n) {
      const int tap = ks >> 2, sub = ks & 3;
      return *reinterpret_cast<const half8_t*>(
          hl + halo_off(2 * wave + n + tap / 3, col + tap % 3, 2 * sub + h));
    };
    floatx16 acc[2][2] = {};
    half8_t fb[3][2];
    v4i_t sv;
    fb[0][0] = ldB(0, 0); fb[0][1] = ldB(0, 1);
    fb[1][0] = ldB(1, 0); fb[1][1] = ldB(1, 1);
#pragma unroll
    for (int ks = 0; ks < kBodyKSteps; ++ks) {
      const int r = ks % 3;
      if ((ks & 3) == 1 && ks < 32) {         // previous tile's stores: 8, one per 4 K-steps
        __builtin_amdgcn_sched_barrier(0);
        sv = stage_read(ks >> 2);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (ks + 2 < kBodyKSteps) { fb[(ks + 2) % 3][0] = ldB(ks + 2, 0); fb[(ks + 2) % 3][1] = ldB(ks + 2, 1); }
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int m = 0; m < 2; ++m)
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wA[ks][m], fb[r][n], acc[m][n], 0, 0, 0);
      if ((ks & 3) == 3 && ks < 32) {
        __builtin_amdgcn_sched_barrier(0);
        stage_store(ks >> 2, sv);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    {                                         // bias + activation -> fp16 -> staging (wave-private)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int pix = n * 32 + col;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const float* bl = bias_l + 32 * m + 16 * h;
          half8_t lo, hi;
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            lo[r] = (half_t)act_fn(acc[m][n][r] + bl[r], act);
            hi[r] = (half_t)act_fn(acc[m][n][r + 8] + bl[r + 8], act);
          }
          const int q = 4 * m + 2 * h;
          *reinterpret_cast<half8_t*>(stg + pix * 128 + 16 * (q ^ (pix & 7))) = lo;
          *reinterpret_cast<half8_t*>(stg + pix * 128 + 16 * ((q + 1) ^ (pix & 7))) = hi;
        }
      }
      const int ncols = min(kTileW, s.W - tx0);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int y = ty0 + 2 * wave + n;
        half_t* row = out + (((size_t)b * s.Hp + y + 1) * s.Wp + tx0 + 1) * kWidth;
        rs[n] = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, y < s.H ? ncols * 128 : 0, 0x00020000);
      }
    }
    // tile t+1 landed: only the DMA of t+2 and this tile's 8 stores are younger
    if (full) asm volatile("s_waitcnt vmcnt(19) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) stage_store(j, stage_read(j));
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
  s.ablate = 0;
  s.trash = nullptr;
  return s;
}

constexpr int kBodyLds = kBodyWBytes + 2 * kHaloDmaBytes + 256;   // 162048 B of the 160 KiB (+ bias)

hipError_t conv_kernels_init() {
  hipError_t e = hipFuncSetAttribute((const void*)conv_body_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, kBodyLds);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)conv_body8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kBodyLds);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)conv_body_ws_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kBodyLds);
  if (e != hipSuccess) return e;
  for (const void* k : {(const void*)conv_body_v3_kernel<false, 2>, (const void*)conv_body_v3_kernel<true, 2>,
                        (const void*)conv_body_v3_kernel<true, 3>}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kV3Lds);
    if (e != hipSuccess) return e;
  }
  e = hipFuncSetAttribute((const void*)conv_body_v4_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kV4Lds);
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
                      int act, int num_cus, int variant, hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  if (variant == 4)
    hipLaunchKernelGGL(conv_body_v4_kernel, dim3(grid), dim3(256), kV4Lds, st, in, out, (const uint4*)w, bias,
                       s, act);
  else if (variant == 5)
    hipLaunchKernelGGL((conv_body_v3_kernel<true, 2>), dim3(grid), dim3(512), kV3Lds, st, in, out, (const uint4*)w,
                       bias, s, act);
  else if (variant == 6)
    hipLaunchKernelGGL((conv_body_v3_kernel<true, 3>), dim3(grid), dim3(512), kV3Lds, st, in, out, (const uint4*)w,
                       bias, s, act);
  else if (variant == 3)
    hipLaunchKernelGGL((conv_body_v3_kernel<false, 2>), dim3(grid), dim3(512), kV3Lds, st, in, out, (const uint4*)w, bias,
                       s, act);
  else if (variant == 2)
    hipLaunchKernelGGL(conv_body_ws_kernel, dim3(grid), dim3(512), kBodyLds, st, in, out, (const uint4*)w, bias,
                       s, act);
  else if (variant == 1)
    hipLaunchKernelGGL(conv_body8_kernel, dim3(grid), dim3(512), kBodyLds, st, in, out, (const uint4*)w, bias,
                       s, act);
  else
    hipLaunchKernelGGL(conv_body_kernel, dim3(grid), dim3(256), kBodyLds, st, in, out, (const uint4*)w, bias,
                       s, act);
}

void launch_conv_tail(const half_t* in, const float* xin, float* xout, const void* w, const float* bias,
                      const ConvShape& s, int C, int residual_sign, int clamp_out, int num_cus,
                      hipStream_t st) {
  const int grid = s.tiles < num_cus ? s.tiles : num_cus;
  hipLaunchKernelGGL(conv_tail_kernel, dim3(grid), dim3(256), kTailLds, st, in, xin, xout,
                     (const uint4*)w, bias, s, C, residual_sign, clamp_out);
}

}  // namespace pnp
