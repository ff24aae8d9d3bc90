// Split-fp16 ("fp16x3") denoiser body and tail for gfx950: near-fp32 convolutions on the fp16
// MFMA.  Every operand is carried as an fp16 pair, x = x_hi + x_lo with x_hi = fp16(x) and
// x_lo = fp16(x - x_hi) (subnormals kept: the f16 MFMA does not flush them), so activations and
// weights keep ~21-22 significant bits; each product is
//     a * w  ~  a_hi w_hi + a_hi w_lo + a_lo w_hi          (the a_lo w_lo term is below fp32's ulp)
// in one fp32 accumulator: three v_mfma_f32_16x16x32_f16 per fp16 product.
//
// Why: the reference denoiser runs in fp32 (models/denoiser.py:37).  fp16 operands hold PSNR
// within 0.01 dB at the metric (ours-A blur, 32-41 dB) but not at high-PSNR regimes: BASELINE
// config 1 (gray 256^2, Id, 45-50 dB) moves 0.067 dB within 23 iterations, and the Poisson
// method (ours-C) drifts 0.19 dB over 3000 iterations.  CPU emulation of this scheme on config 1
// (tools/precision_emu.py): 6e-5 dB against the fp32 oracle, vs 0.06 dB for fp16 operands.
// The fp32-operand path (conv32.hip, v_mfma_f32_32x32x2_f32, 157 TF peak) does the same job
// at 1/16 of the fp16 MFMA rate; three fp16 MFMAs per product cost 1/3.
//
// Reference: models/basic_models.py:25-38 (simple_CNN.forward), KAIR network_dncnn.py:42-77.
//
// Layout.  Hidden activations are two fp16 NHWC64 images (hi, lo) with the same zero border
// (kActPad) as the fp16 path, 128 B per pixel each.  A workgroup (8 waves, 2 per SIMD, one per
// CU: the LDS holds three halo buffers) is persistent over 8 x 16 output tiles.  A tile's
// 10 x 18 input halo sits in LDS pixel-major, hi then lo (128 B per pixel, 192 pixel slots per
// half), its eight 16-B channel chunks XOR-swizzled per halo column: slot s of pixel (pr, pc)
// holds chunk s ^ f(pc), f(pc) = kS3Swz[pc >> 1].  An LDS-DMA piece (buffer_load ... lds, 16 B
// per lane) then fetches 8 whole 128-B pixel lines (lane l: pixel l >> 3, source chunk
// (l & 7) ^ f), 48 pieces per tile = 6 per wave with the same instruction count, and a B
// fragment of v_mfma_f32_16x16x32_f16 (16 pixels x 32 channels: lane l reads chunk
// 4 hs + (l >> 4) of pixel l & 15) hits 16 distinct bank quads in each of the four lane groups
// of a ds_read_b128 for every tap offset (f was found by exhaustive search; an earlier
// chunk-planar form, 16 B per lane from 64 different lines per piece, ran the tail 1.9x
// slower).  The DMA runs two tiles ahead (3-deep ring).
//
// Body (64 -> 64): wave w owns output channels 16 (w & 3) .. +15 of tile rows 4 (w >> 2) .. +3
// (four N-subtiles of 16 pixels).  Its A fragments, hi and lo, for all 18 K-steps stay in
// registers for the launch (144 VGPRs); per K-step it reads 4 hi + 4 lo B fragments and issues
// 12 MFMAs.  The epilogue adds the bias, applies the activation in fp32 and stores the hi and
// lo halves: lane l holds channels 16 (w & 3) + 4 (l >> 4) .. +3 of one pixel (8 B each).
// Tail (64 -> C, C <= 4): one 16-row M-tile (rows >= C zero), wave w = tile row w; the
// epilogue adds the bias and the fp32 residual, clamps, and writes fp32 NCHW.
#include "kernels.h"

namespace pnp {

namespace {

constexpr int kS3HaloW = kS3TileW + 2;                  // 18
constexpr int kS3HaloPix = (kS3TileH + 2) * kS3HaloW;   // 180
constexpr int kS3Half = 192 * 128;                      // 24576 B: hi (or lo) pixels of a halo, 24 DMA pieces
constexpr int kS3Buf = 2 * kS3Half;                     // 49152 B
constexpr int kS3Lds = 3 * kS3Buf;                      // 147456 B
constexpr int kS3KSteps = 18;                           // 9 taps x 2 channel halves of 32
constexpr int kS3Pieces = 6;                            // DMA pieces per wave per tile (48 / 8)

typedef int v2i_t __attribute__((ext_vector_type(2)));
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));

struct S3Geom {
  int tiles_x, tiles_y, tiles;
};

__device__ __forceinline__ void s3_decode(int t, const S3Geom& g, int& b, int& ty0, int& tx0) {
  const int per = g.tiles_x * g.tiles_y;
  b = t / per;
  const int r = t - b * per;
  const int ty = r / g.tiles_x;
  ty0 = ty * kS3TileH;
  tx0 = (r - ty * g.tiles_x) * kS3TileW;
}

// Tile t -> (b, ty0, tx0) stepped by the grid stride G without divisions (two runtime divisions
// per decode cost ~50 instructions per tile and wave): G's mixed-radix digits are added with
// carries; past the last tile the coordinates stay on it (the clamped DMA of the last tiles).
struct S3Iter {
  int t, b, ty, tx, gb, gty, gtx, tiles, tiles_x, tiles_y;
  __device__ __forceinline__ void init(int t0, int G, const S3Geom& g) {
    t = t0;
    tiles = g.tiles;
    tiles_x = g.tiles_x;
    tiles_y = g.tiles_y;
    const int per = g.tiles_x * g.tiles_y, tc = min(t0, g.tiles - 1);
    b = tc / per;
    ty = (tc - b * per) / g.tiles_x;
    tx = tc - b * per - ty * g.tiles_x;
    gb = G / per;
    gty = (G - gb * per) / g.tiles_x;
    gtx = G - gb * per - gty * g.tiles_x;
  }
  __device__ __forceinline__ void next(int G) {
    t += G;
    if (t >= tiles) return;                              // stays on the last tile
    tx += gtx;
    if (tx >= tiles_x) { tx -= tiles_x; ++ty; }
    ty += gty;
    if (ty >= tiles_y) { ty -= tiles_y; ++b; }
    b += gb;
  }
};

// chunk swizzle of halo column pc: f = {0,1,2,4,5,6,2,6,0}[pc >> 1], 3 bits each
__device__ __forceinline__ int s3_swz(int pc) { return (0x00CB5888u >> (3 * (pc >> 1))) & 7; }

__device__ __forceinline__ int xcd_block_s3(int b, int G) {   // as conv.hip xcd_block
  return (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3);
}

// MODE 0: body 64 -> 64 (hi/lo out).  MODE 1: tail 64 -> C + residual + clamp (fp32 NCHW out).
// Body epilogue (round 3, A/B: cfg4 body 1.650 -> 1.639 ms): the bias is the first MFMA's C
// operand, and the activation's max is one v_max_f32 without the compiler's canonicalizing one.
// C operand of a tile's first MFMA: the bias (body) or zero (the tail adds its own)
template <int MODE>
__device__ __forceinline__ floatx4 s3_c0(const float* bl) {
  if (MODE == 0) return floatx4{bl[0], bl[1], bl[2], bl[3]};
  return floatx4{};
}
// fp16x3 body weights are split at 2^8 times their value (pack_body_weights_s3): the low half
// |w_lo| <= 2^-11 |w| is an fp16 subnormal below |w| = 2^-3 at scale 1 -- most DnCNN weights --,
// so it kept fewer bits (r06: ours-C x 3000 landed 2.2e-3 from the reference where fp32 lands
// 5.3e-5; the CPU emulation of the split, tools/split_scale_emu.py, gives 2.0e-3 at scale 1 and
// 2.5e-4 with the weights scaled).  The bias enters the accumulator scaled too and the
// epilogue multiplies by 2^-8: powers of two, so the hi * hi terms round as at scale 1.
constexpr float kS3WScale = kS3BodyScale, kS3WInv = 1.f / kS3BodyScale;
template <int WLO>
__device__ __forceinline__ float s3_bias_scale() { return WLO ? kS3WScale : 1.f; }

// bias (unless already in the accumulator) + activation in fp32, then the hi / lo fp16 halves;
// the accumulator is first unscaled (WLO: kS3WScale, see above)
template <int ACT, int WLO = 0>
__device__ __forceinline__ void s3_split(float a, float b, h4_t& hi, h4_t& lo, int i) {
  (void)b;                                         // the bias is already in the accumulator
  float v = WLO ? a * kS3WInv : a;
  const float t = ACT == 0 ? v * 0.01f : 0.f;
  asm("v_max_f32 %0, %1, %2" : "=v"(v) : "v"(v), "v"(t));
  const half_t h = (half_t)v;
  hi[i] = h;
  lo[i] = (half_t)(v - (float)h);
}

// WLO = 0 (fp16a2, body only): the a_hi w_lo term is dropped, two MFMAs per product on split
// activations and single fp16 weights (pnp_set_denoiser's filter-sum rounding).  Without the
// w_lo registers a wave holds two M-subtiles (32 output channels) of two tile rows instead of one
// M-subtile of four: a B fragment then feeds two MFMAs, so the LDS reads per K-step and CU halve
// (with one M-subtile per wave the 8 reads of 8 MFMAs per wave fill the LDS array's 256 B/clk
// exactly: r05 measured 2.59 ms per layer at the metric against fp16x3's 3.17, not 2/3 of it).
template <int MODE, int ACT, int WLO = 1>
__global__ __launch_bounds__(512, 1) void conv_s3_kernel(const half_t* __restrict__ in_hi,
                                                          const half_t* __restrict__ in_lo,
                                                          half_t* __restrict__ out_hi, half_t* __restrict__ out_lo,
                                                          const uint4* __restrict__ w_hi,
                                                          const uint4* __restrict__ w_lo,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ xin, float* __restrict__ xout,
                                                          ConvShape s, S3Geom g, int C, int residual_sign,
                                                          int clamp_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool A2 = MODE == 0 && !WLO;
  constexpr int NT = MODE == 0 ? (A2 ? 2 : 4) : 1;      // N-subtiles (tile rows) per wave
  constexpr int MW = A2 ? 2 : 1;                        // 16-row M-subtiles per wave
  constexpr int NM = MODE == 0 ? 4 : 1;                 // 16-row M-tiles of the layer
  constexpr int NWL = WLO ? kS3KSteps : 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mt0 = MODE == 0 ? (A2 ? 2 * (wave & 1) : (wave & 3)) : 0;
  const int row0 = MODE == 0 ? (A2 ? 2 * (wave >> 1) : 4 * (wave >> 2)) : wave;
  const int px = lane & 15, grp = lane >> 4;

  half8_t wH[MW][kS3KSteps], wL[NWL];
#pragma unroll
  for (int ks = 0; ks < kS3KSteps; ++ks) {
#pragma unroll
    for (int m = 0; m < MW; ++m)
      wH[m][ks] = __builtin_bit_cast(half8_t, w_hi[(size_t)(ks * NM + mt0 + m) * 64 + lane]);
    if (WLO) wL[ks % NWL] = __builtin_bit_cast(half8_t, w_lo[(size_t)(ks * NM + mt0) * 64 + lane]);
  }
  float bl[MW][4];
#pragma unroll
  for (int m = 0; m < MW; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = MODE == 0 ? 16 * (mt0 + m) + 4 * grp + i : i;
      bl[m][i] = (MODE == 0 || co < C) ? bias[co] * (MODE == 0 ? s3_bias_scale<WLO>() : 1.f) : 0.f;
    }

  // DMA: piece q = 8 j + wave (j < 6) covers half q / 24 (hi, lo), pixels 8 (q % 24) .. +7 (pixels
  // past 179 re-read pixel 179 into the padding slots)
  unsigned doff[kS3Pieces];
#pragma unroll
  for (int j = 0; j < kS3Pieces; ++j) {
    const int k = (8 * j + wave) % 24;
    const int p = min(8 * k + (lane >> 3), kS3HaloPix - 1);
    const int pr = p / kS3HaloW, pc = p - pr * kS3HaloW;
    doff[j] = (unsigned)(((pr * s.Wp + pc) * kWidth + 8 * ((lane & 7) ^ s3_swz(pc))) * 2);
  }
  __amdgpu_buffer_rsrc_t drh, drl;                     // the tile being fetched: hi / lo images, LDS buffer
  unsigned char* ddst;
  auto dma_at = [&](const S3Iter& ti, int bi) {        // clamped: always kS3Pieces pieces
    const int b = ti.b, ty0 = ti.ty * kS3TileH, tx0 = ti.tx * kS3TileW;
    const size_t base = (((size_t)b * s.Hp + ty0 + s.pad - 1) * s.Wp + tx0 + s.pad - 1) * kWidth;
    drh = __builtin_amdgcn_make_buffer_rsrc((void*)(in_hi + base), (short)0, 0x7fffffff, 0x00020000);
    drl = __builtin_amdgcn_make_buffer_rsrc((void*)(in_lo + base), (short)0, 0x7fffffff, 0x00020000);
    ddst = smem + bi * kS3Buf;
  };
  auto dma_piece = [&](int j) {
    const int q = 8 * j + wave, h = q / 24, k = q - 24 * h;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(h ? drl : drh,
                                             (__attribute__((address_space(3))) void*)(ddst + h * kS3Half + k * 1024),
                                             16, doff[j], 0, 0, 0);
  };
  auto issue = [&](const S3Iter& ti, int bi) {
    dma_at(ti, bi);
#pragma unroll
    for (int j = 0; j < kS3Pieces; ++j) dma_piece(j);
  };

  // per-lane part of the B-fragment addresses: tap column dx, channel half hs
  unsigned lofs[3][2];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int hs = 0; hs < 2; ++hs)
      lofs[dx][hs] = (unsigned)((px + dx) * 128 + 16 * ((4 * hs + grp) ^ s3_swz(px + dx)));
  const int G = gridDim.x;
  int t = xcd_block_s3(blockIdx.x, G);
  S3Iter it, itd;                                       // this tile; the tile two strides ahead (DMA)
  it.init(t, G, g);
  itd.init(t, G, g);
  if (t < g.tiles) {
    issue(itd, 0);
    itd.next(G);
    issue(itd, 1);
    itd.next(G);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // tile t landed
  }
  __syncthreads();
  const unsigned plane = (unsigned)(s.H * s.W);
  int cur = 0;
  // MODE 0 (r06): tile t - 1's epilogue (activation, hi / lo split, 8 stores) runs inside tile t's
  // K-steps 1 .. MW NT, one (M-subtile, row) per K-step, so its VALU and stores issue between
  // MFMAs; at the end of the tile both waves of a SIMD used to sit in the epilogue together.  A
  // workgroup's first tile stores its (empty) predecessor through zero-size buffer resources, so
  // every tile issues 8 stores and the vmcnt at its end stays exact.  Same arithmetic, same bits.
  floatx4 pacc[MODE == 0 ? MW : 1][MODE == 0 ? NT : 1] = {};
  int pb = 0, pty0 = 0, ptx0 = 0;
  bool pv = false;
  auto store_mn = [&](int m, int n) {
    const int y = pty0 + row0 + n;
    h4_t hi, lo;
#pragma unroll
    for (int i = 0; i < 4; ++i) s3_split<ACT, WLO>(pacc[m][n][i], bl[m][i], hi, lo, i);
    const size_t rowb = (((size_t)pb * s.Hp + y + s.pad) * s.Wp + ptx0 + s.pad) * kWidth;
    const int nrec = (pv && y < s.H) ? min(kS3TileW, s.W - ptx0) * 128 : 0;
    const unsigned off = (unsigned)(px * 128 + (16 * (mt0 + m) + 4 * grp) * 2);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i_t, hi),
                                          __builtin_amdgcn_make_buffer_rsrc(out_hi + rowb, (short)0, nrec, 0x00020000),
                                          off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i_t, lo),
                                          __builtin_amdgcn_make_buffer_rsrc(out_lo + rowb, (short)0, nrec, 0x00020000),
                                          off, 0, 0);
  };
  for (; t < g.tiles; t += G) {
    const int b = it.b, ty0 = it.ty * kS3TileH, tx0 = it.tx * kS3TileW;
    it.next(G);
    // tail: the residual input, loaded before this tile's DMA issue (so waiting for it never
    // waits on the DMA); always kMaxC loads (c >= C: zero-size descriptor)
    float xi[MODE == 1 ? kMaxC : 1];
    unsigned toff = 0;
    if constexpr (MODE == 1) {
      const int y = ty0 + row0, x = tx0 + px;
      toff = (lane < 16 && y < s.H && x < s.W) ? (unsigned)(y * s.W + x) * 4u : 0x80000000u;
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(xin + ((size_t)b * C + (c < C ? c : 0)) * plane), (short)0, c < C ? (int)(plane * 4u) : 0,
            0x00020000);
        xi[c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, toff, 0, 0));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // MODE 0 (r06): tile t+2's pieces issue one per K-step after the deferred epilogue's stores,
    // between MFMAs, instead of in a burst before the first MFMA of the tile
    static_assert(MODE != 0 || MW * NT + kS3Pieces < kS3KSteps, "the pieces fit in the K-loop");
    dma_at(itd, cur >= 1 ? cur - 1 : 2);
    if constexpr (MODE != 0) {
#pragma unroll
      for (int j = 0; j < kS3Pieces; ++j) dma_piece(j);
    }
    itd.next(G);
    const unsigned char* fb = smem + cur * kS3Buf + row0 * kS3HaloW * 128;
    auto ldB = [&](int ks, int n, int lo) {
      const int tap = ks >> 1, dy = tap / 3, dx = tap - 3 * dy;
      return *reinterpret_cast<const half8_t*>(fb + lofs[dx][ks & 1] + lo * kS3Half + (n + dy) * kS3HaloW * 128);
    };
    // B fragments are read PD K-steps ahead (the body's 12 MFMAs per K-step cover one step of LDS
    // latency; the tail's 3 do not); per K-step the next reads are interleaved with the MFMAs.
    // (fp16a2 at depth 2, r06: 2.361-2.365 vs 2.356-2.363 ms per layer, no change)
    constexpr int PD = MODE == 0 ? 1 : 3;
    floatx4 acc[MW][NT];
    half8_t bh[PD + 1][NT], bo[PD + 1][NT];
#pragma unroll
    for (int d = 0; d < PD; ++d)
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        bh[d][n] = ldB(d, n, 0);
        bo[d][n] = ldB(d, n, 1);
      }
#pragma unroll
    for (int ks = 0; ks < kS3KSteps; ++ks) {
      const int r = ks % (PD + 1);
      if (ks + PD < kS3KSteps) {
        const int w = (ks + PD) % (PD + 1);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          bh[w][n] = ldB(ks + PD, n, 0);
          bo[w][n] = ldB(ks + PD, n, 1);
        }
      }
#pragma unroll
      for (int m = 0; m < MW; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wH[m][ks], bh[r][n],
                                                             ks == 0 ? s3_c0<MODE>(bl[m]) : acc[m][n], 0, 0, 0);
      if (WLO) {
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[0][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wL[ks % NWL], bh[r][n], acc[0][n], 0, 0, 0);
      }
#pragma unroll
      for (int m = 0; m < MW; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wH[m][ks], bo[r][n], acc[m][n], 0, 0, 0);
      if (ks + PD < kS3KSteps) {
        // fp16x3: one LDS read per MFMA, then NT MFMAs; fp16a2: one read per two MFMAs
#pragma unroll
        for (int i = 0; i < 2 * NT; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, MW, 0);
        }
        if (WLO) __builtin_amdgcn_sched_group_barrier(0x008, NT, 0);
      }
      if constexpr (MODE == 0) {
        if (ks >= 1 && ks <= MW * NT) store_mn((ks - 1) / NT, (ks - 1) % NT);   // tile t - 1's epilogue
        if (ks > MW * NT && ks <= MW * NT + kS3Pieces) dma_piece(ks - MW * NT - 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (MODE == 0) {
#pragma unroll
      for (int m = 0; m < MW; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) pacc[m][n] = acc[m][n];
      pb = b;
      pty0 = ty0;
      ptx0 = tx0;
      pv = true;
      // tile t+1 landed: younger than its DMA are tile t-1's 8 stores and the DMA of t+2 (6)
      static_assert(2 * MW * NT == 8, "the vmcnt below counts 8 stores per tile");
      asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)" ::: "memory");
    } else {
      // lanes 0..15 hold channels 0..3 of pixel (row0, px): D rows 4 (l >> 4) + i
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) {
        const float nc = acc[0][0][c] * kSplitWInv + bl[0][c];   // the tail's split weights are scaled too
        float o = residual_sign > 0 ? nc + xi[c] : xi[c] - nc;
        if (clamp_out) o = fminf(fmaxf(o, 0.f), 1.f);
        __builtin_amdgcn_raw_buffer_store_b32(
            __builtin_bit_cast(int, o),
            __builtin_amdgcn_make_buffer_rsrc((void*)(xout + ((size_t)b * C + (c < C ? c : 0)) * plane), (short)0,
                                              c < C ? (int)(plane * 4u) : 0, 0x00020000),
            toff, 0, 0);
      }
      // tile t+1 landed: younger than its DMA are this tile's 4 loads, the DMA of t+2 and 4 stores
      asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
  if constexpr (MODE == 0) {
    if (pv) {                                           // the last tile's epilogue
#pragma unroll
      for (int m = 0; m < MW; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) store_mn(m, n);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may land after the workgroup ends
}

#define PNP_S3_INST(M, A, WL)                                                                                  \
  template __global__ void conv_s3_kernel<M, A, WL>(const half_t* __restrict__, const half_t* __restrict__,       \
                                                half_t* __restrict__, half_t* __restrict__,                    \
                                                const uint4* __restrict__, const uint4* __restrict__,          \
                                                const float* __restrict__, const float* __restrict__,          \
                                                float* __restrict__, ConvShape, S3Geom, int, int, int);
PNP_S3_INST(0, 0, 1)
PNP_S3_INST(0, 1, 1)
PNP_S3_INST(1, 0, 1)
PNP_S3_INST(0, 0, 0)
PNP_S3_INST(0, 1, 0)
#undef PNP_S3_INST

// ------------------------------------------------------------------------------------
// conv_stack_s3: every body layer of a small batch in ONE launch on split fp16 (the
// conv_stack16 protocol of conv.hip for conv_s3's tiles and fragments): a workgroup keeps its
// 8 x 16 tiles for all layers, layer l + 1 of a tile starts once its 3 x 3 neighbourhood has
// published layer l (common.h tile_wait / tile_publish), and the handed-off hi / lo images are
// written and read at device scope (sc1 stores and sc1 LDS-DMA into the same swizzled
// pixel-major image as conv_s3_kernel's).  4 waves, one per SIMD: wave w owns channels 16 w .. +15 of all 8 tile rows
// (two groups of 4 N-subtiles), the same MFMA chain per output as conv_s3_kernel: bit-identical.
// ------------------------------------------------------------------------------------
constexpr int kS3StkLds = 2 * kS3Buf;                   // 98304 B
constexpr int kS3StkPieces = 12;                        // LDS-DMA pieces per wave per tile (48 / 4)
constexpr int kCpolDev = 16;                            // sc1: device-scope load / store

// WLO = 0: fp16a2 (no w_lo term), bit-identical to conv_s3_kernel<0, ACT, 0> launches.
template <int ACT, int WLO = 1>
__global__ __launch_bounds__(256, 1) void conv_stack_s3_kernel(half_t* __restrict__ aH, half_t* __restrict__ aL,
                                                                half_t* __restrict__ bH, half_t* __restrict__ bL,
                                                                const uint4* __restrict__ w_hi,
                                                                const uint4* __restrict__ w_lo,
                                                                const float* __restrict__ bias, int nbody, ConvShape s,
                                                                S3Geom g, int* __restrict__ done, int epoch,
                                                                int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mt = wave, px = lane & 15, grp = lane >> 4;
  const int G = gridDim.x;
  const int K = (g.tiles - (int)blockIdx.x + G - 1) / G;
  unsigned lofs[3][2];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int hs = 0; hs < 2; ++hs)
      lofs[dx][hs] = (unsigned)((px + dx) * 128 + 16 * ((4 * hs + grp) ^ s3_swz(px + dx)));

  // DMA: piece q = 4 j + wave (j < 12) covers half q / 24, pixels 8 (q % 24) .. +7 (as conv_s3_kernel)
  unsigned doff[kS3StkPieces];
#pragma unroll
  for (int j = 0; j < kS3StkPieces; ++j) {
    const int kk = (4 * j + wave) % 24;
    const int p = min(8 * kk + (lane >> 3), kS3HaloPix - 1);
    const int pr = p / kS3HaloW, pc = p - pr * kS3HaloW;
    doff[j] = (unsigned)(((pr * s.Wp + pc) * kWidth + 8 * ((lane & 7) ^ s3_swz(pc))) * 2);
  }
  constexpr int NWL = WLO ? kS3KSteps : 1;
  half8_t wH[kS3KSteps], wL[NWL];
  float bl[4];
  auto load_w = [&](int l) {
#pragma unroll
    for (int ks = 0; ks < kS3KSteps; ++ks) {
      const size_t o = (size_t)l * (kBodyWBytes / 16) + (size_t)(ks * 4 + mt) * 64 + lane;
      wH[ks] = __builtin_bit_cast(half8_t, w_hi[o]);
      if (WLO) wL[ks % NWL] = __builtin_bit_cast(half8_t, w_lo[o]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) bl[i] = bias[l * kWidth + 16 * mt + 4 * grp + i] * s3_bias_scale<WLO>();
  };
  load_w(0);
  for (int l = 0; l < nbody; ++l) {
    const half_t* inH = (l & 1) ? bH : aH;
    const half_t* inL = (l & 1) ? bL : aL;
    half_t* outH = (l & 1) ? aH : bH;
    half_t* outL = (l & 1) ? aL : bL;
    for (int k = 0; k < K; ++k) {
      const int t = (int)blockIdx.x + k * G;
      int b, ty0, tx0;
      s3_decode(t, g, b, ty0, tx0);
      if (l > 0) {
        if (wave == 0) {
          const int ny = ty0 / kS3TileH + lane / 3 - 1, nx = tx0 / kS3TileW + lane % 3 - 1;
          const bool want = lane < 9 && ny >= 0 && ny < g.tiles_y && nx >= 0 && nx < g.tiles_x;
          tile_wait(done, want ? (b * g.tiles_y + ny) * g.tiles_x + nx : 0, want, epoch + l, err);
        }
        __syncthreads();
      }
      unsigned char* hb = smem + (k & 1) * kS3Buf;
      {                                       // halo (hi, lo): device-scope (sc1) LDS-DMA, 12 pieces per wave
        const size_t base = (((size_t)b * s.Hp + ty0 + s.pad - 1) * s.Wp + tx0 + s.pad - 1) * kWidth;
        const __amdgpu_buffer_rsrc_t rh =
            __builtin_amdgcn_make_buffer_rsrc((void*)(inH + base), (short)0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rl =
            __builtin_amdgcn_make_buffer_rsrc((void*)(inL + base), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int j = 0; j < kS3StkPieces; ++j) {
          const int q = 4 * j + wave, h = q / 24, kk = q - 24 * h;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(h ? rl : rh,
                                                   (__attribute__((address_space(3))) void*)(hb + h * kS3Half + kk * 1024),
                                                   16, doff[j], 0, 0, kCpolDev);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
#pragma unroll
      for (int gq = 0; gq < 2; ++gq) {        // tile rows 4 gq .. +3
        const unsigned char* fb = hb + 4 * gq * kS3HaloW * 128;
        auto ldB = [&](int ks, int n, int lo) {
          const int tap = ks >> 1, dy = tap / 3, dx = tap - 3 * dy;
          return *reinterpret_cast<const half8_t*>(fb + lofs[dx][ks & 1] + lo * kS3Half + (n + dy) * kS3HaloW * 128);
        };
        floatx4 acc[4];
        half8_t bh[2][4], bo[2][4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          bh[0][n] = ldB(0, n, 0);
          bo[0][n] = ldB(0, n, 1);
        }
#pragma unroll
        for (int ks = 0; ks < kS3KSteps; ++ks) {
          const int r = ks & 1;
          if (ks + 1 < kS3KSteps) {
#pragma unroll
            for (int n = 0; n < 4; ++n) {
              bh[r ^ 1][n] = ldB(ks + 1, n, 0);
              bo[r ^ 1][n] = ldB(ks + 1, n, 1);
            }
          }
#pragma unroll
          for (int n = 0; n < 4; ++n)
            acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wH[ks], bh[r][n], ks == 0 ? s3_c0<0>(bl) : acc[n], 0, 0, 0);
          if (WLO) {
#pragma unroll
            for (int n = 0; n < 4; ++n)
              acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wL[ks % NWL], bh[r][n], acc[n], 0, 0, 0);
          }
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wH[ks], bo[r][n], acc[n], 0, 0, 0);
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int y = ty0 + 4 * gq + n;
          h4_t hi, lo;
#pragma unroll
          for (int i = 0; i < 4; ++i) s3_split<ACT, WLO>(acc[n][i], bl[i], hi, lo, i);
          const size_t rowb = (((size_t)b * s.Hp + y + s.pad) * s.Wp + tx0 + s.pad) * kWidth;
          const int nrec = y < s.H ? min(kS3TileW, s.W - tx0) * 128 : 0;
          const unsigned off = (unsigned)(px * 128 + (16 * mt + 4 * grp) * 2);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i_t, hi),
                                                __builtin_amdgcn_make_buffer_rsrc(outH + rowb, (short)0, nrec, 0x00020000),
                                                off, 0, kCpolDev);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i_t, lo),
                                                __builtin_amdgcn_make_buffer_rsrc(outL + rowb, (short)0, nrec, 0x00020000),
                                                off, 0, kCpolDev);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) tile_publish(done + t, epoch + l + 1);
    }
    if (l + 1 < nbody) load_w(l + 1);
  }
}

#define PNP_STK_INST(A, WL)                                                                                     \
  template __global__ void conv_stack_s3_kernel<A, WL>(half_t* __restrict__, half_t* __restrict__,              \
                                                       half_t* __restrict__, half_t* __restrict__,              \
                                                       const uint4* __restrict__, const uint4* __restrict__,    \
                                                       const float* __restrict__, int, ConvShape, S3Geom,       \
                                                       int* __restrict__, int, int* __restrict__);
PNP_STK_INST(0, 1)
PNP_STK_INST(1, 1)
PNP_STK_INST(0, 0)
PNP_STK_INST(1, 0)
#undef PNP_STK_INST

S3Geom s3_geom(const ConvShape& s) {
  S3Geom g;
  g.tiles_x = (s.W + kS3TileW - 1) / kS3TileW;
  g.tiles_y = (s.H + kS3TileH - 1) / kS3TileH;
  g.tiles = s.B * g.tiles_x * g.tiles_y;
  return g;
}

inline uint16_t f16_bits(float f) {
  _Float16 h = (_Float16)f;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

}  // namespace

hipError_t conv_s3_kernels_init() {
  for (const void* k : {(const void*)conv_s3_kernel<0, 0, 1>, (const void*)conv_s3_kernel<0, 1, 1>,
                        (const void*)conv_s3_kernel<1, 0, 1>, (const void*)conv_s3_kernel<0, 0, 0>,
                        (const void*)conv_s3_kernel<0, 1, 0>}) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kS3Lds);
    if (e != hipSuccess) return e;
  }
  for (const void* k : {(const void*)conv_stack_s3_kernel<0, 1>, (const void*)conv_stack_s3_kernel<1, 1>,
                        (const void*)conv_stack_s3_kernel<0, 0>, (const void*)conv_stack_s3_kernel<1, 0>}) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kS3StkLds);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// W: [64][64][3][3] fp32 -> hi / lo fragments [18 ks][4 M-tiles][64 lanes][8] fp16: lane l holds
// A[row l & 15][k = 8 (l >> 4) .. +7], row r of M-tile mt = output channel 16 mt + r, k-step ks =
// tap ks >> 1, input channels 32 (ks & 1) + k.  hi = fp16(w), lo = fp16(w - hi).
void pack_body_weights_s3(const float* W, uint16_t* hi, uint16_t* lo, float scale) {
  for (int ks = 0; ks < kS3KSteps; ++ks) {
    const int tap = ks >> 1, ky = tap / 3, kx = tap % 3;
    for (int mt = 0; mt < 4; ++mt)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int co = 16 * mt + (l & 15), ci = 32 * (ks & 1) + 8 * (l >> 4) + j;
          const float w = W[((co * 64 + ci) * 3 + ky) * 3 + kx] * scale;   // exact: a power of two
          const float h = (float)(_Float16)w;
          const size_t o = (((size_t)ks * 4 + mt) * 64 + l) * 8 + j;
          hi[o] = f16_bits(w);
          lo[o] = f16_bits(w - h);
        }
  }
}

void launch_conv_s3_body(const half_t* in_hi, const half_t* in_lo, half_t* out_hi, half_t* out_lo, const void* w_hi,
                         const void* w_lo, const float* bias, const ConvShape& s, int act, int num_cus,
                         hipStream_t st) {
  const S3Geom g = s3_geom(s);
  const int grid = g.tiles < num_cus ? g.tiles : num_cus;
#define S3B(A, WL)                                                                                           \
  hipLaunchKernelGGL((conv_s3_kernel<0, A, WL>), dim3(grid), dim3(512), kS3Lds, st, in_hi, in_lo, out_hi, out_lo, \
                     (const uint4*)w_hi, (const uint4*)w_lo, bias, nullptr, nullptr, s, g, kWidth, 1, 0)
  if (w_lo) {
    if (act == 0) S3B(0, 1);
    else S3B(1, 1);
  } else {                                          // fp16a2: no w_lo term
    if (act == 0) S3B(0, 0);
    else S3B(1, 0);
  }
#undef S3B
}

void launch_conv_s3_tail(const half_t* in_hi, const half_t* in_lo, const float* xin, float* xout, const void* w_hi,
                         const void* w_lo, const float* bias, const ConvShape& s, int C, int residual_sign,
                         int clamp_out, int num_cus, hipStream_t st) {
  const S3Geom g = s3_geom(s);
  const int grid = g.tiles < num_cus ? g.tiles : num_cus;
  hipLaunchKernelGGL((conv_s3_kernel<1, 0>), dim3(grid), dim3(512), kS3Lds, st, in_hi, in_lo, nullptr, nullptr,
                     (const uint4*)w_hi, (const uint4*)w_lo, bias, xin, xout, s, g, C, residual_sign, clamp_out);
}

int s3_tiles(const ConvShape& s) { return s3_geom(s).tiles; }

void launch_conv_stack_s3(half_t* aH, half_t* aL, half_t* bH, half_t* bL, const void* w_hi, const void* w_lo,
                          const float* bias, int nbody, const ConvShape& s, int act, int num_cus, int* done, int epoch,
                          int* err, hipStream_t st) {
  const S3Geom g = s3_geom(s);
  const int grid = g.tiles < num_cus ? g.tiles : num_cus;
  auto k = w_lo ? (act == 0 ? conv_stack_s3_kernel<0, 1> : conv_stack_s3_kernel<1, 1>)
                : (act == 0 ? conv_stack_s3_kernel<0, 0> : conv_stack_s3_kernel<1, 0>);   // no w_lo: fp16a2
  (void)persistent_launch(k, grid, 256, kS3StkLds, st, aH, aL, bH, bL, (const uint4*)w_hi, (const uint4*)w_lo, bias, nbody,
                          s, g, done, epoch, err);
}

}  // namespace pnp
