// Blur passes K1 / K2 (operators.py:7-38 inside iteration.py:50-51) with the stencil on the
// matrix cores (round 3).
//
// The periodic blur of one channel plane is, tap column by tap column, a Toeplitz product: for
// tap column ox, out[i][j] += sum_oy w(oy, ox) x[i + oy][j + ox].  Over a block of 16 output rows
// the sum over oy is a band matrix (its 17 diagonals: the taps' rows -rt .. rb, rt + rb <= 16)
// applied to 32 input rows, so per (tap column, 16 x 16 output block) one v_mfma_f32_16x16x32_f16
// does it: A = the input values (M = 16 output columns, K = 32 input rows), B = the band (K = 32
// input rows, N = 16 output rows), C = the output block transposed (lane l: output row l & 15,
// columns 4 (l >> 4) .. +3, one float4).  blur_1.mat's 109 taps (17 rows x 9 columns) take 9
// MFMAs per block, 2.6x the useful MACs.
//
// Precision: every operand is split into fp16 halves (v = hi + lo, hi = fp16(v), lo = fp16(v -
// hi), ~22 significant bits) and each product is hi*hi + lo*hi + hi*lo in one fp32 accumulator
// (3 MFMAs; lo*lo is below fp32's rounding).  Both sides are scaled by powers of two first so the
// halves stay inside fp16's range: the taps by 2^eh (host, max |w| < 2^15), the data by 2^ed per
// block (max |v| of the block's halo < 2^15).  The result is scaled back exactly.  Absolute error
// ~3e-7 for unit-range images (numpy emulation: tools/blur_mf_emu.py), as the reference's fp32
// FFT; the solver-level comparison with the fp32 VALU stencils is tests/test_gpu_blur_mf.py.
//
// Tile: 64 x 64 outputs of one plane per 256-thread block; wave w computes rows 16w .. 16w+15 x 4
// column blocks.  The halo (80 input rows x 64 + columns - 1) sits in LDS transposed (column-major:
// the 8 consecutive input rows of an A fragment are 16 contiguous bytes) as fp16 hi and lo planes
// with an 88-half (176-B) column pitch: the 16 columns a ds_read_b128 lane group reads are 11 x
// 16 B apart modulo 256 B, 16 distinct bank quads.  The band fragments (tap columns x hi / lo, 8
// VGPRs per tap column) stay in registers.
#include "common.h"
#include "kernels.h"

#include <cmath>
#include <type_traits>
#include <vector>

namespace pnp {

constexpr int kMfT = 64;                              // output tile (rows and columns)
constexpr int kMfRows = 80;                           // input rows i0 - rt .. i0 - rt + 79
constexpr int kMfMaxCols = 80;                        // input columns (64 + tap columns - 1 <= 76 used)
constexpr int kMfPitch = 88;                          // halves per LDS column
constexpr int kMfPlane = (kMfT + kMfMaxTapCols - 1) * kMfPitch;   // halves per plane (hi, lo)
constexpr int kMfPairs = (kMfRows / 2 + 2) / 3;       // 14 row pairs per fill thread (3 threads per column)

typedef float f4v_t __attribute__((ext_vector_type(4)));
#ifndef MF_BEARLY
#define MF_BEARLY 1   // A/B builds: K1's band fragments loaded before the fill (1) or after it (0)
#endif

// Band fragments of tap column c (c < nc <= NCM): hi in bh[c], lo in bl[c]; columns >= nc zero.
// NCM is the compile-time bucket of the kernel's tap-column count (registers: 8 per column).
template <int NCM>
struct MfB {
  half8_t bh[NCM], bl[NCM];
  __device__ __forceinline__ void load(const uint4* __restrict__ tab, int nc, int lane) {
#pragma unroll
    for (int c = 0; c < NCM; ++c) {
      if (c < nc) {
        bh[c] = __builtin_bit_cast(half8_t, tab[(2 * c + 0) * 64 + lane]);
        bl[c] = __builtin_bit_cast(half8_t, tab[(2 * c + 1) * 64 + lane]);
      } else {
        bh[c] = half8_t{};
        bl[c] = half8_t{};
      }
    }
  }
};

// Wrap once, then clamp: rows / columns that need a second wrap are only read by zero taps or
// feed outputs outside the image (rb_gather's rule).
__device__ __forceinline__ int wrap1(int g, int n) {
  g += g < 0 ? n : 0;
  g -= g >= n ? n : 0;
  return min(max(g, 0), n - 1);
}

// Fill geometry: thread t < 240 owns halo column t % 80 (if < ncols) and row pairs
// 2 (t / 80 + 3 k), k < kMfPairs: consecutive threads read consecutive columns of a row.
struct MfFill {
  int col, p0, gj;
  bool on;
  __device__ __forceinline__ void init(int j0, int cl, int ncols, int W) {
    const int t = threadIdx.x;
    col = t % kMfMaxCols;
    p0 = t / kMfMaxCols;
    on = t < 3 * kMfMaxCols && col < ncols;
    gj = wrap1(j0 - cl + col, W);
  }
  __device__ __forceinline__ int row(int k, int h) const { return 2 * (p0 + 3 * k) + h; }   // h: 0 / 1 of the pair
  __device__ __forceinline__ bool has(int k) const { return on && p0 + 3 * k < kMfRows / 2; }
};

// Block max of |v| over the 256 threads -> the data scale exponent ed: max * 2^ed < 2^15.
__device__ __forceinline__ int mf_scale_exp(float m, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  if (!(m > 0.f) || !(m < __builtin_inff())) return 0;   // all zero (or not finite: garbage in, garbage out)
  int e;
  (void)frexpf(m, &e);                                   // m < 2^e
  return 15 - e;
}

// The fill's values (pairs of rows of one column), scaled by 2^ed, split into the hi / lo planes.
__device__ __forceinline__ void mf_store_split(half_t* __restrict__ hs, const MfFill& f, const float (&v)[kMfPairs][2],
                                               int ed) {
  const float sc = ldexpf(1.f, ed);
#pragma unroll
  for (int k = 0; k < kMfPairs; ++k) {
    if (f.has(k)) {
      half_t h[2], l[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float vs = v[k][q] * sc;
        h[q] = (half_t)vs;
        l[q] = (half_t)(vs - (float)h[q]);
      }
      const int o = f.col * kMfPitch + f.row(k, 0);
      *reinterpret_cast<uint32_t*>(hs + o) =
          (uint32_t)__builtin_bit_cast(uint16_t, h[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, h[1]) << 16);
      *reinterpret_cast<uint32_t*>(hs + kMfPlane + o) =
          (uint32_t)__builtin_bit_cast(uint16_t, l[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, l[1]) << 16);
    }
  }
}

// The tile's MFMA stream: acc[cb] = output rows 16 wave + (lane & 15), columns 16 cb + 4 (lane >> 4) ..
template <int NCM>
__device__ __forceinline__ void mf_stencil(const half_t* __restrict__ hs, const MfB<NCM>& Bt, int nc, int wave,
                                           int lane, floatx4 (&acc)[4]) {
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = floatx4{};
  const half_t* base = hs + (lane & 15) * kMfPitch + 16 * wave + 8 * (lane >> 4);
#pragma unroll
  for (int c = 0; c < NCM; ++c) {
    if (c < nc) {                                          // wave-uniform
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const half8_t ah = *reinterpret_cast<const half8_t*>(base + (16 * cb + c) * kMfPitch);
        const half8_t al = *reinterpret_cast<const half8_t*>(base + kMfPlane + (16 * cb + c) * kMfPitch);
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, Bt.bh[c], acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, Bt.bl[c], acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, Bt.bh[c], acc[cb], 0, 0, 0);
      }
    }
  }
}

// float4 of row i, columns j .. j+3 (nv valid; vec = all 4 valid and 16-B aligned)
__device__ __forceinline__ f4v_t ld4(const float* __restrict__ p, size_t idx, int nv, bool vec) {
  if (vec) return __builtin_nontemporal_load(reinterpret_cast<const f4v_t*>(p + idx));
  f4v_t v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < nv) v[q] = p[idx + q];
  return v;
}
__device__ __forceinline__ void st4(float* __restrict__ p, size_t idx, const f4v_t& v, int nv, bool vec) {
  if (vec) {
    __builtin_nontemporal_store(v, reinterpret_cast<f4v_t*>(p + idx));
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < nv) p[idx + q] = v[q];
}

// K1: u = [clamp](x - g1 Phi^T y) -> u32; B (MB): w = s - g1 y.  Block = one (plane, 64 x 64 tile).
template <int NCM, bool MB>
__global__ __launch_bounds__(256, 4) void k1_blur_mf(const float* __restrict__ x, const float* __restrict__ y,
                                                     const float* __restrict__ s, float* __restrict__ u32,
                                                     float* __restrict__ w, const uint4* __restrict__ btab, int nc,
                                                     int rt, int cl, int eh, int H, int W, int tiles_x, int tiles,
                                                     float gamma1, int clamp_in) {
  __shared__ __attribute__((aligned(16))) half_t hs[2 * kMfPlane];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bc = blockIdx.x / tiles, tile = blockIdx.x - bc * tiles;
  const int ty = tile / tiles_x, i0 = ty * kMfT, j0 = (tile - ty * tiles_x) * kMfT;
  const size_t pb = (size_t)bc * H * W;
  MfFill f;
  f.init(j0, cl, kMfT + nc - 1, W);
  MfB<NCM> Bt;
  if (MF_BEARLY) Bt.load(btab, nc, lane);
  float v[kMfPairs][2];
  float m = 0.f;
  {
    const float* yp = y + pb + f.gj;
#pragma unroll
    for (int k = 0; k < kMfPairs; ++k)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        v[k][q] = f.has(k) ? yp[(size_t)wrap1(i0 - rt + f.row(k, q), H) * W] : 0.f;
        m = fmaxf(m, fabsf(v[k][q]));
      }
  }
  const int ed = mf_scale_exp(m, red);
  mf_store_split(hs, f, v, ed);
  if (!MF_BEARLY) Bt.load(btab, nc, lane);
  // the epilogue's x, in flight during the stencil
  const int i = i0 + 16 * wave + (lane & 15);
  const bool al4 = (W & 3) == 0;
  f4v_t xv[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int j = j0 + 16 * cb + 4 * (lane >> 4);
    const int nv = i < H && j < W ? min(4, W - j) : 0;
    xv[cb] = ld4(x, pb + (size_t)min(i, H - 1) * W + j, nv, al4 && nv == 4);
  }
  __syncthreads();
  floatx4 acc[4];
  mf_stencil(hs, Bt, nc, wave, lane, acc);
  const float sc = ldexpf(1.f, -(ed + eh));
  if (i >= H) return;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int j = j0 + 16 * cb + 4 * (lane >> 4);
    const int nv = j < W ? min(4, W - j) : 0;
    if (nv == 0) continue;
    const bool vec = al4 && nv == 4;
    const size_t idx = pb + (size_t)i * W + j;
    f4v_t uo;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float uu = xv[cb][q] - gamma1 * (acc[cb][q] * sc);
      if (clamp_in) uu = fminf(fmaxf(uu, 0.f), 1.f);
      uo[q] = uu;
    }
    st4(u32, idx, uo, nv, vec);
    if (MB) {
      const f4v_t sv = ld4(s, idx, nv, vec), yv = ld4(y, idx, nv, vec);
      f4v_t wo;
#pragma unroll
      for (int q = 0; q < 4; ++q) wo[q] = sv[q] - gamma1 * yv[q];
      st4(w, idx, wo, nv, vec);
    }
  }
}

// K2: v = y + g2 (Phi(2x+ - x) [+ 2 s+ - s]), s+ = shrink(w, theta) (B), the GKL prox (C), and
// the per-cell partial sums, as ops.hip k2_blur_rb (same outputs, same partials layout): d2 per
// 32 x 32 cell, e2 / n2 / t2 (c_n and PSNR sums, iteration.py:187-188) of the tile in its first
// cell, from the fill's own loads of xn / xo (x_true loaded for the tile's pixels only), and the
// tile's (min, max) of x+ for SSIM's data_range.
template <int NCM, int METHOD>
__global__ __launch_bounds__(256, 4) void k2_blur_mf(const float* __restrict__ xn, const float* __restrict__ xo,
                                                     float* __restrict__ y, const float* __restrict__ xobs,
                                                     const float* __restrict__ xtrue, float* __restrict__ s,
                                                     const float* __restrict__ w, const float* __restrict__ theta,
                                                     double* __restrict__ partials, const uint4* __restrict__ btab,
                                                     int nc, int rt, int cl, int eh, int C, int H, int W,
                                                     int tiles_x, int tiles, int cells_x, int cells, double gamma2,
                                                     double inv_g2, double gkl_gamma, double gkl_alpha, int record,
                                                     float* __restrict__ mm) {
  __shared__ __attribute__((aligned(16))) half_t hs[2 * kMfPlane];
  __shared__ float red[4];
  __shared__ double redm[4][3];
  __shared__ float redr[4][2];
  __shared__ double redd[4][2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bc = blockIdx.x / tiles, tile = blockIdx.x - bc * tiles, b = bc / C, c = bc - b * C;
  const int ty = tile / tiles_x, i0 = ty * kMfT, j0 = (tile - ty * tiles_x) * kMfT;
  const size_t pb = (size_t)bc * H * W;
  MfFill f;
  f.init(j0, cl, kMfT + nc - 1, W);
  MfB<NCM> Bt;                                      // (loaded after the fill: 168 B of spills before it)
  const int ie = min(i0 + kMfT, H), je = min(j0 + kMfT, W);
  float v[kMfPairs][2];
  float m = 0.f;
  {
    double e2 = 0, n2 = 0, t2 = 0;
    float lo = __builtin_inff(), hi = -__builtin_inff();
    const float* xnp = xn + pb + f.gj;
    const float* xop = xo + pb + f.gj;
    const float* xtp = xtrue ? xtrue + pb + f.gj : nullptr;
    const int uj = j0 - cl + f.col;                        // unwrapped column
    const bool cin = uj >= j0 && uj < je;
#pragma unroll
    for (int k = 0; k < kMfPairs; ++k)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ui = i0 - rt + f.row(k, q);              // unwrapped row
        const size_t go = (size_t)wrap1(ui, H) * W;
        float a = 0.f, bo = 0.f;
        if (f.has(k)) {
          a = xnp[go];
          bo = xop[go];
        }
        v[k][q] = 2.f * a - bo;
        m = fmaxf(m, fabsf(v[k][q]));
        if (record && f.has(k) && cin && ui >= i0 && ui < ie) {
          const float d = a - bo;
          e2 += (double)(d * d);
          n2 += (double)(bo * bo);
          if (xtp) {
            const float tt = xtp[go] - a;
            t2 += (double)(tt * tt);
          }
          lo = fminf(lo, a);                     // x+ range for SSIM's data_range (utils_eval.py:11)
          hi = fmaxf(hi, a);
        }
      }
    if (record) {
      e2 = wave_sum(e2);
      n2 = wave_sum(n2);
      t2 = wave_sum(t2);
      if (lane == 0) { redm[wave][0] = e2; redm[wave][1] = n2; redm[wave][2] = t2; }
      if (mm) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          lo = fminf(lo, __shfl_xor(lo, o, 64));
          hi = fmaxf(hi, __shfl_xor(hi, o, 64));
        }
        if (lane == 0) { redr[wave][0] = lo; redr[wave][1] = hi; }
      }
    }
  }
  const int ed = mf_scale_exp(m, red);              // (its barrier also publishes redm / redr)
  if (record && mm && tid == 0) {                   // per (image, channel, tile): [B][C * tiles][2]
    const size_t chunk = (size_t)b * C * tiles + (size_t)c * tiles + tile;
    mm[chunk * 2 + 0] = fminf(fminf(redr[0][0], redr[1][0]), fminf(redr[2][0], redr[3][0]));
    mm[chunk * 2 + 1] = fmaxf(fmaxf(redr[0][1], redr[1][1]), fmaxf(redr[2][1], redr[3][1]));
  }
  mf_store_split(hs, f, v, ed);
  Bt.load(btab, nc, lane);
  __syncthreads();
  floatx4 acc[4];
  mf_stencil(hs, Bt, nc, wave, lane, acc);
  const double sc = ldexp(1.0, -(ed + eh));
  const int i = i0 + 16 * wave + (lane & 15);
  const float th = METHOD == M_B ? theta[b] : 0.f;
  const bool al4 = (W & 3) == 0;
  double d2c[2] = {0.0, 0.0};                       // this lane's d2 in the tile's cell columns 0 / 1
  if (i < H) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int j = j0 + 16 * cb + 4 * (lane >> 4);
      const int nv = j < W ? min(4, W - j) : 0;
      if (nv == 0) continue;
      const bool vec = al4 && nv == 4;
      const size_t idx = pb + (size_t)i * W + j;
      const f4v_t yv = ld4(y, idx, nv, vec), bv = ld4(xobs, idx, nv, vec);
      f4v_t sv = {}, wv = {};
      if (METHOD == M_B) {
        sv = ld4(s, idx, nv, vec);
        wv = ld4(w, idx, nv, vec);
      }
      f4v_t yo = yv, so = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= nv) break;
        double gv = (double)(float)((double)acc[cb][q] * sc);   // Phi(2x+ - x) in fp32, as the VALU stencil
        if (METHOD == M_B) {
          const float wq = wv[q];
          const float sp = copysignf(fmaxf(fabsf(wq) - th, 0.f), wq);   // operators.py:98
          gv += 2.0 * (double)sp - (double)sv[q];
          so[q] = sp;
        }
        const double vv = (double)yv[q] + gamma2 * gv;
        const double ob = bv[q];
        if (METHOD == M_C) {
          const double tt = vv * inv_g2 - gkl_gamma * gkl_alpha;
          const double p = 0.5 * (tt + sqrt(tt * tt + 4.0 * gkl_gamma * ob));
          yo[q] = (float)(vv - gamma2 * p);
        } else {
          yo[q] = (float)vv;
          const double dd = vv * inv_g2 - ob;
          d2c[cb >> 1] += dd * dd;
        }
      }
      st4(y, idx, yo, nv, vec);
      if (METHOD == M_B) st4(s, idx, so, nv, vec);
    }
  }
  // d2: cell (cy, cx) = rows 32 cy .. (waves 2 cy, 2 cy + 1), columns 32 cx .. (blocks 2 cx, 2 cx + 1)
  d2c[0] = wave_sum(d2c[0]);
  d2c[1] = wave_sum(d2c[1]);
  if (lane == 0) { redd[wave][0] = d2c[0]; redd[wave][1] = d2c[1]; }
  __syncthreads();
  if (tid < 16) {                                   // 2 x 2 cells x 4 sums
    const int cell = tid >> 2, k = tid & 3, cy = cell >> 1, cx = cell & 1;
    const int gy = i0 / 32 + cy, gx = j0 / 32 + cx;
    double val = 0.0;
    if (k == 0) val = redd[2 * cy][cx] + redd[2 * cy + 1][cx];
    else if (record && cell == 0) val = ((redm[0][k - 1] + redm[1][k - 1]) + redm[2][k - 1]) + redm[3][k - 1];
    if (gy * 32 < H && gx < cells_x)
      partials[(((size_t)b * cells + (size_t)gy * cells_x + gx) * C + c) * 4 + k] = val;
  }
}

// ---- host ------------------------------------------------------------------------------
// Band tables for one tap list (oy, ox, float bits of w): [tap column c][hi, lo][64 lanes][8 x f16];
// lane l, element t: B[k][n] with k = 8 (l >> 4) + t (input row - output row + rt), n = l & 15.
bool build_mf_taps(const int4* taps, int ntaps, std::vector<uint16_t>& tab, MfTapsHost& o) {
  int oy0 = 1 << 20, oy1 = -(1 << 20), ox0 = 1 << 20, ox1 = -(1 << 20);
  float wmax = 0.f;
  for (int t = 0; t < ntaps; ++t) {
    float wv;
    memcpy(&wv, &taps[t].z, 4);
    if (wv == 0.f) continue;
    oy0 = std::min(oy0, taps[t].x);
    oy1 = std::max(oy1, taps[t].x);
    ox0 = std::min(ox0, taps[t].y);
    ox1 = std::max(ox1, taps[t].y);
    wmax = std::max(wmax, std::fabs(wv));
  }
  if (wmax == 0.f || !std::isfinite(wmax)) return false;
  const int nc = ox1 - ox0 + 1, rspan = oy1 - oy0;
  if (nc > kMfMaxTapCols || rspan > 16) return false;
  int e;
  (void)std::frexp(wmax, &e);
  o.eh = 15 - e;
  o.nc = nc;
  o.rt = -oy0;
  o.cl = -ox0;
  std::vector<float> dense((size_t)nc * 17, 0.f);   // [ox - ox0][oy - oy0]
  for (int t = 0; t < ntaps; ++t) {
    float wv;
    memcpy(&wv, &taps[t].z, 4);
    if (wv != 0.f) dense[(size_t)(taps[t].y - ox0) * 17 + (taps[t].x - oy0)] += wv;
  }
  tab.assign((size_t)nc * 2 * 64 * 8, 0);
  for (int c = 0; c < nc; ++c)
    for (int l = 0; l < 64; ++l)
      for (int t = 0; t < 8; ++t) {
        const int n = l & 15, k = 8 * (l >> 4) + t, dy = k - n;   // oy = dy - rt
        const float wv = (dy >= 0 && dy <= rspan) ? dense[(size_t)c * 17 + dy] : 0.f;
        const float ws = std::ldexp(wv, o.eh);
        const _Float16 h = (_Float16)ws, lo = (_Float16)(ws - (float)h);
        uint16_t hb, lb;
        memcpy(&hb, &h, 2);
        memcpy(&lb, &lo, 2);
        tab[(((size_t)c * 2 + 0) * 64 + l) * 8 + t] = hb;
        tab[(((size_t)c * 2 + 1) * 64 + l) * 8 + t] = lb;
      }
  return true;
}

bool mf_usable(const MfTaps& t, int H, int W) { return t.a && H >= 17 && W >= 17; }

// tap-column buckets: blur_1.mat has 9
template <class F>
static void mf_bucket(int nc, F&& f) {
  if (nc <= 5) f(std::integral_constant<int, 5>{});
  else if (nc <= 9) f(std::integral_constant<int, 9>{});
  else f(std::integral_constant<int, 13>{});
}

void launch_k1_mf(hipStream_t st, const float* x, const float* y, const float* s, float* u32, float* w,
                  const MfTaps& t, int B, int C, int H, int W, float gamma1, int clamp_in, int method_b) {
  const int tx = (W + kMfT - 1) / kMfT, tiles = tx * ((H + kMfT - 1) / kMfT);
  const dim3 grid(B * C * tiles);
  mf_bucket(t.nc, [&](auto ncm) {
    constexpr int N = decltype(ncm)::value;
    if (method_b)
      hipLaunchKernelGGL((k1_blur_mf<N, true>), grid, dim3(256), 0, st, x, y, s, u32, w, (const uint4*)t.a, t.nc,
                         t.rt, t.cl, t.eh, H, W, tx, tiles, gamma1, clamp_in);
    else
      hipLaunchKernelGGL((k1_blur_mf<N, false>), grid, dim3(256), 0, st, x, y, s, u32, w, (const uint4*)t.a, t.nc,
                         t.rt, t.cl, t.eh, H, W, tx, tiles, gamma1, clamp_in);
  });
}

void launch_k2_mf(int method, hipStream_t st, const float* xn, const float* xo, float* y, const float* xobs,
                  const float* xtrue, float* s, const float* w, const float* theta, double* partials,
                  const MfTaps& t, int B, int C, int H, int W, int cells_x, int cells, double gamma2,
                  double gkl_gamma, double gkl_alpha, int record, float* mm) {
  const int tx = (W + kMfT - 1) / kMfT, tiles = tx * ((H + kMfT - 1) / kMfT);
  const dim3 grid(B * C * tiles);
  mf_bucket(t.nc, [&](auto ncm) {
    constexpr int N = decltype(ncm)::value;
#define K2MF_ARGS xn, xo, y, xobs, xtrue, s, w, theta, partials, (const uint4*)t.a, t.nc, t.rt, t.cl, t.eh, C, H, W, \
                  tx, tiles, cells_x, cells, gamma2, 1.0 / gamma2, gkl_gamma, gkl_alpha, record, mm
    if (method == M_A) hipLaunchKernelGGL((k2_blur_mf<N, M_A>), grid, dim3(256), 0, st, K2MF_ARGS);
    else if (method == M_B) hipLaunchKernelGGL((k2_blur_mf<N, M_B>), grid, dim3(256), 0, st, K2MF_ARGS);
    else hipLaunchKernelGGL((k2_blur_mf<N, M_C>), grid, dim3(256), 0, st, K2MF_ARGS);
#undef K2MF_ARGS
  });
}

}  // namespace pnp
