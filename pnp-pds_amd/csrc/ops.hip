// Observation operators, proximal operators and the fused primal/dual passes of one
// PnP-PDS iteration (iteration.py:48-63), for gfx950.
//
// State arrays are fp32 B x C x H x W (NCHW).  One iteration is
//   K1  primal_pre : u = [clamp](x - g1 * Phi^T y)            -> u32 (NCHW; the denoiser's input)
//                    (B) w = s - g1 * y
//   L1  l1_select  : (B) per-image l1-ball threshold theta       (operators.py:94-100)
//   D   denoiser   : x+ = D(u)                                    (conv.hip)
//   K2  dual_a     : v = y + g2 (Phi(2x+ - x) [+ 2 s+ - s]),  s+ = shrink(w, theta)
//                    A/B: y <- v,  per-tile partial sums of (v/g2 - xobs)^2 and the metrics
//                    C:   y <- v - g2 proxGKL(v/g2)  (operators.py:114-115), fully elementwise
//   K3  dual_b     : A/B: y <- v - g2 P_ball(v/g2)              (operators.py:102-108)
//                    + per-image c_n / PSNR (iteration.py:187-188, utils_eval.py:4-7)
//
// Phi for 'blur' is the 19x19 centred circular convolution of operators.py:7-22 (its
// FFT form is exactly a periodic stencil), done here as an LDS-tiled stencil over the
// kernel's non-zero taps with wrap-around halo loads; Phi^T is the correlation
// (operators.py:24-38).  'random_sampling' is a pointwise keep-mask (operators.py:40-58).
#include "kernels.h"
#include "taps_gen.h"

#include <type_traits>
#include <utility>

namespace pnp {

constexpr int kST = 32;                 // square pixel tile of the elementwise passes
constexpr int kMaxR = 16;
constexpr int kLdsW = kST + 2 * kMaxR;  // 64

__device__ __forceinline__ int wrapi(int v, int n) {
  v %= n;
  return v < 0 ? v + n : v;
}

// Fill an (kST+2R)^2 LDS tile of one plane, with periodic wrap (the reference's 'wrap'
// padding, operators.py:12,17,27,32).  F(k) returns the source value at linear index k.
template <class F>
__device__ __forceinline__ void fill_halo(float* lds, int LW, int i0, int j0, int R, int H, int W, F val) {
  const int n = LW * LW;
  for (int q = threadIdx.x; q < n; q += 256) {
    const int ly = q / LW, lx = q - ly * LW;
    const int gi = wrapi(i0 - R + ly, H), gj = wrapi(j0 - R + lx, W);
    lds[q] = val((size_t)gi * W + gj);
  }
}

// Thread (tx = tid&31, tg = tid>>5) computes pixels (i0 + 4tg + r, j0 + tx), r = 0..3.
__device__ __forceinline__ void stencil4(const float* lds, int LW, int R, const int4* __restrict__ taps,
                                         int ntaps, float (&acc)[4]) {
  const int tx = threadIdx.x & 31, tg = threadIdx.x >> 5;
  acc[0] = acc[1] = acc[2] = acc[3] = 0.f;
  const float* base = lds + (4 * tg + R) * LW + tx + R;
  for (int t = 0; t < ntaps; ++t) {
    const int4 tp = taps[t];
    const float w = __int_as_float(tp.z);
    const float* p = base + tp.x * LW + tp.y;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = fmaf(w, p[r * LW], acc[r]);
  }
}

// =====================================================================================
// K1: primal step input  (iteration.py:50/55/61 first half; denoiser.py:35-40)
// grid (tiles_x*tiles_y, B), 256 threads
// =====================================================================================
template <int KIND>
__global__ __launch_bounds__(256) void k1_primal_pre(const float* __restrict__ x, const float* __restrict__ y,
                                                      const float* __restrict__ s, float* __restrict__ u32,
                                                      float* __restrict__ w, OpDesc op, int C, int H, int W, int tiles_x,
                                                      float gamma1, int clamp_in, int method_b) {
  __shared__ float lds[kLdsW * kLdsW];
  const int tile = blockIdx.x, b = blockIdx.y;
  const int ty = tile / tiles_x;
  const int i0 = ty * kST, j0 = (tile - ty * tiles_x) * kST;
  const int tx = threadIdx.x & 31, tg = threadIdx.x >> 5;
  const size_t plane = (size_t)H * W;
  float g[kMaxC][4];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    if (c >= C) break;
    const float* yp = y + ((size_t)b * C + c) * plane;
    if (KIND == OP_BLUR) {
      const int LW = kST + 2 * op.R;
      __syncthreads();
      fill_halo(lds, LW, i0, j0, op.R, H, W, [&](size_t k) { return yp[k]; });
      __syncthreads();
      stencil4(lds, LW, op.R, op.taps_adj, op.ntaps, g[c]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + 4 * tg + r, j = j0 + tx;
        float v = 0.f;
        if (i < H && j < W) {
          v = yp[(size_t)i * W + j];
          if (KIND == OP_MASK) v *= (float)op.mask[(size_t)i * W + j];
        }
        g[c][r] = v;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * tg + r, j = j0 + tx;
    if (i >= H || j >= W) continue;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      if (c >= C) break;
      const size_t idx = ((size_t)b * C + c) * plane + (size_t)i * W + j;
      float u = x[idx] - gamma1 * g[c][r];
      if (clamp_in) u = fminf(fmaxf(u, 0.f), 1.f);
      u32[idx] = u;
      if (method_b) w[idx] = s[idx] - gamma1 * y[idx];
    }
  }
}

// =====================================================================================
// K2: dual ascent with Phi and over-relaxation (iteration.py:51/57/62), fused with the
// l1-ball shrink (B), the GKL prox (C), and the per-tile metric / norm partial sums.
// partials: [B][tiles][4] = { sum (v/g2 - xobs)^2, sum (x+ - x)^2, sum x^2, sum (xt - x+)^2 }
// =====================================================================================
template <int KIND, int METHOD>
__global__ __launch_bounds__(256) void k2_dual(const float* __restrict__ xn, const float* __restrict__ xo,
                                                float* __restrict__ y, const float* __restrict__ xobs,
                                                const float* __restrict__ xtrue, float* __restrict__ s,
                                                const float* __restrict__ w, const float* __restrict__ theta,
                                                double* __restrict__ partials, OpDesc op, int C, int H, int W,
                                                int tiles_x, int tiles, double gamma2, double gkl_gamma,
                                                double gkl_alpha, int record) {
  __shared__ float lds[kLdsW * kLdsW];
  __shared__ double red[4];
  const int tile = blockIdx.x, b = blockIdx.y;
  const int ty = tile / tiles_x;
  const int i0 = ty * kST, j0 = (tile - ty * tiles_x) * kST;
  const int tx = threadIdx.x & 31, tg = threadIdx.x >> 5;
  const size_t plane = (size_t)H * W;
  float g[kMaxC][4];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    if (c >= C) break;
    const float* xnp = xn + ((size_t)b * C + c) * plane;
    const float* xop = xo + ((size_t)b * C + c) * plane;
    if (KIND == OP_BLUR) {
      const int LW = kST + 2 * op.R;
      __syncthreads();
      fill_halo(lds, LW, i0, j0, op.R, H, W, [&](size_t k) { return 2.f * xnp[k] - xop[k]; });
      __syncthreads();
      stencil4(lds, LW, op.R, op.taps_fwd, op.ntaps, g[c]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + 4 * tg + r, j = j0 + tx;
        float v = 0.f;
        if (i < H && j < W) {
          const size_t k = (size_t)i * W + j;
          v = 2.f * xnp[k] - xop[k];
          if (KIND == OP_MASK) v *= (float)op.mask[k];
        }
        g[c][r] = v;
      }
    }
  }
  double d2 = 0, e2 = 0, n2 = 0, t2 = 0;
  const float th = METHOD == M_B ? theta[b] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * tg + r, j = j0 + tx;
    if (i >= H || j >= W) continue;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      if (c >= C) break;
      const size_t idx = ((size_t)b * C + c) * plane + (size_t)i * W + j;
      double gv = g[c][r];
      if (METHOD == M_B) {
        const float wv = w[idx];
        const float sp = copysignf(fmaxf(fabsf(wv) - th, 0.f), wv);   // operators.py:98
        gv += 2.0 * (double)sp - (double)s[idx];
        s[idx] = sp;
      }
      const double v = (double)y[idx] + gamma2 * gv;
      const double ob = xobs[idx];
      if (METHOD == M_C) {
        const double vv = v / gamma2;
        const double tt = vv - gkl_gamma * gkl_alpha;
        const double p = 0.5 * (tt + sqrt(tt * tt + 4.0 * gkl_gamma * ob));
        y[idx] = (float)(v - gamma2 * p);
      } else {
        y[idx] = (float)v;
        const double dd = v / gamma2 - ob;
        d2 += dd * dd;
      }
      if (record) {
        const double a = xn[idx], o = xo[idx];
        e2 += (a - o) * (a - o);
        n2 += o * o;
        if (xtrue) {
          const double q = (double)xtrue[idx] - a;
          t2 += q * q;
        }
      }
    }
  }
  d2 = block_sum(d2, red);
  e2 = block_sum(e2, red);
  n2 = block_sum(n2, red);
  t2 = block_sum(t2, red);
  if (threadIdx.x == 0) {
    double* p = partials + ((size_t)b * tiles + tile) * 4;
    p[0] = d2; p[1] = e2; p[2] = n2; p[3] = t2;
  }
}

// =====================================================================================
// K1 / K2 for the pointwise operators ('Id' and 'random_sampling', operators.py:40-79):
// pure streaming passes.  Block = one 32 x 32 tile of an image (all C channels), thread =
// 4 consecutive pixels of one row: 16-B loads and stores where the row allows (W % 4 == 0),
// scalar otherwise.  K2's four partial sums are reduced once per block (wave shuffles, then
// the 4 waves in a fixed order): partials [B][tiles][4], the layout k3 re-reduces.
// =====================================================================================
// VEC (compile time): 16-B accesses; else nv (0..4) guarded scalar ones.  Callers branch
// once on a uniform-per-thread flag into a VEC and a scalar instantiation: with a runtime
// flag inside each access the compiler merged the two paths into partial loads, each behind
// its own branch and vmcnt(0) wait.
template <int KIND, bool VEC>
__device__ __forceinline__ float4 op_apply4(float4 v, const uint8_t* __restrict__ mask, size_t pix, int nv) {
  if (KIND == OP_MASK) {                 // select (t[q] = 0), so a NaN/inf at a dropped pixel cannot leak
    uchar4 m = {0, 0, 0, 0};
    if (VEC) {
      m = *reinterpret_cast<const uchar4*>(mask + pix);
    } else {
      if (nv > 0) m.x = mask[pix];
      if (nv > 1) m.y = mask[pix + 1];
      if (nv > 2) m.z = mask[pix + 2];
      if (nv > 3) m.w = mask[pix + 3];
    }
    v.x = m.x ? v.x : 0.f; v.y = m.y ? v.y : 0.f; v.z = m.z ? v.z : 0.f; v.w = m.w ? v.w : 0.f;
  }
  return v;
}

typedef float f4v_t __attribute__((ext_vector_type(4)));
template <bool VEC>
__device__ __forceinline__ float4 ld4(const float* __restrict__ p, int nv) {
  if (VEC) {
    const f4v_t v = __builtin_nontemporal_load(reinterpret_cast<const f4v_t*>(p));
    return float4{v.x, v.y, v.z, v.w};
  }
  float4 v = {0.f, 0.f, 0.f, 0.f};
  if (nv > 0) v.x = p[0];
  if (nv > 1) v.y = p[1];
  if (nv > 2) v.z = p[2];
  if (nv > 3) v.w = p[3];
  return v;
}
template <bool VEC>
__device__ __forceinline__ void st4(float* __restrict__ p, float4 v, int nv) {
  if (VEC) { __builtin_nontemporal_store(f4v_t{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v_t*>(p)); return; }
  if (nv > 0) p[0] = v.x;
  if (nv > 1) p[1] = v.y;
  if (nv > 2) p[2] = v.z;
  if (nv > 3) p[3] = v.w;
}
__device__ __forceinline__ float f4get(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// K1: thread = one pixel column of 4 rows (consecutive lanes on consecutive pixels).  NC = C
// when it is a compile-time 1 or 3 (all channels' loads in flight together), 0 = runtime C <= 4.
template <int KIND, int NC>
__global__ __launch_bounds__(256) void k1_elem(const float* __restrict__ x, const float* __restrict__ y,
                                                const float* __restrict__ s, float* __restrict__ u32,
                                                float* __restrict__ w, const uint8_t* __restrict__ mask, int Crt, int H, int W, int tiles_x,
                                                float gamma1, int clamp_in, int method_b) {
  constexpr int CM = NC ? NC : kMaxC;
  const int C = NC ? NC : Crt;
  const int tile = blockIdx.x, b = blockIdx.y;
  const int ty = tile / tiles_x;
  const int i0 = ty * kST + 4 * (threadIdx.x >> 5), j = (tile - ty * tiles_x) * kST + (threadIdx.x & 31);
  if (j >= W) return;
  const size_t plane = (size_t)H * W;
  const int nr = min(4, H - i0);
  // all rows' loads first, B's extra streams a compile-time choice (a runtime branch
  // around a load made the compiler wait vmcnt(0) at the join)
  auto body = [&](auto mb_c) {
    constexpr bool MB = decltype(mb_c)::value;
    float xv[4][CM], yv[4][CM], sv[4][CM];
    uint8_t keep[4];                          // compared only after every load is in flight
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r >= nr) break;
      const size_t pix = (size_t)(i0 + r) * W + j;
      keep[r] = KIND == OP_MASK ? mask[pix] : 1;
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        if (c >= C) break;
        const size_t o = ((size_t)b * C + c) * plane + pix;
        xv[r][c] = __builtin_nontemporal_load(x + o);   // streamed once
        yv[r][c] = __builtin_nontemporal_load(y + o);
        if (MB) sv[r][c] = __builtin_nontemporal_load(s + o);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r >= nr) break;
      const int i = i0 + r;
      const size_t pix = (size_t)i * W + j;
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        if (c >= C) break;
        const size_t o = ((size_t)b * C + c) * plane + pix;
        const float g = keep[r] != 0 ? yv[r][c] : 0.f;   // random_sampling: t[q] = 0 (a NaN cannot leak)
        float u = xv[r][c] - gamma1 * g;
        if (clamp_in) u = fminf(fmaxf(u, 0.f), 1.f);
        u32[o] = u;
        if (MB) w[o] = sv[r][c] - gamma1 * yv[r][c];
      }
    }
  };
  if (method_b) body(std::true_type{});
  else body(std::false_type{});
}

template <int KIND, int METHOD, int NC>
__global__ __launch_bounds__(256) void k2_elem(const float* __restrict__ xn, const float* __restrict__ xo,
                                                float* __restrict__ y, const float* __restrict__ xobs,
                                                const float* __restrict__ xtrue, float* __restrict__ s,
                                                const float* __restrict__ w, const float* __restrict__ theta,
                                                double* __restrict__ partials, const uint8_t* __restrict__ mask,
                                                int Crt, int H, int W, int tiles_x, int tiles, double gamma2,
                                                double inv_g2, double gkl_gamma, double gkl_alpha, int record,
                                                float* __restrict__ mm) {
  constexpr int CM = NC ? NC : kMaxC;
  const int C = NC ? NC : Crt;
  __shared__ double red[4][4];
  const int tile = blockIdx.x, b = blockIdx.y;
  const int ty = tile / tiles_x;
  const int i = ty * kST + (threadIdx.x >> 3), j = (tile - ty * tiles_x) * kST + 4 * (threadIdx.x & 7);
  double d2 = 0, e2 = 0, n2 = 0, t2 = 0;
  float lo = __builtin_inff(), hi = -__builtin_inff();   // x+ range for SSIM's data_range
  if (i < H && j < W) {
    const int nv = min(4, W - j);
    const bool vec = (W & 3) == 0 && nv == 4;
    const size_t plane = (size_t)H * W, pix = (size_t)i * W + j;
    const float th = METHOD == M_B ? theta[b] : 0.f;
    auto body = [&](auto vec_c, auto true_c) {
      constexpr bool VEC = decltype(vec_c)::value, TRUE_ = decltype(true_c)::value;   // TRUE_: record && xtrue
      // every channel's loads first (stores to y could otherwise not pass loads of y)
      float4 a4[CM], o4[CM], y4[CM], b4[CM], s4[CM], w4[CM], t4[CM];
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        if (c >= C) break;
        const size_t o = ((size_t)b * C + c) * plane + pix;
        a4[c] = ld4<VEC>(xn + o, nv);
        o4[c] = ld4<VEC>(xo + o, nv);
        y4[c] = ld4<VEC>(y + o, nv);
        b4[c] = ld4<VEC>(xobs + o, nv);
        if (METHOD == M_B) { s4[c] = ld4<VEC>(s + o, nv); w4[c] = ld4<VEC>(w + o, nv); }
        if (TRUE_) t4[c] = ld4<VEC>(xtrue + o, nv);   // compile-time: a runtime branch here waited vmcnt(0)
      }
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        if (c >= C) break;
        const size_t o = ((size_t)b * C + c) * plane + pix;
        float4 g4;
        g4.x = 2.f * a4[c].x - o4[c].x; g4.y = 2.f * a4[c].y - o4[c].y;
        g4.z = 2.f * a4[c].z - o4[c].z; g4.w = 2.f * a4[c].w - o4[c].w;
        g4 = op_apply4<KIND, VEC>(g4, mask, pix, nv);
        float4 sp4 = {}, yo;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          double gv = f4get(g4, k);
          if (METHOD == M_B) {
            const float wv = f4get(w4[c], k);
            const float sp = copysignf(fmaxf(fabsf(wv) - th, 0.f), wv);   // operators.py:98
            gv += 2.0 * (double)sp - (double)f4get(s4[c], k);
            (k == 0 ? sp4.x : k == 1 ? sp4.y : k == 2 ? sp4.z : sp4.w) = sp;
          }
          const double v = (double)f4get(y4[c], k) + gamma2 * gv;
          const double ob = f4get(b4[c], k);
          float yk;
          if (METHOD == M_C) {
            const double tt = v * inv_g2 - gkl_gamma * gkl_alpha;
            const double p = 0.5 * (tt + sqrt(tt * tt + 4.0 * gkl_gamma * ob));
            yk = (float)(v - gamma2 * p);
          } else {
            yk = (float)v;
            const double dd = v * inv_g2 - ob;
            if (k < nv) d2 += dd * dd;
          }
          (k == 0 ? yo.x : k == 1 ? yo.y : k == 2 ? yo.z : yo.w) = yk;
          if (record && k < nv) {
            lo = fminf(lo, f4get(a4[c], k));
            hi = fmaxf(hi, f4get(a4[c], k));
            const double a = f4get(a4[c], k), oo = f4get(o4[c], k);
            e2 += (a - oo) * (a - oo);
            n2 += oo * oo;
            if (TRUE_) {
              const double q = (double)f4get(t4[c], k) - a;
              t2 += q * q;
            }
          }
        }
        st4<VEC>(y + o, yo, nv);
        if (METHOD == M_B) st4<VEC>(s + o, sp4, nv);
      }
    };
    if (record && xtrue) {
      if (vec) body(std::true_type{}, std::true_type{});
      else body(std::false_type{}, std::true_type{});
    } else {
      if (vec) body(std::true_type{}, std::false_type{});
      else body(std::false_type{}, std::false_type{});
    }
  }
  d2 = wave_sum(d2);
  e2 = wave_sum(e2);
  n2 = wave_sum(n2);
  t2 = wave_sum(t2);
  const int wv = threadIdx.x >> 6;
  __shared__ float redr[4][2];
  if (record && mm) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = fminf(lo, __shfl_xor(lo, o, 64));
      hi = fmaxf(hi, __shfl_xor(hi, o, 64));
    }
  }
  if ((threadIdx.x & 63) == 0) {
    red[wv][0] = d2; red[wv][1] = e2; red[wv][2] = n2; red[wv][3] = t2;
    redr[wv][0] = lo; redr[wv][1] = hi;
  }
  __syncthreads();
  if (threadIdx.x < 4)
    partials[((size_t)b * tiles + tile) * 4 + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
  if (record && mm && threadIdx.x == 0) {    // per (image, tile): [B][tiles][2]
    mm[((size_t)b * tiles + tile) * 2 + 0] = fminf(fminf(redr[0][0], redr[1][0]), fminf(redr[2][0], redr[3][0]));
    mm[((size_t)b * tiles + tile) * 2 + 1] = fmaxf(fmaxf(redr[0][1], redr[1][1]), fmaxf(redr[2][1], redr[3][1]));
  }
}

// Deterministic reduction of one image's tile partials (fixed order) in a 256-block.
__device__ __forceinline__ void reduce_partials(const double* __restrict__ partials, int b, int tiles,
                                                double (&out)[4], double* red) {
  double a[4] = {0, 0, 0, 0};
  for (int k = threadIdx.x; k < tiles; k += 256) {
    const double* p = partials + ((size_t)b * tiles + k) * 4;
    a[0] += p[0]; a[1] += p[1]; a[2] += p[2]; a[3] += p[3];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) out[q] = block_sum(a[q], red);
}

__device__ __forceinline__ void write_metrics(double* metrics, int b, int it, int cap, const double (&a)[4],
                                              double n_elem, int has_true) {
  if (it >= cap) return;                                            // (graph replays run past the record)
  double* m = metrics + ((size_t)b * cap + it) * kMetrics;
  m[0] = sqrt(a[1]) / sqrt(a[2]);                                   // iteration.py:187
  m[1] = has_true ? 10.0 * log10(1.0 / (a[3] / n_elem)) : __builtin_nan("");   // utils_eval.py:4-7
}

// =====================================================================================
// K3 (A/B): y <- v - g2 * P_{B(xobs, eps)}(v / g2) = (1 - f)(v - g2 xobs), f = min(1, eps/|v/g2 - xobs|)
// grid (chunks, B); each block re-reduces its image's partials (fixed order).  With the blur
// operator the same update runs inside the next K1's halo fill instead (k1_blur_rb PEND) and
// k3_norm only computes 1 - f per image; k3_l2_dual then finalizes y in place when the host
// asks for the dual state.
// =====================================================================================
__device__ __forceinline__ double l2_dual_omf(const double (&a)[4], double eps) {
  const double nrm = sqrt(a[0]);
  const double f = nrm > eps ? eps / nrm : 1.0;
  return 1.0 - f;
}
// the one expression both K3 and K1's fused fill use (same bits)
__device__ __forceinline__ float l2_dual_y(float v, float ob, double omf, double gamma2) {
  return (float)(omf * ((double)v - gamma2 * (double)ob));
}

__global__ __launch_bounds__(256) void k3_l2_dual(float* __restrict__ y, const float* __restrict__ xobs,
                                                   const double* __restrict__ partials, int tiles, size_t n,
                                                   double gamma2, double eps, double* __restrict__ metrics,
                                                   int it, int cap, int record, int has_true,
                                                   const int* __restrict__ itp) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  if (itp) it = *itp;                        // graph replay: the iteration number from the device counter
  double a[4];
  reduce_partials(partials, b, tiles, a, red);
  const double omf = l2_dual_omf(a, eps);
  if (record && blockIdx.x == 0 && threadIdx.x == 0) write_metrics(metrics, b, it, cap, a, (double)n, has_true);
  float* yb = y + (size_t)b * n;
  const float* ob = xobs + (size_t)b * n;
  const size_t chunk = 2048;
  const size_t beg = (size_t)blockIdx.x * chunk;
  for (size_t k = beg + threadIdx.x; k < beg + chunk && k < n; k += 256)
    yb[k] = l2_dual_y(yb[k], ob[k], omf, gamma2);   // (non-temporal: 0.119 vs 0.099 ms)
}

// K3 without the pass (blur operator): per image 1 - f for the next K1's fused fill, and the
// iteration's metrics.  grid (B).
__global__ __launch_bounds__(256) void k3_norm(const double* __restrict__ partials, int tiles, size_t n,
                                                double eps, double* __restrict__ omf, double* __restrict__ metrics,
                                                int it, int cap, int record, int has_true,
                                                const int* __restrict__ itp) {
  __shared__ double red[4];
  const int b = blockIdx.x;
  if (itp) it = *itp;
  double a[4];
  reduce_partials(partials, b, tiles, a, red);
  if (threadIdx.x == 0) {
    omf[b] = l2_dual_omf(a, eps);
    if (record) write_metrics(metrics, b, it, cap, a, (double)n, has_true);
  }
}

__global__ __launch_bounds__(256) void k3_metrics(const double* __restrict__ partials, int tiles, size_t n,
                                                   double* __restrict__ metrics, int it, int cap, int has_true,
                                                   const int* __restrict__ itp) {
  __shared__ double red[4];
  double a[4];
  if (itp) it = *itp;
  reduce_partials(partials, blockIdx.x, tiles, a, red);
  if (threadIdx.x == 0) write_metrics(metrics, blockIdx.x, it, cap, a, (double)n, has_true);
}

// =====================================================================================
// l1-ball threshold (operators.py:94-100).  The reference sorts |v| and takes
// theta = max(0, max_k (S_k - eta)/k); equivalently theta is the root of
// f(t) = sum max(|v|-t, 0) - eta.  A 3-level radix select on the float bit patterns of |v|
// (11 + 11 + 9 bits): each level builds a histogram (count, sum) of the candidates, finds the
// highest bin whose lower edge still has f >= 0, and descends into it.  After the last level
// every candidate bin is one float value t*, and the counts / sums strictly above it are
// K = #{|v| > t*} and S = sum of those, so theta = (S - eta) / K with no extra pass.
//
// Work split (MI355X: a whole chip of CUs, few images): each level is a histogram launch
// over G workgroups per image (B x G >= 512, slices of >= 16K elements, 16-B loads; each
// workgroup bins its slice in LDS and adds its non-empty bins to the image's histogram in
// HBM with integer atomics) and a pick launch (one wave per image) that scans the bins and
// updates the image's state {prefix, K above, S above}.  Level 1 also yields sum |v|
// (all values are its candidates), which decides the "inside the ball" case.
// Bin sums are kept exactly: every value of a bin shares its float exponent (the bins split
// the bit pattern below the 8 exponent bits), so a bin's sum is (sum of 24-bit significands,
// a uint64 that atomics add in any order to the same result) x 2^(exponent - 150); every
// launch split therefore gives the same theta bits (batch vs single image, sharding).
// =====================================================================================
constexpr int kSelBins = 2048;
constexpr int kSelHistThreads = 256;
struct L1State {
  unsigned prefix;
  unsigned done;          // theta already decided (eta <= 0, inside the ball, or last level)
  double Khi, Shi;        // count / sum of |v| strictly above the current candidate range
};
struct L1Scratch {        // per image, in HBM
  L1State st;
  unsigned cnt[kSelBins];
  unsigned long long sm[kSelBins];
};

__device__ __forceinline__ unsigned sel_significand(unsigned u) {
  const unsigned e = u >> 23, m = u & 0x7fffffu;
  return e ? (m | 0x800000u) : m;
}
template <int SH>
__device__ __forceinline__ double sel_bin_sum(const unsigned long long* sm, unsigned prefix, int j) {
  const int e = (int)(((prefix | ((unsigned)j << SH)) >> 23) & 0xffu);
  // exact while n < 2^29 (a bin's significand sum < n * 2^24 <= 2^53); the callers of
  // launch_l1_select reject larger images (kMaxL1Elems)
  return ldexp((double)sm[j], e ? e - 150 : -149);
}

template <int SH, int NBITS>
__global__ __launch_bounds__(kSelHistThreads) void l1_hist_kernel(const float* __restrict__ v, size_t n, size_t chunk,
                                                                  L1Scratch* __restrict__ scr, double eta) {
  constexpr int nb = 1 << NBITS;
  constexpr unsigned hi_mask = (SH + NBITS >= 31) ? 0u : (0x7fffffffu & ~((1u << (SH + NBITS)) - 1u));
  __shared__ unsigned cnt[nb];
  __shared__ unsigned long long sm[nb];
  const int b = blockIdx.y;
  L1Scratch* sc = scr + b;
  if (!(eta > 0.0) || sc->st.done) return;
  const unsigned prefix = sc->st.prefix;
  for (int j = threadIdx.x; j < nb; j += kSelHistThreads) { cnt[j] = 0; sm[j] = 0ull; }
  __syncthreads();
  const size_t lo = (size_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  const unsigned* vb = reinterpret_cast<const unsigned*>(v + (size_t)b * n);
  auto bin = [&](unsigned u) {
    u &= 0x7fffffffu;
    if ((u & hi_mask) == prefix) {
      const unsigned j = (u >> SH) & (unsigned)(nb - 1);
      atomicAdd(&cnt[j], 1u);
      atomicAdd(&sm[j], (unsigned long long)sel_significand(u));   // exact, so order-independent
    }
  };
  size_t i = lo;
  if ((((uintptr_t)(vb + lo)) & 15) == 0) {     // 16-B loads over the aligned body of the slice
    typedef unsigned u4v_t __attribute__((ext_vector_type(4)));
    const u4v_t* v4 = reinterpret_cast<const u4v_t*>(vb + lo);
    const size_t n4 = (hi - lo) / 4;
    for (size_t k = threadIdx.x; k < n4; k += kSelHistThreads) {
      const u4v_t q = __builtin_nontemporal_load(v4 + k);
      bin(q.x); bin(q.y); bin(q.z); bin(q.w);
    }
    i = lo + 4 * n4;
  }
  for (size_t k = i + threadIdx.x; k < hi; k += kSelHistThreads) bin(vb[k]);
  __syncthreads();
  for (int j = threadIdx.x; j < nb; j += kSelHistThreads)
    if (cnt[j]) {
      atomicAdd(&sc->cnt[j], cnt[j]);
      atomicAdd(&sc->sm[j], sm[j]);
    }
}

// One wave per image: scan the level's bins from the top, keep the highest bin whose lower
// edge has f >= 0, clear the bins for the next level.  Level 1 (FIRST) first decides
// eta <= 0 (projection onto {0}: theta = inf) and sum |v| <= eta (inside: theta = 0); the
// last level writes theta.
template <int SH, int NBITS, bool FIRST, bool LAST>
__global__ __launch_bounds__(64) void l1_pick_kernel(L1Scratch* __restrict__ scr, float* __restrict__ theta,
                                                     double eta) {
  constexpr int nb = 1 << NBITS, per = nb / 64;
  const int b = blockIdx.x, lane = threadIdx.x;
  L1Scratch* sc = scr + b;
  if (sc->st.done) return;
  const unsigned prefix = sc->st.prefix;
  const double Khi = sc->st.Khi, Shi = sc->st.Shi;
  unsigned* cnt = sc->cnt;
  const unsigned long long* sm = sc->sm;
  double kc = 0, sc_ = 0;
  unsigned c[per];
  double sv[per];
#pragma unroll
  for (int q = 0; q < per; ++q) {
    c[q] = cnt[lane * per + q];
    sv[q] = sel_bin_sum<SH>(sm, prefix, lane * per + q);
    kc += c[q];
    sc_ += sv[q];
  }
  if (FIRST) {
    double tot = sc_;                           // fixed-order sum of exact bin sums
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off, 64);
    const bool zero_ball = !(eta > 0.0), inside = tot <= eta;
    if (zero_ball || inside) {
      for (int q = 0; q < per; ++q) { cnt[lane * per + q] = 0; sc->sm[lane * per + q] = 0ull; }
      if (lane == 0) {
        theta[b] = zero_ball ? __builtin_inff() : 0.f;
        sc->st.done = 1;
      }
      return;
    }
  }
  double ks = kc, ss = sc_;                     // inclusive suffix over lanes lane..63
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double tk = __shfl_down(ks, off, 64), ts = __shfl_down(ss, off, 64);
    if (lane + off < 64) { ks += tk; ss += ts; }
  }
  double K = Khi + ks - kc, S = Shi + ss - sc_;   // strictly above this lane's bins
  int found = -1;
  double fK = 0, fS = 0;
  for (int q = per - 1; q >= 0; --q) {
    const int j = lane * per + q;
    const double K2 = K + c[q], S2 = S + sv[q];
    const double lo = (double)__uint_as_float(prefix | ((unsigned)j << SH));
    if (S2 - K2 * lo - eta >= 0.0) { found = j; fK = K; fS = S; break; }
    K = K2; S = S2;
  }
  int best = found;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) best = max(best, __shfl_xor(best, off, 64));
  // bin 0 as the fallback (exact sums make it unreachable: the parent bin had f(lo) >= 0):
  // "above bin 0" = Khi + all bins >= 1, summed in the same fixed order as the scan
  const int own = best >= 0 ? (found == best) : (lane == 0);
  double nK = fK, nS = fS;
  if (best < 0 && lane == 0) {
    nK = Khi; nS = Shi;
    for (int j = nb - 1; j >= 1; --j) { nK += cnt[j]; nS += sel_bin_sum<SH>(sm, prefix, j); }
  }
  const int jsel = best >= 0 ? best : 0;
  __syncthreads();                              // every lane has read its bins
  for (int q = 0; q < per; ++q) { cnt[lane * per + q] = 0; sc->sm[lane * per + q] = 0ull; }
  if (own) {
    const unsigned np = prefix | ((unsigned)jsel << SH);
    if (LAST) {
      const double th = nK > 0 ? (nS - eta) / nK : (double)__uint_as_float(np);
      theta[b] = (float)(th > 0 ? th : 0.0);
      sc->st.done = 1;
    } else {
      sc->st.prefix = np;
      sc->st.Khi = nK;
      sc->st.Shi = nS;
    }
  }
}

__global__ void l1_reset_kernel(L1Scratch* __restrict__ scr, int B) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b < B) scr[b].st = L1State{0u, 0u, 0.0, 0.0};
}

size_t l1_select_scratch_bytes(int B) { return (size_t)B * sizeof(L1Scratch); }

// =====================================================================================
// Standalone operators (pnp_op_*): stencil, l2 projection, shrink, GKL, PSNR, packing.
// =====================================================================================
template <int KIND, int ADJ>
__global__ __launch_bounds__(256) void op_phi_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                      const float* __restrict__ add, OpDesc op, int H, int W,
                                                      int tiles_x) {
  __shared__ float lds[kLdsW * kLdsW];
  const int tile = blockIdx.x, bc = blockIdx.y;
  const int ty = tile / tiles_x;
  const int i0 = ty * kST, j0 = (tile - ty * tiles_x) * kST;
  const int tx = threadIdx.x & 31, tg = threadIdx.x >> 5;
  const size_t plane = (size_t)H * W;
  const float* xp = x + (size_t)bc * plane;
  float acc[4];
  if (KIND == OP_BLUR) {
    const int LW = kST + 2 * op.R;
    fill_halo(lds, LW, i0, j0, op.R, H, W, [&](size_t k) { return xp[k]; });
    __syncthreads();
    stencil4(lds, LW, op.R, ADJ ? op.taps_adj : op.taps_fwd, op.ntaps, acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * tg + r, j = j0 + tx;
    if (i >= H || j >= W) continue;
    const size_t k = (size_t)i * W + j;
    float v;
    if (KIND == OP_BLUR) v = acc[r];
    else if (KIND == OP_MASK) v = op.mask[k] ? xp[k] : 0.f;   // t[q] = 0 (operators.py:49-57), NaN-safe
    else v = xp[k];
    if (add) v += add[(size_t)bc * plane + k];
    out[(size_t)bc * plane + k] = v;
  }
}

// per image partial sums of (x - x0)^2 (or (xt - x)^2 for psnr): grid (chunks, B)
__global__ __launch_bounds__(256) void sqdiff_partials(const float* __restrict__ a, const float* __restrict__ c,
                                                        double* __restrict__ partials, size_t n, int chunks) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  const size_t chunk = 2048, beg = (size_t)blockIdx.x * chunk;
  double acc = 0;
  for (size_t k = beg + threadIdx.x; k < beg + chunk && k < n; k += 256) {
    const double d = (double)a[(size_t)b * n + k] - (double)c[(size_t)b * n + k];
    acc += d * d;
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) partials[(size_t)b * chunks + blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void l2_apply(const float* __restrict__ x, const float* __restrict__ x0,
                                                 float* __restrict__ out, const double* __restrict__ partials,
                                                 size_t n, int chunks, double eps) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  double a = 0;
  for (int k = threadIdx.x; k < chunks; k += 256) a += partials[(size_t)b * chunks + k];
  a = block_sum(a, red);
  const double nrm = sqrt(a);
  const size_t chunk = 2048, beg = (size_t)blockIdx.x * chunk;
  for (size_t k = beg + threadIdx.x; k < beg + chunk && k < n; k += 256) {
    const size_t i = (size_t)b * n + k;
    out[i] = nrm > eps ? (float)((double)x0[i] + eps * ((double)x[i] - (double)x0[i]) / nrm) : x[i];
  }
}

__global__ __launch_bounds__(256) void shrink_kernel(const float* __restrict__ v, float* __restrict__ out,
                                                      const float* __restrict__ theta, size_t n) {
  const int b = blockIdx.y;
  const float th = theta[b];
  const size_t chunk = 2048, beg = (size_t)blockIdx.x * chunk;
  for (size_t k = beg + threadIdx.x; k < beg + chunk && k < n; k += 256) {
    const float x = v[(size_t)b * n + k];
    out[(size_t)b * n + k] = copysignf(fmaxf(fabsf(x) - th, 0.f), x);
  }
}

__global__ __launch_bounds__(256) void gkl_kernel(const float* __restrict__ x, const float* __restrict__ x0,
                                                   float* __restrict__ out, size_t count, double gamma, double alpha) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (size_t)gridDim.x * 256) {
    const double t = (double)x[i] - gamma * alpha;
    out[i] = (float)(0.5 * (t + sqrt(t * t + 4.0 * gamma * (double)x0[i])));
  }
}

// Denoiser input for pnp_op_denoise: u32 = [clamp](x) (the head converts it to fp16).
__global__ __launch_bounds__(256) void pack_input_kernel(const float* __restrict__ x, float* __restrict__ u32,
                                                          size_t total, int clamp_in) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    float u = x[i];
    if (clamp_in) u = fminf(fmaxf(u, 0.f), 1.f);
    u32[i] = u;
  }
}

// =====================================================================================
// Register-blocked blur passes (operators.py:7-38 inside iteration.py:50/51).  The stencil
// over the kernel's non-zero taps runs on a 64 x 64 output tile of one channel plane,
// staged in LDS with its periodic halo; thread (tx, ty) owns columns 2tx, 2tx+1 and rows
// 8ty .. 8ty+7.  For each LDS column pair it touches, the thread loads the (8 + 2R)-row
// column segment once into registers and applies every non-zero tap of the kernel columns
// that use it to its 8 x 2 accumulators.  One block per (plane, tile), 6 blocks per CU.
// (Measured slower and removed: persistent blocks that prefetch the next tile's halo into
// registers while the current tile computes: 3 blocks per CU at 168 VGPRs, K1 0.26 vs
// 0.22 ms, K2 0.56 vs 0.40 ms - the stencil needs the wave count more than the prefetch.)
// The LDS halo is only as wide as the taps' non-zero columns need (blur_1: columns -4..+4
// of 19; rows -8..+8): 72 x 80 floats instead of 80 x 80.
// =====================================================================================
constexpr int kRbW = 64, kRbH = 64, kRbRows = kRbH / 8;   // 8 thread rows x kRbRows rows; 32 threads x 2 columns
// (64 x 32 tiles measured slower, r03: K1 0.206 -> 0.222, K2 0.269 -> 0.276 ms)
static_assert(kRbH == 64 || kRbH == 32, "tiles of whole 32 x 32 metric cells");

typedef float f2_t __attribute__((ext_vector_type(2)));

template <int R>
struct DenseTaps {
  static constexpr int kR = R;
  static constexpr bool kDense = true;
  __host__ __device__ static constexpr uint32_t col(int) { return (1u << (2 * R + 1)) - 1u; }
};

// Geometry of the LDS halo for a tap pattern T.  Column pair P (LDS columns 2tx+2P-kOff and
// +1) is active when kernel column 2P-1, 2P or 2P+1 has a non-zero tap; only pairs
// kPmin..kPmax are read, so the LDS image starts at global column j0 - R + kOff.
template <class T>
struct TapGeom {
  static constexpr int R = T::kR, D = 2 * R + 1;
  static constexpr uint32_t colm(int k) { return k < 0 || k >= D ? 0u : T::col(k); }
  static constexpr bool active(int P) { return (colm(2 * P - 1) | colm(2 * P) | colm(2 * P + 1)) != 0u; }
  static constexpr int pmin() {
    for (int P = 0; P <= R; ++P)
      if (active(P)) return P;
    return 0;
  }
  static constexpr int pmax() {
    for (int P = R; P >= 0; --P)
      if (active(P)) return P;
    return 0;
  }
  static constexpr int kPmin = pmin(), kPmax = pmax();
  static constexpr int kOff = 2 * kPmin;
  static constexpr int LW = kRbW + 2 * (kPmax - kPmin), LH = kRbH + 2 * R;
  static constexpr int N = LW * LH, NF = (N + 255) / 256;
};

// Thread (tx, ty) accumulates rows 8ty..+7 of output columns 2tx, 2tx+1 as float2 pairs
// (v_pk_fma_f32).  LDS columns are read in pairs (A, B = A+1) by ds_read_b64: 32 lanes x
// 8 B contiguous, conflict-free.  Column A feeds output column 0 with kernel column 2P and
// output column 1 with kernel column 2P-1; column B feeds them with kernel columns 2P+1 and
// 2P.  Each pair of taps is one packed FMA with the column value broadcast.  The loop is
// fully unrolled over the compile-time non-zero pattern TAPS (taps_gen.h; DenseTaps<R> for
// any other kernel): no per-tap branches and no loads of LDS columns or weights that only
// zero taps touch.  Tap values are runtime data.  (Measured: one scalar v_fma_f32 per
// non-zero tap instead - 13 % fewer FMAs, 76 % more instructions - is slower, K1 0.27 vs
// 0.22 ms: the packed form issues at the scalar rate.)
// wp: packed tap pairs [p][dyi][2] (float2): [.][.][0] = (W[2p][dyi], W[2p-1][dyi]) for
// LDS column A, [.][.][1] = (W[2p+1][dyi], W[2p][dyi]) for column B (W = column-major
// dense table, out-of-range columns 0), built on the host (pnp_set_operator) so each
// packed FMA takes its weight pair straight from one s_load_dwordx2.
template <class T, int P>
__device__ __forceinline__ void rb_pair(const f2_t* base, const f2_t* __restrict__ wp, f2_t (&acc)[kRbRows]) {
  using G = TapGeom<T>;
  constexpr int R = T::kR, D = G::D;
  constexpr uint32_t m0 = G::colm(2 * P), mm1 = G::colm(2 * P - 1), m1 = G::colm(2 * P + 1);
  constexpr uint32_t mA = m0 | mm1, mB = m1 | m0;
  if constexpr ((mA | mB) != 0u) {
    f2_t cv[kRbRows + 2 * R];
#pragma unroll
    for (int k = 0; k < kRbRows + 2 * R; ++k) cv[k] = base[k * (G::LW / 2) + P - G::kPmin];   // unused rows: dead
#pragma unroll
    for (int dyi = 0; dyi < D; ++dyi) {
      if ((mA >> dyi) & 1u) {
        const f2_t w2 = wp[(P * D + dyi) * 2 + 0];
#pragma unroll
        for (int r = 0; r < kRbRows; ++r)
          acc[r] = __builtin_elementwise_fma(w2, f2_t{cv[r + dyi].x, cv[r + dyi].x}, acc[r]);
      }
      if ((mB >> dyi) & 1u) {
        const f2_t w2 = wp[(P * D + dyi) * 2 + 1];
#pragma unroll
        for (int r = 0; r < kRbRows; ++r)
          acc[r] = __builtin_elementwise_fma(w2, f2_t{cv[r + dyi].y, cv[r + dyi].y}, acc[r]);
      }
    }
  }
}

template <class T, int... Ps>
__device__ __forceinline__ void rb_pair_dispatch(int p, const f2_t* base, const f2_t* __restrict__ wp,
                                                 f2_t (&acc)[kRbRows], std::integer_sequence<int, Ps...>) {
  (void)((p == Ps ? (rb_pair<T, Ps>(base, wp, acc), true) : false) || ...);
}

// The pair loop stays a runtime loop (one straight-line, compile-time-masked body per pair),
// so the weights and the column values of only one pair are live at a time.
template <class T>
__device__ __forceinline__ void rb_stencil(const float* lds, const f2_t* __restrict__ wp, f2_t (&acc)[kRbRows]) {
  using G = TapGeom<T>;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int r = 0; r < kRbRows; ++r) acc[r] = f2_t{0.f, 0.f};
  const f2_t* base = reinterpret_cast<const f2_t*>(lds + ty * kRbRows * G::LW + 2 * tx);
#pragma unroll 1
  for (int p = G::kPmin; p <= G::kPmax; ++p)
    rb_pair_dispatch<T>(p, base, wp, acc, std::make_integer_sequence<int, T::kR + 1>{});
}

// Halo fills: batches of kRbFill elements per thread (the loads of a batch in flight
// together, then their LDS stores), so few registers are live and 6 blocks fit per CU.
constexpr int kRbFill = 8;      // (batches of 14 / 16 / 27 / 32 measured equal or slower)

// Column-wise halo fill (K1): thread t < TPC LW owns LDS column t % LW and rows t / LW +
// TPC i, so the column's wrap is resolved once and each row step is an add and one
// conditional wrap (the element-wise gather above re-derives row and column and wraps both
// for every element).  Loads in batches of kRbFill rows, then their LDS stores.
template <class G, int NB = kRbFill, class FA>
__device__ __forceinline__ void rb_fill_cols(float* lds, int i0, int j0, int H, int W, FA&& la) {
  constexpr int TPC = 256 / G::LW;                   // threads per column (row stride)
  constexpr int NI = (G::LH + TPC - 1) / TPC;        // rows per thread (the last may be past LH)
  const int tid = threadIdx.x;
  if (tid >= TPC * G::LW) return;
  const int lx = tid % G::LW, ly0 = tid / G::LW;
  int gj = j0 - G::R + G::kOff + lx;
  gj += gj < 0 ? W : 0;
  gj -= gj >= W ? W : 0;
  gj = min(max(gj, 0), W - 1);
  int gi = i0 - G::R + ly0;
  gi += gi < 0 ? H : 0;
  gi -= gi >= H ? H : 0;
#pragma unroll
  for (int i0b = 0; i0b < NI; i0b += NB) {
    float a[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if (i0b + i < NI) {
        a[i] = la(min(max(gi, 0), H - 1) * W + gj);
        gi += TPC;
        gi -= gi >= H ? H : 0;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int ly = ly0 + TPC * (i0b + i);
      if (i0b + i < NI && (G::LH % TPC == 0 || ly < G::LH)) lds[ly * G::LW + lx] = a[i];
    }
  }
}

// XCD-aware block -> tile order for the register-blocked passes: blocks b and b + 8 share an
// XCD (MI355X_MICROARCH.md, workgroup dispatch), so XCD x gets the contiguous tile range
// [x n/8, (x+1) n/8) in order and a tile's halo rows and columns (41 % of its fill: the
// neighbouring tiles' pixels) are read while those neighbours are in flight on the same
// XCD's L2 instead of another XCD's.  (A tail of n % 8 blocks keeps the identity order.)
__device__ __forceinline__ int rb_block_tile() {
  const int b = blockIdx.x, n = gridDim.x;
  const int full = n & ~7;
  return b < full ? (b & 7) * (full >> 3) + (b >> 3) : b;
}

__device__ __forceinline__ void rb_tile_origin(int tile, int tiles_x, int& i0, int& j0) {
  const int ty = tile / tiles_x;
  i0 = ty * kRbH;
  j0 = (tile - ty * tiles_x) * kRbW;
}

// Column-pair loads / stores of the blur kernels' epilogues: nv valid columns (0..2);
// vec = both valid and 8-B aligned (one dwordx2), else guarded scalar accesses.
// The epilogue streams (read once / written once per pass: x, y, s, x_obs, w in, u32, y, s, w
// out) are non-temporal: K1 0.162 -> 0.159 ms, K2 0.276 -> 0.272 at the metric (A/B, r03).
__device__ __forceinline__ f2_t ld2g(const float* __restrict__ p, size_t idx, int nv, bool vec) {
  if (vec) return __builtin_nontemporal_load(reinterpret_cast<const f2_t*>(p + idx));
  f2_t v = {0.f, 0.f};
  if (nv > 0) v.x = p[idx];
  if (nv > 1) v.y = p[idx + 1];
  return v;
}
__device__ __forceinline__ void st2g(float* __restrict__ p, size_t idx, const f2_t& v, int nv, bool vec) {
  if (vec) {
    __builtin_nontemporal_store(v, reinterpret_cast<f2_t*>(p + idx));
    return;
  }
  if (nv > 0) p[idx] = v.x;
  if (nv > 1) p[idx + 1] = v.y;
}
constexpr int kRbBatch = 2;                   // K2 epilogue rows whose loads are in flight together (2: 0.351 ms K2, 4: 0.366, 1 per pixel before: 0.392)
constexpr int kRb1Batch = kRbRows;                 // K1: all 8 rows' loads in flight (2: 0.173 ms, 4: 0.170, 8: 0.167)

// Epilogue rows of a thread: rows i0 + 8ty + r, columns j, j + 1 (nv(r) valid of 2); the
// per-row index and count are recomputed (two registers live instead of sixteen).
struct RbRows {
  size_t base;        // plane_base + row0 * W + j
  int rows_left, ncol, W;
  __device__ __forceinline__ void init(size_t plane_base, int i0, int j, int H, int W_) {
    const int row0 = i0 + (threadIdx.x >> 5) * kRbRows;
    W = W_;
    ncol = j < W ? min(2, W - j) : 0;
    rows_left = H - row0;
    base = plane_base + (size_t)row0 * W + j;
  }
  __device__ __forceinline__ int nv(int r) const { return r < rows_left ? ncol : 0; }
  __device__ __forceinline__ size_t ix(int r) const { return base + (size_t)(r < rows_left ? r : 0) * W; }
};

// One plane as a buffer resource: loads take a 32-bit byte offset (no 64-bit address add per
// load) and return 0 past num_records (a null plane: every load 0).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const float* p, int H, int W) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, p ? H * W * 4 : 0, 0x00020000);
}
__device__ __forceinline__ float bld(__amdgpu_buffer_rsrc_t r, int idx) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, idx * 4, 0, 0));
}

// K1's halo fill, laid out as K2's rb_fill_k2_fast (the wrapped halo rows, then the tile's own
// rows by index adds; a ragged bottom row of tiles takes rb_fill_cols).  PEND: the plane holds
// v, K2's dual before the l2-ball step, and the fill applies K3's update per element, y =
// (1 - f)(v - g2 xobs) (l2_dual_y, the bits of k3_l2_dual), so K3's pass over y disappears.
template <class G, int NB, bool PEND>
__device__ __forceinline__ void rb_fill_k1(float* lds, int i0, int j0, int H, int W, const float* yp, const float* op,
                                           double omf, double g2) {
  if (i0 + kRbH > H) {
    rb_fill_cols<G, NB>(lds, i0, j0, H, W,
                        [&](int k) { return PEND ? l2_dual_y(yp[k], op[k], omf, g2) : yp[k]; });
    return;
  }
  constexpr int R = G::R, TPC = 256 / G::LW;
  constexpr int NH = (2 * R + TPC - 1) / TPC;        // halo rows per thread (the last may be past 2R)
  constexpr int NT = (kRbH + TPC - 1) / TPC;         // tile rows per thread (the last may be past kRbH)
  const int tid = threadIdx.x;
  if (tid >= TPC * G::LW) return;
  const int lx = tid % G::LW, ly0 = tid / G::LW;
  int gj = j0 - R + G::kOff + lx;
  gj += gj < 0 ? W : 0;
  gj -= gj >= W ? W : 0;
  gj = min(max(gj, 0), W - 1);
  const __amdgpu_buffer_rsrc_t ry = plane_rsrc(yp, H, W), ro = plane_rsrc(PEND ? op : nullptr, H, W);
  auto val = [&](float v, float o) { return PEND ? l2_dual_y(v, o, omf, g2) : v; };
  {
    float a[NH], bb[NH];
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int q = ly0 + TPC * k;                     // halo row q: LDS row q (above) or q + 64 (below)
      const int ly = q < R ? q : q + kRbH;
      int gi = i0 - R + ly;
      gi += gi < 0 ? H : 0;
      gi -= gi >= H ? H : 0;
      gi = min(max(gi, 0), H - 1);
      const int idx = gi * W + gj;
      a[k] = bld(ry, idx);
      bb[k] = PEND ? bld(ro, idx) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int q = ly0 + TPC * k;
      const int ly = q < R ? q : q + kRbH;
      if ((2 * R) % TPC == 0 || q < 2 * R) lds[ly * G::LW + lx] = val(a[k], bb[k]);
    }
  }
  int idx = (i0 + ly0) * W + gj;
#pragma unroll
  for (int k0 = 0; k0 < NT; k0 += NB) {
    float a[NB], bb[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      if (k0 + k < NT) {
        const int ii = (ly0 + TPC * (k0 + k) < kRbH) ? idx : idx - TPC * W;   // past the last tile row: any loaded row, not stored
        a[k] = bld(ry, ii);
        bb[k] = PEND ? bld(ro, ii) : 0.f;
        idx += TPC * W;
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int r = ly0 + TPC * (k0 + k);
      if (k0 + k < NT && (kRbH % TPC == 0 || r < kRbH)) lds[(R + r) * G::LW + lx] = val(a[k], bb[k]);
    }
  }
}

// K1: u = [clamp](x - g1 Phi^T y) -> u32 (the denoiser's input; its head converts to fp16);
// B (MB): w = s - g1 y.  Block = one (plane, 64 x 64 tile).  B's y comes
// from the halo in LDS (it is the stencil's input), so K1 reads y once.
// LAT (small grids, fewer blocks than CUs: B = 1): every halo load of a thread in flight at
// once instead of in batches of 8 (the batches keep registers low for 6 blocks per CU).
// PEND: y holds v and the fill applies K3's update (omf[b] = 1 - f from k3_norm); yout
// (nullable) receives the tile's y, the next K2's input (a separate buffer: other blocks
// still read v's halo).
template <class T, bool MB, int LAT = 0, bool PEND = false>
// (The batched variants at 7 waves per SIMD, 70-72 VGPRs: the LDS holds 7 blocks per CU; 0.207 -> 0.205 ms at
// the metric, 0.0815 -> 0.079 at cfg3, round 4.  K2 at 7 spilled 10 VGPRs and was no faster.)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LAT ? 1 : (TapGeom<T>::N * 4 * 7 <= 163840 ? 7 : 1))))
void k1_blur_rb(const float* __restrict__ x, const float* __restrict__ y,
                                                   const float* __restrict__ xobs, const double* __restrict__ omf,
                                                   double gamma2, float* __restrict__ yout,
                                                   const float* __restrict__ s, float* __restrict__ u32,
                                                   float* __restrict__ w, const f2_t* __restrict__ wd_adj, int C, int H,
                                                   int W, int tiles_x, int tiles, float gamma1, int clamp_in) {
  using G = TapGeom<T>;
  __shared__ float lds[G::N];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int bt = rb_block_tile();
  const int bc = bt / tiles;                            // plane (image, channel)
  int i0, j0;
  rb_tile_origin(bt - bc * tiles, tiles_x, i0, j0);
  const int j = j0 + 2 * tx;
  const size_t pb = (size_t)bc * H * W;
  const bool al = (W & 1) == 0;              // column pairs 8-B aligned
  RbRows rw;
  rw.init(pb, i0, j, H, W);
  const float* yp = y + pb;
  f2_t xv[kRb1Batch], sv[kRb1Batch];
  auto load_epi = [&](int rb) {                       // the loads of kRb1Batch rows in flight together
#pragma unroll
    for (int k = 0; k < kRb1Batch; ++k) {
      const bool vec = al && rw.nv(rb + k) == 2;
      xv[k] = ld2g(x, rw.ix(rb + k), rw.nv(rb + k), vec);
      if (MB) sv[k] = ld2g(s, rw.ix(rb + k), rw.nv(rb + k), vec);
    }
  };
  if (LAT) load_epi(0);                               // LAT: issued before the halo fill
  rb_fill_k1<G, LAT ? 32 : kRbFill, PEND>(lds, i0, j0, H, W, yp, PEND ? xobs + pb : nullptr,
                                          PEND ? omf[bc / C] : 0.0, gamma2);
  __syncthreads();
  f2_t g[kRbRows];
  rb_stencil<T>(lds, wd_adj, g);
  const float* yc = lds + (ty * kRbRows + G::R) * G::LW + 2 * tx + G::R - G::kOff;   // y at (row 0, col j)
  static_assert(!LAT || kRb1Batch == kRbRows, "LAT preloads every epilogue row");
#pragma unroll
  for (int rb = 0; rb < kRbRows; rb += kRb1Batch) {
    if (!LAT) load_epi(rb);
#pragma unroll
    for (int k = 0; k < kRb1Batch; ++k) {
      const int r = rb + k;
      f2_t uo, wo;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float uu = xv[k][q] - gamma1 * g[r][q];
        if (clamp_in) uu = fminf(fmaxf(uu, 0.f), 1.f);
        uo[q] = uu;
        if (MB) wo[q] = sv[k][q] - gamma1 * yc[r * G::LW + q];
      }
      const bool vec = al && rw.nv(r) == 2;
      st2g(u32, rw.ix(r), uo, rw.nv(r), vec);
      if (MB) st2g(w, rw.ix(r), wo, rw.nv(r), vec);
      if (yout) st2g(yout, rw.ix(r), f2_t{yc[r * G::LW], yc[r * G::LW + 1]}, rw.nv(r), vec);
    }
  }
}

// Standalone Phi / Phi^T of the blur (pnp_op_phi / pnp_op_adj_phi, comparisonB-2's x-step,
// the comparison methods): out = stencil(x) [+ add] on K1's register-blocked tiles (T: the
// forward or the adjoint tap pattern).  Block = one (plane, 64 x 64 tile).
template <class T, bool ADD>
__global__ __launch_bounds__(256) void k0_blur_rb(const float* __restrict__ x, float* __restrict__ out,
                                                   const float* __restrict__ add, const f2_t* __restrict__ wd, int H,
                                                   int W, int tiles_x, int tiles) {
  using G = TapGeom<T>;
  __shared__ float lds[G::N];
  const int tx = threadIdx.x & 31;
  const int bt = rb_block_tile();
  const int bc = bt / tiles;
  int i0, j0;
  rb_tile_origin(bt - bc * tiles, tiles_x, i0, j0);
  const size_t pb = (size_t)bc * H * W;
  const bool al = (W & 1) == 0;
  RbRows rw;
  rw.init(pb, i0, j0 + 2 * tx, H, W);
  const float* xp = x + pb;
  rb_fill_cols<G>(lds, i0, j0, H, W, [&](int k) { return xp[k]; });
  __syncthreads();
  f2_t g[kRbRows];
  rb_stencil<T>(lds, wd, g);
  if (ADD) {
    f2_t av[kRbRows];
#pragma unroll
    for (int r = 0; r < kRbRows; ++r) av[r] = ld2g(add, rw.ix(r), rw.nv(r), al && rw.nv(r) == 2);
#pragma unroll
    for (int r = 0; r < kRbRows; ++r) g[r] += av[r];
  }
#pragma unroll
  for (int r = 0; r < kRbRows; ++r) st2g(out, rw.ix(r), g[r], rw.nv(r), al && rw.nv(r) == 2);
}

// K2 halo fill of 2 xn - xo (Phi's argument) that also accumulates the metric sums of the
// tile's own pixels from the same loads: e2 = sum (xn - xo)^2, n2 = sum xo^2 (c_n,
// iteration.py:187) and t2 = sum (xt - xn)^2 (PSNR, :188; x_true loaded for those pixels
// only).  Column-wise (as rb_fill_cols): thread t < TPC LW owns LDS column t % LW and
// rows t / LW + TPC i, so the column's wrap and its "inside the tile" test are resolved once
// and a row step is an add, one conditional wrap and one row compare (the element-wise form
// of round 2 re-derived and wrapped row and column and tested both per element: 1 240 of the kernel's
// 2 555 VALU instructions per wave, against ~330 for K1's one-plane column fill).  The sums'
// fp32 groups are flushed into fp64 every kRbFill rows of a thread, whatever the load batch
// NB (the latency variant loads all rows at once), so both variants give the same bits.
template <class G, int NB = kRbFill>
__device__ __forceinline__ void rb_fill_k2_cols(float* lds, int i0, int j0, int H, int W, const float* xnp,
                                                const float* xop, const float* xtp, bool record, double& e2,
                                                double& n2, double& t2, float& lo, float& hi) {
  constexpr int TPC = 256 / G::LW;                   // threads per column (row stride)
  constexpr int NI = (G::LH + TPC - 1) / TPC;        // rows per thread (the last may be past LH)
  const int tid = threadIdx.x;
  if (tid >= TPC * G::LW) return;
  const int lx = tid % G::LW, ly0 = tid / G::LW;
  int gj = j0 - G::R + G::kOff + lx;
  const bool colin = record && gj >= j0 && gj < min(j0 + kRbW, W);   // a column of the tile's own pixels
  gj += gj < 0 ? W : 0;
  gj -= gj >= W ? W : 0;
  gj = min(max(gj, 0), W - 1);
  const int rhi = G::R + min(kRbH, H - i0);          // LDS rows R .. rhi-1: the tile's own rows
  int gi = i0 - G::R + ly0;
  gi += gi < 0 ? H : 0;
  gi -= gi >= H ? H : 0;
  float be = 0.f, bn = 0.f, bt = 0.f;
#pragma unroll
  for (int i0b = 0; i0b < NI; i0b += NB) {
    float a[NB], bb[NB], t[NB];
    bool in[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if (i0b + i < NI) {
        const int ly = ly0 + TPC * (i0b + i);
        const int idx = min(max(gi, 0), H - 1) * W + gj;
        a[i] = xnp[idx];
        bb[i] = xop[idx];
        in[i] = colin && ly >= G::R && ly < rhi;
        t[i] = (in[i] && xtp) ? xtp[idx] : 0.f;
        gi += TPC;
        gi -= gi >= H ? H : 0;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if (i0b + i < NI) {
        if ((i0b + i) % kRbFill == 0) {                // fp32 groups of kRbFill rows whatever NB: same bits
          e2 += be;
          n2 += bn;
          t2 += bt;
          be = bn = bt = 0.f;
        }
        const int ly = ly0 + TPC * (i0b + i);
        if (G::LH % TPC == 0 || ly < G::LH) lds[ly * G::LW + lx] = 2.f * a[i] - bb[i];
        const float d = in[i] ? a[i] - bb[i] : 0.f, o = in[i] ? bb[i] : 0.f;
        const float tt = in[i] ? t[i] - a[i] : 0.f;
        be = fmaf(d, d, be);
        bn = fmaf(o, o, bn);
        bt = fmaf(tt, tt, bt);
        lo = in[i] ? fminf(lo, a[i]) : lo;            // x+ range for SSIM's data_range (utils_eval.py:11)
        hi = in[i] ? fmaxf(hi, a[i]) : hi;
      }
    }
  }
  e2 += be;
  n2 += bn;
  t2 += bt;
}

// K2's fill for tiles whose 64 rows lie inside the image (all but a ragged bottom row of
// tiles, which takes rb_fill_k2_cols): the 2R halo rows above and below first (wrapped), then
// the tile's own rows, which need no wrap or clamp (a row step is an index add) and no
// per-element "inside" test: a thread's column is inside the tile or not, so the sums of a
// batch are kept or dropped once per batch.
template <class G, int NB = kRbFill, bool XT = true>   // XT false: no x_true (no loads, t2 stays 0)
__device__ __forceinline__ void rb_fill_k2_fast(float* lds, int i0, int j0, int H, int W, const float* xnp,
                                                const float* xop, const float* xtp, bool record, double& e2,
                                                double& n2, double& t2, float& lo, float& hi) {
  if (i0 + kRbH > H) {
    rb_fill_k2_cols<G, NB>(lds, i0, j0, H, W, xnp, xop, xtp, record, e2, n2, t2, lo, hi);
    return;
  }
  constexpr int R = G::R, TPC = 256 / G::LW;
  constexpr int NH = (2 * R + TPC - 1) / TPC;        // halo rows per thread (the last may be past 2R)
  constexpr int NT = (kRbH + TPC - 1) / TPC;         // tile rows per thread (the last may be past kRbH)
  const int tid = threadIdx.x;
  if (tid >= TPC * G::LW) return;
  const int lx = tid % G::LW, ly0 = tid / G::LW;
  int gj = j0 - R + G::kOff + lx;
  const bool colin = record && gj >= j0 && gj < min(j0 + kRbW, W);
  gj += gj < 0 ? W : 0;
  gj -= gj >= W ? W : 0;
  gj = min(max(gj, 0), W - 1);
  const __amdgpu_buffer_rsrc_t rn = plane_rsrc(xnp, H, W), ro = plane_rsrc(xop, H, W);
  const __amdgpu_buffer_rsrc_t rt = plane_rsrc(record ? xtp : nullptr, H, W);   // none: loads of 0
  {
    float a[NH], bb[NH];
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int q = ly0 + TPC * k;                     // halo row q: LDS row q (above) or q + 64 (below)
      const int ly = q < R ? q : q + kRbH;
      int gi = i0 - R + ly;
      gi += gi < 0 ? H : 0;
      gi -= gi >= H ? H : 0;
      gi = min(max(gi, 0), H - 1);
      const int idx = gi * W + gj;
      a[k] = bld(rn, idx);
      bb[k] = bld(ro, idx);
    }
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int q = ly0 + TPC * k;
      const int ly = q < R ? q : q + kRbH;
      if ((2 * R) % TPC == 0 || q < 2 * R) lds[ly * G::LW + lx] = 2.f * a[k] - bb[k];
    }
  }
  int idx = (i0 + ly0) * W + gj;
  float be = 0.f, bn = 0.f, bt = 0.f, bl = lo, bh = hi;
  auto flush = [&] {
    if (colin) {
      e2 += be;
      n2 += bn;
      t2 += bt;
    }
    be = bn = bt = 0.f;
  };
#pragma unroll
  for (int k0 = 0; k0 < NT; k0 += NB) {
    float a[NB], bb[NB], t[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      if (k0 + k < NT) {
        const int ii = (ly0 + TPC * (k0 + k) < kRbH) ? idx : idx - TPC * W;   // past the last tile row: any loaded row, not stored
        a[k] = bld(rn, ii);
        bb[k] = bld(ro, ii);
        t[k] = XT ? bld(rt, ii) : 0.f;
        idx += TPC * W;
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      if (k0 + k < NT) {
        if ((k0 + k) % kRbFill == 0) flush();        // fp32 groups of kRbFill rows whatever NB: same bits
        const int r = ly0 + TPC * (k0 + k);
        const bool ok = kRbH % TPC == 0 || r < kRbH;
        if (ok) lds[(R + r) * G::LW + lx] = 2.f * a[k] - bb[k];
        const float d = a[k] - bb[k], tt = t[k] - a[k];
        const float o = bb[k];
        be = fmaf(ok ? d : 0.f, d, be);
        bn = fmaf(ok ? o : 0.f, o, bn);
        if (XT) bt = fmaf(ok ? tt : 0.f, tt, bt);
        bl = ok ? fminf(bl, a[k]) : bl;               // x+ range for SSIM's data_range (utils_eval.py:11)
        bh = ok ? fmaxf(bh, a[k]) : bh;
      }
    }
  }
  flush();
  if (colin) {
    lo = bl;
    hi = bh;
  }
}

// K2: v = y + g2 (Phi(2x+ - x) [+ 2 s+ - s]), s+ = shrink(w, theta) (B), the GKL prox (C),
// per-cell partial sums.  Block = one (plane, 64 x 64 tile).  The metric sums come from the
// fill's own loads of xn / xo (plus x_true for the tile's pixels) and are reduced before the
// barrier (no fill value stays live through the stencil), so the epilogue reads only y and
// x_obs (and B's s, w) and nothing is read twice.  partials: [B][cells][C][4] (per 32 x 32
// cell and channel), reduced by k3 in that order: d2 per cell, e2 / n2 / t2 per tile in the
// tile's first cell (zeros in the others).
// ABL (PNP_PROFILING build only, results wrong): phases of K2 removed for the ablation legs of
// tools/gpu_r05_run1.sh: 1 no stencil (each output takes one LDS value), 2 no fp64 partials
// (no metric sums, no d2), 4 no epilogue stores, 8 no halo fill, 16 no epilogue loads, 64 no
// x_true loads (PSNR wrong, the rest right).
// XT: x_true given (false when the SSIM pass sums the PSNR's squared error: no x_true stream)
template <class T, int METHOD, int LAT = 0, int ABL = 0, bool XT = true>   // LAT: as k1_blur_rb, and all 8 epilogue rows' loads in flight
__global__ __launch_bounds__(256) void k2_blur_rb(const float* __restrict__ xn, const float* __restrict__ xo,
                                                   float* __restrict__ y, const float* __restrict__ xobs,
                                                   const float* __restrict__ xtrue, float* __restrict__ s,
                                                   const float* __restrict__ w, const float* __restrict__ theta,
                                                   double* __restrict__ partials, const f2_t* __restrict__ wd_fwd,
                                                   int C, int H, int W, int tiles_x, int tiles, int cells_x, int cells,
                                                   double gamma2, double inv_g2, double gkl_gamma, double gkl_alpha,
                                                   int record, float* __restrict__ mm) {
  using G = TapGeom<T>;
  __shared__ float lds[G::N];
  __shared__ double red[4][2];
  __shared__ double redm[4][3];
  const int tx = threadIdx.x & 31;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bt = rb_block_tile();
  const int bc = bt / tiles, b = bc / C, c = bc - b * C;
  int i0, j0;
  rb_tile_origin(bt - bc * tiles, tiles_x, i0, j0);
  const size_t plane = (size_t)H * W;
  const int j = j0 + 2 * tx;
  const bool al = (W & 1) == 0;              // column pairs 8-B aligned
  RbRows rw;
  rw.init((size_t)bc * plane, i0, j, H, W);
  __shared__ float redr[4][2];
  // EB rows at a time: every stream's loads of the batch are issued before the first use.
  // LAT: all 8 rows, issued before the halo fill (their latency hides behind it)
  constexpr int EB = LAT ? kRbRows : kRbBatch;
  f2_t yv[EB], bv[EB], sv[EB], wv[EB];
  auto load_epi = [&](int rb) {
#pragma unroll
    for (int k = 0; k < EB; ++k) {
      if (ABL & 16) {
        yv[k] = bv[k] = sv[k] = wv[k] = f2_t{0.25f * (float)k, (float)rb};
        continue;
      }
      const bool vec = al && rw.nv(rb + k) == 2;
      yv[k] = ld2g(y, rw.ix(rb + k), rw.nv(rb + k), vec);
      bv[k] = ld2g(xobs, rw.ix(rb + k), rw.nv(rb + k), vec);
      if (METHOD == M_B) {
        sv[k] = ld2g(s, rw.ix(rb + k), rw.nv(rb + k), vec);
        wv[k] = ld2g(w, rw.ix(rb + k), rw.nv(rb + k), vec);
      }
    }
  };
  if (LAT) load_epi(0);
  if (ABL & 2) record = 0;
  {
    double e2 = 0, n2 = 0, t2 = 0;
    float lo = __builtin_inff(), hi = -__builtin_inff();
    if (!(ABL & 8))
      rb_fill_k2_fast<G, LAT ? 32 : kRbFill, XT>(lds, i0, j0, H, W, xn + (size_t)bc * plane, xo + (size_t)bc * plane,
                                            (xtrue && !(ABL & 64)) ? xtrue + (size_t)bc * plane : nullptr,
                                            record != 0, e2, n2, t2, lo, hi);
    if (record) {                            // reduced here, so no fill value stays live past the fill
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
  __syncthreads();
  if (record && mm && threadIdx.x == 0) {    // per (image, channel, tile): [B][C * tiles][2]
    const size_t chunk = (size_t)b * C * tiles + (size_t)c * tiles + (bt - bc * tiles);
    mm[chunk * 2 + 0] = fminf(fminf(redr[0][0], redr[1][0]), fminf(redr[2][0], redr[3][0]));
    mm[chunk * 2 + 1] = fmaxf(fmaxf(redr[0][1], redr[1][1]), fmaxf(redr[2][1], redr[3][1]));
  }
  f2_t g[kRbRows];
  if (ABL & 1) {
#pragma unroll
    for (int r = 0; r < kRbRows; ++r) {
      const float* bp = lds + ((threadIdx.x >> 5) * kRbRows + r + G::R) * G::LW + 2 * tx;
      g[r] = f2_t{bp[0], bp[1]};
    }
  } else {
    rb_stencil<T>(lds, wd_fwd, g);
  }
  // The dual update and the l2-ball partial in fp64 (v is rounded to float32 for the state).  A
  // float32 form for ours-A measured the same time (r05 A/B on one box: 0.2717-0.2733 vs
  // 0.2698-0.2735 ms, profiles/r05/k2_ablation.txt) and moved ours-B's ill-conditioned sigma-0.04
  // golden, so it was not kept.
  double d2 = 0;
  {
    const float th = METHOD == M_B ? theta[b] : 0.f;
#pragma unroll
    for (int rb = 0; rb < kRbRows; rb += EB) {
      if (!LAT) load_epi(rb);
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        const int r = rb + k;
        f2_t yo = yv[k], so = {0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (q >= rw.nv(r)) break;
          double gv = g[r][q];
          if (METHOD == M_B) {
            const float wq = wv[k][q];
            const float sp = copysignf(fmaxf(fabsf(wq) - th, 0.f), wq);   // operators.py:98
            gv += 2.0 * (double)sp - (double)sv[k][q];
            so[q] = sp;
          }
          const double v = (double)yv[k][q] + gamma2 * gv;
          const double ob = bv[k][q];
          if (METHOD == M_C) {
            const double tt = v * inv_g2 - gkl_gamma * gkl_alpha;
            const double p = 0.5 * (tt + sqrt(tt * tt + 4.0 * gkl_gamma * ob));
            yo[q] = (float)(v - gamma2 * p);
          } else {
            yo[q] = (float)v;
            if (!(ABL & 2)) {
              const double dd = v * inv_g2 - ob;
              d2 += dd * dd;
            }
          }
        }
        const bool vec = al && rw.nv(r) == 2;
        if ((ABL & 4) && !(yo[0] == 1234.5f && gamma2 == -7.0)) continue;   // keeps the values live
        st2g(y, rw.ix(r), yo, rw.nv(r), vec);
        if (METHOD == M_B) st2g(s, rw.ix(r), so, rw.nv(r), vec);
      }
    }
  }
  // d2: a wave is two thread rows (2 kRbRows tile rows) x 32 threads; a 32 x 32 cell is 16
  // threads (tx) of WPC = 32 / (2 kRbRows) waves: reduce each wave's two column halves in the
  // wave (lanes {c, c+32}: xor 32, then xor 8..1), then combine the cell's waves through LDS
  // in a fixed order.  e2 / n2 / t2: whole tile, fixed order.
  auto half_sum = [](double v) {
    v += __shfl_xor(v, 32, 64);
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
  d2 = half_sum(d2);
  if ((lane & 47) == 0) red[wave][lane >> 4] = d2;   // lanes 0 / 16: the wave's two half-cells
  __syncthreads();
  constexpr int CY = kRbH / 32, WPC = 4 / CY;          // cell rows per tile, waves per cell
  if (threadIdx.x < 8 * CY) {                          // CY x 2 cells x 4 sums
    const int cell = threadIdx.x >> 2, k = threadIdx.x & 3, cy = cell >> 1, cx = cell & 1;
    const int gy = i0 / 32 + cy, gx = j0 / 32 + cx;
    double v = 0.0;
    if (k == 0) {
      v = red[WPC * cy][cx];
#pragma unroll
      for (int q = 1; q < WPC; ++q) v += red[WPC * cy + q][cx];
    } else if (record && cell == 0) v = ((redm[0][k - 1] + redm[1][k - 1]) + redm[2][k - 1]) + redm[3][k - 1];
    if (gy * 32 < H && gx < cells_x)
      partials[(((size_t)b * cells + (size_t)gy * cells_x + gx) * C + c) * 4 + k] = v;
  }
}

// =====================================================================================
// SSIM (utils/utils_eval.py:9-12): skimage.metrics.structural_similarity(x_true, x,
// data_range = x.max() - x.min(), channel_axis = 0), scikit-image 0.22.0 defaults:
// 7-wide uniform window (scipy uniform_filter: axis 0 then axis 1, float32 between the
// passes), K1 = 0.01, K2 = 0.03, sample covariance, float32 map, mean over the map
// cropped by 3.  channel_axis=0: RGB (C,H,W) -> mean of C 2-D SSIMs; grayscale (H,W) ->
// mean of H 1-D SSIMs over the rows (skimage loops over axis 0).  Cropped pixels' windows
// never leave the image, so no boundary mode is needed.
//   ssim_minmax:  per-image min/max partials of x           (data_range)
//   ssim_rgb:     per (32x32 tile, channel) sums of the cropped SSIM map
//   ssim_gray:    per-row means of the 1-D SSIM map
//   ssim_final:   per image, fixed-order reduction -> metrics[b][it][2]
// =====================================================================================
__global__ __launch_bounds__(256) void ssim_minmax_kernel(const float* __restrict__ x, float* __restrict__ mm,
                                                          size_t n, int chunks) {
  __shared__ float red[2][4];
  const int b = blockIdx.y;
  const size_t beg = (size_t)blockIdx.x * 2048;
  float lo = __builtin_inff(), hi = -__builtin_inff();
  for (size_t k = beg + threadIdx.x; k < beg + 2048 && k < n; k += 256) {
    const float v = x[(size_t)b * n + k];
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o, 64));
    hi = fmaxf(hi, __shfl_xor(hi, o, 64));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = lo; red[1][w] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = red[0][0], c = red[1][0];
    for (int i = 1; i < 4; ++i) { a = fminf(a, red[0][i]); c = fmaxf(c, red[1][i]); }
    mm[((size_t)b * chunks + blockIdx.x) * 2 + 0] = a;
    mm[((size_t)b * chunks + blockIdx.x) * 2 + 1] = c;
  }
}

// data_range of image b from the minmax partials: one wave, lanes stride the chunks
__device__ __forceinline__ float ssim_range_wave(const float* __restrict__ mm, int b, int chunks, int lane) {
  float lo = __builtin_inff(), hi = -__builtin_inff();
  for (int k = lane; k < chunks; k += 64) {
    lo = fminf(lo, mm[((size_t)b * chunks + k) * 2 + 0]);
    hi = fmaxf(hi, mm[((size_t)b * chunks + k) * 2 + 1]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o, 64));
    hi = fmaxf(hi, __shfl_xor(hi, o, 64));
  }
  return hi - lo;                                  // im2.max() - im2.min() in float32
}

__device__ __forceinline__ float ssim_s(float ux, float uy, float uxx, float uyy, float uxy, float cov_norm,
                                        float C1, float C2) {
#pragma clang fp contract(off)   // numpy rounds every product and sum to float32
  const float vx = cov_norm * (uxx - ux * ux);
  const float vy = cov_norm * (uyy - uy * uy);
  const float vxy = cov_norm * (uxy - ux * uy);
  const float A1 = 2.f * ux * uy + C1, A2 = 2.f * vxy + C2;
  const float B1 = ux * ux + uy * uy + C1, B2 = vx + vy + C2;
  // the quotient by the hardware reciprocal and one Newton step (within 1 ulp of numpy's IEEE
  // division; 3 instructions instead of v_div_scale / fmas / fixup's ~10)
  const float n = A1 * A2, d = B1 * B2;
  const float r = __builtin_amdgcn_rcpf(d);
  const float q = n * r;
  return fmaf(fmaf(-d, q, n), r, q);
}

// Window sums in float32 (round 5): running sums over 8 outputs per thread
// (a direct 7-term sum, then + new - old), the mean as sum * (1/7).  Rounds 2-4 kept float64
// running sums, exact for these magnitudes, to reproduce scipy's float64 accumulation bit for
// bit, at ~128 VALU instructions per pixel (half of them fp64 and its conversions: 0.23 ms at the
// metric, 22 % of HBM).  In float32 a window mean is within a few float32 ulps of scipy's, and the
// image SSIM within ~5e-6 of the restatement (numpy emulation on the metric's images; test
// tolerance 2e-5); the SSIM map and the per-tile sums are as before.
constexpr float kInv7f = 1.f / 7.f;
// Output tile 56 x 32: the vertical sums of its 62 columns take one pass of a 64-lane wave,
// the horizontal pass 7 segments of 8 columns per row, and the LDS (40 KiB) fits 4 blocks
// per CU.  (64 x 32 with 70 columns: two vertical passes, 45 KiB, 3 blocks: 0.30 ms.)
constexpr int kSsTW = 56, kSsTH = 32;
constexpr int kSsVW = kSsTW + 6, kSsVS = 63;      // odd LDS row stride

// grid (tiles, B*C), block 256 = 4 waves.  Vertical pass: thread (column, 8-row segment) with
// running sums straight from HBM/L2; horizontal pass: thread (row, 8-column segment) with
// running sums over LDS.  ps[bc][tile] = sum of S over the tile's cropped pixels.
// t2o (PSNR from this pass, round 5): per (bc, tile) the sum of (xt - x)^2 over the tile's own
// pixels, from the vertical pass's loads (K2 then skips its x_true loads: 16 % of its bytes).
__global__ __launch_bounds__(256) void ssim_rgb_kernel(const float* __restrict__ xt, const float* __restrict__ x,
                                                       const float* __restrict__ mm, double* __restrict__ ps,
                                                       double* __restrict__ t2o, int C, int H, int W, int tiles_x,
                                                       int tiles, int chunks) {
  // Two LDS phases (round 5): the axis-0 means of x and y, then of xx, yy and xy, through one
  // 3-quantity array (24 KiB instead of 40: 6 blocks per CU instead of 4); the horizontal pass
  // keeps its 8 outputs' x / y means in registers between them.  Same arithmetic per quantity.
  __shared__ float v[3][kSsTH][kSsVS];
  __shared__ double red[4];
  __shared__ float cst[2];
  const int tile = blockIdx.x, bc = blockIdx.y, b = bc / C;
  const int i0 = (tile / tiles_x) * kSsTH, j0 = (tile % tiles_x) * kSsTW;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (wv == 0) {
    const float R = ssim_range_wave(mm, b, chunks, lane);
    if (lane == 0) { cst[0] = (0.01f * R) * (0.01f * R); cst[1] = (0.03f * R) * (0.03f * R); }
  }
  const __amdgpu_buffer_rsrc_t qa = plane_rsrc(xt + (size_t)bc * H * W, H, W);
  const __amdgpu_buffer_rsrc_t qb = plane_rsrc(x + (size_t)bc * H * W, H, W);
  // ---- vertical loads: columns j0-3+c (c < 62), rows i0 + 8*wv - 3 .. +14 ----
  float se = 0.f;                                  // this thread's own pixels' sum of (xt - x)^2
  const bool vcol = lane < kSsVW;
  const int c = lane;
  float ra[14], rb[14];
  if (vcol) {
    const int gj = min(max(j0 - 3 + c, 0), W - 1);
    const int r0 = i0 + 8 * wv;
    if (__builtin_amdgcn_readfirstlane((int)(r0 >= 3 && r0 + 11 <= H))) {   // no row clamp: an index add per row
      int idx = (r0 - 3) * W + gj;
#pragma unroll
      for (int d = 0; d < 14; ++d, idx += W) {
        ra[d] = bld(qa, idx);
        rb[d] = bld(qb, idx);
      }
    } else {
#pragma unroll
      for (int d = 0; d < 14; ++d) {
        const int idx = min(max(r0 - 3 + d, 0), H - 1) * W + gj;
        ra[d] = bld(qa, idx);
        rb[d] = bld(qb, idx);
      }
    }
    if (t2o && c >= 3 && c < kSsTW + 3 && j0 - 3 + c < W) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float dd = ra[k + 3] - rb[k + 3];
        se = r0 + k < H ? fmaf(dd, dd, se) : se;
      }
    }
    // phase A: the x and y means
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int d = 0; d < 7; ++d) {
      s0 += ra[d]; s1 += rb[d];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k) {
        s0 = (s0 + ra[k + 6]) - ra[k - 1];
        s1 = (s1 + rb[k + 6]) - rb[k - 1];
      }
      const int r = 8 * wv + k;
      v[0][r][c] = s0 * kInv7f;
      v[1][r][c] = s1 * kInv7f;
    }
  }
  __syncthreads();
  // ---- horizontal + SSIM map: row r = t % 32, columns 8*(t / 32) .. +8 (segments 0..6): the
  // 32 lanes of a ds_read_b32 group read one column of 32 rows, stride 63 = -1 mod 32 banks,
  // conflict-free (rows-within-a-lane-group mapping t / 8 had every bank hit twice) ----
  const int r = threadIdx.x & 31, c0 = (threadIdx.x >> 5) * 8;
  const int i = i0 + r;
  const bool hrow = c0 < kSsTW && i >= 3 && i < H - 3;
  float ux[8], uy[8];
  if (hrow) {
    float h0 = 0.f, h1 = 0.f;
#pragma unroll
    for (int d = 0; d < 7; ++d) {
      h0 += v[0][r][c0 + d];
      h1 += v[1][r][c0 + d];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k) {
        h0 = (h0 + v[0][r][c0 + k + 6]) - v[0][r][c0 + k - 1];
        h1 = (h1 + v[1][r][c0 + k + 6]) - v[1][r][c0 + k - 1];
      }
      ux[k] = h0 * kInv7f;
      uy[k] = h1 * kInv7f;
    }
  }
  __syncthreads();
  // phase B: the xx, yy and xy means
  if (vcol) {
    float s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
    for (int d = 0; d < 7; ++d) {
      s2 = fmaf(ra[d], ra[d], s2); s3 = fmaf(rb[d], rb[d], s3); s4 = fmaf(ra[d], rb[d], s4);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k) {
        const float na = ra[k + 6], nb = rb[k + 6], oa = ra[k - 1], ob = rb[k - 1];
        s2 = fmaf(-oa, oa, fmaf(na, na, s2));
        s3 = fmaf(-ob, ob, fmaf(nb, nb, s3));
        s4 = fmaf(-oa, ob, fmaf(na, nb, s4));
      }
      const int rr = 8 * wv + k;
      v[0][rr][c] = s2 * kInv7f;
      v[1][rr][c] = s3 * kInv7f;
      v[2][rr][c] = s4 * kInv7f;
    }
  }
  __syncthreads();
  const float C1 = cst[0], C2 = cst[1];
  float acc = 0.f;
  if (hrow) {
    float h[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      float t = 0.f;
#pragma unroll
      for (int d = 0; d < 7; ++d) t += v[u][r][c0 + d];
      h[u] = t;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k) {
#pragma unroll
        for (int u = 0; u < 3; ++u) h[u] = (h[u] + v[u][r][c0 + k + 6]) - v[u][r][c0 + k - 1];
      }
      const int j = j0 + c0 + k;
      if (j >= 3 && j < W - 3)
        acc += ssim_s(ux[k], uy[k], h[0] * kInv7f, h[1] * kInv7f, h[2] * kInv7f, 49.f / 48.f, C1, C2);
    }
  }
  const double tot = block_sum((double)acc, red);
  if (threadIdx.x == 0) ps[(size_t)bc * tiles + tile] = tot;
  if (t2o) {
    const double te = block_sum((double)se, red);
    if (threadIdx.x == 0) t2o[(size_t)bc * tiles + tile] = te;
  }
}

// grayscale: grid (ceil(H/4), B), one wave per row; rows[b][row] = mean S of the row (float32)
__global__ __launch_bounds__(256) void ssim_gray_kernel(const float* __restrict__ xt, const float* __restrict__ x,
                                                        const float* __restrict__ mm, float* __restrict__ rows,
                                                        double* __restrict__ t2o, int H, int W, int chunks) {
  const int b = blockIdx.y, row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= H) return;
  const float R = ssim_range_wave(mm, b, chunks, lane);
  const float C1 = (0.01f * R) * (0.01f * R), C2 = (0.03f * R) * (0.03f * R);
  const float* a = xt + ((size_t)b * H + row) * W;
  const float* e = x + ((size_t)b * H + row) * W;
  double acc = 0;
  for (int j = 3 + lane; j < W - 3; j += 64) {
    float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = -3; d <= 3; ++d) {
      const float p = a[j + d], q = e[j + d];
      s[0] += p; s[1] += q; s[2] = fmaf(p, p, s[2]); s[3] = fmaf(q, q, s[3]); s[4] = fmaf(p, q, s[4]);
    }
    acc += (double)ssim_s(s[0] * kInv7f, s[1] * kInv7f, s[2] * kInv7f, s[3] * kInv7f, s[4] * kInv7f, 7.f / 6.f, C1, C2);
  }
  acc = wave_sum(acc);
  if (lane == 0) rows[(size_t)b * H + row] = (float)(acc / (double)(W - 6));
  if (t2o) {                                       // PSNR: the row's sum of (xt - x)^2
    float se = 0.f;
    for (int j = lane; j < W; j += 64) {
      const float dd = a[j] - e[j];
      se = fmaf(dd, dd, se);
    }
    const double te = wave_sum((double)se);
    if (lane == 0) t2o[(size_t)b * H + row] = te;
  }
}

// per image: RGB mean over channels of (sum S / cropped count); gray mean over rows
// t2o: PSNR (utils_eval.py:4-7) from the SSIM pass's squared-error sums, fixed order (or null)
__global__ __launch_bounds__(256) void ssim_final_kernel(const double* __restrict__ ps, const float* __restrict__ rows,
                                                         const double* __restrict__ t2o, double* __restrict__ metrics,
                                                         int C, int H, int W, int tiles, int gray, int it, int cap,
                                                         const int* __restrict__ itp) {
  __shared__ double red[4];
  const int b = blockIdx.x;
  if (itp) it = *itp;
  if (it >= cap) return;
  if (t2o) {
    const int nq = gray ? H : C * tiles;
    double a = 0;
    for (int q = threadIdx.x; q < nq; q += 256) a += t2o[(size_t)b * nq + q];
    const double t2 = block_sum(a, red);
    if (threadIdx.x == 0)
      metrics[((size_t)b * cap + it) * kMetrics + 1] = 10.0 * log10(1.0 / (t2 / ((double)C * H * W)));
  }
  double val;
  if (gray) {
    double a = 0;
    for (int r = threadIdx.x; r < H; r += 256) a += rows[(size_t)b * H + r];
    val = block_sum(a, red) / H;
  } else {
    const double cnt = (double)(H - 6) * (double)(W - 6);
    double m = 0;
    for (int c = 0; c < C; ++c) {
      double a = 0;
      for (int t = threadIdx.x; t < tiles; t += 256) a += ps[((size_t)b * C + c) * tiles + t];
      m += (double)(float)(block_sum(a, red) / cnt);   // each channel's mssim is stored as float32
    }
    val = m / C;
  }
  if (threadIdx.x == 0) metrics[((size_t)b * cap + it) * kMetrics + 2] = (double)(float)val;
}

// =====================================================================================
// comparisonB-2 (ADMM with denoiser, iteration.py:127-132, admm.py:30-44): elementwise
// linear combinations and the per-image c_n / PSNR partial sums.
// =====================================================================================
struct LinComb {
  double k, c[4];
  const float* in[4];
};
// out = k + sum_q c[q] * in[q]   (null inputs skipped), evaluated in fp64
__global__ __launch_bounds__(256) void lincomb_kernel(float* __restrict__ out, LinComb lc, size_t count) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (size_t)gridDim.x * 256) {
    double v = lc.k;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (lc.in[q]) v += lc.c[q] * (double)lc.in[q][i];
    out[i] = (float)v;
  }
}

// partials [B][chunks][4] = {0, sum (xn - xo)^2, sum xo^2, sum (xt - xn)^2}, grid (chunks, B)
__global__ __launch_bounds__(256) void metric_partials_kernel(const float* __restrict__ xn,
                                                               const float* __restrict__ xo,
                                                               const float* __restrict__ xt,
                                                               double* __restrict__ partials, size_t n, int chunks) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  const size_t beg = (size_t)blockIdx.x * 2048;
  double e2 = 0, n2 = 0, t2 = 0;
  for (size_t k = beg + threadIdx.x; k < beg + 2048 && k < n; k += 256) {
    const size_t i = (size_t)b * n + k;
    const double a = xn[i], o = xo[i];
    e2 += (a - o) * (a - o);
    n2 += o * o;
    if (xt) {
      const double q = (double)xt[i] - a;
      t2 += q * q;
    }
  }
  e2 = block_sum(e2, red);
  n2 = block_sum(n2, red);
  t2 = block_sum(t2, red);
  if (threadIdx.x == 0) {
    double* p = partials + ((size_t)b * chunks + blockIdx.x) * 4;
    p[0] = 0; p[1] = e2; p[2] = n2; p[3] = t2;
  }
}

// =====================================================================================
// Launchers (host)
// =====================================================================================
struct TileGrid {
  int tiles_x, tiles_y, tiles;
};
inline TileGrid tile_grid(int H, int W) {
  TileGrid g;
  g.tiles_x = (W + kST - 1) / kST;
  g.tiles_y = (H + kST - 1) / kST;
  g.tiles = g.tiles_x * g.tiles_y;
  return g;
}

// The register-blocked kernels wrap the halo once (their fills): images at least Rd on a side.
// Smaller ones (np.pad 'wrap' repeats the image) take the modulo-wrapped stencil4 kernels.
static bool rb_ok(const OpDesc& op, int C, int H, int W) {
  return op.kind == OP_BLUR && op.dense_fwd && op.dense_adj && op.Rd > 0 && C >= 1 && H >= op.Rd && W >= op.Rd;
}

template <class T>
static void launch_k1_rb(hipStream_t st, const float* x, const float* y, const float* s, float* u32, float* w,
                         const OpDesc& op, int B, int C, int H, int W, float gamma1, int clamp_in, int method_b,
                         const float* xobs = nullptr, const double* omf = nullptr, double gamma2 = 0.0,
                         float* yout = nullptr, bool pend = false) {
  const int tx = (W + kRbW - 1) / kRbW, tiles = tx * ((H + kRbH - 1) / kRbH);
  const bool lat = B * C * tiles < op.num_cus;     // one block per CU at most: latency-bound
#define K1RBL(MBV, L, PD)                                                                                   \
  hipLaunchKernelGGL((k1_blur_rb<T, MBV, L, PD>), dim3(B * C * tiles), dim3(256), 0, st, x, y, xobs, omf,   \
                     gamma2, yout, s, u32, w, reinterpret_cast<const f2_t*>(op.dense_adj), C, H, W, tx, tiles, \
                     gamma1, clamp_in)
#define K1RBP(MBV, PD) if (lat) K1RBL(MBV, 1, PD); else K1RBL(MBV, 0, PD);
  if (pend) { if (method_b) { K1RBP(true, true) } else { K1RBP(false, true) } }
  else { if (method_b) { K1RBP(true, false) } else { K1RBP(false, false) } }
#undef K1RBP
#undef K1RBL
}

bool k1_fused_ok(const OpDesc& op, int C, int H, int W) { return op.kind == OP_BLUR && rb_ok(op, C, H, W); }

void launch_k1_fused(const float* x, const float* y, const float* xobs, const double* omf, double gamma2, bool pend,
                     float* yout, const float* s, float* u32, float* w, const OpDesc& op, int B, int C, int H, int W,
                     float gamma1, int clamp_in, int method_b, hipStream_t st) {
#define K1RB(TT) launch_k1_rb<TT>(st, x, y, s, u32, w, op, B, C, H, W, gamma1, clamp_in, method_b, xobs, omf, gamma2, \
                                  yout, pend)
  switch (op.taps_id) {
    case TAPS_BLUR_1: K1RB(Taps_blur_1_Adj); break;
    case TAPS_SQUARE_MINI: K1RB(Taps_square_mini_Adj); break;
    default:
      switch (op.Rd) { case 2: K1RB(DenseTaps<2>); break; case 4: K1RB(DenseTaps<4>); break; default: K1RB(DenseTaps<8>); }
  }
#undef K1RB
}

void launch_k3_norm(const double* partials, const OpDesc& op, int B, int C, int H, int W, double eps, double* omf,
                    double* metrics, int it, int cap, int record, int has_true, hipStream_t st, const int* itp) {
  hipLaunchKernelGGL(k3_norm, dim3(B), dim3(256), 0, st, partials, k2_partials(op, C, H, W), (size_t)C * H * W, eps,
                     omf, metrics, it, cap, record, has_true, itp);
}

void launch_k1(int kind, const float* x, const float* y, const float* s, float* u32, float* w,
               const OpDesc& op, int B, int C, int H, int W, float gamma1, int clamp_in, int method_b,
               hipStream_t st) {
  if (kind == OP_BLUR && rb_ok(op, C, H, W)) {
#define K1RB(TT) launch_k1_rb<TT>(st, x, y, s, u32, w, op, B, C, H, W, gamma1, clamp_in, method_b)
    switch (op.taps_id) {
      case TAPS_BLUR_1: K1RB(Taps_blur_1_Adj); break;
      case TAPS_SQUARE_MINI: K1RB(Taps_square_mini_Adj); break;
      default:
        switch (op.Rd) { case 2: K1RB(DenseTaps<2>); break; case 4: K1RB(DenseTaps<4>); break; default: K1RB(DenseTaps<8>); }
    }
#undef K1RB
    return;
  }
  const TileGrid g = tile_grid(H, W);
  dim3 grid(g.tiles, B);
#define K1_ARGS x, y, s, u32, w, op, C, H, W, g.tiles_x, gamma1, clamp_in, method_b
#define K1E_ARGS x, y, s, u32, w, op.mask, C, H, W, g.tiles_x, gamma1, clamp_in, method_b
#define K1E(KD)                                                                              \
  if (C == 3) hipLaunchKernelGGL((k1_elem<KD, 3>), grid, dim3(256), 0, st, K1E_ARGS);        \
  else if (C == 1) hipLaunchKernelGGL((k1_elem<KD, 1>), grid, dim3(256), 0, st, K1E_ARGS);   \
  else hipLaunchKernelGGL((k1_elem<KD, 0>), grid, dim3(256), 0, st, K1E_ARGS);
  if (kind == OP_BLUR) hipLaunchKernelGGL(k1_primal_pre<OP_BLUR>, grid, dim3(256), 0, st, K1_ARGS);
  else if (kind == OP_MASK) { K1E(OP_MASK) }
  else { K1E(OP_ID) }
#undef K1E
#undef K1E_ARGS
#undef K1_ARGS
}

template <int KIND>
static void launch_k2_kind(int method, dim3 grid, hipStream_t st, const float* xn, const float* xo, float* y,
                           const float* xobs, const float* xtrue, float* s, const float* w, const float* theta,
                           double* partials, const OpDesc& op, int C, int H, int W, int tiles_x, int tiles,
                           double gamma2, double gkl_gamma, double gkl_alpha, int record, float* mm) {
#define K2_ARGS xn, xo, y, xobs, xtrue, s, w, theta, partials, op, C, H, W, tiles_x, tiles, gamma2, gkl_gamma, \
                gkl_alpha, record
#define K2E_ARGS xn, xo, y, xobs, xtrue, s, w, theta, partials, op.mask, C, H, W, tiles_x, tiles, gamma2, \
                 1.0 / gamma2, gkl_gamma, gkl_alpha, record, mm
  if constexpr (KIND == OP_BLUR) {
    if (method == M_A) hipLaunchKernelGGL((k2_dual<KIND, M_A>), grid, dim3(256), 0, st, K2_ARGS);
    else if (method == M_B) hipLaunchKernelGGL((k2_dual<KIND, M_B>), grid, dim3(256), 0, st, K2_ARGS);
    else hipLaunchKernelGGL((k2_dual<KIND, M_C>), grid, dim3(256), 0, st, K2_ARGS);
  } else {
#define K2E(M)                                                                                        \
    if (C == 3) hipLaunchKernelGGL((k2_elem<KIND, M, 3>), grid, dim3(256), 0, st, K2E_ARGS);          \
    else if (C == 1) hipLaunchKernelGGL((k2_elem<KIND, M, 1>), grid, dim3(256), 0, st, K2E_ARGS);     \
    else hipLaunchKernelGGL((k2_elem<KIND, M, 0>), grid, dim3(256), 0, st, K2E_ARGS);
    if (method == M_A) { K2E(M_A) }
    else if (method == M_B) { K2E(M_B) }
    else { K2E(M_C) }
#undef K2E
  }
#undef K2E_ARGS
#undef K2_ARGS
}

#ifdef PNP_PROFILING
static int g_k2_ablate = 0;   // kTuneAblateK2 (profiling build): k2_blur_rb's ABL legs at the metric shape
void set_k2_ablate(int bits) { g_k2_ablate = bits; }
#endif

template <class T>
static void launch_k2_rb(int method, hipStream_t st, const float* xn, const float* xo, float* y, const float* xobs,
                         const float* xtrue, float* s, const float* w, const float* theta, double* partials,
                         const OpDesc& op, int B, int C, int H, int W, int cells_x, int cells, double gamma2,
                         double gkl_gamma, double gkl_alpha, int record, float* mm) {
  const int tx = (W + kRbW - 1) / kRbW, tiles = tx * ((H + kRbH - 1) / kRbH);
  const dim3 grid(B * C * tiles);
  const bool lat = B * C * tiles < op.num_cus;     // one block per CU at most: latency-bound
#define K2RB_ARGS xn, xo, y, xobs, xtrue, s, w, theta, partials, reinterpret_cast<const f2_t*>(op.dense_fwd), C, H, W, \
                  tx, tiles, cells_x, cells, gamma2, 1.0 / gamma2, gkl_gamma, gkl_alpha, record, mm
#ifdef PNP_PROFILING
#define K2RB_ABL(M, A) if (g_k2_ablate == A) { hipLaunchKernelGGL((k2_blur_rb<T, M, 0, A>), grid, dim3(256), 0, st, K2RB_ARGS); return; }
  if (method == M_A && !lat && g_k2_ablate) {
    K2RB_ABL(M_A, 1) K2RB_ABL(M_A, 2) K2RB_ABL(M_A, 4) K2RB_ABL(M_A, 8) K2RB_ABL(M_A, 16) K2RB_ABL(M_A, 3)
    K2RB_ABL(M_A, 6) K2RB_ABL(M_A, 20) K2RB_ABL(M_A, 7) K2RB_ABL(M_A, 9) K2RB_ABL(M_A, 64)
  }
#undef K2RB_ABL
#endif
#define K2RBL(M)                                                                                              \
  if (lat) hipLaunchKernelGGL((k2_blur_rb<T, M, 1>), grid, dim3(256), 0, st, K2RB_ARGS);                       \
  else if (xtrue) hipLaunchKernelGGL((k2_blur_rb<T, M, 0>), grid, dim3(256), 0, st, K2RB_ARGS);               \
  else hipLaunchKernelGGL((k2_blur_rb<T, M, 0, 0, false>), grid, dim3(256), 0, st, K2RB_ARGS);
  if (method == M_A) { K2RBL(M_A) }
  else if (method == M_B) { K2RBL(M_B) }
  else { K2RBL(M_C) }
#undef K2RBL
#undef K2RB_ARGS
}

int launch_k2(int kind, int method, const float* xn, const float* xo, float* y, const float* xobs,
              const float* xtrue, float* s, const float* w, const float* theta, double* partials,
              const OpDesc& op, int B, int C, int H, int W, double gamma2, double gkl_gamma, double gkl_alpha,
              int record, float* mm, hipStream_t st) {
  const TileGrid g = tile_grid(H, W);
  if (!record) mm = nullptr;
  if (kind == OP_BLUR && rb_ok(op, C, H, W)) {
#define K2RB(TT) launch_k2_rb<TT>(method, st, xn, xo, y, xobs, xtrue, s, w, theta, partials, op, B, C, H, W, \
                                  g.tiles_x, g.tiles, gamma2, gkl_gamma, gkl_alpha, record, mm)
    switch (op.taps_id) {
      case TAPS_BLUR_1: K2RB(Taps_blur_1_Fwd); break;
      case TAPS_SQUARE_MINI: K2RB(Taps_square_mini_Fwd); break;
      default:
        switch (op.Rd) { case 2: K2RB(DenseTaps<2>); break; case 4: K2RB(DenseTaps<4>); break; default: K2RB(DenseTaps<8>); }
    }
#undef K2RB
    return mm ? C * ((W + kRbW - 1) / kRbW) * ((H + kRbH - 1) / kRbH) : 0;
  }
  dim3 grid(g.tiles, B);
  if (kind == OP_BLUR) {      // generic stencil path: no x+ range (SSIM computes its own)
    launch_k2_kind<OP_BLUR>(method, grid, st, xn, xo, y, xobs, xtrue, s, w, theta, partials, op, C, H, W,
                            g.tiles_x, g.tiles, gamma2, gkl_gamma, gkl_alpha, record, nullptr);
    return 0;
  }
  if (kind == OP_MASK)
    launch_k2_kind<OP_MASK>(method, grid, st, xn, xo, y, xobs, xtrue, s, w, theta, partials, op, C, H, W,
                            g.tiles_x, g.tiles, gamma2, gkl_gamma, gkl_alpha, record, mm);
  else
    launch_k2_kind<OP_ID>(method, grid, st, xn, xo, y, xobs, xtrue, s, w, theta, partials, op, C, H, W,
                          g.tiles_x, g.tiles, gamma2, gkl_gamma, gkl_alpha, record, mm);
  return mm ? g.tiles : 0;
}

int partial_tiles(int H, int W) { return tile_grid(H, W).tiles; }

int k2_minmax_chunks(int C, int H, int W) {
  const int rb = C * ((W + kRbW - 1) / kRbW) * ((H + kRbH - 1) / kRbH);
  const int el = tile_grid(H, W).tiles;
  return rb > el ? rb : el;
}

template <class TF, class TA>
static bool taps_match(int Rd, const uint32_t* fwd_cols, const uint32_t* adj_cols) {
  if (TF::kR != Rd || TA::kR != Rd) return false;
  for (int k = 0; k < 2 * Rd + 1; ++k)
    if (TF::col(k) != fwd_cols[k] || TA::col(k) != adj_cols[k]) return false;
  return true;
}

void pack_tap_pairs(int Rd, const float* Wc, float* out) {
  const int D = 2 * Rd + 1;
  auto w = [&](int cx, int cy) { return cx >= 0 && cx < D ? Wc[(size_t)cx * D + cy] : 0.f; };
  for (int p = 0; p <= Rd; ++p)
    for (int dy = 0; dy < D; ++dy) {
      float* o = out + ((size_t)p * D + dy) * 4;
      o[0] = w(2 * p, dy);      o[1] = w(2 * p - 1, dy);   // LDS column A: (out col 0, out col 1)
      o[2] = w(2 * p + 1, dy);  o[3] = w(2 * p, dy);       // LDS column B
    }
}

int match_taps(int Rd, const uint32_t* fwd_cols, const uint32_t* adj_cols) {
  if (taps_match<Taps_blur_1_Fwd, Taps_blur_1_Adj>(Rd, fwd_cols, adj_cols)) return TAPS_BLUR_1;
  if (taps_match<Taps_square_mini_Fwd, Taps_square_mini_Adj>(Rd, fwd_cols, adj_cols)) return TAPS_SQUARE_MINI;
  return TAPS_DENSE;
}

int k2_partials(const OpDesc& op, int C, int H, int W) {
  return rb_ok(op, C, H, W) ? tile_grid(H, W).tiles * C : tile_grid(H, W).tiles;
}

void launch_k3(int method, float* y, const float* xobs, const double* partials, const OpDesc& op, int B, int C,
               int H, int W, double gamma2, double eps, double* metrics, int it, int cap, int record, int has_true,
               hipStream_t st, const int* itp) {
  TileGrid g = tile_grid(H, W);
  g.tiles = k2_partials(op, C, H, W);
  const size_t n = (size_t)C * H * W;
  if (method == M_C) {
    if (record) hipLaunchKernelGGL(k3_metrics, dim3(B), dim3(256), 0, st, partials, g.tiles, n, metrics, it, cap,
                                   has_true, itp);
    return;
  }
  const int chunks = (int)((n + 2047) / 2048);
  hipLaunchKernelGGL(k3_l2_dual, dim3(chunks, B), dim3(256), 0, st, y, xobs, partials, g.tiles, n, gamma2, eps,
                     metrics, it, cap, record, has_true, itp);
}

__global__ void it_advance_kernel(int* itp) {
  if (threadIdx.x == 0) *itp += 1;
}
void launch_it_advance(int* itp, hipStream_t st) { hipLaunchKernelGGL(it_advance_kernel, dim3(1), dim3(64), 0, st, itp); }

void launch_l1_select(const float* v, float* theta, void* scratch, int B, size_t n, double eta, hipStream_t st) {
  L1Scratch* scr = reinterpret_cast<L1Scratch*>(scratch);
  // per-image state reset (the bins are left cleared by every pick launch; zeroed at allocation)
  hipLaunchKernelGGL(l1_reset_kernel, dim3((B + 63) / 64), dim3(64), 0, st, scr, B);
  // workgroups per image: B x G >= 512 (two per CU), slices of >= 16K elements, 16-B aligned
  int G = (512 + B - 1) / B;
  const int gmax = (int)((n + 16383) / 16384);
  G = G < gmax ? G : gmax;
  G = G > 0 ? G : 1;
  size_t chunk = (n + G - 1) / G;
  chunk = (chunk + 3) & ~(size_t)3;
  G = (int)((n + chunk - 1) / chunk);
  const dim3 hg(G, B);
  hipLaunchKernelGGL((l1_hist_kernel<20, 11>), hg, dim3(kSelHistThreads), 0, st, v, n, chunk, scr, eta);
  hipLaunchKernelGGL((l1_pick_kernel<20, 11, true, false>), dim3(B), dim3(64), 0, st, scr, theta, eta);
  hipLaunchKernelGGL((l1_hist_kernel<9, 11>), hg, dim3(kSelHistThreads), 0, st, v, n, chunk, scr, eta);
  hipLaunchKernelGGL((l1_pick_kernel<9, 11, false, false>), dim3(B), dim3(64), 0, st, scr, theta, eta);
  hipLaunchKernelGGL((l1_hist_kernel<0, 9>), hg, dim3(kSelHistThreads), 0, st, v, n, chunk, scr, eta);
  hipLaunchKernelGGL((l1_pick_kernel<0, 9, false, true>), dim3(B), dim3(64), 0, st, scr, theta, eta);
}

template <class T>
static void launch_k0_rb(hipStream_t st, const float* x, float* out, const float* add, const void* wd, int BC, int H,
                         int W) {
  const int tx = (W + kRbW - 1) / kRbW, tiles = tx * ((H + kRbH - 1) / kRbH);
  const f2_t* w = reinterpret_cast<const f2_t*>(wd);
  if (add) hipLaunchKernelGGL((k0_blur_rb<T, true>), dim3(BC * tiles), dim3(256), 0, st, x, out, add, w, H, W, tx, tiles);
  else hipLaunchKernelGGL((k0_blur_rb<T, false>), dim3(BC * tiles), dim3(256), 0, st, x, out, add, w, H, W, tx, tiles);
}

void launch_op_phi(int kind, int adj, const float* x, float* out, const OpDesc& op, int BC, int H, int W,
                   hipStream_t st, const float* add) {
  if (kind == OP_BLUR && rb_ok(op, 1, H, W)) {
#define K0RB(TF, TA)                                                           \
  if (adj) launch_k0_rb<TA>(st, x, out, add, op.dense_adj, BC, H, W);          \
  else launch_k0_rb<TF>(st, x, out, add, op.dense_fwd, BC, H, W);
    switch (op.taps_id) {
      case TAPS_BLUR_1: K0RB(Taps_blur_1_Fwd, Taps_blur_1_Adj) break;
      case TAPS_SQUARE_MINI: K0RB(Taps_square_mini_Fwd, Taps_square_mini_Adj) break;
      default:
        switch (op.Rd) {
          case 2: K0RB(DenseTaps<2>, DenseTaps<2>) break;
          case 4: K0RB(DenseTaps<4>, DenseTaps<4>) break;
          default: K0RB(DenseTaps<8>, DenseTaps<8>)
        }
    }
#undef K0RB
    return;
  }
  const TileGrid g = tile_grid(H, W);
  dim3 grid(g.tiles, BC);
#define PHI_ARGS x, out, add, op, H, W, g.tiles_x
  if (kind == OP_BLUR) {
    if (adj) hipLaunchKernelGGL((op_phi_kernel<OP_BLUR, 1>), grid, dim3(256), 0, st, PHI_ARGS);
    else hipLaunchKernelGGL((op_phi_kernel<OP_BLUR, 0>), grid, dim3(256), 0, st, PHI_ARGS);
  } else if (kind == OP_MASK) {
    hipLaunchKernelGGL((op_phi_kernel<OP_MASK, 0>), grid, dim3(256), 0, st, PHI_ARGS);
  } else {
    hipLaunchKernelGGL((op_phi_kernel<OP_ID, 0>), grid, dim3(256), 0, st, PHI_ARGS);
  }
#undef PHI_ARGS
}

int chunk_count(size_t n) { return (int)((n + 2047) / 2048); }

void launch_l2_proj(const float* x, const float* x0, float* out, double* partials, int B, size_t n, double eps,
                    hipStream_t st) {
  const int chunks = chunk_count(n);
  hipLaunchKernelGGL(sqdiff_partials, dim3(chunks, B), dim3(256), 0, st, x, x0, partials, n, chunks);
  hipLaunchKernelGGL(l2_apply, dim3(chunks, B), dim3(256), 0, st, x, x0, out, partials, n, chunks, eps);
}

void launch_sqdiff(const float* a, const float* c, double* partials, int B, size_t n, hipStream_t st) {
  const int chunks = chunk_count(n);
  hipLaunchKernelGGL(sqdiff_partials, dim3(chunks, B), dim3(256), 0, st, a, c, partials, n, chunks);
}

void launch_shrink(const float* v, float* out, const float* theta, int B, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(shrink_kernel, dim3(chunk_count(n), B), dim3(256), 0, st, v, out, theta, n);
}

void launch_gkl(const float* x, const float* x0, float* out, size_t count, double gamma, double alpha,
                hipStream_t st) {
  size_t blocks = (count + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(gkl_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, x0, out, count, gamma, alpha);
}

// Streaming copy (bench.py's measured copy ceiling for the prox passes' HBM fraction): every
// thread moves 4 x 16 B per step, all four loads in flight before the stores, non-temporal
// (tools/probes/copy_bw.hip, 1 GiB: plain 5.5-5.8 TB/s, non-temporal 5.9-6.3 TB/s, best with
// 64 blocks per CU), grid-strided.
__global__ __launch_bounds__(256) void copy_f4_kernel(const floatx4* __restrict__ src, floatx4* __restrict__ dst,
                                                      size_t n4) {
  const size_t stride = (size_t)gridDim.x * 256 * 4;
  for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n4; i += stride) {
    floatx4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + 256 * k < n4) v[k] = __builtin_nontemporal_load(src + i + 256 * k);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + 256 * k < n4) __builtin_nontemporal_store(v[k], dst + i + 256 * k);
  }
}

void launch_copy_f4(const void* src, void* dst, size_t bytes, int num_cus, hipStream_t st) {
  const size_t n4 = bytes / 16;
  size_t blocks = (n4 + 1023) / 1024;
  const size_t cap = (size_t)num_cus * 64;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return;
  hipLaunchKernelGGL(copy_f4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const floatx4*)src, (floatx4*)dst, n4);
}

void launch_pack_input(const float* x, float* u32, int B, int C, int H, int W, int clamp_in, hipStream_t st) {
  const size_t total = (size_t)B * C * H * W;
  size_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (blocks == 0) return;
  hipLaunchKernelGGL(pack_input_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, u32, total, clamp_in);
}

}  // namespace pnp

namespace pnp {

void launch_lincomb(float* out, double k, const float* a, double ca, const float* b, double cb, const float* c,
                    double cc, const float* d, double cd, size_t count, hipStream_t st) {
  LinComb lc;
  lc.k = k;
  lc.c[0] = ca; lc.c[1] = cb; lc.c[2] = cc; lc.c[3] = cd;
  lc.in[0] = a; lc.in[1] = b; lc.in[2] = c; lc.in[3] = d;
  size_t blocks = (count + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(lincomb_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, lc, count);
}

void launch_metrics(const float* xn, const float* xo, const float* xt, double* partials, double* metrics, int B,
                    size_t n, int it, int cap, hipStream_t st, const int* itp) {
  const int chunks = chunk_count(n);
  hipLaunchKernelGGL(metric_partials_kernel, dim3(chunks, B), dim3(256), 0, st, xn, xo, xt, partials, n, chunks);
  hipLaunchKernelGGL(k3_metrics, dim3(B), dim3(256), 0, st, partials, chunks, n, metrics, it, cap, xt ? 1 : 0, itp);
}

}  // namespace pnp

namespace pnp {

size_t ssim_scratch_bytes(int B, int C, int H, int W) {
  const size_t n = (size_t)C * H * W;
  const int tiles = ((W + kSsTW - 1) / kSsTW) * ((H + kSsTH - 1) / kSsTH);
  const size_t t2q = (size_t)B * (C == 1 ? H : C * tiles);
  return (size_t)B * chunk_count(n) * 2 * sizeof(float) + (size_t)B * C * tiles * sizeof(double) +
         t2q * sizeof(double) + (size_t)B * H * sizeof(float) + 256;
}

void launch_ssim(const float* xt, const float* x, void* scratch, double* metrics, int B, int C, int H, int W,
                 int it, int cap, hipStream_t st, const float* mm_ext, int mm_chunks, const int* itp, bool psnr) {
  const size_t n = (size_t)C * H * W;
  int chunks = chunk_count(n);
  const int tx = (W + kSsTW - 1) / kSsTW, tiles = tx * ((H + kSsTH - 1) / kSsTH);
  float* mm = static_cast<float*>(scratch);
  double* ps = reinterpret_cast<double*>(
      (reinterpret_cast<uintptr_t>(mm + (size_t)B * chunks * 2) + 255) & ~(uintptr_t)255);
  double* t2 = ps + (size_t)B * C * tiles;
  float* rows = reinterpret_cast<float*>(t2 + (size_t)B * (C == 1 ? H : C * tiles));
  double* t2o = psnr ? t2 : nullptr;
  if (mm_ext && mm_chunks > 0) {          // x+'s range came from K2 (one pass over x+ fewer)
    mm = const_cast<float*>(mm_ext);
    chunks = mm_chunks;
  } else {
    hipLaunchKernelGGL(ssim_minmax_kernel, dim3(chunks, B), dim3(256), 0, st, x, mm, n, chunks);
  }
  const int gray = C == 1;
  if (gray)
    hipLaunchKernelGGL(ssim_gray_kernel, dim3((H + 3) / 4, B), dim3(256), 0, st, xt, x, mm, rows, t2o, H, W, chunks);
  else
    hipLaunchKernelGGL(ssim_rgb_kernel, dim3(tiles, B * C), dim3(256), 0, st, xt, x, mm, ps, t2o, C, H, W, tx, tiles,
                       chunks);
  hipLaunchKernelGGL(ssim_final_kernel, dim3(B), dim3(256), 0, st, ps, rows, t2o, metrics, C, H, W, tiles, gray, it,
                     cap, itp);
}

}  // namespace pnp
