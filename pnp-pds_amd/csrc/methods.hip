// Kernels of the comparison methods that the PDS kernels do not cover:
// the TV pair D / D^T with prox_l12 (operators.py:110-137; A-PDS-TV, A-FBS-TV,
// comparisonB-3) and the Poisson ADMM x-step (algorithm/admm.py:4-16; C-PnPADMM-DnCNN,
// C-RED-DnCNN).  Everything else those methods need is Phi / Phi^T, the denoiser, the l1 /
// l2 projections and linear combinations, which the PDS path already has.
//
// Layout: x is [B][C][H][W]; the TV dual y1 is [B][2C][H][W] with the C vertical
// differences first, then the C horizontal ones, as D stacks them (operators.py:124).
// Arithmetic in float64 on float32 state, like the rest of the prox kernels.
#include <hip/hip_runtime.h>

#include "common.h"
#include "kernels.h"

namespace pnp {
namespace {

// out = x - gamma1 * (D^T y1 + g)      (iteration.py:88 / :94 / :140; g = Phi^T y2 or the FBS gradient)
// D^T as shipped (operators.py:128-137): row 0 -> -y[0]; rows 1..H-2 -> y[i-1] - y[i];
// row H-1 -> +y[H-1] (the reference keeps the last row of y, which D leaves at 0); same for columns.
__global__ void tv_primal_kernel(const float* __restrict__ x, const float* __restrict__ y1,
                                 const float* __restrict__ g, double gamma1, float* __restrict__ out, int C, int H,
                                 int W, size_t N) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  const size_t plane = (size_t)H * W;
  const int j = (int)(e % W), i = (int)((e / W) % H);
  const size_t bc = e / plane;
  const size_t b = bc / C, c = bc % C;
  const float* yv = y1 + (b * 2 * C + c) * plane;
  const float* yh = y1 + (b * 2 * C + C + c) * plane;
  const size_t p = (size_t)i * W + j;
  double dv, dh;
  if (i == 0) dv = -(double)yv[p];
  else if (i == H - 1) dv = (double)yv[p];
  else dv = -(double)yv[p] + (double)yv[p - W];
  if (j == 0) dh = -(double)yh[p];
  else if (j == W - 1) dh = (double)yh[p];
  else dh = -(double)yh[p] + (double)yh[p - 1];
  const double gv = g ? (double)g[e] : 0.0;
  out[e] = (float)((double)x[e] - gamma1 * ((dv + dh) + gv));
}

// y1 <- y1 + gamma2 D(2 xn - xo);  y1 <- y1 - gamma2 prox_l12(y1 / gamma2, 1 / gamma2)
// (iteration.py:89-90): prox_l12(v, t) = max(1 - t / ||v_pixel||, 0) v over the 2C components.
__global__ void tv_dual_kernel(const float* __restrict__ xn, const float* __restrict__ xo, float* __restrict__ y1,
                               double gamma2, int C, int H, int W, size_t npix) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= npix) return;
  const size_t plane = (size_t)H * W;
  const size_t b = e / plane, p = e % plane;
  const int j = (int)(p % W), i = (int)(p / W);
  double t[2 * kMaxC];
  double ss = 0.0;
  for (int c = 0; c < C; ++c) {
    const size_t base = (b * C + c) * plane;
    const double w0 = 2.0 * xn[base + p] - xo[base + p];
    const double wd = i < H - 1 ? 2.0 * xn[base + p + W] - xo[base + p + W] : w0;
    const double wr = j < W - 1 ? 2.0 * xn[base + p + 1] - xo[base + p + 1] : w0;
    const size_t bv = (b * 2 * C + c) * plane + p, bh = (b * 2 * C + C + c) * plane + p;
    t[c] = (double)y1[bv] + gamma2 * (wd - w0);
    t[C + c] = (double)y1[bh] + gamma2 * (wr - w0);
  }
  for (int k = 0; k < 2 * C; ++k) {
    const double u = t[k] / gamma2;
    ss += u * u;
  }
  const double val = (1.0 / gamma2) / sqrt(ss);          // ss == 0 -> inf -> factor 0 (as numpy fmax)
  const double f = fmax(1.0 - val, 0.0);
  for (int k = 0; k < 2 * C; ++k) {
    const int c = k % C;
    const size_t idx = (b * 2 * C + (k < C ? 0 : C) + c) * plane + p;
    y1[idx] = (float)(t[k] - gamma2 * (f * (t[k] / gamma2)));
  }
}

// out = y / (alpha * t)    (admm.py:11: y / (poisson_alpha * phi(x_n)); 0/0 -> NaN, which
// Phi^T of random sampling then overwrites with 0 exactly as t[q] = 0 does)
__global__ void poisson_ratio_kernel(const float* __restrict__ y, const float* __restrict__ t, double alpha,
                                     float* __restrict__ out, size_t N) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < N) out[e] = (float)((double)y[e] / (alpha * (double)t[e]));
}

// x <- x - gamma * (-g/alpha + c1/alpha + lam (x - v + u))   (admm.py:11-12; g = Phi^T(ratio), c1 = Phi^T 1)
__global__ void admm_poisson_step_kernel(float* __restrict__ x, const float* __restrict__ g,
                                         const float* __restrict__ c1, const float* __restrict__ v,
                                         const float* __restrict__ u, double gamma, double alpha, double lam,
                                         size_t N) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  const double xv = x[e];
  const double grad = -(double)g[e] / alpha + (double)c1[e] / alpha + lam * (xv - (double)v[e] + (double)u[e]);
  x[e] = (float)(xv - gamma * grad);
}

inline unsigned grid_of(size_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

void launch_tv_primal(const float* x, const float* y1, const float* g, double gamma1, float* out, int B, int C, int H,
                      int W, hipStream_t st) {
  const size_t N = (size_t)B * C * H * W;
  hipLaunchKernelGGL(tv_primal_kernel, dim3(grid_of(N)), dim3(256), 0, st, x, y1, g, gamma1, out, C, H, W, N);
}

void launch_tv_dual(const float* xn, const float* xo, float* y1, double gamma2, int B, int C, int H, int W,
                    hipStream_t st) {
  const size_t npix = (size_t)B * H * W;
  hipLaunchKernelGGL(tv_dual_kernel, dim3(grid_of(npix)), dim3(256), 0, st, xn, xo, y1, gamma2, C, H, W, npix);
}

void launch_poisson_ratio(const float* y, const float* t, double alpha, float* out, size_t N, hipStream_t st) {
  hipLaunchKernelGGL(poisson_ratio_kernel, dim3(grid_of(N)), dim3(256), 0, st, y, t, alpha, out, N);
}

void launch_admm_poisson_step(float* x, const float* g, const float* c1, const float* v, const float* u,
                              double gamma, double alpha, double lam, size_t N, hipStream_t st) {
  hipLaunchKernelGGL(admm_poisson_step_kernel, dim3(grid_of(N)), dim3(256), 0, st, x, g, c1, v, u, gamma, alpha,
                     lam, N);
}

}  // namespace pnp
