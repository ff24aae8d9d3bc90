// Observation pipeline on the device: main.py:49-64 with the noise of
// utils/utils_noise.py, reproducing numpy's legacy RandomState stream (np.random.seed(1234)
// before every noise call) so that x_obs has the reference's bit pattern.
//
//   x_obs = Phi(x_true)                                  (float64 here: blur in f64 taps)
//   x_obs += M (sigma * randn(C,H,W))                    add_gaussian_noise       utils_noise.py:35-38
//   x_obs  = poisson(alpha * x_obs)      (if Poisson)    apply_poisson_noise      utils_noise.py:40-43
//   x_obs  = salt & pepper(x_obs, sp_nl)                 add_salt_and_pepper_noise utils_noise.py:3-33
//   x_0    = x_obs (/ alpha if Poisson)                                            main.py:62-64
//
// numpy legacy generator pieces restated (numpy/random: mt19937.c, legacy-distributions.c,
// distributions.c random_loggam, _bounded_integers masked rejection):
//   * MT19937 init_genrand(seed) + twist + tempering: one 256-thread workgroup writes the
//     tempered word stream (3 dependent phases per 624-word block);
//   * randn = legacy_gauss: polar Box-Muller on candidate pairs of legacy doubles (4 words per
//     candidate), each accepted pair emits f*x2 then f*x1 -> parallel by a scan over the
//     acceptance flags;
//   * randint(0, H) = (word & mask) rejected while > H-1, one word per try -> parallel by a
//     scan over the valid words; duplicate / masked pixels resolved by first-occurrence;
//   * poisson = legacy PTRS (lam >= 10) / multiplication (lam < 10): the word consumption of
//     each element depends on its value, so each image walks its stream in one thread.
// The products and sums follow the C sources' evaluation order with contraction off.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"
#include "kernels.h"

namespace pnp {
namespace {

constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMtA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

// ---- MT19937 word stream ------------------------------------------------------------------
__global__ __launch_bounds__(256) void mt_stream_kernel(uint32_t seed, uint32_t* __restrict__ out, size_t nwords) {
  __shared__ uint32_t mt[kMtN];
  const int t = threadIdx.x;
  if (t == 0) {                                        // init_genrand (mt19937_seed)
    uint32_t s = seed;
    for (int i = 0; i < kMtN; ++i) {
      mt[i] = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
  }
  __syncthreads();
  for (size_t base = 0; base < nwords; base += kMtN) {
    // twist in three dependent phases: [0,227) reads old words; [227,454) reads phase-1 words
    // at i-227; [454,624) reads phase-2 words (and i = 623 wraps to the new mt[0]).
#pragma unroll
    for (int ph = 0; ph < 3; ++ph) {
      const int lo = ph * (kMtN - kMtM), hi = ph == 2 ? kMtN : lo + (kMtN - kMtM);
      const int i = lo + t;
      uint32_t v = 0;
      if (i < hi) {
        const uint32_t y = (mt[i] & kUpper) | (mt[(i + 1) % kMtN] & kLower);
        v = mt[(i + kMtM) % kMtN] ^ (y >> 1) ^ ((y & 1u) ? kMtA : 0u);
      }
      __syncthreads();
      if (i < hi) mt[i] = v;
      __syncthreads();
    }
    for (int i = t; i < kMtN; i += 256) {
      if (base + i >= nwords) break;
      uint32_t y = mt[i];
      y ^= y >> 11;
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= y >> 18;
      out[base + i] = y;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ double legacy_double(const uint32_t* w) {   // mt19937_next_double
  const int32_t a = (int32_t)(w[0] >> 5), b = (int32_t)(w[1] >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

// ---- scan (exclusive, u32) over up to ~2^31 flags: block sums, one-block scan, apply -------
constexpr int kScanTile = 1024;   // 256 threads x 4

__global__ __launch_bounds__(256) void scan_sums_kernel(const uint32_t* __restrict__ f, size_t n,
                                                        uint32_t* __restrict__ sums) {
  __shared__ uint32_t red[4];
  const size_t base = (size_t)blockIdx.x * kScanTile + threadIdx.x * 4;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) s += base + k < n ? f[base + k] : 0u;
  s = block_sum(s, red);
  if (threadIdx.x == 0) sums[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void scan_top_kernel(uint32_t* __restrict__ sums, int nb, uint32_t* total) {
  __shared__ uint32_t sh[256];
  uint32_t carry = 0;
  for (int base = 0; base < nb; base += 256) {
    const int i = base + threadIdx.x;
    const uint32_t v = i < nb ? sums[i] : 0u;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {               // Hillis-Steele inclusive
      const uint32_t a = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0u;
      __syncthreads();
      sh[threadIdx.x] += a;
      __syncthreads();
    }
    if (i < nb) sums[i] = carry + sh[threadIdx.x] - v;   // exclusive
    carry += sh[255];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void scan_apply_kernel(const uint32_t* __restrict__ f, size_t n,
                                                         const uint32_t* __restrict__ sums,
                                                         uint32_t* __restrict__ out) {
  __shared__ uint32_t sh[256];
  const size_t base = (size_t)blockIdx.x * kScanTile + threadIdx.x * 4;
  uint32_t v[4], s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = base + k < n ? f[base + k] : 0u;
    s += v[k];
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t a = threadIdx.x >= (unsigned)o ? sh[threadIdx.x - o] : 0u;
    __syncthreads();
    sh[threadIdx.x] += a;
    __syncthreads();
  }
  uint32_t run = sums[blockIdx.x] + sh[threadIdx.x] - s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
}

// ---- Gaussian: legacy_gauss over candidate pairs ------------------------------------------
__global__ void gauss_flags_kernel(const uint32_t* __restrict__ w, size_t ncand, uint32_t* __restrict__ flag) {
#pragma clang fp contract(off)
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ncand) return;
  const double x1 = 2.0 * legacy_double(w + 4 * k) - 1.0;
  const double x2 = 2.0 * legacy_double(w + 4 * k + 2) - 1.0;
  const double r2 = x1 * x1 + x2 * x2;
  flag[k] = (r2 >= 1.0 || r2 == 0.0) ? 0u : 1u;
}

// noise[2j] = f*x2, noise[2j+1] = f*x1 for the j-th accepted candidate (n values)
__global__ void gauss_emit_kernel(const uint32_t* __restrict__ w, size_t ncand, const uint32_t* __restrict__ flag,
                                  const uint32_t* __restrict__ rank, double* __restrict__ noise, size_t n) {
#pragma clang fp contract(off)
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ncand || !flag[k]) return;
  const size_t j = rank[k];   // the noise field is the same for every image (reseeded per call)
  if (2 * j >= n) return;
  const double x1 = 2.0 * legacy_double(w + 4 * k) - 1.0;
  const double x2 = 2.0 * legacy_double(w + 4 * k + 2) - 1.0;
  const double r2 = x1 * x1 + x2 * x2;
  const double f = sqrt(-2.0 * log(r2) / r2);
  noise[2 * j] = f * x2;
  if (2 * j + 1 < n) noise[2 * j + 1] = f * x1;
}

// ---- x_obs = Phi(x_true) + M(sigma * g), float64 ------------------------------------------
// blur: y[i,j] = sum_t v_t x[(i+dy_t) mod H, (j+dx_t) mod W] (operators.py:7-22, centred circular)
__global__ void observe_kernel(const float* __restrict__ xt, const double* __restrict__ noise,
                               const Tap64* __restrict__ taps, int ntaps, const uint8_t* __restrict__ mask, int kind,
                               double sigma, double* __restrict__ img, int B, int C, int H, int W) {
#pragma clang fp contract(off)
  const size_t n = (size_t)C * H * W;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)B * n) return;
  const size_t r = e % n;                               // position inside the image (C,H,W)
  const int j = (int)(r % W), i = (int)((r / W) % H);
  const float* plane = xt + (e - (size_t)i * W - j);
  double v;
  if (kind == OP_BLUR) {
    v = 0.0;
    for (int t = 0; t < ntaps; ++t) {
      int ii = i + taps[t].dy, jj = j + taps[t].dx;
      ii = ((ii % H) + H) % H;
      jj = ((jj % W) + W) % W;
      v += taps[t].v * (double)plane[(size_t)ii * W + jj];
    }
  } else {
    v = (double)xt[e];
  }
  double g = noise ? sigma * noise[r] : 0.0;           // same noise field for every image
  if (kind == OP_MASK && !mask[(size_t)i * W + j]) {
    v = 0.0;                                            // t[q] = 0 (operators.py:49-57)
    g = 0.0;
  }
  img[e] = v + g;
}

// ---- Poisson: one image per thread, walking the shared stream -----------------------------
__device__ double random_loggam(double x) {             // numpy distributions.c
#pragma clang fp contract(off)
  const double a[10] = {8.333333333333333e-02, -2.777777777777778e-03, 7.936507936507937e-04,
                        -5.952380952380952e-04, 8.417508417508418e-04, -1.917526917526918e-03,
                        6.410256410256410e-03, -2.955065359477124e-02, 1.796443723688307e-01,
                        -1.39243221690590e+00};
  if (x == 1.0 || x == 2.0) return 0.0;
  const int64_t n = x < 7.0 ? (int64_t)(7 - x) : 0;
  double x0 = x + n;
  const double x2 = (1.0 / x0) * (1.0 / x0);
  const double lg2pi = 1.8378770664093453e+00;
  double gl0 = a[9];
  for (int k = 8; k >= 0; --k) {
    gl0 *= x2;
    gl0 += a[k];
  }
  double gl = gl0 / x0 + 0.5 * lg2pi + (x0 - 0.5) * log(x0) - x0;
  if (x < 7.0)
    for (int64_t k = 1; k <= n; ++k) {
      gl -= log(x0 - 1.0);
      x0 -= 1.0;
    }
  return gl;
}

// status: [0] = error code (1 lam < 0, 2 lam too large, 3 stream exhausted), [1] = words used (max)
__global__ void poisson_walk_kernel(const uint32_t* __restrict__ w, size_t nwords, double* __restrict__ img,
                                    int B, size_t n, double alpha, unsigned long long* __restrict__ status) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double* x = img + (size_t)b * n;
  for (size_t e = 0; e < n; ++e) {                      // numpy checks every lam before drawing
    const double lam = x[e] * alpha;
    if (lam > 9.2233720064847708e+18) { atomicMax(&status[0], 2ull); return; }   // POISSON_LAM_MAX
    if (!(lam >= 0.0)) { atomicMax(&status[0], 1ull); return; }                   // "lam < 0 or NaN"
  }
  size_t p = 0;
  const size_t lim = nwords & ~(size_t)1;
  for (size_t e = 0; e < n; ++e) {
    const double lam = x[e] * alpha;
    int64_t k = 0;
    if (lam >= 10.0) {                                  // legacy_random_poisson_ptrs
      const double slam = sqrt(lam), loglam = log(lam);
      const double bb = 0.931 + 2.53 * slam;
      const double a = -0.059 + 0.02483 * bb;
      const double invalpha = 1.1239 + 1.1328 / (bb - 3.4);
      const double vr = 0.9277 - 3.6224 / (bb - 2);
      while (true) {
        if (p + 4 > lim) { atomicMax(&status[0], 3ull); atomicMax(&status[1], (unsigned long long)p); return; }
        const double U = legacy_double(w + p) - 0.5;
        const double V = legacy_double(w + p + 2);
        p += 4;
        const double us = 0.5 - fabs(U);
        k = (int64_t)floor((2 * a / us + bb) * U + lam + 0.43);
        if (us >= 0.07 && V <= vr) break;
        if (k < 0 || (us < 0.013 && V > us)) continue;
        if ((log(V) + log(invalpha) - log(a / (us * us) + bb)) <= (-lam + k * loglam - random_loggam(k + 1))) break;
      }
    } else if (lam == 0.0) {
      k = 0;
    } else {                                            // legacy_random_poisson_mult (also NaN -> 0)
      const double enlam = exp(-lam);
      double prod = 1.0;
      while (true) {
        if (p + 2 > lim) { atomicMax(&status[0], 3ull); atomicMax(&status[1], (unsigned long long)p); return; }
        const double U = legacy_double(w + p);
        p += 2;
        prod *= U;
        if (prod > enlam) ++k;
        else break;
      }
    }
    x[e] = (double)k;
  }
  atomicMax(&status[1], (unsigned long long)p);
}

// ---- salt & pepper ------------------------------------------------------------------------
__global__ void sp_valid_kernel(const uint32_t* __restrict__ w, size_t nw, uint32_t mask, uint32_t rng,
                                uint32_t* __restrict__ flag) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nw) flag[k] = (w[k] & mask) <= rng ? 1u : 0u;
}

// draws[rank] = word & mask for the valid words (first ndraw only)
__global__ void sp_compact_kernel(const uint32_t* __restrict__ w, size_t nw, uint32_t mask,
                                  const uint32_t* __restrict__ flag, const uint32_t* __restrict__ rank,
                                  uint32_t* __restrict__ draws, size_t ndraw) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nw && flag[k] && rank[k] < ndraw) draws[rank[k]] = w[k] & mask;
}

// pair i = (x, y) = (draws[2i], draws[2i+1]); noise_target[x][y] == 1 -> first[x*H + y] = min i
__global__ void sp_first_kernel(const uint32_t* __restrict__ draws, int npairs, const uint8_t* __restrict__ tgt,
                                int H, int W, uint32_t* __restrict__ first, unsigned long long* __restrict__ status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npairs) return;
  const uint32_t x = draws[2 * i], y = draws[2 * i + 1];
  if ((int)y >= W) { atomicMax(&status[0], 4ull); return; }   // numpy IndexError (y drawn in [0, H))
  if (tgt && !tgt[(size_t)x * W + y]) return;
  atomicMin(&first[(size_t)x * H + y], (uint32_t)i);
}

__global__ void sp_accept_kernel(const uint32_t* __restrict__ draws, int npairs, const uint8_t* __restrict__ tgt,
                                 int H, int W, const uint32_t* __restrict__ first, uint32_t* __restrict__ acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npairs) return;
  const uint32_t x = draws[2 * i], y = draws[2 * i + 1];
  uint32_t a = 0;
  if ((int)y < W && (!tgt || tgt[(size_t)x * W + y])) a = first[(size_t)x * H + y] == (uint32_t)i;
  acc[i] = a;
}

// the first noise_cnt accepted pixels -> 0, the rest -> 1, in every image and channel
__global__ void sp_apply_kernel(const uint32_t* __restrict__ draws, int npairs, const uint32_t* __restrict__ acc,
                                const uint32_t* __restrict__ rank, int noise_cnt, double* __restrict__ img, int B,
                                int C, int H, int W) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npairs || !acc[i]) return;
  const size_t pix = (size_t)draws[2 * i] * W + draws[2 * i + 1];
  const double v = (int)rank[i] < noise_cnt ? 0.0 : 1.0;
  const size_t plane = (size_t)H * W;
  for (int b = 0; b < B; ++b)
    for (int c = 0; c < C; ++c) img[((size_t)b * C + c) * plane + pix] = v;
}

__global__ void finalize_kernel(const double* __restrict__ img, size_t N, double alpha, int poisson,
                                float* __restrict__ xobs, float* __restrict__ x0, double* __restrict__ xobs64) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  const double v = img[e];
  if (xobs) xobs[e] = (float)v;
  if (xobs64) xobs64[e] = v;
  if (x0) x0[e] = (float)(poisson ? v / alpha : v);   // main.py:62-64: x_0 / alpha
}

inline unsigned grid_of(size_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

void launch_mt_stream(uint32_t seed, uint32_t* out, size_t nwords, hipStream_t st) {
  hipLaunchKernelGGL(mt_stream_kernel, dim3(1), dim3(256), 0, st, seed, out, nwords);
}

size_t scan_scratch_words(size_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

void launch_scan(const uint32_t* f, size_t n, uint32_t* out, uint32_t* scratch, hipStream_t st) {
  const int nb = (int)((n + kScanTile - 1) / kScanTile);
  if (nb == 0) return;
  hipLaunchKernelGGL(scan_sums_kernel, dim3(nb), dim3(256), 0, st, f, n, scratch + 1);
  hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(256), 0, st, scratch + 1, nb, scratch);
  hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(256), 0, st, f, n, scratch + 1, out);
}

void launch_gauss(const uint32_t* w, size_t ncand, uint32_t* flag, uint32_t* rank, uint32_t* scan_scr, double* noise,
                  size_t n, hipStream_t st) {
  hipLaunchKernelGGL(gauss_flags_kernel, dim3(grid_of(ncand)), dim3(256), 0, st, w, ncand, flag);
  launch_scan(flag, ncand, rank, scan_scr, st);
  hipLaunchKernelGGL(gauss_emit_kernel, dim3(grid_of(ncand)), dim3(256), 0, st, w, ncand, flag, rank, noise, n);
}

void launch_observe(const float* xt, const double* noise, const Tap64* taps, int ntaps, const uint8_t* mask, int kind,
                    double sigma, double* img, int B, int C, int H, int W, hipStream_t st) {
  const size_t N = (size_t)B * C * H * W;
  hipLaunchKernelGGL(observe_kernel, dim3(grid_of(N)), dim3(256), 0, st, xt, noise, taps, ntaps, mask, kind, sigma,
                     img, B, C, H, W);
}

void launch_poisson(const uint32_t* w, size_t nwords, double* img, int B, size_t n, double alpha,
                    unsigned long long* status, hipStream_t st) {
  hipLaunchKernelGGL(poisson_walk_kernel, dim3(grid_of(B, 64)), dim3(64), 0, st, w, nwords, img, B, n, alpha, status);
}

void launch_sp_draws(const uint32_t* w, size_t nw, uint32_t mask, uint32_t rng, uint32_t* flag, uint32_t* rank,
                     uint32_t* scan_scr, uint32_t* draws, size_t ndraw, hipStream_t st) {
  hipLaunchKernelGGL(sp_valid_kernel, dim3(grid_of(nw)), dim3(256), 0, st, w, nw, mask, rng, flag);
  launch_scan(flag, nw, rank, scan_scr, st);
  hipLaunchKernelGGL(sp_compact_kernel, dim3(grid_of(nw)), dim3(256), 0, st, w, nw, mask, flag, rank, draws, ndraw);
}

void launch_sp_apply(const uint32_t* draws, int npairs, const uint8_t* tgt, int H, int W, uint32_t* first,
                     uint32_t* acc, uint32_t* rank, uint32_t* scan_scr, int noise_cnt, double* img, int B, int C,
                     unsigned long long* status, hipStream_t st) {
  if (npairs <= 0) return;
  hipLaunchKernelGGL(sp_first_kernel, dim3(grid_of(npairs)), dim3(256), 0, st, draws, npairs, tgt, H, W, first,
                     status);
  hipLaunchKernelGGL(sp_accept_kernel, dim3(grid_of(npairs)), dim3(256), 0, st, draws, npairs, tgt, H, W, first, acc);
  launch_scan(acc, (size_t)npairs, rank, scan_scr, st);
  hipLaunchKernelGGL(sp_apply_kernel, dim3(grid_of(npairs)), dim3(256), 0, st, draws, npairs, acc, rank, noise_cnt,
                     img, B, C, H, W);
}

void launch_degrade_finalize(const double* img, size_t N, double alpha, int poisson, float* xobs, float* x0,
                             double* xobs64, hipStream_t st) {
  hipLaunchKernelGGL(finalize_kernel, dim3(grid_of(N)), dim3(256), 0, st, img, N, alpha, poisson, xobs, x0, xobs64);
}

}  // namespace pnp
