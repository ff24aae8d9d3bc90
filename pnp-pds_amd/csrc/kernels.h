// Launch interface between the host orchestration (capi.hip) and the kernels
// (conv.hip: denoiser, ops.hip: operators / proxes / fused dual passes).
#pragma once
#include "common.h"

namespace pnp {

// ---- denoiser (conv.hip) -----------------------------------------------------------
constexpr int kActPad = 2;   // zero border of the hidden activation images (two-layer halo)
struct ConvShape {
  int B, H, W;       // image size (unpadded)
  int pad;           // zero border of the activation images (kActPad)
  int Hp, Wp;        // padded (H + 2 pad, W + 2 pad)
  int tiles_x, tiles_y, tiles;
};
ConvShape make_conv_shape(int B, int H, int W);
hipError_t conv_kernels_init();
void pack_body_weights(const float* W, uint16_t* out);
void pack_body_weights16(const float* W, uint16_t* out);   // v_mfma_f32_16x16x32_f16 fragments (conv_body_x8)
void pack_head_weights(const float* W, int C, uint16_t* out);
void pack_tail_weights(const float* W, int C, uint16_t* out);
// w_lo (nullable): the split weights' low halves (PNP_PREC_FP16W2 / FP16X3), packed like w.
// out_lo (nullable, FP16X3): the input is split too (three MFMAs per product) and the output is
// written as hi (out) + lo (out_lo) fp16 images.
void launch_conv_head(const float* in32, int C, half_t* out, const void* w, const void* w_lo, const float* bias,
                      const ConvShape& s, int act, int num_cus, int blocks_per_cu, hipStream_t st,
                      half_t* out_lo = nullptr);
// one 64 -> 64 layer; ablate != 0 only in the PNP_PROFILING build (profiling, results wrong)
void launch_conv_body(const half_t* in, half_t* out, const void* w, const float* bias, const ConvShape& s,
                      int act, int num_cus, int ablate, hipStream_t st);
#ifdef PNP_PROFILING
constexpr int kTuneAblate = 99;   // pnp_set_tuning key of the profiling build (not in include/pnppds.h)
constexpr int kTuneAblateK2 = 98; // profiling build: k2_blur_rb ablation legs (ops.hip ABL bits)
#ifdef PNP_PROFILING
void set_k2_ablate(int bits);
#endif
#endif
void launch_conv_tail(const half_t* in, const float* xin, float* xout, const void* w, const void* w_lo,
                      const float* bias, const ConvShape& s, int C, int residual_sign, int clamp_out, int num_cus,
                      hipStream_t st);
// The denoiser's ends inside the first / last two-layer launch (round 5): HEAD = the head layer
// (C -> 64, from the fp32 NCHW input u32) and the first body layer; TAIL = the last body layer and
// the tail (64 -> C + residual + clamp, fp32 NCHW out).  Bit-identical to the separate
// conv_head / conv_tail launches around plain pairs.
struct X8Ends {
  const float* u32 = nullptr;     // HEAD: the denoiser input; TAIL: the residual input
  const void* hw = nullptr;       // HEAD: conv_head's packed weights (pack_head_weights)
  const float* hb = nullptr;
  float* xout = nullptr;          // TAIL: the output x+
  const void* tw = nullptr;       // TAIL: packed tail weights (pack_tail_weights)
  const float* tb = nullptr;
  int C = 0, residual_sign = 1, clamp_out = 1;
};
enum X8Mode { kX8Pair = 0, kX8Head = 1, kX8Tail = 2 };
// two 64 -> 64 layers in one launch, streamed down 32-pixel column strips (needs pad >= 2);
// mode kX8Head: in is not read, layer 1 is the head (ends: u32, C, hw, hb; w16_1 / b1 unused);
// mode kX8Tail: out is not written, layer 2 is the tail (ends: u32, xout, C, tw, tb, residual_sign,
// clamp_out; w16_2 / b2 unused)
void launch_conv_body_f2(const half_t* in, half_t* out, const void* w16_1, const void* w16_2, const void* w32_1,
                         const void* w32_2, const float* b1, const float* b2, const ConvShape& s, int act,
                         int num_cus, hipStream_t st, int mode = kX8Pair, const X8Ends* ends = nullptr);
// all nbody 64 -> 64 layers in one launch for small batches (grid = min(tiles, CUs)); returns
// where the result is (0: a, 1: b).  pairs: two layers per hand-off (conv_stack16x2, even
// nbody), else one.  done: s.tiles progress words (zeroed once), epoch: this launch's tag
// (advance by >= nbody + 1 per launch); err: set on a stuck wait.  u32 != nullptr (only where
// stack16_takes_head): the head layer (fp32 NCHW u32 with C channels, head_w / head_b as for
// launch_conv_head) is computed inside the launch and a is not read.
bool stack16_takes_head(int nbody, bool pairs);
int launch_conv_stack16(half_t* a, half_t* b, const void* w, const float* bias, int nbody, const ConvShape& s,
                        int act, int num_cus, int* done, int epoch, int* err, bool pairs, hipStream_t st,
                        const float* u32 = nullptr, int C = 0, const void* head_w = nullptr,
                        const float* head_b = nullptr);
// one 64 -> 64 layer with split weights W_hi + W_lo (PNP_PREC_FP16W2)
void launch_conv_body_w2(const half_t* in, half_t* out, const void* w, const void* w_lo, const float* bias,
                         const ConvShape& s, int act, int num_cus, hipStream_t st);
// split-fp16 denoiser (conv_s3.hip, PNP_PREC_FP16X3): activations as fp16 hi + lo images (two
// padded NHWC64 buffers), weights hi + lo, three fp16 MFMAs per product; 8 x 16 output tiles.
constexpr int kS3TileH = 8, kS3TileW = 16;
hipError_t conv_s3_kernels_init();
// W [64][64][3][3] -> hi / lo fragments, kBodyWBytes each
// scale: fp16x3's body weights are split at kS3WScale (256) times their value, fp16a2's at 1
void pack_body_weights_s3(const float* W, uint16_t* hi, uint16_t* lo, float scale);
void launch_conv_s3_body(const half_t* in_hi, const half_t* in_lo, half_t* out_hi, half_t* out_lo, const void* w_hi,
                         const void* w_lo, const float* bias, const ConvShape& s, int act, int num_cus,
                         hipStream_t st);
// 64 -> C + residual (x_in fp32 NCHW) + clamp -> fp32 NCHW; weights: pack_tail_weights of hi and lo
void launch_conv_s3_tail(const half_t* in_hi, const half_t* in_lo, const float* xin, float* xout, const void* w_hi,
                         const void* w_lo, const float* bias, const ConvShape& s, int C, int residual_sign,
                         int clamp_out, int num_cus, hipStream_t st);
// all nbody body layers in one launch for small batches (as launch_conv_stack16; result in a* if
// nbody is even); s3_tiles: the 8 x 16 tile count of a batch
int s3_tiles(const ConvShape& s);
void launch_conv_stack_s3(half_t* aH, half_t* aL, half_t* bH, half_t* bL, const void* w_hi, const void* w_lo,
                          const float* bias, int nbody, const ConvShape& s, int act, int num_cus, int* done, int epoch,
                          int* err, hipStream_t st);
// fp32-operand denoiser (conv32.hip, PNP_PREC_FP32): mode 0 = head (NCHW fp32 in), 1 = body,
// 2 = tail (NCHW fp32 out + residual + clamp); activations fp32 padded NHWC64, pad 1.
hipError_t conv32_kernels_init();
size_t conv32_weight_floats(int mode);
void pack_conv32_weights(const float* W, int mode, int cin, int cout, float* out);
size_t act32_bytes(int B, int H, int W);
void launch_conv32(int mode, const float* in, float* out, const float* xin, const float* w, const float* bias,
                   const ConvShape& s, int C, int act, int residual_sign, int clamp_out, int num_cus,
                   hipStream_t st);

// ---- operators / proxes (ops.hip) ----------------------------------------------------
enum { OP_ID = 0, OP_BLUR = 1, OP_MASK = 2 };
enum { M_A = 0, M_B = 1, M_C = 2 };

struct OpDesc {
  int kind;
  const int4* taps_fwd;   // {oy, ox, float bits of w, 0}: Phi:   y[i,j] += w x[i+oy, j+ox] (periodic)
  const int4* taps_adj;   //                               Phi^T: y[i,j] += w x[i+oy, j+ox]
  int ntaps;
  int R;                  // max |offset| (halo radius), <= 16
  const uint8_t* mask;    // H*W keep-mask (random_sampling)
  const float* dense_fwd; // packed tap pairs for the register-blocked stencils (ops.hip rb_stencil):
  const float* dense_adj; //   [p = 0..Rd][oy + Rd][2][2], see pack_tap_pairs
  int Rd;                 // radius of the dense tables: smallest of {2, 4, 8} >= R, 0 if R > 8
  int taps_id;            // compile-time tap pattern (TAPS_*) the stencils are specialised on, 0 = dense
  int num_cus;            // the device's CUs (grids smaller than this take the latency variants)
};
inline int dense_radius(int R) { return R <= 2 ? 2 : R <= 4 ? 4 : R <= 8 ? 8 : 0; }
enum { TAPS_DENSE = 0, TAPS_BLUR_1 = 1, TAPS_SQUARE_MINI = 2 };
// Which generated pattern (taps_gen.h) matches these column-major masks of Phi's dense table.
int match_taps(int Rd, const uint32_t* fwd_cols, const uint32_t* adj_cols);
// Column-major dense table W[ox + Rd][oy + Rd] -> the (Rd+1) x (2Rd+1) x 2 float2 pairs rb_stencil reads.
void pack_tap_pairs(int Rd, const float* W, float* out);

void launch_k1(int kind, const float* x, const float* y, const float* s, float* u32, float* w,
               const OpDesc& op, int B, int C, int H, int W, float gamma1, int clamp_in, int method_b,
               hipStream_t st);
// K1 with K3 fused into its halo fill (blur operator, register-blocked path: k1_fused_ok).
// pend: y holds v (K2's dual before the l2-ball step, omf[b] = 1 - f from launch_k3_norm) and
// the fill applies y = (1 - f)(v - g2 xobs); else y holds the dual.  yout (!= y) receives y.
bool k1_fused_ok(const OpDesc& op, int C, int H, int W);
void launch_k1_fused(const float* x, const float* y, const float* xobs, const double* omf, double gamma2, bool pend,
                     float* yout, const float* s, float* u32, float* w, const OpDesc& op, int B, int C, int H, int W,
                     float gamma1, int clamp_in, int method_b, hipStream_t st);
// K3's per-image part alone: omf[b] = 1 - f from K2's partials, and the metrics when record
void launch_k3_norm(const double* partials, const OpDesc& op, int B, int C, int H, int W, double eps, double* omf,
                    double* metrics, int it, int cap, int record, int has_true, hipStream_t st, const int* itp);
// Returns the number of per-image (min, max) partials of xn it wrote to mm ([B][chunks][2]
// floats, SSIM's data_range; mm may be null), 0 when this path does not produce them.
int launch_k2(int kind, int method, const float* xn, const float* xo, float* y, const float* xobs,
              const float* xtrue, float* s, const float* w, const float* theta, double* partials,
              const OpDesc& op, int B, int C, int H, int W, double gamma2, double gkl_gamma, double gkl_alpha,
              int record, float* mm, hipStream_t st);
// the largest chunk count launch_k2 writes to mm
int k2_minmax_chunks(int C, int H, int W);
void launch_k3(int method, float* y, const float* xobs, const double* partials, const OpDesc& op, int B, int C,
               int H, int W,
               double gamma2, double eps, double* metrics, int it, int cap, int record, int has_true,
               hipStream_t st, const int* itp = nullptr);
int partial_tiles(int H, int W);
int k2_partials(const OpDesc& op, int C, int H, int W);   // partial-sum entries per image written by launch_k2
int chunk_count(size_t n);
// theta per image; n < kMaxL1Elems keeps the radix select's bin sums exact (ops.hip sel_bin_sum).
// scratch: l1_select_scratch_bytes(B), zeroed once at allocation (the launches leave it clean).
constexpr size_t kMaxL1Elems = (size_t)1 << 29;
size_t l1_select_scratch_bytes(int B);
void launch_l1_select(const float* v, float* theta, void* scratch, int B, size_t n, double eta, hipStream_t st);
// out = Phi(x) (or Phi^T x) [+ add]
void launch_op_phi(int kind, int adj, const float* x, float* out, const OpDesc& op, int BC, int H, int W,
                   hipStream_t st, const float* add = nullptr);
void launch_l2_proj(const float* x, const float* x0, float* out, double* partials, int B, size_t n, double eps,
                    hipStream_t st);
void launch_sqdiff(const float* a, const float* c, double* partials, int B, size_t n, hipStream_t st);
void launch_shrink(const float* v, float* out, const float* theta, int B, size_t n, hipStream_t st);
void launch_gkl(const float* x, const float* x0, float* out, size_t count, double gamma, double alpha,
                hipStream_t st);
// ---- observation pipeline (degrade.hip, main.py:49-64 + utils_noise.py) ----
struct Tap64 {   // blur tap in float64: y[i,j] += v * x[(i+dy) mod H, (j+dx) mod W]
  int dy, dx;
  double v;
};
constexpr size_t kMtBlock = 624;   // MT19937 words per twist
void launch_mt_stream(uint32_t seed, uint32_t* out, size_t nwords, hipStream_t st);
size_t scan_scratch_words(size_t n);
// exclusive prefix sum of n u32 flags; scratch[0] receives the total
void launch_scan(const uint32_t* f, size_t n, uint32_t* out, uint32_t* scratch, hipStream_t st);
void launch_gauss(const uint32_t* w, size_t ncand, uint32_t* flag, uint32_t* rank, uint32_t* scan_scr, double* noise,
                  size_t n, hipStream_t st);
void launch_observe(const float* xt, const double* noise, const Tap64* taps, int ntaps, const uint8_t* mask, int kind,
                    double sigma, double* img, int B, int C, int H, int W, hipStream_t st);
void launch_poisson(const uint32_t* w, size_t nwords, double* img, int B, size_t n, double alpha,
                    unsigned long long* status, hipStream_t st);
void launch_sp_draws(const uint32_t* w, size_t nw, uint32_t mask, uint32_t rng, uint32_t* flag, uint32_t* rank,
                     uint32_t* scan_scr, uint32_t* draws, size_t ndraw, hipStream_t st);
void launch_sp_apply(const uint32_t* draws, int npairs, const uint8_t* tgt, int H, int W, uint32_t* first,
                     uint32_t* acc, uint32_t* rank, uint32_t* scan_scr, int noise_cnt, double* img, int B, int C,
                     unsigned long long* status, hipStream_t st);
void launch_degrade_finalize(const double* img, size_t N, double alpha, int poisson, float* xobs, float* x0,
                             double* xobs64, hipStream_t st);

// ---- comparison methods (methods.hip) ----
// out = x - gamma1 (D^T y1 + g); y1 is [B][2C][H][W]; g may be null
void launch_tv_primal(const float* x, const float* y1, const float* g, double gamma1, float* out, int B, int C, int H,
                      int W, hipStream_t st);
// y1 <- y1 + g2 D(2 xn - xo); y1 <- y1 - g2 prox_l12(y1 / g2, 1 / g2)
void launch_tv_dual(const float* xn, const float* xo, float* y1, double gamma2, int B, int C, int H, int W,
                    hipStream_t st);
void launch_poisson_ratio(const float* y, const float* t, double alpha, float* out, size_t N, hipStream_t st);
void launch_admm_poisson_step(float* x, const float* g, const float* c1, const float* v, const float* u,
                              double gamma, double alpha, double lam, size_t N, hipStream_t st);

// per-iteration metrics: metrics[b][it][kMetrics] = {c_n, PSNR, SSIM}
constexpr int kMetrics = 3;
// SSIM of x against xt (utils_eval.py:9-12) into metrics[b][it][2]; scratch >= ssim_scratch_bytes
size_t ssim_scratch_bytes(int B, int C, int H, int W);
// mm_ext / mm_chunks: x's (min, max) partials from launch_k2, or null (then computed here).
// psnr: also PSNR of x against xt into metrics[b][it][1], from this pass's loads (the solver's
// ours-A/B/C path then runs K2 without x_true)
void launch_ssim(const float* xt, const float* x, void* scratch, double* metrics, int B, int C, int H, int W,
                 int it, int cap, hipStream_t st, const float* mm_ext = nullptr, int mm_chunks = 0, const int* itp = nullptr,
                 bool psnr = false);
// comparisonB-2: out = k + ca*a + cb*b + cc*c + cd*d (null inputs skipped), fp64 arithmetic
void launch_lincomb(float* out, double k, const float* a, double ca, const float* b, double cb, const float* c,
                    double cc, const float* d, double cd, size_t count, hipStream_t st);
// c_n / PSNR of xn against xo / xt into metrics[b][it] (partials: B * chunk_count(n) * 4 doubles)
void launch_metrics(const float* xn, const float* xo, const float* xt, double* partials, double* metrics, int B,
                    size_t n, int it, int cap, hipStream_t st, const int* itp = nullptr);
// graph replays: the iteration number (metrics row) lives in device memory, advanced per iteration
void launch_it_advance(int* itp, hipStream_t st);
void launch_pack_input(const float* x, float* u32, int B, int C, int H, int W, int clamp_in,
                       hipStream_t st);
// dst = src, bytes a multiple of 16 (16-B aligned pointers): float4 streaming copy
void launch_copy_f4(const void* src, void* dst, size_t bytes, int num_cus, hipStream_t st);

}  // namespace pnp
