// C ABI (include/pnppds.h): device context, denoiser/operator state and the on-device
// PnP-PDS solver loop.  Host orchestration only; kernels live in ops.hip / conv.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pnppds.h"
#include "kernels.h"


using namespace pnp;

namespace {

thread_local std::string g_thread_err;

struct PnpError {
  int code;
};

// A device allocation owned by its context: freed by its destructor (pnp_destroy deletes the
// context with its device current), so no buffer can be left out of a release list.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  long long geom = -1;   // zero-border buffers: the (H,W) the whole allocation was zeroed for
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

struct ProfEntry {
  const char* name;
  hipEvent_t a, b;
};

}  // namespace

struct pnp_ctx {
  int device = 0;
  int num_cus = 256;
  double act_budget = 36e9;   // denoiser activation bytes per pass: totalGlobalMem / 8
  hipStream_t stream = nullptr;
  std::string err;

  // denoiser
  int den_C = 0, den_depth = 0, den_act = 0, den_residual = 1, den_clamp = 1;
  int den_chunk = 0;   // images per denoiser pass; 0 = auto
  int ablate = 0;         // PNP_PROFILING build only: parts of conv_body_v3 skipped, results wrong
  int fuse_ends = 1;      // PNP_TUNE_FUSE_ENDS: head / tail inside the first / last pair launch
  int body_layers = 0;    // PNP_TUNE_BODY_LAYERS: 0 auto, 1 conv_body_v3, 2 conv_body_f2, 3 conv_stack16(x2), 4 conv_stack16
  bool den_ready = false;
  int prec_req = PNP_PREC_AUTO;   // pnp_set_precision (default: the per-solve policy, auto_precision)
  int prec = PNP_PREC_FP16X3;     // the operands the denoiser runs with now (resolved from prec_req)
  // PNP_PREC_CONVERGE (converge_check): per image, auto's operands until the image's own c_n
  // falls below conv_c, split activations from then on.  conv_row: pinned host rows of c_n (two
  // slots of B doubles) copied after each watched iteration, conv_ev / conv_slot_it: their events
  // and the iteration each slot holds.
  double conv_c = 3e-3;
  bool conv_switched = false;     // every image has switched
  int conv_switch_it = -1;        // the first iteration every image ran split (-1: not yet)
  std::vector<int> conv_img_it;   // per image: its first split iteration (-1: not yet)
  int conv_nsw = 0;               // images switched
  double* conv_row = nullptr;
  int conv_row_B = 0;
  hipEvent_t conv_ev[2] = {nullptr, nullptr};
  int conv_slot_it[2] = {-1, -1};
  DevBuf head_w, head_b, body_w, body_b, tail_w, tail_b;
  DevBuf body_w16;                       // 16x16x32 MFMA fragments of the body layers (conv_body_x8)
  DevBuf head_w32, body_w32, tail_w32;   // fp32 MFMA fragments (PNP_PREC_FP32)
  DevBuf head_wlo, body_wlo, tail_wlo;   // fp16 low halves W - fp16(W) (PNP_PREC_FP16W2 / FP16X3)
  DevBuf body_s3h, body_s3l;             // conv_s3 body fragments, hi / lo (PNP_PREC_FP16X3)
  DevBuf body_s3f;                       // conv_s3 body fragments of the fp16 weights (PNP_PREC_FP16A2)
  DevBuf head_wx3, head_wlox3, tail_wx3, tail_wlox3;   // split head / tail weights at kSplitWScale (FP16X3 / A2)

  // operator
  int op_kind = PNP_OP_ID;
  int op_H = 0, op_W = 0;
  int op_ntaps = 0, op_R = 0, op_taps_id = 0;
  DevBuf taps_fwd, taps_adj, mask, dense_fwd, dense_adj, taps64;

  // solver
  int method = -1, B = 0, C = 0, H = 0, W = 0, cap = 0, it = 0;
  bool loaded = false, has_true = false;
  pnp_params prm{};
  int cur = 0;
  DevBuf x[2], y, s, w, xobs, xtrue, u32, act[2], partials, metrics, theta;
  // A / B on the blur operator (k1_fused_ok): K3 runs inside the next K1 (launch_k1_fused). The
  // dual then alternates between y (cur 0) and y2 (cur 1) like x; ypend: it holds v, K2's dual
  // before the l2-ball step, and omf[b] = 1 - f (finalize_dual applies it in place).
  DevBuf y2, omf;
  bool ypend = false;
  DevBuf act_lo[2]; // low halves of the hidden activations (PNP_PREC_FP16X3)
  DevBuf z, p, t;   // comparisonB-2 and the other comparison methods
  DevBuf y1, d, c1; // TV dual [B][2C][H][W]; Poisson-ADMM d and Phi^T 1
  DevBuf ssim_scr;  // SSIM partials (record_ssim)
  DevBuf ssim_mm;   // x+ (min, max) partials written by K2 for SSIM's data_range

  // observation pipeline (pnp_degrade)
  DevBuf dg_words, dg_flag, dg_rank, dg_scan, dg_noise, dg_img, dg_draws, dg_first, dg_status;
  size_t dg_nwords = 0;
  uint32_t dg_seed = 0;

  // scratch for single ops
  DevBuf scr_u32, scr_act[2], scr_act_lo[2], scr_part, scr_theta;
  DevBuf act32[2];   // fp32 hidden activations (PNP_PREC_FP32) of the solver
  DevBuf l1_scr;     // l1-ball select histograms + per-image state (launch_l1_select) of the solver
  // the stream-parameterised single ops (pnp_op_*) keep their own stateful scratch, so they never
  // share zero-border or cleared-bin buffers with the solver across streams or graph replays
  DevBuf scr_act32[2], scr_l1;

  // graph replay of the iteration launches (small batches): PNP_TUNE_GRAPH
  int graph_mode = 0;          // 0 off (default), 1 on
  long long gen = 0;           // bumped by every setter and buffer (re)allocation: a graph built at
  long long warm_gen = -1;     //   another generation is stale; warm_gen: gen after the last plain step
  hipGraphExec_t gexec = nullptr;
  long long gexec_gen = -1;
  bool capturing = false;      // solver_step is being captured: record unconditionally, itp set
  const int* itp = nullptr;    // device iteration counter the metric kernels read while captured
  DevBuf it_dev;

  // persistent small-batch denoiser (conv_stack16): per-tile progress words, one array for the
  // solver's stream and one for the single ops (concurrent launches must not share them)
  DevBuf stack_done, scr_stack_done, stack_err, scr_stack_err;
  int stack_epoch = 0, scr_stack_epoch = 0;

  // profiling
  int prof = 0;           // pnp_profile_enable: 0 off, 1 every launch, 2 body launches only
  std::vector<ProfEntry> prof_log;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
};

namespace {

void fail(pnp_ctx* ctx, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  g_thread_err = buf;
  throw PnpError{code};
}

#define HIPCHK(ctx, expr)                                                                     \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) fail(ctx, PNP_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                               __FILE__, __LINE__);                                           \
  } while (0)

void check_launch(pnp_ctx* ctx, const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(ctx, PNP_E_HIP, "launch %s: %s", what, hipGetErrorString(e));
}

template <class F>
int guarded(pnp_ctx* ctx, F&& f) {
  try {
    if (ctx) {
      hipError_t e = hipSetDevice(ctx->device);
      if (e != hipSuccess) fail(ctx, PNP_E_HIP, "hipSetDevice(%d): %s", ctx->device, hipGetErrorString(e));
    }
    f();
    return PNP_OK;
  } catch (const PnpError& e) {
    return e.code;
  } catch (const std::exception& e) {
    if (ctx) ctx->err = e.what();
    g_thread_err = e.what();
    return PNP_E_ARG;
  }
}

void ensure(pnp_ctx* ctx, DevBuf& b, size_t bytes, bool zero = false) {
  if (bytes == 0) bytes = 16;
  if (b.p && b.bytes >= bytes) return;
  // before the grow path: its stream sync and hipFree would invalidate the capture
  if (ctx->capturing) fail(ctx, PNP_E_STATE, "allocation inside a graph capture");
  if (b.p) {
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHK(ctx, hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
  }
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) fail(ctx, PNP_E_OOM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  ctx->gen++;
  b.bytes = bytes;
  b.geom = -1;
  if (zero) HIPCHK(ctx, hipMemsetAsync(b.p, 0, bytes, ctx->stream));
}

void release(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

template <class T>
T* P(DevBuf& b) {
  return reinterpret_cast<T*>(b.p);
}

hipStream_t pick_stream(pnp_ctx* ctx, void* stream) {
  return stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
}

// -------- profiling (hipEvents around each launch group on the solver stream) ---------
hipEvent_t next_event(pnp_ctx* ctx) {
  if (ctx->ev_used == ctx->ev_pool.size()) {
    hipEvent_t e;
    HIPCHK(ctx, hipEventCreate(&e));
    ctx->ev_pool.push_back(e);
  }
  return ctx->ev_pool[ctx->ev_used++];
}

struct ProfScope {
  pnp_ctx* ctx;
  const char* name;
  hipStream_t st;
  hipEvent_t a = nullptr;
  // prof 2: only the denoiser's body launches (the bench's timed region: the dominant kernel's
  // duration without the other scopes' event packets between launches)
  static bool body(const char* n) {
    return !strncmp(n, "conv_body", 9) || !strncmp(n, "conv32_body", 11) || !strncmp(n, "conv_stack", 10);
  }
  bool on() const { return ctx->prof == 1 || (ctx->prof == 2 && body(name)); }
  ProfScope(pnp_ctx* c, const char* n, hipStream_t s) : ctx(c), name(n), st(s) {
    if (on()) {
      a = next_event(ctx);
      HIPCHK(ctx, hipEventRecord(a, st));
    }
  }
  ~ProfScope() noexcept(false) {
    if (a) {
      hipEvent_t b = next_event(ctx);
      HIPCHK(ctx, hipEventRecord(b, st));
      ctx->prof_log.push_back({name, a, b});
    }
  }
};

// -------- fp16 weights: rounding that keeps each 3x3 filter's sum -----------------------
// The fp16 operand precisions store every weight as an fp16 value.  Plain round-to-nearest
// leaves each (c_out, c_in) filter's DC gain off by the sum of its nine rounding errors, and on
// the reference's smooth images that sum is what the error of a layer's output mostly is
// (fp16 weights cost cfg1 0.069 dB over 40 iterations, fp16 activations 0.009).
// Here each filter starts from round-to-nearest and moves taps to their other fp16 neighbour
// (the other side of the fp32 weight), cheapest added error first, while a move shrinks
// |sum of the filter's errors|; every error stays below one fp16 ulp (emulated: cfg1 0.066 ->
// 0.011 dB).  The sums are exact in double (a few dozen bits span), so the choice does not
// depend on summation order; ties go to the lower tap index.  The test oracle
// (fp16_filter_round) restates it for the fp16-emulating checker.
uint16_t f16_step(uint16_t b, bool up) {   // the next fp16 toward +inf (up) or -inf
  const bool neg = (b & 0x8000) != 0, zero = (b & 0x7fff) == 0;
  if (zero) return up ? 0x0001 : 0x8001;
  return (up != neg) ? (uint16_t)(b + 1) : (uint16_t)(b - 1);
}
float f16_value(uint16_t b) {
  _Float16 h;
  std::memcpy(&h, &b, 2);
  return (float)h;
}
void fp16_filter_round(const float* w, size_t nfilt, float* out) {
  for (size_t f = 0; f < nfilt; ++f) {
    const float* wf = w + 9 * f;
    float r[9], alt[9];
    double cost[9];
    bool used[9];
    double S = 0.0;
    for (int k = 0; k < 9; ++k) {
      const _Float16 h = (_Float16)wf[k];
      uint16_t hb;
      std::memcpy(&hb, &h, 2);
      r[k] = (float)h;
      alt[k] = r[k] == wf[k] ? r[k] : f16_value(f16_step(hb, r[k] < wf[k]));
      cost[k] = std::fabs((double)alt[k] - wf[k]) - std::fabs((double)r[k] - wf[k]);
      used[k] = false;
      S += (double)r[k] - (double)wf[k];
    }
    for (;;) {
      int best = -1;
      for (int k = 0; k < 9; ++k) {
        if (used[k]) continue;
        const double d = (double)alt[k] - (double)r[k];
        if (std::fabs(S + d) < std::fabs(S) && (best < 0 || cost[k] < cost[best])) best = k;
      }
      if (best < 0) break;
      S += (double)alt[best] - (double)r[best];
      r[best] = alt[best];
      used[best] = true;
    }
    std::memcpy(out + 9 * f, r, sizeof(r));
  }
}

// -------- operator descriptor --------------------------------------------------------
OpDesc op_desc(pnp_ctx* ctx) {
  OpDesc d;
  d.kind = ctx->op_kind;
  d.taps_fwd = P<const int4>(ctx->taps_fwd);
  d.taps_adj = P<const int4>(ctx->taps_adj);
  d.ntaps = ctx->op_ntaps;
  d.R = ctx->op_R;
  d.mask = P<const uint8_t>(ctx->mask);
  d.dense_fwd = ctx->op_kind == PNP_OP_BLUR ? P<const float>(ctx->dense_fwd) : nullptr;
  d.dense_adj = ctx->op_kind == PNP_OP_BLUR ? P<const float>(ctx->dense_adj) : nullptr;
  d.Rd = ctx->op_kind == PNP_OP_BLUR ? dense_radius(ctx->op_R) : 0;
  d.taps_id = ctx->op_kind == PNP_OP_BLUR ? ctx->op_taps_id : TAPS_DENSE;
  d.num_cus = ctx->num_cus;
  return d;
}

void check_operator_shape(pnp_ctx* ctx, int H, int W) {
  if (ctx->op_kind == PNP_OP_RANDOM_SAMPLING && (H != ctx->op_H || W != ctx->op_W))
    fail(ctx, PNP_E_ARG, "random_sampling mask is %dx%d, image is %dx%d", ctx->op_H, ctx->op_W, H, W);
  if (ctx->op_kind == PNP_OP_BLUR && (H < 1 || W < 1))
    fail(ctx, PNP_E_ARG, "bad image size");
}

// -------- denoiser forward: u32 (NCHW fp32) -> xout ------------------------------------
size_t act_bytes(int B, int H, int W, int ch, int pad) {
  // + slack: partial tiles read up to 12 rows / 36 pixels past the last image
  const size_t Wp = (size_t)W + 2 * pad;
  return ((size_t)B * (H + 2 * pad) * Wp + 16 * Wp + 64) * ch * sizeof(half_t);
}

// Padded activation images: the one-pixel border must be zero for the geometry in use.
// Kernels never write the border, so a buffer is zeroed once per (H, W) it serves, over its
// whole allocation: an image's slot (offset and border) does not depend on the batch size, so
// any batch the allocation holds finds its borders zero (PNP_PREC_CONVERGE's per-image passes
// alternate batch sizes every iteration).  Reusing it for another image size (whose border
// lands on stale interior data) re-zeroes; growing it reallocates (ensure resets geom).
void ensure_padded(pnp_ctx* ctx, DevBuf& b, int B, int H, int W, int ch, int pad, hipStream_t st) {
  const size_t bytes = act_bytes(B, H, W, ch, pad);
  const long long geom = ((long long)H << 20) ^ (long long)W;
  ensure(ctx, b, bytes);
  if (b.geom != geom) {
    HIPCHK(ctx, hipMemsetAsync(b.p, 0, b.bytes, st));
    b.geom = geom;
  }
}

void ensure_act(pnp_ctx* ctx, DevBuf (&act)[2], int B, int H, int W, hipStream_t st) {
  for (int i = 0; i < 2; ++i) ensure_padded(ctx, act[i], B, H, W, kWidth, kActPad, st);
}

// Images per denoiser pass: see denoise_chunk / split_passes below.  (Passes sized to stay in
// the 256 MB Infinity Cache measured no faster at 256x256: conv_body is not HBM-bound.)
// Two body layers per launch (conv_body_f2) when its strips fill the chip: one workgroup per
// 32-column strip walks the strip's rows serially, so a batch with fewer strips than CUs (B = 1
// at 256^2: 8 strips, 0.23 ms per layer pair) runs one layer per launch over 8 x 32 tiles
// (256 workgroups, 0.013 ms per layer).  Auto = at least one strip per CU and >= 80 % of the
// last round of strips busy.
bool use_pair(pnp_ctx* ctx, int mb, int W) {
  if (ctx->body_layers) return ctx->body_layers == 2;
  const long long strips = (long long)mb * ((W + kTileW - 1) / kTileW), cus = ctx->num_cus;
  const long long rounds = (strips + cus - 1) / cus;
  return strips >= cus && strips * 5 >= rounds * cus * 4;
}

// All body layers in one persistent launch (conv_stack16) for small batches: at most 2 tiles
// of 8 x 32 per CU (B = 1 at 256^2: 256 tiles), where per-layer launches are fixed-cost-bound
// (~11 us each for ~2 us of MFMA work).  Not while a graph is captured: the launch's epoch tag
// is a kernel argument, which a replay would repeat.  Only on the context's own stream (the
// solver's, and single ops called without a stream), so two of the context's persistent grids
// never compete for CUs (common.h persistent_launch).
bool use_stack(pnp_ctx* ctx, int tiles, hipStream_t st) {
  if (ctx->capturing || st != ctx->stream) return false;   // one persistent grid at a time per context
  if (ctx->body_layers) return ctx->body_layers >= 3;
  return tiles <= 2 * ctx->num_cus;
}

// The progress words, this launch's epoch (advanced by nbody + 1 per launch; the words are
// reset before the tag could wrap) and the error word a stuck wait sets: the solver's
// (checked by pnp_solver_fetch) or the single ops' (checked by pnp_op_status).
int* stack_flags(pnp_ctx* ctx, bool solver, int tiles, int nbody, hipStream_t st, int& epoch, int*& err) {
  DevBuf& d = solver ? ctx->stack_done : ctx->scr_stack_done;
  DevBuf& ew = solver ? ctx->stack_err : ctx->scr_stack_err;
  int& e = solver ? ctx->stack_epoch : ctx->scr_stack_epoch;
  if (!d.p || d.bytes < (size_t)tiles * sizeof(int)) {
    ensure(ctx, d, (size_t)std::max(tiles, 4096) * sizeof(int));
    HIPCHK(ctx, hipMemsetAsync(d.p, 0, d.bytes, st));
    e = 0;
  }
  if (!ew.p) {
    ensure(ctx, ew, sizeof(int));
    HIPCHK(ctx, hipMemsetAsync(ew.p, 0, sizeof(int), st));
  }
  if (e > (1 << 30)) {
    HIPCHK(ctx, hipMemsetAsync(d.p, 0, d.bytes, st));
    e = 0;
  }
  epoch = e + 1;
  e += nbody + 1;
  err = P<int>(ew);
  return P<int>(d);
}

// split activations (hi + lo images): fp16x3, and fp16a2 (its body without the a_hi w_lo term)
bool split_acts(int prec) { return prec == PNP_PREC_FP16X3 || prec == PNP_PREC_FP16A2; }

// Images per denoiser pass.  The two ping-pong activation buffers may take an eighth of the
// card's HBM (36 GB of the MI355X's 288 GB: cfg5's 64 x 1024^2 shard, 17.3 GB, is one pass),
// and a batch that needs several passes is split into equal ones: a small remainder pass
// has fewer 32-column strips than CUs and falls back to one body layer per launch (cfg5
// with the former 8 GB budget: passes of 29 + 29 + 6 images, the 6-image pass on one-layer
// launches).  Per-image results do not depend on the split (test_batch_equals_single_images).
int split_passes(int B, double per_img, double budget) {
  const int m = std::max(1, std::min((int)std::floor(budget / per_img), B));
  const int passes = (B + m - 1) / m;
  return (B + passes - 1) / passes;
}

int denoise_chunk(pnp_ctx* ctx, int B, int H, int W) {
  if (ctx->den_chunk > 0) return std::min(ctx->den_chunk, B);
  const double planes = split_acts(ctx->prec) ? 4.0 : 2.0;   // X3 / A2: hi + lo ping-pong pairs
  const double per_img = planes * (H + 2 * kActPad) * (W + 2 * kActPad) * kWidth * sizeof(half_t);
  return split_passes(B, per_img, ctx->act_budget);
}

// fp32-operand forward (PNP_PREC_FP32): u32 (NCHW, clamped input) -> xout, conv32.hip.
void run_denoiser32(pnp_ctx* ctx, const float* u32, float* xout, DevBuf (&act32)[2], int B, int H, int W,
                    hipStream_t st) {
  const double per_img = 2.0 * act32_bytes(1, H, W);
  const int m = ctx->den_chunk > 0 ? std::min(ctx->den_chunk, B) : split_passes(B, per_img, ctx->act_budget);
  for (int i = 0; i < 2; ++i) {                 // one-pixel zero border, zeroed once per geometry
    const long long geom = ((long long)m << 40) ^ ((long long)H << 20) ^ (long long)W;
    ensure(ctx, act32[i], act32_bytes(m, H, W));
    if (act32[i].geom != geom) {
      HIPCHK(ctx, hipMemsetAsync(act32[i].p, 0, act32_bytes(m, H, W), st));
      act32[i].geom = geom;
    }
  }
  const int C = ctx->den_C, nbody = ctx->den_depth - 2;
  const size_t wb = conv32_weight_floats(1);
  for (int b0 = 0; b0 < B; b0 += m) {
    const int mb = std::min(m, B - b0);
    ConvShape s = make_conv_shape(mb, H, W);
    const float* xin = u32 + (size_t)b0 * C * H * W;
    float* xo = xout + (size_t)b0 * C * H * W;
    {
      ProfScope ps(ctx, "conv32_head", st);
      launch_conv32(0, xin, P<float>(act32[0]), nullptr, P<float>(ctx->head_w32), P<float>(ctx->head_b), s, C,
                    ctx->den_act, 1, 0, ctx->num_cus, st);
      check_launch(ctx, "conv32_head");
    }
    int cur = 0;
    for (int l = 0; l < nbody; ++l, cur ^= 1) {
      ProfScope ps(ctx, "conv32_body", st);
      launch_conv32(1, P<float>(act32[cur]), P<float>(act32[cur ^ 1]), nullptr,
                    P<float>(ctx->body_w32) + (size_t)l * wb, P<float>(ctx->body_b) + l * kWidth, s, C, ctx->den_act,
                    1, 0, ctx->num_cus, st);
      check_launch(ctx, "conv32_body");
    }
    {
      ProfScope ps(ctx, "conv32_tail", st);
      launch_conv32(2, P<float>(act32[cur]), xo, xin, P<float>(ctx->tail_w32), P<float>(ctx->tail_b), s, C,
                    ctx->den_act, ctx->den_residual, ctx->den_clamp, ctx->num_cus, st);
      check_launch(ctx, "conv32_tail");
    }
  }
}

// Denoiser forward over B images with the operands ctx->prec: u32 (NCHW fp32: the head's input
// and the residual) -> xout.
void run_denoiser_prec(pnp_ctx* ctx, const float* u32, float* xout, DevBuf (&act)[2], int B, int H,
                       int W, hipStream_t st) {
  if (!ctx->den_ready) fail(ctx, PNP_E_STATE, "denoiser not set (pnp_set_denoiser)");
  if (ctx->prec == PNP_PREC_FP32) {
    run_denoiser32(ctx, u32, xout, &act[0] == &ctx->act[0] ? ctx->act32 : ctx->scr_act32, B, H, W, st);
    return;
  }
  const int m = denoise_chunk(ctx, B, H, W);
  ensure_act(ctx, act, m, H, W, st);
  const int C = ctx->den_C;
  if (split_acts(ctx->prec)) {                 // split fp16 (conv_s3.hip): hi images in act, lo in act_lo
    const bool a2 = ctx->prec == PNP_PREC_FP16A2;   // a2: fp16 weights in the body (two MFMAs per product)
    DevBuf(&alo)[2] = &act[0] == &ctx->act[0] ? ctx->act_lo : ctx->scr_act_lo;
    ensure_act(ctx, alo, m, H, W, st);
    for (int b0 = 0; b0 < B; b0 += m) {
      const int mb = std::min(m, B - b0);
      ConvShape s = make_conv_shape(mb, H, W);
      const float* xin = u32 + (size_t)b0 * C * H * W;
      float* xo = xout + (size_t)b0 * C * H * W;
      {
        ProfScope ps(ctx, "conv_head", st);
        launch_conv_head(xin, C, P<half_t>(act[0]), ctx->head_wx3.p, ctx->head_wlox3.p, P<float>(ctx->head_b), s,
                         ctx->den_act, ctx->num_cus, 4, st, P<half_t>(alo[0]));
        check_launch(ctx, "conv_head");
      }
      int cur = 0;
      const int nbody = ctx->den_depth - 2;
      const bool stack = nbody > 0 && use_stack(ctx, s3_tiles(s), st);
      if (stack) {                                 // every body layer in one launch
        ProfScope ps(ctx, "conv_stack_s3", st);
        int epoch = 0;
        int* err = nullptr;
        int* done = stack_flags(ctx, &act[0] == &ctx->act[0], s3_tiles(s), nbody, st, epoch, err);
        launch_conv_stack_s3(P<half_t>(act[0]), P<half_t>(alo[0]), P<half_t>(act[1]), P<half_t>(alo[1]),
                             a2 ? ctx->body_s3f.p : ctx->body_s3h.p, a2 ? nullptr : ctx->body_s3l.p,
                             P<float>(ctx->body_b), nbody, s, ctx->den_act,
                             ctx->num_cus, done, epoch, err, st);
        check_launch(ctx, "conv_stack_s3");
        cur = nbody & 1;
      }
      for (int l = stack ? nbody : 0; l < nbody; ++l, cur ^= 1) {
        ProfScope ps(ctx, a2 ? "conv_body_a2" : "conv_body_s3", st);
        launch_conv_s3_body(P<half_t>(act[cur]), P<half_t>(alo[cur]), P<half_t>(act[cur ^ 1]), P<half_t>(alo[cur ^ 1]),
                            (const char*)(a2 ? ctx->body_s3f.p : ctx->body_s3h.p) + (size_t)l * kBodyWBytes,
                            a2 ? nullptr : (const char*)ctx->body_s3l.p + (size_t)l * kBodyWBytes,
                            P<float>(ctx->body_b) + l * kWidth, s, ctx->den_act, ctx->num_cus, st);
        check_launch(ctx, "conv_body_s3");
      }
      {
        ProfScope ps(ctx, "conv_tail_s3", st);
        launch_conv_s3_tail(P<half_t>(act[cur]), P<half_t>(alo[cur]), xin, xo, ctx->tail_wx3.p, ctx->tail_wlox3.p,
                            P<float>(ctx->tail_b), s, C, ctx->den_residual, ctx->den_clamp, ctx->num_cus, st);
        check_launch(ctx, "conv_tail_s3");
      }
    }
    return;
  }
  for (int b0 = 0; b0 < B; b0 += m) {
    const int mb = std::min(m, B - b0);
    ConvShape s = make_conv_shape(mb, H, W);
    const float* xin = u32 + (size_t)b0 * C * H * W;
    float* xo = xout + (size_t)b0 * C * H * W;
    const bool w2 = ctx->prec == PNP_PREC_FP16W2;
    int cur = 0;
    const int nbody = ctx->den_depth - 2;
    const bool pair = use_pair(ctx, mb, W);
    const bool stack = !w2 && !ctx->ablate && nbody > 0 && use_stack(ctx, s.tiles, st);
    const bool stack_pairs = ctx->body_layers != 4;
    // the two-layer stack computes the head itself (its first pair's input halo)
    const bool head_in_stack = stack && stack16_takes_head(nbody, stack_pairs);
    // head + L0 and L(n-1) + tail in the first and last pair launches (conv_body_x8_kernel's HEAD /
    // TAIL modes): the pairs L1 .. L(n-2) between need an even body depth
    // (HEAD / TAIL address the pass's fp32 input through one buffer resource: under 2 GB)
    const bool fuse = !w2 && pair && !stack && !ctx->ablate && ctx->fuse_ends && nbody >= 2 && nbody % 2 == 0 &&
                      C <= kMaxC && (size_t)mb * C * H * W * sizeof(float) < ((size_t)1 << 31);
    if (fuse) {
      ProfScope ps(ctx, "conv_body_f2h", st);
      X8Ends e;
      e.u32 = xin;
      e.hw = ctx->head_w.p;
      e.hb = P<float>(ctx->head_b);
      e.C = C;
      const char* w16 = (const char*)ctx->body_w16.p;
      launch_conv_body_f2(nullptr, P<half_t>(act[0]), w16, w16, ctx->body_w.p, ctx->body_w.p, P<float>(ctx->body_b),
                          P<float>(ctx->body_b), s, ctx->den_act, ctx->num_cus, st, kX8Head, &e);
      check_launch(ctx, "conv_body_f2h");
    } else if (!head_in_stack) {
      ProfScope ps(ctx, "conv_head", st);
      launch_conv_head(xin, C, P<half_t>(act[0]), ctx->head_w.p, w2 ? ctx->head_wlo.p : nullptr, P<float>(ctx->head_b),
                       s, ctx->den_act, ctx->num_cus, 4, st);
      check_launch(ctx, "conv_head");
    }
    if (stack) {                                 // every body layer in one launch
      ProfScope ps(ctx, "conv_stack16", st);
      int epoch = 0;
      int* err = nullptr;
      int* done = stack_flags(ctx, &act[0] == &ctx->act[0], s.tiles, nbody, st, epoch, err);
      cur = launch_conv_stack16(P<half_t>(act[0]), P<half_t>(act[1]), ctx->body_w.p, P<float>(ctx->body_b), nbody,
                                s, ctx->den_act, ctx->num_cus, done, epoch, err, stack_pairs, st,
                                head_in_stack ? xin : nullptr, C, ctx->head_w.p, P<float>(ctx->head_b));
      check_launch(ctx, "conv_stack16");
    }
    for (int l = stack ? nbody : fuse ? 1 : 0; l < (fuse ? nbody - 1 : nbody);) {
      const char* wl = (const char*)ctx->body_w.p + (size_t)l * kBodyWBytes;
      const float* bl = P<float>(ctx->body_b) + l * kWidth;
      if (!w2 && pair && !ctx->ablate && l + 1 < nbody) {   // layers l, l+1 in one launch
        ProfScope ps(ctx, "conv_body_f2", st);
        const char* w16 = (const char*)ctx->body_w16.p + (size_t)l * kBodyWBytes;
        launch_conv_body_f2(P<half_t>(act[cur]), P<half_t>(act[cur ^ 1]), w16, w16 + kBodyWBytes, wl,
                            wl + kBodyWBytes, bl, bl + kWidth, s, ctx->den_act, ctx->num_cus, st);
        check_launch(ctx, "conv_body_f2");
        l += 2;
        cur ^= 1;
        continue;
      }
      if (w2) {
        ProfScope ps(ctx, "conv_body_w2", st);
        launch_conv_body_w2(P<half_t>(act[cur]), P<half_t>(act[cur ^ 1]), wl,
                            (const char*)ctx->body_wlo.p + (size_t)l * kBodyWBytes, bl, s, ctx->den_act, ctx->num_cus,
                            st);
        check_launch(ctx, "conv_body_w2");
      } else {
        ProfScope ps(ctx, "conv_body", st);
        launch_conv_body(P<half_t>(act[cur]), P<half_t>(act[cur ^ 1]), wl, bl, s, ctx->den_act, ctx->num_cus,
                         ctx->ablate, st);
        check_launch(ctx, "conv_body");
      }
      l += 1;
      cur ^= 1;
    }
    if (fuse) {
      ProfScope ps(ctx, "conv_body_f2t", st);
      X8Ends e;
      e.u32 = xin;
      e.xout = xo;
      e.tw = ctx->tail_w.p;
      e.tb = P<float>(ctx->tail_b);
      e.C = C;
      e.residual_sign = ctx->den_residual;
      e.clamp_out = ctx->den_clamp;
      const size_t l = nbody - 1;
      const char* w16 = (const char*)ctx->body_w16.p + l * kBodyWBytes;
      const char* wl = (const char*)ctx->body_w.p + l * kBodyWBytes;
      const float* bl = P<float>(ctx->body_b) + l * kWidth;
      launch_conv_body_f2(P<half_t>(act[cur]), nullptr, w16, w16, wl, wl, bl, bl, s, ctx->den_act, ctx->num_cus, st,
                          kX8Tail, &e);
      check_launch(ctx, "conv_body_f2t");
    } else {
      ProfScope ps(ctx, "conv_tail", st);
      launch_conv_tail(P<half_t>(act[cur]), xin, xo, ctx->tail_w.p, w2 ? ctx->tail_wlo.p : nullptr,
                       P<float>(ctx->tail_b), s, C, ctx->den_residual, ctx->den_clamp, ctx->num_cus, st);
      check_launch(ctx, "conv_tail");
    }
  }
}

int converge_precision(int fast);

// Denoiser forward over B images: u32 (NCHW fp32: the head's input and the residual) -> xout.
// A solver pass under PNP_PREC_CONVERGE while only some images have switched runs each maximal
// run of consecutive images with one precision as its own pass (ctx->prec for the images still
// on auto's operands, converge_precision(ctx->prec) for the switched ones).  Per-image results
// do not depend on how a batch is split into passes (test_batch_equals_single_images), so an
// image's bits depend only on its own c_n history, not on its batch or shard.
void run_denoiser(pnp_ctx* ctx, const float* u32, float* xout, DevBuf (&act)[2], int B, int H,
                  int W, hipStream_t st) {
  if (&act[0] != &ctx->act[0] || ctx->prec_req != PNP_PREC_CONVERGE || ctx->conv_switched || ctx->conv_nsw == 0 ||
      B != ctx->B || (int)ctx->conv_img_it.size() != B) {
    run_denoiser_prec(ctx, u32, xout, act, B, H, W, st);
    return;
  }
  const int fast = ctx->prec, slow = converge_precision(fast);
  struct Restore {
    pnp_ctx* c;
    int p;
    ~Restore() { c->prec = p; }
  } restore{ctx, fast};
  const size_t img = (size_t)ctx->den_C * H * W;
  for (int b0 = 0; b0 < B;) {
    const bool sw = ctx->conv_img_it[b0] >= 0;
    int b1 = b0 + 1;
    while (b1 < B && (ctx->conv_img_it[b1] >= 0) == sw) ++b1;
    ctx->prec = sw ? slow : fast;
    run_denoiser_prec(ctx, u32 + b0 * img, xout + b0 * img, act, b1 - b0, H, W, st);
    b0 = b1;
  }
}

// l1-ball threshold per image into theta.  The scratch (histogram bins every launch leaves
// cleared) is grown and zeroed on demand on the stream that uses it: the solver's (ctx->l1_scr,
// ctx->stream) or a single op's (ctx->scr_l1, the caller's stream).
void l1_select(pnp_ctx* ctx, DevBuf& scr, const float* v, float* theta, int B, size_t n, double eta,
               hipStream_t st) {
  const size_t need = l1_select_scratch_bytes(B);
  if (!scr.p || scr.bytes < need) {
    ensure(ctx, scr, need);
    HIPCHK(ctx, hipMemsetAsync(scr.p, 0, scr.bytes, st));
  }
  launch_l1_select(v, theta, scr.p, B, n, eta, st);
}

// -------- one solver iteration -------------------------------------------------------
double l2_eps(pnp_ctx* ctx, size_t n) {
  const pnp_params& p = ctx->prm;
  const double r = ctx->method == PNP_METHOD_B ? p.r : 1.0;   // A passes no r (iteration.py:52)
  return std::sqrt((double)n * (1.0 - p.sp_nl)) * r * p.alpha_n * p.gaussian_nl;
}

// iteration.py:189: ssim_data[i] = eval_ssim(x_true, x_n), only when asked (record_ssim)
bool want_ssim(pnp_ctx* ctx) {
  const pnp_params& p = ctx->prm;
  return p.record_metrics && p.record_ssim && ctx->has_true && (ctx->capturing || ctx->it < ctx->cap);
}

// mm_chunks > 0: K2 already wrote x+'s (min, max) partials to ctx->ssim_mm.  psnr: the PSNR of
// this iteration comes from the SSIM pass too (it loads x_true and x+ anyway): K2 then skipped its
// x_true loads (r05 A/B at the metric: K2 0.279 -> 0.239 ms), and what k3_norm wrote from K2's
// partials for the PSNR is overwritten here, later in the same iteration.
void record_ssim(pnp_ctx* ctx, const float* xn, hipStream_t st, int mm_chunks = 0, bool psnr = false) {
  if (!want_ssim(ctx)) return;
  ProfScope ps(ctx, "ssim", st);
  launch_ssim(P<float>(ctx->xtrue), xn, ctx->ssim_scr.p, P<double>(ctx->metrics), ctx->B, ctx->C, ctx->H, ctx->W,
              ctx->it, ctx->cap, st, mm_chunks > 0 ? P<float>(ctx->ssim_mm) : nullptr, mm_chunks, ctx->itp, psnr);
  check_launch(ctx, "ssim");
}

// K3 fused into the next K1 (ours-A / ours-B on the register-blocked blur path)
bool dual_fused(pnp_ctx* ctx, const OpDesc& od) {
  return (ctx->method == PNP_METHOD_A || ctx->method == PNP_METHOD_B) && k1_fused_ok(od, ctx->C, ctx->H, ctx->W);
}
float* dual_buf(pnp_ctx* ctx, int i) { return P<float>(i ? ctx->y2 : ctx->y); }

// The dual state as the reference holds it: applies a pending l2-ball step (K3) in place.
void finalize_dual(pnp_ctx* ctx) {
  if (!ctx->ypend) return;
  const OpDesc od = op_desc(ctx);
  const size_t n = (size_t)ctx->C * ctx->H * ctx->W;
  launch_k3(ctx->method, dual_buf(ctx, ctx->cur), P<float>(ctx->xobs), P<double>(ctx->partials), od, ctx->B, ctx->C,
            ctx->H, ctx->W, ctx->prm.gamma2, l2_eps(ctx, n), P<double>(ctx->metrics), 0, ctx->cap, 0, ctx->has_true,
            ctx->stream);
  check_launch(ctx, "k3 (finalize)");
  ctx->ypend = false;
  ctx->gen++;   // a captured graph holds the pending-dual K1: the next run recaptures
}

void solver_iteration(pnp_ctx* ctx) {
  hipStream_t st = ctx->stream;
  const pnp_params& p = ctx->prm;
  const int B = ctx->B, C = ctx->C, H = ctx->H, W = ctx->W;
  const size_t n = (size_t)C * H * W;
  const OpDesc od = op_desc(ctx);
  float* xo = P<float>(ctx->x[ctx->cur]);
  float* xn = P<float>(ctx->x[ctx->cur ^ 1]);
  const bool mb = ctx->method == PNP_METHOD_B;
  const int record = p.record_metrics && (ctx->capturing || ctx->it < ctx->cap);
  const bool fused = dual_fused(ctx, od);
  float* y = fused ? dual_buf(ctx, ctx->cur ^ 1) : P<float>(ctx->y);   // the dual K2 reads and updates
  const bool psnr_in_ssim = want_ssim(ctx);   // the SSIM pass computes the PSNR (record_ssim)
  {
    ProfScope ps(ctx, "k1_primal_pre", st);
    if (fused)
      launch_k1_fused(xo, dual_buf(ctx, ctx->cur), P<float>(ctx->xobs), P<double>(ctx->omf), p.gamma2, ctx->ypend, y,
                      P<float>(ctx->s), P<float>(ctx->u32), P<float>(ctx->w), od, B, C, H, W, (float)p.gamma1,
                      ctx->den_clamp, mb, st);
    else
      launch_k1(od.kind, xo, P<float>(ctx->y), P<float>(ctx->s), P<float>(ctx->u32),
                P<float>(ctx->w), od, B, C, H, W, (float)p.gamma1, ctx->den_clamp, mb, st);
    check_launch(ctx, "k1");
  }
  if (mb) {
    ProfScope ps(ctx, "l1_select", st);
    const double eta = p.alpha_s * (double)n * p.sp_nl * p.r * 0.5;   // operators.py:96
    l1_select(ctx, ctx->l1_scr, P<float>(ctx->w), P<float>(ctx->theta), B, n, eta, st);
    check_launch(ctx, "l1_select");
  }
  run_denoiser(ctx, P<float>(ctx->u32), xn, ctx->act, B, H, W, st);
  int mm_chunks = 0;
  {
    ProfScope ps(ctx, "k2_dual", st);
    const double gkl_gamma = p.my_lambda / p.gamma2;   // iteration.py:63
    mm_chunks = launch_k2(od.kind, ctx->method, xn, xo, y, P<float>(ctx->xobs),
                          ctx->has_true && !psnr_in_ssim ? P<float>(ctx->xtrue) : nullptr, P<float>(ctx->s), P<float>(ctx->w),
                          P<float>(ctx->theta), P<double>(ctx->partials), od, B, C, H, W, p.gamma2, gkl_gamma,
                          p.poisson_alpha, record, want_ssim(ctx) ? P<float>(ctx->ssim_mm) : nullptr, st);
    check_launch(ctx, "k2");
  }
  if (fused) {
    ProfScope ps(ctx, "k3_norm", st);
    launch_k3_norm(P<double>(ctx->partials), od, B, C, H, W, l2_eps(ctx, n), P<double>(ctx->omf),
                   P<double>(ctx->metrics), ctx->it, ctx->cap, record, ctx->has_true, st, ctx->itp);
    check_launch(ctx, "k3_norm");
    ctx->ypend = true;
  } else {
    ProfScope ps(ctx, "k3_dual", st);
    launch_k3(ctx->method, P<float>(ctx->y), P<float>(ctx->xobs), P<double>(ctx->partials), od, B, C, H, W, p.gamma2,
              l2_eps(ctx, n), P<double>(ctx->metrics), ctx->it, ctx->cap, record, ctx->has_true, st, ctx->itp);
    check_launch(ctx, "k3");
  }
  record_ssim(ctx, xn, st, mm_chunks, psnr_in_ssim);
  if (ctx->capturing) launch_it_advance(P<int>(ctx->it_dev), st);
  ctx->cur ^= 1;
  ctx->it += 1;
}

// comparisonB-2 (iteration.py:127-132): ADMM with the denoiser as the x-step prox.
//   x = 1; m1 x { x <- D(x - Phi^T(Phi x + s - z + y) / g1) }        (admm.py:30-36)
//   s = 1; m2 x { s <- P_l1(s - (Phi x + s - z + y) / g1) }          (admm.py:38-44, r = 1)
//   z = P_l2(Phi x + s + y; x_obs)  (r = 1);  y <- y + Phi x + s - z
void solver_iteration_admm(pnp_ctx* ctx) {
  hipStream_t st = ctx->stream;
  const pnp_params& p = ctx->prm;
  const int B = ctx->B, C = ctx->C, H = ctx->H, W = ctx->W;
  const size_t n = (size_t)C * H * W, N = (size_t)B * n;
  const OpDesc od = op_desc(ctx);
  float* xo = P<float>(ctx->x[ctx->cur]);
  float* xn = P<float>(ctx->x[ctx->cur ^ 1]);
  float *y = P<float>(ctx->y), *sv = P<float>(ctx->s), *z = P<float>(ctx->z), *w = P<float>(ctx->w);
  float *pp = P<float>(ctx->p), *t = P<float>(ctx->t);
  const double g = 1.0 / p.gamma1;
  {
    ProfScope ps(ctx, "admm_x_init", st);
    launch_lincomb(w, 0.0, sv, 1.0, y, 1.0, z, -1.0, nullptr, 0.0, N, st);     // s - z + y (fixed in the x-step)
    launch_lincomb(xn, 1.0, nullptr, 0.0, nullptr, 0.0, nullptr, 0.0, nullptr, 0.0, N, st);   // admm.py:32
    check_launch(ctx, "admm_x_init");
  }
  for (int i = 0; i < p.m1; ++i) {
    {
      ProfScope ps(ctx, "admm_x_grad", st);
      launch_op_phi(od.kind, 0, xn, t, od, B * C, H, W, st, w);               // Phi x + s - z + y
      launch_k1(od.kind, xn, t, nullptr, P<float>(ctx->u32), nullptr, od, B, C, H, W,
                (float)g, ctx->den_clamp, 0, st);                              // x - Phi^T(.) / g1 -> denoiser input
      check_launch(ctx, "admm_x_grad");
    }
    run_denoiser(ctx, P<float>(ctx->u32), xn, ctx->act, B, H, W, st);   // admm.py:35
  }
  {
    ProfScope ps(ctx, "admm_s_step", st);
    launch_op_phi(od.kind, 0, xn, pp, od, B * C, H, W, st);                   // Phi x (fixed from here on)
    launch_lincomb(sv, 1.0, nullptr, 0.0, nullptr, 0.0, nullptr, 0.0, nullptr, 0.0, N, st);   // admm.py:40
    const double eta = p.alpha_s * (double)n * p.sp_nl * 0.5;               // operators.py:96, r = 1
    for (int i = 0; i < p.m2; ++i) {
      launch_lincomb(w, 0.0, sv, 1.0 - g, pp, -g, y, -g, z, g, N, st);       // s - (Phi x + s - z + y) / g1
      l1_select(ctx, ctx->l1_scr, w, P<float>(ctx->theta), B, n, eta, st);
      launch_shrink(w, sv, P<float>(ctx->theta), B, n, st);
    }
    check_launch(ctx, "admm_s_step");
  }
  {
    ProfScope ps(ctx, "admm_zy", st);
    const double eps = std::sqrt((double)n * (1.0 - p.sp_nl)) * p.alpha_n * p.gaussian_nl;   // r = 1
    launch_lincomb(t, 0.0, pp, 1.0, sv, 1.0, y, 1.0, nullptr, 0.0, N, st);
    launch_l2_proj(t, P<float>(ctx->xobs), z, P<double>(ctx->partials), B, n, eps, st);
    launch_lincomb(y, 0.0, y, 1.0, pp, 1.0, sv, 1.0, z, -1.0, N, st);      // iteration.py:132
    if (p.record_metrics && ctx->it < ctx->cap)
      launch_metrics(xn, xo, ctx->has_true ? P<float>(ctx->xtrue) : nullptr, P<double>(ctx->partials),
                     P<double>(ctx->metrics), B, n, ctx->it, ctx->cap, st);
    check_launch(ctx, "admm_zy");
  }
  record_ssim(ctx, xn, st);
  ctx->cur ^= 1;
  ctx->it += 1;
}

bool is_tv(int m) { return m == PNP_METHOD_A_PDS_TV || m == PNP_METHOD_A_FBS_TV || m == PNP_METHOD_B_HTV; }
bool is_poisson_admm(int m) { return m == PNP_METHOD_C_PNPADMM || m == PNP_METHOD_C_RED; }

// The comparison methods of iteration.py:71-180 (BM3D excluded), composed from the PDS
// path's kernels plus methods.hip.  x_o = x_n of the reference on entry, x_n on exit.
void solver_iteration_cmp(pnp_ctx* ctx) {
  hipStream_t st = ctx->stream;
  const pnp_params& p = ctx->prm;
  const int B = ctx->B, C = ctx->C, H = ctx->H, W = ctx->W, m = ctx->method;
  const size_t n = (size_t)C * H * W, N = (size_t)B * n;
  const OpDesc od = op_desc(ctx);
  float* xo = P<float>(ctx->x[ctx->cur]);
  float* xn = P<float>(ctx->x[ctx->cur ^ 1]);
  float *y = P<float>(ctx->y), *sv = P<float>(ctx->s), *xobs = P<float>(ctx->xobs);
  float *t = P<float>(ctx->t), *pp = P<float>(ctx->p), *w = P<float>(ctx->w), *z = P<float>(ctx->z);
  const float* xt = ctx->has_true ? P<float>(ctx->xtrue) : nullptr;
  const int record = p.record_metrics && ctx->it < ctx->cap;
  auto phi = [&](const float* in, float* out, const float* add = nullptr) {
    launch_op_phi(od.kind, 0, in, out, od, B * C, H, W, st, add);
  };
  auto adj = [&](const float* in, float* out) { launch_op_phi(od.kind, 1, in, out, od, B * C, H, W, st); };
  auto lin = [&](float* out, double k, const float* a, double ca, const float* b = nullptr, double cb = 0.0,
                 const float* c = nullptr, double cc = 0.0, const float* d = nullptr, double cd = 0.0) {
    launch_lincomb(out, k, a, ca, b, cb, c, cc, d, cd, N, st);
  };
  auto denoise = [&](const float* in, float* out) {          // Denoiser_J.denoise / KAIR forward
    launch_pack_input(in, P<float>(ctx->u32), B, C, H, W, ctx->den_clamp, st);
    run_denoiser(ctx, P<float>(ctx->u32), out, ctx->act, B, H, W, st);
  };
  const double eta = p.alpha_s * (double)n * p.sp_nl * 0.5;                         // proj_l1_ball, r = 1
  const double eps = std::sqrt((double)n * (1.0 - p.sp_nl)) * p.alpha_n * p.gaussian_nl;  // proj_l2_ball, r = 1
  auto l1proj = [&](const float* in, float* out) {
    l1_select(ctx, ctx->l1_scr, in, P<float>(ctx->theta), B, n, eta, st);
    launch_shrink(in, out, P<float>(ctx->theta), B, n, st);
  };
  auto metrics = [&] {
    if (record)
      launch_metrics(xn, xo, xt, P<double>(ctx->partials), P<double>(ctx->metrics), B, n, ctx->it, ctx->cap, st);
  };
  // Phi x + s - x_obs  (grad_s_l2, operators.py:91-92), into out
  auto residual = [&](const float* x, const float* s, float* out) {
    phi(x, out, s);
    lin(out, 0.0, out, 1.0, xobs, -1.0);
  };
  ProfScope ps(ctx, "cmp_iteration", st);
  switch (m) {
    case PNP_METHOD_A_PNPFBS: {      // iteration.py:71-73
      residual(xo, nullptr, t);
      adj(t, pp);
      lin(pp, 0.0, xo, 1.0, pp, -(p.gamma1 * p.my_lambda * 0.5) * 2.0);
      denoise(pp, xn);
      metrics();
      break;
    }
    case PNP_METHOD_A_RED: {         // iteration.py:98-103
      denoise(xo, xn);
      residual(xo, nullptr, t);
      adj(t, pp);
      const double ig = 1.0 / (p.gamma1 * p.gamma1), mu = 2.0 / (ig + p.my_lambda);
      lin(xn, 0.0, xo, 1.0 - mu * p.my_lambda, pp, -mu * ig, xn, mu * p.my_lambda);
      metrics();
      break;
    }
    case PNP_METHOD_B_RED: {         // iteration.py:146-151
      denoise(xo, xn);
      residual(xo, sv, t);
      adj(t, pp);
      lin(xn, 0.0, xo, 1.0 - p.gamma1, pp, -p.gamma1 * p.my_lambda, xn, p.gamma1);
      residual(xn, sv, t);
      lin(w, 0.0, sv, 1.0, t, -p.gamma1);
      l1proj(w, sv);
      metrics();
      break;
    }
    case PNP_METHOD_B_PNPFBS: {      // iteration.py:152-155
      residual(xo, sv, t);
      adj(t, pp);
      lin(pp, 0.0, xo, 1.0, pp, -p.gamma1 * 2.0);
      denoise(pp, xn);
      residual(xn, sv, t);
      lin(w, 0.0, sv, 1.0, t, -p.gamma1);
      l1proj(w, sv);
      metrics();
      break;
    }
    case PNP_METHOD_A_PDS_TV:        // iteration.py:86-91
    case PNP_METHOD_B_HTV: {         // iteration.py:139-145
      float* y1 = P<float>(ctx->y1);
      adj(y, pp);
      launch_tv_primal(xo, y1, pp, p.gamma1, xn, B, C, H, W, st);
      const int mb = m == PNP_METHOD_B_HTV;
      if (mb) {
        lin(w, 0.0, sv, 1.0, y, -p.gamma1);
        l1_select(ctx, ctx->l1_scr, w, P<float>(ctx->theta), B, n, eta, st);
      }
      launch_tv_dual(xn, xo, y1, p.gamma2, B, C, H, W, st);
      launch_k2(od.kind, mb ? PNP_METHOD_B : PNP_METHOD_A, xn, xo, y, xobs, xt, sv, w, P<float>(ctx->theta),
                P<double>(ctx->partials), od, B, C, H, W, p.gamma2, 0.0, p.poisson_alpha, record, nullptr, st);
      launch_k3(mb ? PNP_METHOD_B : PNP_METHOD_A, y, xobs, P<double>(ctx->partials), od, B, C, H, W, p.gamma2, eps,
                P<double>(ctx->metrics), ctx->it, ctx->cap, record, ctx->has_true, st);
      break;
    }
    case PNP_METHOD_A_FBS_TV: {      // iteration.py:92-96
      residual(xo, nullptr, t);
      adj(t, pp);
      launch_tv_primal(xo, P<float>(ctx->y1), pp, p.gamma1, xn, B, C, H, W, st);
      launch_tv_dual(xn, xo, P<float>(ctx->y1), p.gamma2, B, C, H, W, st);
      metrics();
      break;
    }
    case PNP_METHOD_C_PNPADMM:       // iteration.py:163-166
    case PNP_METHOD_C_RED: {         // iteration.py:167-173
      float* d = P<float>(ctx->d);
      lin(xn, 1.0, nullptr, 0.0);                                       // admm.py:9 x_n = ones
      for (int i = 0; i < p.m1; ++i) {                                  // admm.py:10-12
        phi(xn, t);
        launch_poisson_ratio(xobs, t, p.poisson_alpha, t, N, st);
        adj(t, pp);
        launch_admm_poisson_step(xn, pp, P<float>(ctx->c1), z, d, p.gamma_in_admm_step1, p.poisson_alpha,
                                 p.my_lambda, N, st);
      }
      if (m == PNP_METHOD_C_PNPADMM) {
        lin(pp, 0.0, xn, 1.0, d, 1.0);
        denoise(pp, z);                                                 // z = D(x + d)
      } else {                                                          // admm.py:18-27
        const double beta = p.my_lambda, lam2 = p.gamma1;
        lin(pp, 0.0, xn, 1.0, d, 1.0);                                  // z_str
        for (int i = 0; i < p.m2; ++i) {
          denoise(z, z);
          lin(z, 0.0, z, (1.0 / (beta + lam2)) * lam2, pp, (1.0 / (beta + lam2)) * beta);
        }
      }
      lin(d, 0.0, d, 1.0, xn, 1.0, z, -1.0);                            // d = d + x - z
      metrics();
      break;
    }
    default:
      fail(ctx, PNP_E_UNSUPPORTED, "method %d", m);
  }
  check_launch(ctx, "cmp_iteration");
  record_ssim(ctx, xn, st);
  ctx->cur ^= 1;
  ctx->it += 1;
}

void solver_step(pnp_ctx* ctx) {
  if (ctx->method == PNP_METHOD_ADMM_B2) solver_iteration_admm(ctx);
  else if (ctx->method <= PNP_METHOD_C) solver_iteration(ctx);
  else solver_iteration_cmp(ctx);
}

// ---- graph replay ----------------------------------------------------------------------
// Two iterations (x ping-pong back to the same buffer) are captured once into a hipGraph and
// replayed; the metric kernels then take the iteration number (their metrics row) from a
// device counter the graph advances.  The kernels and their arguments are those of the plain
// path, so the results are the same bits.  Any setter or (re)allocation bumps ctx->gen and
// the next run recaptures.  Off by default: measured at B = 1 (cfg1 / cfg2, 0.22-0.25 ms per
// iteration) the GPU work outlasts the host's launches, so replays gain nothing there; it is
// for hosts that are slower or busy (small batches).
bool graph_enabled(pnp_ctx* ctx) {
  if (ctx->prof || ctx->graph_mode != 1) return false;
  return ctx->method == PNP_METHOD_A || ctx->method == PNP_METHOD_B || ctx->method == PNP_METHOD_C;
}

void graph_release(pnp_ctx* ctx) {
  if (ctx->gexec) (void)hipGraphExecDestroy(ctx->gexec);
  ctx->gexec = nullptr;
  ctx->gexec_gen = -1;
}

void graph_build(pnp_ctx* ctx) {
  graph_release(ctx);
  ensure(ctx, ctx->it_dev, sizeof(int));
  const int it0 = ctx->it, cur0 = ctx->cur;
  hipGraph_t g = nullptr;
  HIPCHK(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
  ctx->capturing = true;
  ctx->itp = P<int>(ctx->it_dev);
  try {
    solver_step(ctx);
    solver_step(ctx);
  } catch (...) {
    ctx->capturing = false;
    ctx->itp = nullptr;
    (void)hipStreamEndCapture(ctx->stream, &g);
    if (g) (void)hipGraphDestroy(g);
    ctx->it = it0;
    ctx->cur = cur0;
    throw;
  }
  ctx->capturing = false;
  ctx->itp = nullptr;
  ctx->it = it0;
  ctx->cur = cur0;
  HIPCHK(ctx, hipStreamEndCapture(ctx->stream, &g));
  const hipError_t e = hipGraphInstantiate(&ctx->gexec, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    ctx->gexec = nullptr;
    fail(ctx, PNP_E_HIP, "hipGraphInstantiate: %s", hipGetErrorString(e));
  }
  ctx->gexec_gen = ctx->gen;
}

// n iterations: plain steps until the state is warm (no allocation pending) and x sits in
// buffer 0, then graph replays of two iterations, then a plain step for an odd remainder.
// PNP_PREC_AUTO: a reduced precision only where the reference's long
// trajectories (tests/test_gpu_long.py, at the experiments' own lengths) keep every
// iteration's PSNR within half the 0.01 dB bound.
//  * Blur operator, ours-A / ours-B / comparisonB-2 / PnP-FBS / RED (the operator's low-pass
//    damps the network's rounding), sigma <= 0.01: fp16 operands (largest max |dPSNR| 0.0035
//    dB, comparisonB-2 over 200 outer iterations).
//  * Above sigma 0.01 the fp16 drift keeps growing through the run (sigma 0.02: ours-A 0.0055,
//    ours-B 0.0055 dB; sigma 0.04: ours-A 0.0068, ours-B / PnP-FBS / RED 0.031-0.050).  ours-A
//    and comparisonB-2 then run fp16 activations with split hi + lo weights (fp16w2, two MFMAs
//    per product: <= 0.0005 dB at sigma 0.02 / 0.04); ours-B, PnP-FBS and RED split fp16
//    (their fp16w2 trajectories reach 0.011 / 0.0039 / 0.0023 dB at sigma 0.04).
//  * Everything else: split fp16 (fp16x3, three MFMAs per product, near-fp32): the Id and
//    random-sampling operators, whose restorations reach 42-50 dB (fp16: gray Id 256^2 0.037 dB
//    over 1200, ours-A random sampling 0.051 / 0.113 dB over 3000; fp16w2 0.011 / 0.0135), the
//    Poisson methods (ours-C: fp16 0.19 dB, fp16w2 0.10 over 3000) and the TV / sparse
//    comparison methods (no long-trajectory evidence for less).
constexpr double kAutoFp16MaxSigma = 0.01;
int auto_precision(int method, int op_kind, double sigma) {
  if (op_kind != PNP_OP_BLUR) return PNP_PREC_FP16X3;
  const bool w2_ok = method == PNP_METHOD_A || method == PNP_METHOD_ADMM_B2;
  const bool fp16_ok = w2_ok || method == PNP_METHOD_B || method == PNP_METHOD_A_PNPFBS || method == PNP_METHOD_A_RED;
  if (fp16_ok && sigma <= kAutoFp16MaxSigma * (1.0 + 1e-9)) return PNP_PREC_FP16;
  return w2_ok ? PNP_PREC_FP16W2 : PNP_PREC_FP16X3;
}

// PNP_PREC_CONVERGE after its hand-over: split activations.  Where auto runs fp16 activations
// (the blur family, fp16 / fp16w2) fp16a2 (single fp16 weights, two MFMAs per product: r05
// probe, every such golden within 0.0007 dB and its c_n within 1 % of the reference's down to
// 1e-6); elsewhere auto already runs fp16x3 and the solve switches at once.
int converge_precision(int fast) {
  return (fast == PNP_PREC_FP16 || fast == PNP_PREC_FP16W2) ? PNP_PREC_FP16A2 : PNP_PREC_FP16X3;
}

int effective_precision(const pnp_ctx* ctx) {
  if (ctx->prec_req == PNP_PREC_CONVERGE && ctx->conv_switched)
    return converge_precision(ctx->method >= 0 ? auto_precision(ctx->method, ctx->op_kind, ctx->prm.gaussian_nl)
                                               : PNP_PREC_FP16X3);
  if (ctx->prec_req != PNP_PREC_AUTO && ctx->prec_req != PNP_PREC_CONVERGE) return ctx->prec_req;
  return ctx->method >= 0 ? auto_precision(ctx->method, ctx->op_kind, ctx->prm.gaussian_nl) : PNP_PREC_FP16X3;
}

// ---- PNP_PREC_CONVERGE: a precision hand-over at a c_n threshold --------------------------
// With fp16 activations the iteration settles on the fp16-rounded map's fixed point: c_n
// (iteration.py:187) stalls near 3e-4 where the reference's keeps contracting.
// CONVERGE runs auto's operands while c_n is far above that floor, then split activations
// (fp16a2 or fp16x3, converge_precision: c_n follows the reference's down to ~1e-7) for the rest
// of the solve.  The switch is per image: image b runs split activations from iteration i + 2
// on once its c_n at iteration i is below conv_c (the host reads iteration i's c_n row while
// iteration i + 1 runs: a fixed lag of one, so the decision does not depend on timing), and
// while only some images have switched each denoiser pass is split into runs of one precision
// (run_denoiser).  An image's iterates therefore depend only on its own c_n, whatever batch or
// shard it is solved in.  Without recorded metrics (record_metrics 0, or the metrics capacity
// reached) there is no c_n to watch, and the images not yet switched switch at once.
// pnp_get_precision_switches reports each image's switch iteration, pnp_get_precision_switch
// the iteration from which the whole batch runs split.
void converge_reset(pnp_ctx* ctx) {
  ctx->conv_switched = false;
  ctx->conv_switch_it = -1;
  ctx->conv_slot_it[0] = ctx->conv_slot_it[1] = -1;
  ctx->conv_img_it.assign(std::max(ctx->B, 0), -1);
  ctx->conv_nsw = 0;
}

void converge_switch_image(pnp_ctx* ctx, int b) {
  if (ctx->conv_img_it[b] >= 0) return;
  ctx->conv_img_it[b] = ctx->it;
  if (++ctx->conv_nsw == ctx->B) {
    ctx->conv_switched = true;
    ctx->conv_switch_it = ctx->it;
  }
}

void converge_switch(pnp_ctx* ctx) {
  if ((int)ctx->conv_img_it.size() != ctx->B) converge_reset(ctx);
  for (int b = 0; b < ctx->B; ++b) converge_switch_image(ctx, b);
  ctx->conv_switched = true;
  if (ctx->conv_switch_it < 0) ctx->conv_switch_it = ctx->it;
}

// true when every image has switched (before iteration ctx->it)
bool converge_check(pnp_ctx* ctx) {
  if (ctx->conv_switched) return true;
  if ((int)ctx->conv_img_it.size() != ctx->B) converge_reset(ctx);
  const int i = ctx->it;
  if (auto_precision(ctx->method, ctx->op_kind, ctx->prm.gaussian_nl) == PNP_PREC_FP16X3 ||
      !ctx->prm.record_metrics || i >= ctx->cap) {
    converge_switch(ctx);
    return true;
  }
  const int k = i & 1;                        // slot of iteration i - 2
  if (i >= 2 && ctx->conv_slot_it[k] == i - 2) {
    HIPCHK(ctx, hipEventSynchronize(ctx->conv_ev[k]));
    const int before = ctx->conv_nsw;
    for (int b = 0; b < ctx->B; ++b)          // NaN compares false: never triggers a switch
      if (ctx->conv_img_it[b] < 0 && ctx->conv_row[(size_t)k * ctx->B + b] < ctx->conv_c) converge_switch_image(ctx, b);
    if (ctx->conv_nsw != before) ctx->gen++;  // the passes' split changed (no graph runs before the end anyway)
  }
  return ctx->conv_switched;
}

// after a watched iteration i (ctx->it == i + 1 now): queue the copy of its c_n row
void converge_watch(pnp_ctx* ctx) {
  const int i = ctx->it - 1, k = i & 1, B = ctx->B;
  if (!ctx->conv_row || ctx->conv_row_B < B) {
    if (ctx->conv_row) {
      HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
      (void)hipHostFree(ctx->conv_row);
      ctx->conv_row = nullptr;
    }
    HIPCHK(ctx, hipHostMalloc((void**)&ctx->conv_row, 2 * (size_t)B * sizeof(double), hipHostMallocDefault));
    ctx->conv_row_B = B;
    ctx->conv_slot_it[0] = ctx->conv_slot_it[1] = -1;
  }
  for (int e = 0; e < 2; ++e)
    if (!ctx->conv_ev[e]) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->conv_ev[e], hipEventDisableTiming));
  const size_t pitch = (size_t)ctx->cap * kMetrics * sizeof(double);   // metrics[b][it][kMetrics]
  HIPCHK(ctx, hipMemcpy2DAsync(ctx->conv_row + (size_t)k * B, sizeof(double),
                               P<double>(ctx->metrics) + (size_t)i * kMetrics, pitch, sizeof(double), B,
                               hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipEventRecord(ctx->conv_ev[k], ctx->stream));
  ctx->conv_slot_it[k] = i;
}

void solver_run(pnp_ctx* ctx, int n) {
  if (ctx->prec_req == PNP_PREC_CONVERGE) {   // watched steps until the hand-over (plain launches)
    while (n > 0 && !converge_check(ctx)) {
      const int eff = effective_precision(ctx);
      if (ctx->prec != eff) {
        ctx->prec = eff;
        ctx->gen++;
      }
      solver_step(ctx);
      ctx->warm_gen = ctx->gen;
      converge_watch(ctx);
      --n;
    }
  }
  const int eff = effective_precision(ctx);
  if (ctx->prec != eff) {                      // a captured graph holds the other precision's kernels
    ctx->prec = eff;
    ctx->gen++;
  }
  auto plain = [&] {
    solver_step(ctx);
    ctx->warm_gen = ctx->gen;
  };
  if (!graph_enabled(ctx)) {
    for (int i = 0; i < n; ++i) plain();
    return;
  }
  while (n > 0 && (ctx->cur != 0 || ctx->warm_gen != ctx->gen)) {
    plain();
    --n;
  }
  if (n >= 2) {
    if (!ctx->gexec || ctx->gexec_gen != ctx->gen) graph_build(ctx);
    HIPCHK(ctx, hipMemsetD32Async((hipDeviceptr_t)ctx->it_dev.p, ctx->it, 1, ctx->stream));
    for (int k = 0; k < n / 2; ++k) HIPCHK(ctx, hipGraphLaunch(ctx->gexec, ctx->stream));
    ctx->it += 2 * (n / 2);
    n &= 1;
  }
  if (n) plain();
}

void solver_setup(pnp_ctx* ctx, int method, const pnp_params* params, int B, int C, int H, int W, int cap) {
  ctx->gen++;
  if (!params) fail(ctx, PNP_E_ARG, "params is NULL");
  if (method < PNP_METHOD_A || method > PNP_METHOD_C_RED)
    fail(ctx, PNP_E_UNSUPPORTED, "method %d not supported on device", method);
  if (method == PNP_METHOD_ADMM_B2 && (params->m1 < 0 || params->m2 < 0 || params->gamma1 == 0.0))
    fail(ctx, PNP_E_ARG, "comparisonB-2 needs m1, m2 >= 0 and gamma1 != 0");
  if (is_poisson_admm(method) && (params->m1 < 0 || params->m2 < 0 || params->poisson_alpha == 0.0))
    fail(ctx, PNP_E_ARG, "Poisson ADMM needs m1, m2 >= 0 and poisson_alpha != 0");
  if (is_tv(method) && (H < 3 || W < 3 || C > kMaxC))
    fail(ctx, PNP_E_ARG, "TV methods need H, W >= 3 (operators.py:128-137)");
  if (B < 1 || C < 1 || C > kMaxC || H < 1 || W < 1) fail(ctx, PNP_E_ARG, "bad shape B=%d C=%d H=%d W=%d", B, C, H, W);
  if (!is_tv(method)) {   // the TV methods use no denoiser
    if (!ctx->den_ready) fail(ctx, PNP_E_STATE, "denoiser not set");
    if (ctx->den_C != C) fail(ctx, PNP_E_ARG, "denoiser has %d channels, images have %d", ctx->den_C, C);
  }
  check_operator_shape(ctx, H, W);
  if (ctx->op_kind == PNP_OP_BLUR && (ctx->op_R > H || ctx->op_R > W))
    fail(ctx, PNP_E_ARG, "blur kernel radius %d larger than the image", ctx->op_R);
  if (params->gamma2 == 0.0) fail(ctx, PNP_E_ARG, "gamma2 must be non-zero");
  if ((size_t)C * H * W >= kMaxL1Elems && (method == PNP_METHOD_B || method == PNP_METHOD_ADMM_B2 ||
                                            method == PNP_METHOD_B_HTV || method == PNP_METHOD_B_RED ||
                                            method == PNP_METHOD_B_PNPFBS))
    fail(ctx, PNP_E_UNSUPPORTED, "l1-ball methods need C*H*W < 2^29 per image");
  ctx->method = method;
  ctx->prm = *params;
  ctx->B = B; ctx->C = C; ctx->H = H; ctx->W = W;
  ctx->cap = std::max(cap, 0);
  const size_t N = (size_t)B * C * H * W, fb = N * sizeof(float);
  for (int i = 0; i < 2; ++i) ensure(ctx, ctx->x[i], fb);
  ensure(ctx, ctx->y, fb);
  if (method == PNP_METHOD_A || method == PNP_METHOD_B) {
    ensure(ctx, ctx->y2, fb);
    ensure(ctx, ctx->omf, (size_t)B * sizeof(double));
  }
  ctx->ypend = false;
  ensure(ctx, ctx->s, fb);
  ensure(ctx, ctx->xobs, fb);
  ensure(ctx, ctx->xtrue, fb);
  ensure(ctx, ctx->u32, fb);
  if (method != PNP_METHOD_A && method != PNP_METHOD_C) ensure(ctx, ctx->w, fb);
  if (method >= PNP_METHOD_ADMM_B2) {
    ensure(ctx, ctx->z, fb);
    ensure(ctx, ctx->p, fb);
    ensure(ctx, ctx->t, fb);
  }
  if (is_tv(method)) ensure(ctx, ctx->y1, 2 * fb);
  if (is_poisson_admm(method)) {
    ensure(ctx, ctx->d, fb);
    ensure(ctx, ctx->c1, fb);
  }
  ensure(ctx, ctx->partials,
         (size_t)B * std::max(partial_tiles(H, W) * C, chunk_count((size_t)C * H * W)) * 4 * sizeof(double));
  ensure(ctx, ctx->metrics, (size_t)B * std::max(ctx->cap, 1) * kMetrics * sizeof(double));
  if (params->record_ssim) {
    ensure(ctx, ctx->ssim_scr, ssim_scratch_bytes(B, C, H, W));
    ensure(ctx, ctx->ssim_mm, (size_t)B * k2_minmax_chunks(C, H, W) * 2 * sizeof(float));
  }
  ensure(ctx, ctx->theta, (size_t)B * sizeof(float));
  ctx->loaded = false;
  ctx->it = 0;
  converge_reset(ctx);
}

void solver_reset_state(pnp_ctx* ctx) {
  ctx->gen++;
  check_operator_shape(ctx, ctx->H, ctx->W);
  if (ctx->op_kind == PNP_OP_BLUR && (ctx->op_R > ctx->H || ctx->op_R > ctx->W))
    fail(ctx, PNP_E_ARG, "blur kernel radius %d larger than the image", ctx->op_R);
  const size_t fb = (size_t)ctx->B * ctx->C * ctx->H * ctx->W * sizeof(float);
  HIPCHK(ctx, hipMemsetAsync(ctx->y.p, 0, fb, ctx->stream));          // iteration.py:24
  ctx->ypend = false;
  HIPCHK(ctx, hipMemsetAsync(ctx->s.p, 0, fb, ctx->stream));          // iteration.py:27
  if (ctx->method >= PNP_METHOD_ADMM_B2) HIPCHK(ctx, hipMemsetAsync(ctx->z.p, 0, fb, ctx->stream));
  if (is_tv(ctx->method)) HIPCHK(ctx, hipMemsetAsync(ctx->y1.p, 0, 2 * fb, ctx->stream));   // iteration.py:25
  if (is_poisson_admm(ctx->method)) {
    HIPCHK(ctx, hipMemsetAsync(ctx->d.p, 0, fb, ctx->stream));                            // iteration.py:29
    const OpDesc od = op_desc(ctx);                                                     // c1 = Phi^T 1 (admm.py:11)
    launch_lincomb(P<float>(ctx->t), 1.0, nullptr, 0.0, nullptr, 0.0, nullptr, 0.0, nullptr, 0.0, fb / 4,
                   ctx->stream);
    launch_op_phi(od.kind, 1, P<float>(ctx->t), P<float>(ctx->c1), od, ctx->B * ctx->C, ctx->H, ctx->W, ctx->stream);
  }
  if (ctx->cap) {
    std::vector<double> nanbuf((size_t)ctx->B * ctx->cap * kMetrics, std::nan(""));
    HIPCHK(ctx, hipMemcpyAsync(ctx->metrics.p, nanbuf.data(), nanbuf.size() * sizeof(double), hipMemcpyHostToDevice,
                               ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  }
  ctx->cur = 0;
  ctx->it = 0;
  ctx->loaded = true;
  converge_reset(ctx);
}

// A persistent denoiser whose neighbour wait hit its spin bound: the results are wrong, so the
// fetch (or pnp_op_status for the single ops) fails loudly instead of returning them.  The
// stacks are plain launches (common.h persistent_launch), not cooperative ones: co-residency
// rests on one persistent grid per context at a time (use_stack), so a timeout is a fault or
// contention with another process's grid on the same device.  The caller has synchronized
// ctx->stream, the only stream the persistent launches run on; the word is read and cleared
// on that stream.
void check_stack_err(pnp_ctx* ctx, DevBuf& ew) {
  if (!ew.p) return;
  int e = 0;
  HIPCHK(ctx, hipMemcpyAsync(&e, ew.p, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  if (e) {
    HIPCHK(ctx, hipMemsetAsync(ew.p, 0, sizeof(int), ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    fail(ctx, PNP_E_INTERNAL, "persistent denoiser: a tile's neighbour wait timed out (results invalid)");
  }
}

void solver_fetch(pnp_ctx* ctx, float* x_out, float* s_out, double* c_out, double* psnr_out, double* ssim_out) {
  if (!ctx->loaded) fail(ctx, PNP_E_STATE, "solver not loaded");
  const size_t N = (size_t)ctx->B * ctx->C * ctx->H * ctx->W;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  check_stack_err(ctx, ctx->stack_err);
  if (x_out) HIPCHK(ctx, hipMemcpy(x_out, ctx->x[ctx->cur].p, N * sizeof(float), hipMemcpyDeviceToHost));
  if (s_out) {
    HIPCHK(ctx, hipMemcpy(s_out, ctx->s.p, N * sizeof(float), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < N; ++i) s_out[i] += 0.5f;                // iteration.py:196
  }
  if ((c_out || psnr_out || ssim_out) && ctx->cap) {
    std::vector<double> m((size_t)ctx->B * ctx->cap * kMetrics);
    HIPCHK(ctx, hipMemcpy(m.data(), ctx->metrics.p, m.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < (size_t)ctx->B * ctx->cap; ++i) {
      if (c_out) c_out[i] = m[kMetrics * i];
      if (psnr_out) psnr_out[i] = m[kMetrics * i + 1];
      if (ssim_out) ssim_out[i] = m[kMetrics * i + 2];
    }
  }
}

}  // namespace

// =====================================================================================
// extern "C"
// =====================================================================================
extern "C" {

int pnp_abi_version(void) { return PNP_ABI_VERSION; }

#ifndef PNP_SRC_HASH
#define PNP_SRC_HASH "unknown"
#endif
const char* pnp_build_id(void) { return PNP_SRC_HASH; }

int pnp_device_count(int* count) {
  return guarded(nullptr, [&] {
    if (!count) fail(nullptr, PNP_E_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) fail(nullptr, PNP_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    *count = n;
  });
}

int pnp_create(int device, pnp_ctx** out) {
  return guarded(nullptr, [&] {
    if (!out) fail(nullptr, PNP_E_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
      fail(nullptr, PNP_E_HIP, "no HIP device available (%s)", hipGetErrorString(e));
    if (device < 0 || device >= n) fail(nullptr, PNP_E_ARG, "device %d out of range (%d devices)", device, n);
    auto* ctx = new pnp_ctx();
    ctx->device = device;
    try {
      HIPCHK(ctx, hipSetDevice(device));
      hipDeviceProp_t prop;
      HIPCHK(ctx, hipGetDeviceProperties(&prop, device));
      if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        fail(ctx, PNP_E_UNSUPPORTED, "device %d is %s; this library is built for gfx950 only", device,
             prop.gcnArchName);
      ctx->num_cus = prop.multiProcessorCount;
      ctx->act_budget = (double)prop.totalGlobalMem / 8;
      HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
      HIPCHK(ctx, conv_kernels_init());
      HIPCHK(ctx, conv32_kernels_init());
      HIPCHK(ctx, conv_s3_kernels_init());
    } catch (const PnpError&) {
      g_thread_err = ctx->err;
      delete ctx;
      throw;
    }
    *out = ctx;
  });
}

int pnp_destroy(pnp_ctx* ctx) {
  if (!ctx) return PNP_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  graph_release(ctx);
  for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->conv_ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->conv_row) (void)hipHostFree(ctx->conv_row);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;   // every DevBuf member frees its allocation (device ctx->device is current)
  return PNP_OK;
}

const char* pnp_last_error(const pnp_ctx* ctx) { return ctx ? ctx->err.c_str() : g_thread_err.c_str(); }

int pnp_synchronize(pnp_ctx* ctx) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] { HIPCHK(ctx, hipStreamSynchronize(ctx->stream)); });
}

int pnp_set_tuning(pnp_ctx* ctx, int key, int value) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    ctx->gen++;
    if (key == PNP_TUNE_GRAPH) {
      if (value < 0 || value > 1) fail(ctx, PNP_E_ARG, "graph mode must be 0 (off) or 1 (on)");
      ctx->graph_mode = value;
      return;
    }
    if (key == PNP_TUNE_DENOISE_CHUNK) {
      if (value < 0) fail(ctx, PNP_E_ARG, "chunk must be >= 0");
      ctx->den_chunk = value;
      return;
    }
    if (key == PNP_TUNE_CONVERGE_C) {
      if (value < 1) fail(ctx, PNP_E_ARG, "the c_n threshold (units of 1e-6) must be >= 1");
      ctx->conv_c = value * 1e-6;
      return;
    }
    if (key == PNP_TUNE_FUSE_ENDS) {
      if (value < 0 || value > 1) fail(ctx, PNP_E_ARG, "fuse-ends must be 0 (off) or 1 (on)");
      ctx->fuse_ends = value;
      return;
    }
    if (key == PNP_TUNE_BODY_LAYERS) {
      if (value < 0 || value > 4)
        fail(ctx, PNP_E_ARG, "body layers per launch must be 0 (auto), 1, 2, 3 (all) or 4 (all, one per hand-off)");
      ctx->body_layers = value;
      return;
    }
#ifdef PNP_PROFILING
    if (key == kTuneAblate) {              // profiling build only
      ctx->ablate = value;
      return;
    }
    if (key == kTuneAblateK2) {            // profiling build only (a process-wide setting)
      set_k2_ablate(value);
      return;
    }
#endif
    fail(ctx, PNP_E_UNSUPPORTED, "tuning key %d", key);
  });
}

int pnp_set_precision(pnp_ctx* ctx, int precision) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (precision != PNP_PREC_FP16 && precision != PNP_PREC_FP32 && precision != PNP_PREC_FP16W2 &&
        precision != PNP_PREC_FP16X3 && precision != PNP_PREC_AUTO && precision != PNP_PREC_CONVERGE &&
        precision != PNP_PREC_FP16A2)
      fail(ctx, PNP_E_UNSUPPORTED, "precision %d not supported", precision);
    ctx->prec_req = precision;   // resolved (and the graph invalidated if it changes) when the solver runs
  });
}

int pnp_get_precision(pnp_ctx* ctx, int* requested, int* effective) {
  if (!ctx) return PNP_E_ARG;
  if (requested) *requested = ctx->prec_req;
  if (effective) *effective = effective_precision(ctx);
  return PNP_OK;
}

int pnp_get_precision_switch(pnp_ctx* ctx, int* iteration) {
  if (!ctx || !iteration) return PNP_E_ARG;
  *iteration = ctx->conv_switch_it;
  return PNP_OK;
}

int pnp_get_precision_switches(pnp_ctx* ctx, int* iterations, int n) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!iterations || n < ctx->B)
      fail(ctx, PNP_E_ARG, "need room for %d switch iterations (one per image), got %d", ctx->B, n);
    for (int b = 0; b < ctx->B; ++b)
      iterations[b] = b < (int)ctx->conv_img_it.size() ? ctx->conv_img_it[b] : -1;
  });
}

int pnp_set_denoiser(pnp_ctx* ctx, int channels, int depth, int width, const float* params, size_t n_params,
                     int activation, int residual_sign, int clamp_io) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    ctx->gen++;
    if (width != kWidth) fail(ctx, PNP_E_UNSUPPORTED, "width %d unsupported (only 64)", width);
    if (channels < 1 || channels > kMaxC) fail(ctx, PNP_E_UNSUPPORTED, "channels %d unsupported (1..4)", channels);
    if (depth < 3) fail(ctx, PNP_E_UNSUPPORTED, "depth %d < 3", depth);
    if (activation != PNP_ACT_LEAKY_RELU && activation != PNP_ACT_RELU) fail(ctx, PNP_E_ARG, "bad activation");
    if (residual_sign != 1 && residual_sign != -1) fail(ctx, PNP_E_ARG, "residual_sign must be +1 or -1");
    const size_t n_head = (size_t)kWidth * channels * 9 + kWidth;
    const size_t n_body = (size_t)kWidth * kWidth * 9 + kWidth;
    const size_t n_tail = (size_t)channels * kWidth * 9 + channels;
    const size_t expect = n_head + (size_t)(depth - 2) * n_body + n_tail;
    if (!params || n_params != expect)
      fail(ctx, PNP_E_ARG, "expected %zu parameters for C=%d depth=%d, got %zu", expect, channels, depth, n_params);
    // rp: the parameters with every conv weight replaced by its fp16 value (fp16_filter_round):
    // the fp16 operand paths' weights and the high halves of the split ones
    std::vector<float> rp(params, params + n_params);
    {
      size_t off = 0;
      auto round_layer = [&](size_t nw, size_t nb) {
        fp16_filter_round(params + off, nw / 9, rp.data() + off);
        off += nw + nb;
      };
      round_layer((size_t)kWidth * channels * 9, kWidth);
      for (int l = 0; l < depth - 2; ++l) round_layer((size_t)kWidth * kWidth * 9, kWidth);
      round_layer((size_t)channels * kWidth * 9, channels);
    }
    const float* p = rp.data();
    std::vector<uint16_t> hw(kHeadWBytes / 2), bw((size_t)(depth - 2) * kBodyWBytes / 2), tw(kTailWBytes / 2);
    std::vector<float> hb(kWidth), bb((size_t)(depth - 2) * kWidth), tb(kMaxC, 0.f);
    pack_head_weights(p, channels, hw.data());
    std::memcpy(hb.data(), p + kWidth * channels * 9, kWidth * sizeof(float));
    p += n_head;
    std::vector<uint16_t> bw16(bw.size());
    for (int l = 0; l < depth - 2; ++l) {
      pack_body_weights(p, bw.data() + (size_t)l * kBodyWBytes / 2);
      pack_body_weights16(p, bw16.data() + (size_t)l * kBodyWBytes / 2);
      std::memcpy(bb.data() + (size_t)l * kWidth, p + kWidth * kWidth * 9, kWidth * sizeof(float));
      p += n_body;
    }
    pack_tail_weights(p, channels, tw.data());
    {                                        // low halves W - hi for PNP_PREC_FP16W2 / FP16X3, packed like W
      auto lo_of = [&](const float* w, size_t n) {   // hi: the same weights in rp (the fp16 values)
        const float* hi = rp.data() + (w - params);
        std::vector<float> lo(n);
        for (size_t i = 0; i < n; ++i) lo[i] = w[i] - hi[i];
        return lo;
      };
      std::vector<uint16_t> hl(hw.size()), bl(bw.size()), tl(tw.size());
      const float* q = params;
      pack_head_weights(lo_of(q, (size_t)kWidth * channels * 9).data(), channels, hl.data());
      q += n_head;
      for (int l = 0; l < depth - 2; ++l, q += n_body)
        pack_body_weights(lo_of(q, (size_t)kWidth * kWidth * 9).data(), bl.data() + (size_t)l * kBodyWBytes / 2);
      pack_tail_weights(lo_of(q, (size_t)channels * kWidth * 9).data(), channels, tl.data());
      std::vector<uint16_t> sh(bw.size()), sl(bw.size());   // conv_s3 body fragments (PNP_PREC_FP16X3)
      std::vector<uint16_t> sf(bw.size()), sz(bw.size());   // ... of the fp16 weights (FP16A2; lo = 0)
      q = params + n_head;
      for (int l = 0; l < depth - 2; ++l, q += n_body) {
        // fp16x3 at kS3BodyScale x the weights (the low halves stay normal fp16)
        pack_body_weights_s3(q, sh.data() + (size_t)l * kBodyWBytes / 2, sl.data() + (size_t)l * kBodyWBytes / 2,
                             kS3BodyScale);
        pack_body_weights_s3(rp.data() + (q - params), sf.data() + (size_t)l * kBodyWBytes / 2,
                             sz.data() + (size_t)l * kBodyWBytes / 2, 1.f);
      }
      ensure(ctx, ctx->body_s3f, sf.size() * 2);
      HIPCHK(ctx, hipMemcpy(ctx->body_s3f.p, sf.data(), sf.size() * 2, hipMemcpyHostToDevice));
      ensure(ctx, ctx->body_s3h, sh.size() * 2);
      ensure(ctx, ctx->body_s3l, sl.size() * 2);
      HIPCHK(ctx, hipMemcpy(ctx->body_s3h.p, sh.data(), sh.size() * 2, hipMemcpyHostToDevice));
      HIPCHK(ctx, hipMemcpy(ctx->body_s3l.p, sl.data(), sl.size() * 2, hipMemcpyHostToDevice));
      {                                      // the split (FP16X3 / A2) head and tail at kSplitWScale
        auto scaled = [&](const float* w, size_t n, bool lo_half) {
          const float* hi = rp.data() + (w - params);
          std::vector<float> v(n);
          for (size_t i = 0; i < n; ++i) v[i] = (lo_half ? w[i] - hi[i] : hi[i]) * kSplitWScale;
          return v;
        };
        std::vector<uint16_t> hx(hw.size()), hlx(hw.size()), tx(tw.size()), tlx(tw.size());
        const size_t nh = (size_t)kWidth * channels * 9, nt = (size_t)channels * kWidth * 9;
        const float* tail_p = params + n_head + (size_t)(depth - 2) * n_body;
        pack_head_weights(scaled(params, nh, false).data(), channels, hx.data());
        pack_head_weights(scaled(params, nh, true).data(), channels, hlx.data());
        pack_tail_weights(scaled(tail_p, nt, false).data(), channels, tx.data());
        pack_tail_weights(scaled(tail_p, nt, true).data(), channels, tlx.data());
        ensure(ctx, ctx->head_wx3, hx.size() * 2);
        ensure(ctx, ctx->head_wlox3, hlx.size() * 2);
        ensure(ctx, ctx->tail_wx3, tx.size() * 2);
        ensure(ctx, ctx->tail_wlox3, tlx.size() * 2);
        HIPCHK(ctx, hipMemcpy(ctx->head_wx3.p, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(ctx->head_wlox3.p, hlx.data(), hlx.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(ctx->tail_wx3.p, tx.data(), tx.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(ctx->tail_wlox3.p, tlx.data(), tlx.size() * 2, hipMemcpyHostToDevice));
      }
      ensure(ctx, ctx->head_wlo, hl.size() * 2);
      ensure(ctx, ctx->body_wlo, bl.size() * 2);
      ensure(ctx, ctx->tail_wlo, tl.size() * 2);
      HIPCHK(ctx, hipMemcpy(ctx->head_wlo.p, hl.data(), hl.size() * 2, hipMemcpyHostToDevice));
      HIPCHK(ctx, hipMemcpy(ctx->body_wlo.p, bl.data(), bl.size() * 2, hipMemcpyHostToDevice));
      HIPCHK(ctx, hipMemcpy(ctx->tail_wlo.p, tl.data(), tl.size() * 2, hipMemcpyHostToDevice));
    }
    {                                        // fp32 fragments for PNP_PREC_FP32
      std::vector<float> h32(conv32_weight_floats(0)), b32(conv32_weight_floats(1) * (depth - 2)),
          t32(conv32_weight_floats(2));
      const float* q = params;
      pack_conv32_weights(q, 0, channels, kWidth, h32.data());
      q += n_head;
      for (int l = 0; l < depth - 2; ++l, q += n_body)
        pack_conv32_weights(q, 1, kWidth, kWidth, b32.data() + (size_t)l * conv32_weight_floats(1));
      pack_conv32_weights(q, 2, kWidth, channels, t32.data());
      ensure(ctx, ctx->head_w32, h32.size() * 4);
      ensure(ctx, ctx->body_w32, b32.size() * 4);
      ensure(ctx, ctx->tail_w32, t32.size() * 4);
      HIPCHK(ctx, hipMemcpy(ctx->head_w32.p, h32.data(), h32.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(ctx, hipMemcpy(ctx->body_w32.p, b32.data(), b32.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(ctx, hipMemcpy(ctx->tail_w32.p, t32.data(), t32.size() * 4, hipMemcpyHostToDevice));
    }
    std::memcpy(tb.data(), p + channels * kWidth * 9, channels * sizeof(float));
    ensure(ctx, ctx->head_w, hw.size() * 2);
    ensure(ctx, ctx->head_b, hb.size() * 4);
    ensure(ctx, ctx->body_w, bw.size() * 2);
    ensure(ctx, ctx->body_b, bb.size() * 4);
    ensure(ctx, ctx->tail_w, tw.size() * 2);
    ensure(ctx, ctx->tail_b, tb.size() * 4);
    HIPCHK(ctx, hipMemcpy(ctx->head_w.p, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->head_b.p, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->body_w.p, bw.data(), bw.size() * 2, hipMemcpyHostToDevice));
    ensure(ctx, ctx->body_w16, bw16.size() * 2);
    HIPCHK(ctx, hipMemcpy(ctx->body_w16.p, bw16.data(), bw16.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->body_b.p, bb.data(), bb.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->tail_w.p, tw.data(), tw.size() * 2, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->tail_b.p, tb.data(), tb.size() * 4, hipMemcpyHostToDevice));
    ctx->den_C = channels;
    ctx->den_depth = depth;
    ctx->den_act = activation;
    ctx->den_residual = residual_sign;
    ctx->den_clamp = clamp_io ? 1 : 0;
    ctx->den_ready = true;
  });
}

int pnp_set_operator(pnp_ctx* ctx, int kind, const double* h, int kh, int kw, const uint8_t* keep_mask, int H,
                     int W) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    ctx->gen++;
    // the loaded solver state depends on the operator (the Poisson-ADMM c1 = Phi^T 1 and the
    // shape checks of solver_setup): a new operator needs pnp_solver_load / pnp_run again
    ctx->loaded = false;
    if (kind == PNP_OP_ID) {
      ctx->op_kind = kind;
      return;
    }
    if (kind == PNP_OP_BLUR) {
      if (!h || kh < 1 || kw < 1) fail(ctx, PNP_E_ARG, "blur needs a kernel");
      if (kh != kw) fail(ctx, PNP_E_UNSUPPORTED, "blur kernel must be square (operators.py:9 uses h.shape[0])");
      // operators.py:7-38: Phi   y[i,j] = sum h[a,b] x[i - a + mf, j - b + mf], mf = (l-1)//2
      //                    Phi^T y[i,j] = sum h[a,b] x[i + a - ma, j + b - ma], ma = l//2
      const int l = kh, mf = (l - 1) / 2, ma = l / 2;
      std::vector<int4> fwd, adj;
      std::vector<Tap64> f64;
      int R = 0;
      for (int a = 0; a < kh; ++a)
        for (int b = 0; b < kw; ++b) {
          const double v = h[a * kw + b];
          if (v == 0.0) continue;
          const float fv = (float)v;
          int bits;
          std::memcpy(&bits, &fv, 4);
          fwd.push_back(make_int4(mf - a, mf - b, bits, 0));
          f64.push_back(Tap64{mf - a, mf - b, v});
          adj.push_back(make_int4(a - ma, b - ma, bits, 0));
          R = std::max({R, std::abs(mf - a), std::abs(mf - b), std::abs(a - ma), std::abs(b - ma)});
        }
      if (R > 16) fail(ctx, PNP_E_UNSUPPORTED, "blur support radius %d > 16", R);
      if (fwd.empty()) fwd.push_back(make_int4(0, 0, 0, 0)), adj.push_back(make_int4(0, 0, 0, 0));
      ensure(ctx, ctx->taps_fwd, fwd.size() * sizeof(int4));
      ensure(ctx, ctx->taps_adj, adj.size() * sizeof(int4));
      HIPCHK(ctx, hipMemcpy(ctx->taps_fwd.p, fwd.data(), fwd.size() * sizeof(int4), hipMemcpyHostToDevice));
      HIPCHK(ctx, hipMemcpy(ctx->taps_adj.p, adj.data(), adj.size() * sizeof(int4), hipMemcpyHostToDevice));
      if (const int Rd = dense_radius(R)) {   // dense (2Rd+1)^2 tables for the register-blocked stencils
        const int D = 2 * Rd + 1;
        std::vector<float> df((size_t)D * D, 0.f), da((size_t)D * D, 0.f);
        for (size_t i = 0; i < fwd.size(); ++i) {
          float v;
          std::memcpy(&v, &fwd[i].z, 4);
          df[(size_t)(fwd[i].y + Rd) * D + fwd[i].x + Rd] += v;   // column-major: [ox + Rd][oy + Rd]
          da[(size_t)(adj[i].y + Rd) * D + adj[i].x + Rd] += v;
        }
        std::vector<uint32_t> mf(D, 0u), mad(D, 0u);   // non-zero pattern, column-major like the tables
        for (int cx = 0; cx < D; ++cx)
          for (int cy = 0; cy < D; ++cy) {
            if (df[(size_t)cx * D + cy] != 0.f) mf[cx] |= 1u << cy;
            if (da[(size_t)cx * D + cy] != 0.f) mad[cx] |= 1u << cy;
          }
        ctx->op_taps_id = match_taps(Rd, mf.data(), mad.data());
        std::vector<float> pf((size_t)(Rd + 1) * D * 4), pa((size_t)(Rd + 1) * D * 4);
        pack_tap_pairs(Rd, df.data(), pf.data());
        pack_tap_pairs(Rd, da.data(), pa.data());
        ensure(ctx, ctx->dense_fwd, pf.size() * sizeof(float));
        ensure(ctx, ctx->dense_adj, pa.size() * sizeof(float));
        HIPCHK(ctx, hipMemcpy(ctx->dense_fwd.p, pf.data(), pf.size() * sizeof(float), hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(ctx->dense_adj.p, pa.data(), pa.size() * sizeof(float), hipMemcpyHostToDevice));
      }
      if (f64.empty()) f64.push_back(Tap64{0, 0, 0.0});
      ensure(ctx, ctx->taps64, f64.size() * sizeof(Tap64));
      HIPCHK(ctx, hipMemcpy(ctx->taps64.p, f64.data(), f64.size() * sizeof(Tap64), hipMemcpyHostToDevice));
      ctx->op_ntaps = (int)fwd.size();
      ctx->op_R = R;
      ctx->op_kind = kind;
      return;
    }
    if (kind == PNP_OP_RANDOM_SAMPLING) {
      if (!keep_mask || H < 1 || W < 1) fail(ctx, PNP_E_ARG, "random_sampling needs an HxW keep mask");
      ensure(ctx, ctx->mask, (size_t)H * W);
      HIPCHK(ctx, hipMemcpy(ctx->mask.p, keep_mask, (size_t)H * W, hipMemcpyHostToDevice));
      ctx->op_H = H;
      ctx->op_W = W;
      ctx->op_kind = kind;
      return;
    }
    fail(ctx, PNP_E_UNSUPPORTED, "operator kind %d", kind);
  });
}

int pnp_solver_setup(pnp_ctx* ctx, int method, const pnp_params* params, int B, int C, int H, int W,
                     int metrics_capacity) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] { solver_setup(ctx, method, params, B, C, H, W, metrics_capacity); });
}

int pnp_solver_load(pnp_ctx* ctx, const float* x0, const float* xobs, const float* xtrue) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (ctx->method < 0) fail(ctx, PNP_E_STATE, "pnp_solver_setup first");
    if (!x0 || !xobs) fail(ctx, PNP_E_ARG, "x0 and xobs are required");
    const size_t fb = (size_t)ctx->B * ctx->C * ctx->H * ctx->W * sizeof(float);
    HIPCHK(ctx, hipMemcpy(ctx->x[0].p, x0, fb, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->xobs.p, xobs, fb, hipMemcpyHostToDevice));
    ctx->has_true = xtrue != nullptr;
    if (xtrue) HIPCHK(ctx, hipMemcpy(ctx->xtrue.p, xtrue, fb, hipMemcpyHostToDevice));
    solver_reset_state(ctx);
  });
}

int pnp_solver_load_device(pnp_ctx* ctx, const float* d_x0, const float* d_xobs, const float* d_xtrue) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (ctx->method < 0) fail(ctx, PNP_E_STATE, "pnp_solver_setup first");
    if (!d_x0 || !d_xobs) fail(ctx, PNP_E_ARG, "x0 and xobs are required");
    const size_t fb = (size_t)ctx->B * ctx->C * ctx->H * ctx->W * sizeof(float);
    HIPCHK(ctx, hipMemcpyAsync(ctx->x[0].p, d_x0, fb, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->xobs.p, d_xobs, fb, hipMemcpyDeviceToDevice, ctx->stream));
    ctx->has_true = d_xtrue != nullptr;
    if (d_xtrue) HIPCHK(ctx, hipMemcpyAsync(ctx->xtrue.p, d_xtrue, fb, hipMemcpyDeviceToDevice, ctx->stream));
    solver_reset_state(ctx);
  });
}

int pnp_solver_iterate(pnp_ctx* ctx, int n_iter) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!ctx->loaded) fail(ctx, PNP_E_STATE, "pnp_solver_load first");
    if (n_iter < 0) fail(ctx, PNP_E_ARG, "n_iter < 0");
    if (ctx->prof) {
      ctx->prof_log.clear();
      ctx->ev_used = 0;
    }
    solver_run(ctx, n_iter);
  });
}

int pnp_solver_fetch(pnp_ctx* ctx, float* x_out, float* s_out, double* c_out, double* psnr_out,
                     double* ssim_out) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] { solver_fetch(ctx, x_out, s_out, c_out, psnr_out, ssim_out); });
}

int pnp_solver_iterations_done(pnp_ctx* ctx, int* n) {
  if (!ctx || !n) return PNP_E_ARG;
  *n = ctx->it;
  return PNP_OK;
}

int pnp_solver_state(pnp_ctx* ctx, const float** d_x, const float** d_y, const float** d_s) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!ctx->loaded) fail(ctx, PNP_E_STATE, "solver not loaded");
    if (d_x) *d_x = P<const float>(ctx->x[ctx->cur]);
    if (d_y) {
      finalize_dual(ctx);
      *d_y = dual_buf(ctx, dual_fused(ctx, op_desc(ctx)) ? ctx->cur : 0);
    }
    if (d_s) *d_s = P<const float>(ctx->s);
  });
}

int pnp_run(pnp_ctx* ctx, int method, const pnp_params* params, int B, int C, int H, int W, const float* x0,
            const float* xobs, const float* xtrue, int max_iter, float* x_out, float* s_out, double* c_out,
            double* psnr_out, double* ssim_out, double* avg_time_s) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (max_iter < 0) fail(ctx, PNP_E_ARG, "max_iter < 0");
    solver_setup(ctx, method, params, B, C, H, W, max_iter);
    if (!x0 || !xobs) fail(ctx, PNP_E_ARG, "x0 and xobs are required");
    const size_t fb = (size_t)B * C * H * W * sizeof(float);
    HIPCHK(ctx, hipMemcpy(ctx->x[0].p, x0, fb, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->xobs.p, xobs, fb, hipMemcpyHostToDevice));
    ctx->has_true = xtrue != nullptr;
    if (xtrue) HIPCHK(ctx, hipMemcpy(ctx->xtrue.p, xtrue, fb, hipMemcpyHostToDevice));
    solver_reset_state(ctx);
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    const auto t0 = std::chrono::steady_clock::now();
    solver_run(ctx, max_iter);
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (avg_time_s) *avg_time_s = max_iter ? dt / max_iter : 0.0;
    solver_fetch(ctx, x_out, s_out, c_out, psnr_out, ssim_out);
  });
}

int pnp_profile_enable(pnp_ctx* ctx, int enable) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (enable < 0 || enable > 2) fail(ctx, PNP_E_ARG, "profile mode must be 0 (off), 1 (every launch) or 2 (body launches)");
    ctx->gen++;   // a captured graph holds the other mode's event packets
    ctx->prof = enable;
    ctx->prof_log.clear();
    ctx->ev_used = 0;
  });
}

int pnp_profile_read(pnp_ctx* ctx, int cap, const char** names, double* avg_ms, int* calls, int* n) {
  if (!ctx || !n) return PNP_E_ARG;
  return guarded(ctx, [&] {
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<std::string> keys;
    std::vector<double> tot;
    std::vector<int> cnt;
    for (const ProfEntry& e : ctx->prof_log) {
      float ms = 0;
      HIPCHK(ctx, hipEventElapsedTime(&ms, e.a, e.b));
      size_t k = 0;
      while (k < keys.size() && keys[k] != e.name) ++k;
      if (k == keys.size()) { keys.push_back(e.name); tot.push_back(0); cnt.push_back(0); }
      tot[k] += ms;
      cnt[k] += 1;
    }
    const int m = (int)keys.size();
    for (int i = 0; i < m && i < cap; ++i) {
      if (names) {
        // names point at string literals from ProfScope (static storage)
        for (const ProfEntry& e : ctx->prof_log)
          if (keys[i] == e.name) { names[i] = e.name; break; }
      }
      if (avg_ms) avg_ms[i] = tot[i] / cnt[i];
      if (calls) calls[i] = cnt[i];
    }
    *n = m;
  });
}

// ---- single operators ------------------------------------------------------------------
int pnp_op_phi(pnp_ctx* ctx, const float* x, float* y, int B, int C, int H, int W, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!x || !y || B < 1 || C < 1 || H < 1 || W < 1) fail(ctx, PNP_E_ARG, "bad arguments");
    check_operator_shape(ctx, H, W);
    launch_op_phi(ctx->op_kind, 0, x, y, op_desc(ctx), B * C, H, W, pick_stream(ctx, stream));
    check_launch(ctx, "op_phi");
  });
}

int pnp_op_adj_phi(pnp_ctx* ctx, const float* x, float* y, int B, int C, int H, int W, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!x || !y || B < 1 || C < 1 || H < 1 || W < 1) fail(ctx, PNP_E_ARG, "bad arguments");
    check_operator_shape(ctx, H, W);
    launch_op_phi(ctx->op_kind, 1, x, y, op_desc(ctx), B * C, H, W, pick_stream(ctx, stream));
    check_launch(ctx, "op_adj_phi");
  });
}

int pnp_op_proj_l2_ball(pnp_ctx* ctx, const float* x, const float* x0, float* out, int B, int64_t n,
                        double alpha_n, double gaussian_nl, double sp_nl, double r, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!x || !x0 || !out || B < 1 || n < 1) fail(ctx, PNP_E_ARG, "bad arguments");
    ensure(ctx, ctx->scr_part, (size_t)B * chunk_count((size_t)n) * sizeof(double));
    const double eps = std::sqrt((double)n * (1.0 - sp_nl)) * r * alpha_n * gaussian_nl;   // operators.py:104
    launch_l2_proj(x, x0, out, P<double>(ctx->scr_part), B, (size_t)n, eps, pick_stream(ctx, stream));
    check_launch(ctx, "l2_proj");
  });
}

int pnp_op_proj_l1_ball(pnp_ctx* ctx, const float* x, float* out, int B, int64_t n, double alpha_s, double sp_nl,
                        double r, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!x || !out || B < 1 || n < 1) fail(ctx, PNP_E_ARG, "bad arguments");
    if ((size_t)n >= kMaxL1Elems) fail(ctx, PNP_E_UNSUPPORTED, "l1-ball projection of %lld >= 2^29 elements per image",
                                      (long long)n);
    ensure(ctx, ctx->scr_theta, (size_t)B * sizeof(float));
    const double eta = alpha_s * (double)n * sp_nl * r * 0.5;    // operators.py:96
    hipStream_t st = pick_stream(ctx, stream);
    l1_select(ctx, ctx->scr_l1, x, P<float>(ctx->scr_theta), B, (size_t)n, eta, st);
    check_launch(ctx, "l1_select");
    launch_shrink(x, out, P<float>(ctx->scr_theta), B, (size_t)n, st);
    check_launch(ctx, "shrink");
  });
}

int pnp_op_prox_gkl(pnp_ctx* ctx, const float* x, const float* x0, float* out, int64_t count, double gamma,
                    double alpha, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!x || !x0 || !out || count < 0) fail(ctx, PNP_E_ARG, "bad arguments");
    if (count == 0) return;
    launch_gkl(x, x0, out, (size_t)count, gamma, alpha, pick_stream(ctx, stream));
    check_launch(ctx, "gkl");
  });
}

int pnp_op_denoise(pnp_ctx* ctx, const float* x, float* out, int B, int C, int H, int W, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!x || !out || B < 1 || H < 1 || W < 1) fail(ctx, PNP_E_ARG, "bad arguments");
    if (!ctx->den_ready) fail(ctx, PNP_E_STATE, "denoiser not set");
    if (C != ctx->den_C) fail(ctx, PNP_E_ARG, "denoiser has %d channels, input has %d", ctx->den_C, C);
    hipStream_t st = pick_stream(ctx, stream);
    ensure(ctx, ctx->scr_u32, (size_t)B * C * H * W * sizeof(float));
    launch_pack_input(x, P<float>(ctx->scr_u32), B, C, H, W, ctx->den_clamp, st);
    check_launch(ctx, "pack_input");
    // this call's precision (auto: split fp16, the reference denoiser's fp32 to ~2e-7); the
    // solver's resolved precision (and its captured graph) is left as it was
    struct Restore {
      pnp_ctx* c;
      int p;
      ~Restore() { c->prec = p; }
    } restore{ctx, ctx->prec};
    ctx->prec = (ctx->prec_req == PNP_PREC_AUTO || ctx->prec_req == PNP_PREC_CONVERGE) ? PNP_PREC_FP16X3
                                                                                         : ctx->prec_req;
    run_denoiser(ctx, P<float>(ctx->scr_u32), out, ctx->scr_act, B, H, W, st);
  });
}

int pnp_fp16_filter_round(const float* w, size_t n_filters, float* out) {
  if (!w || !out) return PNP_E_ARG;
  fp16_filter_round(w, n_filters, out);
  return PNP_OK;
}

int pnp_auto_precision(int method, int op_kind, double gaussian_nl) {
  if (method < PNP_METHOD_A || method > PNP_METHOD_C_RED || op_kind < PNP_OP_ID || op_kind > PNP_OP_RANDOM_SAMPLING)
    return PNP_E_ARG;
  return auto_precision(method, op_kind, gaussian_nl);
}

int pnp_op_status(pnp_ctx* ctx, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    // the persistent single-op launches run on ctx->stream only (use_stack), whatever stream the
    // caller passes: synchronize both, so a failure that is still being written is not missed
    HIPCHK(ctx, hipStreamSynchronize(pick_stream(ctx, stream)));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    check_stack_err(ctx, ctx->scr_stack_err);
  });
}

int pnp_device_copy(pnp_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!dst || !src || bytes % 16 || ((uintptr_t)dst | (uintptr_t)src) % 16)
      fail(ctx, PNP_E_ARG, "copy needs 16-B aligned pointers and a multiple of 16 bytes");
    launch_copy_f4(src, dst, bytes, ctx->num_cus, pick_stream(ctx, stream));
    check_launch(ctx, "copy_f4");
  });
}

int pnp_op_psnr(pnp_ctx* ctx, const float* x_true, const float* x, int B, int64_t n, double* psnr_out,
                void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!x_true || !x || !psnr_out || B < 1 || n < 1) fail(ctx, PNP_E_ARG, "bad arguments");
    const int chunks = chunk_count((size_t)n);
    ensure(ctx, ctx->scr_part, (size_t)B * chunks * sizeof(double));
    hipStream_t st = pick_stream(ctx, stream);
    launch_sqdiff(x_true, x, P<double>(ctx->scr_part), B, (size_t)n, st);
    check_launch(ctx, "sqdiff");
    std::vector<double> part((size_t)B * chunks);
    HIPCHK(ctx, hipMemcpyAsync(part.data(), ctx->scr_part.p, part.size() * sizeof(double), hipMemcpyDeviceToHost,
                               st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    for (int b = 0; b < B; ++b) {
      double s = 0;
      for (int k = 0; k < chunks; ++k) s += part[(size_t)b * chunks + k];
      psnr_out[b] = 10.0 * std::log10(1.0 / (s / (double)n));       // utils_eval.py:4-7
    }
  });
}

int pnp_op_ssim(pnp_ctx* ctx, const float* x_true, const float* x, int B, int C, int H, int W, double* ssim_out,
                void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!x_true || !x || !ssim_out || B < 1 || C < 1 || H < 1 || W < 1) fail(ctx, PNP_E_ARG, "bad arguments");
    if (C == 1 ? W < 7 : (H < 7 || W < 7)) fail(ctx, PNP_E_ARG, "SSIM needs a 7x7 window inside the image");
    ensure(ctx, ctx->scr_part, ssim_scratch_bytes(B, C, H, W) + (size_t)B * kMetrics * sizeof(double) + 256);
    hipStream_t st = pick_stream(ctx, stream);
    double* m = P<double>(ctx->scr_part);                     // metrics[b][0][kMetrics]
    void* scr = reinterpret_cast<char*>(ctx->scr_part.p) + (((size_t)B * kMetrics * sizeof(double) + 255) & ~(size_t)255);
    launch_ssim(x_true, x, scr, m, B, C, H, W, 0, 1, st);
    check_launch(ctx, "ssim");
    std::vector<double> h((size_t)B * kMetrics);
    HIPCHK(ctx, hipMemcpyAsync(h.data(), m, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    for (int b = 0; b < B; ++b) ssim_out[b] = h[(size_t)b * kMetrics + 2];
  });
}

// main.py:49-64 on the device; see degrade.hip for the numpy-stream restatement.
int pnp_degrade(pnp_ctx* ctx, const pnp_degrade_params* p, int B, int C, int H, int W, const float* d_xtrue,
                float* d_xobs, float* d_x0, double* d_xobs64, void* stream) {
  if (!ctx) return PNP_E_ARG;
  return guarded(ctx, [&] {
    if (!p || !d_xtrue || (!d_xobs && !d_x0 && !d_xobs64)) fail(ctx, PNP_E_ARG, "bad arguments");
    if (B < 1 || H < 1 || W < 1 || (C != 1 && C != 3))
      fail(ctx, PNP_E_ARG, "bad shape B=%d C=%d H=%d W=%d (utils_noise.py handles (H,W) and (3,H,W))", B, C, H, W);
    if (p->poisson_noise && !(p->poisson_alpha > 0.0)) fail(ctx, PNP_E_ARG, "poisson_alpha must be > 0");
    check_operator_shape(ctx, H, W);
    hipStream_t st = pick_stream(ctx, stream);
    const size_t n = (size_t)C * H * W, N = (size_t)B * n;
    const int noise_cnt = (int)((double)H * W * p->sp_nl / 2.0);      // utils_noise.py:4
    const size_t npairs = noise_cnt > 0 ? 2 * (size_t)noise_cnt : 0;  // utils_noise.py:11
    const size_t ndraw = 2 * npairs;
    const size_t half = (n + 1) / 2, ncand = half + half / 2 + 4096;  // legacy_gauss acceptance pi/4
    const uint32_t rng = (uint32_t)(H - 1);                           // randint(0, img.shape[-2])
    uint32_t mask = rng;
    for (int sh = 1; sh < 32; sh <<= 1) mask |= mask >> sh;
    size_t want = 0;
    if (p->gaussian_nl != 0.0) want = std::max(want, 4 * ncand);
    if (npairs && rng) want = std::max(want, 3 * ndraw + 4096);
    if (p->poisson_noise) want = std::max(want, 6 * n + 65536);
    const size_t scan_n = std::max({ncand, want, npairs, (size_t)1});
    ensure(ctx, ctx->dg_flag, scan_n * 4);
    ensure(ctx, ctx->dg_rank, scan_n * 4);
    ensure(ctx, ctx->dg_scan, scan_scratch_words(scan_n) * 4);
    ensure(ctx, ctx->dg_noise, n * sizeof(double));
    ensure(ctx, ctx->dg_img, N * sizeof(double));
    ensure(ctx, ctx->dg_status, 2 * sizeof(unsigned long long));
    auto stream_words = [&](size_t nw) {       // the tempered MT19937 stream of np.random.seed(seed)
      nw = (nw + kMtBlock - 1) / kMtBlock * kMtBlock;
      if (ctx->dg_nwords >= nw && ctx->dg_seed == p->seed) return;
      ensure(ctx, ctx->dg_words, nw * 4);
      launch_mt_stream(p->seed, P<uint32_t>(ctx->dg_words), nw, st);
      check_launch(ctx, "mt_stream");
      ctx->dg_nwords = nw;
      ctx->dg_seed = p->seed;
    };
    auto read_status = [&](unsigned long long* h) {
      HIPCHK(ctx, hipMemcpyAsync(h, ctx->dg_status.p, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipStreamSynchronize(st));
    };
    stream_words(std::max(want, (size_t)kMtBlock));
    // 1) x_obs = Phi(x_true) + M(sigma randn)        utils_noise.py:35-38
    const double* noise = nullptr;
    if (p->gaussian_nl != 0.0) {
      launch_gauss(P<uint32_t>(ctx->dg_words), ncand, P<uint32_t>(ctx->dg_flag), P<uint32_t>(ctx->dg_rank),
                   P<uint32_t>(ctx->dg_scan), P<double>(ctx->dg_noise), n, st);
      check_launch(ctx, "gauss");
      uint32_t acc = 0;
      HIPCHK(ctx, hipMemcpyAsync(&acc, ctx->dg_scan.p, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipStreamSynchronize(st));
      if (acc < half) fail(ctx, PNP_E_INTERNAL, "gaussian stream too short (%u of %zu pairs)", acc, half);
      noise = P<double>(ctx->dg_noise);
    }
    const OpDesc od = op_desc(ctx);
    for (int attempt = 0;; ++attempt) {
      launch_observe(d_xtrue, noise, P<Tap64>(ctx->taps64), ctx->op_ntaps, od.mask, ctx->op_kind, p->gaussian_nl,
                     P<double>(ctx->dg_img), B, C, H, W, st);
      check_launch(ctx, "observe");
      if (!p->poisson_noise) break;
      // 2) x_obs = poisson(alpha x_obs)              utils_noise.py:40-43
      HIPCHK(ctx, hipMemsetAsync(ctx->dg_status.p, 0, 2 * sizeof(unsigned long long), st));
      launch_poisson(P<uint32_t>(ctx->dg_words), ctx->dg_nwords, P<double>(ctx->dg_img), B, n, p->poisson_alpha,
                     P<unsigned long long>(ctx->dg_status), st);
      check_launch(ctx, "poisson");
      unsigned long long hs[2];
      read_status(hs);
      if (hs[0] == 1) fail(ctx, PNP_E_ARG, "poisson: lam < 0 or NaN (numpy raises ValueError)");
      if (hs[0] == 2) fail(ctx, PNP_E_ARG, "poisson: lam value too large");
      if (hs[0] != 3) break;
      if (attempt >= 6) fail(ctx, PNP_E_INTERNAL, "poisson stream exhausted");
      stream_words(2 * ctx->dg_nwords);            // deterministic: a longer prefix of the same stream
    }
    // 3) salt & pepper                               utils_noise.py:3-33
    if (npairs) {
      const uint8_t* tgt = ctx->op_kind == PNP_OP_RANDOM_SAMPLING ? od.mask : nullptr;
      const size_t side = (size_t)H * std::max(H, W);
      ensure(ctx, ctx->dg_draws, ndraw * 4);
      ensure(ctx, ctx->dg_first, side * 4);
      HIPCHK(ctx, hipMemsetAsync(ctx->dg_first.p, 0xff, side * 4, st));
      HIPCHK(ctx, hipMemsetAsync(ctx->dg_status.p, 0, 2 * sizeof(unsigned long long), st));
      if (rng == 0) {
        HIPCHK(ctx, hipMemsetAsync(ctx->dg_draws.p, 0, ndraw * 4, st));   // randint(0, 1) draws nothing
      } else {
        size_t nw = std::min(ctx->dg_nwords, 3 * ndraw + 4096);   // words scanned for the draws
        for (int attempt = 0;; ++attempt) {
          ensure(ctx, ctx->dg_flag, nw * 4);
          ensure(ctx, ctx->dg_rank, nw * 4);
          ensure(ctx, ctx->dg_scan, scan_scratch_words(nw) * 4);
          launch_sp_draws(P<uint32_t>(ctx->dg_words), nw, mask, rng, P<uint32_t>(ctx->dg_flag),
                          P<uint32_t>(ctx->dg_rank), P<uint32_t>(ctx->dg_scan), P<uint32_t>(ctx->dg_draws), ndraw, st);
          check_launch(ctx, "sp_draws");
          uint32_t valid = 0;
          HIPCHK(ctx, hipMemcpyAsync(&valid, ctx->dg_scan.p, 4, hipMemcpyDeviceToHost, st));
          HIPCHK(ctx, hipStreamSynchronize(st));
          if (valid >= ndraw) break;
          if (attempt >= 6) fail(ctx, PNP_E_INTERNAL, "salt-and-pepper stream exhausted");
          nw *= 2;
          stream_words(nw);
        }
      }
      launch_sp_apply(P<uint32_t>(ctx->dg_draws), (int)npairs, tgt, H, W, P<uint32_t>(ctx->dg_first),
                      P<uint32_t>(ctx->dg_flag), P<uint32_t>(ctx->dg_rank), P<uint32_t>(ctx->dg_scan), noise_cnt,
                      P<double>(ctx->dg_img), B, C, P<unsigned long long>(ctx->dg_status), st);
      check_launch(ctx, "sp_apply");
      unsigned long long hs[2];
      read_status(hs);
      if (hs[0] == 4) fail(ctx, PNP_E_ARG, "salt-and-pepper: column index out of range (the reference draws "
                                           "columns in [0, H) and raises IndexError when H > W)");
    }
    // 4) x_obs (float32 state of the solver), x_0 = x_obs (/ alpha)   main.py:62-64
    launch_degrade_finalize(P<double>(ctx->dg_img), N, p->poisson_alpha, p->poisson_noise, d_xobs, d_x0, d_xobs64, st);
    check_launch(ctx, "degrade_finalize");
    HIPCHK(ctx, hipStreamSynchronize(st));
  });
}

}  // extern "C"
