/*
 * pnppds.h — C ABI of the MI355X-native PnP-PDS inner loop (libpnppds.so).
 *
 * Drop-in boundary for the reference's solver path (yodai49/PnP-PDS):
 *   iteration.test_iter            iteration.py:10-196       -> pnp_run / pnp_solver_*
 *   get_observation_operators      operators.py:60-79        -> pnp_set_operator
 *   Denoiser(file_name, ch)        models/denoiser.py:9-32   -> pnp_set_denoiser
 *   Denoiser.denoise / apply_model models/denoiser.py:14-46  -> pnp_op_denoise
 *   get_blur_operator / _adj_      operators.py:7-38         -> pnp_op_phi / pnp_op_adj_phi
 *   get_random_sampling_operator   operators.py:40-58        -> pnp_op_phi / pnp_op_adj_phi
 *   proj_l2_ball                   operators.py:102-108      -> pnp_op_proj_l2_ball
 *   proj_l1_ball                   operators.py:94-100       -> pnp_op_proj_l1_ball
 *   prox_GKL                       operators.py:114-115      -> pnp_op_prox_gkl
 *   eval_psnr                      utils/utils_eval.py:4-7   -> pnp_op_psnr
 *
 * Conventions
 *   - Images are B x C x H x W, C-contiguous float32 (the reference's (C,H,W) numpy
 *     layout with a leading batch axis).  C in {1, 3} (any C <= 4 works).
 *   - Host pointers are borrowed for the duration of the call; the library copies.
 *   - Device pointers (pnp_op_*) are hipMalloc'd memory on the context's device.
 *   - Every entry returns PNP_OK (0) or a negative PNP_E_* code; pnp_last_error()
 *     returns a message for the last failure on that context (or the thread, if the
 *     context is NULL).
 *   - A context is bound to one device and is not thread-safe.  Different contexts
 *     may be driven from different host threads (one per GPU).
 *   - No CPU fallback: without a usable HIP device every compute entry fails.
 */
#ifndef PNPPDS_H
#define PNPPDS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNP_ABI_VERSION 8

typedef struct pnp_ctx pnp_ctx;

enum pnp_status {
  PNP_OK = 0,
  PNP_E_ARG = -1,         /* bad argument / shape                                     */
  PNP_E_UNSUPPORTED = -2, /* method / operator / denoiser shape not supported          */
  PNP_E_HIP = -3,         /* HIP runtime error (message has the hipError string)      */
  PNP_E_OOM = -4,         /* device allocation failed                                 */
  PNP_E_STATE = -5,       /* call out of order (e.g. iterate before load)             */
  PNP_E_INTERNAL = -6     /* internal limit reached (message says which)              */
};

/* iteration.py:48-63 ('A-Proposed' / 'B-Proposed' / 'C-Proposed'; README: ours-A/B/C)
 * and iteration.py:127-132 ('comparisonB-2', ADMM inner steps of algorithm/admm.py)   */
enum pnp_method {
  PNP_METHOD_A = 0,       /* Gaussian noise, l2-ball data constraint                  */
  PNP_METHOD_B = 1,       /* Gaussian + sparse noise, l2 ball + l1 ball on s           */
  PNP_METHOD_C = 2,       /* Poisson noise, generalised-KL prox                       */
  PNP_METHOD_ADMM_B2 = 3, /* comparisonB-2: ADMM, denoiser x-step (admm.py:30-44)    */
  /* comparison methods (iteration.py:71-180; the BM3D ones are not available)       */
  PNP_METHOD_A_PNPFBS = 4,  /* A-PnPFBS-DnCNN:  x = D(x - g1 lam Phi^T(Phi x - x_obs))    */
  PNP_METHOD_A_PDS_TV = 5,  /* A-PDS-TV:  PDS with TV (D, D^T, prox_l12) + l2 ball        */
  PNP_METHOD_A_FBS_TV = 6,  /* A-FBS-TV:  additive data term + TV dual                    */
  PNP_METHOD_A_RED = 7,     /* A-RED-DnCNN: RED steepest descent                          */
  PNP_METHOD_B_HTV = 8,     /* comparisonB-3: TV + l1 ball on s + l2 ball                 */
  PNP_METHOD_B_RED = 9,     /* comparisonB-4: RED with the sparse component               */
  PNP_METHOD_B_PNPFBS = 10, /* comparisonB-5: PnP-FBS with the sparse component           */
  PNP_METHOD_C_PNPADMM = 11,/* C-PnPADMM-DnCNN: Poisson ADMM, denoiser z-step             */
  PNP_METHOD_C_RED = 12     /* C-RED-DnCNN: Poisson ADMM, RED z-step                      */
  /* A-PnPPDS-unstable-DnCNN / C-PnP-unstable-DnCNN are METHOD_A / METHOD_C with the
   * KAIR DnCNN set as the denoiser (residual_sign -1, ReLU, clamp_io 0).             */
};

/* operators.py:60-79 */
enum pnp_operator_kind {
  PNP_OP_ID = 0,
  PNP_OP_BLUR = 1,            /* centred circular convolution with h (kh x kw)        */
  PNP_OP_RANDOM_SAMPLING = 2  /* pointwise 0/1 keep-mask shared by all channels      */
};

enum pnp_activation { PNP_ACT_LEAKY_RELU = 0 /* slope 0.01 */, PNP_ACT_RELU = 1 };

enum pnp_precision {
  PNP_PREC_FP16 = 0, /* fp16 MFMA operands, fp32 accumulation (default)            */
  PNP_PREC_FP32 = 1, /* fp32 operands and accumulation (v_mfma_f32_32x32x2_f32): the
                        reference denoiser's own precision (models/denoiser.py:37), the
                        parity fallback; about 1/10 of the fp16 path's throughput     */
  PNP_PREC_FP16W2 = 2,/* fp16 activations, weights split into fp16 hi + lo halves (two
                        MFMAs per product, ~22-bit weights), fp32 accumulation         */
  PNP_PREC_FP16X3 = 3,/* activations and weights both split into fp16 hi + lo halves,
                        three fp16 MFMAs per product (hi*hi + hi*lo + lo*hi), fp32
                        accumulation: near-fp32 results at 1/3 of the fp16 MFMA rate
                        (ABI 4)                                                      */
  PNP_PREC_AUTO = 4,  /* default (ABI 4): per solve, on the blur operator: FP16 for
                        A/B-Proposed, comparisonB-2, A-PnPFBS-DnCNN and A-RED-DnCNN up
                        to gaussian_nl = 0.01; above it FP16W2 for A-Proposed (measured
                        within 0.0005 dB of the reference over 1200 iterations at sigma
                        0.02 / 0.04) and comparisonB-2 (0.0002 dB over 30 outer
                        iterations at sigma 0.04); FP16X3 otherwise; single denoiser
                        calls (pnp_op_denoise) run FP16X3.
                        Where it runs FP16 or FP16W2, x and PSNR follow the reference
                        (<= 0.0035 dB) but c_n (iteration.py:187) does not below ~3e-4:
                        the fp16 activations' rounding sets a floor where successive
                        iterates stop contracting (the reference's c_n reaches ~7e-8).
                        Use PNP_PREC_CONVERGE where the c_n curve matters.            */
  PNP_PREC_CONVERGE = 5, /* (ABI 7; per image since ABI 8) per solve and per image: AUTO's
                        operands while the image's own c_n is above a threshold
                        (PNP_TUNE_CONVERGE_C, default 3e-3, ten times the fp16 floor), then
                        split activations for the rest of the solve: FP16A2 where AUTO runs
                        FP16 / FP16W2, FP16X3 elsewhere (where AUTO already runs FP16X3 it
                        switches at once).  Needs recorded metrics (record_metrics, iterations
                        within metrics_capacity) to watch c_n; without them every image
                        switches at once.  The switch is decided on the host one iteration
                        behind the device (pnp_solver_iterate then blocks per iteration until
                        every image has switched); while only some have, each denoiser pass
                        runs the batch as runs of consecutive images of one precision, so an
                        image's results do not depend on its batch or shard.  See
                        pnp_get_precision_switch(es).  Single denoiser calls run FP16X3.    */
  PNP_PREC_FP16A2 = 6   /* (ABI 7) activations split into fp16 hi + lo halves, single fp16
                        weights (rounded per filter as FP16's): two fp16 MFMAs per product in
                        the 64->64 layers (hi*w + lo*w); head and tail as FP16X3           */
};

/* Scalar parameters of iteration.test_iter (iteration.py:10), same names/meaning. */
typedef struct pnp_params {
  double gamma1, gamma2;          /* PDS step sizes                                   */
  double alpha_s, alpha_n;        /* l1-ball / l2-ball radius factors                  */
  double my_lambda;               /* GKL weight (C-Proposed)                           */
  int32_t m1, m2;                 /* ADMM inner iterations (comparisonB-2)             */
  double gamma_in_admm_step1;     /* unused by the supported methods (kept for parity) */
  double gaussian_nl, sp_nl;      /* sigma, salt-and-pepper rate                       */
  double poisson_alpha;           /* Poisson scale                                     */
  double r;                       /* sampling rate; also scales the B-method balls     */
  int32_t record_metrics;         /* 1: c_n and PSNR every iteration (iteration.py:187-188) */
  int32_t record_ssim;            /* 1 (with record_metrics): also SSIM (iteration.py:189)  */
} pnp_params;

/* ---- library / context -------------------------------------------------------- */
int pnp_abi_version(void);
/* SHA-256 prefix (16 hex digits) of the library's sources (pnp-pds_amd/Makefile HASHSRC),
 * baked in at build time: lets a caller detect a library built from other sources.    */
const char* pnp_build_id(void);
int pnp_device_count(int* count);
int pnp_create(int device, pnp_ctx** out);
int pnp_destroy(pnp_ctx* ctx);
const char* pnp_last_error(const pnp_ctx* ctx);
int pnp_synchronize(pnp_ctx* ctx);

/* Denoiser (models/denoiser.py:23-32 + basic_models.py:8-38, or the KAIR DnCNN of
 * network_dncnn.py:42-77).  `params` = [w0, b0, w1, b1, ...] in forward order, each
 * w_i in PyTorch layout (cout, cin, 3, 3) float32.  Layer 0: channels -> width, the
 * last layer: width -> channels, all others width -> width.  Only width == 64.
 * residual_sign: +1 => out = net(x) + x (simple_CNN), -1 => out = x - net(x) (KAIR).
 * clamp_io: 1 => clamp input and output to [0,1] (denoiser.py:40,42).            */
int pnp_set_denoiser(pnp_ctx* ctx, int channels, int depth, int width, const float* params,
                     size_t n_params, int activation, int residual_sign, int clamp_io);
/* Denoiser operand precision (pnp_precision); applies to every later denoiser call.
 * pnp_get_precision: the requested value and the one the next solver step will use.   */
int pnp_set_precision(pnp_ctx* ctx, int precision);
int pnp_get_precision(pnp_ctx* ctx, int* requested, int* effective);
/* (ABI 7) PNP_PREC_CONVERGE: the first iteration of the current solve from which every image
 * ran split activations (FP16A2 / FP16X3), or -1 while some image has not switched (or the
 * solve does not run PNP_PREC_CONVERGE).  For B = 1, the image's switch iteration.          */
int pnp_get_precision_switch(pnp_ctx* ctx, int* iteration);
/* (ABI 8) PNP_PREC_CONVERGE: per image b of the current solve, the first iteration it ran split
 * activations (-1: not yet).  n must be at least the solve's batch B (PNP_E_ARG otherwise).  */
int pnp_get_precision_switches(pnp_ctx* ctx, int* iterations, int n);

/* Performance knobs (no effect on results; PNP_TUNE_CONVERGE_C excepted).
 * PNP_TUNE_DENOISE_CHUNK: images per denoiser pass (0 = auto: the whole batch, unless its
 * activation ping-pong pair would exceed an eighth of the device's memory; then equal passes). */
enum pnp_tuning_key {
  PNP_TUNE_DENOISE_CHUNK = 1,
  PNP_TUNE_BODY_LAYERS = 2,  /* 64->64 layers per launch: 0 = auto (default: all of them in one
                                persistent launch when the batch has at most 2 tiles per CU,
                                e.g. one 256^2 image; else 2 when it has at least one 32-column
                                strip per CU, else 1), 1 (conv_body_v3), 2 (conv_body_f2, the
                                intermediate stays in LDS), 3 (all: conv_stack16x2, two layers
                                per tile hand-off when their number is even) or 4 (all:
                                conv_stack16, one layer per hand-off).  Bit-identical results. */
  PNP_TUNE_GRAPH = 3,         /* 1: iteration launches replayed from a hipGraph (two iterations
                                per replay, methods A/B/C); 0: direct launches (default).
                                Same results either way.                                       */
  PNP_TUNE_CONVERGE_C = 4,    /* (ABI 7) PNP_PREC_CONVERGE's c_n threshold in units of 1e-6
                                (default 3000 = 3e-3).  Changes when the solve switches, so it
                                changes results (within the tolerances of DESIGN.md §4).        */
  PNP_TUNE_FUSE_ENDS = 5      /* (ABI 7) 1 (default): when the two-layer launches run (FP16, even
                                body depth), the head runs inside the first one and the tail
                                inside the last; 0: separate head / tail launches.  Bit-identical. */
};
int pnp_set_tuning(pnp_ctx* ctx, int key, int value);

/* Observation operator (operators.py:60-79).  BLUR: h is kh x kw float64 row-major
 * (blur_models/blur_1.mat: 19x19); RANDOM_SAMPLING: keep_mask is H x W uint8 (1 keeps
 * the pixel; the reference drops RandomState(1234).permutation(H*W)[:round(H*W*(1-r))]).
 * ID: both NULL.                                                                  */
int pnp_set_operator(pnp_ctx* ctx, int kind, const double* h, int kh, int kw,
                     const uint8_t* keep_mask, int H, int W);

/* ---- whole solver (iteration.test_iter) ---------------------------------------- */
/* Batched test_iter: B independent images.  x0/xobs: B*C*H*W float32; xtrue may be
 * NULL (then psnr_out and ssim_out are NaN).  Outputs (any may be NULL): x_out, s_out
 * (= s + 0.5 as iteration.py:196 returns), c_out, psnr_out and ssim_out (B x max_iter
 * float64, row-major; ssim_out is NaN unless params->record_ssim),
 * avg_time_s = wall seconds per iteration on the device.                            */
int pnp_run(pnp_ctx* ctx, int method, const pnp_params* params, int B, int C, int H, int W,
            const float* x0, const float* xobs, const float* xtrue, int max_iter,
            float* x_out, float* s_out, double* c_out, double* psnr_out, double* ssim_out,
            double* avg_time_s);

/* Staged form of pnp_run, with state resident in HBM between calls (bench / drivers). */
int pnp_solver_setup(pnp_ctx* ctx, int method, const pnp_params* params, int B, int C, int H,
                     int W, int metrics_capacity);
int pnp_solver_load(pnp_ctx* ctx, const float* x0, const float* xobs, const float* xtrue);
int pnp_solver_load_device(pnp_ctx* ctx, const float* d_x0, const float* d_xobs,
                           const float* d_xtrue);
int pnp_solver_iterate(pnp_ctx* ctx, int n_iter);   /* enqueue only (async) */
int pnp_solver_fetch(pnp_ctx* ctx, float* x_out, float* s_out, double* c_out, double* psnr_out,
                     double* ssim_out);
int pnp_solver_iterations_done(pnp_ctx* ctx, int* n);
/* Device pointers of the solver's primal / dual state (read-only views, B*C*H*W).  ours-A / ours-B
 * on the blur operator keep the dual's l2-ball step pending between iterations (it runs inside
 * the next iteration's first pass); this call applies it first (enqueued on the solver stream),
 * so d_y is the dual as iteration.py holds it. */
int pnp_solver_state(pnp_ctx* ctx, const float** d_x, const float** d_y, const float** d_s);

/* Per-kernel timing of the last iterate() call: fills up to `cap` entries of
 * name/avg-ms pairs measured with hipEvents on the solver stream (profiling aid).  enable:
 * 0 off, 1 every launch, 2 (ABI 7) only the denoiser's body launches (conv_body*, conv32_body*,
 * conv_stack*), so the other launches run without event packets between them.            */
int pnp_profile_enable(pnp_ctx* ctx, int enable);
int pnp_profile_read(pnp_ctx* ctx, int cap, const char** names, double* avg_ms, int* calls, int* n);

/* ---- single operators on device pointers (stream NULL => context stream) -------- */
int pnp_op_phi(pnp_ctx* ctx, const float* x, float* y, int B, int C, int H, int W, void* stream);
int pnp_op_adj_phi(pnp_ctx* ctx, const float* x, float* y, int B, int C, int H, int W, void* stream);
/* per image b (n elements each): out = P_{B(x0_b, eps)}(x_b), eps = sqrt(n(1-sp_nl)) r alpha_n sigma */
int pnp_op_proj_l2_ball(pnp_ctx* ctx, const float* x, const float* x0, float* out, int B, int64_t n,
                        double alpha_n, double gaussian_nl, double sp_nl, double r, void* stream);
/* per image: projection onto {|s|_1 <= alpha_s * n * sp_nl * r / 2} */
int pnp_op_proj_l1_ball(pnp_ctx* ctx, const float* x, float* out, int B, int64_t n, double alpha_s,
                        double sp_nl, double r, void* stream);
int pnp_op_prox_gkl(pnp_ctx* ctx, const float* x, const float* x0, float* out, int64_t count,
                    double gamma, double alpha, void* stream);
int pnp_op_denoise(pnp_ctx* ctx, const float* x, float* out, int B, int C, int H, int W, void* stream);
/* (ABI 5) Synchronizes `stream` and the context's own stream (the persistent small-batch
 * launches run there whatever stream a single op is given) and reports whether a single-op
 * denoiser call's persistent launch failed (PNP_E_INTERNAL: its results are invalid).  The
 * solver's own launches are checked by pnp_solver_fetch.                               */
int pnp_op_status(pnp_ctx* ctx, void* stream);
/* (ABI 5, host only, no device) The fp16 values the fp16 operand precisions store for conv
 * weights: n_filters 3x3 filters (9 floats each, [c_out][c_in][3][3] order) rounded to fp16
 * so that each filter's rounding errors sum to ~0 (capi.hip fp16_filter_round).  out holds
 * float32 copies of the fp16 values; w and out may alias.                              */
int pnp_fp16_filter_round(const float* w, size_t n_filters, float* out);
/* (ABI 6, host only, no device) What PNP_PREC_AUTO resolves to for a solve of `method` on
 * operator `op_kind` at Gaussian noise level `gaussian_nl` (pnp_params.gaussian_nl): a
 * pnp_precision value, or PNP_E_ARG for an unknown method / operator.                    */
int pnp_auto_precision(int method, int op_kind, double gaussian_nl);
/* dst = src on the device (float4 streaming copy; 16-B aligned, bytes % 16 == 0).  The
 * measured copy ceiling bench.py reports the prox passes' HBM fraction against.        */
int pnp_device_copy(pnp_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream);
/* psnr_out: host array of B doubles (synchronous). */
int pnp_op_psnr(pnp_ctx* ctx, const float* x_true, const float* x, int B, int64_t n, double* psnr_out,
                void* stream);

/* ---- observation pipeline (main.py:49-64, utils/utils_noise.py) ------------------ */
typedef struct pnp_degrade_params {
  double gaussian_nl;      /* sigma of add_gaussian_noise (0: no Gaussian noise)          */
  double sp_nl;            /* add_salt_and_pepper_noise rate (0: none)                     */
  double poisson_alpha;    /* apply_poisson_noise scale                                    */
  int32_t poisson_noise;   /* 1: Poisson noise, and x_0 = x_obs / poisson_alpha            */
  uint32_t seed;           /* np.random.seed of utils_noise.py (1234)                      */
} pnp_degrade_params;
/* x_obs = SP(Poisson(Phi(x_true) + M(sigma g))) with the operator set by pnp_set_operator,
 * reproducing numpy's legacy RandomState draws (every image gets the reference's noise
 * field, as main.py reseeds per image).  Device pointers, B*C*H*W each; C is 1 ((H,W)
 * gray) or 3.  Outputs may be NULL: d_xobs / d_x0 float32, d_xobs64 the float64 x_obs the
 * reference hands to test_iter.  Synchronous on `stream`.                               */
int pnp_degrade(pnp_ctx* ctx, const pnp_degrade_params* p, int B, int C, int H, int W,
                const float* d_xtrue, float* d_xobs, float* d_x0, double* d_xobs64, void* stream);

/* utils_eval.py:9-12 eval_ssim per image: skimage structural_similarity(x_true, x,
 * data_range = x.max() - x.min(), channel_axis = 0) with scikit-image 0.22 defaults.
 * C == 1 images are the reference's (H, W) grayscale arrays (mean of per-row 1-D SSIMs).
 * ssim_out: host array of B doubles (synchronous).                                  */
int pnp_op_ssim(pnp_ctx* ctx, const float* x_true, const float* x, int B, int C, int H, int W,
                double* ssim_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PNPPDS_H */
