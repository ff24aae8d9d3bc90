// Shared definitions for the PnP-PDS HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

typedef _Float16 half_t;
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace pnp {

constexpr int kWave = 64;
constexpr int kWidth = 64;             // hidden channels of the denoiser
constexpr int kMaxC = 4;               // image channels handled by head/tail (C <= 4)

// ---- denoiser activation layout (HBM) ------------------------------------------------
// Hidden activations: fp16 [B][H+2][W+2][64] ("padded NHWC64"): a zero border of one
// pixel implements conv padding=1 with no boundary branches; 128 B per pixel.
// Head input:         fp16 [B][H+2][W+2][4]  ("padded NHWC4"), channels >= C are zero.
// Conv tiles: 8 output rows x 32 output columns; halo tile 10 x 34 pixels.
constexpr int kTileH = 8;
constexpr int kTileW = 32;
constexpr int kHaloH = kTileH + 2;
constexpr int kHaloW = kTileW + 2;
constexpr int kHaloPix = kHaloH * kHaloW;          // 340
constexpr int kBodyKSteps = 36;                    // 9 taps x 64 cin / 16
constexpr int kBodyWBytes = kBodyKSteps * 2 * kWave * 16;   // 73728: [s][m][lane][8 x f16]
constexpr int kHeadKSteps = 3;                     // 9 taps x 4 ch = 36 -> 48 / 16
// Split fp16 (PNP_PREC_FP16X3) weights are split at 2^8 times their value: |w_lo| <= 2^-11 |w|
// is an fp16 subnormal below |w| = 2^-3 at scale 1 (most DnCNN weights), so it kept fewer bits;
// the kernels unscale the accumulator by 2^-8 (exact) before the bias (conv_s3.hip, r06).
constexpr float kSplitWScale = 256.f, kSplitWInv = 1.f / 256.f;
constexpr float kS3BodyScale = kSplitWScale;     // the 64 -> 64 layers' split (conv_s3 body, stack)
constexpr int kHeadWBytes = kHeadKSteps * 2 * kWave * 16;   // 6144
constexpr int kTailKSteps = 18;                    // 9 taps x 64 cin / 32
constexpr int kTailWBytes = kTailKSteps * kWave * 16;       // 18432: [s][lane][8 x f16]

// Row i (0..31) of a 32x32x16 MFMA A-tile <-> output channel within the 32-channel
// M-tile, chosen so that accumulator register r of lane-half h holds channel 16h + r
// (C/D map: row = (r&3) + 8*(r>>2) + 4*h).  Each lane then owns 16 consecutive
// output channels of one pixel -> two 16-byte stores in the epilogue.
__host__ __device__ inline int mfma32_row_to_channel(int i) {
  return 16 * ((i >> 2) & 1) + (i & 3) + 4 * (i >> 3);
}

// LDS image of a halo tile (hidden activations): pixel (row pr, column pc) of the
// 10 x 34 halo occupies 128 B at p = pr*34 + pc; its eight 16-B channel chunks are
// XOR-swizzled by ((pc >> 1) & 7) so that the 16-lane groups of a ds_read_b128 over 16
// consecutive pixels of a row hit 16 distinct bank slots (34 is even, so p & 1 == pc & 1).
// The swizzle depends on the column only: a wave's tap offsets differ by whole rows, so
// the per-lane part of every fragment address is one of (3 columns x chunk) values and
// the row steps fold into immediate offsets.
__device__ __forceinline__ int halo_off(int pr, int pc, int chunk) {
  return (pr * kHaloW + pc) * 128 + 16 * (chunk ^ ((pc >> 1) & 7));
}
__device__ __forceinline__ int halo_chunk_offset(int p, int chunk) {
  const int pr = p / kHaloW;
  return halo_off(pr, p - pr * kHaloW, chunk);
}

__device__ __forceinline__ float act_fn(float v, int act) {
  return act == 0 ? (v > 0.f ? v : 0.01f * v) : (v > 0.f ? v : 0.f);
}

// ---- tile hand-off between workgroups (persistent small-batch denoiser) ------------------
// A layer's output tile is published with a per-tile progress word: the producer stores the
// tile with device-scope (sc1) stores, its storing waves drain (s_waitcnt vmcnt(0)), the
// workgroup barriers, then one lane stores done[t] = value (device scope).  A consumer polls
// with device-scope loads and then reads the tile with device-scope loads (the per-XCD L2s
// and per-CU L1s are not coherent with each other: MI355X_MICROARCH.md, inter-workgroup
// visibility).  Every spin is bounded: a stuck wait sets *err and proceeds (results wrong,
// no hang).
// The contract is sc1-only, not a language-level release / acquire: the flag store and poll
// are relaxed (agent-scope release / acquire fences measured slower: DESIGN.md §3, small
// batches), and the ordering comes from (1) every access to handed-off data using the device-
// scope cache policy kCpolDevice (sc1 stores, sc1 LDS-DMA loads), (2) the storing waves'
// s_waitcnt vmcnt(0) and (3) the workgroup barrier before the flag store.  A new access to a
// handed-off buffer must use kCpolDevice too.  tests/test_isa_handoff.py checks (1)-(3) on the
// built code object of every stack kernel.
constexpr int kTileSpinMax = 1 << 20;   // polls of ~0.1-1 us each: ~0.1-1 s before giving up

__device__ __forceinline__ void tile_publish(int* flag, int value) {
  __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave-level: lanes with want set poll flags[idx] until >= target (wrap-safe); every lane
// returns after all of them saw it (or the spin bound hit: *err = 1).  Call from one wave,
// then the workgroup barrier.
__device__ __forceinline__ void tile_wait(const int* flags, int idx, bool want, int target, int* err) {
  for (int it = 0; it < kTileSpinMax; ++it) {
    bool ok = true;
    if (want) ok = (__hip_atomic_load(flags + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) >= 0;
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) return;
    __builtin_amdgcn_s_sleep(1);
  }
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Launch of a persistent kernel whose workgroups wait on each other (the tile hand-off above),
// with the arguments converted to the kernel's parameter types as hipLaunchKernelGGL does.  The
// grid is at most one workgroup per CU and each needs most of a CU's LDS, so all of it is
// resident unless another persistent grid holds CUs at the same time: within a context only
// the solver's stream launches these kernels (capi.hip use_stack), and a wait that still hits
// its spin bound (another process's persistent grid) sets the error word, which
// pnp_solver_fetch / pnp_op_status turn into PNP_E_INTERNAL.  hipLaunchCooperativeKernel
// would guarantee co-residency but measured +30 us per launch at B = 1 (cfg2 0.184 -> 0.213
// ms per iteration, round 4), a sixth of the iteration.
template <typename... KArgs>
inline hipError_t persistent_launch_impl(void (*kernel)(KArgs...), int grid, int block, unsigned lds,
                                         hipStream_t st, KArgs... args) {
  void* ptrs[] = {static_cast<void*>(&args)...};
  return hipLaunchKernel(reinterpret_cast<const void*>(kernel), dim3(grid), dim3(block), ptrs, lds, st);
}
template <typename... KArgs, typename... Args>
inline hipError_t persistent_launch(void (*kernel)(KArgs...), int grid, int block, unsigned lds, hipStream_t st,
                                    Args... args) {
  static_assert(sizeof...(KArgs) == sizeof...(Args), "argument count");
  return persistent_launch_impl<KArgs...>(kernel, grid, block, lds, st, static_cast<KArgs>(args)...);
}

// Workgroup barrier for an LDS hand-off: this wave's LDS accesses complete (lgkmcnt(0)), then
// s_barrier.  __syncthreads' release fence also waits vmcnt(0), i.e. for every outstanding
// global store and load of the wave (measured in the ISA: the step barrier of conv_body_x8
// drained the layer-l+1 waves' HBM stores every step); callers wait for their LDS-DMA with a
// counted vmcnt themselves.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- block reductions ------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over a 256-thread block in a fixed order (deterministic); result valid in all threads.
template <typename T, int NT = 256>
__device__ __forceinline__ T block_sum(T v, T* scratch /* >= NT/64 */) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += scratch[i];
  return s;
}

}  // namespace pnp
