// Probe: device copy bandwidth of float4 streaming-copy variants (1 GiB each way, best of 10).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/copy_bw.hip -o tools/probes/copy_bw && ./tools/probes/copy_bw
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const f4* __restrict__ s, f4* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
    f4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + 256 * k < n) v[k] = NT ? __builtin_nontemporal_load(s + i + 256 * k) : s[i + 256 * k];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (i + 256 * k < n) {
        if (NT) __builtin_nontemporal_store(v[k], d + i + 256 * k);
        else d[i + 256 * k] = v[k];
      }
  }
}

template <int U, bool NT>
void run(const char* name, f4* a, f4* b, size_t n, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9f;
  for (int r = 0; r < 10; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((copy_k<U, NT>), dim3(blocks), dim3(256), 0, 0, a, b, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  printf("%-28s blocks %6d: %7.1f GB/s\n", name, blocks, 2.0 * n * 16 / (best * 1e-3) / 1e9);
}

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 16;
  f4 *a, *b;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes);
  hipMemset(a, 1, bytes);
  for (int blocks : {2048, 4096, 8192, 16384}) {
    run<4, false>("U4", a, b, n, blocks);
    run<4, true>("U4 nontemporal", a, b, n, blocks);
    run<8, false>("U8", a, b, n, blocks);
    run<2, false>("U2", a, b, n, blocks);
  }
  run<1, false>("U1 one pass", a, b, n, (int)((n + 255) / 256));
  return 0;
}
