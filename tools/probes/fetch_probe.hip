// Probe: calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the prox
// passes use.  Streams over a 2 GiB buffer (8x the 256 MiB Infinity Cache,
// so no re-read is absorbed on die) with 4, 8 and 16 B per lane reads, then writes it with 4 and
// 16 B per lane stores.  Each kernel's algorithmic bytes are 2 GiB; compare with the counters:
//   hipcc --offload-arch=gfx950 -O3 tools/probes/fetch_probe.hip -o tools/probes/fetch_probe
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -- tools/probes/fetch_probe
//   rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir> -- tools/probes/fetch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ __launch_bounds__(256) void read_k(const T* __restrict__ s, size_t n, float* __restrict__ sink) {
  float acc = 0.f;
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const T v = s[i];
    const float* f = reinterpret_cast<const float*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc += f[k];
  }
  sink[(size_t)blockIdx.x * 256 + threadIdx.x] = acc;   // 4 MiB of sink writes, not counted as reads
}

template <typename T>
__global__ __launch_bounds__(256) void write_k(T* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256;
  T v;
  float* f = reinterpret_cast<float*>(&v);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); ++k) f[k] = 1.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) d[i] = v;
}

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename T>
void time_it(const char* name, void (*launch)(void*, size_t), void* p, size_t bytes) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  launch(p, bytes / sizeof(T));
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-12s %6.3f ms  %7.1f GB/s (%zu bytes)\n", name, ms, bytes / (ms * 1e-3) / 1e9, bytes);
}

static float* g_sink;
constexpr int kBlocks = 4096;

int main() {
  const size_t bytes = 2ull << 30;
  void* a;
  hipMalloc(&a, bytes);
  hipMalloc(&g_sink, (size_t)kBlocks * 256 * sizeof(float));
  hipMemset(a, 0, bytes);
  hipDeviceSynchronize();
  time_it<float>("read_b32", [](void* p, size_t n) {
    hipLaunchKernelGGL(read_k<float>, dim3(kBlocks), dim3(256), 0, 0, (const float*)p, n, g_sink); }, a, bytes);
  time_it<f2>("read_b64", [](void* p, size_t n) {
    hipLaunchKernelGGL(read_k<f2>, dim3(kBlocks), dim3(256), 0, 0, (const f2*)p, n, g_sink); }, a, bytes);
  time_it<f4>("read_b128", [](void* p, size_t n) {
    hipLaunchKernelGGL(read_k<f4>, dim3(kBlocks), dim3(256), 0, 0, (const f4*)p, n, g_sink); }, a, bytes);
  time_it<float>("write_b32", [](void* p, size_t n) {
    hipLaunchKernelGGL(write_k<float>, dim3(kBlocks), dim3(256), 0, 0, (float*)p, n); }, a, bytes);
  time_it<f4>("write_b128", [](void* p, size_t n) {
    hipLaunchKernelGGL(write_k<f4>, dim3(kBlocks), dim3(256), 0, 0, (f4*)p, n); }, a, bytes);
  hipDeviceSynchronize();
  return 0;
}
