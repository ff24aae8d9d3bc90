// Probe: does v_mfma_f32_32x32x16_f16 keep fp16 subnormal A inputs (default kernel mode)?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
__global__ void k(float* out, float aval) {
  half8_t a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)aval; b[j] = (_Float16)1.0f; }
  floatx16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  if (threadIdx.x == 0) out[0] = acc[0];
}
int main() {
  float* d; hipMalloc(&d, 4);
  const float vals[] = {1e-5f, 3e-6f, 6.1e-5f, 1e-3f};
  for (float v : vals) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, v);
    float h; hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("a=%g (fp16 %g): mfma sum over k=16 -> %g (expect %g)\n", v, (float)(_Float16)v, h, 16.f * (float)(_Float16)v);
  }
  return 0;
}
