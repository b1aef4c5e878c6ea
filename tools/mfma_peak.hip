// Calibration: back-to-back v_mfma_f32_32x32x16_bf16 from registers, 8 waves
// per CU (2 per SIMD), every CU busy: the achievable dense bf16 rate.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_peak.hip -o tools/pbin/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void __launch_bounds__(512) k(float* out, int iters) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(i * 0.5f); }
  f32x16 c0 = {}, c1 = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    }
  }
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
  if (s == 1.2345f) out[threadIdx.x] = s;
}
int main() {
  float* o; (void)hipMalloc(&o, 4096);
  const int iters = 4000, grid = 256 * 4;
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, 0, o, iters);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double fl = 2.0 * 32 * 32 * 16 * 16.0 * iters * 8.0 * grid;
    printf("mfma peak probe: %.3f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
  }
  return 0;
}
