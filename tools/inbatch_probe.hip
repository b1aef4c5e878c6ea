// Development probe for the fused in-batch softmax CE (tt_inbatch.hip): times
// tt_inbatch_softmax_xent at the C3 shape (B = 16384, E = 128) on relu(N(0,1))
// rows, so two builds of the kernel file can be compared on one box.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics \
//     -mllvm -amdgpu-mfma-vgpr-form -I include -I hm-retrieval-two-tower_amd/csrc \
//     tools/inbatch_probe.hip hm-retrieval-two-tower_amd/csrc/tt_api.cpp -o /tmp/probe
#include <hiprand/hiprand_kernel.h>

#include <cstdio>
#include <cstdlib>

#include "tt_inbatch.hip"

__global__ void fill(float* x, int64_t n, unsigned long long seed, float scale, int relu) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  hiprandStatePhilox4_32_10_t st;
  hiprand_init(seed, i, 0, &st);
  const float v = hiprand_normal(&st) * scale;
  x[i] = relu && v < 0.0f ? 0.0f : v;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 16384;
  const int dim = 128, reps = argc > 2 ? atoi(argv[2]) : 50;
  float *q, *c, *logq, *lse, *loss, *dq, *dc;
  hipMalloc(&q, n * dim * 4);
  hipMalloc(&c, n * dim * 4);
  hipMalloc(&dq, n * dim * 4);
  hipMalloc(&dc, n * dim * 4);
  hipMalloc(&logq, n * 4);
  hipMalloc(&lse, n * 4);
  hipMalloc(&loss, n * 4);
  fill<<<(n * dim + 255) / 256, 256>>>(q, n * dim, 1, 0.3f, 1);
  fill<<<(n * dim + 255) / 256, 256>>>(c, n * dim, 2, 0.3f, 1);
  fill<<<(n + 255) / 256, 256>>>(logq, n, 3, 1.0f, 0);
  const size_t wb = tt_inbatch_fused_workspace_size(n, dim);
  void* ws;
  hipMalloc(&ws, wb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 10; ++i)
    if (tt_inbatch_softmax_xent(q, dim, c, dim, n, dim, logq, lse, loss, dq, dc, ws, wb, nullptr))
      return printf("inbatch: %s\n", tt_last_error()), 1;
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) tt_inbatch_softmax_xent(q, dim, c, dim, n, dim, logq, lse, loss, dq, dc, ws, wb, nullptr);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  float l0;
  hipMemcpy(&l0, loss, 4, hipMemcpyDeviceToHost);
  printf("n=%lld: %.1f us per entry  (loss[0] %.6f)\n", (long long)n, ms * 1e3 / reps, l0);
  return 0;
}
