// Development probe for the brute-force index kernels: builds tt_index.hip
// with its probe hooks and times search on relu(N(0,1)) data of the C4 shape.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics \
//     -I include -I hm-retrieval-two-tower_amd/csrc [-DTT_INDEX_STATS] [-DTT_INDEX_NOINSERT (screen keeps nothing)] \
//     tools/index_probe.hip hm-retrieval-two-tower_amd/csrc/tt_api.cpp -o /tmp/probe
#include <hiprand/hiprand_kernel.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tt_index.hip"

__global__ void fill_relu(float* x, int64_t n, unsigned long long seed, int zero_every, int dim) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  hiprandStatePhilox4_32_10_t st;
  hiprand_init(seed, i, 0, &st);
  const float v = hiprand_normal(&st);
  x[i] = (zero_every > 0 && (i / dim) % zero_every == 0) ? 0.0f : (v > 0.0f ? v : 0.0f);
}

int main(int argc, char** argv) {
  const int64_t nq = argc > 1 ? atoll(argv[1]) : 65536;
  const int64_t nc = argc > 2 ? atoll(argv[2]) : 105542;
  const int dim = 128, k = argc > 3 ? atoi(argv[3]) : 100;
  float *C, *Q, *S;
  int32_t* I;
  hipMalloc(&C, nc * dim * 4);
  hipMalloc(&Q, nq * dim * 4);
  hipMalloc(&S, nq * k * 4);
  hipMalloc(&I, nq * k * 4);
  fill_relu<<<(nc * dim + 255) / 256, 256>>>(C, nc * dim, 1, 0, dim);
  fill_relu<<<(nq * dim + 255) / 256, 256>>>(Q, nq * dim, 2, 100, dim);
  const size_t ib = tt_bruteforce_index_bytes(nc, dim);
  const size_t wb = tt_bruteforce_workspace_size(nq, nc, dim, k);
  void *idx, *ws;
  hipMalloc(&idx, ib);
  hipMalloc(&ws, wb);
  if (tt_bruteforce_build(C, dim, nc, dim, idx, ib, nullptr)) return printf("build: %s\n", tt_last_error()), 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
#ifdef TT_INDEX_STATS
    unsigned long long z[4] = {0, 0, 0, 0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_index_stats), z, sizeof(z));
#endif
    hipEventRecord(e0);
    if (tt_bruteforce_search(idx, C, dim, nc, dim, Q, dim, nq, k, 0, S, I, ws, wb, nullptr))
      return printf("search: %s\n", tt_last_error()), 1;
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("nq=%lld nc=%lld: %.3f ms  %.1f TFLOP/s  %.2f MQPS\n", (long long)nq, (long long)nc, ms,
           2.0 * nq * nc * dim / ms / 1e9, nq / ms / 1e3);
#ifdef TT_INDEX_STATS
    unsigned long long st[4];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_index_stats), sizeof(st));
    printf("  list entries/query %.1f  fallbacks %llu  cut entries/query %.1f\n", double(st[0]) / nq, st[1],
           double(st[2]) / nq);
#endif
  }
  std::vector<int32_t> hi(k);
  hipMemcpy(hi.data(), I + 1 * k, k * 4, hipMemcpyDeviceToHost);
  printf("q1 top5: %d %d %d %d %d\n", hi[0], hi[1], hi[2], hi[3], hi[4]);
  return 0;
}
