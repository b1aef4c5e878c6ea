// Development probe: times tt_inbatch_softmax_xent at B=16384, E=128 (C3) and
// the rows/cols ops separately, replayed from a hipGraph.  -DTT_INBATCH_* knobs.
#include <cstdio>
#include <vector>

#include "tt_inbatch.hip"

__global__ void fill(float* x, int64_t n, unsigned seed) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = ((h & 0xFFFF) / 65535.0f - 0.5f) * 0.2f;
  }
}

int main() {
  const int64_t n = 16384;
  const int dim = 128;
  float *q, *c, *logq, *lse, *loss, *dq, *dc;
  hipMalloc(&q, n * dim * 4); hipMalloc(&c, n * dim * 4); hipMalloc(&logq, n * 4);
  hipMalloc(&lse, n * 4); hipMalloc(&loss, n * 4); hipMalloc(&dq, n * dim * 4); hipMalloc(&dc, n * dim * 4);
  fill<<<(n * dim + 255) / 256, 256>>>(q, n * dim, 1);
  fill<<<(n * dim + 255) / 256, 256>>>(c, n * dim, 2);
  fill<<<(n + 255) / 256, 256>>>(logq, n, 3);
  const size_t wb = tt_inbatch_fused_workspace_size(n, dim);
  void* ws; hipMalloc(&ws, wb);
  hipStream_t st; hipStreamCreate(&st);
  for (int i = 0; i < 3; ++i)
    if (tt_inbatch_softmax_xent(q, dim, c, dim, n, dim, logq, lse, loss, dq, dc, ws, wb, st)) return printf("err %s\n", tt_last_error()), 1;
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 20; ++i) tt_inbatch_softmax_xent(q, dim, c, dim, n, dim, logq, lse, loss, dq, dc, ws, wb, st);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, st); hipStreamSynchronize(st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, st); hipGraphLaunch(ge, st); hipEventRecord(e1, st); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double fl = 8.0 * n * n * 128;
  std::vector<float> h(4); hipMemcpy(h.data(), loss, 16, hipMemcpyDeviceToHost);
  printf("target=%d: fused %.1f us  %.0f TF/s  loss[0]=%.6f\n", TT_INBATCH_WG_TARGET, ms / 20 * 1e3, fl / (ms / 20 * 1e-3) / 1e12, h[0]);
  return 0;
}
