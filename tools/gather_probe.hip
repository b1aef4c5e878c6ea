// Development probe: times tt_gather_multi on the C3 main.py schema shape
// (query 128+2+128 cols, candidate 128+4+4+8+32+4+16+4 cols, B=16384) with
// Zipf/uniform ids, replayed from a hipGraph.  Built with -DTT_GATHER_* knobs.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "tt_gather.hip"

int main() {
  const int B = 16384;
  struct T { int rows, dim; double zipf; };
  std::vector<T> q = {{1371981, 128, 1.6}, {5, 2, 0}, {352000, 128, 0}};
  std::vector<T> c = {{105543, 128, 2.1}, {132, 4, 0}, {132, 4, 0}, {51, 8, 0}, {251, 32, 0}, {11, 4, 0}, {57, 16, 0}, {22, 4, 0}};
  std::mt19937_64 rng(1);
  auto make = [&](std::vector<T>& ts, std::vector<tt_gather_segment>& segs, int& width, double& bytes) {
    width = 0;
    for (auto& t : ts) {
      float* tab; int32_t* ids;
      hipMalloc(&tab, size_t(t.rows) * t.dim * 4);
      hipMemset(tab, 0, size_t(t.rows) * t.dim * 4);
      std::vector<int32_t> h(B);
      for (int i = 0; i < B; ++i) {
        if (t.zipf > 0) { double u = std::uniform_real_distribution<double>(0, 1)(rng); h[i] = int(std::fmod(std::pow(1 - u, -1.0 / (t.zipf - 1)), t.rows - 1)) + 1; }
        else h[i] = int(rng() % (t.rows - 1)) + 1;
      }
      hipMalloc(&ids, B * 4);
      hipMemcpy(ids, h.data(), B * 4, hipMemcpyHostToDevice);
      segs.push_back({tab, ids, t.rows, t.dim, width});
      width += t.dim;
      bytes += double(B) * (4 + 8.0 * t.dim);
    }
  };
  std::vector<tt_gather_segment> sq, sc;
  int wq, wc; double bytes = 0;
  make(q, sq, wq, bytes); make(c, sc, wc, bytes);
  const int ldq = (wq + 3) / 4 * 4, ldc = (wc + 3) / 4 * 4;
  float *oq, *oc;
  hipMalloc(&oq, size_t(B) * ldq * 4); hipMalloc(&oc, size_t(B) * ldc * 4);
  tt_gather_call calls[2] = {{sq.data(), (int)sq.size(), oq, ldq}, {sc.data(), (int)sc.size(), oc, ldc}};
  hipStream_t st; hipStreamCreate(&st);
  for (int i = 0; i < 3; ++i) tt_gather_multi(calls, 2, B, st);
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 100; ++i) tt_gather_multi(calls, 2, B, st);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, st); hipStreamSynchronize(st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, st); hipGraphLaunch(ge, st); hipEventRecord(e1, st); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("iters=%d threads=%d: %.2f us/launch  %.0f GB/s (%.1f MB)\n", TT_GATHER_ITERS, TT_GATHER_THREADS, ms * 10, bytes / (ms / 100 * 1e-3) / 1e9, bytes / 1e6);
  return 0;
}
