// Development check: rows pass lse vs a host fp64 computation, per row, at a
// few shapes; prints the worst rows so layout bugs show their pattern.
#include <cmath>
#include <cstdio>
#include <vector>

#include "tt_inbatch.hip"

static float frand(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return ((s >> 8) & 0xFFFF) / 65535.0f;
}

int run(int64_t n, int dim, bool logq_on) {
  std::vector<float> q(n * dim), c(n * dim), lq(n);
  unsigned s = 12345u + (unsigned)n;
  for (auto& x : q) x = std::max(0.0f, (frand(s) - 0.3f));
  for (auto& x : c) x = std::max(0.0f, (frand(s) - 0.3f));
  for (auto& x : lq) x = logf(1e-6f + frand(s) * 1e-2f);
  float *dq_, *dc_, *dl, *dlse, *dloss, *ddq;
  hipMalloc(&dq_, n * dim * 4); hipMalloc(&dc_, n * dim * 4); hipMalloc(&dl, n * 4);
  hipMalloc(&dlse, n * 4); hipMalloc(&dloss, n * 4); hipMalloc(&ddq, n * dim * 4);
  hipMemcpy(dq_, q.data(), n * dim * 4, hipMemcpyHostToDevice);
  hipMemcpy(dc_, c.data(), n * dim * 4, hipMemcpyHostToDevice);
  hipMemcpy(dl, lq.data(), n * 4, hipMemcpyHostToDevice);
  const size_t wb = tt_inbatch_workspace_size(n, n, dim);
  void* ws; hipMalloc(&ws, wb);
  if (tt_inbatch_xent_rows(dq_, dim, n, dc_, dim, n, dim, logq_on ? dl : nullptr, 0, dlse, dloss, ddq, ws, wb, 0))
    return printf("err %s\n", tt_last_error()), 1;
  hipDeviceSynchronize();
  std::vector<float> lse(n);
  hipMemcpy(lse.data(), dlse, n * 4, hipMemcpyDeviceToHost);
  double worst = 0; int64_t wi = -1; int bad = 0;
  for (int64_t i = 0; i < n; ++i) {
    double m = -1e300;
    std::vector<double> sc(n);
    for (int64_t j = 0; j < n; ++j) {
      double d = 0;
      for (int e = 0; e < dim; ++e) d += (double)q[i * dim + e] * c[j * dim + e];
      if (logq_on) d -= lq[j];
      sc[j] = d; m = std::max(m, d);
    }
    double l = 0;
    for (int64_t j = 0; j < n; ++j) l += exp(sc[j] - m);
    const double ref = m + log(l);
    const double err = fabs(lse[i] - ref);
    if (err > 1e-2 * std::max(1.0, fabs(ref))) { if (bad < 6) printf("  row %lld got %.5f ref %.5f\n", (long long)i, lse[i], ref); ++bad; }
    if (err > worst) { worst = err; wi = i; }
  }
  printf("n=%lld dim=%d logq=%d: worst |dlse| %.3g at row %lld, %d bad rows\n", (long long)n, dim, (int)logq_on, worst, (long long)wi, bad);
  hipFree(dq_); hipFree(dc_); hipFree(dl); hipFree(dlse); hipFree(dloss); hipFree(ddq); hipFree(ws);
  return 0;
}

int main() {
  run(64, 16, false);
  run(64, 16, true);
  run(200, 64, true);
  run(1024, 128, true);
  run(3000, 128, true);
  return 0;
}
