// K4 glue: the non-GEMM parts of the tower MLP backward (Dense + ReLU layers,
// /root/reference/pkg/modelling/models/tower.py:45,48; TF computes them as
// ReluGrad and BiasAddGrad beside the MatMul gradients).
//
//   tt_relu_bias_grad: gout = (act > 0) * s * gin and db = column sums of
//     gout, in one pass over [rows, cols] (s = *gscale, the loss's incoming
//     gradient, so the loss backward needs no separate scaling pass).
//     Column sums are deterministic: 64-row blocks summed in row order, the
//     block partials in 16 consecutive chunks (each in order), then the 16
//     chunk sums in order.
//   tt_sum_slices: out = sum over S slices of [n] (slice order) — the split-K
//     reduction of a weight gradient computed as S batched partial GEMMs.
// Both are HBM streams: one read of every input byte, one write of every
// output byte.
#include "tt_common.h"

namespace tt {
namespace {

constexpr int kRowsPerBlock = 64;

// One block: 64 rows x all columns; thread t owns columns t, t+256, ...
// (coalesced row reads).  part[blk][col] = sum of the block's masked rows.
__global__ void __launch_bounds__(256) relu_bias_grad_kernel(const float* __restrict__ gin, int64_t ldg,
                                                             const float* __restrict__ gscale,
                                                             const float* __restrict__ act, int64_t lda,
                                                             int64_t rows, int cols, float* gout, int64_t ldo,
                                                             float* __restrict__ part) {
  const float s = gscale ? *gscale : 1.0f;
  const int64_t r0 = blockIdx.x * static_cast<int64_t>(kRowsPerBlock);
  const int nr = static_cast<int>(rows - r0 < kRowsPerBlock ? rows - r0 : kRowsPerBlock);
  for (int c = threadIdx.x; c < cols; c += 256) {
    float acc = 0.0f;
    int r = 0;
    for (; r + 8 <= nr; r += 8) {
      float g[8], a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        g[u] = gin[(r0 + r + u) * ldg + c];
        a[u] = act[(r0 + r + u) * lda + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float v = a[u] > 0.0f ? g[u] * s : 0.0f;
        gout[(r0 + r + u) * ldo + c] = v;
        acc += v;
      }
    }
    for (; r < nr; ++r) {
      const float v = act[(r0 + r) * lda + c] > 0.0f ? gin[(r0 + r) * ldg + c] * s : 0.0f;
      gout[(r0 + r) * ldo + c] = v;
      acc += v;
    }
    part[blockIdx.x * static_cast<int64_t>(cols) + c] = acc;
  }
}

// db[c] from the block partials part[nblk][cols]: 16 chunks of consecutive
// partials summed in order by 16 threads per column, then the 16 chunk sums
// in order (a fixed, deterministic order with 16 loads in flight per thread).
__global__ void __launch_bounds__(1024) column_total_kernel(const float* __restrict__ part, int nblk, int cols,
                                                            float* __restrict__ db) {
  __shared__ float red[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int i = threadIdx.x >> 6;
  const int chunk = (nblk + 15) / 16;
  const int b0 = i * chunk, b1 = min(b0 + chunk, nblk);
  float acc = 0.0f;
  if (c < cols)
    for (int bb = b0; bb < b1; bb += 16) {  // 16 loads in flight (index clamped), added in order
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = part[static_cast<int64_t>(min(bb + u, b1 - 1)) * cols + c];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (bb + u < b1) acc += v[u];
    }
  red[i][threadIdx.x & 63] = acc;
  __syncthreads();
  if (i == 0 && c < cols) {
    float t = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][threadIdx.x];
    db[c] = t;
  }
}

// out[i] = sum_{s < S} parts[s * n + i], slices in order.
__global__ void __launch_bounds__(256) sum_slices_kernel(const float* __restrict__ parts, int nslices, int64_t n,
                                                         float* __restrict__ out) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    float acc = 0.0f;
    int s = 0;
    for (; s + 8 <= nslices; s += 8) {  // 8 loads in flight, added in slice order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = parts[(s + u) * n + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; s < nslices; ++s) acc += parts[s * n + i];
    out[i] = acc;
  }
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" size_t tt_relu_bias_grad_workspace_size(int64_t rows, int32_t cols) {
  if (rows < 0 || cols < 1) return 0;
  return static_cast<size_t>(ceil_div(rows > 0 ? rows : 1, kRowsPerBlock)) * cols * sizeof(float);
}

extern "C" int tt_relu_bias_grad(const float* gin, int64_t ldg, const float* gscale, const float* act, int64_t lda,
                                 int64_t rows, int32_t cols, float* gout, int64_t ldo, float* db, void* workspace,
                                 size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(rows >= 0 && cols >= 1, "tt_relu_bias_grad: bad shape %lld x %d", static_cast<long long>(rows), cols);
  TT_REQUIRE(db != nullptr, "tt_relu_bias_grad: NULL db");
  TT_REQUIRE(rows == 0 || (gin && act && gout), "tt_relu_bias_grad: NULL operand");
  TT_REQUIRE(ldg >= cols && lda >= cols && ldo >= cols, "tt_relu_bias_grad: leading dimension < cols");
  hipStream_t st = to_stream(stream);
  if (rows == 0) {
    TT_CHECK_HIP(hipMemsetAsync(db, 0, cols * sizeof(float), st));
    return TT_OK;
  }
  const size_t need = tt_relu_bias_grad_workspace_size(rows, cols);
  if (!workspace || workspace_bytes < need)
    return fail(TT_ERR_WORKSPACE, "tt_relu_bias_grad: workspace %zu < required %zu", workspace_bytes, need);
  const int64_t nblk = ceil_div(rows, kRowsPerBlock);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(relu_bias_grad_kernel, dim3(static_cast<unsigned>(nblk)), dim3(256), 0, st, gin, ldg, gscale,
                     act, lda, rows, cols, gout, ldo, part);
  TT_CHECK_LAUNCH();
  hipLaunchKernelGGL(column_total_kernel, dim3(static_cast<unsigned>(ceil_div(cols, 64))), dim3(1024), 0, st, part,
                     static_cast<int>(nblk), cols, db);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_sum_slices(const float* parts, int32_t nslices, int64_t n, float* out, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(nslices >= 1 && n >= 0, "tt_sum_slices: bad shape");
  TT_REQUIRE(n == 0 || (parts && out), "tt_sum_slices: NULL pointer");
  if (n == 0) return TT_OK;
  int64_t blocks = ceil_div(n, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(sum_slices_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, to_stream(stream), parts,
                     nslices, n, out);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
