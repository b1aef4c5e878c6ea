// K14 recall hits and the per-shard top-k merge; the loss reduction.
//
// tt_recall_hits restates IndexRecall.__call__
// (/root/reference/pkg/modelling/metrics/index_recall.py:52-58):
//   hits[k] += sum(equal(true_ids[B,1], candidates[:, :k]))
// (every equal position counts, as the reference's reduce_sum does).
//
// tt_topk_merge merges sorted per-shard top-k lists (score desc, index asc)
// into the global top-k with the same order as tf.math.top_k over the
// concatenated candidates (brute_force.py:81): one wave per query, a k-way
// head merge with a wave-wide argmax over the list heads per output slot.
#include "tt_common.h"

namespace tt {
namespace {

constexpr int kMaxKs = 16;

// loss = scale * sum(x[0..n)): one workgroup, thread t sums t, t+1024, ...
// in order, then a fixed-shape LDS tree (deterministic; the reference's
// reduce_sum over the per-example CE, runner.py:78-83 with reduction SUM).
__global__ void __launch_bounds__(1024) sum_kernel(const float* __restrict__ x, int64_t n, float scale,
                                                   float* __restrict__ out) {
  __shared__ float red[1024];
  float acc = 0.0f;
  int64_t i = threadIdx.x;
  for (; i + 3 * 1024 < n; i += 4 * 1024) {
    const float a = x[i], b = x[i + 1024], c = x[i + 2048], d = x[i + 3072];
    acc = ((acc + a) + b) + c;
    acc = acc + d;
  }
  for (; i < n; i += 1024) acc += x[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0] * scale;
}

struct RecallArgs {
  const int32_t* true_ids;
  const int32_t* cand;
  int64_t batch;
  int32_t k_total;
  int32_t num_ks;
  int32_t ks[kMaxKs];
  unsigned long long* hits;
};

__global__ void __launch_bounds__(256) recall_hits_kernel(const RecallArgs a) {
  __shared__ unsigned long long part[kMaxKs];
  if (threadIdx.x < kMaxKs) part[threadIdx.x] = 0;
  __syncthreads();
  const int64_t b = blockIdx.x * 256ll + threadIdx.x;
  unsigned cnt[kMaxKs];
#pragma unroll
  for (int t = 0; t < kMaxKs; ++t) cnt[t] = 0;
  if (b < a.batch) {
    const int32_t want = a.true_ids[b];
    const int32_t* row = a.cand + b * a.k_total;
    for (int j = 0; j < a.k_total; ++j) {
      if (row[j] == want) {
#pragma unroll
        for (int t = 0; t < kMaxKs; ++t)
          if (t < a.num_ks && j < a.ks[t]) ++cnt[t];
      }
    }
  }
#pragma unroll
  for (int t = 0; t < kMaxKs; ++t) {
    if (t < a.num_ks) {
      unsigned long long s = static_cast<unsigned long long>(wave_sum_i32(static_cast<int>(cnt[t])));
      if (lane_id() == 0 && s) atomicAdd(&part[t], s);
    }
  }
  __syncthreads();
  if (threadIdx.x < a.num_ks && part[threadIdx.x]) atomicAdd(&a.hits[threadIdx.x], part[threadIdx.x]);
}

// Composite ordering key: larger = better (higher score, then lower index).
__device__ __forceinline__ unsigned long long merge_key(float s, int32_t idx) {
  return (static_cast<unsigned long long>(float_order_key(s)) << 32) |
         static_cast<unsigned long long>(0xFFFFFFFFu - static_cast<unsigned>(idx));
}

__global__ void __launch_bounds__(256) topk_merge_kernel(const float* __restrict__ scores,
                                                         const int32_t* __restrict__ idx, int num_lists,
                                                         int64_t n_queries, int k_in, int k_out,
                                                         float* __restrict__ out_s, int32_t* __restrict__ out_i) {
  const int64_t q = blockIdx.x * 4ll + threadIdx.x / kWave;
  if (q >= n_queries) return;
  const int lane = lane_id();
  const int64_t list_stride = n_queries * static_cast<int64_t>(k_in);
  int ptr = 0;  // head position of list `lane`
  const bool owner = lane < num_lists;
  const float* ls = scores + lane * list_stride + q * k_in;
  const int32_t* li = idx + lane * list_stride + q * k_in;
  unsigned long long head = 0;
  float hs = 0.f;
  int32_t hi = 0;
  auto load_head = [&]() {
    if (owner && ptr < k_in) {
      hs = ls[ptr];
      hi = li[ptr];
      head = merge_key(hs, hi);
    } else {
      head = 0;  // exhausted
    }
  };
  load_head();
  for (int o = 0; o < k_out; ++o) {
    unsigned long long best = head;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const unsigned long long other = __shfl_xor(best, m, kWave);
      best = other > best ? other : best;
    }
    if (head == best && head != 0) {  // keys are unique per query (distinct indices)
      out_s[q * k_out + o] = hs;
      out_i[q * k_out + o] = hi;
      ++ptr;
      load_head();
    }
  }
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" int tt_recall_hits(const int32_t* true_ids, const int32_t* cand_ids, int64_t batch, int32_t k_total,
                              const int32_t* ks_host, int32_t num_ks, int64_t* hits, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(num_ks >= 1 && num_ks <= kMaxKs, "tt_recall_hits: num_ks=%d outside [1,%d]", num_ks, kMaxKs);
  TT_REQUIRE(ks_host && hits, "tt_recall_hits: NULL ks/hits");
  TT_REQUIRE(batch >= 0 && k_total >= 1, "tt_recall_hits: bad batch/k_total");
  if (batch == 0) return TT_OK;
  TT_REQUIRE(true_ids && cand_ids, "tt_recall_hits: NULL ids");
  RecallArgs a{};
  a.true_ids = true_ids;
  a.cand = cand_ids;
  a.batch = batch;
  a.k_total = k_total;
  a.num_ks = num_ks;
  for (int t = 0; t < num_ks; ++t) {
    TT_REQUIRE(ks_host[t] >= 0, "tt_recall_hits: negative k");
    a.ks[t] = ks_host[t] < k_total ? ks_host[t] : k_total;
  }
  a.hits = reinterpret_cast<unsigned long long*>(hits);
  hipLaunchKernelGGL(recall_hits_kernel, dim3(ceil_div(batch, 256)), dim3(256), 0, to_stream(stream), a);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_sum(const float* x, int64_t n, float scale, float* out, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(n >= 0 && out != nullptr && (n == 0 || x != nullptr), "tt_sum: bad arguments");
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, to_stream(stream), x, n, scale, out);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_topk_merge(const float* scores, const int32_t* idx, int32_t num_lists, int64_t n_queries,
                             int32_t k_in, int32_t k_out, float* out_scores, int32_t* out_idx,
                             tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(num_lists >= 1 && num_lists <= kWave, "tt_topk_merge: num_lists=%d outside [1,64]", num_lists);
  TT_REQUIRE(k_in >= 1 && k_out >= 1 && k_out <= static_cast<int64_t>(num_lists) * k_in,
             "tt_topk_merge: need 1 <= k_out <= num_lists*k_in");
  TT_REQUIRE(n_queries >= 0, "tt_topk_merge: negative n_queries");
  if (n_queries == 0) return TT_OK;
  TT_REQUIRE(scores && idx && out_scores && out_idx, "tt_topk_merge: NULL pointer");
  hipLaunchKernelGGL(topk_merge_kernel, dim3(ceil_div(n_queries, 4)), dim3(256), 0, to_stream(stream), scores, idx,
                     num_lists, n_queries, k_in, k_out, out_scores, out_idx);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
