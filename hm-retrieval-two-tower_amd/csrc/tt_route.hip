// Request routing for row-sharded embedding tables.
//
// The reference has no multi-GPU path; this is the exchange step the
// data-parallel train step needs once the large tables are row-sharded
// (global row r on rank r % world).  Per step each rank turns its lookups
// into one deduplicated request list, bucketed by owner:
//
//   tt_route_requests  lookups (table tag, ids [B]) ->
//       send [R, 2] = (global row, tag), owner-major; inside an owner by tag,
//                     then row ascending, an invalid id (outside the table)
//                     as row -1 first and owned by rank world-1
//       counts [world] (int64) requests per owner, R = their sum
//       idx [L, B]    position of each lookup's request in `send`
//   tt_route_owner     the requests an owner received ->
//       tags [n], local rows [n] (-1 for invalid), and per table the local
//       rows of its own requests (-1 elsewhere) for the sparse update.
//
// MI355X shape: one launch builds 64-bit keys (owner, tag, row+1) with the
// lookup index as value, one rocPRIM radix sort over the key bits in use,
// then two coalesced passes over the sorted keys (one key per thread): block
// head counts, and per block its prefix (a wave sums the earlier blocks'
// counts), an in-block scan and the send / idx / per-owner count writes.
// (A single-workgroup scan with a contiguous run per thread took 166 us at
// 49k lookups: every load instruction touched 64 lines and each thread's
// loop was a chain of dependent misses.)
#include <algorithm>
#include <rocprim/device/device_radix_sort.hpp>

#include "tt_common.h"

namespace tt {
namespace {

constexpr int kMaxRouteLookups = 32;
constexpr int kMaxWorld = 1024;
constexpr int kScanThreads = 1024;

struct RouteLookup {
  const int32_t* ids;
  int64_t num_rows;
  int32_t tag;
};

struct RouteArgs {
  RouteLookup lk[kMaxRouteLookups];
  int32_t num;
  int64_t batch;
  int32_t world;
  int32_t num_tags;
  int32_t id_bits;
  unsigned long long* keys_in;
  uint32_t* vals_in;
};

__global__ void __launch_bounds__(256) route_keys_kernel(const RouteArgs a) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  const int64_t total = a.batch * a.num;
  if (i >= total) return;
  const int l = static_cast<int>(i / a.batch);
  const int64_t b = i - l * a.batch;
  const RouteLookup& L = a.lk[l];
  const int32_t r = L.ids[b];
  const bool ok = r >= 0 && r < L.num_rows;
  const unsigned long long owner = ok ? static_cast<unsigned long long>(r % a.world) : a.world - 1;
  const unsigned long long rowp1 = ok ? static_cast<unsigned long long>(r) + 1ull : 0ull;
  a.keys_in[i] = ((owner * a.num_tags + static_cast<unsigned long long>(L.tag)) << a.id_bits) | rowp1;
  a.vals_in[i] = static_cast<uint32_t>(i);
}

// Heads of the sorted key runs = distinct requests.  Pass 1: per block of
// kScanThreads consecutive sorted keys (one per thread, coalesced), the
// number of heads.  Pass 2: each block adds up the counts of the blocks
// before it (wave-parallel), scans its own heads and writes send / idx and
// its per-owner counts (LDS, then one atomic per owner per block into the
// zeroed counts); the last block writes the request total.
__global__ void __launch_bounds__(kScanThreads) route_heads_kernel(const unsigned long long* keys, int64_t total,
                                                                   int32_t* block_heads, long long* counts,
                                                                   int32_t world) {
  // the per-owner counts route_write_kernel adds into are zeroed here, by a
  // kernel, not by a captured hipMemsetAsync: with the memset node (and the
  // counts' block recycled inside the step's graph) the overflow word picked
  // up garbage in 2 of 2 graphed runs; a standalone probe of memset nodes
  // (tools/graph_replay_overlap_probe.py) stayed ordered, so that cause is
  // not pinned down, and the kernel-zeroed version has run clean since
  if (blockIdx.x == 0)
    for (int o = threadIdx.x; o < world; o += kScanThreads) counts[o] = 0;
  __shared__ int wsum[kScanThreads / kWave];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kScanThreads + threadIdx.x;
  const int head = (i < total && (i == 0 || keys[i] != keys[i - 1])) ? 1 : 0;
  const int c = __popcll(__ballot(head));
  if (lane_id() == 0) wsum[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int k = 0; k < kScanThreads / kWave; ++k) t += wsum[k];
    block_heads[blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(kScanThreads) route_write_kernel(const unsigned long long* keys, const uint32_t* vals,
                                                                   int64_t total, int32_t world, int32_t num_tags,
                                                                   int32_t id_bits, const int32_t* block_heads,
                                                                   int32_t* send, int32_t* idx, long long* counts,
                                                                   int32_t* num_requests) {
  __shared__ int wsum[kScanThreads / kWave + 1];
  __shared__ int cnt[kMaxWorld];
  __shared__ int base_s;
  for (int o = threadIdx.x; o < world; o += kScanThreads) cnt[o] = 0;
  const int lane = lane_id(), w = threadIdx.x / kWave;
  if (w == 0) {  // requests in the blocks before this one
    int t = 0;
    for (int b = lane; b < static_cast<int>(blockIdx.x); b += kWave) t += block_heads[b];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m, kWave);
    if (lane == 0) base_s = t;
  }
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kScanThreads + threadIdx.x;
  const unsigned long long k = i < total ? keys[i] : 0ull;
  const int head = (i < total && (i == 0 || k != keys[i - 1])) ? 1 : 0;
  const uint64_t m = __ballot(head);
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int incl = __popcll(m & (lt | (1ull << lane)));  // heads up to and including this lane
  if (lane == kWave - 1) wsum[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int q = 0; q < kScanThreads / kWave; ++q) {
      const int t = wsum[q];
      wsum[q] = run;
      run += t;
    }
    wsum[kScanThreads / kWave] = run;
  }
  __syncthreads();
  if (i < total) {
    const int u = base_s + wsum[w] + incl - 1;  // request index of this key's run
    if (head) {
      const unsigned long long mask = (1ull << id_bits) - 1ull;
      const unsigned long long ot = k >> id_bits;
      send[2 * static_cast<int64_t>(u)] = static_cast<int32_t>(static_cast<long long>(k & mask) - 1);
      send[2 * static_cast<int64_t>(u) + 1] = static_cast<int32_t>(ot % num_tags);
      atomicAdd(&cnt[static_cast<int>(ot / num_tags)], 1);
    }
    idx[vals[i]] = u;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < world; o += kScanThreads)
    if (cnt[o]) atomicAdd(reinterpret_cast<unsigned long long*>(counts + o), static_cast<unsigned long long>(cnt[o]));
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *num_requests = base_s + wsum[kScanThreads / kWave];
}

__global__ void __launch_bounds__(256) route_owner_kernel(const int32_t* recv, int64_t n, int32_t world,
                                                          int32_t num_tags, int32_t* tags, int32_t* rows,
                                                          int32_t* table_ids) {
  const int64_t j = blockIdx.x * 256ll + threadIdx.x;
  if (j >= n) return;
  const int32_t gid = recv[2 * j], tag = recv[2 * j + 1];
  const int32_t row = gid >= 0 ? gid / world : -1;
  tags[j] = tag;
  rows[j] = row;
  for (int t = 0; t < num_tags; ++t) table_ids[t * n + j] = (t == tag) ? row : -1;
}

// Fixed per-owner slots (tt_route_pad): every block computes the owners'
// start offsets in LDS from the device counts (world <= kMaxWorld), then one
// thread per padded slot copies its request (or writes the (-1, -1) filler)
// and one thread per lookup rewrites its request index to the padded slot.
__global__ void __launch_bounds__(256) route_pad_kernel(const int32_t* send, const long long* counts,
                                                        const int32_t* idx, int64_t num_lookups, int32_t world,
                                                        int64_t cap, int32_t* send_padded, int32_t* idx_padded,
                                                        int32_t* overflow) {
  __shared__ long long start[kMaxWorld + 1];
  if (threadIdx.x == 0) {
    long long run = 0;
    for (int o = 0; o < world; ++o) {
      start[o] = run;
      run += counts[o];
    }
    start[world] = run;
  }
  __syncthreads();
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int64_t slots = static_cast<int64_t>(world) * cap;
  if (t < slots) {
    const int o = static_cast<int>(t / cap);
    const int64_t j = t - static_cast<int64_t>(o) * cap;
    const long long n = start[o + 1] - start[o];
    int32_t row = -1, tag = -1;
    if (j < n) {
      const long long u = start[o] + j;
      row = send[2 * u];
      tag = send[2 * u + 1];
    }
    send_padded[2 * t] = row;
    send_padded[2 * t + 1] = tag;
    if (j == cap - 1 && n > cap && overflow) atomicAdd(overflow, static_cast<int32_t>(n - cap));
  }
  if (t < num_lookups) {
    const long long u = idx[t];
    int lo = 0, hi = world - 1;  // the owner o with start[o] <= u < start[o + 1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (start[mid] <= u) lo = mid; else hi = mid - 1;
    }
    long long j = u - start[lo];
    if (j >= cap) j = cap - 1;  // dropped request (counted in *overflow): a defined slot
    idx_padded[t] = static_cast<int32_t>(static_cast<int64_t>(lo) * cap + j);
  }
}

int bits_for(int64_t x) {  // bits needed to represent values in [0, x]
  int b = 1;
  while ((int64_t(1) << b) <= x) ++b;
  return b;
}

struct RoutePlan {
  int64_t total;
  int id_bits;
  int end_bit;
  size_t sort_bytes;
};

int plan_route(const tt_route_lookup* lookups, int32_t num, int64_t batch, int32_t world, int32_t num_tags,
               RoutePlan* p) {
  TT_REQUIRE(num >= 1 && num <= kMaxRouteLookups, "route: 1..%d lookups, got %d", kMaxRouteLookups, num);
  TT_REQUIRE(batch >= 1, "route: empty batch");
  TT_REQUIRE(world >= 1 && world <= kMaxWorld, "route: world %d out of range", world);
  TT_REQUIRE(num_tags >= 1, "route: num_tags must be >= 1");
  TT_REQUIRE(batch * num < (int64_t(1) << 31), "route: too many lookups");
  int64_t max_rows = 1;
  for (int l = 0; l < num; ++l) {
    TT_REQUIRE(lookups == nullptr || (lookups[l].tag >= 0 && lookups[l].tag < num_tags),
               "route: lookup %d tag out of range", l);
    if (lookups) max_rows = std::max<int64_t>(max_rows, lookups[l].num_rows);
  }
  p->total = batch * num;
  p->id_bits = bits_for(max_rows);
  p->end_bit = p->id_bits + bits_for(static_cast<int64_t>(world) * num_tags - 1);
  TT_REQUIRE(p->end_bit <= 64, "route: key does not fit 64 bits");
  size_t sb = 0;
  unsigned long long* kp = nullptr;
  uint32_t* vp = nullptr;
  hipError_t e = rocprim::radix_sort_pairs<SortConfig>(nullptr, sb, kp, kp, vp, vp, static_cast<unsigned>(p->total), 0,
                                           p->end_bit, nullptr, false);
  p->sort_bytes = (e == hipSuccess) ? sb : static_cast<size_t>(p->total) * 24 + (size_t(4) << 20);
  return TT_OK;
}

struct RouteWs {
  unsigned long long *keys_in, *keys;
  uint32_t *vals_in, *vals;
  void* sort_tmp;
  int32_t* block_heads;
};

RouteWs carve_route(Carver& cv, const RoutePlan& p) {
  RouteWs w;
  w.keys_in = cv.take<unsigned long long>(p.total);
  w.keys = cv.take<unsigned long long>(p.total);
  w.vals_in = cv.take<uint32_t>(p.total);
  w.vals = cv.take<uint32_t>(p.total);
  w.sort_tmp = cv.take<char>(static_cast<int64_t>(p.sort_bytes) + 256);
  w.block_heads = cv.take<int32_t>(ceil_div(p.total, kScanThreads));
  return w;
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" size_t tt_route_workspace_size(int32_t num_lookups, int64_t batch, int32_t world, int64_t max_rows,
                                          int32_t num_tags) {
  RoutePlan p;
  if (num_lookups < 1 || batch < 1 || world < 1 || num_tags < 1) return 0;
  p.total = batch * num_lookups;
  p.id_bits = bits_for(max_rows > 0 ? max_rows : 1);
  p.end_bit = p.id_bits + bits_for(static_cast<int64_t>(world) * num_tags - 1);
  size_t sb = 0;
  unsigned long long* kp = nullptr;
  uint32_t* vp = nullptr;
  hipError_t e = rocprim::radix_sort_pairs<SortConfig>(nullptr, sb, kp, kp, vp, vp, static_cast<unsigned>(p.total), 0,
                                           p.end_bit, nullptr, false);
  p.sort_bytes = (e == hipSuccess) ? sb : static_cast<size_t>(p.total) * 24 + (size_t(4) << 20);
  Carver cv(nullptr, 0);
  carve_route(cv, p);
  return cv.used();
}

extern "C" int tt_route_requests(const tt_route_lookup* lookups, int32_t num_lookups, int64_t batch, int32_t world,
                                 int32_t num_tags, int32_t* send, long long* counts, int32_t* num_requests,
                                 int32_t* idx, void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(lookups && send && counts && num_requests && idx, "tt_route_requests: NULL pointer");
  for (int l = 0; l < num_lookups && l < kMaxRouteLookups; ++l)
    TT_REQUIRE(lookups[l].ids && lookups[l].num_rows >= 1 && lookups[l].num_rows < (int64_t(1) << 31),
               "tt_route_requests: lookup %d ids/num_rows invalid", l);
  RoutePlan p;
  int rc = plan_route(lookups, num_lookups, batch, world, num_tags, &p);
  if (rc) return rc;
  Carver cv(workspace, workspace_bytes);
  RouteWs w = carve_route(cv, p);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_route_requests: workspace %zu < required %zu", workspace_bytes, cv.used());
  hipStream_t st = to_stream(stream);
  RouteArgs a{};
  for (int l = 0; l < num_lookups; ++l) a.lk[l] = RouteLookup{lookups[l].ids, lookups[l].num_rows, lookups[l].tag};
  a.num = num_lookups;
  a.batch = batch;
  a.world = world;
  a.num_tags = num_tags;
  a.id_bits = p.id_bits;
  a.keys_in = w.keys_in;
  a.vals_in = w.vals_in;
  hipLaunchKernelGGL(route_keys_kernel, dim3(static_cast<unsigned>(ceil_div(p.total, 256))), dim3(256), 0, st, a);
  TT_CHECK_LAUNCH();
  size_t sb = p.sort_bytes;
  TT_CHECK_HIP(rocprim::radix_sort_pairs<SortConfig>(w.sort_tmp, sb, w.keys_in, w.keys, w.vals_in, w.vals,
                                         static_cast<unsigned>(p.total), 0, p.end_bit, st, false));
  const unsigned nb = static_cast<unsigned>(ceil_div(p.total, kScanThreads));
  hipLaunchKernelGGL(route_heads_kernel, dim3(nb), dim3(kScanThreads), 0, st, w.keys, p.total, w.block_heads, counts,
                     world);
  TT_CHECK_LAUNCH();
  hipLaunchKernelGGL(route_write_kernel, dim3(nb), dim3(kScanThreads), 0, st, w.keys, w.vals, p.total, world,
                     num_tags, p.id_bits, w.block_heads, send, idx, counts, num_requests);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_route_owner(const int32_t* recv, int64_t n, int32_t world, int32_t num_tags, int32_t* tags,
                              int32_t* rows, int32_t* table_ids, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(n >= 0 && world >= 1 && num_tags >= 1, "tt_route_owner: bad arguments");
  if (n == 0) return TT_OK;
  TT_REQUIRE(recv && tags && rows && table_ids, "tt_route_owner: NULL pointer");
  hipLaunchKernelGGL(route_owner_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0,
                     to_stream(stream), recv, n, world, num_tags, tags, rows, table_ids);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_route_pad(const int32_t* send, const long long* counts, const int32_t* idx, int64_t num_lookups,
                            int32_t world, int64_t cap, int32_t* send_padded, int32_t* idx_padded, int32_t* overflow,
                            tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(send && counts && idx && send_padded && idx_padded, "tt_route_pad: NULL pointer");
  TT_REQUIRE(world >= 1 && world <= kMaxWorld, "tt_route_pad: world %d out of range", world);
  TT_REQUIRE(cap >= 1 && num_lookups >= 1, "tt_route_pad: cap %lld / lookups %lld must be >= 1",
             static_cast<long long>(cap), static_cast<long long>(num_lookups));
  TT_REQUIRE(static_cast<int64_t>(world) * cap < (int64_t(1) << 31), "tt_route_pad: world * cap exceeds int32");
  const int64_t n = std::max<int64_t>(static_cast<int64_t>(world) * cap, num_lookups);
  hipLaunchKernelGGL(route_pad_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0, to_stream(stream),
                     send, counts, idx, num_lookups, world, cap, send_padded, idx_padded, overflow);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
