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
// then ONE workgroup (1024 threads, each a contiguous run of sorted keys)
// finds the heads, block-scans them and writes send / idx / counts; a few
// hundred thousand lookups per step make that a ~10 us pass, with no
// device-wide scan or atomics.
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

__global__ void __launch_bounds__(kScanThreads) route_scan_kernel(const unsigned long long* keys, const uint32_t* vals,
                                                                  int64_t total, int32_t world, int32_t num_tags,
                                                                  int32_t id_bits, int32_t* send, int32_t* idx,
                                                                  long long* counts, int32_t* num_requests) {
  __shared__ int wsum[kScanThreads / kWave + 1];
  __shared__ int cnt[kMaxWorld];
  for (int o = threadIdx.x; o < world; o += kScanThreads) cnt[o] = 0;
  const int64_t per = (total + kScanThreads - 1) / kScanThreads;
  const int64_t i0 = threadIdx.x * per;
  const int64_t i1 = i0 + per < total ? i0 + per : total;
  int heads = 0;
  for (int64_t i = i0; i < i1; ++i) heads += (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
  // block exclusive scan of the per-thread head counts
  const int lane = lane_id(), w = threadIdx.x / kWave;
  int x = heads;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int y = __shfl_up(x, off, kWave);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int k = 0; k < kScanThreads / kWave; ++k) {
      const int t = wsum[k];
      wsum[k] = run;
      run += t;
    }
    wsum[kScanThreads / kWave] = run;
  }
  __syncthreads();
  int u = wsum[w] + x - heads - 1;  // index of the current request
  const unsigned long long mask = (1ull << id_bits) - 1ull;
  for (int64_t i = i0; i < i1; ++i) {
    const unsigned long long k = keys[i];
    if (i == 0 || k != keys[i - 1]) {
      ++u;
      const unsigned long long ot = k >> id_bits;
      const int owner = static_cast<int>(ot / num_tags);
      send[2 * static_cast<int64_t>(u)] = static_cast<int32_t>(static_cast<long long>(k & mask) - 1);
      send[2 * static_cast<int64_t>(u) + 1] = static_cast<int32_t>(ot % num_tags);
      atomicAdd(&cnt[owner], 1);
    }
    idx[vals[i]] = u;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < world; o += kScanThreads) counts[o] = cnt[o];
  if (threadIdx.x == 0) *num_requests = wsum[kScanThreads / kWave];
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
  hipError_t e = rocprim::radix_sort_pairs(nullptr, sb, kp, kp, vp, vp, static_cast<unsigned>(p->total), 0,
                                           p->end_bit, nullptr, false);
  p->sort_bytes = (e == hipSuccess) ? sb : static_cast<size_t>(p->total) * 24 + (size_t(4) << 20);
  return TT_OK;
}

struct RouteWs {
  unsigned long long *keys_in, *keys;
  uint32_t *vals_in, *vals;
  void* sort_tmp;
};

RouteWs carve_route(Carver& cv, const RoutePlan& p) {
  RouteWs w;
  w.keys_in = cv.take<unsigned long long>(p.total);
  w.keys = cv.take<unsigned long long>(p.total);
  w.vals_in = cv.take<uint32_t>(p.total);
  w.vals = cv.take<uint32_t>(p.total);
  w.sort_tmp = cv.take<char>(static_cast<int64_t>(p.sort_bytes) + 256);
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
  hipError_t e = rocprim::radix_sort_pairs(nullptr, sb, kp, kp, vp, vp, static_cast<unsigned>(p.total), 0,
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
  TT_CHECK_HIP(rocprim::radix_sort_pairs(w.sort_tmp, sb, w.keys_in, w.keys, w.vals_in, w.vals,
                                         static_cast<unsigned>(p.total), 0, p.end_bit, st, false));
  hipLaunchKernelGGL(route_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, w.keys, w.vals, p.total, world, num_tags,
                     p.id_bits, send, idx, counts, num_requests);
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
