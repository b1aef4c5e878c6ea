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
#include <cstdlib>
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
  void* keys_in;  // KeyT [total]
  uint32_t* vals_in;
};

// KeyT: uint32_t when the key bits in use fit 32 (every config here: the
// sort then moves and compares half the key bytes), else 64-bit
template <typename KeyT>
__global__ void __launch_bounds__(256) route_keys_kernel(const RouteArgs a) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  const int64_t total = a.batch * a.num;
  if (i >= total) return;
  const int l = static_cast<int>(i / a.batch);
  const int64_t b = i - l * a.batch;
  const RouteLookup& L = a.lk[l];
  const int32_t r = L.ids[b];
  const bool ok = r >= 0 && r < L.num_rows;
  const KeyT owner = ok ? static_cast<KeyT>(r % a.world) : static_cast<KeyT>(a.world - 1);
  const KeyT rowp1 = ok ? static_cast<KeyT>(r) + KeyT(1) : KeyT(0);
  static_cast<KeyT*>(a.keys_in)[i] = ((owner * static_cast<KeyT>(a.num_tags) + static_cast<KeyT>(L.tag)) << a.id_bits) |
                                     rowp1;
  a.vals_in[i] = static_cast<uint32_t>(i);
}

// World-1 fixed slots written by the head / write passes themselves (no
// route_pad launch): the one owner's requests start at slot 0, so request u
// IS slot u (u < cap; the rest are dropped and counted).  The heads pass
// fills every slot with (-1, -1) and the owner view with -1; the write pass
// then overwrites the requests' slots.  send == NULL: not this mode.
struct World1Slots {
  int64_t cap;
  int32_t* send;      // [cap, 2]
  int32_t* idx;       // [total]: each lookup's slot
  int32_t* overflow;  // optional
  int32_t* tags;      // [cap]
  int32_t* rows;      // [cap]
  int32_t* tids;      // [num_tags, cap]
  int32_t num_tags;
};

// Heads of the sorted key runs = distinct requests.  Pass 1: per block of
// kScanThreads consecutive sorted keys (one per thread, coalesced), the
// number of heads.  Pass 2: each block adds up the counts of the blocks
// before it (wave-parallel), scans its own heads and writes send / idx and
// its per-owner counts (LDS, then one atomic per owner per block into the
// zeroed counts); the last block writes the request total.
template <typename KeyT>
__global__ void __launch_bounds__(kScanThreads) route_heads_kernel(const KeyT* keys, int64_t total,
                                                                   int32_t* block_heads, long long* counts,
                                                                   int32_t world, int32_t* grp_first, int32_t* grp_last,
                                                                   int32_t groups, const World1Slots w1) {
  // the per-owner counts route_write_kernel adds into are zeroed here, by a
  // kernel, not by a captured hipMemsetAsync: with the memset node (and the
  // counts' block recycled inside the step's graph) the overflow word picked
  // up garbage in 2 of 2 graphed runs; a standalone probe of memset nodes
  // (tools/graph_replay_overlap_probe.py) stayed ordered, so that cause is
  // not pinned down, and the kernel-zeroed version has run clean since
  if (blockIdx.x == 0)
    for (int o = threadIdx.x; o < world; o += kScanThreads) counts[o] = 0;
  // (owner, tag) group bounds (optional): empty groups read [0, -1]
  if (grp_first && blockIdx.x == gridDim.x - 1)
    for (int g = threadIdx.x; g < groups; g += kScanThreads) {
      grp_first[g] = 0;
      grp_last[g] = -1;
    }
  if (w1.send)  // world-1 slots: every slot empty until the write pass fills the requests'
    for (int64_t t = static_cast<int64_t>(blockIdx.x) * kScanThreads + threadIdx.x; t < w1.cap;
         t += static_cast<int64_t>(gridDim.x) * kScanThreads) {
      w1.send[2 * t] = -1;
      w1.send[2 * t + 1] = -1;
      if (w1.tags) {
        w1.tags[t] = -1;
        w1.rows[t] = -1;
        for (int q = 0; q < w1.num_tags; ++q) w1.tids[static_cast<int64_t>(q) * w1.cap + t] = -1;
      }
    }
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

template <typename KeyT>
__global__ void __launch_bounds__(kScanThreads) route_write_kernel(const KeyT* keys, const uint32_t* vals,
                                                                   int64_t total, int32_t world, int32_t num_tags,
                                                                   int32_t id_bits, const int32_t* block_heads,
                                                                   int32_t* send, int32_t* idx, long long* counts,
                                                                   int32_t* num_requests, int32_t* order,
                                                                   int32_t* grp_first, int32_t* grp_last,
                                                                   const World1Slots w1) {
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
  const KeyT k = i < total ? keys[i] : KeyT(0);
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
      const KeyT mask = (KeyT(1) << id_bits) - KeyT(1);
      const KeyT ot = k >> id_bits;
      const int32_t row = static_cast<int32_t>(static_cast<long long>(k & mask) - 1);
      const int32_t tag = static_cast<int32_t>(ot % num_tags);
      if (w1.send) {
        if (u < w1.cap) {
          w1.send[2 * static_cast<int64_t>(u)] = row;
          w1.send[2 * static_cast<int64_t>(u) + 1] = tag;
          if (w1.tags) {
            w1.tags[u] = tag;
            w1.rows[u] = row;
            w1.tids[static_cast<int64_t>(tag) * w1.cap + u] = row;
          }
        }
      } else {
        send[2 * static_cast<int64_t>(u)] = row;
        send[2 * static_cast<int64_t>(u) + 1] = tag;
      }
      atomicAdd(&cnt[static_cast<int>(ot / num_tags)], 1);
    }
    // a dropped request's lookups get the sentinel -1 - owner (owner 0 here):
    // gathers read a zero row for them, the sparse sums skip them
    if (w1.send) w1.idx[vals[i]] = static_cast<int32_t>(u < w1.cap ? u : -1);
    else idx[vals[i]] = u;
    if (order) order[i] = static_cast<int32_t>(vals[i]);
    if (grp_first) {  // first / last sorted position of each (owner, tag) group
      const KeyT g = k >> id_bits;
      if (i == 0 || (keys[i - 1] >> id_bits) != g) grp_first[g] = static_cast<int32_t>(i);
      if (i == total - 1 || (keys[i + 1] >> id_bits) != g) grp_last[g] = static_cast<int32_t>(i);
    }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < world; o += kScanThreads)
    if (cnt[o]) atomicAdd(reinterpret_cast<unsigned long long*>(counts + o), static_cast<unsigned long long>(cnt[o]));
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    const int n = base_s + wsum[kScanThreads / kWave];
    *num_requests = n;
    if (w1.send && w1.overflow && n > w1.cap) atomicAdd(w1.overflow, static_cast<int32_t>(n - w1.cap));
  }
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
// own_tags / own_rows / own_tids (optional, world 1): tt_route_owner's view
// of the slots written in the same pass.
__global__ void __launch_bounds__(256) route_pad_kernel(const int32_t* send, const long long* counts,
                                                        const int32_t* idx, int64_t num_lookups, int32_t world,
                                                        int64_t cap, int32_t* send_padded, int32_t* idx_padded,
                                                        int32_t* overflow, int32_t num_tags, int32_t* own_tags,
                                                        int32_t* own_rows, int32_t* own_tids) {
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
    if (own_tags) {  // world 1: the local row is the row
      own_tags[t] = tag;
      own_rows[t] = row;
      for (int q = 0; q < num_tags; ++q) own_tids[static_cast<int64_t>(q) * slots + t] = q == tag ? row : -1;
    }
    if (j == cap - 1 && n > cap && overflow) atomicAdd(overflow, static_cast<int32_t>(n - cap));
  }
  if (t < num_lookups) {
    const long long u = idx[t];
    int lo = 0, hi = world - 1;  // the owner o with start[o] <= u < start[o + 1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (start[mid] <= u) lo = mid; else hi = mid - 1;
    }
    const long long j = u - start[lo];
    // dropped request (counted in *overflow): the sentinel -1 - owner (no slot;
    // a gather reads a zero row, the sparse sums skip it)
    idx_padded[t] = j < cap ? static_cast<int32_t>(static_cast<int64_t>(lo) * cap + j) : -1 - lo;
  }
}

// ---- fused fixed-capacity route for small batches (tt_route_fixed) --------
// One 1024-thread workgroup does the whole route of <= kRsMax lookups whose
// keys fit 32 bits: key build into LDS, a stable LSD radix sort of the
// positions (8-bit-or-narrower digits; per wave a contiguous slice, ranks by
// ballots of equal digits, so equal keys keep lookup order — the rocPRIM
// path's order), the request scan, then the padded slots, each lookup's slot,
// the per-owner counts and overflow, optionally the sorted order / group
// bounds, and at world 1 the owner view (tags / rows / table_ids) of the
// slots — the outputs of tt_route_requests_ordered + tt_route_pad (+
// tt_route_owner) in one launch instead of ~11 (key build, ~6 sort
// launches, heads, write, pad, owner: each a few microseconds of launch
// and drain at a 2048-row step).
#ifdef TT_ROUTE_STAMPS
__device__ unsigned long long g_route_stamps[8];  // phase end times (wall clock), thread 0
#define TT_RS_STAMP(i)                                            \
  if (threadIdx.x == 0) g_route_stamps[i] = wall_clock64();
#else
#define TT_RS_STAMP(i)
#endif
constexpr int kRsThreads = 1024;
constexpr int kRsWaves = kRsThreads / kWave;
// the one-workgroup route wins only at small batches (one CU's LDS radix
// passes: 25 vs 31 us per call at 3 x 1024 lookups, 44 vs 46 at 3 x 2048,
// 108 vs 46 at 3 x 5461 — tools/time_route.py, profiles/r05_route_fused.txt)
constexpr int kRsMax = 8192;
constexpr int kRsPer = kRsMax / kRsThreads;  // lookups staged per thread
constexpr int kRsTiles = kRsMax / kRsWaves / kWave;  // 64-lane tiles per wave at the maximum
constexpr int kRsHistStride = kRsWaves + 1;
constexpr size_t kRsLdsBytes = size_t(kRsMax) * 4 + size_t(2) * kRsMax * 2 + size_t(256) * kRsHistStride * 4 +
                               size_t(2) * (kMaxWorld + 1) * 4;

struct RouteFixedArgs {
  RouteLookup lk[kMaxRouteLookups];
  int32_t num;
  int64_t batch;
  int32_t world, num_tags, id_bits, end_bit;
  int64_t cap;
  int32_t* send_padded;
  int32_t* idx_padded;
  long long* counts;
  int32_t* overflow;
  int32_t* order;
  int32_t* grp_first;
  int32_t* grp_last;
  int32_t* own_tags;
  int32_t* own_rows;
  int32_t* own_tids;
};

// lanes of this wave holding the same digit among the active lanes (one
// ballot per digit bit, nbits <= 8, wave-uniform)
__device__ __forceinline__ uint64_t rs_peers(uint32_t d, bool act, int nbits) {
  const uint64_t a = __ballot(act);
  uint32_t lo = static_cast<uint32_t>(a), hi = static_cast<uint32_t>(a >> 32);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if (b >= nbits) break;
    const uint32_t bit = (d >> b) & 1u;
    const uint64_t bal = __ballot(bit);
    const uint32_t flip = bit - 1u;
    lo &= static_cast<uint32_t>(bal) ^ flip;
    hi &= static_cast<uint32_t>(bal >> 32) ^ flip;
  }
  return act ? (static_cast<uint64_t>(hi) << 32 | lo) : 0;
}

// block-wide exclusive scan of one int per thread; *total = the sum
__device__ __forceinline__ int rs_scan(int v, int* wsum, int* total) {
  const int lane = lane_id(), w = threadIdx.x / kWave;
  int x = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  __syncthreads();  // wsum free (an earlier scan's readers are done)
  if (lane == kWave - 1) wsum[w] = x;
  __syncthreads();
  int ex = x - v, t = 0;
  for (int q = 0; q < kRsWaves; ++q) {
    const int c = wsum[q];
    ex += q < w ? c : 0;
    t += c;
  }
  *total = t;
  return ex;
}

__global__ void __launch_bounds__(kRsThreads) route_fixed_small_kernel(const RouteFixedArgs a) {
  extern __shared__ __attribute__((aligned(16))) char rsm[];
  uint32_t* lkey = reinterpret_cast<uint32_t*>(rsm);
  uint16_t* pb0 = reinterpret_cast<uint16_t*>(rsm + kRsMax * 4);
  uint16_t* pb1 = pb0 + kRsMax;
  uint32_t* hist = reinterpret_cast<uint32_t*>(rsm + kRsMax * 8);  // [256][kRsHistStride]
  int* cnt = reinterpret_cast<int*>(rsm + kRsMax * 8 + 256 * kRsHistStride * 4);
  int* start = cnt + (kMaxWorld + 1);
  __shared__ int wsum[kRsWaves];
  TT_RS_STAMP(5)
  const int tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
  const int n = static_cast<int>(a.batch * a.num);
  const int W = a.world, T = a.num_tags;
  // keys: (owner, tag, row + 1) as in route_keys_kernel, 32 bits; every id
  // load of the thread issued before the first is used
  {
    const int B = static_cast<int>(a.batch);
    int32_t r[kRsPer];
    int lk[kRsPer];
#pragma unroll
    for (int u = 0; u < kRsPer; ++u) {
      const int i = tid + u * kRsThreads;
      const int l = i < n ? i / B : 0;
      lk[u] = l;
      r[u] = i < n ? a.lk[l].ids[i - l * B] : 0;
    }
#pragma unroll
    for (int u = 0; u < kRsPer; ++u) {
      const int i = tid + u * kRsThreads;
      if (i < n) {
        const RouteLookup& L = a.lk[lk[u]];
        const bool ok = r[u] >= 0 && r[u] < L.num_rows;
        const uint32_t owner = ok ? static_cast<uint32_t>(r[u] % W) : static_cast<uint32_t>(W - 1);
        const uint32_t rowp1 = ok ? static_cast<uint32_t>(r[u]) + 1u : 0u;
        lkey[i] = ((owner * static_cast<uint32_t>(T) + static_cast<uint32_t>(L.tag)) << a.id_bits) | rowp1;
        pb0[i] = static_cast<uint16_t>(i);
      }
    }
  }
  for (int o = tid; o <= W; o += kRsThreads) cnt[o] = 0;
  if (a.grp_first)
    for (int g = tid; g < W * T; g += kRsThreads) {
      a.grp_first[g] = 0;
      a.grp_last[g] = -1;
    }
  TT_RS_STAMP(0)
  // stable LSD radix sort of the positions by key
  const int per = ((n + kRsWaves - 1) / kRsWaves + kWave - 1) / kWave * kWave;
  const int wbeg = w * per, wend = min(n, wbeg + per);
  const uint64_t lt = (uint64_t(1) << lane) - 1u;
  const int passes = (a.end_bit + 7) / 8;
  const int width = (a.end_bit + passes - 1) / passes;
  const uint32_t dmask = (1u << width) - 1u;
  uint16_t* src = pb0;
  uint16_t* dst = pb1;
  for (int p = 0; p < passes; ++p) {
    const int sh = p * width;
    for (int e = tid; e < 256 * kRsHistStride; e += kRsThreads) hist[e] = 0u;
    __syncthreads();
    uint16_t pos[kRsTiles];
    uint32_t dig[kRsTiles];
    uint64_t peer[kRsTiles];
#pragma unroll
    for (int q = 0; q < kRsTiles; ++q) {
      const int i = wbeg + q * kWave + lane;
      pos[q] = 0;
      dig[q] = 0;
      if (i < wend) {
        pos[q] = src[i];
        dig[q] = (lkey[pos[q]] >> sh) & dmask;
      }
    }
#pragma unroll
    for (int q = 0; q < kRsTiles; ++q) {
      peer[q] = 0;
      if (wbeg + q * kWave < wend) {  // wave-uniform
        peer[q] = rs_peers(dig[q], wbeg + q * kWave + lane < wend, width);
        if (peer[q] != 0 && __builtin_ctzll(peer[q]) == lane) hist[dig[q] * kRsHistStride + w] += __popcll(peer[q]);
      }
    }
    __syncthreads();
    {  // counts -> exclusive offsets in (digit, wave) order: 4 words per thread
      uint32_t h[4], run = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int L = 4 * tid + u;
        h[u] = hist[(L / kRsWaves) * kRsHistStride + L % kRsWaves];
        run += h[u];
      }
      int tot;
      uint32_t ex = static_cast<uint32_t>(rs_scan(static_cast<int>(run), wsum, &tot));
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int L = 4 * tid + u;
        hist[(L / kRsWaves) * kRsHistStride + L % kRsWaves] = ex;
        ex += h[u];
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kRsTiles; ++q) {
      if (wbeg + q * kWave < wend) {  // wave-uniform
        const uint64_t m = peer[q];
        if (m != 0) {
          uint32_t* slot = &hist[dig[q] * kRsHistStride + w];
          const uint32_t off = *slot;
          dst[off + __popcll(m & lt)] = pos[q];
          if (__builtin_ctzll(m) == lane) *slot = off + __popcll(m);
        }
      }
    }
    __syncthreads();
    uint16_t* t = src;
    src = dst;
    dst = t;
  }
  TT_RS_STAMP(1)
  // requests: heads of the sorted key runs; each thread a contiguous run of
  // sorted positions
  const int E = (n + kRsThreads - 1) / kRsThreads;
  const int p0 = min(n, tid * E), p1 = min(n, p0 + E);
  const uint32_t omask = (1u << a.id_bits) - 1u;
  // (a thread's sorted keys have non-decreasing owners: one LDS atomic per
  // owner run, not per request — at world 1 every request has owner 0)
  int heads = 0, run_owner = -1, run_n = 0;
  uint32_t kprev = p0 > 0 ? lkey[src[p0 - 1]] : ~0u;
  for (int p = p0; p < p1; ++p) {
    const uint32_t k = lkey[src[p]];
    if (p == 0 || k != kprev) {
      ++heads;
      const int o = static_cast<int>((k >> a.id_bits) / static_cast<uint32_t>(T));
      if (o != run_owner) {
        if (run_n) atomicAdd(&cnt[run_owner], run_n);
        run_owner = o;
        run_n = 0;
      }
      ++run_n;
    }
    kprev = k;
  }
  if (run_n) atomicAdd(&cnt[run_owner], run_n);
  int nreq;
  const int ubase = rs_scan(heads, wsum, &nreq);
  {  // owners' first request: exclusive scan of cnt (W <= kRsThreads)
    int tot;
    const int c = tid < W ? cnt[tid] : 0;
    const int ex = rs_scan(c, wsum, &tot);
    if (tid < W) start[tid] = ex;
  }
  __syncthreads();
  TT_RS_STAMP(2)
  int u = ubase - 1;
  for (int p = p0; p < p1; ++p) {
    const int pos = src[p];
    const uint32_t k = lkey[pos];
    const uint32_t kp = p > 0 ? lkey[src[p - 1]] : ~0u;
    const bool head = p == 0 || k != kp;
    u += head ? 1 : 0;
    const uint32_t g = k >> a.id_bits;
    const int o = static_cast<int>(g / static_cast<uint32_t>(T));
    const int tag = static_cast<int>(g - static_cast<uint32_t>(o * T));
    const int64_t j = u - start[o];
    const int64_t slot = static_cast<int64_t>(o) * a.cap + j;
    a.idx_padded[pos] = j < a.cap ? static_cast<int32_t>(slot) : -1 - o;  // dropped: sentinel -1 - owner
    if (a.order) a.order[p] = pos;
    if (a.grp_first) {
      if (p == 0 || (kp >> a.id_bits) != g) a.grp_first[g] = p;
      if (p == n - 1 || (lkey[src[p + 1]] >> a.id_bits) != g) a.grp_last[g] = p;
    }
    if (head && j < a.cap) {
      const int32_t row = static_cast<int32_t>(static_cast<int64_t>(k & omask) - 1);
      a.send_padded[2 * slot] = row;
      a.send_padded[2 * slot + 1] = tag;
      if (a.own_tags) {  // world 1: the owner's local row is the row
        a.own_tags[slot] = tag;
        a.own_rows[slot] = row;
        for (int t = 0; t < T; ++t) a.own_tids[static_cast<int64_t>(t) * W * a.cap + slot] = t == tag ? row : -1;
      }
    }
  }
  TT_RS_STAMP(3)
  // unused slots, counts, overflow
  const int64_t slots = static_cast<int64_t>(W) * a.cap;
  for (int64_t t = tid; t < slots; t += kRsThreads) {
    const int o = static_cast<int>(t / a.cap);
    if (t - static_cast<int64_t>(o) * a.cap >= cnt[o]) {
      a.send_padded[2 * t] = -1;
      a.send_padded[2 * t + 1] = -1;
      if (a.own_tags) {
        a.own_tags[t] = -1;
        a.own_rows[t] = -1;
        for (int q = 0; q < T; ++q) a.own_tids[static_cast<int64_t>(q) * slots + t] = -1;
      }
    }
  }
  if (tid < W) {
    a.counts[tid] = cnt[tid];
    if (a.overflow && cnt[tid] > a.cap) atomicAdd(a.overflow, static_cast<int32_t>(cnt[tid] - a.cap));
  }
  TT_RS_STAMP(4)
}

// The route's sort configuration: rocPRIM's defaults, or (TT_ROUTE_SORT_BS >
// 0) a merge-sort path whose block sort covers TT_ROUTE_SORT_BS x
// TT_ROUTE_SORT_IPT keys (fewer merge launches).
#ifndef TT_ROUTE_SORT_BS
#define TT_ROUTE_SORT_BS 0
#endif
#ifndef TT_ROUTE_SORT_IPT
#define TT_ROUTE_SORT_IPT 4
#endif
#if TT_ROUTE_SORT_BS > 0
using RouteSortConfig =
    rocprim::radix_sort_config<rocprim::default_config,
                               rocprim::merge_sort_config<TT_ROUTE_SORT_BS, TT_ROUTE_SORT_BS, TT_ROUTE_SORT_IPT>,
                               rocprim::default_config, TT_SORT_MERGE_LIMIT>;
#else
using RouteSortConfig = SortConfig;
#endif

// The route's device sort: rocPRIM's merge path below TT_SORT_MERGE_LIMIT
// (block sort + ~6 merge launches at 65,536 keys).  Its onesweep radix path
// (histogram + one launch per 8-bit digit) measured slower at C5: 0.19 vs
// 0.13 ms per step (tools/runs/gpu_s05_route3.sh).
size_t route_sort_bytes(int64_t total, int end_bit) {
  size_t a = 0;
  uint32_t* vp = nullptr;
  hipError_t e;
  if (end_bit <= 32) {
    uint32_t* kp = nullptr;
    e = rocprim::radix_sort_pairs<RouteSortConfig>(nullptr, a, kp, kp, vp, vp, static_cast<unsigned>(total), 0, end_bit,
                                              nullptr, false);
  } else {
    unsigned long long* kp = nullptr;
    e = rocprim::radix_sort_pairs<RouteSortConfig>(nullptr, a, kp, kp, vp, vp, static_cast<unsigned>(total), 0, end_bit,
                                              nullptr, false);
  }
  return e == hipSuccess ? a : static_cast<size_t>(total) * 24 + (size_t(4) << 20);
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
  p->sort_bytes = route_sort_bytes(p->total, p->end_bit);
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
  p.sort_bytes = route_sort_bytes(p.total, p.end_bit);
  Carver cv(nullptr, 0);
  carve_route(cv, p);
  return cv.used();
}

namespace tt {
namespace {
int route_requests(const tt_route_lookup* lookups, int32_t num_lookups, int64_t batch, int32_t world,
                   int32_t num_tags, int32_t* send, long long* counts, int32_t* num_requests, int32_t* idx,
                   int32_t* order, int32_t* grp_first, int32_t* grp_last, void* workspace, size_t workspace_bytes,
                   tt_stream_t stream, const World1Slots& w1) {
  TT_REQUIRE(lookups && send && counts && num_requests && idx, "tt_route_requests: NULL pointer");
  TT_REQUIRE((grp_first == nullptr) == (grp_last == nullptr), "tt_route_requests: grp_first / grp_last: both or neither");
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
  const auto run = [&](auto key_tag) -> int {
    using KeyT = decltype(key_tag);
    KeyT* kin = reinterpret_cast<KeyT*>(w.keys_in);
    KeyT* kout = reinterpret_cast<KeyT*>(w.keys);
    hipLaunchKernelGGL(route_keys_kernel<KeyT>, dim3(static_cast<unsigned>(ceil_div(p.total, 256))), dim3(256), 0, st,
                       a);
    TT_CHECK_LAUNCH();
    size_t sb = p.sort_bytes;
    TT_CHECK_HIP(rocprim::radix_sort_pairs<RouteSortConfig>(w.sort_tmp, sb, kin, kout, w.vals_in, w.vals,
                                                       static_cast<unsigned>(p.total), 0, p.end_bit, st, false));
    const unsigned nb = static_cast<unsigned>(ceil_div(p.total, kScanThreads));
    hipLaunchKernelGGL(route_heads_kernel<KeyT>, dim3(nb), dim3(kScanThreads), 0, st, kout, p.total, w.block_heads,
                       counts, world, grp_first, grp_last, world * num_tags, w1);
    TT_CHECK_LAUNCH();
    hipLaunchKernelGGL(route_write_kernel<KeyT>, dim3(nb), dim3(kScanThreads), 0, st, kout, w.vals, p.total, world,
                       num_tags, p.id_bits, w.block_heads, send, idx, counts, num_requests, order, grp_first,
                       grp_last, w1);
    TT_CHECK_LAUNCH();
    return TT_OK;
  };
  return p.end_bit <= 32 ? run(uint32_t{}) : run(static_cast<unsigned long long>(0));
}
}  // namespace
}  // namespace tt

extern "C" int tt_route_requests_ordered(const tt_route_lookup* lookups, int32_t num_lookups, int64_t batch,
                                         int32_t world, int32_t num_tags, int32_t* send, long long* counts,
                                         int32_t* num_requests, int32_t* idx, int32_t* order, int32_t* grp_first,
                                         int32_t* grp_last, void* workspace, size_t workspace_bytes,
                                         tt_stream_t stream) {
  clear_error();
  return route_requests(lookups, num_lookups, batch, world, num_tags, send, counts, num_requests, idx, order,
                        grp_first, grp_last, workspace, workspace_bytes, stream, World1Slots{});
}

extern "C" int tt_route_requests(const tt_route_lookup* lookups, int32_t num_lookups, int64_t batch, int32_t world,
                                 int32_t num_tags, int32_t* send, long long* counts, int32_t* num_requests,
                                 int32_t* idx, void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  return tt_route_requests_ordered(lookups, num_lookups, batch, world, num_tags, send, counts, num_requests, idx,
                                   nullptr, nullptr, nullptr, workspace, workspace_bytes, stream);
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
                     send, counts, idx, num_lookups, world, cap, send_padded, idx_padded, overflow, 1, nullptr,
                     nullptr, nullptr);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

namespace tt {
namespace {
// the multi-launch path's scratch after the route workspace: compact send,
// idx and the request count
struct FixedWs {
  RouteWs rw;
  int32_t* send;
  int32_t* idx;
  int32_t* nreq;
};
FixedWs carve_fixed(Carver& cv, const RoutePlan& p) {
  FixedWs f;
  f.rw = carve_route(cv, p);
  f.send = cv.take<int32_t>(2 * p.total);
  f.idx = cv.take<int32_t>(p.total);
  f.nreq = cv.take<int32_t>(1);
  return f;
}
bool route_w1_slots() {  // TT_ROUTE_W1_SLOTS=0: world 1 through route_pad as well (A/B)
  static const bool off = [] {
    const char* e = std::getenv("TT_ROUTE_W1_SLOTS");
    return e && e[0] == '0';
  }();
  return !off;
}
bool route_fused(const RoutePlan& p) {
  static const bool off = [] {
    const char* e = std::getenv("TT_ROUTE_FUSED");
    return e && e[0] == '0';
  }();
  return !off && p.total <= kRsMax && p.end_bit <= 32;
}
}  // namespace
}  // namespace tt

extern "C" size_t tt_route_fixed_workspace_size(int32_t num_lookups, int64_t batch, int32_t world, int64_t max_rows,
                                                int32_t num_tags) {
  if (num_lookups < 1 || batch < 1 || world < 1 || num_tags < 1) return 0;
  const size_t base = tt_route_workspace_size(num_lookups, batch, world, max_rows, num_tags);
  const int64_t total = batch * num_lookups;
  return base + ((static_cast<size_t>(total) * 12 + 4 + 3 * 256) & ~size_t(255)) + 256;
}

extern "C" int tt_route_fixed(const tt_route_lookup* lookups, int32_t num_lookups, int64_t batch, int32_t world,
                              int32_t num_tags, int64_t cap, int32_t* send_padded, int32_t* idx_padded,
                              long long* counts, int32_t* overflow, int32_t* order, int32_t* grp_first,
                              int32_t* grp_last, int32_t* owner_tags, int32_t* owner_rows, int32_t* owner_table_ids,
                              void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(lookups && send_padded && idx_padded && counts, "tt_route_fixed: NULL pointer");
  TT_REQUIRE((grp_first == nullptr) == (grp_last == nullptr), "tt_route_fixed: grp_first / grp_last: both or neither");
  const bool owner = owner_tags != nullptr;
  TT_REQUIRE(owner == (owner_rows != nullptr) && owner == (owner_table_ids != nullptr),
             "tt_route_fixed: owner_tags / owner_rows / owner_table_ids: all or none");
  TT_REQUIRE(!owner || world == 1, "tt_route_fixed: the owner view is the world-1 shortcut (world %d)", world);
  TT_REQUIRE(cap >= 1 && static_cast<int64_t>(world) * cap < (int64_t(1) << 31), "tt_route_fixed: bad cap");
  for (int l = 0; l < num_lookups && l < kMaxRouteLookups; ++l)
    TT_REQUIRE(lookups[l].ids && lookups[l].num_rows >= 1 && lookups[l].num_rows < (int64_t(1) << 31),
               "tt_route_fixed: lookup %d ids/num_rows invalid", l);
  RoutePlan p;
  int rc = plan_route(lookups, num_lookups, batch, world, num_tags, &p);
  if (rc) return rc;
  hipStream_t st = to_stream(stream);
  if (route_fused(p)) {
    RouteFixedArgs a{};
    for (int l = 0; l < num_lookups; ++l) a.lk[l] = RouteLookup{lookups[l].ids, lookups[l].num_rows, lookups[l].tag};
    a.num = num_lookups;
    a.batch = batch;
    a.world = world;
    a.num_tags = num_tags;
    a.id_bits = p.id_bits;
    a.end_bit = p.end_bit;
    a.cap = cap;
    a.send_padded = send_padded;
    a.idx_padded = idx_padded;
    a.counts = counts;
    a.overflow = overflow;
    a.order = order;
    a.grp_first = grp_first;
    a.grp_last = grp_last;
    a.own_tags = owner_tags;
    a.own_rows = owner_rows;
    a.own_tids = owner_table_ids;
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(route_fixed_small_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       static_cast<int>(kRsLdsBytes));
    TT_CHECK_HIP(attr);
    hipLaunchKernelGGL(route_fixed_small_kernel, dim3(1), dim3(kRsThreads), kRsLdsBytes, st, a);
    TT_CHECK_LAUNCH();
    return TT_OK;
  }
  Carver cv(workspace, workspace_bytes);
  FixedWs f = carve_fixed(cv, p);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_route_fixed: workspace %zu < required %zu", workspace_bytes, cv.used());
  const size_t rbytes = static_cast<size_t>(reinterpret_cast<char*>(f.send) - static_cast<char*>(workspace));
  if (world == 1 && route_w1_slots()) {
    // one owner: the head / write passes lay the slots out themselves
    const World1Slots w1{cap, send_padded, idx_padded, overflow, owner_tags, owner_rows, owner_table_ids, num_tags};
    return route_requests(lookups, num_lookups, batch, world, num_tags, f.send, counts, f.nreq, f.idx, order,
                          grp_first, grp_last, workspace, rbytes, stream, w1);
  }
  rc = route_requests(lookups, num_lookups, batch, world, num_tags, f.send, counts, f.nreq, f.idx, order, grp_first,
                      grp_last, workspace, rbytes, stream, World1Slots{});
  if (rc) return rc;
  // tt_route_pad, with the world-1 owner view written by the same pass
  const int64_t n = std::max<int64_t>(static_cast<int64_t>(world) * cap, p.total);
  hipLaunchKernelGGL(route_pad_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0, st, f.send,
                     counts, f.idx, p.total, world, cap, send_padded, idx_padded, overflow, num_tags, owner_tags,
                     owner_rows, owner_table_ids);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

#ifdef TT_ROUTE_STAMPS
// timing builds only: the fused route kernel's phase stamps (wall clock ticks)
extern "C" int tt_route_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_route_stamps), sizeof(g_route_stamps)) == hipSuccess ? TT_OK
                                                                                                      : TT_ERR_BAD_ARG;
}
#endif
