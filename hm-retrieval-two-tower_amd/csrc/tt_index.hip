// K11+K12: brute-force scoring with fused top-K
// (BruteForceIndex.call, /root/reference/pkg/modelling/indices/brute_force.py:75-83:
//  scores = matmul(Q, C^T); top_k(scores, k) sorted descending, ties -> lower
//  index; int32 indices).
//
// Exactness contract: the returned indices are bit-exact against the fp32
// reference in which every score is the k-ordered fmaf chain
//   s = fmaf(q[D-1], c[D-1], ... fmaf(q[0], c[0], 0))
// and the returned scores are those fp32 values.
//
// Screening bound.  A bf16 MFMA score s~ differs from the exact chain s by at
// most M_q = eps * |q| * max_c |c| with eps = 2^-7 + 2^-14: bf16 has 8
// significant bits, so round-to-nearest moves each operand by at most 2^-8 of
// itself and a product of two rounded operands by at most 2^-7 + 2^-16
// (summed over k: <= (2^-7 + 2^-16) sum_k |q_k c_k| <= ... |q| |c|); fp32
// accumulation of <= 128 exact bf16 products and the exact chain's own
// rounding add below 2^-17 each.  If tau is a lower bound of the
// K-th largest screened score, every member of the exact top-K has
// s~ >= tau - 2 M_q, so "s~ > next_down(tau - 2 M_q)" loses nothing.
//
// Design (MI355X):
//  screen (k <= 128, the bins path) — one workgroup = 8 waves x 32 queries;
//    the queries' bf16 fragments stay in VGPRs (B operand), 64-candidate
//    bf16 tiles stream through double-buffered, XOR-swizzled LDS with global
//    loads issued two tiles ahead, and are scored with
//    v_mfma_f32_32x32x16_bf16 (S^T: each lane holds 16 candidates of one
//    query).  Per register: one v_max into a per-lane "bin" (64 bins per lane,
//    128 per query, each the running maximum over a fixed residue class of
//    candidates) and one v_cmp against the query's threshold; survivors are
//    appended to a lane-private HBM shortlist (no atomics, no cross-lane
//    work).  At geometrically spaced tiles the lanes refresh their
//    threshold in parallel from the bins: the K-th largest of 128 bin maxima
//    (distinct candidates) is a lower bound of the K-th screened score.
//    Small query batches split the candidates over up to 8 workgroups per
//    query block (split = blockIdx % S keeps a split on fixed XCDs, so its
//    slice stays in that L2); splits share thresholds through a per-query
//    atomicMax.
//  screen (k > 128, the compaction path) — per-query wave shortlists compacted
//    by a bitwise K-th search when they fill.
//  finalize — one wave per query: shortlist entries above the final
//    threshold are gathered into LDS, cut by a coarse K-th search,
//    rescored with the exact fp32 fmaf chain, the exact top-K is selected on
//    (score, -index) and ranked with an LDS bitonic sort.  A query whose
//    shortlist cannot be bounded (massive near-ties) is answered by an exact
//    fp32 scan with the same machinery.
#include <cmath>

#include "tt_common.h"

// Probe hooks for tools/index_probe.hip (never defined in the library build):
//   TT_INDEX_STATS    count inserts / compactions / overflows
//   TT_INDEX_NOINSERT screening threshold pinned above every score
#ifdef TT_INDEX_STATS
__device__ unsigned long long g_index_stats[4];
#define TT_STAT(i, v) atomicAdd(&g_index_stats[i], static_cast<unsigned long long>(v))
#else
#define TT_STAT(i, v) ((void)0)
#endif

namespace tt {
namespace {

#ifndef TT_SCREEN_WAVES
#define TT_SCREEN_WAVES 8
#endif
constexpr int kScreenWaves = TT_SCREEN_WAVES;
constexpr int kScreenThreads = kScreenWaves * kWave;
constexpr int kQPerWave = 32;
constexpr int kQPerWG = kScreenWaves * kQPerWave;  // 256 queries
constexpr int kCTile = 64;                         // candidates per LDS tile
#ifndef TT_BINS
#define TT_BINS 64
#endif
constexpr int kBins = TT_BINS;                     // per lane (128 per query)
constexpr int kBinsMaxK = 2 * kBins;               // bins path serves k <= 128
#ifndef TT_LANE_CAP
#define TT_LANE_CAP 1024
#endif
constexpr int kLaneCap = TT_LANE_CAP;              // entries per (query, split, lane half)
constexpr int kMaxSplits = 8;
constexpr float kScreenEps = 0.00787353515625f;    // 2^-7 + 2^-14
constexpr int64_t kMaxChunk = 65536;               // queries per screening pass
#ifndef TT_SHORTLIST_BUDGET
#define TT_SHORTLIST_BUDGET (size_t(1) << 30)
#endif
constexpr size_t kShortlistBudget = TT_SHORTLIST_BUDGET;  // bytes of shortlists per pass

struct IndexHeader {
  int64_t n;
  int64_t n_pad;
  int32_t dim;
  int32_t D;
  unsigned maxnorm_bits;  // max_c |c|_2 as float bits (non-negative)
  unsigned pad[9];
};
static_assert(sizeof(IndexHeader) == 64, "header");

inline int pick_dpad(int dim) {
  if (dim <= 32) return 32;
  if (dim <= 64) return 64;
  if (dim <= 128) return 128;
  return 0;
}

inline int cap_for_k(int k) {
  int c = 1024;
  while (c < 2 * k + 2 * kCTile) c <<= 1;
  return c;
}

inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

size_t index_bytes(int64_t n, int dim) {
  const int D = pick_dpad(dim);
  const int64_t n_pad = round_up(n, kCTile);
  return 64 + static_cast<size_t>(n_pad) * D * 2 + static_cast<size_t>(n_pad) * 4;
}

__device__ __forceinline__ const __bf16* index_rows(const void* idx) {
  return reinterpret_cast<const __bf16*>(static_cast<const char*>(idx) + 64);
}
__device__ __forceinline__ const float* index_bias(const void* idx, int64_t n_pad, int D) {
  return reinterpret_cast<const float*>(static_cast<const char*>(idx) + 64 + n_pad * D * 2);
}

// ---- build ----------------------------------------------------------------
// Row-major bf16 image (zero padded to n_pad rows, D columns), bias (0 / -inf
// for padding rows) and max row norm (one atomic per workgroup of 64 rows).
constexpr int kBuildRowsPerWave = 16;
__global__ void __launch_bounds__(256) build_kernel(const float* __restrict__ cand, int64_t ldc, int64_t n, int dim,
                                                    int64_t n_pad, int D, void* index) {
  __shared__ float wmax[4];
  IndexHeader* hdr = static_cast<IndexHeader*>(index);
  __bf16* rows = reinterpret_cast<__bf16*>(static_cast<char*>(index) + 64);
  float* bias = reinterpret_cast<float*>(static_cast<char*>(index) + 64 + n_pad * D * 2);
  const int wave = threadIdx.x / kWave;
  const int lane = lane_id();
  float mx = 0.0f;
  for (int i = 0; i < kBuildRowsPerWave; ++i) {
    const int64_t r = (blockIdx.x * 4ll + wave) * kBuildRowsPerWave + i;
    if (r >= n_pad) break;
    float ss = 0.0f;
    for (int e2 = lane; e2 < D / 2; e2 += kWave) {
      const int e = 2 * e2;
      const float x0 = (r < n && e < dim) ? cand[r * ldc + e] : 0.0f;
      const float x1 = (r < n && e + 1 < dim) ? cand[r * ldc + e + 1] : 0.0f;
      ss = __builtin_fmaf(x0, x0, __builtin_fmaf(x1, x1, ss));
      reinterpret_cast<unsigned*>(rows + r * D)[e2] = pack_bf16x2(x0, x1);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, kWave);
    if (lane == 0) bias[r] = (r < n) ? 0.0f : -INFINITY;
    if (r < n) mx = fmaxf(mx, sqrtf(ss));
  }
  if (lane == 0) wmax[wave] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    // round the norm up so the bound stays an upper bound
    atomicMax(&hdr->maxnorm_bits, __float_as_uint(m * (1.0f + 1e-5f)));
    if (blockIdx.x == 0) {
      hdr->n = n;
      hdr->n_pad = n_pad;
      hdr->dim = dim;
      hdr->D = D;
    }
  }
}

// ---- query prep ----------------------------------------------------------
// bf16 rows [nq_pad, D] and the per-query screening margin 2*M_q.
__global__ void query_prep_kernel(const float* __restrict__ q, int64_t ldq, int64_t nq, int dim, int64_t nq_pad,
                                  int D, const void* index, __bf16* __restrict__ qb, float* __restrict__ margin2) {
  const int64_t r = blockIdx.x * 4ll + threadIdx.x / kWave;
  if (r >= nq_pad) return;
  const int lane = lane_id();
  float ss = 0.0f;
  bool nz = false;
  for (int e2 = lane; e2 < D / 2; e2 += kWave) {
    const int e = 2 * e2;
    const float x0 = (r < nq && e < dim) ? q[r * ldq + e] : 0.0f;
    const float x1 = (r < nq && e + 1 < dim) ? q[r * ldq + e + 1] : 0.0f;
    ss = __builtin_fmaf(x0, x0, __builtin_fmaf(x1, x1, ss));
    nz = nz || x0 != 0.0f || x1 != 0.0f;
    reinterpret_cast<unsigned*>(qb + r * D)[e2] = pack_bf16x2(x0, x1);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, kWave);
  const bool nonzero = __ballot(nz) != 0;
  if (lane == 0) {
    const float maxc = __uint_as_float(static_cast<const IndexHeader*>(index)->maxnorm_bits);
    const float qn = sqrtf(ss) * (1.0f + 1e-5f);
    // 2 * eps * |q| * max|c|, rounded up; tiny absolute floor for subnormals.
    // A zero query scores exactly +0 against every candidate in both paths, so
    // its margin is 0 and ties resolve by index.
    margin2[r] = (r < nq && nonzero) ? (2.0f * kScreenEps * qn * maxc) * (1.0f + 1e-5f) + 1e-30f : 0.0f;
  }
}

__device__ __forceinline__ unsigned long long make_key(float s, unsigned idx) {
  return (static_cast<unsigned long long>(float_order_key(s)) << 32) |
         static_cast<unsigned long long>(0xFFFFFFFFu - idx);
}

// Largest float strictly below x (x finite).
__device__ __forceinline__ float next_down(float x) {
  if (x == 0.0f) return -__uint_as_float(1u);
  const unsigned u = __float_as_uint(x);
  return __uint_as_float(x > 0.0f ? u - 1u : u + 1u);
}

__device__ __forceinline__ uint64_t lanemask_lt64() {
  const int l = lane_id();
  return (l == 0) ? 0ull : (~0ull >> (64 - l));
}

// Largest v such that at least K of the wave's keys are >= v (keys distinct:
// the K-th largest).  Keys of empty slots are 0.
template <int NPL>
__device__ unsigned long long kth_largest(const unsigned long long (&key)[NPL], int K) {
  unsigned long long res = 0;
#pragma unroll 1
  for (int bit = 63; bit >= 0; --bit) {
    const unsigned long long cand = res | (1ull << bit);
    int c = 0;
#pragma unroll
    for (int i = 0; i < NPL; ++i) c += __popcll(__ballot(key[i] >= cand));
    if (c >= K) res = cand;
  }
  return res;
}

// ---- screen, bins path (k <= 128) -------------------------------------------
struct ScreenArgs {
  const void* index;
  const __bf16* qb;      // [nq_pad, D]
  const float* margin2;  // [nq_pad]
  int64_t nq;            // real queries in this chunk
  int64_t n;             // real candidates (rows >= n are zero padding)
  int64_t n_pad;
  int k;
  int S;                 // candidate splits
  int R;                 // entries per (query, split, half) region
  uint2* buf;            // [nq_pad][S][2][R] (score bits, candidate)
  int* count;            // [nq_pad][S][2]; -1 = region overflowed
  unsigned* thr;         // [nq_pad] order key of a valid strict threshold (0 = none)
};

// s_waitcnt with only the vector-memory counter constrained (gfx9 encoding).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// Keeps the entries of region[0..n) scoring above thr; returns their count.
__device__ __noinline__ int compact_region(uint2* region, int n, float thr) {
  int m = 0;
  for (int j0 = 0; j0 < n; j0 += 16) {
    uint2 e[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) e[u] = (j0 + u < n) ? region[j0 + u] : make_uint2(0u, 0u);
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (j0 + u < n && __uint_as_float(e[u].x) > thr) region[m++] = e[u];
  }
  return m;
}

constexpr int kStages = 4;     // LDS ring: tile i computed while tiles i+1..i+3 land
#ifndef TT_WARM_TILES
#define TT_WARM_TILES 64
#endif
constexpr int kWarmTiles = TT_WARM_TILES;  // bins-only warm-up tiles per split (4096 candidates)

template <int D>
__global__ void __launch_bounds__(kScreenThreads) screen_bins_kernel(const ScreenArgs a) {
  constexpr int KS = D / 16, CH = D / 8, RB = D * 2;
  constexpr int TILE_BYTES = kCTile * RB;                 // 16 KiB at D = 128
  constexpr int PIECES = TILE_BYTES / 1024;               // 1 KiB LDS-DMA pieces per tile
  constexpr int PPW = PIECES >= kScreenWaves ? PIECES / kScreenWaves : 1;
  __shared__ __attribute__((aligned(1024))) char smem[kStages * TILE_BYTES];  // tile ring (LDS-DMA)
  const int tid = threadIdx.x;
  const int wave = tid / kWave;
  const int lane = lane_id();
  const int h = lane >> 5, l32 = lane & 31;
  const int split = static_cast<int>(blockIdx.x % a.S);
  const int64_t qg = static_cast<int64_t>(blockIdx.x / a.S) * kQPerWG + wave * kQPerWave + l32;
  const int ntiles = static_cast<int>(a.n_pad / kCTile);
  const int per = (ntiles + a.S - 1) / a.S;
  const int tb = split * per;
  const int nt = max(min(ntiles, tb + per) - tb, 0);
  const __bf16* crow = index_rows(a.index);
  const bool my_pieces = wave * PPW < PIECES;  // D = 32: waves 4..7 stage nothing

  bf16x8 bfrag[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) bfrag[s] = *reinterpret_cast<const bf16x8*>(a.qb + qg * D + 16 * s + 8 * h);
  const float m2 = a.margin2[qg];
  wait_vmcnt<0>();  // ordinary loads retired before the LDS-DMA ring starts
  const bool live = qg < a.nq;
  float thr = live ? -INFINITY : INFINITY;  // insertion threshold (strict)
  float gthr = -INFINITY;                   // best globally valid strict threshold
  float bins[kBins];
#pragma unroll
  for (int i = 0; i < kBins; ++i) bins[i] = -INFINITY;
  uint2* region = a.buf + ((qg * a.S + split) * 2 + h) * static_cast<int64_t>(a.R);
  int cnt = 0;
  bool ovf = false;

  // LDS image of a tile: row-major RB-byte rows, 16-B chunks XOR-swizzled by
  // row; the swizzle is applied to the per-lane SOURCE address so that every
  // 1 KiB DMA piece lands lane-linear.
  auto issue = [&](int tile, int stage) {
    const int64_t base = static_cast<int64_t>(tile) * kCTile;
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const int p = wave * PPW + u;
      if (p < PIECES) {
        const int off = p * 1024 + lane * 16;
        const int row = off / RB, chp = (off % RB) / 16;
        const int ch = chp ^ ((row * CH / 16) % CH);
        const __bf16* src = crow + (base + row) * D + ch * 8;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src),
                                         (__attribute__((address_space(3))) void*)(smem + stage * TILE_BYTES + p * 1024),
                                         16, 0, 0);
      }
    }
  };
  // wait until at most `ahead` tiles of this wave's DMA are still in flight
  auto wait_tiles = [&](int ahead) {
    if (!my_pieces || ahead <= 0) {
      wait_vmcnt<0>();
    } else if (ahead == 1) {
      wait_vmcnt<PPW>();
    } else {
      wait_vmcnt<2 * PPW>();
    }
  };

  // Lane-parallel threshold refresh: K-th largest of the pair's 128 bins by a
  // 16-bit prefix search of their order keys (a lower bound of the K-th).
  auto refresh = [&](bool warm) {
    unsigned res = 0;
#pragma unroll 1
    for (int bit = 15; bit >= 0; --bit) {
      const unsigned c = res | (1u << bit);
      const float f = order_key_float(c << 16);  // smallest float with this key prefix (NaN: none)
      int n = 0;
#pragma unroll
      for (int i = 0; i < kBins; ++i) n += (bins[i] >= f) ? 1 : 0;
      n += __shfl_xor(n, 32, kWave);
      if (n >= a.k) res = c;
    }
    const float tau = order_key_float(res << 16);
    // A zero query (m2 == 0, every score exactly 0) relies on a strict local
    // threshold that is valid only for candidates after the certifying ones;
    // the warm-up tiles are scanned again, so it skips the warm-up threshold
    // and restarts its bins.
    if (warm && m2 == 0.0f) {
#pragma unroll
      for (int i = 0; i < kBins; ++i) bins[i] = -INFINITY;
    } else if (tau > -INFINITY && tau < INFINITY) {
      const float local = m2 > 0.0f ? next_down(tau - m2) : tau;
      const float pub = m2 > 0.0f ? local : next_down(tau);
      gthr = fmaxf(gthr, pub);
      thr = fmaxf(thr, local);
    }
    if (a.S > 1) {
      unsigned g = float_order_key(gthr);
      if (h == 0 && live) g = max(g, atomicMax(&a.thr[qg], g));
      const unsigned g2 = __shfl_xor(g, 32, kWave);
      gthr = fmaxf(gthr, order_key_float(g2 > g ? g2 : g));
      thr = fmaxf(thr, gthr);
    }
    thr = fmaxf(thr, __shfl_xor(thr, 32, kWave));
#ifdef TT_INDEX_NOINSERT
    thr = 3.0e38f;
#endif
  };

  // A lane whose region is nearly full drops the entries the globally valid
  // threshold rules out (the strict local one of a zero-margin query is only
  // valid for later candidates); if that does not make room the query is
  // answered by the exact fallback.
  auto self_compact = [&]() {
    if (cnt > a.R - 2 * 16) {
      cnt = compact_region(region, cnt, gthr);
      TT_STAT(1, 1);
      if (cnt > a.R - 2 * 16) {
        ovf = true;
        thr = INFINITY;
        TT_STAT(2, 1);
      }
    }
  };

  // Warm-up: the first `pre` tiles of the split are scanned once for the bins
  // only (no inserts), so the insertion threshold starts near the top few
  // percent instead of at -inf; then the split is scanned from its start.
  // Virtual tile v < pre is tile tb + v, v >= pre is tile tb + v - pre.
  // pre is a multiple of 4 so a tile re-scanned after the warm-up lands in the
  // same bins (Q = v & 3): every bin stays a maximum over distinct candidates.
  const int pre = min(kWarmTiles, nt / 4) & ~3;
  const int nv = pre + nt;
  auto vtile = [&](int v) { return tb + (v < pre ? v : v - pre); };
#pragma unroll
  for (int s = 0; s < kStages - 1; ++s)
    if (s < nv) issue(vtile(s), s);
  wait_tiles(min(nv, kStages - 1) - 1);
  __builtin_amdgcn_s_barrier();

  // Software pipeline at 32-candidate block granularity: the 8 MFMAs of a
  // block are issued with the filter of the previous block (bins, threshold
  // test, inserts) in their issue gaps.
  // Tile v: [MFMA(v,0) | filter(v-1,1)] then [MFMA(v,1) | filter(v,0)].
  // Q = v & 3 selects a tile's bins (static under the unroll by 4).
  constexpr int PPS = 8 / KS;  // filter pairs per MFMA slot
  f32x16 accf = {};            // block waiting to be filtered: tile v-1, block 1
  int64_t cbase_f = 0;         // first candidate of that tile
  bool scan_f = false;

  auto filter_pair = [&](const f32x16& acc, const int Qb, const int t, const int pr, int64_t cbase, float tins) {
    const float x = acc[2 * pr], y = acc[2 * pr + 1];
    const float pm = __builtin_elementwise_maximum(x, y);
    constexpr int NQ = kBins / 16;  // tile parities with their own bins
    bins[(Qb % NQ) * 16 + t * 8 + pr] = __builtin_elementwise_maximum(bins[(Qb % NQ) * 16 + t * 8 + pr], pm);
#ifndef TT_PROBE_LIGHT
    if (pm > tins) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float val = u ? y : x;
        const int r = 2 * pr + u;
        if (val > tins) {
          const unsigned cidx = static_cast<unsigned>(cbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h);
          region[cnt] = make_uint2(__float_as_uint(val), cidx);
          ++cnt;
          TT_STAT(0, 1);
        }
      }
    }
#endif
  };
  auto mask_pad = [&](f32x16& acc, const int t, int64_t cbase) {  // zero padding rows of the last tile
    if (cbase + kCTile > a.n) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (cbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h >= a.n) acc[r] = -INFINITY;
    }
  };
  // after the filter of main-scan tile j-1: refresh on a geometric schedule;
  // j == 1 (pre > 0) is the first refresh after the warm-up tiles.
  auto after_filter = [&](int j) {
    const bool warm = pre > 0 && j == 1;
    const bool due = warm || (j >= 2 && (j & (j - 1)) == 0) || (j > 0 && j % 128 == 0);
    const bool full = __any(cnt > a.R - 2 * 32);
    if (due || full) refresh(warm);
    if (full) self_compact();
  };

  auto tile_body = [&](int v, const int Q) {
    const int Qp = (Q + 3) & 3;
    if (v + kStages - 1 < nv) issue(vtile(v + kStages - 1), (v + kStages - 1) % kStages);
#ifdef TT_PROBE_NOLDS
    const char* B = smem;  // probe: always the same stage (fragments stay cached)
#else
    const char* B = smem + (v % kStages) * TILE_BYTES;
#endif
    const int64_t cbase = static_cast<int64_t>(vtile(v)) * kCTile;
    const bool scan = v >= pre;
    const bool have_prev = v > 0;
    const float tins_f = scan_f ? thr : INFINITY;
    if (have_prev) mask_pad(accf, 1, cbase_f);
    f32x16 acc0 = {}, acc1 = {};
    auto block0 = [&](const bool with_filter) {  // block 0 of tile v | filter block 1 of tile v-1
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int row = l32, ch = 2 * s + h;
        const int swz = (row * CH / 16) % CH;
#ifdef TT_PROBE_REGA
        const bf16x8 af = bfrag[(s + 1) % KS];  // probe: no LDS reads
#else
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(B + row * RB + ((ch ^ swz) << 4));
#endif
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfrag[s], acc0, 0, 0, 0);
        if (with_filter) {
#pragma unroll
          for (int u = 0; u < PPS; ++u) filter_pair(accf, Qp, 1, s * PPS + u, cbase_f, tins_f);
        }
      }
    };
    if (have_prev) {
      block0(true);
      after_filter(v - pre);
    } else {
      block0(false);
    }
    mask_pad(acc0, 0, cbase);
    const float tins = scan ? thr : INFINITY;
#pragma unroll
    for (int s = 0; s < KS; ++s) {  // block 1 of tile v | filter block 0 of tile v
      const int row = 32 + l32, ch = 2 * s + h;
      const int swz = (row * CH / 16) % CH;
#ifdef TT_PROBE_REGA
      const bf16x8 af = bfrag[(s + 2) % KS];  // probe: no LDS reads
#else
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(B + row * RB + ((ch ^ swz) << 4));
#endif
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfrag[s], acc1, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < PPS; ++u) filter_pair(acc0, Q, 0, s * PPS + u, cbase, tins);
    }
    accf = acc1;
    cbase_f = cbase;
    scan_f = scan;
#ifndef TT_PROBE_NOBARRIER
    if (v + 1 < nv) wait_tiles(min(v + kStages - 1, nv - 1) - (v + 1));  // tile v+1 landed
    __builtin_amdgcn_s_barrier();
#endif
  };

#ifdef TT_PROBE_NOUNROLL
  for (int v = 0; v < nv; ++v) tile_body(v, 0);  // probe: one code copy (bins aliased)
#else
  for (int v = 0; v < nv; v += 4) {
    tile_body(v, 0);
    if (v + 1 < nv) tile_body(v + 1, 1);
    if (v + 2 < nv) tile_body(v + 2, 2);
    if (v + 3 < nv) tile_body(v + 3, 3);
  }
#endif
  if (nv > 0) {  // drain: filter the last block, final refresh
    mask_pad(accf, 1, cbase_f);
    const int Ql = (nv - 1) & 3;
    const float tins_f = scan_f ? thr : INFINITY;
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) {
      switch (Ql) {  // static bin index per case
        case 0: filter_pair(accf, 0, 1, pr, cbase_f, tins_f); break;
        case 1: filter_pair(accf, 1, 1, pr, cbase_f, tins_f); break;
        case 2: filter_pair(accf, 2, 1, pr, cbase_f, tins_f); break;
        default: filter_pair(accf, 3, 1, pr, cbase_f, tins_f); break;
      }
    }
    refresh(false);
  }
  a.count[(qg * a.S + split) * 2 + h] = ovf ? -1 : cnt;
  if (h == 0 && live && gthr > -INFINITY) atomicMax(&a.thr[qg], float_order_key(gthr));
}

// ---- screen, compaction path (k > 128) ---------------------------------------
struct ScreenCArgs {
  const void* index;
  const __bf16* qb;
  const float* margin2;
  int64_t nq;
  int64_t n_pad;
  int k;
  int cap;
  uint2* buf;    // [nq_pad][cap]
  int* count;    // [nq_pad]; -1 = overflow
};

// Compacts the shortlist buf[0..n) of one query with the whole wave.  Keeps
// every entry that might still belong to the exact top-K given screened
// scores within +-M of the exact ones (margin2 = 2M).  n <= 64*NPL.
template <int NPL>
__device__ int compact_shortlist(uint2* buf, int n, int K, float margin2, float* thr_out) {
  const int lane = lane_id();
  unsigned long long key[NPL];
  uint2 ent[NPL];
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int j = i * kWave + lane;
    ent[i] = (j < n) ? buf[j] : make_uint2(0u, 0u);
    key[i] = (j < n) ? make_key(__uint_as_float(ent[i].x), ent[i].y) : 0ull;
  }
  if (n <= K) {
    *thr_out = -INFINITY;
    return n;
  }
  const unsigned long long kk = kth_largest<NPL>(key, K);
  const float sK = order_key_float(static_cast<unsigned>(kk >> 32));
  const unsigned idxK = 0xFFFFFFFFu - static_cast<unsigned>(kk & 0xFFFFFFFFull);
  float thr = sK - margin2;
  if (margin2 > 0.0f) thr = next_down(thr);
  int out = 0;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int j = i * kWave + lane;
    const float s = __uint_as_float(ent[i].x) + 0.0f;
    const bool keep = (j < n) && (s > thr || (s == thr && ent[i].y <= idxK));
    const uint64_t m = __ballot(keep);
    if (keep) buf[out + __popcll(m & lanemask_lt64())] = ent[i];
    out += __popcll(m);
  }
  __threadfence_block();
  *thr_out = thr;
  return out;
}

template <int D, int NPL>
__global__ void __launch_bounds__(kScreenThreads) screen_compact_kernel(const ScreenCArgs a) {
  constexpr int KS = D / 16, CH = D / 8;
  constexpr int A_BYTES = kCTile * D * 2;
  constexpr int BUF_BYTES = A_BYTES + kCTile * 4;
  constexpr int CPT = (kCTile * CH + kScreenThreads - 1) / kScreenThreads;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES];
  __shared__ int cnt_s[kQPerWG];
  __shared__ float thr_s[kQPerWG];
  const int tid = threadIdx.x;
  const int wave = tid / kWave;
  const int lane = lane_id();
  const int h = lane >> 5, l32 = lane & 31;
  const int ql = wave * kQPerWave + l32;
  const int64_t qg = static_cast<int64_t>(blockIdx.x) * kQPerWG + ql;
  const __bf16* crow = index_rows(a.index);
  const float* cbias = index_bias(a.index, a.n_pad, D);

  bf16x8 bfrag[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) bfrag[s] = *reinterpret_cast<const bf16x8*>(a.qb + qg * D + 16 * s + 8 * h);
  const float margin2 = a.margin2[qg];
  if (tid < kQPerWG) {
    const int64_t q = static_cast<int64_t>(blockIdx.x) * kQPerWG + tid;
    cnt_s[tid] = 0;
    thr_s[tid] = (q < a.nq) ? -INFINITY : INFINITY;
  }
  uint2* mybuf_base = a.buf + (static_cast<int64_t>(blockIdx.x) * kQPerWG + wave * kQPerWave) * a.cap;
  bool ovf = false;

  u32x4 ra[CPT];
  float rb = 0.0f;
  auto gload = [&](int64_t base) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + kScreenThreads * i;
      if (c < kCTile * CH) {
        const int row = c / CH, ch = c % CH;
        ra[i] = *reinterpret_cast<const u32x4*>(crow + (base + row) * D + ch * 8);
      }
    }
    if (tid < kCTile) rb = cbias[base + tid];
  };
  auto lstore = [&](int b) {
    char* B = smem + b * BUF_BYTES;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + kScreenThreads * i;
      if (c < kCTile * CH) {
        const int row = c / CH, ch = c % CH;
        const int swz = (row * CH / 16) % CH;
        *reinterpret_cast<u32x4*>(B + row * (CH * 16) + ((ch ^ swz) << 4)) = ra[i];
      }
    }
    if (tid < kCTile) reinterpret_cast<float*>(B + A_BYTES)[tid] = rb;
  };

  const int ntiles = static_cast<int>(a.n_pad / kCTile);
  gload(0);
  lstore(0);
  __syncthreads();
  float thr = thr_s[ql];

  for (int tile = 0; tile < ntiles; ++tile) {
    const int cur = tile & 1;
    const bool more = tile + 1 < ntiles;
    if (more) gload(static_cast<int64_t>(tile + 1) * kCTile);
    const char* B = smem + cur * BUF_BYTES;
    const float* bias = reinterpret_cast<const float*>(B + A_BYTES);

    const bool need = cnt_s[ql] > a.cap - kCTile;
    uint64_t needm = __ballot(need) & 0xFFFFFFFFull;
    if (needm) __threadfence_block();
    while (needm) {
      const int qq = __ffsll(static_cast<long long>(needm)) - 1;
      needm &= needm - 1;
      const float mq = __shfl(margin2, qq, kWave);
      float nthr;
      const int nc = compact_shortlist<NPL>(mybuf_base + static_cast<int64_t>(qq) * a.cap,
                                            cnt_s[wave * kQPerWave + qq], a.k, mq, &nthr);
      if (lane == 0) {
        if (nc > a.cap - kCTile) {  // cannot make room: exact fallback in finalize
          cnt_s[wave * kQPerWave + qq] = 0;
          thr_s[wave * kQPerWave + qq] = INFINITY;
        } else {
          cnt_s[wave * kQPerWave + qq] = nc;
          thr_s[wave * kQPerWave + qq] = nthr;
        }
      }
      if (nc > a.cap - kCTile && l32 == qq) ovf = true;
      __builtin_amdgcn_wave_barrier();
    }
    thr = thr_s[ql];

    const int64_t cbase = static_cast<int64_t>(tile) * kCTile;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 acc;
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias + 32 * t + 8 * r4 + 4 * h);
        acc[4 * r4 + 0] = b4[0];
        acc[4 * r4 + 1] = b4[1];
        acc[4 * r4 + 2] = b4[2];
        acc[4 * r4 + 3] = b4[3];
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int row = 32 * t + l32, ch = 2 * s + h;
        const int swz = (row * CH / 16) % CH;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(B + row * (CH * 16) + ((ch ^ swz) << 4));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfrag[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool hit = acc[r] > thr;
        if (__any(hit)) {
          if (hit) {
            const int slot = atomicAdd(&cnt_s[ql], 1);
            const unsigned cidx = static_cast<unsigned>(cbase + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h);
            mybuf_base[static_cast<int64_t>(l32) * a.cap + slot] = make_uint2(__float_as_uint(acc[r]), cidx);
          }
        }
      }
    }
    if (more) lstore(cur ^ 1);
    __syncthreads();
  }
  if (h == 0) a.count[qg] = ovf ? -1 : cnt_s[ql];
}

// ---- finalize ------------------------------------------------------------
// Exact score: k-ordered fmaf chain over the fp32 rows (dim real columns).
// qs is the query row in LDS (broadcast reads); the candidate row is loaded in
// batches (16 x float4 or 16 scalars in flight) ahead of the dependent chain.
__device__ __forceinline__ float exact_score(const float* __restrict__ qs, const float* __restrict__ c, int dim,
                                             bool vec4) {
  float acc = 0.0f;
  if (vec4) {  // c 16-byte aligned, dim % 4 == 0
    for (int e0 = 0; e0 < dim; e0 += 64) {
      f32x4 v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (e0 + 4 * i < dim) v[i] = *reinterpret_cast<const f32x4*>(c + e0 + 4 * i);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (e0 + 4 * i < dim) {
#pragma unroll
          for (int u = 0; u < 4; ++u) acc = __builtin_fmaf(qs[e0 + 4 * i + u], v[i][u], acc);
        }
    }
  } else {
    for (int e0 = 0; e0 < dim; e0 += 16) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = (e0 + i < dim) ? c[e0 + i] : 0.0f;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (e0 + i < dim) acc = __builtin_fmaf(qs[e0 + i], v[i], acc);
    }
  }
  return acc;
}

struct FinalArgs {
  const float* q;  // fp32 queries of this chunk
  int64_t ldq;
  const float* cand;
  int64_t ldc;
  int64_t n;
  int dim;
  int k;
  int S;     // splits
  int H;     // regions per split (2 bins path, 1 compaction path)
  int R;     // entries per region
  int L;     // LDS list capacity
  int P;     // bitonic sort size (pow2 >= k)
  int vec4;  // candidate rows are 16-byte aligned float4 rows
  int pairs; // entries are (max of candidates c, c+1; c) pairs (bins path)
  int64_t nq;
  int64_t index_offset;
  const float* margin2;
  const uint2* buf;
  const int* count;
  const unsigned* thr;  // null for the compaction path
  float* out_s;
  int32_t* out_i;
};

// Keeps list entries with sc > thr (in place, whole wave).  Returns the count.
__device__ __forceinline__ int filter_list(float* sc, unsigned* id, int n, float thr) {
  int out = 0;
  for (int j0 = 0; j0 < n; j0 += kWave) {
    const int j = j0 + lane_id();
    const float s = j < n ? sc[j] : 0.0f;
    const unsigned i = j < n ? id[j] : 0u;
    const bool keep = j < n && s > thr;
    const uint64_t m = __ballot(keep);
    __syncthreads();  // all reads of this chunk before any write into it
    if (keep) {
      const int p = out + __popcll(m & lanemask_lt64());
      sc[p] = s;
      id[p] = i;
    }
    out += __popcll(m);
  }
  __syncthreads();
  return out;
}

// Radix select on the list's score order keys with 8-bit digits and an LDS
// histogram (one wave): after `passes` digits, `prefix` holds the top
// 8*passes bits of the K-th largest key, `above` = #keys whose top bits are
// greater, `at` = #keys sharing the prefix (above < K <= above + at).
struct Kth {
  unsigned prefix;
  int above;
  int at;
};

__device__ Kth radix_select(const float* sc, int n, int K, int passes, unsigned* hist) {
  const int lane = lane_id();
  unsigned prefix = 0;
  int above = 0, at = n;
  for (int d = 0; d < passes; ++d) {
    const int shift = 24 - 8 * d;
    const unsigned hi_mask = d == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
#pragma unroll
    for (int u = 0; u < 4; ++u) hist[4 * lane + u] = 0;
    __syncthreads();
    for (int j = lane; j < n; j += kWave) {
      const unsigned key = float_order_key(sc[j]);
      if ((key & hi_mask) == prefix) atomicAdd(&hist[(key >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    // counts at or above each bin: lane L owns bins 4L..4L+3
    unsigned h4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) h4[u] = hist[4 * lane + u];
    const unsigned mine = h4[0] + h4[1] + h4[2] + h4[3];
    unsigned suffix = mine;  // inclusive suffix sum over lanes >= L
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const unsigned o = __shfl_down(suffix, off, kWave);
      if (lane + off < kWave) suffix += o;
    }
    unsigned cum[4];  // keys in bins >= 4L+u (within the prefix)
    cum[3] = suffix - mine + h4[3];
    cum[2] = cum[3] + h4[2];
    cum[1] = cum[2] + h4[1];
    cum[0] = cum[1] + h4[0];
    const int need = K - above;
    int best = -1;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (static_cast<int>(cum[u]) >= need) best = 4 * lane + u;
    const uint64_t m = __ballot(best >= 0);
    const int src = 63 - __clzll(m);
    const int b = __shfl(best, src, kWave);
    const int u = b & 3;
    const unsigned cb = __shfl(cum[0], src, kWave), cb1 = __shfl(cum[1], src, kWave),
                   cb2 = __shfl(cum[2], src, kWave), cb3 = __shfl(cum[3], src, kWave);
    const unsigned cumb = u == 0 ? cb : u == 1 ? cb1 : u == 2 ? cb2 : cb3;
    const unsigned hb = hist[b];
    above += static_cast<int>(cumb - hb);
    at = static_cast<int>(hb);
    prefix |= static_cast<unsigned>(b) << shift;
    __syncthreads();
  }
  return Kth{prefix, above, at};
}

// Screened cut: tau = lower bound of the K-th largest screened score (16-bit
// key prefix); keeps s > next_down(tau - margin2).  Raises *thr.
__device__ int coarse_cut(float* sc, unsigned* id, int n, int K, float margin2, float* thr, unsigned* hist) {
  if (n <= K) return n;
  const Kth r = radix_select(sc, n, K, 2, hist);
  const float tau = order_key_float(r.prefix);
  if (!(tau > -INFINITY)) return n;
  const float t = next_down(margin2 > 0.0f ? tau - margin2 : tau);
  if (t <= *thr) return n;
  *thr = t;
  return filter_list(sc, id, n, t);
}

// Exact selection: keeps exactly the K best entries by (score desc, index
// asc); *thr = the K-th score (later candidates of an in-order scan need a
// strictly larger score).
__device__ int exact_select(float* sc, unsigned* id, int n, int K, float* thr, unsigned* hist) {
  if (n <= K) {
    *thr = -INFINITY;
    return n;
  }
  const Kth r = radix_select(sc, n, K, 4, hist);
  const unsigned res = r.prefix;  // exact key of the K-th score
  const int need = K - r.above;   // ties at the K-th score to keep, lowest indices first
  unsigned cut = 0xFFFFFFFFu;
  if (need < r.at) {
    // need-th smallest index among the ties: largest v with #(idx < v) < need
    unsigned v = 0;
#pragma unroll 1
    for (int bit = 31; bit >= 0; --bit) {
      const unsigned c = v | (1u << bit);
      int lt = 0;
      for (int j0 = 0; j0 < n; j0 += kWave) {
        const int j = j0 + lane_id();
        lt += __popcll(__ballot(j < n && float_order_key(sc[j]) == res && id[j] < c));
      }
      if (lt < need) v = c;
    }
    cut = v;
  }
  int out = 0;
  for (int j0 = 0; j0 < n; j0 += kWave) {
    const int j = j0 + lane_id();
    const float s = j < n ? sc[j] : 0.0f;
    const unsigned i = j < n ? id[j] : 0u;
    const unsigned key = float_order_key(s);
    const bool keep = j < n && (key > res || (key == res && i <= cut));
    const uint64_t m = __ballot(keep);
    __syncthreads();
    if (keep) {
      const int p = out + __popcll(m & lanemask_lt64());
      sc[p] = s;
      id[p] = i;
    }
    out += __popcll(m);
  }
  __syncthreads();
  *thr = order_key_float(res);
  return out;
}

__global__ void __launch_bounds__(kWave) finalize_kernel(const FinalArgs a) {
  extern __shared__ __attribute__((aligned(16))) char fsm[];
  float* qs = reinterpret_cast<float*>(fsm);  // query row (dim <= 128)
  float* sc = qs + 128;
  unsigned* id = reinterpret_cast<unsigned*>(sc + a.L);
  unsigned long long* sk = reinterpret_cast<unsigned long long*>(id + a.L);
  unsigned* hist = reinterpret_cast<unsigned*>(sk + a.P);  // 256 radix bins
  const int64_t q = blockIdx.x;
  const int lane = lane_id();
#ifdef TT_INDEX_NOINSERT
  return;  // probe build: the screen inserted nothing
#endif
  for (int e = lane; e < a.dim; e += kWave) qs[e] = a.q[q * a.ldq + e];
  const float m2 = a.margin2[q];
  float thr = (a.thr && a.thr[q]) ? order_key_float(a.thr[q]) : -INFINITY;
  const int nreg = a.S * a.H;
  bool ovf = false;
  for (int r = 0; r < nreg; ++r) ovf = ovf || a.count[q * nreg + r] < 0;
  __syncthreads();

  int n = 0;
  if (!ovf) {
    // Gather the entries above the final threshold; cut whenever the list fills.
    for (int r = 0; r < nreg && !ovf; ++r) {
      const int c = a.count[q * nreg + r];
      const uint2* reg = a.buf + (q * nreg + r) * static_cast<int64_t>(a.R);
      for (int j0 = 0; j0 < c && !ovf; j0 += 4 * kWave) {
        uint2 e[4];  // four chunks in flight
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + u * kWave + lane;
          e[u] = j < c ? reg[j] : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + u * kWave + lane;
          const float s = __uint_as_float(e[u].x);
          const bool keep = j < c && s > thr;
          const uint64_t m = __ballot(keep);
          if (keep) {
            const int p = n + __popcll(m & lanemask_lt64());
            sc[p] = s;
            id[p] = e[u].y;
          }
          n += __popcll(m);
          if (n > a.L - kWave) {
            __syncthreads();
            if (m2 > 0.0f) {
              n = coarse_cut(sc, id, n, a.k, m2, &thr, hist);
            } else {  // zero query: screened scores are exact, cut ties by index
              float t;
              n = exact_select(sc, id, n, a.k, &t, hist);
              thr = fmaxf(thr, next_down(t));
            }
            if (n > a.L - kWave) {
              ovf = true;
              break;
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if (!ovf) {
    n = coarse_cut(sc, id, n, a.k, m2, &thr, hist);
    ovf = n < a.k;  // cannot happen with a valid screen; answer exactly regardless
  }
  if (!ovf && a.pairs) {
    // expand pair entries into their two candidates (c, c + 1), top chunk first
    if (2 * n > a.L) {
      ovf = true;
    } else {
      for (int j0 = (n - 1) / kWave * kWave; j0 >= 0; j0 -= kWave) {
        const int j = j0 + lane;
        const unsigned c = j < n ? id[j] : 0u;
        __syncthreads();
        if (j < n) {
          id[2 * j] = c;
          id[2 * j + 1] = c + 1;
        }
        __syncthreads();
      }
      n *= 2;
    }
  }
  if (!ovf) {
    for (int j = lane; j < n; j += kWave) {
      const unsigned c = id[j];
      sc[j] = c < static_cast<uint64_t>(a.n)
                  ? exact_score(qs, a.cand + static_cast<int64_t>(c) * a.ldc, a.dim, a.vec4 != 0) + 0.0f
                  : -INFINITY;  // c + 1 past the last candidate
    }
    __syncthreads();
  } else {
    // Exact fallback: scan every candidate with the fp32 chain (in index
    // order, so a strict threshold at the K-th score is exact).
    float ethr = -INFINITY;
    n = 0;
    for (int64_t c0 = 0; c0 < a.n; c0 += kWave) {
      const int64_t c = c0 + lane;
      float s = -INFINITY;
      if (c < a.n) s = exact_score(qs, a.cand + c * a.ldc, a.dim, a.vec4 != 0) + 0.0f;
      const bool keep = c < a.n && s > ethr;
      const uint64_t m = __ballot(keep);
      if (keep) {
        const int p = n + __popcll(m & lanemask_lt64());
        sc[p] = s;
        id[p] = static_cast<unsigned>(c);
      }
      n += __popcll(m);
      if (n > a.L - kWave) {
        __syncthreads();
        n = exact_select(sc, id, n, a.k, &ethr, hist);
      }
    }
    __syncthreads();
  }
  float kth;
  n = exact_select(sc, id, n, a.k, &kth, hist);
  // Rank: bitonic sort of (score, -index) keys, descending.
  for (int j = lane; j < a.P; j += kWave) sk[j] = j < n ? make_key(sc[j], id[j]) : 0ull;
  for (int size = 2; size <= a.P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = lane; i < a.P / 2; i += kWave) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const unsigned long long x = sk[lo], y = sk[hi];
        if ((x < y) == desc) {
          sk[lo] = y;
          sk[hi] = x;
        }
      }
    }
  }
  __syncthreads();
  for (int t = lane; t < a.k; t += kWave) {
    const unsigned long long key = sk[t];
    a.out_s[q * a.k + t] = order_key_float(static_cast<unsigned>(key >> 32));
    a.out_i[q * a.k + t] =
        static_cast<int32_t>(static_cast<int64_t>(0xFFFFFFFFu - static_cast<unsigned>(key)) + a.index_offset);
  }
}

// ---- host plan -------------------------------------------------------------
struct SearchPlan {
  bool bins;
  int S, H, R, L, P;
  int64_t chunk;
};

SearchPlan plan_search(int64_t nq, int64_t n_cand, int k) {
  SearchPlan p{};
  const int64_t ntiles = ceil_div(n_cand, kCTile);
  p.P = next_pow2(k < 2 ? 2 : k);
  p.bins = k <= kBinsMaxK;
  p.H = p.bins ? 2 : 1;
  p.R = p.bins ? kLaneCap : cap_for_k(k);
  p.L = p.bins ? 1024 : (p.R > 2048 ? p.R : 2048);
  p.S = 1;
  p.chunk = nq < kMaxChunk ? (nq > 0 ? nq : 1) : kMaxChunk;
  for (int pass = 0; pass < 3; ++pass) {
    if (p.bins) {  // enough workgroups for the chip: split the candidates of few query blocks
      const int64_t qblocks = ceil_div(p.chunk, kQPerWG);
      p.S = 1;
      while (p.S < kMaxSplits && qblocks * p.S * kScreenWaves < 2048 && ntiles / (2 * p.S) >= 64) p.S *= 2;
#ifdef TT_FORCE_SPLITS
      p.S = TT_FORCE_SPLITS;
#endif
    }
    const size_t per_query = static_cast<size_t>(p.S) * p.H * p.R * sizeof(uint2);
    int64_t chunk = static_cast<int64_t>(kShortlistBudget / per_query) / kQPerWG * kQPerWG;
    if (chunk < kQPerWG) chunk = kQPerWG;
    if (chunk > p.chunk) chunk = p.chunk;
    p.chunk = chunk;
  }
  return p;
}

size_t final_lds_bytes(const SearchPlan& p) {
  return 128 * sizeof(float) + static_cast<size_t>(p.L) * 8 + static_cast<size_t>(p.P) * 8 + 256 * sizeof(unsigned);
}

struct SearchWs {
  __bf16* qb;
  float* margin2;
  uint2* buf;
  int* count;
  unsigned* thr;
};

SearchWs carve_search(Carver& cv, int64_t nq, int D, const SearchPlan& p) {
  const int64_t chunk = nq < p.chunk ? nq : p.chunk;
  const int64_t nq_pad = round_up(chunk > 0 ? chunk : 1, kQPerWG);
  SearchWs w;
  w.qb = cv.take<__bf16>(nq_pad * D);
  w.margin2 = cv.take<float>(nq_pad);
  w.buf = cv.take<uint2>(nq_pad * p.S * p.H * static_cast<int64_t>(p.R));
  w.count = cv.take<int>(nq_pad * p.S * p.H);
  w.thr = cv.take<unsigned>(nq_pad);
  return w;
}

template <int D>
int launch_screen(const SearchPlan& p, const ScreenArgs& sa, const ScreenCArgs& ca, int64_t nq_pad, hipStream_t st) {
  if (p.bins) {
    hipLaunchKernelGGL(screen_bins_kernel<D>, dim3((nq_pad / kQPerWG) * p.S), dim3(kScreenThreads), 0, st, sa);
    TT_CHECK_LAUNCH();
    return TT_OK;
  }
  const dim3 grid(nq_pad / kQPerWG), block(kScreenThreads);
  switch (p.R / kWave) {
    case 16: hipLaunchKernelGGL((screen_compact_kernel<D, 16>), grid, block, 0, st, ca); break;
    case 32: hipLaunchKernelGGL((screen_compact_kernel<D, 32>), grid, block, 0, st, ca); break;
    case 64: hipLaunchKernelGGL((screen_compact_kernel<D, 64>), grid, block, 0, st, ca); break;
    case 128: hipLaunchKernelGGL((screen_compact_kernel<D, 128>), grid, block, 0, st, ca); break;
    default: return fail(TT_ERR_UNSUPPORTED, "tt_bruteforce_search: shortlist capacity %d", p.R);
  }
  TT_CHECK_LAUNCH();
  return TT_OK;
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" size_t tt_bruteforce_index_bytes(int64_t n_cand, int32_t dim) {
  if (n_cand < 1 || pick_dpad(dim) == 0) return 0;
  return index_bytes(n_cand, dim);
}

extern "C" int tt_bruteforce_build(const float* cand, int64_t ldc, int64_t n_cand, int32_t dim, void* index,
                                   size_t index_bytes_avail, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(cand && index, "tt_bruteforce_build: NULL pointer");
  TT_REQUIRE(n_cand >= 1 && n_cand < (1ll << 31) - kCTile, "tt_bruteforce_build: n_cand out of range");
  TT_REQUIRE(dim >= 1 && ldc >= dim, "tt_bruteforce_build: bad dim/ldc");
  if (pick_dpad(dim) == 0) return fail(TT_ERR_UNSUPPORTED, "tt_bruteforce_build: dim=%d > 128", dim);
  const size_t need = index_bytes(n_cand, dim);
  if (index_bytes_avail < need)
    return fail(TT_ERR_WORKSPACE, "tt_bruteforce_build: index buffer %zu < %zu", index_bytes_avail, need);
  hipStream_t st = to_stream(stream);
  TT_CHECK_HIP(hipMemsetAsync(index, 0, 64, st));
  const int D = pick_dpad(dim);
  const int64_t n_pad = round_up(n_cand, kCTile);
  hipLaunchKernelGGL(build_kernel, dim3(ceil_div(n_pad, 4 * kBuildRowsPerWave)), dim3(256), 0, st, cand, ldc, n_cand,
                     dim, n_pad, D, index);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" size_t tt_bruteforce_workspace_size(int64_t n_queries, int64_t n_cand, int32_t dim, int32_t k) {
  if (n_queries < 1 || n_cand < 1 || k < 1 || pick_dpad(dim) == 0) return 0;
  const SearchPlan p = plan_search(n_queries, n_cand, k);
  Carver cv(nullptr, 0);
  carve_search(cv, n_queries, pick_dpad(dim), p);
  return cv.used();
}

extern "C" int tt_bruteforce_search(const void* index, const float* cand, int64_t ldc, int64_t n_cand, int32_t dim,
                                    const float* queries, int64_t ldq, int64_t n_queries, int32_t k,
                                    int64_t index_offset, float* out_scores, int32_t* out_idx, void* workspace,
                                    size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(index && cand, "tt_bruteforce_search: NULL index/cand");
  TT_REQUIRE(n_cand >= 1 && dim >= 1 && ldc >= dim && ldq >= dim, "tt_bruteforce_search: bad shapes");
  if (pick_dpad(dim) == 0) return fail(TT_ERR_UNSUPPORTED, "tt_bruteforce_search: dim=%d > 128", dim);
  TT_REQUIRE(k >= 1, "tt_bruteforce_search: k must be >= 1");
  TT_REQUIRE(k <= n_cand, "tt_bruteforce_search: k=%d > number of candidates %lld", k,
             static_cast<long long>(n_cand));
  TT_REQUIRE(k <= 4000, "tt_bruteforce_search: k=%d > 4000", k);
  TT_REQUIRE(n_queries >= 0, "tt_bruteforce_search: negative n_queries");
  TT_REQUIRE(index_offset >= 0 && index_offset + n_cand < (1ll << 31), "tt_bruteforce_search: index_offset range");
  if (n_queries == 0) return TT_OK;
  TT_REQUIRE(queries && out_scores && out_idx, "tt_bruteforce_search: NULL queries/outputs");
  const int D = pick_dpad(dim);
  const SearchPlan p = plan_search(n_queries, n_cand, k);
  Carver cv(workspace, workspace_bytes);
  SearchWs w = carve_search(cv, n_queries, D, p);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_bruteforce_search: workspace %zu < required %zu", workspace_bytes, cv.used());
  hipStream_t st = to_stream(stream);
  const int64_t n_pad = round_up(n_cand, kCTile);
  const size_t shm = final_lds_bytes(p);
  if (shm > 65536)
    TT_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(finalize_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(shm)));
  const int vec4 = (reinterpret_cast<uintptr_t>(cand) % 16 == 0 && ldc % 4 == 0 && dim % 4 == 0) ? 1 : 0;
  for (int64_t q0 = 0; q0 < n_queries; q0 += p.chunk) {
    const int64_t nq = (n_queries - q0 < p.chunk) ? n_queries - q0 : p.chunk;
    const int64_t nq_pad = round_up(nq, kQPerWG);
    if (p.bins) TT_CHECK_HIP(hipMemsetAsync(w.thr, 0, nq_pad * sizeof(unsigned), st));
    hipLaunchKernelGGL(query_prep_kernel, dim3(ceil_div(nq_pad, 4)), dim3(256), 0, st, queries + q0 * ldq, ldq, nq,
                       dim, nq_pad, D, index, w.qb, w.margin2);
    TT_CHECK_LAUNCH();
    ScreenArgs sa{index, w.qb, w.margin2, nq, n_cand, n_pad, k, p.S, p.R, w.buf, w.count, w.thr};
    ScreenCArgs ca{index, w.qb, w.margin2, nq, n_pad, k, p.R, w.buf, w.count};
    int rc;
    probe_begin(TT_PROBE_INDEX_SCREEN, st);
    switch (D) {
      case 32: rc = launch_screen<32>(p, sa, ca, nq_pad, st); break;
      case 64: rc = launch_screen<64>(p, sa, ca, nq_pad, st); break;
      default: rc = launch_screen<128>(p, sa, ca, nq_pad, st); break;
    }
    probe_end(TT_PROBE_INDEX_SCREEN, st);
    if (rc) return rc;
    FinalArgs fa{queries + q0 * ldq, ldq, cand, ldc, n_cand, dim, k, p.S, p.H, p.R, p.L, p.P, vec4, 0, nq,
                 index_offset, w.margin2, w.buf, w.count, p.bins ? w.thr : nullptr, out_scores + q0 * k,
                 out_idx + q0 * k};
    probe_begin(TT_PROBE_INDEX_FINALIZE, st);
    hipLaunchKernelGGL(finalize_kernel, dim3(nq), dim3(kWave), shm, st, fa);
    probe_end(TT_PROBE_INDEX_FINALIZE, st);
    TT_CHECK_LAUNCH();
  }
  return TT_OK;
}
