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
// Screening bound.  A bf16 MFMA score s~ and the exact chain s differ by at
// most eps * sum_k |q_k c_k| with eps = 2^-7 + 2^-10: round-to-nearest bf16
// moves each operand by at most 2^-8 of itself, so a product of two rounded
// operands by at most 2^-7 + 2^-16; the bf16 products are exact in fp32 and
// the fp32 accumulation of <= 128 of them, like the exact chain's own
// rounding, adds below 2^-16 each.  Two forms of the bound:
//   relative  (query and every candidate non-negative, e.g. the towers' final
//             ReLU, tower.py:48): sum |q_k c_k| = s, so
//             s in [s~(1 - eps) - tiny, s~(1 + eps) + tiny];
//   absolute  (otherwise): |s - s~| <= M_q = eps |q|_2 max_c |c|_2.
// lb(s~) / ub(s~) below are those interval ends.
//
// Design (MI355X, one chip):
//  prep     bf16 query rows, per-query bound mode / margin, zero-query flag.
//  screen   one workgroup = 8 waves x 64 queries (two 32-query sets per wave,
//           their bf16 fragments in VGPRs as the B operand); 64-candidate bf16
//           tiles stream through a 4-stage LDS ring filled by LDS-DMA
//           (global_load_lds, chunk-pair planes: tile_frag_lane_off) and are scored with
//           v_mfma_f32_32x32x16_bf16 (S^T: each lane holds 16 candidates of one
//           query).  Phase 1 scans a spread sample of the split's tiles and
//           keeps per-register running maxima ("bins": 64 per query, each over
//           a fixed residue class of sampled candidates); the j-th largest bin
//           is an ESTIMATE tau of the score at rank ~R of the split (R ~ 3k).
//           Phase 2 scans every tile once: a score s~ > tau is appended to a
//           lane-private list (no atomics); that is one compare per score and
//           a store for ~R/N of them.  tau is NOT assumed to be a bound.
//  finalize one wave per query: radix-selects the k-th largest screened score
//           sK over its lists, certifies the screen — X = lb(sK) > ub(tau)
//           of every list means every candidate that can still belong to the
//           exact top-k (ub(s~) >= X) scored above its list's tau and was
//           kept — keeps the entries with ub(s~) >= X, rescores them with the
//           exact fp32 chain, selects the exact top-k on (score, -index) and
//           ranks them with an LDS bitonic sort.  A query that fails the
//           certificate, overflows a list, or cannot be cut into LDS goes to
//           the fallback list.
//  fallback persistent grid: an exact fp32 scan of every candidate for each
//           failed query (rare: estimation tails, massive exact ties).
//  Zero queries score exactly +0 against every candidate in both paths; their
//  answer (indices 0..k-1 by the tie rule) is written directly.
#include <cmath>
#include <cstdlib>

#include "tt_common.h"

#ifdef TT_INDEX_STATS
__device__ unsigned long long g_index_stats[4];  // list entries, certificate fails, cut sizes, other fails
#define TT_STAT(i, v) atomicAdd(&g_index_stats[i], static_cast<unsigned long long>(v))
#define TT_STAT0(i, v) \
  if (lane_id() == 0) atomicAdd(&g_index_stats[i], static_cast<unsigned long long>(v))
#else
#define TT_STAT(i, v) ((void)0)
#define TT_STAT0(i, v) ((void)0)
#endif

namespace tt {
namespace {

#ifndef TT_SCREEN_WAVES
#define TT_SCREEN_WAVES 8
#endif
constexpr int kSWaves = TT_SCREEN_WAVES;
constexpr int kSThreads = kSWaves * kWave;       // 512
constexpr int kQPerWave = 64;                    // two 32-query sets
constexpr int kQPerWG = kSWaves * kQPerWave;     // 512
constexpr int kCTile = 64;                       // candidates per LDS tile
constexpr int kStages = 4;                       // LDS ring depth
#ifndef TT_INDEX_MAX_SAMPLE
#define TT_INDEX_MAX_SAMPLE 128
#endif
constexpr int kMaxSample = TT_INDEX_MAX_SAMPLE;  // sample tiles per split
#ifndef TT_INDEX_MAX_SPLITS
#define TT_INDEX_MAX_SPLITS 32
#endif
#ifndef TT_INDEX_SPLIT_TILES
#define TT_INDEX_SPLIT_TILES 32  // a split is halved only while each half keeps >= this many tiles
#endif
constexpr int kMaxSplits = TT_INDEX_MAX_SPLITS;
#ifndef TT_INDEX_MAX_SCAN_SPLITS
#define TT_INDEX_MAX_SCAN_SPLITS 64
#endif
#ifndef TT_INDEX_SCAN_TILES
#define TT_INDEX_SCAN_TILES 16  // a scan split is halved only while each half keeps >= this many tiles
#endif
constexpr float kEps = 0.0087890625f;            // 2^-7 + 2^-10
constexpr float kTiny = 1e-30f;
#ifndef TT_LIST_BUDGET
#define TT_LIST_BUDGET (size_t(2) << 30)
#endif
constexpr size_t kListBudget = TT_LIST_BUDGET;   // bytes of screened lists per chunk

enum : int { kQZero = 1, kQRel = 2 };

struct IndexHeader {
  int64_t n;
  int64_t n_pad;
  int32_t dim;
  int32_t D;
  unsigned maxnorm_bits;  // max_c |c|_2 as float bits (non-negative)
  unsigned has_neg;       // some candidate coordinate < 0
  unsigned maxcb_bits;    // max_c |bf16(c)|_2 (rounded up)
  unsigned maxrc_bits;    // max_c |c - bf16(c)|_2 (rounded up)
  unsigned pad[6];
};
static_assert(sizeof(IndexHeader) == 64, "header");

inline int pick_dpad(int dim) {
  if (dim <= 32) return 32;
  if (dim <= 64) return 64;
  if (dim <= 128) return 128;
  return 0;
}

inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Index image: 64-B header, bf16 rows [n_pad, D], then per row the norms
// (|bf16(c)|_2, |c - bf16(c)|_2) as float2 (rounded up) for the per-row
// screen bound.
size_t index_bytes(int64_t n, int dim) {
  const int D = pick_dpad(dim);
  const size_t n_pad = static_cast<size_t>(round_up(n, kCTile));
  return 64 + n_pad * D * 2 + n_pad * sizeof(float2);
}

__device__ __forceinline__ const __bf16* index_rows(const void* idx) {
  return reinterpret_cast<const __bf16*>(static_cast<const char*>(idx) + 64);
}

__host__ __device__ __forceinline__ size_t norms_offset(int64_t n_pad, int D) {
  return 64 + static_cast<size_t>(n_pad) * D * 2;
}

// Per-row screen bound.  With qb = bf16(q), rq = q - qb, cb = bf16(c),
// rc = c - cb (componentwise exact in fp32):
//   q.c = qb.cb + qb.rc + rq.cb + rq.rc,
//   |s~ - qb.cb|      <= g |qb| |cb|   (fp32 accumulation of the exact bf16
//                                       products, any order, g = 2 D 2^-24),
//   |s_chain - q.c|   <= g |q| |c|     (the exact fmaf chain's own rounding),
// so |s~ - s_chain| <= |qb||rc| + |rq|(|cb| + |rc|) + 2g(|qb| + |rq|)(|cb| + |rc|)
// (Cauchy-Schwarz; |q| <= |qb| + |rq|, |c| <= |cb| + |rc|).  The bf16
// residuals are ~2^-9 of their vectors, so this is typically 2-3x tighter
// than eps * s (relative form): fewer screened entries survive the cut.
constexpr float kGam2 = 2.0f * 2.0f * 128.0f * 5.9604645e-8f;  // 2g at D <= 128
__device__ __forceinline__ float row_err(float qb, float qr, float cb, float cr) {
  return (qb * cr + qr * (cb + cr) + kGam2 * (qb + qr) * (cb + cr)) * (1.0f + 1e-5f) + kTiny;
}

__device__ __forceinline__ float lb_of(float s, float m, bool rel) {
  return rel ? s * (1.0f - kEps) - kTiny : s - m;
}
__device__ __forceinline__ float ub_of(float s, float m, bool rel) {
  return rel ? s * (1.0f + kEps) + kTiny : s + m;
}

__device__ __forceinline__ uint64_t lanemask_lt64() {
  const int l = lane_id();
  return (l == 0) ? 0ull : (~0ull >> (64 - l));
}

// Orders this wave's LDS accesses around it (a wave's LDS operations execute
// in order; this stops the compiler moving them across).  The finalize and
// fallback helpers below are wave-local, so several waves of one workgroup
// may run them on their own LDS regions.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ unsigned long long make_key(float s, unsigned idx) {
  return (static_cast<unsigned long long>(float_order_key(s)) << 32) |
         static_cast<unsigned long long>(0xFFFFFFFFu - idx);
}

// ---- build ----------------------------------------------------------------
// Row-major bf16 image (zero padded to n_pad rows, D columns), max row norm
// and the has-negative flag (one atomic of each per workgroup).
constexpr int kBuildRowsPerWave = 16;
__global__ void __launch_bounds__(256) build_kernel(const float* __restrict__ cand, int64_t ldc, int64_t n, int dim,
                                                    int64_t n_pad, int D, void* index) {
  __shared__ float wmax[3][4];
  __shared__ int wneg[4];
  IndexHeader* hdr = static_cast<IndexHeader*>(index);
  __bf16* rows = reinterpret_cast<__bf16*>(static_cast<char*>(index) + 64);
  float2* norms = reinterpret_cast<float2*>(static_cast<char*>(index) + norms_offset(n_pad, D));
  const int wave = threadIdx.x / kWave;
  const int lane = lane_id();
  float mx = 0.0f, mcb = 0.0f, mrc = 0.0f;
  bool neg = false;
  for (int i = 0; i < kBuildRowsPerWave; ++i) {
    const int64_t r = (blockIdx.x * 4ll + wave) * kBuildRowsPerWave + i;
    if (r >= n_pad) break;
    float ss = 0.0f, sb = 0.0f, sr = 0.0f;
    for (int e2 = lane; e2 < D / 2; e2 += kWave) {
      const int e = 2 * e2;
      const float x0 = (r < n && e < dim) ? cand[r * ldc + e] : 0.0f;
      const float x1 = (r < n && e + 1 < dim) ? cand[r * ldc + e + 1] : 0.0f;
      ss = __builtin_fmaf(x0, x0, __builtin_fmaf(x1, x1, ss));
      neg = neg || x0 < 0.0f || x1 < 0.0f;
      const unsigned pk = pack_bf16x2(x0, x1);
      reinterpret_cast<unsigned*>(rows + r * D)[e2] = pk;
      const float b0 = __uint_as_float(pk << 16), b1 = __uint_as_float(pk & 0xFFFF0000u);
      const float d0 = x0 - b0, d1 = x1 - b1;  // exact in fp32
      sb = __builtin_fmaf(b0, b0, __builtin_fmaf(b1, b1, sb));
      sr = __builtin_fmaf(d0, d0, __builtin_fmaf(d1, d1, sr));
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      ss += __shfl_xor(ss, m, kWave);
      sb += __shfl_xor(sb, m, kWave);
      sr += __shfl_xor(sr, m, kWave);
    }
    // rounded up (the sums of <= 128 squares and the sqrt: relative < 1e-5)
    const float nb = sqrtf(sb) * (1.0f + 1e-5f), nr = sqrtf(sr) * (1.0f + 1e-5f);
    if (lane == 0) norms[r] = make_float2(nb, nr);
    if (r < n) {
      mx = fmaxf(mx, sqrtf(ss));
      mcb = fmaxf(mcb, nb);
      mrc = fmaxf(mrc, nr);
    }
  }
  const bool wn = __ballot(neg) != 0;
  if (lane == 0) {
    wmax[0][wave] = mx;
    wmax[1][wave] = mcb;
    wmax[2][wave] = mrc;
    wneg[wave] = wn ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(wmax[0][0], wmax[0][1]), fmaxf(wmax[0][2], wmax[0][3]));
    // round the norm up so the bound stays an upper bound
    atomicMax(&hdr->maxnorm_bits, __float_as_uint(m * (1.0f + 1e-5f)));
    atomicMax(&hdr->maxcb_bits, __float_as_uint(fmaxf(fmaxf(wmax[1][0], wmax[1][1]), fmaxf(wmax[1][2], wmax[1][3]))));
    atomicMax(&hdr->maxrc_bits, __float_as_uint(fmaxf(fmaxf(wmax[2][0], wmax[2][1]), fmaxf(wmax[2][2], wmax[2][3]))));
    if (wneg[0] | wneg[1] | wneg[2] | wneg[3]) atomicOr(&hdr->has_neg, 1u);
    if (blockIdx.x == 0) {
      hdr->n = n;
      hdr->n_pad = n_pad;
      hdr->dim = dim;
      hdr->D = D;
    }
  }
}

// ---- query prep ----------------------------------------------------------
// bf16 rows [nq_pad, D]; per query the bound mode (relative when the query and
// every candidate are non-negative), the absolute margin M_q, the zero flag.
__global__ void query_prep_kernel(const float* __restrict__ q, int64_t ldq, int64_t nq, int dim, int64_t nq_pad,
                                  int D, const void* index, __bf16* __restrict__ qb, int* __restrict__ qflags,
                                  float* __restrict__ qmarg, float2* __restrict__ qnorm) {
  const int64_t r = blockIdx.x * 4ll + threadIdx.x / kWave;
  if (r >= nq_pad) return;
  const int lane = lane_id();
  float ss = 0.0f, sb = 0.0f, sr = 0.0f;
  bool nz = false, neg = false;
  for (int e2 = lane; e2 < D / 2; e2 += kWave) {
    const int e = 2 * e2;
    const float x0 = (r < nq && e < dim) ? q[r * ldq + e] : 0.0f;
    const float x1 = (r < nq && e + 1 < dim) ? q[r * ldq + e + 1] : 0.0f;
    ss = __builtin_fmaf(x0, x0, __builtin_fmaf(x1, x1, ss));
    nz = nz || x0 != 0.0f || x1 != 0.0f;
    neg = neg || x0 < 0.0f || x1 < 0.0f;
    const unsigned pk = pack_bf16x2(x0, x1);
    if (qb) reinterpret_cast<unsigned*>(qb + r * D)[e2] = pk;
    const float b0 = __uint_as_float(pk << 16), b1 = __uint_as_float(pk & 0xFFFF0000u);
    const float d0 = x0 - b0, d1 = x1 - b1;
    sb = __builtin_fmaf(b0, b0, __builtin_fmaf(b1, b1, sb));
    sr = __builtin_fmaf(d0, d0, __builtin_fmaf(d1, d1, sr));
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    ss += __shfl_xor(ss, m, kWave);
    sb += __shfl_xor(sb, m, kWave);
    sr += __shfl_xor(sr, m, kWave);
  }
  if (lane == 0) qnorm[r] = make_float2(sqrtf(sb) * (1.0f + 1e-5f), sqrtf(sr) * (1.0f + 1e-5f));
  const bool nonzero = __ballot(nz) != 0;
  const bool qneg = __ballot(neg) != 0;
  if (lane == 0) {
    const IndexHeader* hdr = static_cast<const IndexHeader*>(index);
    const float maxc = __uint_as_float(hdr->maxnorm_bits);
    const float qn = sqrtf(ss) * (1.0f + 1e-5f);
    const bool rel = !qneg && hdr->has_neg == 0;
    qflags[r] = (nonzero ? 0 : kQZero) | (rel ? kQRel : 0);
    qmarg[r] = (kEps * qn * maxc) * (1.0f + 1e-5f) + kTiny;
  }
}

// ---- screen ----------------------------------------------------------------
struct ScreenArgs {
  const void* index;
  const __bf16* qb;   // [nq_pad, D]
  int64_t nq;         // real queries in this chunk
  int64_t row0;       // candidate rows [row0, row1) of the image are screened
  int64_t row1;
  int S;              // candidate splits
  int NS;             // sample tiles per split (0: keep every score)
  int jsel;           // tau = jsel-th largest of a query's 64 bins
  int cap;            // entries per (query, split) list; the last slot is scratch
  unsigned index_offset;  // id of image row r = index_offset + r
  uint2* buf;         // [nq_pad][S][cap] (score bits, id)
  int* count;         // [nq_pad][S]; -1 = list overflowed
  float* tau_split;   // sample pass output [nq_pad][S]
  const float* tau;   // scan pass input [nq_pad]: keep s~ > tau[q]
  float* bins;        // pooled estimate (non-NULL): the sample pass writes [nq_pad][S][64] bin maxima instead
};

// s_waitcnt with only the vector-memory counter constrained (gfx9 encoding).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// Waits until at most n of this wave's vector-memory ops are in flight (n
// rounded down to a bucket: waiting for more is always safe).
// n is read as a wave-uniform (scalar) value: the tests are scalar compares
// and branches, the small counts (the scan's steady state) first.
__device__ __forceinline__ void wait_vmcnt_atmost(int n) {
  n = __builtin_amdgcn_readfirstlane(n);
  if (n < 16) {
    if (n >= 8) {
      if (n >= 12) wait_vmcnt<12>();
      else wait_vmcnt<8>();
    } else if (n >= 4) {
      if (n >= 6) wait_vmcnt<6>();
      else wait_vmcnt<4>();
    } else if (n >= 2) {
      wait_vmcnt<2>();
    } else {
      wait_vmcnt<0>();
    }
  } else if (n >= 32) {
    if (n >= 63) wait_vmcnt<63>();
    else if (n >= 48) wait_vmcnt<48>();
    else wait_vmcnt<32>();
  } else if (n >= 24) {
    wait_vmcnt<24>();
  } else {
    wait_vmcnt<16>();
  }
}

// LDS image of one 64-candidate bf16 tile (sample and scan rings), in 16-B
// chunks: plane s holds chunks 2s and 2s + 1 of every row (64 rows x 32 B =
// 2 KiB at s * 2048); row r's pair sits at r * 32 with its two chunks swapped
// when bit 3 of r is set.  A lane's fragment of k-step s is then at a
// lane-constant offset + s * 2048 + t * 1024 (an instruction immediate, no
// address arithmetic per read), and the 16 lanes of each ds_read_b128 lane
// group ({0-3, 12-15, 20-27}, ...) hit 16 distinct 16-B bank slots.
__device__ __forceinline__ int tile_frag_lane_off(int l32, int h) {
  return l32 * 32 + ((h ^ ((l32 >> 3) & 1)) << 4);
}
// Source chunk of the 16 B that LDS-DMA piece p's lane writes (piece = 1 KiB
// = half a plane: 32 rows x 32 B): its row in the tile and chunk in the row.
__device__ __forceinline__ void tile_piece_src(int p, int lane, int& row, int& ch) {
  const int plane = p >> 1, w = (p & 1) * 1024 + lane * 16;
  row = w >> 5;
  ch = 2 * plane + (((w >> 4) & 1) ^ ((row >> 3) & 1));
}

// jsel-th largest of the 64 values {bins of this lane, bins of lane ^ 32},
// to a 16-bit order-key prefix (rounded down); -inf if fewer than jsel bins.
__device__ float bins_select(const float (&ba)[16], const float (&bb)[16], int jsel) {
  unsigned res = 0;
#pragma unroll 1
  for (int bit = 15; bit >= 0; --bit) {
    const unsigned c = res | (1u << bit);
    const float f = order_key_float(c << 16);  // smallest float with this prefix (NaN: none)
    int n = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) n += ((ba[i] >= f) ? 1 : 0) + ((bb[i] >= f) ? 1 : 0);
    n += __shfl_xor(n, 32, kWave);
    if (n >= jsel) res = c;
  }
  const float t = order_key_float(res << 16);
  return (t > -INFINITY) ? t : -INFINITY;  // NaN (no prefix found) -> keep everything
}

// The estimate pass (phase 1) over the split's spread sample tiles: writes
// tau[q][split].  (scan_kernel below is phase 2.)
template <int D>
__global__ void __launch_bounds__(kSThreads) sample_kernel(const ScreenArgs a) {
  constexpr bool SAMPLE = true;
  constexpr int KS = D / 16, RB = D * 2;
  constexpr int TILE_BYTES = kCTile * RB;                 // 16 KiB at D = 128
  constexpr int PIECES = TILE_BYTES / 1024;               // 1 KiB LDS-DMA pieces per tile
  constexpr int PPW = PIECES >= kSWaves ? PIECES / kSWaves : 1;
  __shared__ __attribute__((aligned(1024))) char smem[kStages * TILE_BYTES];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);  // wave-uniform (scalar)
  const int lane = lane_id();
  const int h = lane >> 5, l32 = lane & 31;
  const int split = static_cast<int>(blockIdx.x % a.S);
  const int64_t q0 = static_cast<int64_t>(blockIdx.x / a.S) * kQPerWG + wave * kQPerWave + l32;
  const int64_t q1 = q0 + 32;
  const int t0 = static_cast<int>(a.row0 / kCTile);
  const int ntiles = static_cast<int>((a.row1 + kCTile - 1) / kCTile) - t0;
  const int per = (ntiles + a.S - 1) / a.S;
  const int tb = t0 + split * per;
  const int nt = max(min(ntiles - split * per, per), 0);
  const int ns = min(a.NS, nt);
  const __bf16* crow = index_rows(a.index);
  const bool my_pieces = wave * PPW < PIECES;  // D = 32: waves 4..7 stage nothing

  bf16x8 bq0[KS], bq1[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    bq0[s] = *reinterpret_cast<const bf16x8*>(a.qb + q0 * D + 16 * s + 8 * h);
    bq1[s] = *reinterpret_cast<const bf16x8*>(a.qb + q1 * D + 16 * s + 8 * h);
  }
  wait_vmcnt<0>();  // ordinary loads retired before the LDS-DMA ring starts

  // tile sequence: the spread sample, or every tile of the split
  auto phys = [&](int u) { return SAMPLE ? tb + (u * nt) / ns : tb + u; };
  const int nv = SAMPLE ? ns : nt;

  auto issue = [&](int tile, int stage) {
    const int64_t base = static_cast<int64_t>(tile) * kCTile;
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const int p = wave * PPW + u;
      if (p < PIECES) {
        int row, ch;
        tile_piece_src(p, lane, row, ch);
        const __bf16* src = crow + (base + row) * D + ch * 8;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src),
                                         (__attribute__((address_space(3))) void*)(smem + stage * TILE_BYTES + p * 1024),
                                         16, 0, 0);
      }
    }
  };
  auto wait_tiles = [&](int ahead) {  // at most `ahead` of this wave's tiles still in flight
    if (!my_pieces || ahead <= 0) {
      wait_vmcnt<0>();
    } else if (ahead == 1) {
      wait_vmcnt<PPW>();
    } else {
      wait_vmcnt<2 * PPW>();
    }
  };
  const int frag_off = tile_frag_lane_off(l32, h);
  auto frag = [&](const char* B, int t, int s) {
    return *reinterpret_cast<const bf16x8*>(B + frag_off + s * 2048 + t * 1024);
  };
  auto mask_pad = [&](f32x16& acc, int64_t cfirst) {  // rows outside [row0, row1) (edge tiles only)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t c = cfirst + (r & 3) + 8 * (r >> 2);
      if (c < a.row0 || c >= a.row1) acc[r] = -INFINITY;
    }
  };
  auto edge = [&](int64_t cbase) { return cbase < a.row0 || cbase + kCTile > a.row1; };
  auto advance = [&](int u) {  // (sample) tile u consumed: wait for u + 1, barrier
    if (u + 1 < nv) wait_tiles(min(u + kStages - 1, nv - 1) - (u + 1));
    __builtin_amdgcn_s_barrier();
  };

#pragma unroll
  for (int s = 0; s < kStages - 1; ++s)
    if (s < nv) issue(phys(s), s);
  wait_tiles(min(nv, kStages - 1) - 1);
  __builtin_amdgcn_s_barrier();

  if constexpr (SAMPLE) {
  // ---- phase 1: sample tiles, bins only ------------------------------------
    // bins: per lane and query set, 16 register positions x the 2 blocks of a tile
    // (64 per query with the partner lane), running maxima of the sample.
    float b0a[16], b0b[16], b1a[16], b1b[16];
  #pragma unroll
    for (int r = 0; r < 16; ++r) b0a[r] = b0b[r] = b1a[r] = b1b[r] = -INFINITY;
    for (int u = 0; u < ns; ++u) {
      if (u + kStages - 1 < nv) issue(phys(u + kStages - 1), (u + kStages - 1) % kStages);
      const char* B = smem + (u % kStages) * TILE_BYTES;
      const int64_t cbase = static_cast<int64_t>(phys(u)) * kCTile;
  #pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x16 c0 = {}, c1 = {};
  #pragma unroll
        for (int s = 0; s < KS; ++s) {
          const bf16x8 af = frag(B, t, s);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bq0[s], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bq1[s], c1, 0, 0, 0);
        }
        if (edge(cbase)) {
          mask_pad(c0, cbase + 32 * t + 4 * h);
          mask_pad(c1, cbase + 32 * t + 4 * h);
        }
        float (&x0)[16] = t == 0 ? b0a : b0b;  // static under the unroll
        float (&x1)[16] = t == 0 ? b1a : b1b;
  #pragma unroll
        for (int r = 0; r < 16; ++r) {
          x0[r] = __builtin_elementwise_maximum(x0[r], c0[r]);
          x1[r] = __builtin_elementwise_maximum(x1[r], c1[r]);
        }
      }
      advance(u);
    }
    if (a.bins) {  // pooled estimate: this lane's 32 of the query's 64 bins of this split
      float* o0 = a.bins + (q0 * a.S + split) * 64 + 32 * h;
      float* o1 = a.bins + (q1 * a.S + split) * 64 + 32 * h;
  #pragma unroll
      for (int r = 0; r < 16; r += 4) {
        *reinterpret_cast<f32x4*>(o0 + r) = f32x4{b0a[r], b0a[r + 1], b0a[r + 2], b0a[r + 3]};
        *reinterpret_cast<f32x4*>(o0 + 16 + r) = f32x4{b0b[r], b0b[r + 1], b0b[r + 2], b0b[r + 3]};
        *reinterpret_cast<f32x4*>(o1 + r) = f32x4{b1a[r], b1a[r + 1], b1a[r + 2], b1a[r + 3]};
        *reinterpret_cast<f32x4*>(o1 + 16 + r) = f32x4{b1b[r], b1b[r + 1], b1b[r + 2], b1b[r + 3]};
      }
    } else {
      const float tq0 = ns > 0 ? bins_select(b0a, b0b, a.jsel) : -INFINITY;
      const float tq1 = ns > 0 ? bins_select(b1a, b1b, a.jsel) : -INFINITY;
      if (h == 0) {
        a.tau_split[q0 * a.S + split] = tq0;
        a.tau_split[q1 * a.S + split] = tq1;
      }
    }
  }
}

// ---- scan: every tile of the split once, keep s~ > tau ----------------------
// Staged hit rows per wave: a lane whose 16 scores of a block hold one above
// its query's tau copies the whole row (16 scores + tag) into its wave's LDS
// stage; once >= 64 rows are staged the wave filters them one row per lane
// and appends the hits to the queries' lists.  The per-block filter is thus
// a 16-way max per query set and one compare (branch-free, interleaved with
// the next block's MFMAs); the per-score work runs on full waves of hit rows.
constexpr int kStageRows = 128;  // a wave's ring of staged rows: < 64 pending before a set, + <= 64 per set
constexpr int kRowF = 20;        // floats per staged row: 16 scores, candidate base, query, 2 pad (80 B: no
                                 // bank conflicts when 8 lanes read 8 consecutive rows by ds_read_b128)

template <int D>
struct ScanGeo {
  static constexpr int TILE_BYTES = kCTile * D * 2;
  static constexpr int RING = kStages * TILE_BYTES;
};

// (IEEE maximum: v_maximum3_f32, no NaN-quieting canonicalisations as fmaxf
// needs; a NaN score makes the max NaN, which stages nothing.)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ __forceinline__ float max16(const f32x16& c) {
  const float x0 = max3f(c[0], c[1], c[2]);
  const float x1 = max3f(c[3], c[4], c[5]);
  const float x2 = max3f(c[6], c[7], c[8]);
  const float x3 = max3f(c[9], c[10], c[11]);
  const float x4 = max3f(c[12], c[13], c[14]);
  return max3f(max3f(x0, x1, x2), max3f(x3, x4, c[15]), -INFINITY);
}

template <int D>
__global__ void __launch_bounds__(kSThreads) scan_kernel(const ScreenArgs a) {
  using G = ScanGeo<D>;
  constexpr int KS = D / 16;
  constexpr int TILE_BYTES = G::TILE_BYTES;
  constexpr int PIECES = TILE_BYTES / 1024;               // 1 KiB LDS-DMA pieces per tile
  constexpr int PPW = PIECES >= kSWaves ? PIECES / kSWaves : 1;
  // separate LDS objects: the compiler can tell the staging area from the
  // LDS-DMA ring, so staging does not wait for the ring's loads (vmcnt)
  __shared__ __attribute__((aligned(1024))) char smem[G::RING];
  __shared__ __attribute__((aligned(16))) float s_rows[kSWaves * kStageRows * kRowF];
  __shared__ float s_tau[kQPerWG];
  __shared__ int s_cnt[kQPerWG];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);  // wave-uniform (scalar)
  const int lane = lane_id();
  const int h = lane >> 5, l32 = lane & 31;
  const int split = static_cast<int>(blockIdx.x % a.S);
  const int64_t qblk = static_cast<int64_t>(blockIdx.x / a.S) * kQPerWG;
  const int ql0 = wave * kQPerWave + l32, ql1 = ql0 + 32;  // this lane's queries in the workgroup
  const int64_t q0 = qblk + ql0, q1 = qblk + ql1;
  const int t0 = static_cast<int>(a.row0 / kCTile);
  const int ntiles = static_cast<int>((a.row1 + kCTile - 1) / kCTile) - t0;
  const int per = (ntiles + a.S - 1) / a.S;
  const int tb = t0 + split * per;
  const int nv = max(min(ntiles - split * per, per), 0);
  const __bf16* crow = index_rows(a.index);
  const bool my_pieces = wave * PPW < PIECES;  // D = 32: waves 4..7 stage nothing
  float* const srow = s_rows + wave * kStageRows * kRowF;
  float* const tau_l = s_tau;
  int* const cnt_l = s_cnt;

  bf16x8 bq0[KS], bq1[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    bq0[s] = *reinterpret_cast<const bf16x8*>(a.qb + q0 * D + 16 * s + 8 * h);
    bq1[s] = *reinterpret_cast<const bf16x8*>(a.qb + q1 * D + 16 * s + 8 * h);
  }
  // the sample pass's estimate; queries past nq keep nothing
#ifndef TT_INDEX_NOINSERT
  const float tau0 = q0 < a.nq ? a.tau[q0] : INFINITY;
  const float tau1 = q1 < a.nq ? a.tau[q1] : INFINITY;
#else  // probe build: scan cost without staging (tau +inf, opaque to the compiler)
  const float tau0 = __uint_as_float(a.cap > 0 ? 0x7f800000u : 0u), tau1 = tau0;
#endif
  if (h == 0) {  // each wave owns its 64 queries' LDS words
    tau_l[ql0] = tau0;
    tau_l[ql1] = tau1;
    cnt_l[ql0] = 0;
    cnt_l[ql1] = 0;
  }
  wait_vmcnt<0>();  // ordinary loads retired before the LDS-DMA ring starts

  auto issue = [&](int tile, int stage) {
    const int64_t base = static_cast<int64_t>(tile) * kCTile;
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const int p = wave * PPW + u;
      if (p < PIECES) {
        int row, ch;
        tile_piece_src(p, lane, row, ch);
        const __bf16* src = crow + (base + row) * D + ch * 8;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src),
                                         (__attribute__((address_space(3))) void*)(smem + stage * TILE_BYTES + p * 1024),
                                         16, 0, 0);
      }
    }
  };
  const int frag_off = tile_frag_lane_off(l32, h);
  auto frag = [&](const char* B, int t, int s) {
    return *reinterpret_cast<const bf16x8*>(B + frag_off + s * 2048 + t * 1024);
  };
  auto load_frags = [&](bf16x8 (&f)[KS], const char* B, int t) {
#pragma unroll
    for (int s = 0; s < KS; ++s) f[s] = frag(B, t, s);
  };
  auto mask_pad = [&](f32x16& acc, int64_t cfirst) {  // rows outside [row0, row1) (edge tiles only)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t c = cfirst + (r & 3) + 8 * (r >> 2);
      if (c < a.row0 || c >= a.row1) acc[r] = -INFINITY;
    }
  };
  auto edge = [&](int64_t cbase) { return cbase < a.row0 || cbase + kCTile > a.row1; };

  // ---- vector-memory accounting (as in the ring loop of the sample pass,
  // plus the list stores of the flushes, which share vmcnt with the LDS-DMA):
  // windows wa / wb / wc = ops issued from the DMA of tile u + 1 / u + 2 /
  // u + 3 up to the next DMA; da / db / dc = that DMA's pieces.
  const int dpieces = my_pieces ? PPW : 0;
  int wa, wb, wc, da, db, dc;
  int head = 0, tail = 0;  // staged rows [tail, head) of the wave's ring (wave-uniform counters)
  // the workgroup's lists: (query ql, split) at entry (ql * S + split) * cap
  const __amdgpu_buffer_rsrc_t lists = __builtin_amdgcn_make_buffer_rsrc(
      a.buf + qblk * a.S * static_cast<int64_t>(a.cap), 0, 0x7fffffff, 0x00020000);

  // Filters nrows staged rows from the tail (one per lane) and appends their
  // hits to the lists: per register r, the lanes whose score r beats their
  // row's tau store it at their list's next slot.  Branch-free: 16 stores per
  // flush, a lane without a hit in r addressing past the buffer resource's
  // range (the store drops it; 4.53 -> 4.35 ms per 131k-query chunk against
  // one branch per register).
  auto flush = [&](int nrows) {
    wsync();
    const float* row = srow + ((tail + lane) & (kStageRows - 1)) * kRowF;
    const bool valid = lane < nrows;
    f32x4 x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = reinterpret_cast<const f32x4*>(row)[i];
    const f32x4 tg4 = reinterpret_cast<const f32x4*>(row)[4];
    const unsigned pcr = __float_as_uint(tg4[0]);
    const int ql = valid ? static_cast<int>(__float_as_uint(tg4[1])) : 0;
    const float tr = valid ? tau_l[ql] : INFINITY;
#ifndef TT_SCAN_FLUSH_LOOP
#define TT_SCAN_FLUSH_LOOP 1
#endif
    unsigned hm = 0;  // the row's registers above tau
#pragma unroll
    for (int r = 0; r < 16; ++r) hm |= (x[r >> 2][r & 3] > tr) ? (1u << r) : 0u;
    const int n = __popc(hm);
    int pos = 0;
    if (n) {  // reserve n list slots (an LDS atomic the compiler would order behind the ring's loads)
      const unsigned addr = static_cast<unsigned>(
          reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) int*)(cnt_l + ql)));
      asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(pos) : "v"(addr), "v"(n) : "memory");
    }
    const unsigned lbase = static_cast<unsigned>((ql * a.S + split) * a.cap) * 8u;
    const int last = a.cap - 1;  // scratch slot: entries past it are dropped with the list
    // branch-free: one store per register for the whole wave; a lane with no
    // hit in it addresses past the resource's range, and the store drops it
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    if (TT_SCAN_FLUSH_LOOP) {
      // one store per round for the whole wave, each lane storing its next
      // hit (lowest register first: the same entries at the same slots as
      // the per-register form), the score re-read from the staged row in
      // LDS; rounds = the most hits in one row (usually 2), not 16
      int rounds = 0;
      while (__ballot(hm != 0u)) {
        const int r = __builtin_ctz(hm | 0x10000u);  // 16 (the row's tag word) when none is left
        const float v = row[r];
        const u32x2 e = {__float_as_uint(v), pcr + static_cast<unsigned>((r & 3) + 8 * (r >> 2))};
        const unsigned off = hm != 0u ? lbase + static_cast<unsigned>(min(pos, last)) * 8u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b64(e, lists, off, 0, 0);
        pos += hm != 0u ? 1 : 0;
        hm &= hm - 1u;
        ++rounds;
      }
      wc = __builtin_amdgcn_readfirstlane(wc + rounds);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = x[r >> 2][r & 3];
        const bool keepit = v > tr;
        const u32x2 e = {__float_as_uint(v), pcr + static_cast<unsigned>((r & 3) + 8 * (r >> 2))};
        const unsigned off = keepit ? lbase + static_cast<unsigned>(min(pos, last)) * 8u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b64(e, lists, off, 0, 0);
        pos += keepit ? 1 : 0;
      }
      wc = __builtin_amdgcn_readfirstlane(wc + 16);
    }
    tail += nrows;
    wsync();
  };
  // Stages the rows of this block's lanes whose max beats their tau.
  auto stage = [&](const f32x16& c, bool hit, int ql, unsigned pc) {
    const uint64_t m = __ballot(hit);
    if (m) {
      if (hit) {
        // slot = head + #hit lanes below this one (v_mbcnt adds head in)
        const unsigned slot = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(m), head));
        f32x4* d = reinterpret_cast<f32x4*>(srow + (slot & (kStageRows - 1)) * kRowF);
        d[0] = f32x4{c[0], c[1], c[2], c[3]};
        d[1] = f32x4{c[4], c[5], c[6], c[7]};
        d[2] = f32x4{c[8], c[9], c[10], c[11]};
        d[3] = f32x4{c[12], c[13], c[14], c[15]};
        reinterpret_cast<uint2*>(d + 4)[0] = make_uint2(pc, static_cast<unsigned>(ql));
      }
      head += __popcll(m);
      if (head - tail >= kWave) flush(kWave);
    }
  };
#ifndef TT_SCAN_PAIR_STAGE
#define TT_SCAN_PAIR_STAGE 1
#endif
  // Both query sets' rows of one block in ONE round of row stores: a lane
  // stages its set-0 row if that hits, else its set-1 row (selected in
  // registers); the lanes where both hit (~0.4 % of lanes) store their set-1
  // row in a second round.  The stores' LDS issue — five instructions per
  // round whatever the hit lanes, the filter's main cost — is then ~1.2
  // rounds per block pair instead of ~2 (the same rows, in another order).
  auto stage2 = [&](const f32x16& x0, const f32x16& x1, bool h0, bool h1, unsigned pc) {
    const uint64_t m = __ballot(h0 || h1);
    if (m) {
      if (h0 || h1) {
        const unsigned slot = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(m), head));
        f32x4* d = reinterpret_cast<f32x4*>(srow + (slot & (kStageRows - 1)) * kRowF);
        f32x16 y;
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = h0 ? x0[r] : x1[r];
        d[0] = f32x4{y[0], y[1], y[2], y[3]};
        d[1] = f32x4{y[4], y[5], y[6], y[7]};
        d[2] = f32x4{y[8], y[9], y[10], y[11]};
        d[3] = f32x4{y[12], y[13], y[14], y[15]};
        reinterpret_cast<uint2*>(d + 4)[0] = make_uint2(pc, static_cast<unsigned>(h0 ? ql0 : ql1));
      }
      head += __popcll(m);
      if (head - tail >= kWave) flush(kWave);
      stage(x1, h0 && h1, ql1, pc);
    }
  };

#pragma unroll
  for (int s = 0; s < kStages - 1; ++s)
    if (s < nv) issue(tb + s, s);
  if (!my_pieces || nv <= 1) wait_vmcnt<0>();
  else if (nv == 2) wait_vmcnt<PPW>();
  else wait_vmcnt<2 * PPW>();
  __builtin_amdgcn_s_barrier();

  // entering: tile 0 landed (barrier passed), tiles up to 2 issued, the
  // stage of tile 3 free
  dc = 0;
  if (3 < nv) {
    issue(tb + 3, 3);
    dc = dpieces;
  }
  da = wa = (1 < nv) ? dpieces : 0;
  db = wb = (2 < nv) ? dpieces : 0;
  wc = dc;
  // Two accumulator pairs, A for the first half of a tile (block (u, 0)),
  // B for the second (u, 1), and two fragment sets F0 / F1.  A half issues
  // one pair's 16 MFMAs from fragments read during the previous half, then
  // the next block's fragment reads, then filters the other pair (whose
  // MFMAs finished during the previous half).  The ring barrier sits between
  // the halves: every wave has read stage u by then (refill it; tile u + 1
  // has landed).
  bf16x8 f0[KS], f1[KS];
  f32x16 a0 = {}, a1 = {}, b0 = {}, b1 = {};
#ifndef TT_SCAN_PRIO
#define TT_SCAN_PRIO 0
#endif
  // 1: the younger half of the workgroup (waves 4-7) at priority 1 for the
  // whole loop; 2: priority 1 around each MFMA cluster
  if (TT_SCAN_PRIO == 1 && __builtin_amdgcn_readfirstlane(tid) >= kSThreads / 2) __builtin_amdgcn_s_setprio(1);
  auto mfmas = [&](const bf16x8 (&f)[KS], f32x16& x0, f32x16& x1) {
    x0 = f32x16{};
    x1 = f32x16{};
    if (TT_SCAN_PRIO == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      x0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[s], bq0[s], x0, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[s], bq1[s], x1, 0, 0, 0);
    }
    if (TT_SCAN_PRIO == 2) __builtin_amdgcn_s_setprio(0);
  };
  // block (tile u, half t) held in (x0, x1): edge mask, candidate base, maxima
  struct Pend {
    unsigned pc;
    float m0, m1;
  };
  // the split's only tiles that can reach outside [row0, row1): its first and
  // last (scalar tile indices, -1 when that tile is whole)
  const int ue0 = (nv > 0 && edge(static_cast<int64_t>(tb) * kCTile)) ? 0 : -1;
  const int ue1 = (nv > 0 && edge(static_cast<int64_t>(tb + nv - 1) * kCTile)) ? nv - 1 : -1;
  auto prep = [&](f32x16& x0, f32x16& x1, int u, int t) {
    const int64_t cb = static_cast<int64_t>(tb + u) * kCTile + 32 * t;
    if (u == ue0 || u == ue1) {
      mask_pad(x0, cb + 4 * h);
      mask_pad(x1, cb + 4 * h);
    }
    return Pend{a.index_offset + static_cast<unsigned>(cb + 4 * h), max16(x0), max16(x1)};
  };
#ifndef TT_SCAN_PROBE
#define TT_SCAN_PROBE 0
#endif
  // probe builds (timing only, results unused): 1 = maxima without the
  // ballot / staging branches, 2 = no filter work at all
  float probe_acc = 0.f;
  auto stage_pair = [&](const f32x16& x0, const f32x16& x1, const Pend& p) {
    if (TT_SCAN_PROBE == 1) {
      probe_acc = fmaxf(probe_acc, fmaxf(p.m0, p.m1));
    } else if (TT_SCAN_PROBE == 2) {
      probe_acc += x0[0] + x1[5];
    } else if (TT_SCAN_PAIR_STAGE) {
      stage2(x0, x1, p.m0 > tau0, p.m1 > tau1, p.pc);
    } else {
      stage(x0, p.m0 > tau0, ql0, p.pc);
      stage(x1, p.m1 > tau1, ql1, p.pc);
    }
  };
  if (nv > 0) load_frags(f0, smem, 0);
  for (int u = 0; u < nv; ++u) {
    // half A: MFMAs (u, 0) into A (F0 read during the previous half), then
    // read F1 <- (u, 1), then filter (u - 1, 1) from B
#ifndef TT_SCAN_LATE_B
#define TT_SCAN_LATE_B 1
#endif
    // (TT_SCAN_LATE_B: filter B after the ring barrier, so the LDS drain the
    // barrier needs covers the fragment reads only, not B's row stores)
    mfmas(f0, a0, a1);
    load_frags(f1, smem + (u % kStages) * TILE_BYTES, 1);
    if (!TT_SCAN_LATE_B && u > 0) stage_pair(b0, b1, prep(b0, b1, u - 1, 1));
    if (u + 1 < nv) {  // next tile: landed, every wave done with tile u, refill its stage
      wait_vmcnt_atmost((wa - da) + wb + wc);
      // compiler-visible wait + barrier: it then knows the fragment reads
      // before it are complete and puts no wait in front of the next MFMAs
      __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt(63) expcnt(7) lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      wa = wb;
      da = db;
      wb = wc;
      db = dc;
      dc = 0;
      if (u + 4 < nv) {
        issue(tb + u + 4, (u + 4) % kStages);
        dc = dpieces;
      }
      wc = dc;
    }
    if (TT_SCAN_LATE_B && u > 0) stage_pair(b0, b1, prep(b0, b1, u - 1, 1));
    // half B: MFMAs (u, 1) into B, then read F0 <- (u + 1, 0) (stale after the
    // last tile: unused), then filter (u, 0) from A
    mfmas(f1, b0, b1);
    load_frags(f0, smem + ((u + 1) % kStages) * TILE_BYTES, 0);
    stage_pair(a0, a1, prep(a0, a1, u, 0));
#ifndef TT_SCAN_FLUSH_TILES
#define TT_SCAN_FLUSH_TILES 0
#endif
    // optional: every wave flushes at the same tiles (so no wave flushing
    // alone holds the others at the next ring barrier).  Off by default: a
    // wave flushes when 64 rows are staged and at the end (1M x k=100: 44.7
    // vs 45.2 ms with a flush every 4 tiles; every 8: much slower)
#if TT_SCAN_FLUSH_TILES > 0
    if (u % TT_SCAN_FLUSH_TILES == TT_SCAN_FLUSH_TILES - 1)
      while (head > tail) flush(min(head - tail, kWave));
#endif
  }
  if (nv > 0) stage_pair(b0, b1, prep(b0, b1, nv - 1, 1));
  if (TT_SCAN_PROBE && probe_acc == 12345.f) a.count[0] = -2;  // keeps the probe's work alive
  while (head > tail) flush(min(head - tail, kWave));
  if (h == 0) {
    const int n0c = cnt_l[ql0], n1c = cnt_l[ql1];
    a.count[q0 * a.S + split] = n0c > a.cap - 1 ? -1 : n0c;  // slot cap - 1 is scratch
    a.count[q1 * a.S + split] = n1c > a.cap - 1 ? -1 : n1c;
  }
  TT_STAT(0, (h == 0 ? cnt_l[ql0] + cnt_l[ql1] : 0));
}

// Zeroes n words (the failure counters and the image header): a kernel, not
// a hipMemsetAsync, so a captured search holds no memset node (round 5's route
// counts picked up garbage in graphed runs with one: DESIGN.md §8).
__global__ void zero_words_kernel(int* __restrict__ p, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0;
}

void zero_words(void* p, int n, hipStream_t st) {
  hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(256), 0, st, static_cast<int*>(p), n);
}

// tau[q] = min over the splits' estimates (the lowest is the safest: more
// entries, fewer failed certificates).
__global__ void tau_min_kernel(const float* __restrict__ tau_split, int S, int64_t nq, float* __restrict__ tau) {
  const int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (q >= nq) return;
  float t = tau_split[q * S];
  for (int s = 1; s < S; ++s) t = fminf(t, tau_split[q * S + s]);
  tau[q] = t;
}

// tau[q] = the J-th largest of the query's S x 64 bin maxima (all splits'
// samples pooled: one estimate of the rank-R score over the whole candidate
// set, far less noisy than the least of S per-split estimates), to a 16-bit
// order-key prefix (rounded down); -inf if fewer than J bins.  One wave per
// query, S <= 64.
__global__ void __launch_bounds__(256) tau_pool_kernel(const float* __restrict__ bins, int S, int64_t nq, int J,
                                                       float* __restrict__ tau) {
  const int64_t q = blockIdx.x * 4ll + threadIdx.x / kWave;
  const int lane = lane_id();
  if (q >= nq) return;
  const float* b = bins + q * S * 64;
  float v[kWave];
#pragma unroll
  for (int s = 0; s < kWave; ++s) v[s] = s < S ? b[s * 64 + lane] : -INFINITY;
  unsigned res = 0;
#pragma unroll 1
  for (int bit = 15; bit >= 0; --bit) {
    const unsigned c = res | (1u << bit);
    const float f = order_key_float(c << 16);  // smallest float with this prefix (NaN: none)
    int n = 0;
#pragma unroll
    for (int s = 0; s < kWave; ++s) n += v[s] >= f ? 1 : 0;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) n += __shfl_xor(n, m, kWave);
    if (n >= J) res = c;
  }
  const float t = order_key_float(res << 16);
  if (lane == 0) tau[q] = (t > -INFINITY) ? t : -INFINITY;
}

// ---- finalize ------------------------------------------------------------
// Exact score: k-ordered fmaf chain over the fp32 rows (dim real columns).
// qs is the query row in LDS (broadcast reads); the candidate row is loaded in
// batches (16 x float4 or 16 scalars in flight) ahead of the dependent chain.
#ifndef TT_EXACT_CHUNK
#define TT_EXACT_CHUNK 8  // float4 loads in flight per row chunk
#endif
__device__ __forceinline__ float exact_score(const float* __restrict__ qs, const float* __restrict__ c, int dim,
                                             bool vec4) {
  float acc = 0.0f;
  if (vec4) {  // c 16-byte aligned, dim % 4 == 0
    constexpr int NC = TT_EXACT_CHUNK;
    for (int e0 = 0; e0 < dim; e0 += 4 * NC) {
      f32x4 v[NC];
#pragma unroll
      for (int i = 0; i < NC; ++i)
        if (e0 + 4 * i < dim) v[i] = *reinterpret_cast<const f32x4*>(c + e0 + 4 * i);
#pragma unroll
      for (int i = 0; i < NC; ++i)
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

// Lists of one query: `nseg` segments; segment j of query q holds
// count[q * cq + j * cj] entries (-1: overflowed) starting at
// buf + (q * nseg + j) * cap (region form) or at off[q * cq + j * cj] (CSR
// form, cap == 0, entries as int64 = id << 32 | score bits, the same bytes as
// uint2 {score bits, id}); their screens kept s~ > tau[q].
static_assert(TT_INDEX_MAX_SCAN_SPLITS <= kWave, "the finalize prefixes at most 64 list segments");
struct Lists {
  const uint2* buf;
  const int* count;
  const float* tau;
  int nseg;
  int cap;
  const int64_t* off;
  int64_t cq;
  int64_t cj;
};

__device__ __forceinline__ int seg_count(const Lists& L, int64_t q, int j) { return L.count[q * L.cq + j * L.cj]; }
__device__ __forceinline__ const uint2* seg_ptr(const Lists& L, int64_t q, int j) {
  return L.cap ? L.buf + (q * L.nseg + j) * static_cast<int64_t>(L.cap) : L.buf + L.off[q * L.cq + j * L.cj];
}

// Group primitives.  A "group" is the NW waves (NW * 64 threads) that work on
// one query together: NW = 1 is one wave of a workgroup (the helpers are
// wave-local then, so several waves of one workgroup may run them on their own
// LDS regions: the fallback), NW > 1 is the whole workgroup.
template <int NW>
__device__ __forceinline__ void gsync() {
  if constexpr (NW == 1) wsync();
  else __syncthreads();
}
template <int NW>
__device__ __forceinline__ int gtid() {
  if constexpr (NW == 1) return lane_id();
  else return static_cast<int>(threadIdx.x);
}
// Group-wide stream compaction of one chunk of NW * 64 items: returns the
// output slot of this thread's item (meaningful when keep) and advances n by
// the chunk's kept count (uniform over the group).  wcnt: 2 * NW ints of LDS
// (double-buffered by chunk parity `par`).  For NW > 1 it contains a barrier,
// so every thread of the group must call it; for NW = 1 the caller orders its
// LDS reads before its writes (wsync).
template <int NW>
__device__ __forceinline__ int compact_slot(bool keep, int& n, int* wcnt, int& par) {
  const uint64_t m = __ballot(keep);
  const int before = __popcll(m & lanemask_lt64());
  if constexpr (NW == 1) {
    const int p = n + before;
    n += __popcll(m);
    return p;
  } else {
    int* wc = wcnt + (par & 1) * NW;
    ++par;
    const int wave = static_cast<int>(threadIdx.x) / kWave;
    if (lane_id() == 0) wc[wave] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int c = wc[w];
      off += w < wave ? c : 0;
      tot += c;
    }
    const int p = n + off + before;
    n += tot;
    return p;
  }
}

// Group-wide min / max of the threads' values (uniform result); ends with the
// group's LDS writes ordered (gsync).  scratch: 2 * NW words (NW > 1).
template <int NW>
__device__ __forceinline__ void group_minmax(unsigned& mn, unsigned& mx, int* scratch) {
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    mn = min(mn, static_cast<unsigned>(__shfl_xor(static_cast<int>(mn), off, kWave)));
    mx = max(mx, static_cast<unsigned>(__shfl_xor(static_cast<int>(mx), off, kWave)));
  }
  if constexpr (NW > 1) {
    const int wave = static_cast<int>(threadIdx.x) / kWave;
    if (lane_id() == 0) {
      scratch[wave] = static_cast<int>(mn);
      scratch[NW + wave] = static_cast<int>(mx);
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      mn = min(mn, static_cast<unsigned>(scratch[w]));
      mx = max(mx, static_cast<unsigned>(scratch[NW + w]));
    }
  }
  gsync<NW>();
}

// Radix select with 8-bit digits and an LDS histogram over keys the group
// adds with `fill(prefix, hi_mask, shift)` (LDS atomics, any thread).  After
// `passes` digits, `prefix` holds the top 8*passes bits of the K-th largest
// key, `above` = #keys whose top bits are greater, `at` = #keys sharing the
// prefix (above < K <= above + at); at = -1: fewer than K keys.  The bin
// search runs on the group's first wave; bc: 4 words of LDS (NW > 1).
struct Kth {
  unsigned prefix;
  int above;
  int at;
};

// The keys' common top bits, when the caller knows them (kmin / kmax: the
// smallest and largest key), are skipped: resolution starts below them, and
// the last digit may overlap resolved bits (their value is the same for every
// counted key, so the bin order is the digit order).  Bits >= stop_lo are
// resolved (stop_lo = 8: a 24-bit prefix; 0: the exact key).
template <int NW = 1, class Hist>
__device__ Kth radix_select(Hist&& fill, int K, int stop_lo, unsigned* hist, unsigned* bc = nullptr,
                            unsigned kmin = 0u, unsigned kmax = 0xFFFFFFFFu) {
  const int lane = lane_id();
  const int t = gtid<NW>();
  const bool w0 = NW == 1 || t < kWave;
  const int kb = (kmin ^ kmax) == 0 ? 32 : __clz(kmin ^ kmax);  // common top bits
  int lo = 32 - kb;                                               // bits below lo unresolved
  if (lo <= stop_lo) lo = stop_lo + 1;                            // at least one digit pass
  unsigned prefix = lo >= 32 ? 0u : (kmin & (0xFFFFFFFFu << lo));
  int above = 0, at = 0;
  for (; lo > stop_lo;) {
    const int shift = lo - 8 > 0 ? lo - 8 : 0;
    const unsigned hi_mask = lo >= 32 ? 0u : (0xFFFFFFFFu << lo);
    for (int u = t; u < 256; u += NW * kWave) hist[u] = 0;
    gsync<NW>();
    fill(prefix, hi_mask, shift);
    gsync<NW>();
    bool none = false;
    if (w0) {
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
      if (m == 0) {  // fewer than K keys
        none = true;
      } else {
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
      }
      if (NW > 1 && lane == 0) {
        bc[0] = prefix;
        bc[1] = static_cast<unsigned>(above);
        bc[2] = static_cast<unsigned>(at);
        bc[3] = none ? 1u : 0u;
      }
    }
    gsync<NW>();
    if constexpr (NW > 1) {
      prefix = bc[0];
      above = static_cast<int>(bc[1]);
      at = static_cast<int>(bc[2]);
      none = bc[3] != 0;
      __syncthreads();  // bc read by all before the next pass's first wave rewrites it
    }
    if (none) return Kth{0u, 0, -1};
    lo = shift;
  }
  return Kth{prefix, above, at};
}

// Exact selection in LDS: keeps exactly the K best entries by (score desc,
// index asc); *thr = the K-th score (later candidates of an in-order scan need
// a strictly larger score).  aux (NW > 1): 2 * NW + 4 words of LDS.
template <int NW = 1>
__device__ int exact_select(float* sc, unsigned* id, int n, int K, float* thr, unsigned* hist,
                            unsigned* aux = nullptr, unsigned kmin = 0u, unsigned kmax = 0xFFFFFFFFu) {
  if (n <= K) {
    *thr = -INFINITY;
    return n;
  }
  const int t = gtid<NW>();
  constexpr int NT = NW * kWave;
  const Kth r = radix_select<NW>(
      [&](unsigned prefix, unsigned hi_mask, int shift) {
        for (int j = t; j < n; j += NT) {
          const unsigned key = float_order_key(sc[j]);
          if ((key & hi_mask) == prefix) atomicAdd(&hist[(key >> shift) & 0xFFu], 1u);
        }
      },
      K, 0, hist, aux, kmin, kmax);
  const unsigned res = r.prefix;  // exact key of the K-th score
  const int need = K - r.above;   // ties at the K-th score to keep, lowest indices first
  unsigned cut = 0xFFFFFFFFu;
  if (need < r.at) {
    // need-th smallest index among the ties: largest v with #(idx < v) < need
    // (the group's first wave; rare)
    if (NW == 1 || t < kWave) {
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
      if (NW > 1 && t == 0) aux[0] = v;
    }
    if constexpr (NW > 1) {
      __syncthreads();
      cut = aux[0];
      __syncthreads();
    }
  }
  int out = 0, par = 0;
  int* wcnt = reinterpret_cast<int*>(aux) + 4;
  for (int j0 = 0; j0 < n; j0 += NT) {
    const int j = j0 + t;
    const float s = j < n ? sc[j] : 0.0f;
    const unsigned i = j < n ? id[j] : 0u;
    const unsigned key = float_order_key(s);
    const bool keep = j < n && (key > res || (key == res && i <= cut));
    const int p = compact_slot<NW>(keep, out, wcnt, par);
    if constexpr (NW == 1) wsync();
    if (keep) {  // p <= j: a chunk's writes never reach entries not yet read
      sc[p] = s;
      id[p] = i;
    }
  }
  gsync<NW>();
  *thr = order_key_float(res);
  return out;
}

// Ranks the n <= P entries (score desc, index asc) and writes the first k.
// Sort sizes up to kAliasP build their keys in registers, so the key array
// may alias the (score, index) arrays it is built from (the finalize's LDS).
constexpr int kAliasP = 1024;
template <int NW = 1>
__device__ void rank_and_write(const float* sc, const unsigned* id, int n, int k, int P, unsigned long long* sk,
                               float* out_s, int32_t* out_i) {
  const int t = gtid<NW>();
  constexpr int NT = NW * kWave;
  if (NW == 1 && P <= 4 * kWave) {
    // one wave, P <= 256: the whole bitonic network in registers (element
    // i = slot * 64 + lane; strides < 64 between lanes by shuffles, >= 64
    // between a lane's slots) — no LDS round trip or wave barrier per stage
    constexpr int EM = 4;
    const int E = P / kWave > 0 ? P / kWave : 1;
    const int lane = lane_id();
    unsigned long long kv[EM];
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      const int j = e * kWave + lane;
      kv[e] = (e < E && j < n) ? make_key(sc[j], id[j]) : 0ull;
    }
    const int PP = E * kWave;
    for (int size = 2; size <= PP; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        if (stride >= kWave) {
          const int es = stride / kWave;
#pragma unroll
          for (int e = 0; e < EM; ++e) {
            if (e >= E || (e & es)) continue;
            const int i = e * kWave + lane;  // the lower element of the pair (e, e + es)
            const bool desc = (i & size) == 0;
            const unsigned long long x = kv[e], y = kv[e + es];
            const bool sw = (x < y) == desc;
            kv[e] = sw ? y : x;
            kv[e + es] = sw ? x : y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < EM; ++e) {
            if (e >= E) continue;
            const int i = e * kWave + lane;
            const unsigned long long o = __shfl_xor(kv[e], stride, kWave);
            const bool lower = (i & stride) == 0;
            const bool desc = (i & size) == 0;
            const unsigned long long mx = kv[e] > o ? kv[e] : o, mn = kv[e] > o ? o : kv[e];
            kv[e] = (lower == desc) ? mx : mn;
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      const int j = e * kWave + lane;
      if (e < E && j < k) {
        out_s[j] = order_key_float(static_cast<unsigned>(kv[e] >> 32));
        out_i[j] = static_cast<int32_t>(0xFFFFFFFFu - static_cast<unsigned>(kv[e]));
      }
    }
    return;
  }
  if (P <= kAliasP) {
    // keys built in registers first: sk may alias sc / id
    constexpr int PER = (kAliasP + NT - 1) / NT;
    unsigned long long kv[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = t + NT * u;
      kv[u] = j < n ? make_key(sc[j], id[j]) : 0ull;
    }
    gsync<NW>();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int j = t + NT * u;
      if (j < P) sk[j] = kv[u];
    }
  } else {
    for (int j = t; j < P; j += NT) sk[j] = j < n ? make_key(sc[j], id[j]) : 0ull;
  }
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      gsync<NW>();
      for (int i = t; i < P / 2; i += NT) {
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
  gsync<NW>();
  for (int j = t; j < k; j += NT) {
    const unsigned long long key = sk[j];
    out_s[j] = order_key_float(static_cast<unsigned>(key >> 32));
    out_i[j] = static_cast<int32_t>(0xFFFFFFFFu - static_cast<unsigned>(key));
  }
}

struct FinalArgs {
  const float* q;       // fp32 queries of this chunk
  int64_t ldq;
  const float* cand;    // fp32 rows; entry id e is row e - cand_offset
  int64_t ldc;
  int64_t n_rows;
  int64_t cand_offset;
  int64_t zero_base;    // id of row 0 in the output numbering (zero queries)
  int dim;
  int k;
  int L;                // LDS capacity: the whole screened list when it fits (staged), then the cut
  int P;                // bitonic sort size (pow2 >= k)
  int vec4;             // candidate rows are 16-byte aligned float4 rows
  int64_t nq;
  const int* qflags;
  const float* qmarg;
  const float2* qnorm;      // per query (|bf16(q)|, |q - bf16(q)|)
  const float2* cnorm;      // per candidate row of the index: (|bf16(c)|, |c - bf16(c)|)
  const IndexHeader* hdr;   // the maxima of cnorm (the certificate's bound for unlisted rows)
  Lists lists;
  float* out_s;
  int32_t* out_i;
  int* fail_count;
  int* fail_list;
  // candidate-sharded two-phase form (tt_bruteforce_shard_*):
  float* kth_lb;        // select pass: per query lb(k-th screened score) (-inf: certificate failed), then stop
  const float* floor;   // rescore pass: per query lower bound on the GLOBAL k-th exact score
};

// LDS of one finalize group: query row, (score, id) list of L, the ranking
// keys when they cannot alias the list, 256 radix bins, 2 NW + 4 aux words
__host__ __device__ inline size_t final_lds_bytes(int L, int P, int NW = 1) {
  return 128 * sizeof(float) + static_cast<size_t>(L) * 8 + (P <= kAliasP ? 0 : static_cast<size_t>(P) * 8) +
         256 * sizeof(unsigned) + static_cast<size_t>(2 * NW + 4) * sizeof(unsigned);
}

// One query per group of NW waves (the workgroup).  NW > 1 splits every
// phase's loops over the waves (large k: long lists, many survivors, a
// P-element sort), so a query's latency chain shrinks while its list stays
// in LDS.
#ifndef TT_FINAL_WPE
#define TT_FINAL_WPE 0  // > 0: the finalize compiled for at least that many waves per SIMD
#endif
template <int NW>
__global__ void __launch_bounds__(NW * kWave)
#if TT_FINAL_WPE > 0
    __attribute__((amdgpu_waves_per_eu(TT_FINAL_WPE)))
#endif
    finalize_kernel(const FinalArgs a) {
  constexpr int NT = NW * kWave;
  extern __shared__ __attribute__((aligned(16))) char fsm[];
  float* qs = reinterpret_cast<float*>(fsm);  // query row (dim <= 128)
  float* sc = qs + 128;
  unsigned* id = reinterpret_cast<unsigned*>(sc + a.L);
  // for P <= kAliasP the ranking's keys reuse the LDS of sc / id (P <= L)
  const bool alias = a.P <= kAliasP;
  unsigned long long* sk = alias ? reinterpret_cast<unsigned long long*>(sc)
                                 : reinterpret_cast<unsigned long long*>(id + a.L);
  unsigned* hist = alias ? id + a.L : reinterpret_cast<unsigned*>(sk + a.P);  // 256 radix bins
  unsigned* aux = hist + 256;                                                // 2 NW + 4 words
  int* wcnt = reinterpret_cast<int*>(aux) + 4;
  const int64_t q = blockIdx.x;
  const int t = gtid<NW>();
  const int K = a.k;
  const Lists& Ls = a.lists;
#ifdef TT_INDEX_NOINSERT
  return;  // probe build: the screen kept nothing
#endif
  float* out_s = a.out_s + q * K;
  int32_t* out_i = a.out_i + q * K;
  const int fl = a.qflags[q];
  if (fl & kQZero) {  // every score is exactly +0: indices 0..k-1 by the tie rule
    if (a.kth_lb) {
      if (t == 0) a.kth_lb[q] = 0.0f;
      return;
    }
    for (int j = t; j < K; j += NT) {
      out_s[j] = 0.0f;
      out_i[j] = static_cast<int32_t>(a.zero_base + j);
    }
    return;
  }
  const bool rel = (fl & kQRel) != 0;
  const float m = a.qmarg[q];
  const float2 qn = a.qnorm[q];
  // the per-row screen bound of list entry id (row_err)
  auto err_row = [&](unsigned idv) {
    const float2 cn = a.cnorm[static_cast<int64_t>(idv) - a.cand_offset];
    return row_err(qn.x, qn.y, cn.x, cn.y);
  };
  // the segments' counts, one load each by the first wave, to an exclusive
  // prefix pre[0..64] in LDS (the radix bins, cleared by the select later;
  // padded with the total), so the list is read as one flat index space
  // rather than segment by segment (64 dependent round trips at S = 64)
  int* const pre = reinterpret_cast<int*>(hist);
  if (t < kWave) {
    const int c = t < Ls.nseg ? seg_count(Ls, q, t) : 0;
    int v = c;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const int o = __shfl_up(v, off, kWave);
      if (t >= off) v += o;
    }
    pre[t + 1] = v;
    if (t == 0) pre[0] = 0;
    const bool bad = __ballot(c < 0) != 0;
    if (t == 0) pre[kWave + 1] = bad ? 1 : 0;
  }
  gsync<NW>();
  const int ntot = pre[kWave];
  bool fail = pre[kWave + 1] != 0 || ntot < K;
  const float tmax = Ls.tau[q];
  float X = -INFINITY;
  // the whole list read once into LDS when it fits (the select's passes and
  // the cut then read LDS, not the lists in memory)
  const bool staged = !fail && ntot <= a.L;
  unsigned kmin = 0xFFFFFFFFu, kmax = 0u;  // the staged list's key range (radix select skips its common bits)
  if (staged) {
    for (int i0 = 0; i0 < ntot; i0 += 4 * NT) {
      uint2 en[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * NT + t;
        if (i < ntot) {
          int j = 0;  // the segment holding flat entry i: the last j with pre[j] <= i
#pragma unroll
          for (int st = kWave / 2; st > 0; st >>= 1) j += pre[j + st] <= i ? st : 0;
          en[u] = seg_ptr(Ls, q, j)[i - pre[j]];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * NT + t;
        if (i < ntot) {
          sc[i] = __uint_as_float(en[u].x);
          id[i] = en[u].y;
          const unsigned k = float_order_key(__uint_as_float(en[u].x));
          kmin = min(kmin, k);
          kmax = max(kmax, k);
        }
      }
    }
    group_minmax<NW>(kmin, kmax, wcnt);
  } else {
    gsync<NW>();  // pre read by all before the select clears the bins
  }
#if defined(TT_FINAL_STOP) && TT_FINAL_STOP == 1  // timing probe: phases up to here only
  for (int j = t; j < K; j += NT) out_s[j] = sc[j];
  return;
#endif

  if (!fail) {
    // K-th largest screened score to a 24-bit key prefix (rounded down)
    const Kth r = radix_select<NW>(
        [&](unsigned prefix, unsigned hi_mask, int shift) {
          if (staged) {
            for (int i = t; i < ntot; i += NT) {
              const unsigned key = float_order_key(sc[i]);
              if ((key & hi_mask) == prefix) atomicAdd(&hist[(key >> shift) & 0xFFu], 1u);
            }
            return;
          }
          for (int j = 0; j < Ls.nseg; ++j) {
            const int c = seg_count(Ls, q, j);
            const uint2* e = seg_ptr(Ls, q, j);
            for (int i = t; i < c; i += NT) {
              const unsigned key = float_order_key(__uint_as_float(e[i].x));
              if ((key & hi_mask) == prefix) atomicAdd(&hist[(key >> shift) & 0xFFu], 1u);
            }
          }
        },
        K, 8, hist, aux, staged ? kmin : 0u, staged ? kmax : 0xFFFFFFFFu);
    fail = r.at < 0;
    if (!fail) {
      // certificate (below) is the only reason counted in stats[1]
      X = lb_of(order_key_float(r.prefix), m, rel);
      // per-row bounds: the >= K entries at or above the K-th key prefix each
      // score at least max(lb(s~), s~ - err_row) exactly, so X = the least of
      // those lower bounds has >= K candidates at or above it (and is >= the
      // relative / absolute form's lb(prefix))
#ifndef TT_INDEX_ROW_X
#define TT_INDEX_ROW_X 0
#endif
      if (TT_INDEX_ROW_X) {
      unsigned xk = 0xFFFFFFFFu, unused = 0u;
      auto visit = [&](float sv, unsigned iv) {
        if (float_order_key(sv) >= r.prefix)
          xk = min(xk, float_order_key(fmaxf(lb_of(sv, m, rel), sv - err_row(iv))));
      };
      if (staged) {
        for (int i = t; i < ntot; i += NT) visit(sc[i], id[i]);
      } else {
        for (int j = 0; j < Ls.nseg; ++j) {
          const int c = seg_count(Ls, q, j);
          const uint2* e = seg_ptr(Ls, q, j);
          for (int i = t; i < c; i += NT) visit(__uint_as_float(e[i].x), e[i].y);
        }
      }
      group_minmax<NW>(xk, unused, wcnt);
      if (xk != 0xFFFFFFFFu) X = fmaxf(X, order_key_float(xk));
      }
      // certificate: every list kept all s~ > tau, and an unlisted row's
      // exact score is <= min(ub(tau), tau + the per-row bound at the index's
      // largest row norms) < X, which rules it out of the exact top-K (K
      // members >= X)
      const float ubt = fminf(ub_of(tmax, m, rel),
                              tmax + row_err(qn.x, qn.y, __uint_as_float(a.hdr->maxcb_bits),
                                             __uint_as_float(a.hdr->maxrc_bits)));
      fail = !(X > ubt);
      if (fail && t == 0) TT_STAT(1, 1);
    }
  }
  if (a.kth_lb) {  // select pass: at least K rows of these candidates score >= X exactly
    if (t == 0) a.kth_lb[q] = fail ? -INFINITY : X;
    return;
  }
#if defined(TT_FINAL_STOP) && TT_FINAL_STOP == 2  // timing probe: phases up to here only
  for (int j = t; j < K; j += NT) out_s[j] = sc[j];
  return;
#endif

  // a member of the global top-K scores >= floor: only those can matter
  if (a.floor) X = fmaxf(X, a.floor[q]);
  int n = 0, par = 0;
  if (!fail && staged) {
    for (int e = t; e < a.dim; e += NT) qs[e] = a.q[q * a.ldq + e];
    // in-place compaction of the kept ids (writes never pass the reads)
    for (int i0 = 0; i0 < ntot; i0 += NT) {
      const int i = i0 + t;
      const float sv = i < ntot ? sc[i] : 0.0f;
      const unsigned iv = i < ntot ? id[i] : 0u;
      // ub = min(relative / absolute form, s~ + per-row bound): its row
      // norms are read only for the entries the first form keeps
      const bool keepit = i < ntot && ub_of(sv, m, rel) >= X && sv + err_row(iv) >= X;
      const int p = compact_slot<NW>(keepit, n, wcnt, par);
      if constexpr (NW == 1) wsync();
      if (keepit) id[p] = iv;
      if constexpr (NW == 1) wsync();
    }
  } else if (!fail) {
    for (int e = t; e < a.dim; e += NT) qs[e] = a.q[q * a.ldq + e];
    for (int j = 0; j < Ls.nseg && !fail; ++j) {
      const int c = seg_count(Ls, q, j);
      const uint2* e = seg_ptr(Ls, q, j);
      for (int i0 = 0; i0 < c; i0 += NT) {
        const int i = i0 + t;
        const uint2 en = i < c ? e[i] : make_uint2(0u, 0u);
        const bool keepit = i < c && ub_of(__uint_as_float(en.x), m, rel) >= X &&
                            __uint_as_float(en.x) + err_row(en.y) >= X;
        const int p = compact_slot<NW>(keepit, n, wcnt, par);
        if (n > a.L) {  // uniform over the group
          fail = true;
          break;
        }
        if (keepit) id[p] = en.y;
      }
    }
  }
  gsync<NW>();
  if (fail) {
    if (t == 0) {
      const int slot = atomicAdd(a.fail_count, 1);
      a.fail_list[slot] = static_cast<int>(q);
      TT_STAT(3, 1);
    }
    return;
  }
  if (t == 0) TT_STAT(2, n);
#if defined(TT_FINAL_STOP) && TT_FINAL_STOP == 3  // timing probe: phases up to here only
  for (int j = t; j < K; j += NT) out_s[j] = sc[j];
  return;
#endif
  unsigned emin = 0xFFFFFFFFu, emax = 0u;
  for (int j = t; j < n; j += NT) {
    const int64_t row = static_cast<int64_t>(id[j]) - a.cand_offset;
#ifdef TT_FINAL_NORESCORE  // timing probe only: no candidate rows read (results wrong, no ties)
    sc[j] = static_cast<float>(row);
#else
    sc[j] = exact_score(qs, a.cand + row * a.ldc, a.dim, a.vec4 != 0) + 0.0f;
#endif
    const unsigned k = float_order_key(sc[j]);
    emin = min(emin, k);
    emax = max(emax, k);
  }
  group_minmax<NW>(emin, emax, wcnt);
#if defined(TT_FINAL_STOP) && TT_FINAL_STOP == 4  // timing probe: phases up to here only
  for (int j = t; j < K; j += NT) out_s[j] = sc[j];
  return;
#endif
  float kth;
  n = exact_select<NW>(sc, id, n, K, &kth, hist, aux, emin, emax);
#if defined(TT_FINAL_STOP) && TT_FINAL_STOP == 5  // timing probe: phases up to here only
  for (int j = t; j < K; j += NT) out_s[j] = sc[j];
  return;
#endif

  rank_and_write<NW>(sc, id, n, min(n, K), a.P, sk, out_s, out_i);
  // with a floor fewer than K may remain: pad (sorts after every real entry)
  for (int j = n + t; j < K; j += NT) {
    out_s[j] = -INFINITY;
    out_i[j] = 0x7FFFFFFF;
  }
}

// Exact fallback for the queries the finalize could not certify.  A
// persistent grid of 4-wave workgroups takes work items from a global
// counter: item (f, p) scans part p of the candidate rows for failed query f
// with the fp32 chain (wave w takes the part's 64-row chunks w, w + 4, ... in
// index order, so a strict threshold at its running K-th score is exact),
// merges its waves' exact top-K lists and writes them to scratch slot (f, p);
// the workgroup that completes a query's last part merges the P lists and
// writes the answer.  Queries beyond the scratch slots are scanned whole by
// one workgroup.
constexpr int kFbWaves = 4;
constexpr int kFbSlots = 1024;       // failed queries served by the parallel form per chunk
constexpr int kFbGrid = 512;         // persistent workgroups

struct FallbackArgs {
  const float* q;
  int64_t ldq;
  const float* cand;  // the rows to scan (all of them)
  int64_t ldc;
  int64_t n_rows;
  int64_t id_base;    // output id of row 0
  int dim;
  int k;
  int L;              // per-wave list capacity
  int P;              // bitonic sort size
  int parts;          // candidate parts per failed query (parts * k <= 8192)
  int vec4;
  const int* fail_count;
  const int* fail_list;
  int* ctrl;          // [0] item counter, [1 + f] parts done of slot f (zeroed per chunk)
  uint2* scratch;     // [kFbSlots][parts][k]
  int* scratch_n;     // [kFbSlots][parts]
  float* out_s;
  int32_t* out_i;
};

__host__ __device__ inline int fallback_merge_cap(int parts, int k) {
  return parts * k > kFbWaves * k ? parts * k : kFbWaves * k;
}
__host__ __device__ inline size_t fallback_lds_bytes(int L, int P, int parts, int k) {
  return 128 * sizeof(float) + static_cast<size_t>(kFbWaves) * (static_cast<size_t>(L) * 8 + 256 * sizeof(unsigned)) +
         static_cast<size_t>(fallback_merge_cap(parts, k)) * 8 + static_cast<size_t>(P) * 8 + 16 * sizeof(int);
}

__global__ void __launch_bounds__(kFbWaves * kWave) fallback_kernel(const FallbackArgs a) {
  extern __shared__ __attribute__((aligned(16))) char fsm[];
  const int wave = threadIdx.x / kWave;
  const int lane = lane_id();
  const int K = a.k, PT = a.parts;
  float* qs = reinterpret_cast<float*>(fsm);
  char* wbase = fsm + 128 * sizeof(float) + static_cast<size_t>(wave) * (static_cast<size_t>(a.L) * 8 + 1024);
  float* sc = reinterpret_cast<float*>(wbase);
  unsigned* id = reinterpret_cast<unsigned*>(sc + a.L);
  unsigned* hist = id + a.L;
  const int MC = fallback_merge_cap(PT, K);
  char* mbase = fsm + 128 * sizeof(float) + static_cast<size_t>(kFbWaves) * (static_cast<size_t>(a.L) * 8 + 1024);
  float* msc = reinterpret_cast<float*>(mbase);
  unsigned* mid = reinterpret_cast<unsigned*>(msc + MC);
  unsigned long long* sk = reinterpret_cast<unsigned long long*>(mid + MC);
  int* sh = reinterpret_cast<int*>(sk + a.P);  // [0] item, [1..4] wave counts, [5] merge flag
  const int nf = *a.fail_count;
  const int npar = nf < kFbSlots ? nf : kFbSlots;
  const int total = npar * PT + (nf - npar);
  for (;;) {
    __syncthreads();
    if (threadIdx.x == 0) sh[0] = atomicAdd(&a.ctrl[0], 1);
    __syncthreads();
    const int item = sh[0];
    if (item >= total) break;
    const bool part = item < npar * PT;
    const int f = part ? item / PT : npar + (item - npar * PT);
    const int pi = part ? item % PT : 0;
    const int64_t q = a.fail_list[f];
    const int64_t r0 = part ? (a.n_rows * pi) / PT : 0;
    const int64_t r1 = part ? (a.n_rows * (pi + 1)) / PT : a.n_rows;
    for (int e = threadIdx.x; e < a.dim; e += blockDim.x) qs[e] = a.q[q * a.ldq + e];
    __syncthreads();
    float ethr = -INFINITY;
    int n = 0;
    for (int64_t c0 = r0 + static_cast<int64_t>(wave) * kWave; c0 < r1; c0 += kFbWaves * kWave) {
      const int64_t c = c0 + lane;
      float sv = -INFINITY;
      if (c < r1) sv = exact_score(qs, a.cand + c * a.ldc, a.dim, a.vec4 != 0) + 0.0f;
      const bool keepit = c < r1 && sv > ethr;
      const uint64_t m = __ballot(keepit);
      if (keepit) {
        const int pp = n + __popcll(m & lanemask_lt64());
        sc[pp] = sv;
        id[pp] = static_cast<unsigned>(a.id_base + c);
      }
      n += __popcll(m);
      if (n > a.L - kWave) {
        wsync();
        n = exact_select(sc, id, n, K, &ethr, hist);
      }
    }
    wsync();
    float kth;
    n = exact_select(sc, id, n, K, &kth, hist);
    for (int j = lane; j < n; j += kWave) {
      msc[wave * K + j] = sc[j];
      mid[wave * K + j] = id[j];
    }
    if (lane == 0) sh[1 + wave] = n;
    __syncthreads();
    if (wave == 0) {
      int nm = sh[1];
      for (int w = 1; w < kFbWaves; ++w) {  // compact the wave lists to the front
        const int cw = sh[1 + w];
        for (int j0 = 0; j0 < cw; j0 += kWave) {
          const int j = j0 + lane;
          const float sv = j < cw ? msc[w * K + j] : 0.0f;
          const unsigned iv = j < cw ? mid[w * K + j] : 0u;
          wsync();
          if (j < cw) {
            msc[nm + j] = sv;
            mid[nm + j] = iv;
          }
          wsync();
        }
        nm += cw;
      }
      nm = exact_select(msc, mid, nm, K, &kth, hist);
      if (!part) {
        rank_and_write(msc, mid, nm, K, a.P, sk, a.out_s + q * K, a.out_i + q * K);
        if (lane == 0) sh[5] = 0;
      } else {
        uint2* dst = a.scratch + (static_cast<int64_t>(f) * PT + pi) * K;
        for (int j = lane; j < nm; j += kWave) dst[j] = make_uint2(__float_as_uint(msc[j]), mid[j]);
        if (lane == 0) a.scratch_n[f * PT + pi] = nm;
        __threadfence();  // the part's list is visible chip-wide before it is counted
        int last = 0;
        if (lane == 0) last = atomicAdd(&a.ctrl[1 + f], 1) == PT - 1;
        last = __shfl(last, 0, kWave);
        if (lane == 0) sh[5] = last;
      }
    }
    __syncthreads();
    if (part && sh[5] && wave == 0) {  // every part of query f is in scratch: merge them
      __threadfence();
      int nm = 0;
      for (int pj = 0; pj < PT; ++pj) {
        const int cj = a.scratch_n[f * PT + pj];
        const uint2* src = a.scratch + (static_cast<int64_t>(f) * PT + pj) * K;
        for (int j = lane; j < cj; j += kWave) {
          const uint2 e = src[j];
          msc[nm + j] = __uint_as_float(e.x);
          mid[nm + j] = e.y;
        }
        nm += cj;
      }
      wsync();
      nm = exact_select(msc, mid, nm, K, &kth, hist);
      rank_and_write(msc, mid, nm, K, a.P, sk, a.out_s + q * K, a.out_i + q * K);
    }
  }
}

// ---- host plan -------------------------------------------------------------
#ifndef TT_INDEX_R_MUL  // target screened entries per query: TT_INDEX_R_MUL * k + TT_INDEX_R_ADD
#define TT_INDEX_R_MUL 3.0
#endif
#ifndef TT_INDEX_R_MUL_BIG  // the same for k >= 512 (rank estimates far from the sample's tail)
#define TT_INDEX_R_MUL_BIG 1.2
#endif
#ifndef TT_INDEX_POOL  // 1: the pooled rank estimate when the sample pass splits the candidates (k < 512)
#define TT_INDEX_POOL 1
#endif
#ifndef TT_INDEX_R_ADD
#define TT_INDEX_R_ADD 100.0
#endif
struct SearchPlan {
  int S, NS, jsel, cap, L, LF, P, k, parts;
  int pool;  // pooled estimate (> 1 sample splits): tau = the J-th largest of a query's Ss x 64 bins
  int J;
  int Ss;  // sample-pass splits (<= S): their estimates give one tau per query
  int NW;  // waves per finalize workgroup (one query each)
  int64_t chunk;
};

// Finalize group size: one wave per query for small k (many queries in
// flight hide each other's latency); four for large k, whose long lists,
// ~1.3k rescored rows and P-element sort make one query's chain the latency.
// TT_FINAL_WAVES (1 / 2 / 4) overrides, TT_FINAL_LF the staged list size.
inline int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

// R = target list entries per query over the whole candidate set (3k + 100),
// split evenly over the S splits x `shards` ranks screening disjoint ranges;
// each split estimates its share and the query keeps the lowest estimate.
SearchPlan plan_search(int64_t nq, int64_t n_rows, int k, int shards) {
  SearchPlan p{};
  const int64_t ntiles = ceil_div(n_rows, kCTile) + 1;  // + 1: a range need not start on a tile
  p.P = next_pow2(k < 2 ? 2 : k);
  p.k = k;
  p.parts = 8192 / k < 1 ? 1 : (8192 / k > 64 ? 64 : 8192 / k);
  p.L = static_cast<int>(round_up(2 * static_cast<int64_t>(k) + 256, kWave));
#ifndef TT_INDEX_LF
#define TT_INDEX_LF 1024
#endif
  p.LF = p.L > TT_INDEX_LF ? p.L : TT_INDEX_LF;  // finalize: a query's whole list (~3k + 100 entries) fits
  static const int nw_env = env_int("TT_FINAL_WAVES", 0), lf_env = env_int("TT_FINAL_LF", 0);
  p.NW = nw_env == 1 || nw_env == 2 || nw_env == 4 ? nw_env : (k >= 512 ? 4 : 1);
  if (p.NW > 1) {  // the whole list staged in the group's LDS
    const int lf = static_cast<int>(round_up(static_cast<int64_t>(3.5 * k) + 128, kWave));
    if (lf > p.LF) p.LF = lf;
  }
  if (lf_env >= p.L) p.LF = static_cast<int>(round_up(lf_env, kWave));
  const int64_t qblocks = ceil_div(nq > 0 ? nq : 1, kQPerWG);
  p.S = 1;  // enough workgroups for the 256 CUs: split the candidates of few query blocks
  while (p.S < kMaxSplits && qblocks * p.S < 256 && ntiles / (2 * p.S) >= TT_INDEX_SPLIT_TILES) p.S *= 2;
  p.Ss = p.S;
  const int64_t nts = ceil_div(ntiles, p.S);  // tiles per split
  const double ns_cand = static_cast<double>(nts) * kCTile;
  // 3k + 100 below k = 512; 1.2k + 100 from there (at the runner's 2048 x
  // k = 1000: 3k -> 1.5k + 100 took the lists from 4642 to 2704 entries per
  // query after the min over 32 split estimates, 0.705 -> 0.607 ms per
  // search; 1.5k -> 1.2k: 0.54 -> 0.46 ms, and 1.0k-1.15k no faster;
  // bit-exact index tests green at each — profiles/r05_index_scan_ab.txt)
  const double rmul = k >= 512 ? TT_INDEX_R_MUL_BIG : TT_INDEX_R_MUL;
  const double R = (rmul * k + TT_INDEX_R_ADD) / (static_cast<double>(p.S) * (shards > 0 ? shards : 1));
  double mu;  // expected entries per (query, split)
  if (nts < 16 || R >= 0.25 * ns_cand) {
    p.NS = 0;  // keep every score of the split
    p.jsel = 1;
    mu = ns_cand;
  } else {
    // 64 bins of NS samples each; the smallest bin must sit well below
    // rank R: NS <= N ln64 / (1.5 R)
    const double ns_max = ns_cand * std::log(64.0) / (1.5 * R);
    int NS = static_cast<int>(nts / 4 < kMaxSample ? nts / 4 : kMaxSample);
    if (NS > ns_max) NS = static_cast<int>(ns_max);
    if (NS < 1) NS = 1;
    p.NS = NS;
    const double pbin = 1.0 - std::exp(-1.0 * NS * R / ns_cand);
    int j = static_cast<int>(std::lround(64.0 * pbin));
    p.jsel = j < 1 ? 1 : (j > 64 ? 64 : j);
    mu = R;
    // pooled: every split's 64 bins estimate the same global rank (R per
    // split x Ss splits), so the J-th largest of all Ss x 64 estimates it
    // once — lists near their target instead of above it (2048 x k = 100:
    // 0.31 -> 0.20 ms per search).  Not for k >= 512: there the rank sits
    // deep in the bins (pbin near 1) and the pooled estimate lands high
    // enough to fail certificates (runner point 0.46 -> 1.7 ms at 1.3k + 100,
    // no gain at 1.5k + 100; profiles/r05_index_scan_ab.txt)
    if (TT_INDEX_POOL && p.Ss > 1 && p.Ss <= 64 && k < 512) {
      const int64_t jj = std::llround(64.0 * p.Ss * pbin);
      p.pool = 1;
      p.J = static_cast<int>(jj < 1 ? 1 : (jj > 64 * p.Ss ? 64 * p.Ss : jj));
    }
  }
  if (p.NS > 0) {
    // the scan needs only the per-query tau (the min over the sample
    // splits), so it may split the candidates further than the sample pass
    // (whose per-split estimates need enough tiles): a 2048-query batch gets
    // 4 x 64 instead of 4 x 32 workgroups
    while (p.S < TT_INDEX_MAX_SCAN_SPLITS && qblocks * p.S < 256 && ntiles / (2 * p.S) >= TT_INDEX_SCAN_TILES) {
      p.S *= 2;
      mu *= 0.5;
    }
  }
  // the lowest of S (x shards) estimates lands lower than each: room for it
  p.cap = next_pow2(static_cast<int>(3.0 * mu * (p.S > 1 ? 2.0 : 1.0)) + 64);
  const size_t per_query = static_cast<size_t>(p.S) * p.cap * sizeof(uint2);
  int64_t chunk = static_cast<int64_t>(kListBudget / per_query) / kQPerWG * kQPerWG;
  if (chunk < kQPerWG) chunk = kQPerWG;
  const int64_t need = round_up(nq > 0 ? nq : 1, kQPerWG);
  p.chunk = chunk < need ? chunk : need;
  return p;
}

struct SearchWs {
  __bf16* qb;
  int* qflags;
  float* qmarg;
  float2* qnorm;
  uint2* buf;
  int* count;
  float* tau_split;
  float* tau;
  float* bins;      // pooled estimate: [nq_pad][Ss][64] bin maxima
  int* fail_count;  // [0] failures, then the fallback's ctrl words
  int* fail_list;
  uint2* fb_scratch;
  int* fb_scratch_n;
};

SearchWs carve_search(Carver& cv, int D, const SearchPlan& p, bool lists, bool finalize) {
  const int64_t nq_pad = p.chunk;
  SearchWs w{};
  w.qb = cv.take<__bf16>(nq_pad * D);
  w.qflags = cv.take<int>(nq_pad);
  w.qmarg = cv.take<float>(nq_pad);
  w.qnorm = cv.take<float2>(nq_pad);
  if (lists) {
    w.buf = cv.take<uint2>(nq_pad * p.S * static_cast<int64_t>(p.cap));
    w.count = cv.take<int>(nq_pad * p.S);
    w.tau_split = cv.take<float>(nq_pad * p.Ss);
    w.tau = cv.take<float>(nq_pad);
    if (p.pool) w.bins = cv.take<float>(nq_pad * p.Ss * 64);
  }
  if (finalize) {
    w.fail_count = cv.take<int>(2 + kFbSlots);
    w.fail_list = cv.take<int>(nq_pad);
    w.fb_scratch = cv.take<uint2>(static_cast<int64_t>(kFbSlots) * p.parts * p.k);
    w.fb_scratch_n = cv.take<int>(static_cast<int64_t>(kFbSlots) * p.parts);
  }
  return w;
}

template <int D>
void launch_pass(const ScreenArgs& sa, int64_t nq_pad, bool sample, hipStream_t st) {
  const dim3 grid((nq_pad / kQPerWG) * sa.S), block(kSThreads);
  if (sample) {
    hipLaunchKernelGGL((sample_kernel<D>), grid, block, 0, st, sa);
  } else {
    probe_begin(TT_PROBE_INDEX_SCREEN, st);
    hipLaunchKernelGGL((scan_kernel<D>), grid, block, 0, st, sa);
    probe_end(TT_PROBE_INDEX_SCREEN, st);
  }
}

int run_pass(int D, const ScreenArgs& sa, int64_t nq_pad, bool sample, hipStream_t st) {
  switch (D) {
    case 32: launch_pass<32>(sa, nq_pad, sample, st); break;
    case 64: launch_pass<64>(sa, nq_pad, sample, st); break;
    default: launch_pass<128>(sa, nq_pad, sample, st); break;
  }
  TT_CHECK_LAUNCH();
  return TT_OK;
}

int run_prep(const float* q, int64_t ldq, int64_t nq, int dim, int D, const void* index, const SearchWs& w,
             bool with_rows, hipStream_t st) {
  const int64_t nq_pad = round_up(nq, kQPerWG);
  hipLaunchKernelGGL(query_prep_kernel, dim3(ceil_div(nq_pad, 4)), dim3(256), 0, st, q, ldq, nq, dim, nq_pad, D, index,
                     with_rows ? w.qb : nullptr, w.qflags, w.qmarg, w.qnorm);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

// sample pass + min over the splits -> tau[0..nq)
int run_estimate(int D, const void* index, int64_t row0, int64_t row1, int64_t nq, const SearchPlan& p,
                 const SearchWs& w, float* tau, hipStream_t st) {
  const int64_t nq_pad = round_up(nq, kQPerWG);
  ScreenArgs sa{index, w.qb, nq, row0, row1, p.Ss, p.NS, p.jsel, p.cap, 0u, nullptr, nullptr, w.tau_split, nullptr,
                p.pool ? w.bins : nullptr};
  if (int rc = run_pass(D, sa, nq_pad, true, st)) return rc;
  if (p.pool)
    hipLaunchKernelGGL(tau_pool_kernel, dim3(ceil_div(nq, 4)), dim3(256), 0, st, w.bins, p.Ss, nq, p.J, tau);
  else
    hipLaunchKernelGGL(tau_min_kernel, dim3(ceil_div(nq, 256)), dim3(256), 0, st, w.tau_split, p.Ss, nq, tau);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

int run_scan(int D, const void* index, int64_t row0, int64_t row1, int64_t nq, const SearchPlan& p, const SearchWs& w,
             const float* tau, unsigned index_offset, hipStream_t st) {
  const int64_t nq_pad = round_up(nq, kQPerWG);
  ScreenArgs sa{index, w.qb, nq, row0, row1, p.S, p.NS, p.jsel, p.cap, index_offset, w.buf, w.count, nullptr, tau};
  return run_pass(D, sa, nq_pad, false, st);
}

template <int NW>
int launch_finalize_nw(const FinalArgs& fa, int64_t nq, const SearchPlan& p, hipStream_t st) {
  const size_t shm = final_lds_bytes(p.LF, p.P, NW);
  if (shm > 65536)
    TT_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(finalize_kernel<NW>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(shm)));
  hipLaunchKernelGGL(finalize_kernel<NW>, dim3(nq), dim3(NW * kWave), shm, st, fa);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

int launch_finalize(const FinalArgs& fa, int64_t nq, const SearchPlan& p, hipStream_t st) {
  switch (p.NW) {
    case 4: return launch_finalize_nw<4>(fa, nq, p, st);
    case 2: return launch_finalize_nw<2>(fa, nq, p, st);
    default: return launch_finalize_nw<1>(fa, nq, p, st);
  }
}

int run_finalize(const FinalArgs& fa, const FallbackArgs& fb, int64_t nq, const SearchPlan& p, hipStream_t st) {
  const size_t fshm = fallback_lds_bytes(p.L, p.P, p.parts, p.k);
  if (fshm > 65536)
    TT_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fallback_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(fshm)));
  probe_begin(TT_PROBE_INDEX_FINALIZE, st);
  if (int rc = launch_finalize(fa, nq, p, st)) return rc;
  probe_end(TT_PROBE_INDEX_FINALIZE, st);
  hipLaunchKernelGGL(fallback_kernel, dim3(kFbGrid), dim3(kFbWaves * kWave), fshm, st, fb);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

inline const float2* index_norms(const void* index, int64_t n_cand, int D) {
  return reinterpret_cast<const float2*>(static_cast<const char*>(index) + norms_offset(round_up(n_cand, kCTile), D));
}
inline const IndexHeader* index_header(const void* index) { return static_cast<const IndexHeader*>(index); }

inline bool is_vec4(const float* cand, int64_t ldc, int dim) {
  return reinterpret_cast<uintptr_t>(cand) % 16 == 0 && ldc % 4 == 0 && dim % 4 == 0;
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
  zero_words(index, 16, st);
  const int D = pick_dpad(dim);
  const int64_t n_pad = round_up(n_cand, kCTile);
  hipLaunchKernelGGL(build_kernel, dim3(ceil_div(n_pad, 4 * kBuildRowsPerWave)), dim3(256), 0, st, cand, ldc, n_cand,
                     dim, n_pad, D, index);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" size_t tt_bruteforce_workspace_size(int64_t n_queries, int64_t n_cand, int32_t dim, int32_t k) {
  if (n_queries < 1 || n_cand < 1 || k < 1 || pick_dpad(dim) == 0) return 0;
  const SearchPlan p = plan_search(n_queries, n_cand, k, 1);
  Carver cv(nullptr, 0);
  carve_search(cv, pick_dpad(dim), p, true, true);
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
  const SearchPlan p = plan_search(n_queries, n_cand, k, 1);
  Carver cv(workspace, workspace_bytes);
  SearchWs w = carve_search(cv, D, p, true, true);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_bruteforce_search: workspace %zu < required %zu", workspace_bytes, cv.used());
  hipStream_t st = to_stream(stream);
  const int vec4 = is_vec4(cand, ldc, dim) ? 1 : 0;
  for (int64_t q0 = 0; q0 < n_queries; q0 += p.chunk) {
    const int64_t nq = (n_queries - q0 < p.chunk) ? n_queries - q0 : p.chunk;
    const float* qc = queries + q0 * ldq;
    zero_words(w.fail_count, 2 + kFbSlots, st);
    if (int rc = run_prep(qc, ldq, nq, dim, D, index, w, true, st)) return rc;
    if (int rc = run_estimate(D, index, 0, n_cand, nq, p, w, w.tau, st)) return rc;
    if (int rc = run_scan(D, index, 0, n_cand, nq, p, w, w.tau, static_cast<unsigned>(index_offset), st)) return rc;
    Lists ls{w.buf, w.count, w.tau, p.S, p.cap, nullptr, p.S, 1};
    FinalArgs fa{qc, ldq, cand, ldc, n_cand, index_offset, index_offset, dim, k, p.LF, p.P, vec4,
                 nq, w.qflags, w.qmarg, w.qnorm, index_norms(index, n_cand, D), index_header(index), ls,
                 out_scores + q0 * k, out_idx + q0 * k, w.fail_count, w.fail_list,
                 nullptr, nullptr};
    FallbackArgs fb{qc, ldq, cand, ldc, n_cand, index_offset, dim, k, p.L, p.P, p.parts, vec4,
                    w.fail_count, w.fail_list, w.fail_count + 1, w.fb_scratch, w.fb_scratch_n,
                    out_scores + q0 * k, out_idx + q0 * k};
    if (int rc = run_finalize(fa, fb, nq, p, st)) return rc;
  }
  return TT_OK;
}

// ---- candidate-sharded two-phase search (ShardedBruteForceIndex) ----------
// A shard's exact top-k over its own rows, cut by a lower bound on the GLOBAL
// k-th score so each shard rescores only its share of the global candidates:
//   screen   (this shard) prep + estimate + scan + the finalize's select:
//            kth_lb[q] = lb(k-th largest screened score) — at least k rows of
//            the shard, hence of the whole matrix, score >= it exactly;
//   (caller) floor = all_reduce(MAX) of kth_lb over the shards;
//   finalize rescoring of the entries with ub(s~) >= max(own cut, floor):
//            every member of the global top-k on this shard is among them
//            (it is in the shard's top-k and scores >= the global k-th >=
//            floor), so the merged lists hold the global top-k exactly; fewer
//            than k are padded with (-inf, INT32_MAX).
// Queries whose certificate fails are scanned exactly over the shard's rows.
// Queries go in chunks: every call pair of one search plans with the same
// `plan_queries` (the chunk the workspace was sized for, which every rank of
// the search must use alike: tt_bruteforce_shard_chunk is a per-shard
// recommendation, the caller takes the minimum over the shards) and carries
// n_queries <= plan_queries of them; the pair shares the workspace (its lists
// live there between the two calls).
extern "C" int64_t tt_bruteforce_shard_chunk(int64_t n_queries, int64_t n_cand, int32_t dim, int32_t k) {
  if (n_queries < 1 || n_cand < 1 || k < 1 || pick_dpad(dim) == 0) return 0;
  return plan_search(n_queries, n_cand, k, 1).chunk;
}

namespace {
// the plan of every chunk of a shard search: sized for plan_queries queries
SearchPlan shard_plan(int64_t plan_queries, int64_t n_cand, int k) {
  SearchPlan p = plan_search(plan_queries, n_cand, k, 1);
  p.chunk = round_up(plan_queries, kQPerWG);
  return p;
}
}  // namespace

extern "C" size_t tt_bruteforce_shard_workspace_size(int64_t plan_queries, int64_t n_cand, int32_t dim, int32_t k) {
  if (plan_queries < 1 || n_cand < 1 || k < 1 || pick_dpad(dim) == 0) return 0;
  const SearchPlan p = shard_plan(plan_queries, n_cand, k);
  Carver cv(nullptr, 0);
  carve_search(cv, pick_dpad(dim), p, true, true);
  return cv.used();
}

namespace {
int shard_check(const char* fn, const void* index, int64_t n_cand, int32_t dim, int64_t n_queries,
                int64_t plan_queries, int32_t k, void* workspace, size_t workspace_bytes, const SearchPlan& p,
                SearchWs* w) {
  TT_REQUIRE(index, "%s: NULL index", fn);
  TT_REQUIRE(n_cand >= 1 && dim >= 1, "%s: bad shapes", fn);
  if (pick_dpad(dim) == 0) return fail(TT_ERR_UNSUPPORTED, "%s: dim=%d > 128", fn, dim);
  TT_REQUIRE(k >= 1 && k <= n_cand && k <= 4000, "%s: bad k=%d", fn, k);
  TT_REQUIRE(n_queries >= 1 && n_queries <= plan_queries, "%s: n_queries=%lld outside [1, plan_queries %lld]", fn,
             static_cast<long long>(n_queries), static_cast<long long>(plan_queries));
  Carver cv(workspace, workspace_bytes);
  *w = carve_search(cv, pick_dpad(dim), p, true, true);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "%s: workspace %zu < required %zu", fn, workspace_bytes, cv.used());
  return TT_OK;
}
}  // namespace

extern "C" int tt_bruteforce_shard_screen(const void* index, int64_t n_cand, int32_t dim, const float* queries,
                                          int64_t ldq, int64_t n_queries, int64_t plan_queries, int32_t k,
                                          int64_t index_offset, float* kth_lb, void* workspace,
                                          size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(plan_queries >= 1, "tt_bruteforce_shard_screen: plan_queries must be >= 1");
  const SearchPlan p = shard_plan(plan_queries, n_cand, k);
  SearchWs w;
  if (int rc = shard_check("tt_bruteforce_shard_screen", index, n_cand, dim, n_queries, plan_queries, k, workspace,
                           workspace_bytes, p, &w))
    return rc;
  TT_REQUIRE(queries && kth_lb && ldq >= dim, "tt_bruteforce_shard_screen: NULL queries/kth_lb or bad ldq");
  TT_REQUIRE(index_offset >= 0 && index_offset + n_cand < (1ll << 31),
             "tt_bruteforce_shard_screen: index_offset range");
  const int D = pick_dpad(dim);
  hipStream_t st = to_stream(stream);
  if (int rc = run_prep(queries, ldq, n_queries, dim, D, index, w, true, st)) return rc;
  if (int rc = run_estimate(D, index, 0, n_cand, n_queries, p, w, w.tau, st)) return rc;
  // the lists carry the ids the finalize call outputs (index_offset + row)
  if (int rc = run_scan(D, index, 0, n_cand, n_queries, p, w, w.tau, static_cast<unsigned>(index_offset), st))
    return rc;
  Lists ls{w.buf, w.count, w.tau, p.S, p.cap, nullptr, p.S, 1};
  FinalArgs fa{queries, ldq, nullptr, 0, n_cand, index_offset, index_offset, dim, k, p.LF, p.P, 0,
               n_queries, w.qflags, w.qmarg, w.qnorm, index_norms(index, n_cand, D), index_header(index), ls, nullptr,
               nullptr, nullptr, nullptr, kth_lb, nullptr};
  return launch_finalize(fa, n_queries, p, st);
}

extern "C" int tt_bruteforce_shard_finalize(const void* index, const float* cand, int64_t ldc, int64_t n_cand,
                                            int32_t dim, const float* queries, int64_t ldq, int64_t n_queries,
                                            int64_t plan_queries, int32_t k, int64_t index_offset,
                                            const float* floor, float* out_scores, int32_t* out_idx,
                                            void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(plan_queries >= 1, "tt_bruteforce_shard_finalize: plan_queries must be >= 1");
  const SearchPlan p = shard_plan(plan_queries, n_cand, k);
  SearchWs w;
  if (int rc = shard_check("tt_bruteforce_shard_finalize", index, n_cand, dim, n_queries, plan_queries, k,
                           workspace, workspace_bytes, p, &w))
    return rc;
  TT_REQUIRE(cand && ldc >= dim && queries && ldq >= dim && floor && out_scores && out_idx,
             "tt_bruteforce_shard_finalize: NULL argument or bad leading dimension");
  TT_REQUIRE(index_offset >= 0 && index_offset + n_cand < (1ll << 31),
             "tt_bruteforce_shard_finalize: index_offset range");
  hipStream_t st = to_stream(stream);
  const int vec4 = is_vec4(cand, ldc, dim) ? 1 : 0;
  zero_words(w.fail_count, 2 + kFbSlots, st);
  Lists ls{w.buf, w.count, w.tau, p.S, p.cap, nullptr, p.S, 1};
  FinalArgs fa{queries, ldq, cand, ldc, n_cand, index_offset, index_offset, dim, k, p.LF, p.P, vec4,
               n_queries, w.qflags, w.qmarg, w.qnorm, index_norms(index, n_cand, pick_dpad(dim)), index_header(index), ls,
               out_scores, out_idx, w.fail_count, w.fail_list, nullptr, floor};
  FallbackArgs fb{queries, ldq, cand, ldc, n_cand, index_offset, dim, k, p.L, p.P, p.parts, vec4,
                  w.fail_count, w.fail_list, w.fail_count + 1, w.fb_scratch, w.fb_scratch_n, out_scores, out_idx};
  return run_finalize(fa, fb, n_queries, p, st);
}
