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
// Design (MI355X):
//  screen   — one workgroup = 8 waves x 32 queries; the queries' bf16
//             fragments stay in VGPRs (B operand), candidates stream through
//             double-buffered, XOR-swizzled LDS tiles of 64 rows and are scored
//             with v_mfma_f32_32x32x16_bf16 (S^T tile: each lane holds 16
//             candidates of one query).  Per register a single v_cmp against
//             the query's running threshold and a wave-uniform branch filter
//             the tile; survivors are appended to a per-query HBM shortlist.
//             When a shortlist fills, the wave compacts it: the K-th best
//             screened (score, index) key is found by a 64-step bitwise search
//             and everything that provably cannot reach the exact top-K is
//             dropped.  Screened scores err from the exact chain by at most
//             M_q = eps * |q| * max_c |c| (eps = 2^-7 covers bf16 rounding of
//             both operands and fp32 accumulation twice over); the threshold
//             is thr = s_K - 2 M_q and a later candidate survives iff s > thr.
//  finalize — one wave per query: the surviving shortlist is rescored with
//             the exact fp32 fmaf chain (row gathers of the fp32 candidates),
//             the exact top-K selected by the same bitwise search on
//             (score, ~index) keys and ranked.  A query whose shortlist cannot
//             be compacted below capacity (massive near-ties) falls back to an
//             exact fp32 scan with the same machinery and margin 0.
#include <cmath>

#include "tt_common.h"

namespace tt {
namespace {

constexpr int kScreenWaves = 8;
constexpr int kScreenThreads = kScreenWaves * kWave;
constexpr int kQPerWave = 32;
constexpr int kQPerWG = kScreenWaves * kQPerWave;  // 256 queries
constexpr int kCTile = 64;                         // candidates per LDS tile
constexpr float kScreenEps = 0.0078125f;           // 2^-7
constexpr int64_t kQueryChunk = 131072;            // queries per screening pass
constexpr int kFinalWaves = 4;

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
// for padding rows) and max row norm.
__global__ void build_kernel(const float* __restrict__ cand, int64_t ldc, int64_t n, int dim, int64_t n_pad, int D,
                             void* index) {
  IndexHeader* hdr = static_cast<IndexHeader*>(index);
  __bf16* rows = reinterpret_cast<__bf16*>(static_cast<char*>(index) + 64);
  float* bias = reinterpret_cast<float*>(static_cast<char*>(index) + 64 + n_pad * D * 2);
  const int64_t r = blockIdx.x * 4ll + threadIdx.x / kWave;  // one wave per row
  if (r >= n_pad) return;
  const int lane = lane_id();
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
  if (lane == 0) {
    bias[r] = (r < n) ? 0.0f : -INFINITY;
    // round the norm up by a few ulps so the bound stays an upper bound
    const float nr = sqrtf(ss) * (1.0f + 1e-6f);
    atomicMax(&hdr->maxnorm_bits, __float_as_uint(nr));
    if (r == 0) {
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
  for (int e2 = lane; e2 < D / 2; e2 += kWave) {
    const int e = 2 * e2;
    const float x0 = (r < nq && e < dim) ? q[r * ldq + e] : 0.0f;
    const float x1 = (r < nq && e + 1 < dim) ? q[r * ldq + e + 1] : 0.0f;
    ss = __builtin_fmaf(x0, x0, __builtin_fmaf(x1, x1, ss));
    reinterpret_cast<unsigned*>(qb + r * D)[e2] = pack_bf16x2(x0, x1);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, kWave);
  if (lane == 0) {
    const float maxc = __uint_as_float(static_cast<const IndexHeader*>(index)->maxnorm_bits);
    const float qn = sqrtf(ss) * (1.0f + 1e-6f);
    // 2 * eps * |q| * max|c|, rounded up; tiny absolute floor for subnormals.
    margin2[r] = (r < nq) ? (2.0f * kScreenEps * qn * maxc) * (1.0f + 1e-5f) + 1e-30f : 0.0f;
  }
}

__device__ __forceinline__ unsigned long long make_key(float s, unsigned idx) {
  return (static_cast<unsigned long long>(float_order_key(s)) << 32) |
         static_cast<unsigned long long>(0xFFFFFFFFu - idx);
}

// Largest key v such that at least K of the wave's keys are >= v, i.e. the
// K-th largest key (keys are distinct).  Keys of empty slots are 0.
template <int NPL>
__device__ unsigned long long kth_largest(const unsigned long long (&key)[NPL], int K) {
  unsigned long long res = 0;
#pragma unroll 1
  for (int bit = 63; bit >= 0; --bit) {
    const unsigned long long cand = res | (1ull << bit);
    int c = 0;
#pragma unroll
    for (int i = 0; i < NPL; ++i) c += (key[i] >= cand) ? 1 : 0;
    c = wave_sum_i32(c);
    if (c >= K) res = cand;
  }
  return res;
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

// Compacts the shortlist buf[0..n) of one query with the whole wave.
// Keeps every entry that might still belong to the exact top-K given screened
// scores within +-M of the exact ones (margin2 = 2M).  Returns the new count
// and the new strict insert threshold.  n <= 64*NPL.
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
  if (margin2 > 0.0f) thr = next_down(thr);  // round the threshold down
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
  __threadfence_block();  // other lanes of this wave re-read the shortlist
  *thr_out = thr;
  return out;
}

struct ScreenArgs {
  const void* index;
  const __bf16* qb;      // [nq_pad, D]
  const float* margin2;  // [nq_pad]
  int64_t nq;            // real queries in this chunk
  int64_t n_pad;
  int k;
  int cap;
  uint2* buf;            // [nq_pad, cap]
  int* count;            // [nq_pad]
  int* overflow;         // [nq_pad]
};

template <int D, int NPL>
__global__ void __launch_bounds__(kScreenThreads) screen_kernel(const ScreenArgs a) {
  constexpr int KS = D / 16, CH = D / 8;
  constexpr int A_BYTES = kCTile * D * 2;
  constexpr int BUF_BYTES = A_BYTES + kCTile * 4;
  constexpr int CPT = (kCTile * CH + kScreenThreads - 1) / kScreenThreads;  // chunks per thread
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES];
  __shared__ int cnt_s[kQPerWG];
  __shared__ float thr_s[kQPerWG];
  const int tid = threadIdx.x;
  const int wave = tid / kWave;
  const int lane = lane_id();
  const int h = lane >> 5, l32 = lane & 31;
  const int ql = wave * kQPerWave + l32;  // query slot in the WG
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
    thr_s[tid] = (q < a.nq) ? -INFINITY : INFINITY;  // padding queries never insert
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

    // Make room: a tile adds at most kCTile entries per query.
    const bool need = cnt_s[ql] > a.cap - kCTile;
    uint64_t needm = __ballot(need) & 0xFFFFFFFFull;
    if (needm) __threadfence_block();  // inserts of earlier tiles visible to the wave
    while (needm) {
      const int qq = __ffsll(static_cast<long long>(needm)) - 1;
      needm &= needm - 1;
      const float m2 = __shfl(margin2, qq, kWave);
      float nthr;
      const int nc = compact_shortlist<NPL>(mybuf_base + static_cast<int64_t>(qq) * a.cap,
                                            cnt_s[wave * kQPerWave + qq], a.k, m2, &nthr);
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
  if (h == 0) {
    a.count[qg] = cnt_s[ql];
    a.overflow[qg] = ovf ? 1 : 0;
  }
}

// Exact score: k-ordered fmaf chain over the fp32 rows (dim real columns).
__device__ __forceinline__ float exact_score(const float* __restrict__ qs, const float* __restrict__ c, int dim) {
  float acc = 0.0f;
  for (int e = 0; e < dim; ++e) acc = __builtin_fmaf(qs[e], c[e], acc);
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
  int cap;
  int64_t nq;
  int64_t index_offset;
  const float* margin2;
  uint2* buf;
  const int* count;
  const int* overflow;
  float* out_s;
  int32_t* out_i;
};

template <int NPL>
__global__ void __launch_bounds__(kFinalWaves * kWave) finalize_kernel(const FinalArgs a) {
  extern __shared__ __attribute__((aligned(16))) char fsm[];
  const int wave = threadIdx.x / kWave;
  const int lane = lane_id();
  const int64_t q = blockIdx.x * static_cast<int64_t>(kFinalWaves) + wave;
  if (q >= a.nq) return;
  float* qs = reinterpret_cast<float*>(fsm) + wave * 128;  // query row (dim <= 128)
  for (int e = lane; e < a.dim; e += kWave) qs[e] = a.q[q * a.ldq + e];
  __threadfence_block();
  uint2* buf = a.buf + q * a.cap;
  int n = a.count[q];

  if (a.overflow[q]) {
    // Exact fallback: scan every candidate with the fp32 chain, keep an exact
    // shortlist (margin 0: compaction always reduces to exactly K).
    float thr = -INFINITY;
    n = 0;
    for (int64_t c0 = 0; c0 < a.n; c0 += kWave) {
      const int64_t c = c0 + lane;
      float s = -INFINITY;
      if (c < a.n) s = exact_score(qs, a.cand + c * a.ldc, a.dim);
      const bool hit = (c < a.n) && (s + 0.0f > thr);
      const uint64_t m = __ballot(hit);
      if (hit) buf[n + __popcll(m & lanemask_lt64())] = make_uint2(__float_as_uint(s + 0.0f), static_cast<unsigned>(c));
      n += __popcll(m);
      if (n > a.cap - kWave) {
        __threadfence_block();
        n = compact_shortlist<NPL>(buf, n, a.k, 0.0f, &thr);
      }
    }
  } else {
    // Drop what the final screened threshold rules out, then rescore exactly.
    float thr;
    n = compact_shortlist<NPL>(buf, n, a.k, a.margin2[q], &thr);
    for (int j = lane; j < n; j += kWave) {
      const uint2 e = buf[j];
      const float s = exact_score(qs, a.cand + static_cast<int64_t>(e.y) * a.ldc, a.dim);
      buf[j] = make_uint2(__float_as_uint(s + 0.0f), e.y);
    }
    __threadfence_block();
  }
  // Exact selection of the top-K (distinct keys -> exactly K remain).
  __threadfence_block();
  float thr0;
  n = compact_shortlist<NPL>(buf, n, a.k, 0.0f, &thr0);
  // Rank the K survivors: rank = #keys greater than own key.
  for (int j = lane; j < n; j += kWave) {
    const uint2 e = buf[j];
    const unsigned long long mine = make_key(__uint_as_float(e.x), e.y);
    int rank = 0;
    for (int i = 0; i < n; ++i) {
      const uint2 o = buf[i];
      rank += (make_key(__uint_as_float(o.x), o.y) > mine) ? 1 : 0;
    }
    if (rank < a.k) {
      a.out_s[q * a.k + rank] = __uint_as_float(e.x);
      a.out_i[q * a.k + rank] = static_cast<int32_t>(static_cast<int64_t>(e.y) + a.index_offset);
    }
  }
}

template <int D, int NPL>
int launch_screen(const ScreenArgs& sa, int64_t nq_pad, hipStream_t st) {
  hipLaunchKernelGGL((screen_kernel<D, NPL>), dim3(nq_pad / kQPerWG), dim3(kScreenThreads), 0, st, sa);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

template <int NPL>
int launch_screen_d(int D, const ScreenArgs& sa, int64_t nq_pad, hipStream_t st) {
  switch (D) {
    case 32: return launch_screen<32, NPL>(sa, nq_pad, st);
    case 64: return launch_screen<64, NPL>(sa, nq_pad, st);
    default: return launch_screen<128, NPL>(sa, nq_pad, st);
  }
}

template <int NPL>
int launch_final(const FinalArgs& fa, hipStream_t st) {
  const size_t shm = kFinalWaves * 128 * sizeof(float);
  hipLaunchKernelGGL(finalize_kernel<NPL>, dim3(ceil_div(fa.nq, kFinalWaves)), dim3(kFinalWaves * kWave), shm, st,
                     fa);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

struct SearchWs {
  __bf16* qb;
  float* margin2;
  uint2* buf;
  int* count;
  int* overflow;
};

SearchWs carve_search(Carver& cv, int64_t nq, int D, int cap) {
  const int64_t chunk = nq < kQueryChunk ? nq : kQueryChunk;
  const int64_t nq_pad = round_up(chunk > 0 ? chunk : 1, kQPerWG);
  SearchWs w;
  w.qb = cv.take<__bf16>(nq_pad * D);
  w.margin2 = cv.take<float>(nq_pad);
  w.buf = cv.take<uint2>(nq_pad * cap);
  w.count = cv.take<int>(nq_pad);
  w.overflow = cv.take<int>(nq_pad);
  return w;
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
  hipLaunchKernelGGL(build_kernel, dim3(ceil_div(n_pad, 4)), dim3(256), 0, st, cand, ldc, n_cand, dim, n_pad, D,
                     index);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" size_t tt_bruteforce_workspace_size(int64_t n_queries, int64_t n_cand, int32_t dim, int32_t k) {
  (void)n_cand;
  if (n_queries < 1 || k < 1 || pick_dpad(dim) == 0) return 0;
  Carver cv(nullptr, 0);
  carve_search(cv, n_queries, pick_dpad(dim), cap_for_k(k));
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
  TT_REQUIRE(k <= 4096, "tt_bruteforce_search: k=%d > 4096", k);
  TT_REQUIRE(n_queries >= 0, "tt_bruteforce_search: negative n_queries");
  TT_REQUIRE(index_offset >= 0 && index_offset + n_cand < (1ll << 31), "tt_bruteforce_search: index_offset range");
  if (n_queries == 0) return TT_OK;
  TT_REQUIRE(queries && out_scores && out_idx, "tt_bruteforce_search: NULL queries/outputs");
  const int D = pick_dpad(dim);
  const int cap = cap_for_k(k);
  Carver cv(workspace, workspace_bytes);
  SearchWs w = carve_search(cv, n_queries, D, cap);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_bruteforce_search: workspace %zu < required %zu", workspace_bytes, cv.used());
  hipStream_t st = to_stream(stream);
  const int64_t n_pad = round_up(n_cand, kCTile);
  for (int64_t q0 = 0; q0 < n_queries; q0 += kQueryChunk) {
    const int64_t nq = (n_queries - q0 < kQueryChunk) ? n_queries - q0 : kQueryChunk;
    const int64_t nq_pad = round_up(nq, kQPerWG);
    hipLaunchKernelGGL(query_prep_kernel, dim3(ceil_div(nq_pad, 4)), dim3(256), 0, st, queries + q0 * ldq, ldq, nq,
                       dim, nq_pad, D, index, w.qb, w.margin2);
    TT_CHECK_LAUNCH();
    ScreenArgs sa{index, w.qb, w.margin2, nq, n_pad, k, cap, w.buf, w.count, w.overflow};
    FinalArgs fa{queries + q0 * ldq, ldq, cand, ldc, n_cand, dim, k, cap, nq, index_offset, w.margin2,
                 w.buf, w.count, w.overflow, out_scores + q0 * k, out_idx + q0 * k};
    int rc;
    switch (cap / kWave) {
      case 16: rc = launch_screen_d<16>(D, sa, nq_pad, st); if (!rc) rc = launch_final<16>(fa, st); break;
      case 32: rc = launch_screen_d<32>(D, sa, nq_pad, st); if (!rc) rc = launch_final<32>(fa, st); break;
      case 64: rc = launch_screen_d<64>(D, sa, nq_pad, st); if (!rc) rc = launch_final<64>(fa, st); break;
      case 128: rc = launch_screen_d<128>(D, sa, nq_pad, st); if (!rc) rc = launch_final<128>(fa, st); break;
      default: return fail(TT_ERR_UNSUPPORTED, "tt_bruteforce_search: shortlist capacity %d", cap);
    }
    if (rc) return rc;
  }
  return TT_OK;
}
