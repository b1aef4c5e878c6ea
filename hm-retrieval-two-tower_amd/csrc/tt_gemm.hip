// K4: the tower MLP GEMMs (Dense layers, /root/reference/pkg/modelling/models/
// tower.py:41-49: relu(x W + b) per layer; their gradients dW = x^T G,
// db = colsum(G), dx = G W^T with G = relu'(y) * dy, the TF MatMul /
// BiasAddGrad / ReluGrad trio of the tape).
//
//   C[i][j] (+= over split z) = sum_r opA(i, r) * opB(r, j)
//
// fp32 operands in HBM, staged through LDS as bf16 and multiplied on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation.  Two precisions:
//   bf16    one MFMA per step on bf16(a) * bf16(b);
//   bf16x3  a = a_hi + a_lo, b = b_hi + b_lo (hi = bf16(x), lo = bf16(x - hi));
//           a_hi b_hi + a_hi b_lo + a_lo b_hi, i.e. every product to ~2^-17
//           relative — fp32-faithful at 3 MFMAs, still ~5x the fp32 MFMA rate.
// Operand options, fused into the tile loads so the backward needs no
// separate ReluGrad / BiasAddGrad passes:
//   * A row-major (A[i*lda + r]) or column-major (A[r*lda + i]);
//     B row-major (B[r*ldb + j]) or column-major (B[j*ldb + r]);
//   * a relu mask on A or on B: v -> (mask > 0) ? s * v : 0 (mask = the
//     layer's relu output in the operand's layout, s = *scale);
//   * a row of ones in A (row `ones_row`): with A = x^T that row of C is
//     colsum(G) = db, which the flat parameter layout stores right after dW;
//   * epilogue: + bias[j], relu;
//   * split-K over blockIdx.z into C + z * slice (reduced by tt_sum_slices in
//     slice order, so the result is deterministic).
// Tiles: 256 threads = 4 waves, each a 64x64 sub-tile (2x2 MFMA blocks);
// BM x BN = 64 x 256 (N > 128) or 128 x 128.  32-deep k stages, double
// buffered; the next stage's global loads are in flight during this stage's
// MFMAs.  LDS holds each stage in MFMA fragment order (one 16-B slot per lane
// per 32x16 block), so every fragment read is a lane-linear ds_read_b128.
#include <algorithm>

#include "tt_common.h"

namespace tt {
namespace {

constexpr int kBK = 32;
constexpr int kGemmThreads = 256;

struct GemmArgs {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  const float* mask;  // relu mask of the masked operand (same layout), or NULL
  int64_t ldm;
  const float* scale; // device scalar applied with the mask (NULL -> 1)
  const float* bias;  // [N] (NULL -> none)
  float* C;
  int64_t ldc;
  int64_t slice;      // split z writes C + z * slice
  int64_t M, N, K;
  int64_t a_rows;     // rows of A that hold data (the ones row, if any, is a_rows)
  int ones_row;       // -1: none
  int relu;
  int64_t k_per_split;  // multiple of kBK
  int vec_a, vec_b, vec_m;
};

// Element slot of (row x, depth k) inside one stage plane in fragment order:
// block (x / 32, k / 16), lane (x % 32) + 32 * ((k % 16) / 8), element k % 8.
__device__ __forceinline__ int frag_slot(int x, int k) {
  return ((((x >> 5) * 2 + (k >> 4)) * 64 + (x & 31) + 32 * ((k >> 3) & 1)) << 3) + (k & 7);
}

__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = static_cast<__bf16>(v);
  lo = static_cast<__bf16>(v - static_cast<float>(hi));
}

// Loads 4 consecutive elements along an operand's contiguous dimension:
// p = base + other * ld + c; elements c..c+3 valid below `lim`, the whole
// vector invalid when !ok.  vec: 16-B loads allowed (ld % 4 == 0, aligned).
__device__ __forceinline__ f32x4 load4(const float* base, int64_t other, int64_t ld, int64_t c, int64_t lim,
                                       bool ok, bool vec) {
  f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
  if (!ok || c >= lim) return v;
  const float* p = base + other * ld + c;
  if (vec) {
    v = *reinterpret_cast<const f32x4*>(p);
    if (c + 4 > lim) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c + e >= lim) v[e] = 0.0f;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (c + e < lim) ? p[e] : 0.0f;
  }
  return v;
}

__device__ __forceinline__ f32x4 apply_mask(f32x4 v, f32x4 m, float s) {
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = m[e] > 0.0f ? v[e] * s : 0.0f;
  return v;
}

template <int BM, bool ACOL, bool BCOL, int MASK, bool X3>
__global__ void __launch_bounds__(kGemmThreads) gemm_kernel(const GemmArgs a) {
  constexpr int BN = 16384 / BM;
  constexpr int WN = BN / 64;                 // waves along N
  constexpr int A_VEC = BM * kBK / 4 / kGemmThreads;  // float4 per thread per stage
  constexpr int B_VEC = BN * kBK / 4 / kGemmThreads;
  constexpr int A_ELEMS = BM * kBK, B_ELEMS = BN * kBK;
  constexpr int PLANES = X3 ? 2 : 1;
  constexpr int STAGE = (A_ELEMS + B_ELEMS) * PLANES;  // bf16 elements per stage
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = lane_id();
  const int wm = wave / WN, wn = wave % WN;
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * BM;
  const int64_t n0 = static_cast<int64_t>(blockIdx.y) * BN;
  const int64_t kb = static_cast<int64_t>(blockIdx.z) * a.k_per_split;
  const int64_t ke = min(a.K, kb + a.k_per_split);
  const int nk = ke > kb ? static_cast<int>((ke - kb + kBK - 1) / kBK) : 0;
  const float s = a.scale ? *a.scale : 1.0f;
  const bool wave_live = (m0 + wm * 64 < a.M) && (n0 + wn * 64 < a.N);

  f32x4 ra[A_VEC], rb[B_VEC];

  // A stage = BM rows x kBK depths, B stage = BN columns x kBK depths, both
  // cut into "quads" (one row / column, 4 consecutive depths) = one 8-byte
  // LDS write per plane.  Thread -> quad mapping follows the operand's
  // contiguous dimension so global loads coalesce: depth-contiguous operands
  // (A row-major, B column-major) take one 16-B load per quad with lanes
  // walking depth first; row-contiguous ones (A column-major, B row-major)
  // take 4 scalar loads per quad with lanes walking rows first (each load
  // instruction reads 64 consecutive floats).
  auto quad_a = [&](int q, int& x, int& r) {
    if (!ACOL) { x = q / (kBK / 4); r = (q % (kBK / 4)) * 4; }
    else       { x = q % BM;        r = (q / BM) * 4; }
  };
  auto quad_b = [&](int q, int& x, int& r) {
    if (BCOL) { x = q / (kBK / 4); r = (q % (kBK / 4)) * 4; }
    else      { x = q % BN;        r = (q / BN) * 4; }
  };
  // 4 depths k0+r .. k0+r+3 of row x of a row-contiguous operand (element
  // (x, k) at base[k * ld + x]); x valid below xlim.
  auto load_cols = [&](const float* base, int64_t ld, int64_t x, int64_t xlim, int64_t k) {
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
    if (x < xlim) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k + e < ke) v[e] = base[(k + e) * ld + x];
    }
    return v;
  };

  // Interior stages (every row, column and depth of the tile in range) take
  // a fast path: per-thread 32-bit element offsets fixed for the whole loop
  // against a wave-uniform stage base pointer, no predicates.
  int offA[A_VEC], offAm[A_VEC], offB[B_VEC], offBm[B_VEC];
#pragma unroll
  for (int u = 0; u < A_VEC; ++u) {
    int x, r;
    quad_a(tid + u * kGemmThreads, x, r);
    offA[u] = ACOL ? r * static_cast<int>(a.lda) + x : x * static_cast<int>(a.lda) + r;
    offAm[u] = ACOL ? r * static_cast<int>(a.ldm) + x : x * static_cast<int>(a.ldm) + r;
  }
#pragma unroll
  for (int u = 0; u < B_VEC; ++u) {
    int x, r;
    quad_b(tid + u * kGemmThreads, x, r);
    offB[u] = BCOL ? x * static_cast<int>(a.ldb) + r : r * static_cast<int>(a.ldb) + x;
    offBm[u] = BCOL ? x * static_cast<int>(a.ldm) + r : r * static_cast<int>(a.ldm) + x;
  }
  const bool rows_in = (m0 + BM <= a.a_rows) && (n0 + BN <= a.N) && a.ones_row < 0 && a.vec_a && a.vec_b &&
                       (MASK == 0 || a.vec_m) && BM * a.lda < (1ll << 31) && BN * a.ldb < (1ll << 31) &&
                       (MASK == 0 || (MASK == 1 ? BM : BN) * a.ldm < (1ll << 31)) &&
                       kBK * (a.lda + a.ldb + a.ldm) < (1ll << 31);

  // fast path: stage at depth k0 fully inside [kb, ke)
  auto fetch_fast = [&](int64_t k0) {
    const float* Ab = a.A + (ACOL ? k0 * a.lda + m0 : m0 * a.lda + k0);
    const float* Bb = a.B + (BCOL ? n0 * a.ldb + k0 : k0 * a.ldb + n0);
    const float* Mb = MASK == 1 ? a.mask + (ACOL ? k0 * a.ldm + m0 : m0 * a.ldm + k0)
                                : a.mask + (BCOL ? n0 * a.ldm + k0 : k0 * a.ldm + n0);
#pragma unroll
    for (int u = 0; u < A_VEC; ++u) {
      if (!ACOL) {
        ra[u] = *reinterpret_cast<const f32x4*>(Ab + offA[u]);
        if (MASK == 1) ra[u] = apply_mask(ra[u], *reinterpret_cast<const f32x4*>(Mb + offAm[u]), s);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) ra[u][e] = Ab[offA[u] + e * a.lda];
        if (MASK == 1) {
          f32x4 m;
#pragma unroll
          for (int e = 0; e < 4; ++e) m[e] = Mb[offAm[u] + e * a.ldm];
          ra[u] = apply_mask(ra[u], m, s);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < B_VEC; ++u) {
      if (BCOL) {
        rb[u] = *reinterpret_cast<const f32x4*>(Bb + offB[u]);
        if (MASK == 2) rb[u] = apply_mask(rb[u], *reinterpret_cast<const f32x4*>(Mb + offBm[u]), s);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) rb[u][e] = Bb[offB[u] + e * a.ldb];
        if (MASK == 2) {
          f32x4 m;
#pragma unroll
          for (int e = 0; e < 4; ++e) m[e] = Mb[offBm[u] + e * a.ldm];
          rb[u] = apply_mask(rb[u], m, s);
        }
      }
    }
  };

  // general path: every element predicated (tile edges, ones row, unaligned)
  auto fetch_slow = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < A_VEC; ++u) {
      int x, r;
      quad_a(tid + u * kGemmThreads, x, r);
      const int64_t gi = m0 + x, gk = k0 + r;
      if (!ACOL) {
        ra[u] = load4(a.A, gi, a.lda, gk, ke, gi < a.a_rows, a.vec_a);
        if (MASK == 1) ra[u] = apply_mask(ra[u], load4(a.mask, gi, a.ldm, gk, ke, gi < a.a_rows, a.vec_m), s);
      } else {
        ra[u] = load_cols(a.A, a.lda, gi, a.a_rows, gk);
        if (MASK == 1) ra[u] = apply_mask(ra[u], load_cols(a.mask, a.ldm, gi, a.a_rows, gk), s);
      }
      if (gi == a.ones_row) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ra[u][e] = (gk + e < ke) ? 1.0f : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < B_VEC; ++u) {
      int x, r;
      quad_b(tid + u * kGemmThreads, x, r);
      const int64_t gj = n0 + x, gk = k0 + r;
      if (BCOL) {
        rb[u] = load4(a.B, gj, a.ldb, gk, ke, gj < a.N, a.vec_b);
        if (MASK == 2) rb[u] = apply_mask(rb[u], load4(a.mask, gj, a.ldm, gk, ke, gj < a.N, a.vec_m), s);
      } else {
        rb[u] = load_cols(a.B, a.ldb, gj, a.N, gk);
        if (MASK == 2) rb[u] = apply_mask(rb[u], load_cols(a.mask, a.ldm, gj, a.N, gk), s);
      }
    }
  };

  auto put_quad = [&](__bf16* hi, __bf16* lo, int x, int r, const f32x4& v) {
    __bf16 h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) split_bf16(v[e], h[e], l[e]);
    const int slot = frag_slot(x, r);  // 4 consecutive elements of one lane slot
    *reinterpret_cast<uint2*>(hi + slot) = make_uint2(__builtin_bit_cast(unsigned, bf16x2{h[0], h[1]}),
                                                      __builtin_bit_cast(unsigned, bf16x2{h[2], h[3]}));
    if (X3)
      *reinterpret_cast<uint2*>(lo + slot) = make_uint2(__builtin_bit_cast(unsigned, bf16x2{l[0], l[1]}),
                                                        __builtin_bit_cast(unsigned, bf16x2{l[2], l[3]}));
  };

  // registers -> LDS stage (bf16 hi [, lo] planes in fragment order)
  auto stash = [&](int buf) {
    __bf16* Ah = smem + buf * STAGE;
    __bf16* Al = Ah + A_ELEMS;
    __bf16* Bh = Ah + A_ELEMS * PLANES;
    __bf16* Bl = Bh + B_ELEMS;
#pragma unroll
    for (int u = 0; u < A_VEC; ++u) {
      int x, r;
      quad_a(tid + u * kGemmThreads, x, r);
      put_quad(Ah, Al, x, r, ra[u]);
    }
#pragma unroll
    for (int u = 0; u < B_VEC; ++u) {
      int x, r;
      quad_b(tid + u * kGemmThreads, x, r);
      put_quad(Bh, Bl, x, r, rb[u]);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = f32x16{};

  auto compute = [&](int buf) {
    const __bf16* Ah = smem + buf * STAGE;
    const __bf16* Al = Ah + A_ELEMS;
    const __bf16* Bh = Ah + A_ELEMS * PLANES;
    const __bf16* Bl = Bh + B_ELEMS;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int fa = ((((wm * 2 + x) * 2 + ks) * 64) + lane) * 8;
        const int fb = ((((wn * 2 + x) * 2 + ks) * 64) + lane) * 8;
        ah[x] = *reinterpret_cast<const bf16x8*>(Ah + fa);
        bh[x] = *reinterpret_cast<const bf16x8*>(Bh + fb);
        if (X3) {
          al[x] = *reinterpret_cast<const bf16x8*>(Al + fa);
          bl[x] = *reinterpret_cast<const bf16x8*>(Bl + fb);
        }
      }
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
          if (X3) {
            acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[bi], bh[bj], acc[bi][bj], 0, 0, 0);
            acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[bi], bl[bj], acc[bi][bj], 0, 0, 0);
          }
          acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[bi], bh[bj], acc[bi][bj], 0, 0, 0);
        }
    }
  };

  if (nk > 0) {
    auto fetch = [&](int64_t k0) {
      if (rows_in && k0 + kBK <= ke) fetch_fast(k0);
      else fetch_slow(k0);
    };
    fetch(kb);
    stash(0);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      const bool more = t + 1 < nk;
      if (more) fetch(kb + static_cast<int64_t>(t + 1) * kBK);
      if (wave_live) compute(t & 1);
      if (more) stash((t + 1) & 1);
      __syncthreads();
    }
  }

  // epilogue: acc[bi][bj][v] is C[i][j] with
  // i = 64 wm + 32 bi + (v & 3) + 8 (v >> 2) + 4 (lane >> 5), j = 64 wn + 32 bj + lane % 32
  if (!wave_live) return;
  // bias + relu in registers first; stores then depend on no outstanding load
#pragma unroll
  for (int bj = 0; bj < 2; ++bj) {
    const int64_t j = n0 + wn * 64 + bj * 32 + (lane & 31);
    const float bv = (a.bias && j < a.N) ? a.bias[j] : 0.0f;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const float x = acc[bi][bj][v] + bv;
        acc[bi][bj][v] = a.relu ? fmaxf(x, 0.0f) : x;
      }
  }
  float* C = a.C + static_cast<int64_t>(blockIdx.z) * a.slice + (m0 + wm * 64 + 4 * (lane >> 5)) * a.ldc + n0 +
             wn * 64 + (lane & 31);
  if (m0 + wm * 64 + 64 <= a.M && n0 + wn * 64 + 64 <= a.N && 64 * a.ldc < (1ll << 31)) {
    const int ldc = static_cast<int>(a.ldc);
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int v = 0; v < 16; ++v) C[(bi * 32 + (v & 3) + 8 * (v >> 2)) * ldc + bj * 32] = acc[bi][bj][v];
  } else {
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) {
      const bool jok = n0 + wn * 64 + bj * 32 + (lane & 31) < a.N;
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = bi * 32 + (v & 3) + 8 * (v >> 2);
          if (jok && m0 + wm * 64 + r + 4 * (lane >> 5) < a.M) C[r * a.ldc + bj * 32] = acc[bi][bj][v];
        }
    }
  }
}

// ---- weight-stationary form (y = x W, dx = G W^T) ---------------------------
// The weight operand is small (<= 288 x 272 bf16 = 153 KiB): it is packed
// once per call into a bf16 MFMA B-fragment image (pack_weight_kernel), every
// workgroup copies the whole image into LDS, and every wave then streams
// 32-row panels of the tall operand straight from HBM into A-fragment
// registers (two 16-B loads per lane per 16-deep step, prefetched a chunk of
// 4 steps ahead) and produces the panel's full output width, so the tall
// operand is read exactly once and never touches LDS.
constexpr int kWsWaves = 4;
constexpr size_t kWsLdsMax = 160 * 1024;

struct WsArgs {
  const float* A;     // tall operand [M, K] row-major
  int64_t lda;
  const float* mask;  // optional relu mask of A (same shape), ldm
  int64_t ldm;
  const float* scale;
  const __bf16* img;  // packed weight image (pack_weight_kernel)
  const float* bias;
  float* C;
  int64_t ldc;
  int64_t M;
  int N, K, Kp;       // Kp = K rounded up to 16
  int relu;
  int vec;            // A (and mask) rows 16-B loadable
  int probe;          // timing probes only (tools/): bit0 skip weight copy, bit1 skip MFMAs, bit2 skip stores
};

// Weight image: opB(k, j) for k < Kp, j < 32*NB as bf16 in MFMA B-fragment
// order ([Kp/16][NB][64 lanes][8]); zero outside K x N.  One thread per
// 4-depth quad; lanes walk the weight's contiguous dimension.
template <bool BCOL>
__global__ void __launch_bounds__(256) pack_weight_kernel(const float* __restrict__ W, int64_t ldw, int K, int N,
                                                           int Kp, int NB, __bf16* __restrict__ img) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  const int nq = (Kp / 4) * (NB * 32);
  if (q >= nq) return;
  int j, k;
  if (!BCOL) { j = q % (NB * 32); k = (q / (NB * 32)) * 4; }
  else       { k = (q % (Kp / 4)) * 4; j = q / (Kp / 4); }
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bool ok = j < N && k + e < K;
    v[e] = ok ? (BCOL ? W[static_cast<int64_t>(j) * ldw + k + e] : W[static_cast<int64_t>(k + e) * ldw + j]) : 0.0f;
  }
  const int slot = ((((k >> 4) * NB + (j >> 5)) * 64 + (j & 31) + 32 * ((k >> 3) & 1)) << 3) + (k & 7);
  *reinterpret_cast<uint2*>(img + slot) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}

// Tall-operand staging: a wave's 32-row panel moves in 32-deep chunks.  A
// chunk is read row-contiguously (load instruction i: lane l reads 16 B at
// row 8i + l/8, depth 4(l%8): 8 rows x 128 B per instruction, the pattern
// that streams at the CU's full load rate; loading straight into MFMA
// fragments would put 32 rows in every instruction), converted to bf16 with
// the relu mask applied, written to the wave's own LDS chunk buffer in
// fragment order, and read back as A fragments.  Up to P chunks are in flight
// (a register ring indexed at compile time under full unrolling).
constexpr int kWsMaxChunks = 9;  // K <= 288
constexpr int kWsChunkElems = 32 * 32;  // bf16 per wave chunk buffer

template <int NB, bool MASKA>
__global__ void __launch_bounds__(256) gemm_wstat_kernel(const WsArgs a) {
  constexpr int P = MASKA ? 4 : (NB >= 9 ? 6 : kWsMaxChunks);  // chunks in flight
  extern __shared__ __attribute__((aligned(16))) __bf16 wlds[];  // [Kp/16][NB][64 lanes][8] + chunk buffers
  const int tid = threadIdx.x, wave = tid / kWave, lane = lane_id();
  const int nw = blockDim.x / kWave, nthreads = blockDim.x;
  const float s = a.scale ? *a.scale : 1.0f;
  const int nks = a.Kp / 16;
  const int nchunks = (a.K + 31) / 32;
  const int64_t panels = (a.M + 31) / 32;
  __bf16* abuf = wlds + static_cast<size_t>(a.Kp) * NB * 32 + wave * 2 * kWsChunkElems;
  const int lr = lane >> 3, lk = 4 * (lane & 7);  // row within 8, depth within the chunk

  f32x4 ring[P][4], mring[MASKA ? P : 1][4];
  auto issue = [&](int64_t p, int c, f32x4 (&dst)[4], f32x4 (&mdst)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = p * 32 + 8 * i + lr;
      const int k = 32 * c + lk;
      f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f}, m = {1.0f, 1.0f, 1.0f, 1.0f};
      if (row < a.M && k < a.K) {
        const float* ap = a.A + row * a.lda + k;
        const float* mp = MASKA ? a.mask + row * a.ldm + k : nullptr;
        if (a.vec && k + 4 <= a.lda && (!MASKA || k + 4 <= a.ldm)) {
          v = *reinterpret_cast<const f32x4*>(ap);
          if (MASKA) m = *reinterpret_cast<const f32x4*>(mp);
          if (k + 4 > a.K) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (k + e >= a.K) v[e] = 0.0f;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (k + e < a.K) {
              v[e] = ap[e];
              if (MASKA) m[e] = mp[e];
            }
        }
      }
      dst[i] = v;
      if (MASKA) mdst[i] = m;
    }
  };

  int64_t p = static_cast<int64_t>(blockIdx.x) * nw + wave;
  if (p < panels) {  // first chunks in flight while the weight is staged
#pragma unroll
    for (int c = 0; c < P; ++c)
      if (c < nchunks) issue(p, c, ring[c], mring[MASKA ? c : 0]);
  }

  // copy the packed weight image into LDS: 16-B pieces, 8 in flight per
  // thread, start rotated per workgroup so the workgroups do not all hit the
  // same L2 lines at once
  {
    const int npieces = a.Kp * NB * 32 / 8;
    const int rot = (static_cast<int>(blockIdx.x) * 1024) % npieces;
    const u32x4* src = reinterpret_cast<const u32x4*>(a.img);
    u32x4* dst = reinterpret_cast<u32x4*>(wlds);
    for (int i0 = (a.probe & 1) ? npieces : tid; i0 < npieces; i0 += nthreads * 8) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        int i = i0 + u * nthreads;
        i = i < npieces ? (i + rot) % npieces : -1;
        if (i >= 0) v[u] = src[i];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * nthreads;
        if (i < npieces) dst[(i + rot) % npieces] = v[u];
      }
    }
  }
  __syncthreads();

  for (; p < panels; p += static_cast<int64_t>(gridDim.x) * nw) {
    const int64_t pnext = p + static_cast<int64_t>(gridDim.x) * nw;
    f32x16 acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = f32x16{};
#pragma unroll
    for (int c = 0; c < kWsMaxChunks; ++c) {
      if (c < nchunks) {
        __bf16* buf = abuf + (c & 1) * kWsChunkElems;
        // chunk c -> bf16 fragments in this wave's buffer: element (row r,
        // depth k) at lane slot (r + 32 * ((k / 8) % 2)) of step k / 16
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f32x4 v = ring[c % P][i];
          if (MASKA) v = apply_mask(v, mring[c % P][i], s);
          const int r = 8 * i + lr;
          const int slot = ((((lk >> 4) * 64) + r + 32 * ((lk >> 3) & 1)) << 3) + (lk & 7);
          *reinterpret_cast<uint2*>(buf + slot) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        }
        if (c + P < nchunks) issue(p, c + P, ring[c % P], mring[MASKA ? c % P : 0]);
        else if (c + P - nchunks < P && pnext < panels)  // next panel's first chunks
          issue(pnext, c + P - nchunks, ring[c % P], mring[MASKA ? c % P : 0]);
        if (a.probe & 2) continue;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int ks = 2 * c + t;
          if (ks >= nks) break;
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(buf + ((t * 64 + lane) << 3));
          bf16x8 bf[NB];  // all of the step's B fragments in flight before the MFMAs
#pragma unroll
          for (int b = 0; b < NB; ++b)
            bf[b] = *reinterpret_cast<const bf16x8*>(wlds + (((ks * NB + b) * 64 + lane) << 3));
#pragma unroll
          for (int b = 0; b < NB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf[b], acc[b], 0, 0, 0);
        }
      }
    }
    // bias + relu applied in registers first, so the stores below depend on
    // no outstanding load (a predicated store after a load makes the waitcnt
    // pass serialise every store behind vmcnt(0))
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int j = b * 32 + (lane & 31);
      const float bv = (a.bias && j < a.N) ? a.bias[j] : 0.0f;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const float x = acc[b][v] + bv;
        acc[b][v] = a.relu ? fmaxf(x, 0.0f) : x;
      }
    }
    if (a.probe & 4) {  // keep the accumulators live without storing them
      float t = 0.0f;
#pragma unroll
      for (int b = 0; b < NB; ++b) t += acc[b][0] + acc[b][15];
      if (t == 12345.678f) a.C[0] = t;
      continue;
    }
    float* cp = a.C + (p * 32 + 4 * (lane >> 5)) * a.ldc + (lane & 31);
    const int ldc = static_cast<int>(a.ldc);  // 32 rows x ldc fit in 32 bits (checked on the host)
    if (p * 32 + 32 <= a.M && NB * 32 <= a.N) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int v = 0; v < 16; ++v) cp[((v & 3) + 8 * (v >> 2)) * ldc + b * 32] = acc[b][v];
    } else {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const bool jok = b * 32 + (lane & 31) < a.N;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int r = (v & 3) + 8 * (v >> 2);
          if (jok && p * 32 + r + 4 * (lane >> 5) < a.M) cp[r * ldc + b * 32] = acc[b][v];
        }
      }
    }
  }
}

template <int NB, bool MASKA>
int launch_wstat_nb(const WsArgs& w, hipStream_t st) {
  const int64_t panels = (w.M + 31) / 32;
  // one workgroup per CU (the weight image fills LDS): 2 waves per workgroup
  // once there are >= 512 panels so all 256 CUs stream, else 4
  const int nw = (w.probe >> 8) ? (w.probe >> 8) : (panels >= 512 ? 2 : kWsWaves);
  const size_t lds = static_cast<size_t>(w.Kp) * NB * 32 * sizeof(__bf16) +
                     static_cast<size_t>(nw) * 2 * kWsChunkElems * sizeof(__bf16);
  const int64_t grid = std::min<int64_t>(ceil_div(panels, nw), 256);
  static bool attr_set = false;  // allow > 64 KiB of dynamic LDS (once per instantiation)
  if (!attr_set) {
    TT_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_wstat_kernel<NB, MASKA>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kWsLdsMax)));
    attr_set = true;
  }
  if (lds > kWsLdsMax) return fail(TT_ERR_UNSUPPORTED, "tt_gemm: weight image + chunk buffers exceed LDS");
  hipLaunchKernelGGL((gemm_wstat_kernel<NB, MASKA>), dim3(static_cast<unsigned>(grid)), dim3(nw * kWave), lds,
                     st, w);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

template <bool MASKA>
int launch_wstat(const WsArgs& w, int nb, hipStream_t st) {
  switch (nb) {
    case 1: return launch_wstat_nb<1, MASKA>(w, st);
    case 2: return launch_wstat_nb<2, MASKA>(w, st);
    case 3: return launch_wstat_nb<3, MASKA>(w, st);
    case 4: return launch_wstat_nb<4, MASKA>(w, st);
    case 5: return launch_wstat_nb<5, MASKA>(w, st);
    case 6: return launch_wstat_nb<6, MASKA>(w, st);
    case 7: return launch_wstat_nb<7, MASKA>(w, st);
    case 8: return launch_wstat_nb<8, MASKA>(w, st);
    case 9: return launch_wstat_nb<9, MASKA>(w, st);
    default: return fail(TT_ERR_UNSUPPORTED, "tt_gemm: weight-stationary form needs N <= 288");
  }
}

template <int BM, bool ACOL, bool BCOL, int MASK>
int launch_gemm(const GemmArgs& g, int splits, bool x3, hipStream_t st) {
  constexpr int BN = 16384 / BM;
  const dim3 grid(static_cast<unsigned>(ceil_div(g.M, BM)), static_cast<unsigned>(ceil_div(g.N, BN)),
                  static_cast<unsigned>(splits));
  if (x3)
    hipLaunchKernelGGL((gemm_kernel<BM, ACOL, BCOL, MASK, true>), grid, dim3(kGemmThreads), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, ACOL, BCOL, MASK, false>), grid, dim3(kGemmThreads), 0, st, g);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

template <bool ACOL, bool BCOL, int MASK>
int dispatch_bm(const GemmArgs& g, int splits, bool x3, hipStream_t st) {
  if (g.N > 128) return launch_gemm<64, ACOL, BCOL, MASK>(g, splits, x3, st);
  return launch_gemm<128, ACOL, BCOL, MASK>(g, splits, x3, st);
}

int g_gemm_probe = 0;  // tt_gemm_set_probe (timing tools only)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace
}  // namespace tt

using namespace tt;

// Not in tt.h: timing-probe switch for tools/gemm_probe.py (never set by the package).
extern "C" void tt_gemm_set_probe(int bits) { g_gemm_probe = bits; }

extern "C" size_t tt_gemm_workspace_size(int64_t N, int64_t K) {
  if (N <= 0 || K < 0) return 0;
  return static_cast<size_t>(round_up(K > 0 ? K : 1, 16)) * round_up(N, 32) * sizeof(uint16_t);
}

extern "C" int tt_gemm(int32_t a_col_major, int32_t b_col_major, int64_t M, int64_t N, int64_t K, const float* A,
                       int64_t lda, const float* B, int64_t ldb, int32_t mask_operand, const float* mask, int64_t ldm,
                       const float* scale, int64_t ones_row, const float* bias, int32_t relu, float* C, int64_t ldc,
                       int32_t splits, int64_t slice, int32_t precision, void* workspace,
                       size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(M >= 0 && N >= 0 && K >= 0, "tt_gemm: negative shape");
  TT_REQUIRE(splits >= 1 && splits <= 65535, "tt_gemm: splits %d out of range", splits);
  TT_REQUIRE(precision == TT_GEMM_BF16 || precision == TT_GEMM_BF16X3, "tt_gemm: unknown precision %d", precision);
  TT_REQUIRE(mask_operand >= 0 && mask_operand <= 2, "tt_gemm: mask_operand must be 0, 1 (A) or 2 (B)");
  TT_REQUIRE(mask_operand == 0 || mask != nullptr, "tt_gemm: NULL mask");
  TT_REQUIRE(ones_row < 0 || ones_row == M - 1, "tt_gemm: ones_row must be the last row of C");
  const int64_t a_rows = ones_row >= 0 ? M - 1 : M;
  if (M == 0 || N == 0) return TT_OK;
  TT_REQUIRE(C != nullptr && ldc >= N, "tt_gemm: bad C / ldc");
  TT_REQUIRE(splits == 1 || slice >= (M - 1) * ldc + N, "tt_gemm: slice stride too small");
  TT_REQUIRE(K == 0 || a_rows == 0 || (A != nullptr && lda >= (a_col_major ? a_rows : K)), "tt_gemm: bad A / lda");
  TT_REQUIRE(K == 0 || (B != nullptr && ldb >= (b_col_major ? K : N)), "tt_gemm: bad B / ldb");
  const int64_t mask_w = mask_operand == 1 ? (a_col_major ? a_rows : K) : (b_col_major ? K : N);
  TT_REQUIRE(mask_operand == 0 || ldm >= mask_w, "tt_gemm: ldm < mask width");
  TT_REQUIRE(!(splits > 1 && (bias || relu)), "tt_gemm: bias / relu epilogue needs splits == 1");
  GemmArgs g{};
  g.A = A;
  g.lda = lda;
  g.B = B;
  g.ldb = ldb;
  g.mask = mask;
  g.ldm = ldm;
  g.scale = scale;
  g.bias = bias;
  g.C = C;
  g.ldc = ldc;
  g.slice = slice;
  g.M = M;
  g.N = N;
  g.K = K;
  g.a_rows = a_rows;
  g.ones_row = ones_row >= 0 ? static_cast<int>(ones_row) : -1;
  g.relu = relu ? 1 : 0;
  g.k_per_split = round_up(ceil_div(K > 0 ? K : 1, splits), kBK);
  g.vec_a = (lda % 4 == 0) && aligned16(A);
  g.vec_b = (ldb % 4 == 0) && aligned16(B);
  g.vec_m = mask_operand ? ((ldm % 4 == 0) && aligned16(mask)) : 0;
  const bool x3 = precision == TT_GEMM_BF16X3;
  hipStream_t st = to_stream(stream);
  // bf16, y = x W (+bias, relu) or dx = G W^T (masked A), weight small enough
  // to sit in LDS whole: weight-stationary form.
  {
    const int64_t Kp = round_up(K > 0 ? K : 1, 16);
    const bool form = !x3 && splits == 1 && !a_col_major && ones_row < 0 && mask_operand != 2 && N <= 288 &&
                      K <= 32 * kWsMaxChunks &&
                      static_cast<size_t>(Kp) * round_up(N, 32) * sizeof(uint16_t) +
                              static_cast<size_t>(M >= 512 * 32 ? 2 : kWsWaves) * 2 * kWsChunkElems * sizeof(uint16_t) <=
                          kWsLdsMax &&
                      (mask_operand == 0 || b_col_major) && ldc * 32 < (1ll << 31) &&
                      workspace != nullptr && workspace_bytes >= tt_gemm_workspace_size(N, K);
    if (form) {
      WsArgs w{};
      w.A = A;
      w.lda = lda;
      w.mask = mask;
      w.ldm = ldm;
      w.scale = scale;
      w.img = static_cast<const __bf16*>(workspace);
      w.bias = bias;
      w.C = C;
      w.ldc = ldc;
      w.M = M;
      w.N = static_cast<int>(N);
      w.K = static_cast<int>(K);
      w.Kp = static_cast<int>(Kp);
      w.relu = relu ? 1 : 0;
      w.vec = (lda % 4 == 0) && aligned16(A) && (mask_operand == 0 || ((ldm % 4 == 0) && aligned16(mask)));
      w.probe = g_gemm_probe;
      const int nb = static_cast<int>(ceil_div(N, 32));
      const int nq = static_cast<int>(Kp / 4) * nb * 32;
      if (b_col_major)
        hipLaunchKernelGGL(pack_weight_kernel<true>, dim3(static_cast<unsigned>(ceil_div(nq, 256))), dim3(256), 0, st,
                           B, ldb, static_cast<int>(K), static_cast<int>(N), static_cast<int>(Kp), nb,
                           static_cast<__bf16*>(workspace));
      else
        hipLaunchKernelGGL(pack_weight_kernel<false>, dim3(static_cast<unsigned>(ceil_div(nq, 256))), dim3(256), 0, st,
                           B, ldb, static_cast<int>(K), static_cast<int>(N), static_cast<int>(Kp), nb,
                           static_cast<__bf16*>(workspace));
      TT_CHECK_LAUNCH();
      return mask_operand ? launch_wstat<true>(w, nb, st) : launch_wstat<false>(w, nb, st);
    }
  }
  const int ac = a_col_major ? 1 : 0, bc = b_col_major ? 1 : 0;
  // the three layouts the tower uses, each with its mask placement
  if (!ac && !bc && mask_operand == 0) return dispatch_bm<false, false, 0>(g, splits, x3, st);  // y = x W
  if (!ac && bc && mask_operand == 1) return dispatch_bm<false, true, 1>(g, splits, x3, st);    // dx = G W^T
  if (ac && !bc && mask_operand == 2) return dispatch_bm<true, false, 2>(g, splits, x3, st);    // dW = x^T G
  if (!ac && bc && mask_operand == 0) return dispatch_bm<false, true, 0>(g, splits, x3, st);
  if (ac && !bc && mask_operand == 0) return dispatch_bm<true, false, 0>(g, splits, x3, st);
  return fail(TT_ERR_UNSUPPORTED, "tt_gemm: layout (a_col=%d, b_col=%d, mask=%d) not built", ac, bc, mask_operand);
}
