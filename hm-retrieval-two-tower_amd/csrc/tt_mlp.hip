// K4 (tower MLP), row-streaming form: C = epi(maskA(A) . B) for a tall fp32
// activation A [M, K] and a small weight operand B [K, N] (K, N <= 288),
// the shape of every Dense-layer GEMM of the towers except the weight
// gradients (/root/reference/pkg/modelling/models/tower.py:41-49):
//   forward   h = relu(x W + b)                       B = W,   epi bias + relu
//   backward  g_in = (g_out * relu'(y) * s) W^T        B = W^T, maskA = relu'(y) * s,
//             (optionally * relu'(x) for the layer below: epi cmask)
//
// Precision: bf16x3 on v_mfma_f32_32x32x16_bf16 with fp32 accumulation:
// a = a_hi + a_lo, b = b_hi + b_lo (hi = bf16(x), lo = bf16(x - hi)),
// a_lo b_hi + a_hi b_lo + a_hi b_hi — every product to ~2^-17 relative,
// i.e. fp32-faithful (the model-level parity tests hold the fp32 tolerance).
//
// Layout (MI355X): B is tiny and read by every workgroup, so it is split
// ONCE per call into a bf16 hi/lo image already in MFMA B-fragment order
// (tt_mlp_pack): one wave's fragment for (k-step, 32-column block, plane) is
// 1 KiB contiguous, so each wave loads its fragments straight from L2 into
// VGPRs with fully coalesced 16-B-per-lane loads, 3 k-steps ahead.  A is
// streamed once: 64 rows per workgroup (256 workgroups fill the 256 CUs at
// M = 16384), 64-deep fp32 stages loaded row-contiguous by range-checked
// buffer loads two stages ahead (rows past M and depths past K read as 0),
// masked, split into hi/lo and written to a double-buffered XOR-swizzled LDS
// tile, read back as A fragments with conflict-free ds_read_b128.  The main
// loop is branch-free (the image is zero-padded to whole stages and to 4
// column blocks per wave row), so the compiler's vmcnt waits are exact.
// 4 waves; wave w computes rows 0..63 x the 32-column blocks w, w+4, w+8
// (each B fragment is loaded by exactly one wave of the workgroup).
#include <type_traits>

#include <cstdlib>

#include "tt_common.h"
#include "tt_mlp_pack.h"

namespace tt {
namespace {

constexpr int kMlpThreads = 256;
#ifndef TT_MLP_BM
#define TT_MLP_BM 64
#endif
constexpr int kMlpBM = TT_MLP_BM;  // rows per workgroup (32 or 64)
constexpr int kMlpRB = kMlpBM / 32;  // 32-row MFMA blocks per wave
constexpr int kMlpUQ = kMlpBM / 16;  // A rows per thread per stage
constexpr int kMlpBK = 64;       // depth per A stage (4 MFMA k-steps)
constexpr int kMlpMaxCB = 3;     // 32-column blocks per wave (N <= 384)


struct MlpArgs {
  const float* A;
  int64_t lda;
  const float* amask;  // A := (amask > 0) ? A * s : 0   (HAS_MASK)
  int64_t ldam;
  const float* scale;  // device scalar s (NULL: 1)
  const __bf16* img;   // B image [KSp][NBp][2][64][8]
  int64_t M;
  int K, N, KSp, NBp;
  const float* bias;   // epilogue + bias[n] (NULL: none)
  int relu;
  const float* cmask;  // epilogue: C := (cmask > 0) ? C : 0 (NULL: none)
  int64_t ldcm;
  float* C;
  int64_t ldc;
  float* parts;        // optional [gridDim.x][N]: per-workgroup column sums of C
};

// Raw buffer resource over `bytes` bytes: loads past the end return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mlp_desc(const void* base, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                           static_cast<int>(bytes > 0x7fffffffull ? 0x7fffffffu : bytes),
                                           0x00020000);
}

__device__ __forceinline__ f32x4 mlp_load4(__amdgpu_buffer_rsrc_t d, unsigned voff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(d, voff, 0, 0));
}
// voff per lane (loop-invariant), soff uniform (e.g. the stage's row offset)
__device__ __forceinline__ f32x4 mlp_load4s(__amdgpu_buffer_rsrc_t d, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(d, voff, soff, 0));
}

using pack::bf16_bits;
using pack::bf16_val;
using pack::pack_fragment;
using pack::PackJob;
using pack::PackJobs;
using pack::kMaxPackJobs;
using pack::mlp_ks;
using pack::mlp_nb;

// LDS A tile: plane p, row r (0..63), 16-B chunk c (0..7) of the 64-deep stage
// at byte (p * 64 + r) * 128 + ((c ^ ((r >> 1) & 7)) << 4): the 16 lanes of
// one ds_read_b128 cycle (16 consecutive rows, one chunk) cover all 64 banks.
__device__ __forceinline__ int a_lds_off(int plane, int row, int chunk) {
  return ((plane * kMlpBM + row) << 7) + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// A stages (2 x 2 planes x 64 rows x 128 B = 32 KiB), then the output tile
// [64][NCB * 128 + 4] fp32 of the epilogue (<= 97 KiB)
template <int NCB>
struct MlpSmem {
  static constexpr int OUT_LD = NCB * 128 + 4;
  static constexpr int BYTES = kMlpBM * OUT_LD * 4 > 2 * 2 * kMlpBM * 128 ? kMlpBM * OUT_LD * 4 : 2 * 2 * kMlpBM * 128;
};

// One workgroup's rows [bid * kMlpBM, +kMlpBM) of one problem; smem_raw holds
// MlpSmem<NCB>::BYTES.
template <int NCB, bool HAS_MASK>
__device__ __forceinline__ void mlp_rows_block(const MlpArgs& a, const int64_t bid, char* smem_raw) {
  constexpr int OUT_LD = MlpSmem<NCB>::OUT_LD;
  char (*smem)[2 * kMlpBM * 128] = reinterpret_cast<char (*)[2 * kMlpBM * 128]>(smem_raw);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = lane_id();
  const int l32 = lane & 31, h = lane >> 5;
  const int64_t m0 = bid * kMlpBM;
  const float s = a.scale ? *a.scale : 1.0f;

  // ---- A stages: thread -> rows qrow + 16 u (u < 4), depths qk .. qk + 3 ------
  // (16 threads per row: 256 contiguous bytes per row per stage)
  const int qrow = tid >> 4, qk = (tid & 15) * 4;
  const __amdgpu_buffer_rsrc_t da = mlp_desc(a.A + m0 * a.lda, static_cast<uint64_t>(a.M - m0) * a.lda * 4);
  const __amdgpu_buffer_rsrc_t dm = mlp_desc(HAS_MASK ? a.amask + m0 * a.ldam : a.A, static_cast<uint64_t>(a.M - m0) * a.ldam * 4);
  f32x4 ra[2][kMlpUQ], rm[2][kMlpUQ];
  auto fetch_a = [&](int k0, auto slot_c) {
    constexpr int SL = decltype(slot_c)::value;
#pragma unroll
    for (int u = 0; u < kMlpUQ; ++u) {
      const int row = qrow + 16 * u;
      ra[SL][u] = mlp_load4(da, static_cast<unsigned>((row * a.lda + k0 + qk) * 4));
      if constexpr (HAS_MASK) rm[SL][u] = mlp_load4(dm, static_cast<unsigned>((row * a.ldam + k0 + qk) * 4));
    }
  };
  auto stash_a = [&](int k0, auto slot_c, int buf) {
    constexpr int SL = decltype(slot_c)::value;
    char* base = smem[buf];
#pragma unroll
    for (int u = 0; u < kMlpUQ; ++u) {
      const int row = qrow + 16 * u;
      unsigned hb[4], lb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = (k0 + qk + e < a.K) ? ra[SL][u][e] : 0.0f;  // depths past K (or a ragged row's tail)
        if constexpr (HAS_MASK) v = (rm[SL][u][e] > 0.0f) ? v * s : 0.0f;
        hb[e] = bf16_bits(v);
        lb[e] = bf16_bits(v - bf16_val(hb[e]));
      }
      const int chunk = qk >> 3, half = (qk >> 2) & 1;
      *reinterpret_cast<uint2*>(base + a_lds_off(0, row, chunk) + 8 * half) =
          make_uint2(hb[0] | (hb[1] << 16), hb[2] | (hb[3] << 16));
      *reinterpret_cast<uint2*>(base + a_lds_off(1, row, chunk) + 8 * half) =
          make_uint2(lb[0] | (lb[1] << 16), lb[2] | (lb[3] << 16));
    }
  };

  // ---- B fragments: k-step ks, block i (column block wave + 4 i), plane p ----
  const bf16x8* img = reinterpret_cast<const bf16x8*>(a.img) + lane;
  const int64_t kstride = static_cast<int64_t>(a.NBp) * 2 * 64;  // bf16x8 per k-step
  bf16x8 bq[4][NCB][2];  // k-step ks in slot ks % 4 (static under the 2-stage unroll)
  auto load_b = [&](int ks, auto slot_c) {
    constexpr int SL = decltype(slot_c)::value;
    const int kc = ks < a.KSp ? ks : a.KSp - 1;  // past the end: a harmless re-read
#pragma unroll
    for (int i = 0; i < NCB; ++i) {
      const bf16x8* p = img + kc * kstride + ((wave + 4 * i) * 2) * 64;
      bq[SL][i][0] = p[0];
      bq[SL][i][1] = p[64];
    }
  };

  f32x16 acc[kMlpRB][NCB];
#pragma unroll
  for (int rb = 0; rb < kMlpRB; ++rb)
#pragma unroll
    for (int i = 0; i < NCB; ++i) acc[rb][i] = f32x16{};

  const int nstage = (a.K + kMlpBK - 1) / kMlpBK;  // KSp = 4 nstage
  const int ks_end = (a.K + 15) / 16;               // k-steps holding data
  load_b(0, std::integral_constant<int, 0>());
  load_b(1, std::integral_constant<int, 1>());
  load_b(2, std::integral_constant<int, 2>());
  fetch_a(0, std::integral_constant<int, 0>());
  fetch_a(kMlpBK, std::integral_constant<int, 1>());
  stash_a(0, std::integral_constant<int, 0>(), 0);
  __syncthreads();
  // stage st (parity PAR): A of stage st + 1 sits in ra[1 - PAR], stage st + 2
  // is fetched into ra[PAR]; k-steps 4 st .. 4 st + 3 use B slots 0..3 and
  // prefetch k-steps 4 st + 3 .. 4 st + 6.
  auto stage = [&](int st, auto par_c) {
    constexpr int PAR = decltype(par_c)::value;
    fetch_a((st + 2) * kMlpBK, std::integral_constant<int, PAR>());
    const char* base = smem[PAR];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int ks = 4 * st + kk;
      if (kk == 0) load_b(ks + 3, std::integral_constant<int, 3>());
      if (kk == 1) load_b(ks + 3, std::integral_constant<int, 0>());
      if (kk == 2) load_b(ks + 3, std::integral_constant<int, 1>());
      if (kk == 3) load_b(ks + 3, std::integral_constant<int, 2>());
      if (ks >= ks_end) continue;  // the zero padding of the last stage (uniform)
      bf16x8 ah[kMlpRB], al[kMlpRB];
#pragma unroll
      for (int rb = 0; rb < kMlpRB; ++rb) {
        const int row = 32 * rb + l32, chunk = 2 * kk + h;
        ah[rb] = *reinterpret_cast<const bf16x8*>(base + a_lds_off(0, row, chunk));
        al[rb] = *reinterpret_cast<const bf16x8*>(base + a_lds_off(1, row, chunk));
      }
#pragma unroll
      for (int i = 0; i < NCB; ++i)
#pragma unroll
        for (int rb = 0; rb < kMlpRB; ++rb) {
          acc[rb][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[rb], bq[kk][i][0], acc[rb][i], 0, 0, 0);
          acc[rb][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[rb], bq[kk][i][1], acc[rb][i], 0, 0, 0);
          acc[rb][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[rb], bq[kk][i][0], acc[rb][i], 0, 0, 0);
        }
    }
    if (st + 1 < nstage) {
      stash_a((st + 1) * kMlpBK, std::integral_constant<int, 1 - PAR>(), 1 - PAR);
      lds_barrier();  // LDS hand-off only: the A / B prefetches stay in flight
    }
  };
  for (int st = 0; st < nstage; st += 2) {
    stage(st, std::integral_constant<int, 0>());
    if (st + 1 < nstage) stage(st + 1, std::integral_constant<int, 1>());
  }

  // ---- epilogue: lane (l32, h), register r -> row (r & 3) + 8 (r >> 2) + 4 h, column l32
  // acc (+ bias, relu) -> LDS tile [64][OUT_LD] (column = 32 cb + l32 of this
  // wave's blocks, in block order cb = wave + 4 i), then row-contiguous vector
  // stores of C with the epilogue mask read the same way (coalesced).
  __syncthreads();  // every wave is done reading the A stages
  float* tile = reinterpret_cast<float*>(smem_raw);
#pragma unroll
  for (int i = 0; i < NCB; ++i) {
    const int col = (wave + 4 * i) * 32 + l32;
    const float b = (a.bias && col < a.N) ? a.bias[col] : 0.0f;
#pragma unroll
    for (int rb = 0; rb < kMlpRB; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = acc[rb][i][r] + b;
        if (a.relu) v = v > 0.0f ? v : 0.0f;
        tile[(32 * rb + (r & 3) + 8 * (r >> 2) + 4 * h) * OUT_LD + col] = v;
      }
  }
  __syncthreads();
  const int64_t rows = a.M - m0 < kMlpBM ? a.M - m0 : kMlpBM;
  float* C = a.C + m0 * a.ldc;
  const float* cm = a.cmask ? a.cmask + m0 * a.ldcm : nullptr;
  // 16-B stores of whole rows; a ragged N writes its row's padding columns
  // (zeros: the image is zero there) when the row pitch has room for them
  const int n4 = (a.N + 3) / 4 * 4;
  const bool v4 = (a.ldc % 4 == 0) && (a.ldc >= n4) && (reinterpret_cast<uintptr_t>(a.C) % 16 == 0) &&
                  (!cm || ((a.N % 4 == 0) && (a.ldcm % 4 == 0) && (reinterpret_cast<uintptr_t>(a.cmask) % 16 == 0)));
  if (v4) {
    const int per_row = n4 / 4;
    for (int idx = tid; idx < rows * per_row; idx += kMlpThreads) {
      const int row = idx / per_row, c4 = (idx - row * per_row) * 4;
      f32x4 v = *reinterpret_cast<const f32x4*>(tile + row * OUT_LD + c4);
      if (cm) {
        const f32x4 mk = *reinterpret_cast<const f32x4*>(cm + row * a.ldcm + c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = mk[e] > 0.0f ? v[e] : 0.0f;
        if (a.parts) *reinterpret_cast<f32x4*>(tile + row * OUT_LD + c4) = v;  // masked, for the column sums
      }
      *reinterpret_cast<f32x4*>(C + row * a.ldc + c4) = v;
    }
  } else {
    for (int idx = tid; idx < rows * a.N; idx += kMlpThreads) {
      const int row = idx / a.N, c = idx - row * a.N;
      float v = tile[row * OUT_LD + c];
      if (cm && !(cm[row * a.ldcm + c] > 0.0f)) v = 0.0f;
      if (cm && a.parts) tile[row * OUT_LD + c] = v;
      C[row * a.ldc + c] = v;
    }
  }
  if (a.parts == nullptr) return;
  // column sums (the bias gradient of the layer below when C is its masked
  // output gradient): this workgroup's rows in order; mlp_colsum_kernel then
  // adds the workgroups' partials in workgroup order (deterministic).
  __syncthreads();
  for (int c = tid; c < a.N; c += kMlpThreads) {
    float sum = 0.0f;
    for (int row = 0; row < rows; ++row) sum += tile[row * OUT_LD + c];  // already masked
    a.parts[bid * a.N + c] = sum;
  }
}

template <int NCB, bool HAS_MASK>
__global__ void __launch_bounds__(kMlpThreads) mlp_rows_kernel(const MlpArgs a) {
  __shared__ __attribute__((aligned(16))) char smem_raw[MlpSmem<NCB>::BYTES];
  mlp_rows_block<NCB, HAS_MASK>(a, blockIdx.x, smem_raw);
}

// Two independent problems in one launch (the two towers' layers): blocks
// [0, split) are a0's, the rest a1's.
template <int NCB0, int NCB1, bool HAS_MASK>
__global__ void __launch_bounds__(kMlpThreads) mlp_rows_pair_kernel(const MlpArgs a0, const MlpArgs a1,
                                                                    const int split) {
  constexpr int B0 = MlpSmem<NCB0>::BYTES, B1 = MlpSmem<NCB1>::BYTES;
  __shared__ __attribute__((aligned(16))) char smem_raw[B0 > B1 ? B0 : B1];
  const int b = blockIdx.x;
  if (b < split) mlp_rows_block<NCB0, HAS_MASK>(a0, b, smem_raw);
  else mlp_rows_block<NCB1, HAS_MASK>(a1, b - split, smem_raw);
}

// out[c] = sum over b of parts[b][c] in b order; 64 columns x 16 row groups
// per block, the 16 group sums added in order in LDS.
__global__ void __launch_bounds__(1024) mlp_colsum_kernel(const float* __restrict__ parts, int nblk, int N,
                                                          float* __restrict__ out) {
  __shared__ float red[16][65];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const int per = (nblk + 15) / 16;
  float sum = 0.0f;
  if (c < N) {
    const int b1 = min(nblk, (grp + 1) * per);
    for (int bb = grp * per; bb < b1; bb += 16) {  // 16 loads in flight (index clamped), added in order
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = parts[static_cast<int64_t>(min(bb + u, b1 - 1)) * N + c];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (bb + u < b1) sum += v[u];
    }
  }
  red[grp][threadIdx.x & 63] = sum;
  __syncthreads();
  if (grp == 0 && c < N) {
    float t = red[0][threadIdx.x];
#pragma unroll
    for (int g = 1; g < 16; ++g) t += red[g][threadIdx.x];
    out[c] = t;
  }
}


// ---------------------------------------------------------------------------
// Weight gradient of a Dense layer (the tape's MatMul for the kernel and
// BiasAddGrad for the bias, tower.py:41-49):
//   [dW; db] = [A | 1]^T . Gm    (A [M, Ka] activations, Gm [M, N] the
//   layer's output gradient, optionally Gm = (gmask > 0) ? G * s : 0 — the
//   ReluGrad of the layer's own relu folded into the load)
// The output [Ka + 1, N] is exactly the flat parameter layout (kernel rows
// then the bias row).  Split-K over the batch: grid = S splits x 64 x 64
// output tiles; each workgroup reduces its split's rows for one tile into
// its split's partial [Ka + 1, N], and mlp_sum_parts_kernel adds the
// partials in split order (deterministic).  The tiles of one split sit on
// one XCD (blockIdx % 8 picks the XCD), so the split's rows that its tiles
// all stage come from that XCD's L2.
// Both MFMA operands need 8 consecutive BATCH rows per lane; the staged
// 32-row stages are written ROW-major (as loaded: each thread converts 8
// consecutive columns of one row to bf16 hi / lo and stores 16 B per plane)
// and the fragments are read with the hardware transposing read
// ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group, delivered
// column-major).  Rows are 192 B apart (128 B of data): the 4 rows x 2 groups
// of a 32-lane half then start at banks 48q + 8g mod 64, all distinct.
// 4 waves; wave w owns the 32 x 32 block (w & 1, w >> 1) of the tile;
// bf16x3 (a_lo b_hi + a_hi b_lo + a_hi b_hi), fp32 accumulation.
constexpr int kWgThreads = 256;
constexpr int kWgTile = 64;       // output tile: 64 rows of [A | 1]^T x 64 columns of Gm
constexpr int kWgBK = 32;         // batch rows per stage (2 MFMA k-steps)
constexpr int kWgRowB = 192;      // LDS bytes per staged row
constexpr int kWgPlaneB = kWgBK * kWgRowB;       // 6 KiB
constexpr int kWgStageB = 4 * kWgPlaneB;         // A hi, A lo, G hi, G lo: 24 KiB
constexpr int kWgDepth = 3;       // stages of global loads in flight

struct WgradArgs {
  const float* A;
  int64_t lda;
  const float* G;
  int64_t ldg;
  const float* gmask;  // (MASK) Gm = (gmask > 0) ? G * s : 0
  int64_t ldgm;
  const float* scale;
  int64_t M;
  int Ka, N;
  int TI, TJ, S;       // tiles along [A | 1] columns and Gm columns, splits
  int64_t rows_per_split;
  float* parts;        // [S][(Ka + 1) * N]
};

typedef __bf16 wg_bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) wg_bf16x4 lds_bf16x4_t;

// Workgroup b of one problem; wsm holds 2 * kWgStageB bytes.
template <bool MASK>
__device__ __forceinline__ void mlp_wgrad_block(const WgradArgs& a, const int b, char* wsm) {
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = lane_id();
  // b -> (split, tile); the tiles of a split on one XCD when S % 8 == 0
  const int tiles = a.TI * a.TJ;
  int split, tile;
  {
    if (a.S % 8 == 0) {
      const int q = b >> 3;
      tile = q % tiles;
      split = (q / tiles) * 8 + (b & 7);
    } else {
      tile = b % tiles;
      split = b / tiles;
    }
  }
  const int i0 = (tile / a.TJ) * kWgTile;  // first [A | 1] column (= output row)
  const int j0 = (tile % a.TJ) * kWgTile;  // first Gm column
  const int64_t r0 = static_cast<int64_t>(split) * a.rows_per_split;
  int64_t r1 = r0 + a.rows_per_split;
  if (r1 > a.M) r1 = a.M;
  // a split starting past M (rows_per_split is rounded up to whole stages)
  // has no rows: its descriptors get 0 bytes, so the prologue's loads return
  // zeros instead of reading past the operands
  if (r1 < r0) r1 = r0;
  const int nstage = r1 > r0 ? static_cast<int>((r1 - r0 + kWgBK - 1) / kWgBK) : 0;
  const float s = a.scale ? *a.scale : 1.0f;

  // loader: thread t stages row t / 8 of a stage, columns 8 (t % 8) .. + 7 of
  // both operand tiles; range-checked buffer loads (rows past the split read 0)
  const int lrow = tid >> 3, lcol = (tid & 7) * 8;
  const __amdgpu_buffer_rsrc_t dA = mlp_desc(a.A + r0 * a.lda, static_cast<uint64_t>(r1 - r0) * a.lda * 4);
  const __amdgpu_buffer_rsrc_t dG = mlp_desc(a.G + r0 * a.ldg, static_cast<uint64_t>(r1 - r0) * a.ldg * 4);
  const __amdgpu_buffer_rsrc_t dM =
      mlp_desc(MASK ? a.gmask + r0 * a.ldgm : a.G, static_cast<uint64_t>(r1 - r0) * (MASK ? a.ldgm : a.ldg) * 4);
  const unsigned lda4 = static_cast<unsigned>(a.lda) * 4, ldg4 = static_cast<unsigned>(a.ldg) * 4,
                 ldm4 = static_cast<unsigned>(MASK ? a.ldgm : a.ldg) * 4;
  // columns past Ka (A) / N (Gm) are zeroed after the load (their loads read
  // on into the row's padding or the next row, or 0 past the split)
  const int ca = i0 + lcol, cg = j0 + lcol;
  const unsigned oa = lrow * lda4 + static_cast<unsigned>(ca) * 4;
  const unsigned og = lrow * ldg4 + static_cast<unsigned>(cg) * 4;
  const unsigned om = lrow * ldm4 + static_cast<unsigned>(cg) * 4;
  f32x4 va[kWgDepth][2], vg[kWgDepth][2], vm[kWgDepth][MASK ? 2 : 1];
  auto fetch = [&](int st, auto slot_c) {
    constexpr int SL = decltype(slot_c)::value;
    const unsigned sa = static_cast<unsigned>(st * kWgBK) * lda4, sg = static_cast<unsigned>(st * kWgBK) * ldg4,
                   sm = static_cast<unsigned>(st * kWgBK) * ldm4;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      va[SL][e] = mlp_load4s(dA, oa + 16 * e, sa);
      vg[SL][e] = mlp_load4s(dG, og + 16 * e, sg);
      if constexpr (MASK) vm[SL][e] = mlp_load4s(dM, om + 16 * e, sm);
    }
  };
  // 8 values -> 16 B of hi and 16 B of lo at (plane pair, this thread's row, columns)
  auto put8 = [&](char* base, const float (&x)[8]) {
    unsigned hw[4], lw[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned h0 = bf16_bits(x[2 * e]), h1 = bf16_bits(x[2 * e + 1]);
      const unsigned l0 = bf16_bits(x[2 * e] - bf16_val(h0)), l1 = bf16_bits(x[2 * e + 1] - bf16_val(h1));
      hw[e] = h0 | (h1 << 16);
      lw[e] = l0 | (l1 << 16);
    }
    char* p = base + lrow * kWgRowB + lcol * 2;
    *reinterpret_cast<u32x4*>(p) = u32x4{hw[0], hw[1], hw[2], hw[3]};
    *reinterpret_cast<u32x4*>(p + kWgPlaneB) = u32x4{lw[0], lw[1], lw[2], lw[3]};
  };
  auto stash = [&](int st, int buf, auto slot_c) {
    constexpr int SL = decltype(slot_c)::value;
    char* base = wsm + buf * kWgStageB;
    const bool live = r0 + static_cast<int64_t>(st) * kWgBK + lrow < r1;
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // [A | 1]: the ones column is the bias row of the output
      const int col = ca + e;
      x[e] = col < a.Ka ? va[SL][e >> 2][e & 3] : ((col == a.Ka && live) ? 1.0f : 0.0f);
    }
    put8(base, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = cg + e;
      float v = col < a.N ? vg[SL][e >> 2][e & 3] : 0.0f;
      if constexpr (MASK) v = vm[SL][e >> 2][e & 3] > 0.0f ? v * s : 0.0f;
      x[e] = v;
    }
    put8(base + 2 * kWgPlaneB, x);
  };

  // fragments: 16-lane group g -> MFMA rows / columns 16 (g & 1) .. + 15 of
  // the wave's 32-block, batch rows 8 (g >> 1) .. + 7 of the k-step; lane
  // 4q + p of the group addresses row q, columns 4p .. 4p + 3
  const int ib = wave & 1, jb = wave >> 1;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int frow = 8 * (g >> 1) + q;
  const int fa = frow * kWgRowB + (32 * ib + 16 * (g & 1) + 4 * p) * 2;
  const int fg = 2 * kWgPlaneB + frow * kWgRowB + (32 * jb + 16 * (g & 1) + 4 * p) * 2;
  auto frag = [&](const char* base, int off) {
    const wg_bf16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(base + off));
    const wg_bf16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(base + off + 4 * kWgRowB));
    return __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  f32x16 acc = {};
  auto compute = [&](int buf) {
    const char* base = wsm + buf * kWgStageB;
#pragma unroll
    for (int ks = 0; ks < kWgBK / 16; ++ks) {
      const int ko = ks * 16 * kWgRowB;
      const bf16x8 ah = frag(base, fa + ko), al = frag(base + kWgPlaneB, fa + ko);
      const bf16x8 gh = frag(base, fg + ko), gl = frag(base + kWgPlaneB, fg + ko);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, gh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, gl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, gh, acc, 0, 0, 0);
    }
  };

  // pipeline: kWgDepth stages of loads in flight; stage st is stashed into
  // buffer st % 2 right after its loads land, one barrier per stage (a wave
  // passes it only after computing stage st - 1 from the other buffer)
  static_assert(kWgDepth == 3, "the stage loop below is unrolled 3x");
  fetch(0, std::integral_constant<int, 0>());  // issued in stage order (the waits count on it)
  __builtin_amdgcn_sched_barrier(0);
  fetch(1, std::integral_constant<int, 1>());
  __builtin_amdgcn_sched_barrier(0);
  fetch(2, std::integral_constant<int, 2>());
  auto step = [&](int st, auto slot_c) {
    // nothing crosses a step boundary: the scheduler would otherwise hoist the
    // later steps' conversions to the loop top and wait for every load there
    __builtin_amdgcn_sched_barrier(0);
    stash(st, st & 1, slot_c);
    __builtin_amdgcn_sched_barrier(0);
    fetch(st + kWgDepth, slot_c);  // past the split: zeros, unused
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
    compute(st & 1);
  };
  // branch-free body (stages past the split stage zeros, which add nothing),
  // so the compiler's vmcnt waits stay exact across the stages in flight
  for (int st = 0; st < nstage; st += 3) {
    step(st, std::integral_constant<int, 0>());
    step(st + 1, std::integral_constant<int, 1>());
    step(st + 2, std::integral_constant<int, 2>());
  }

  // this block of the split's partial: lane (l32, h), register r -> row
  // 32 ib + (r & 3) + 8 (r >> 2) + 4 h, column 32 jb + l32
  const int rows_out = a.Ka + 1;
  float* P = a.parts + static_cast<int64_t>(split) * rows_out * a.N;
  const int n = j0 + 32 * jb + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = i0 + 32 * ib + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (n < a.N && row < rows_out) P[static_cast<int64_t>(row) * a.N + n] = acc[r];
  }
}

template <bool MASK>
__global__ void __launch_bounds__(kWgThreads) mlp_wgrad_kernel(const WgradArgs a) {
  __shared__ __attribute__((aligned(16))) char wsm[2 * kWgStageB];
  mlp_wgrad_block<MASK>(a, blockIdx.x, wsm);
}

// Two problems in one launch: blocks [0, split) are a0's (split % 8 == 0
// keeps the second problem's split -> XCD mapping).
template <bool MASK>
__global__ void __launch_bounds__(kWgThreads) mlp_wgrad_pair_kernel(const WgradArgs a0, const WgradArgs a1,
                                                                    const int split) {
  __shared__ __attribute__((aligned(16))) char wsm[2 * kWgStageB];
  const int b = blockIdx.x;
  if (b < split) mlp_wgrad_block<MASK>(a0, b, wsm);
  else mlp_wgrad_block<MASK>(a1, b - split, wsm);
}

// out[e] = sum over splits of parts[sp][e] (deterministic): a block covers 64
// float4 of the output; group g of 16 adds splits [g S/16, (g+1) S/16) in
// order (their loads all in flight), then the 16 group sums are added in
// group order.  len % 4 == 0.
// Optional Adagrad on the summed gradient (tt_mlp_wgrad_adagrad): the layer's
// parameters and accumulator, the same per-element arithmetic as
// tt_dense_adagrad.
struct PartsAdagrad {
  float* param;  // NULL: none
  float* accum;
  float lr, eps;
};

__device__ __forceinline__ void mlp_sum_parts_block(const float* __restrict__ parts, int S, int64_t len,
                                                    float* __restrict__ out, const int64_t bid, f32x4 (*red)[64],
                                                    const PartsAdagrad& ad = PartsAdagrad{}) {
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t e4 = (bid * 64 + lane) * 4;
  const int per = (S + 15) / 16;
  const int s0 = grp * per, s1 = min(S, s0 + per);
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  if (e4 < len) {
    f32x4 v[8];
    for (int sb = s0; sb < s1; sb += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (sb + u < s1) v[u] = *reinterpret_cast<const f32x4*>(parts + (sb + u) * len + e4);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (sb + u < s1) {
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] += v[u][q];
        }
    }
  }
  red[grp][lane] = acc;
  __syncthreads();
  if (grp == 0 && e4 < len) {
    f32x4 t = red[0][lane];
    for (int g = 1; g < 16; ++g) {
      const f32x4 r = red[g][lane];
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] += r[q];
    }
    *reinterpret_cast<f32x4*>(out + e4) = t;
    if (ad.param) {
      f32x4 pa = *reinterpret_cast<const f32x4*>(ad.param + e4);
      f32x4 ac = *reinterpret_cast<const f32x4*>(ad.accum + e4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gi = t[q];
        const float a = ac[q] + gi * gi;
        ac[q] = a;
        pa[q] = pa[q] - (gi * ad.lr) / (sqrtf(a) + ad.eps);
      }
      *reinterpret_cast<f32x4*>(ad.accum + e4) = ac;
      *reinterpret_cast<f32x4*>(ad.param + e4) = pa;
    }
  }
}

__global__ void __launch_bounds__(1024) mlp_sum_parts_kernel(const float* __restrict__ parts, int S, int64_t len,
                                                             float* __restrict__ out, const PartsAdagrad ad) {
  __shared__ f32x4 red[16][64];
  mlp_sum_parts_block(parts, S, len, out, blockIdx.x, red, ad);
}

// Both problems' partial sums in one launch: blocks [0, split) are the first's.
__global__ void __launch_bounds__(1024) mlp_sum_parts_pair_kernel(const float* __restrict__ p0, int S0, int64_t len0,
                                                                  float* __restrict__ o0, const float* __restrict__ p1,
                                                                  int S1, int64_t len1, float* __restrict__ o1,
                                                                  const int split) {
  __shared__ f32x4 red[16][64];
  const int b = blockIdx.x;
  if (b < split) mlp_sum_parts_block(p0, S0, len0, o0, b, red);
  else mlp_sum_parts_block(p1, S1, len1, o1, b - split, red);
}

__global__ void __launch_bounds__(256) mlp_pack_kernel(const float* __restrict__ w, int64_t ldw, int K, int N,
                                                       int trans, int KS, int NB, __bf16* __restrict__ img) {
  const int64_t t = blockIdx.x * 256ll + threadIdx.x;
  if (t >= static_cast<int64_t>(KS) * NB * 64) return;
  const int lane = static_cast<int>(t & 63);
  pack_fragment(w, ldw, K, N, trans, static_cast<int>((t >> 6) / NB), static_cast<int>((t >> 6) % NB), NB, lane, img);
}

__global__ void __launch_bounds__(256) mlp_pack_many_kernel(const PackJobs jobs, int64_t total) {
  const int64_t t = blockIdx.x * 256ll + threadIdx.x;
  if (t >= total) return;
  pack::pack_many_thread(jobs, t);
}



}  // namespace
}  // namespace tt

using namespace tt;

extern "C" size_t tt_mlp_pack_bytes(int32_t K, int32_t N) {
  if (K < 1 || N < 1) return 0;
  return static_cast<size_t>(mlp_ks(K)) * mlp_nb(N) * 2 * 64 * 8 * sizeof(__bf16);
}

extern "C" int tt_mlp_pack(const float* w, int64_t ldw, int32_t K, int32_t N, int32_t trans, void* img,
                           size_t img_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(w && img, "tt_mlp_pack: NULL pointer");
  TT_REQUIRE(K >= 1 && N >= 1, "tt_mlp_pack: bad K/N");
  TT_REQUIRE(ldw >= (trans ? K : N), "tt_mlp_pack: ldw too small");
  TT_REQUIRE(img_bytes >= tt_mlp_pack_bytes(K, N), "tt_mlp_pack: image too small");
  const int KS = mlp_ks(K), NB = mlp_nb(N);
  const int64_t threads = static_cast<int64_t>(KS) * NB * 64;
  hipLaunchKernelGGL(mlp_pack_kernel, dim3(ceil_div(threads, 256)), dim3(256), 0, to_stream(stream), w, ldw, K, N,
                     trans ? 1 : 0, KS, NB, static_cast<__bf16*>(img));
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_mlp_pack_many(const tt_mlp_pack_job* jobs, int32_t num_jobs, tt_stream_t stream) {
  clear_error();
  PackJobs pj;
  int64_t total = 0;
  if (int rc = pack::make_pack_jobs(jobs, num_jobs, &pj, &total, "tt_mlp_pack_many")) return rc;
  hipLaunchKernelGGL(mlp_pack_many_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, to_stream(stream), pj, total);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" size_t tt_mlp_rows_workspace_size(int64_t M, int32_t N) {
  if (M < 0 || N < 1) return 0;
  return static_cast<size_t>(ceil_div(M, kMlpBM)) * N * sizeof(float);
}

// Validates one tt_mlp_rows problem (no colsum) into its kernel arguments;
// *ncb = column blocks per wave.  TT_OK or the error code (message set).
static int rows_setup(const char* fn, const float* A, int64_t lda, const float* amask, int64_t ldam,
                      const float* scale, int64_t M, int32_t K, const void* img, int32_t N, const float* bias,
                      int32_t relu, const float* cmask, int64_t ldcm, float* C, int64_t ldc, MlpArgs& a, int& ncb) {
  // a problem of no rows may come with NULL A / C (empty tensors have no storage)
  TT_REQUIRE(img && (M == 0 || (A && C)), "%s: NULL A/img/C", fn);
  TT_REQUIRE(M >= 0 && K >= 1 && N >= 1, "%s: bad M/K/N", fn);
  const int NB = mlp_nb(N);
  TT_REQUIRE(NB <= 4 * kMlpMaxCB, "%s: N=%d > %d unsupported", fn, N, 32 * 4 * kMlpMaxCB);
  TT_REQUIRE(M * lda < (int64_t(1) << 30) && (!amask || M * ldam < (int64_t(1) << 30)),
             "%s: operand too large for 32-bit buffer offsets", fn);
  TT_REQUIRE(lda >= K && ldc >= N && (!amask || ldam >= K) && (!cmask || ldcm >= N),
             "%s: leading dimension too small", fn);
  TT_REQUIRE(reinterpret_cast<uintptr_t>(A) % 16 == 0 && lda % 4 == 0 &&
                 (!amask || (reinterpret_cast<uintptr_t>(amask) % 16 == 0 && ldam % 4 == 0)),
             "%s: A / amask rows must be 16-B aligned (ld %% 4 == 0)", fn);
  a = MlpArgs{};
  a.A = A;
  a.lda = lda;
  a.amask = amask;
  a.ldam = ldam;
  a.scale = scale;
  a.img = static_cast<const __bf16*>(img);
  a.M = M;
  a.K = K;
  a.N = N;
  a.KSp = mlp_ks(K);
  a.NBp = NB;
  a.bias = bias;
  a.relu = relu ? 1 : 0;
  a.cmask = cmask;
  a.ldcm = ldcm;
  a.C = C;
  a.ldc = ldc;
  ncb = NB / 4;
  return TT_OK;
}

template <bool HM>
static void launch_rows(const MlpArgs& a, int ncb, hipStream_t st) {
  const dim3 grid(static_cast<unsigned>(ceil_div(a.M, kMlpBM)));
  if (ncb == 1) hipLaunchKernelGGL((mlp_rows_kernel<1, HM>), grid, dim3(kMlpThreads), 0, st, a);
  else if (ncb == 2) hipLaunchKernelGGL((mlp_rows_kernel<2, HM>), grid, dim3(kMlpThreads), 0, st, a);
  else hipLaunchKernelGGL((mlp_rows_kernel<3, HM>), grid, dim3(kMlpThreads), 0, st, a);
}

template <int NCB0, bool HM>
static void launch_rows_pair1(const MlpArgs& a0, const MlpArgs& a1, int ncb1, int split, dim3 grid,
                              hipStream_t st) {
  if (ncb1 == 1) hipLaunchKernelGGL((mlp_rows_pair_kernel<NCB0, 1, HM>), grid, dim3(kMlpThreads), 0, st, a0, a1, split);
  else if (ncb1 == 2) hipLaunchKernelGGL((mlp_rows_pair_kernel<NCB0, 2, HM>), grid, dim3(kMlpThreads), 0, st, a0, a1, split);
  else hipLaunchKernelGGL((mlp_rows_pair_kernel<NCB0, 3, HM>), grid, dim3(kMlpThreads), 0, st, a0, a1, split);
}

template <bool HM>
static void launch_rows_pair(const MlpArgs& a0, int ncb0, const MlpArgs& a1, int ncb1, hipStream_t st) {
  const int split = static_cast<int>(ceil_div(a0.M, kMlpBM));
  const dim3 grid(static_cast<unsigned>(split + ceil_div(a1.M, kMlpBM)));
  if (ncb0 == 1) launch_rows_pair1<1, HM>(a0, a1, ncb1, split, grid, st);
  else if (ncb0 == 2) launch_rows_pair1<2, HM>(a0, a1, ncb1, split, grid, st);
  else launch_rows_pair1<3, HM>(a0, a1, ncb1, split, grid, st);
}

extern "C" int tt_mlp_rows(const float* A, int64_t lda, const float* amask, int64_t ldam, const float* scale,
                           int64_t M, int32_t K, const void* img, int32_t N, const float* bias, int32_t relu,
                           const float* cmask, int64_t ldcm, float* C, int64_t ldc, float* colsum, void* workspace,
                           size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  MlpArgs a;
  int ncb = 0;
  const int rc = rows_setup("tt_mlp_rows", A, lda, amask, ldam, scale, M, K, img, N, bias, relu, cmask, ldcm, C, ldc,
                            a, ncb);
  if (rc != TT_OK) return rc;
  if (M == 0) return TT_OK;
  if (colsum) {
    TT_REQUIRE(workspace && workspace_bytes >= tt_mlp_rows_workspace_size(M, N),
               "tt_mlp_rows: colsum needs a workspace of tt_mlp_rows_workspace_size bytes");
    a.parts = static_cast<float*>(workspace);
  }
  hipStream_t st = to_stream(stream);
  if (amask) launch_rows<true>(a, ncb, st);
  else launch_rows<false>(a, ncb, st);
  TT_CHECK_LAUNCH();
  if (colsum) {
    hipLaunchKernelGGL(mlp_colsum_kernel, dim3(ceil_div(N, 64)), dim3(1024), 0, st, a.parts,
                       static_cast<int>(ceil_div(M, kMlpBM)), N, colsum);
  }
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_mlp_rows_pair(const tt_mlp_rows_problem* p, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(p, "tt_mlp_rows_pair: NULL problems");
  MlpArgs a[2];
  int ncb[2];
  for (int i = 0; i < 2; ++i) {
    const tt_mlp_rows_problem& q = p[i];
    const int rc = rows_setup("tt_mlp_rows_pair", q.A, q.lda, q.amask, q.ldam, q.scale, q.M, q.K, q.img, q.N,
                              q.bias, q.relu, q.cmask, q.ldcm, q.C, q.ldc, a[i], ncb[i]);
    if (rc != TT_OK) return rc;
  }
  hipStream_t st = to_stream(stream);
  const bool hm0 = a[0].amask != nullptr, hm1 = a[1].amask != nullptr;
  if (a[0].M == 0 || a[1].M == 0 || hm0 != hm1) {  // one problem, or masks differ: one launch each
    for (int i = 0; i < 2; ++i) {
      if (a[i].M == 0) continue;
      if (a[i].amask) launch_rows<true>(a[i], ncb[i], st);
      else launch_rows<false>(a[i], ncb[i], st);
    }
  } else if (hm0) {
    launch_rows_pair<true>(a[0], ncb[0], a[1], ncb[1], st);
  } else {
    launch_rows_pair<false>(a[0], ncb[0], a[1], ncb[1], st);
  }
  TT_CHECK_LAUNCH();
  return TT_OK;
}

static int wgrad_splits(int64_t M, int Ka, int N) {
  const int tiles = static_cast<int>(ceil_div(Ka + 1, kWgTile) * ceil_div(N, kWgTile));
  // TT_WGRAD_WGS: workgroups to aim for (default 1024: ~4 per CU, so the
  // loads of co-resident workgroups hide each other's latency)
  static const int64_t target = [] {
    const char* e = std::getenv("TT_WGRAD_WGS");
    return static_cast<int64_t>(e ? std::atoi(e) : 1024);
  }();
  int64_t S = 1;
  while (S < 256 && tiles * S * 2 <= target && M / (2 * S) >= 128) S *= 2;
  return static_cast<int>(S);
}

extern "C" size_t tt_mlp_wgrad_workspace_size(int64_t M, int32_t Ka, int32_t N) {
  if (M < 0 || Ka < 0 || N < 1) return 0;
  return static_cast<size_t>(wgrad_splits(M, Ka, N)) * (Ka + 1) * N * sizeof(float);
}

// Validates one tt_mlp_wgrad problem into its kernel arguments (parts unset).
static int wgrad_setup(const char* fn, const float* A, int64_t lda, const float* G, int64_t ldg, const float* gmask,
                       int64_t ldgm, const float* scale, int64_t M, int32_t Ka, int32_t N, float* dwb,
                       WgradArgs& a) {
  TT_REQUIRE(dwb && (M == 0 || (A && G)), "%s: NULL A/G/dwb", fn);
  TT_REQUIRE(M >= 0 && Ka >= 1 && Ka <= 4096, "%s: Ka=%d outside [1, 4096]", fn, Ka);
  TT_REQUIRE(N >= 4 && N <= 4096 && N % 4 == 0, "%s: N=%d must be a multiple of 4 in [4, 4096]", fn, N);
  TT_REQUIRE(lda >= Ka && ldg >= N && (!gmask || ldgm >= N), "%s: leading dimension too small", fn);
  // 16-B vector loads of 8-column groups
  TT_REQUIRE(lda % 4 == 0, "%s: lda must be a multiple of 4", fn);
  TT_REQUIRE(reinterpret_cast<uintptr_t>(A) % 16 == 0 && ldg % 4 == 0 && reinterpret_cast<uintptr_t>(G) % 16 == 0 &&
                 (!gmask || (ldgm % 4 == 0 && reinterpret_cast<uintptr_t>(gmask) % 16 == 0)),
             "%s: A / G / gmask rows must be 16-B aligned", fn);
  const int S = wgrad_splits(M, Ka, N);
  const int64_t rps = round_up(ceil_div(M > 0 ? M : 1, S), kWgBK);
  // per-split byte offsets are 32-bit (buffer loads)
  TT_REQUIRE(rps * std::max<int64_t>(lda, std::max<int64_t>(ldg, gmask ? ldgm : 0)) * 4 < (int64_t(1) << 31),
             "%s: a split's rows exceed 2 GiB", fn);
  a = WgradArgs{};
  a.A = A;
  a.lda = lda;
  a.G = G;
  a.ldg = ldg;
  a.gmask = gmask;
  a.ldgm = ldgm;
  a.scale = scale;
  a.M = M;
  a.Ka = Ka;
  a.N = N;
  a.TI = static_cast<int>(ceil_div(Ka + 1, kWgTile));
  a.TJ = static_cast<int>(ceil_div(N, kWgTile));
  a.S = S;
  a.rows_per_split = rps;
  return TT_OK;
}

static void launch_wgrad(const WgradArgs& a, hipStream_t st) {
  const dim3 grid(static_cast<unsigned>(a.S * a.TI * a.TJ));
  if (a.gmask) hipLaunchKernelGGL((mlp_wgrad_kernel<true>), grid, dim3(kWgThreads), 0, st, a);
  else hipLaunchKernelGGL((mlp_wgrad_kernel<false>), grid, dim3(kWgThreads), 0, st, a);
}

namespace {
int wgrad_one(const char* fn, const float* A, int64_t lda, const float* G, int64_t ldg, const float* gmask,
              int64_t ldgm, const float* scale, int64_t M, int32_t Ka, int32_t N, float* dwb, void* workspace,
              size_t workspace_bytes, tt_stream_t stream, const PartsAdagrad& ad) {
  WgradArgs a;
  const int rc = wgrad_setup(fn, A, lda, G, ldg, gmask, ldgm, scale, M, Ka, N, dwb, a);
  if (rc != TT_OK) return rc;
  TT_REQUIRE(workspace && workspace_bytes >= tt_mlp_wgrad_workspace_size(M, Ka, N), "%s: workspace %zu < %zu", fn,
             workspace_bytes, tt_mlp_wgrad_workspace_size(M, Ka, N));
  a.parts = static_cast<float*>(workspace);
  hipStream_t st = to_stream(stream);
  launch_wgrad(a, st);
  TT_CHECK_LAUNCH();
  const int64_t len = static_cast<int64_t>(Ka + 1) * N;
  hipLaunchKernelGGL(mlp_sum_parts_kernel, dim3(ceil_div(len, 256)), dim3(1024), 0, st, a.parts, a.S, len, dwb, ad);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
}  // namespace

extern "C" int tt_mlp_wgrad(const float* A, int64_t lda, const float* G, int64_t ldg, const float* gmask,
                            int64_t ldgm, const float* scale, int64_t M, int32_t Ka, int32_t N, float* dwb,
                            void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  return wgrad_one("tt_mlp_wgrad", A, lda, G, ldg, gmask, ldgm, scale, M, Ka, N, dwb, workspace, workspace_bytes,
                   stream, PartsAdagrad{});
}

extern "C" int tt_mlp_wgrad_adagrad(const float* A, int64_t lda, const float* G, int64_t ldg, const float* gmask,
                                    int64_t ldgm, const float* scale, int64_t M, int32_t Ka, int32_t N, float* dwb,
                                    float* param, float* accum, float lr, float epsilon, void* workspace,
                                    size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(param && accum, "tt_mlp_wgrad_adagrad: NULL param / accum");
  TT_REQUIRE(reinterpret_cast<uintptr_t>(param) % 16 == 0 && reinterpret_cast<uintptr_t>(accum) % 16 == 0,
             "tt_mlp_wgrad_adagrad: param / accum must be 16-B aligned");
  return wgrad_one("tt_mlp_wgrad_adagrad", A, lda, G, ldg, gmask, ldgm, scale, M, Ka, N, dwb, workspace,
                   workspace_bytes, stream, PartsAdagrad{param, accum, lr, epsilon});
}

// the second problem's partials start 256-B aligned after the first's
static size_t wgrad_pair_offset(const tt_mlp_wgrad_problem* p) {
  return static_cast<size_t>(round_up(static_cast<int64_t>(tt_mlp_wgrad_workspace_size(p[0].M, p[0].Ka, p[0].N)), 256));
}

extern "C" size_t tt_mlp_wgrad_pair_workspace_size(const tt_mlp_wgrad_problem* p) {
  if (!p) return 0;
  return wgrad_pair_offset(p) + tt_mlp_wgrad_workspace_size(p[1].M, p[1].Ka, p[1].N);
}

extern "C" int tt_mlp_wgrad_pair(const tt_mlp_wgrad_problem* p, void* workspace, size_t workspace_bytes,
                                 tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(p, "tt_mlp_wgrad_pair: NULL problems");
  WgradArgs a[2];
  for (int i = 0; i < 2; ++i) {
    const tt_mlp_wgrad_problem& q = p[i];
    const int rc = wgrad_setup("tt_mlp_wgrad_pair", q.A, q.lda, q.G, q.ldg, q.gmask, q.ldgm, q.scale, q.M, q.Ka, q.N,
                               q.dwb, a[i]);
    if (rc != TT_OK) return rc;
  }
  const size_t need = tt_mlp_wgrad_pair_workspace_size(p);
  TT_REQUIRE(workspace && workspace_bytes >= need, "tt_mlp_wgrad_pair: workspace %zu < %zu", workspace_bytes, need);
  a[0].parts = static_cast<float*>(workspace);
  a[1].parts = reinterpret_cast<float*>(static_cast<char*>(workspace) + wgrad_pair_offset(p));
  hipStream_t st = to_stream(stream);
  const int nb0 = a[0].S * a[0].TI * a[0].TJ, nb1 = a[1].S * a[1].TI * a[1].TJ;
  if ((a[0].gmask != nullptr) != (a[1].gmask != nullptr) || nb0 % 8 != 0) {
    launch_wgrad(a[0], st);
    launch_wgrad(a[1], st);
  } else {
    const dim3 grid(static_cast<unsigned>(nb0 + nb1));
    if (a[0].gmask) hipLaunchKernelGGL((mlp_wgrad_pair_kernel<true>), grid, dim3(kWgThreads), 0, st, a[0], a[1], nb0);
    else hipLaunchKernelGGL((mlp_wgrad_pair_kernel<false>), grid, dim3(kWgThreads), 0, st, a[0], a[1], nb0);
  }
  TT_CHECK_LAUNCH();
  const int64_t len0 = static_cast<int64_t>(a[0].Ka + 1) * a[0].N, len1 = static_cast<int64_t>(a[1].Ka + 1) * a[1].N;
  const int sb0 = static_cast<int>(ceil_div(len0, 256));
  hipLaunchKernelGGL(mlp_sum_parts_pair_kernel, dim3(static_cast<unsigned>(sb0 + ceil_div(len1, 256))), dim3(1024), 0,
                     st, a[0].parts, a[0].S, len0, p[0].dwb, a[1].parts, a[1].S, len1, p[1].dwb, sb0);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
