// K5+K6+K7: fused in-batch scores, logQ correction and softmax cross-entropy
// (reduction SUM) with its gradient, on bf16 MFMA (v_mfma_f32_32x32x16_bf16)
// with fp32 accumulation.  The [rows, cols] score matrix never leaves
// registers.
//
// Reference chain (/root/reference):
//   TwoTowerModel.call        S = Q C^T                  two_tower_model.py:92
//   LogQCorrection.__call__   S' = S - log p[cand]       logq_correction.py:66-71
//   eye labels + CE(from_logits, SUM)                    two_tower_model.py:119-122,
//                                                        runner.py:78-83
//   loss = sum_i [lse_i(S'_i.) - S'_ii];  dS = softmax(S') - I
//   dQ = dS C,  dC = dS^T Q
//
// Two streaming passes, each "flash"-structured over the other operand:
//   rows pass (F): per query row i, online softmax over all candidate columns
//     accumulating O_i = sum_j exp(S'_ij - m_i) c_j -> lse_i and
//     dq_i = O_i / l_i - c_pos(i)   (the forward IS attention with K = V = C).
//   cols pass (G): per candidate column j, with lse known,
//     dc_j = sum_i exp(S'_ij - lse_i) q_i - q_pos(j); the -logq_j shift is
//     applied as the exact factor exp(-logq_j) on the column sum.
// 4 B^2 E flops each (S recompute + P.V), i.e. 8 B^2 E per train step.
//
// Wave layout (32x32x16 bf16 MFMA, 64-wide wave): a wave owns 32 stationary
// rows whose bf16 fragments stay in VGPRs for the whole pass (B operand).
// Streamed rows arrive in 64-row tiles through a 4-stage LDS-DMA ring
// (XOR-swizzled so every ds_read_b128 fragment read is bank-conflict free):
//   S^T tile [32 streamed x 32 stationary] = A(streamed rows) . B(stationary)
// so each lane holds 16 scores of ONE stationary row; the per-row bias
// (-logq_j for F, -lse_i for G) is loaded as the accumulator's initial value.
// The S^T accumulator is exactly the B operand of the next MFMA
// (O^T += X^T . P^T) after a bf16 pack, so P never touches LDS; the streamed
// operand's transposed image X^T is prepared once in HBM with the MFMA's
// k-permutation baked in (16-byte fragment reads).
// The stationary extent is split into 128-row workgroups and the streamed
// extent into S splits (flash-decoding) so that >= 256 workgroups fill the
// 256 CUs; tiny combine kernels merge the splits.
#include <cmath>

#include "tt_common.h"

namespace tt {
namespace {

constexpr int kWavesPerWG = 4;
constexpr int kThreads = kWavesPerWG * kWave;
constexpr int kRowsPerWave = 32;
constexpr int kRowsPerWG = kWavesPerWG * kRowsPerWave;  // stationary rows per WG
constexpr int kTile = 64;                                // streamed rows per LDS tile
constexpr int kMaxSplit = 16;
constexpr int kRingStages = 4;                           // LDS tile ring depth
constexpr float kLog2e = 1.4426950408889634f;

template <int D>
struct Geo {
  static constexpr int KS = D / 16;           // MFMA k-steps over the embedding
  static constexpr int DT = D / 32;           // 32-row output tiles of O^T
  static constexpr int CH = D / 8;            // 16-byte chunks per bf16 row
  static constexpr int A_BYTES = kTile * D * 2;   // streamed rows, row-major
  static constexpr int T_BYTES = D * kTile * 2;   // transposed image [D][64]
  static constexpr int STAGE_BYTES = A_BYTES + T_BYTES + kTile * 4;  // + 64 biases
  static constexpr int LDS_BYTES = kRingStages * STAGE_BYTES;
  static constexpr int PPW = (A_BYTES / 1024) / 2;  // 1 KiB DMA pieces per wave
};

// Swizzled byte offset of 16-B chunk `ch` of row `row` in the [64][D] image.
template <int D>
__device__ __forceinline__ int a_off(int row, int ch) {
  constexpr int CH = D / 8;
  const int swz = (row * CH / 16) % CH;
  return row * (CH * 16) + ((ch ^ swz) << 4);
}
// Swizzled byte offset of 16-B chunk `ch` (0..7) of row `e` in the [D][64] image.
__device__ __forceinline__ int t_off(int e, int ch) { return e * 128 + ((ch ^ ((e >> 1) & 7)) << 4); }

// Position of streamed row offset o (0..15) inside its 16-row group of the
// transposed image: MFMA k element j of lane half h is row 8(j>>2)+4h+(j&3).
__device__ __forceinline__ int perm16(int o) {
  const int a = o >> 3, h = (o >> 2) & 1, b = o & 3;
  return 8 * h + 4 * a + b;
}

// ---------------------------------------------------------------------------
// Prep: fp32 [n, ld] -> bf16 row-major [n_pad, D] of scale * src (zero padded)
// and optionally the permuted transposed image [D, n_pad] of src (unscaled).
// One block = 64 rows.
template <int D>
__global__ void __launch_bounds__(256) prep_kernel(const float* __restrict__ src, int64_t ld, int64_t n,
                                                   int dim, int64_t n_pad, float scale, __bf16* __restrict__ dst,
                                                   __bf16* __restrict__ dstT) {
  __shared__ float tile[64][D + 1];
  const int64_t r0 = blockIdx.x * 64ll;
  for (int i = threadIdx.x; i < 64 * D; i += 256) {
    const int r = i / D, e = i % D;
    const int64_t gr = r0 + r;
    tile[r][e] = (gr < n && e < dim) ? src[gr * ld + e] : 0.0f;
  }
  __syncthreads();
  // row-major: each thread packs 8 consecutive elements (16 B).
  for (int i = threadIdx.x; i < 64 * D / 8; i += 256) {
    const int r = i / (D / 8), c8 = (i % (D / 8)) * 8;
    u32x4 v;
    v.x = pack_bf16x2(scale * tile[r][c8 + 0], scale * tile[r][c8 + 1]);
    v.y = pack_bf16x2(scale * tile[r][c8 + 2], scale * tile[r][c8 + 3]);
    v.z = pack_bf16x2(scale * tile[r][c8 + 4], scale * tile[r][c8 + 5]);
    v.w = pack_bf16x2(scale * tile[r][c8 + 6], scale * tile[r][c8 + 7]);
    *reinterpret_cast<u32x4*>(dst + (r0 + r) * D + c8) = v;
  }
  if (dstT) {
    // transposed: image row e holds the 64 rows of this block, permuted per 16.
    for (int i = threadIdx.x; i < D * 8; i += 256) {
      const int e = i / 8, p8 = (i % 8) * 8;  // positions p8..p8+7 within the 64
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = p8 + j;
        const int g = p >> 4, pp = p & 15;
        // inverse of perm16: position pp holds row offset o with perm16(o) == pp
        const int h = pp >> 3, a = (pp >> 2) & 1, b = pp & 3;
        const int o = 8 * a + 4 * h + b;
        x[j] = tile[16 * g + o][e];
      }
      u32x4 v;
      v.x = pack_bf16x2(x[0], x[1]);
      v.y = pack_bf16x2(x[2], x[3]);
      v.z = pack_bf16x2(x[4], x[5]);
      v.w = pack_bf16x2(x[6], x[7]);
      *reinterpret_cast<u32x4*>(dstT + static_cast<int64_t>(e) * n_pad + r0 + p8) = v;
    }
  }
}

// bias[i] = sign * v[i] (v may be NULL -> 0) for i < n; pad value beyond.
__global__ void bias_kernel(const float* __restrict__ v, int64_t n, int64_t n_pad, float sign, float pad,
                            float* __restrict__ out) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n_pad) return;
  out[i] = (i < n) ? (v ? sign * v[i] : 0.0f) : pad;
}

// bias1[i] = -log2(e) logq[i] (0 if logq NULL) for i < n, -inf for n <= i < n_pad;
// bias2[i] = -inf for n <= i < n_pad (its [0, n) is written by combine_rows).
__global__ void dual_bias_kernel(const float* __restrict__ logq, int64_t n, int64_t n_pad, float* __restrict__ bias1,
                                 float* __restrict__ bias2) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n_pad) return;
  bias1[i] = (i < n) ? (logq ? -kLog2e * logq[i] : 0.0f) : -INFINITY;
  if (i >= n) bias2[i] = -INFINITY;
}

struct PassArgs {
  const __bf16* stat;     // [n_stat_pad, D] stationary rows (B operand)
  const __bf16* strm;     // [n_strm_pad, D] streamed rows (A operand of S)
  const __bf16* strmT;    // [D, n_strm_pad] permuted transposed image
  const float* bias;      // [n_strm_pad] accumulator init per streamed row
  int64_t n_stat_pad;
  int64_t n_strm_pad;
  int64_t per_split;      // streamed rows per split (multiple of kTile)
  float* part_m;          // [S, n_stat_pad]   (rows pass)
  float* part_l;          // [S, n_stat_pad]   (rows pass)
  float* part_o;          // [S, n_stat_pad, D]
};

// ---------------------------------------------------------------------------
// The pass kernel (MODE 0: rows pass, online softmax; MODE 1: cols pass, lse
// known), software-pipelined so that the MFMA pipe never waits on the softmax:
//   iteration t:  [S(t+1) = A(t+1) . B  ||  p(t) = exp2(S(t)), bf16 pack]
//                 [O^T += X^T(t) . P^T(t) ||  l += sum p(t), max S(t+1)]
// i.e. the exp/pack work of tile t issues between the score MFMAs of tile
// t+1, and the row-sum / next max between the P.V MFMAs of tile t.
// Tiles arrive by LDS-DMA (buffer_load ... lds: zero VGPR staging, the tile
// offset is a scalar) into a 4-stage ring; one counted vmcnt + one s_barrier
// per tile.  Waves 0-1 fetch the row-major image, waves 2-3 the transposed
// one, wave 0 also the 64 biases.
// Scores are in log2 units: the row-major image of q is prepared scaled by
// log2(e) and the biases likewise, so p = exp2(s - m) is one subtract + one
// v_exp per score.  (The row sum stays an fp32 add chain: a v_dot2 over the
// packed weights miscompiles with this hipcc — it re-reads one source pair.)
// Rows pass: lazy rescaling — the running max m only moves when a tile's max
// exceeds it by more than 8 (log2 units), so p <= 2^8 and the 64-register O
// rescale leaves the steady state (m, l, O stay consistent: lse = m + log l).
constexpr float kLazyRescale = 8.0f;  // log2 units
constexpr float kLn2 = 0.6931471805599453f;

template <int N>
__device__ __forceinline__ void ib_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int D, int MODE>
__global__ void __launch_bounds__(kThreads) inbatch_pipe_kernel(const PassArgs a) {
  using G = Geo<D>;
  extern __shared__ __attribute__((aligned(16))) char ring[];
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  const int lane = lane_id();
  const int h = lane >> 5;
  const int l32 = lane & 31;
  const int64_t stat_row = static_cast<int64_t>(blockIdx.x) * kRowsPerWG + wave * kRowsPerWave + l32;
  const int split = blockIdx.y;
  const int64_t s_begin = split * a.per_split;
  int64_t s_end = s_begin + a.per_split;
  if (s_end > a.n_strm_pad) s_end = a.n_strm_pad;
  const int ntiles = s_begin < s_end ? static_cast<int>((s_end - s_begin) / kTile) : 0;

  bf16x8 bfrag[G::KS];
#pragma unroll
  for (int s = 0; s < G::KS; ++s)
    bfrag[s] = *reinterpret_cast<const bf16x8*>(a.stat + stat_row * D + 16 * s + 8 * h);

  // DMA plan of this wave: PPW pieces of the A image (waves 0-1) or of the
  // T image (waves 2-3); lane offsets are tile-invariant, the tile moves the
  // scalar offset only.  Swizzle applied on the source so pieces land
  // lane-linear in the XOR-swizzled layout.
  const bool is_t = wave >= 2;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      is_t ? (void*)a.strmT : (void*)a.strm, 0, static_cast<int>(a.n_strm_pad * D * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t brsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.bias, 0, static_cast<int>(a.n_strm_pad * 4), 0x00020000);
  unsigned voff[G::PPW];
#pragma unroll
  for (int u = 0; u < G::PPW; ++u) {
    const int p = (wave & 1) * G::PPW + u;
    const int off = p * 1024 + lane * 16;
    if (!is_t) {
      const int row = off / (D * 2), chp = (off % (D * 2)) / 16;
      const int ch = chp ^ ((row * G::CH / 16) % G::CH);
      voff[u] = static_cast<unsigned>(row * D * 2 + ch * 16);
    } else {
      const int e = off / 128, chp = (off % 128) / 16;
      const int ch = chp ^ ((e >> 1) & 7);
      voff[u] = static_cast<unsigned>(static_cast<int64_t>(e) * a.n_strm_pad * 2 + ch * 16);
    }
  }
  const int dst0 = (is_t ? G::A_BYTES : 0) + (wave & 1) * G::PPW * 1024;
  auto issue = [&](int tile) {
    const int64_t row0 = s_begin + static_cast<int64_t>(tile) * kTile;
    const unsigned soff = static_cast<unsigned>(is_t ? row0 * 2 : row0 * D * 2);
    char* st = ring + (tile % kRingStages) * G::STAGE_BYTES;
#pragma unroll
    for (int u = 0; u < G::PPW; ++u)
      // (the explicit copy of voff[u] is needed: passing the captured array
      // element itself drops the kernel's host-side stub with this hipcc)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(st + dst0 + u * 1024),
                                               16, static_cast<unsigned>(voff[u]), soff, 0, 0);
    if (wave == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (__attribute__((address_space(3))) void*)(st + G::A_BYTES + G::T_BYTES),
                                               4, lane * 4, static_cast<unsigned>(row0 * 4), 0, 0);
  };
  // Wait until at most `ahead` issued tiles of this wave are still in flight.
  auto wait_tiles = [&](int ahead) {
    if (wave == 0) {
      if (ahead >= 2) ib_wait_vmcnt<2 * (G::PPW + 1)>();
      else if (ahead == 1) ib_wait_vmcnt<G::PPW + 1>();
      else ib_wait_vmcnt<0>();
    } else {
      if (ahead >= 2) ib_wait_vmcnt<2 * G::PPW>();
      else if (ahead == 1) ib_wait_vmcnt<G::PPW>();
      else ib_wait_vmcnt<0>();
    }
  };

  f32x16 o[G::DT];
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.0f;
  float m_run = -1.0e30f;
  float l_run = 0.0f;

  auto scores = [&](int tile, f32x16* sacc) {
    const char* B = ring + (tile % kRingStages) * G::STAGE_BYTES;
    const float* bias = reinterpret_cast<const float*>(B + G::A_BYTES + G::T_BYTES);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias + 32 * t + 8 * r4 + 4 * h);
        sacc[t][4 * r4 + 0] = b4[0];
        sacc[t][4 * r4 + 1] = b4[1];
        sacc[t][4 * r4 + 2] = b4[2];
        sacc[t][4 * r4 + 3] = b4[3];
      }
#pragma unroll
    for (int s = 0; s < G::KS; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(B + a_off<D>(32 * t + l32, 2 * s + h));
        sacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfrag[s], sacc[t], 0, 0, 0);
      }
  };
  auto tile_max = [&](const f32x16* sacc) {
    float m0 = sacc[0][0], m1 = sacc[1][0];
#pragma unroll
    for (int r = 1; r < 16; r += 2) {
      m0 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m0, sacc[0][r]), sacc[0][r + 1 < 16 ? r + 1 : r]);
      m1 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m1, sacc[1][r]), sacc[1][r + 1 < 16 ? r + 1 : r]);
    }
    const float m = __builtin_elementwise_maximum(m0, m1);
    return __builtin_elementwise_maximum(m, __shfl_xor(m, 32, kWave));
  };

  const int pre = ntiles < kRingStages ? ntiles : kRingStages;
  for (int t = 0; t < pre; ++t) issue(t);
  f32x16 sa[2], sb[2];
  float mx = -INFINITY;
  if (ntiles > 0) {
    wait_tiles(pre - 1);  // tile 0 landed
    __builtin_amdgcn_s_barrier();
    scores(0, sa);
    if constexpr (MODE == 0) mx = tile_max(sa);
  }

  // One tile: sc holds S(tile) (log2 units), sn receives S(tile+1).
  auto step = [&](int tile, f32x16* sc, f32x16* sn) {
    if constexpr (MODE == 0) {
      if (__any(mx > m_run + kLazyRescale)) {
        const float m_new = __builtin_elementwise_maximum(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        l_run *= alpha;
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        m_run = m_new;
      }
    }
    if (tile == 0 && ntiles > 1) {
      // tile 1 must be resident before the first look-ahead scores
      wait_tiles(pre - 2);
      __builtin_amdgcn_s_barrier();
    }

    // Region A: next scores || exp + pack of this tile.  (After the last
    // tile the look-ahead reads a stale stage: harmless, never used.)
    scores(tile + 1, sn);
    const float mb = (MODE == 0) ? m_run : 0.0f;
    bf16x8 pf[4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] = __builtin_amdgcn_exp2f(sc[t][8 * s2 + j] - mb);
        u32x4 pk;
        pk.x = pack_bf16x2(p[0], p[1]);
        pk.y = pack_bf16x2(p[2], p[3]);
        pk.z = pack_bf16x2(p[4], p[5]);
        pk.w = pack_bf16x2(p[6], p[7]);
        pf[2 * t + s2] = __builtin_bit_cast(bf16x8, pk);
        if constexpr (MODE == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) l_run += p[j];
        }
      }

    // Region B: P.V of this tile || the next tile's max.
    const char* B = ring + (tile % kRingStages) * G::STAGE_BYTES;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) {
          const int e = 32 * dt + l32;
          const bf16x8 tf = *reinterpret_cast<const bf16x8*>(B + G::A_BYTES + t_off(e, 4 * t + 2 * s2 + h));
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tf, pf[2 * t + s2], o[dt], 0, 0, 0);
        }
    if constexpr (MODE == 0) mx = tile_max(sn);

    // Ring: tile+2 resident for the next step, this tile's stage free.
    if (tile + 2 < ntiles) {
      wait_tiles(tile + 3 < ntiles ? 1 : 0);
      __builtin_amdgcn_s_barrier();
      if (tile + kRingStages < ntiles) issue(tile + kRingStages);
    }
  };
  // Unrolled by two so the S(t) / S(t+1) register sets swap roles without copies.
  for (int tile = 0; tile < ntiles; tile += 2) {
    step(tile, sa, sb);
    if (tile + 1 < ntiles) step(tile + 1, sb, sa);
  }

  const int64_t prow = static_cast<int64_t>(split) * a.n_stat_pad + stat_row;
  if constexpr (MODE == 0) {
    const float l_tot = l_run + __shfl_xor(l_run, 32, kWave);
    if (h == 0) {
      a.part_m[prow] = m_run * kLn2;  // natural-log units for the combine
      a.part_l[prow] = l_tot;
    }
  }
  float* po = a.part_o + prow * D;
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      f32x4 v;
      v[0] = o[dt][4 * r4 + 0];
      v[1] = o[dt][4 * r4 + 1];
      v[2] = o[dt][4 * r4 + 2];
      v[3] = o[dt][4 * r4 + 3];
      *reinterpret_cast<f32x4*>(po + 32 * dt + 8 * r4 + 4 * h) = v;
    }
}

// Rows combine: one wave per row.  lse, row loss, dq.
__global__ void __launch_bounds__(256) combine_rows_kernel(
    const float* __restrict__ part_m, const float* __restrict__ part_l, const float* __restrict__ part_o,
    int nsplit, int64_t n_stat_pad, int D, const float* __restrict__ q, int64_t ldq, const float* __restrict__ c,
    int64_t ldc, const float* __restrict__ logq, int64_t n_rows, int dim, int64_t pos_offset,
    float* __restrict__ lse_out, float* __restrict__ loss_out, float* __restrict__ dq,
    float* __restrict__ neg_lse_bias) {
  const int64_t i = blockIdx.x * 4ll + threadIdx.x / kWave;
  if (i >= n_rows) return;
  const int lane = lane_id();
  float M = -1.0e30f;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, part_m[s * n_stat_pad + i]);
  float L = 0.0f;
  for (int s = 0; s < nsplit; ++s) L += part_l[s * n_stat_pad + i] * expf(part_m[s * n_stat_pad + i] - M);
  const float lse = M + logf(L);
  const int64_t pos = i + pos_offset;
  float dot = 0.0f;
  for (int e = lane; e < dim; e += kWave) {
    float oe = 0.0f;
    for (int s = 0; s < nsplit; ++s)
      oe += part_o[(s * n_stat_pad + i) * D + e] * expf(part_m[s * n_stat_pad + i] - M);
    const float ce = c[pos * ldc + e];
    if (dq) dq[i * dim + e] = oe / L - ce;
    dot = __builtin_fmaf(q[i * ldq + e], ce, dot);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) dot += __shfl_xor(dot, m, kWave);
  if (lane == 0) {
    const float pos_logit = dot - (logq ? logq[pos] : 0.0f);
    lse_out[i] = lse;
    loss_out[i] = lse - pos_logit;
    if (neg_lse_bias) neg_lse_bias[i] = -kLog2e * lse;
  }
}

// Cols combine: dc_j = exp(-logq_j) * sum_s O_s[j] - q_pos(j).
__global__ void __launch_bounds__(256) combine_cols_kernel(const float* __restrict__ part_o, int nsplit,
                                                           int64_t n_stat_pad, int D, const float* __restrict__ q,
                                                           int64_t ldq, const float* __restrict__ logq,
                                                           int64_t n_cols, int dim, int64_t pos_offset,
                                                           float* __restrict__ dc) {
  const int64_t j = blockIdx.x * 4ll + threadIdx.x / kWave;
  if (j >= n_cols) return;
  const int lane = lane_id();
  const float scale = logq ? expf(-logq[j]) : 1.0f;
  const int64_t pos = j + pos_offset;
  for (int e = lane; e < dim; e += kWave) {
    float oe = 0.0f;
    for (int s = 0; s < nsplit; ++s) oe += part_o[(s * n_stat_pad + j) * D + e];
    dc[j * dim + e] = oe * scale - q[pos * ldq + e];
  }
}

int pick_dpad(int dim) {
  if (dim <= 32) return 32;
  if (dim <= 64) return 64;
  if (dim <= 128) return 128;
  return 0;
}

#ifndef TT_INBATCH_WG_TARGET
#define TT_INBATCH_WG_TARGET 256
#endif
// Splits of the streamed extent so that the grid has >= TT_INBATCH_WG_TARGET
// workgroups (several per CU: two waves per SIMD hide each other's softmax).
int pick_split(int64_t n_stat_pad, int64_t n_strm_pad) {
  const int64_t wgs = n_stat_pad / kRowsPerWG;
  int64_t s = ceil_div(TT_INBATCH_WG_TARGET, wgs);
  const int64_t tiles = n_strm_pad / kTile;
  if (s > tiles) s = tiles;
  if (s > kMaxSplit) s = kMaxSplit;
  if (s < 1) s = 1;
  return static_cast<int>(s);
}

struct Plan {
  int D;
  int64_t stat_pad, strm_pad;
  int split;
  int64_t per_split;
};

Plan make_plan(int64_t n_stat, int64_t n_strm, int dim) {
  Plan p;
  p.D = pick_dpad(dim);
  p.stat_pad = round_up(n_stat > 0 ? n_stat : 1, kRowsPerWG);
  p.strm_pad = round_up(n_strm > 0 ? n_strm : 1, kTile);
  p.split = pick_split(p.stat_pad, p.strm_pad);
  p.per_split = round_up(ceil_div(p.strm_pad, p.split), kTile);
  return p;
}

struct PassWs {
  __bf16* stat;
  __bf16* strm;
  __bf16* strmT;
  float* bias;
  float* part_m;
  float* part_l;
  float* part_o;
};

PassWs carve_pass(Carver& cv, const Plan& p) {
  PassWs w;
  w.stat = cv.take<__bf16>(p.stat_pad * p.D);
  w.strm = cv.take<__bf16>(p.strm_pad * p.D);
  w.strmT = cv.take<__bf16>(p.strm_pad * p.D);
  w.bias = cv.take<float>(p.strm_pad);
  w.part_m = cv.take<float>(int64_t(p.split) * p.stat_pad);
  w.part_l = cv.take<float>(int64_t(p.split) * p.stat_pad);
  w.part_o = cv.take<float>(int64_t(p.split) * p.stat_pad * p.D);
  return w;
}

size_t pass_bytes(int64_t n_stat, int64_t n_strm, int dim) {
  Carver cv(nullptr, 0);
  carve_pass(cv, make_plan(n_stat, n_strm, dim));
  return cv.used();
}

template <int D>
int launch_prep(const float* src, int64_t ld, int64_t n, int dim, int64_t n_pad, float scale, __bf16* dst,
                __bf16* dstT, hipStream_t st) {
  hipLaunchKernelGGL(prep_kernel<D>, dim3(n_pad / 64), dim3(256), 0, st, src, ld, n, dim, n_pad, scale, dst, dstT);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

// scale applies to the row-major image only (log2(e) for q, 1 for c).
int prep(int D, const float* src, int64_t ld, int64_t n, int dim, int64_t n_pad, float scale, __bf16* dst,
         __bf16* dstT, hipStream_t st) {
  switch (D) {
    case 32: return launch_prep<32>(src, ld, n, dim, n_pad, scale, dst, dstT, st);
    case 64: return launch_prep<64>(src, ld, n, dim, n_pad, scale, dst, dstT, st);
    default: return launch_prep<128>(src, ld, n, dim, n_pad, scale, dst, dstT, st);
  }
}

template <int D, int MODE>
int launch_pass_d(dim3 grid, const PassArgs& a, hipStream_t st) {
  constexpr int shm = Geo<D>::LDS_BYTES;
  if (shm > 65536) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(inbatch_pipe_kernel<D, MODE>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, shm);
    TT_CHECK_HIP(attr);
  }
  hipLaunchKernelGGL((inbatch_pipe_kernel<D, MODE>), grid, dim3(kThreads), shm, st, a);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

template <int MODE>
int launch_pass(const Plan& p, const PassArgs& a, hipStream_t st) {
  // buffer descriptors address the bf16 images with 32-bit byte offsets
  if (p.strm_pad * p.D * 2 >= (1ll << 31))
    return fail(TT_ERR_UNSUPPORTED, "inbatch: %lld x %d streamed batch too large", (long long)p.strm_pad, p.D);
  dim3 grid(static_cast<unsigned>(p.stat_pad / kRowsPerWG), static_cast<unsigned>(p.split));
  switch (p.D) {
    case 32: return launch_pass_d<32, MODE>(grid, a, st);
    case 64: return launch_pass_d<64, MODE>(grid, a, st);
    default: return launch_pass_d<128, MODE>(grid, a, st);
  }
}

int check_common(const float* q, int64_t ldq, int64_t n_rows, const float* c, int64_t ldc, int64_t n_cols,
                 int32_t dim) {
  TT_REQUIRE(q && c, "inbatch: NULL q/c");
  TT_REQUIRE(n_rows >= 1 && n_cols >= 1, "inbatch: empty batch");
  TT_REQUIRE(n_rows < (1ll << 30) && n_cols < (1ll << 30), "inbatch: batch too large");
  TT_REQUIRE(dim >= 1, "inbatch: dim must be >= 1");
  if (pick_dpad(dim) == 0) return fail(TT_ERR_UNSUPPORTED, "inbatch: dim=%d > 128 not supported", dim);
  TT_REQUIRE(ldq >= dim && ldc >= dim, "inbatch: leading dimension smaller than dim");
  return TT_OK;
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" size_t tt_inbatch_workspace_size(int64_t n_rows, int64_t n_cols, int32_t dim) {
  if (n_rows < 1 || n_cols < 1 || pick_dpad(dim) == 0) return 0;
  const size_t a = pass_bytes(n_rows, n_cols, dim);
  const size_t b = pass_bytes(n_cols, n_rows, dim);
  return a > b ? a : b;
}

extern "C" int tt_inbatch_xent_rows(const float* q, int64_t ldq, int64_t n_rows, const float* c, int64_t ldc,
                                    int64_t n_cols, int32_t dim, const float* logq, int64_t pos_offset,
                                    float* lse, float* row_loss, float* dq, void* workspace,
                                    size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  int rc = check_common(q, ldq, n_rows, c, ldc, n_cols, dim);
  if (rc) return rc;
  TT_REQUIRE(lse && row_loss, "tt_inbatch_xent_rows: NULL lse/row_loss");
  TT_REQUIRE(pos_offset >= 0 && n_rows + pos_offset <= n_cols,
             "tt_inbatch_xent_rows: positives [pos_offset, pos_offset+n_rows) exceed n_cols");
  const Plan p = make_plan(n_rows, n_cols, dim);
  Carver cv(workspace, workspace_bytes);
  PassWs w = carve_pass(cv, p);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_inbatch_xent_rows: workspace %zu < required %zu", workspace_bytes, cv.used());
  hipStream_t st = to_stream(stream);
  if ((rc = prep(p.D, q, ldq, n_rows, dim, p.stat_pad, kLog2e, w.stat, nullptr, st))) return rc;
  if ((rc = prep(p.D, c, ldc, n_cols, dim, p.strm_pad, 1.0f, w.strm, w.strmT, st))) return rc;
  hipLaunchKernelGGL(bias_kernel, dim3(ceil_div(p.strm_pad, 256)), dim3(256), 0, st, logq, n_cols, p.strm_pad,
                     -kLog2e, -INFINITY, w.bias);
  TT_CHECK_LAUNCH();
  PassArgs a{w.stat, w.strm, w.strmT, w.bias, p.stat_pad, p.strm_pad, p.per_split, w.part_m, w.part_l, w.part_o};
  if ((rc = launch_pass<0>(p, a, st))) return rc;
  hipLaunchKernelGGL(combine_rows_kernel, dim3(ceil_div(n_rows, 4)), dim3(256), 0, st, w.part_m, w.part_l,
                     w.part_o, p.split, p.stat_pad, p.D, q, ldq, c, ldc, logq, n_rows, dim, pos_offset, lse,
                     row_loss, dq, nullptr);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_inbatch_xent_cols(const float* q, int64_t ldq, int64_t n_rows, const float* lse, const float* c,
                                    int64_t ldc, int64_t n_cols, int32_t dim, const float* logq,
                                    int64_t pos_offset, float* dc, void* workspace, size_t workspace_bytes,
                                    tt_stream_t stream) {
  clear_error();
  int rc = check_common(q, ldq, n_rows, c, ldc, n_cols, dim);
  if (rc) return rc;
  TT_REQUIRE(lse && dc, "tt_inbatch_xent_cols: NULL lse/dc");
  TT_REQUIRE(pos_offset >= 0 && n_cols + pos_offset <= n_rows,
             "tt_inbatch_xent_cols: positives [pos_offset, pos_offset+n_cols) exceed n_rows");
  const Plan p = make_plan(n_cols, n_rows, dim);  // stationary = columns, streamed = rows
  Carver cv(workspace, workspace_bytes);
  PassWs w = carve_pass(cv, p);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_inbatch_xent_cols: workspace %zu < required %zu", workspace_bytes, cv.used());
  hipStream_t st = to_stream(stream);
  if ((rc = prep(p.D, c, ldc, n_cols, dim, p.stat_pad, 1.0f, w.stat, nullptr, st))) return rc;
  if ((rc = prep(p.D, q, ldq, n_rows, dim, p.strm_pad, kLog2e, w.strm, w.strmT, st))) return rc;
  hipLaunchKernelGGL(bias_kernel, dim3(ceil_div(p.strm_pad, 256)), dim3(256), 0, st, lse, n_rows, p.strm_pad,
                     -kLog2e, -INFINITY, w.bias);
  TT_CHECK_LAUNCH();
  PassArgs a{w.stat, w.strm, w.strmT, w.bias, p.stat_pad, p.strm_pad, p.per_split, nullptr, nullptr, w.part_o};
  if ((rc = launch_pass<1>(p, a, st))) return rc;
  hipLaunchKernelGGL(combine_cols_kernel, dim3(ceil_div(n_cols, 4)), dim3(256), 0, st, w.part_o, p.split,
                     p.stat_pad, p.D, q, ldq, logq, n_cols, dim, pos_offset, dc);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

// ---------------------------------------------------------------------------
// Single-device fused loss: rows and cols passes share one bf16 preparation of
// q and c (row-major + transposed images), the cols pass's -lse bias is
// written by the rows combine.  7 launches in total.
namespace tt {
namespace {
struct FusedWs {
  __bf16 *qb, *qbT, *cb, *cbT;
  float *bias_logq, *bias_lse;
  float *part_m, *part_l, *part_o_rows, *part_o_cols;
};
struct FusedPlan {
  int D;
  int64_t n_pad;
  int split;
  int64_t per_split;
};
FusedPlan fused_plan(int64_t n, int dim) {
  FusedPlan p;
  p.D = pick_dpad(dim);
  p.n_pad = round_up(n > 0 ? n : 1, kRowsPerWG);  // multiple of both 128 and 64
  p.split = pick_split(p.n_pad, p.n_pad);
  p.per_split = round_up(ceil_div(p.n_pad, p.split), kTile);
  return p;
}
FusedWs carve_fused(Carver& cv, const FusedPlan& p) {
  FusedWs w;
  w.qb = cv.take<__bf16>(p.n_pad * p.D);
  w.qbT = cv.take<__bf16>(p.n_pad * p.D);
  w.cb = cv.take<__bf16>(p.n_pad * p.D);
  w.cbT = cv.take<__bf16>(p.n_pad * p.D);
  w.bias_logq = cv.take<float>(p.n_pad);
  w.bias_lse = cv.take<float>(p.n_pad);
  w.part_m = cv.take<float>(int64_t(p.split) * p.n_pad);
  w.part_l = cv.take<float>(int64_t(p.split) * p.n_pad);
  w.part_o_rows = cv.take<float>(int64_t(p.split) * p.n_pad * p.D);
  w.part_o_cols = cv.take<float>(int64_t(p.split) * p.n_pad * p.D);
  return w;
}
}  // namespace
}  // namespace tt

extern "C" size_t tt_inbatch_fused_workspace_size(int64_t n, int32_t dim) {
  if (n < 1 || pick_dpad(dim) == 0) return 0;
  Carver cv(nullptr, 0);
  carve_fused(cv, fused_plan(n, dim));
  return cv.used();
}

extern "C" int tt_inbatch_softmax_xent(const float* q, int64_t ldq, const float* c, int64_t ldc, int64_t n,
                                       int32_t dim, const float* logq, float* lse, float* row_loss, float* dq,
                                       float* dc, void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  int rc = check_common(q, ldq, n, c, ldc, n, dim);
  if (rc) return rc;
  TT_REQUIRE(lse && row_loss && dq && dc, "tt_inbatch_softmax_xent: NULL output");
  const FusedPlan p = fused_plan(n, dim);
  Carver cv(workspace, workspace_bytes);
  FusedWs w = carve_fused(cv, p);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_inbatch_softmax_xent: workspace %zu < required %zu", workspace_bytes,
                cv.used());
  hipStream_t st = to_stream(stream);
  if ((rc = prep(p.D, q, ldq, n, dim, p.n_pad, kLog2e, w.qb, w.qbT, st))) return rc;
  if ((rc = prep(p.D, c, ldc, n, dim, p.n_pad, 1.0f, w.cb, w.cbT, st))) return rc;
  hipLaunchKernelGGL(dual_bias_kernel, dim3(ceil_div(p.n_pad, 256)), dim3(256), 0, st, logq, n, p.n_pad, w.bias_logq,
                     w.bias_lse);
  TT_CHECK_LAUNCH();
  const Plan pl{p.D, p.n_pad, p.n_pad, p.split, p.per_split};
  PassArgs ar{w.qb, w.cb, w.cbT, w.bias_logq, p.n_pad, p.n_pad, p.per_split, w.part_m, w.part_l, w.part_o_rows};
  if ((rc = launch_pass<0>(pl, ar, st))) return rc;
  hipLaunchKernelGGL(combine_rows_kernel, dim3(ceil_div(n, 4)), dim3(256), 0, st, w.part_m, w.part_l, w.part_o_rows,
                     p.split, p.n_pad, p.D, q, ldq, c, ldc, logq, n, dim, (int64_t)0, lse, row_loss, dq, w.bias_lse);
  TT_CHECK_LAUNCH();
  PassArgs ac{w.cb, w.qb, w.qbT, w.bias_lse, p.n_pad, p.n_pad, p.per_split, nullptr, nullptr, w.part_o_cols};
  if ((rc = launch_pass<1>(pl, ac, st))) return rc;
  hipLaunchKernelGGL(combine_cols_kernel, dim3(ceil_div(n, 4)), dim3(256), 0, st, w.part_o_cols, p.split, p.n_pad,
                     p.D, q, ldq, logq, n, dim, (int64_t)0, dc);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
