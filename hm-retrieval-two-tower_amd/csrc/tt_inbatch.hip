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
// Streamed rows arrive in 64-row tiles, by LDS-DMA, into a 4-stage ring of
// ONE row-major image per tile, read two ways:
//   S^T tile [32 streamed x 32 stationary] = A(streamed rows) . B(stationary)
//     with row reads (ds_read_b128), so each lane holds 16 scores of ONE
//     stationary row; the per-row bias (-logq_j for F, -lse_i for G) is the
//     accumulator's initial value;
//   O^T [E x 32 stationary] += X^T . P^T, where the S^T accumulator packed to
//     bf16 IS the B operand P^T (P never touches LDS) and X^T comes from the
//     same image through the hardware transposing read ds_read_b64_tr_b16.
// The image's XOR swizzle keeps both kinds of read bank-conflict free.
// The stationary extent is split into 128-row workgroups and the streamed
// extent into S splits (flash-decoding) so that >= 256 workgroups fill the
// 256 CUs; small combine kernels merge the splits.  (Merging them inside the
// passes instead — write-through partials, the last of a block's S
// workgroups merging them — measured 10-30 us per step slower: the merging
// workgroups' dependent reads form a serial tail of the pass.)
#include <cmath>
#include <cstdlib>
#include <type_traits>

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
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kLazyRescale = 8.0f;  // log2 units

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int D>
struct Geo {
  static constexpr int KS = D / 16;                        // MFMA k-steps over the embedding
  static constexpr int DT = D / 32;                        // 32-row output tiles of O^T
  static constexpr int CH = D / 8;                         // 16-byte chunks per bf16 row
  static constexpr int A_BYTES = kTile * D * 2;            // one tile image = one ring stage
  static constexpr int BIAS_OFF = kRingStages * A_BYTES;   // then kRingStages x 64 biases
  static constexpr int LDS_BYTES = BIAS_OFF + kRingStages * kTile * 4;
  static constexpr int PPW = A_BYTES / 1024 / kWavesPerWG; // 1 KiB DMA pieces per wave per tile
};

// Byte offset of 16-B chunk ch of tile row `row` (rows of 2D bytes).  The XOR
// swizzle makes both the 16-lane ds_read_b128 groups of the row reads (rows
// {0-3,12-15,20-27}, one chunk) and the 32-lane halves of the transposed reads
// (4 consecutive rows x 4 aligned chunks) hit 64 distinct banks.
template <int D>
__device__ __forceinline__ int a_off(int row, int ch) {
  int f;
  if constexpr (D == 128) f = ((row & 3) << 2) | ((row >> 2) & 3);
  else if constexpr (D == 64) f = (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
  else f = (row >> 2) & 3;
  return row * (D * 2) + ((ch ^ f) << 4);
}

// ---------------------------------------------------------------------------
// Prep: fp32 [n, ld] -> bf16 [n_pad, D] (zero padded), optionally with the
// pass's per-row bias vector: bias[i] = sign * bv[i] (0 if bv NULL) for i < n
// and -inf for padded rows; bias2 (if set) gets -inf on padded rows (its
// [0, n) is written later by combine_rows).  One launch preps up to two
// matrices (blockIdx.y); one block = 32 rows, 8 elements per thread.
struct PrepJob {
  const float* src;
  int64_t ld;
  int64_t n;
  __bf16* dst;
  const float* bv;
  float sign;
  float* bias;
  float* bias2;
  int vec;  // src 16-B aligned, ld % 4 == 0, dim % 4 == 0: float4 loads
  __bf16* dst_lo;  // x3 mode: also the residual plane bf16(x - bf16(x)) (NULL: none)
};

template <int D>
__global__ void __launch_bounds__(256) prep_kernel(PrepJob j0, PrepJob j1, int dim) {
  const PrepJob& j = blockIdx.y ? j1 : j0;
  const int64_t r0 = blockIdx.x * 32ll;
  constexpr int TPR = D / 8;  // threads per row
  for (int i = threadIdx.x; i < 32 * TPR; i += 256) {
    const int64_t r = r0 + i / TPR;
    const int c8 = (i % TPR) * 8;
    float x[8];
    if (r < j.n && j.vec) {
      const float* row = j.src + r * j.ld + c8;
      const f32x4 lo = c8 < dim ? *reinterpret_cast<const f32x4*>(row) : f32x4{0, 0, 0, 0};
      const f32x4 hi = c8 + 4 < dim ? *reinterpret_cast<const f32x4*>(row + 4) : f32x4{0, 0, 0, 0};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        x[u] = lo[u];
        x[4 + u] = hi[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = (r < j.n && c8 + u < dim) ? j.src[r * j.ld + c8 + u] : 0.0f;
    }
    u32x4 v;
    v.x = pack_bf16x2(x[0], x[1]);
    v.y = pack_bf16x2(x[2], x[3]);
    v.z = pack_bf16x2(x[4], x[5]);
    v.w = pack_bf16x2(x[6], x[7]);
    *reinterpret_cast<u32x4*>(j.dst + r * D + c8) = v;
    if (j.dst_lo) {  // x = hi + lo + O(2^-16 |x|): the bf16x3 products' operands
      float e[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) e[u] = x[u] - static_cast<float>(static_cast<__bf16>(x[u]));
      u32x4 w;
      w.x = pack_bf16x2(e[0], e[1]);
      w.y = pack_bf16x2(e[2], e[3]);
      w.z = pack_bf16x2(e[4], e[5]);
      w.w = pack_bf16x2(e[6], e[7]);
      *reinterpret_cast<u32x4*>(j.dst_lo + r * D + c8) = w;
    }
  }
  if (j.bias && threadIdx.x < 32) {
    const int64_t r = r0 + threadIdx.x;
    j.bias[r] = (r < j.n) ? (j.bv ? j.sign * j.bv[r] : 0.0f) : -INFINITY;
    if (j.bias2 && r >= j.n) j.bias2[r] = -INFINITY;
  }
}

struct PassArgs {
  const __bf16* stat;     // [n_stat_pad, D] stationary rows (B operand)
  const __bf16* strm;     // [n_strm_pad, D] streamed rows
  const float* bias;      // [n_strm_pad] accumulator init per streamed row
  int64_t n_stat_pad;
  int64_t n_strm_pad;
  int64_t per_split;      // streamed rows per split (multiple of kTile)
  int64_t diag_off;       // stationary row r's positive is streamed row r + diag_off (excluded from the sums)
  float* part_m;          // [S, n_stat_pad]   (rows pass; log2 units, integer valued)
  float* part_l;          // [S, n_stat_pad]   (rows pass)
  float* part_o;          // [S, n_stat_pad, D]
  const __bf16* stat_lo;  // x3 mode: residual planes of the stationary / streamed rows
  const __bf16* strm_lo;
};

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Raw buffer descriptor (stride 0, byte-range checked) from wave-uniform values.
__device__ __forceinline__ i32x4 buffer_desc(const void* base, unsigned bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  i32x4 d;
  d.x = __builtin_amdgcn_readfirstlane(static_cast<int>(b & 0xffffffffu));
  d.y = __builtin_amdgcn_readfirstlane(static_cast<int>((b >> 32) & 0xffffu));
  d.z = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  d.w = 0x00020000;
  return d;
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return static_cast<unsigned>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char*)p));
}

// LDS-DMA (buffer_load ... lds, 64 lanes x 16 B or x 4 B at LDS address lds)
// in inline asm: the compiler then does not track these LDS writes, and so
// does not put an s_waitcnt vmcnt(0) in front of every ds_read_b64_tr_b16 (it
// does for the builtin form).  Ordering against the reads is the explicit
// counted vmcnt + s_barrier of the tile ring.
__device__ __forceinline__ void dma_b128(i32x4 desc, unsigned voff, unsigned soff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               :
               : "v"(voff), "s"(desc), "s"(soff), "s"(lds)
               : "memory");  // m0 is compiler-reserved and unused by this kernel otherwise
}
__device__ __forceinline__ void dma_b32(i32x4 desc, unsigned voff, unsigned soff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %0, %1, %2 offen lds"
               :
               : "v"(voff), "s"(desc), "s"(soff), "s"(lds)
               : "memory");  // m0 is compiler-reserved and unused by this kernel otherwise
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// ---------------------------------------------------------------------------
// The pass kernel.  MODE 0: rows pass (online softmax).  MODE 1: cols pass
// (lse known: p = exp(S + bias) directly).
//
// Software pipeline, per tile t (one wave, 32 stationary rows):
//   region A: the 2*KS score MFMAs of tile t+1 (look-ahead)  ||  exp2 + bf16
//             pack of tile t's scores (the VALU fills the MFMA gaps);
//   region B: the 4*DT P.V MFMAs of tile t  ||  row sums of tile t and the
//             max of tile t+1 (rows pass).
// Every MFMA step issues the fragment read AHEAD steps later, then its MFMA,
// then its share of the VALU; __builtin_amdgcn_sched_barrier(0) pins that
// order (left alone, the scheduler keeps one or two reads in flight and waits
// lgkmcnt(0) before most MFMAs).  Unrolled by the ring period (4): the S(t) /
// S(t+1) register sets swap roles without copies and all LDS offsets fold.
// Tiles arrive by buffer_load ... lds (no VGPR staging; the tile offset is a
// scalar soffset) into the ring; one counted vmcnt + one s_barrier per tile.
// Rows pass: lazy rescaling — the running max m only moves when a tile's max
// exceeds it by more than 8 (log2 units), so p <= 2^8 and the 64-register O
// rescale leaves the steady state (m, l, O stay consistent: lse = m + log l).
// Two workgroups per CU (<= 256 registers per lane): the second hides the
// first's barrier and DMA waits.  At one per CU (the mask_diag of the
// contract commit in its 64-bit form needed 302) the passes ran 25 % slower.
//
// X3 (opt-in, tt_inbatch_softmax_xent_x3): fp32-faithful products — S and
// P.V both from bf16x3 products hi.hi + hi.lo + lo.hi of split operands (x =
// hi + lo, both bf16; P split the same way in registers), three MFMAs where
// the default issues one; the streamed rows' lo image has a ring of its own
// (LDS 129 KB at D = 128: one workgroup per CU).
template <int D, int MODE, bool X3 = false>
__global__ void __launch_bounds__(kThreads, X3 ? 1 : 2) inbatch_pass_kernel(const PassArgs a) {
  using G = Geo<D>;
  constexpr int IMG = X3 ? 2 : 1;                           // bf16 images per streamed tile
  constexpr int LO_OFF = kRingStages * G::A_BYTES;          // the lo ring (X3)
  constexpr int BIAS_OFF = IMG * kRingStages * G::A_BYTES;
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
  bf16x8 bfrag_lo[X3 ? G::KS : 1];
  if constexpr (X3) {
#pragma unroll
    for (int s = 0; s < G::KS; ++s)
      bfrag_lo[s] = *reinterpret_cast<const bf16x8*>(a.stat_lo + stat_row * D + 16 * s + 8 * h);
  }

  // DMA plan: every wave moves PPW 1 KiB pieces of each tile image, wave 0
  // also the 64 biases.  Per-lane source offsets are tile-invariant (the
  // swizzle is applied on the source so pieces land lane-linear).
  const i32x4 desc = buffer_desc(a.strm, static_cast<unsigned>(a.n_strm_pad * D * 2));
  const i32x4 bdesc = buffer_desc(a.bias, static_cast<unsigned>(a.n_strm_pad * 4));
  const i32x4 ldesc = buffer_desc(X3 ? a.strm_lo : a.strm, static_cast<unsigned>(a.n_strm_pad * D * 2));
  unsigned voff[G::PPW];
#pragma unroll
  for (int u = 0; u < G::PPW; ++u) {
    const int off = (wave * G::PPW + u) * 1024 + lane * 16;
    const int row = off / (D * 2), chp = (off % (D * 2)) / 16;
    // chunk ch lands in slot chp of its row iff a_off(row, ch) == row*2D + 16*chp
    const int ch = (a_off<D>(row, chp) - row * (D * 2)) >> 4;  // the swizzle is an involution
    voff[u] = static_cast<unsigned>(row * D * 2 + ch * 16);
  }
  const unsigned ring_lds = lds_addr(ring);
  auto issue = [&](int tile) {
    const unsigned row0 = static_cast<unsigned>(s_begin + static_cast<int64_t>(tile) * kTile);
    const int stage = tile % kRingStages;
    const unsigned st = ring_lds + stage * G::A_BYTES;
#pragma unroll
    for (int u = 0; u < G::PPW; ++u) dma_b128(desc, voff[u], row0 * (D * 2), st + (wave * G::PPW + u) * 1024);
    if constexpr (X3) {
#pragma unroll
      for (int u = 0; u < G::PPW; ++u)
        dma_b128(ldesc, voff[u], row0 * (D * 2), st + LO_OFF + (wave * G::PPW + u) * 1024);
    }
    if (wave == 0) dma_b32(bdesc, lane * 4, row0 * 4, ring_lds + BIAS_OFF + stage * (kTile * 4));
  };
  // Wait until at most `ahead` issued tiles of this wave are still in flight.
  auto wait_tiles = [&](int ahead) {
    if (wave == 0) {
      if (ahead >= 2) wait_vmcnt<2 * (IMG * G::PPW + 1)>();
      else if (ahead == 1) wait_vmcnt<IMG * G::PPW + 1>();
      else wait_vmcnt<0>();
    } else {
      if (ahead >= 2) wait_vmcnt<2 * IMG * G::PPW>();
      else if (ahead == 1) wait_vmcnt<IMG * G::PPW>();
      else wait_vmcnt<0>();
    }
  };

  f32x16 o[G::DT];
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.0f;
  float m_run = -1.0e30f;  // log2 units, integer valued
  float l_run = 0.0f;

  // Fragment reads.  Score step i: k-step i >> 1, sub-tile i & 1.
  // P.V step j = (2 t + s2) DT + dt: X^T rows e = 32 dt + l32, k = streamed
  // rows 32t + 16s2 + 8(k>>2) + 4h + (k&3) — the S^T accumulator's row order,
  // gathered by two transposing reads of 4 rows x 16 columns per lane group.
  // Every read is a per-lane base (the swizzle depends only on the low row
  // bits) plus a compile-time offset (stage, sub-tile, row group): no address
  // arithmetic in the loop.
  int rbase[G::KS];        // row reads: a_off(l32, 2s + h)
  int tbase[G::DT][2];     // transposed reads: rows 4h + tq + 8u, chunk 4dt + 2tg + tp/2
  {
    const int tq = (lane & 15) >> 2, tp = lane & 3, tg = (lane >> 4) & 1;
#pragma unroll
    for (int s = 0; s < G::KS; ++s) rbase[s] = a_off<D>(l32, 2 * s + h);
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        tbase[dt][u] = a_off<D>(4 * h + tq + 8 * u, 4 * dt + 2 * tg + (tp >> 1)) + 8 * (tp & 1);
  }
  auto rd_a = [&](int stage, int i) {
    return *reinterpret_cast<const bf16x8*>(ring + rbase[i >> 1] + (stage * G::A_BYTES + (i & 1) * 32 * 2 * D));
  };
  auto rd_a_lo = [&](int stage, int i) {  // X3: the same fragment of the lo image
    return *reinterpret_cast<const bf16x8*>(ring + rbase[i >> 1] +
                                            (LO_OFF + stage * G::A_BYTES + (i & 1) * 32 * 2 * D));
  };
  auto rd_t = [&](int stage, int j) {
    const int dt = j % G::DT, g = j / G::DT;  // g = 2t + s2
    typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
    const int roff = stage * G::A_BYTES + 16 * g * 2 * D;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(ring + tbase[dt][0] + roff));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(ring + tbase[dt][1] + roff));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto rd_t_lo = [&](int stage, int j) {  // X3: the same transposed read of the lo image
    const int dt = j % G::DT, g = j / G::DT;
    typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
    const int roff = LO_OFF + stage * G::A_BYTES + 16 * g * 2 * D;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(ring + tbase[dt][0] + roff));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(ring + tbase[dt][1] + roff));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto rd_bias = [&](int stage, f32x16* sacc) {
    const float* bias = reinterpret_cast<const float*>(ring + BIAS_OFF + stage * (kTile * 4)) + 4 * h;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias + 32 * t + 8 * r4);
#pragma unroll
        for (int u = 0; u < 4; ++u) sacc[t][4 * r4 + u] = b4[u];
      }
  };

  auto scores_plain = [&](f32x16* sacc) {  // prologue: tile 0, stage 0
    rd_bias(0, sacc);
#pragma unroll
    for (int i = 0; i < 2 * G::KS; ++i) {
      const bf16x8 ah = rd_a(0, i);
      sacc[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bfrag[i >> 1], sacc[i & 1], 0, 0, 0);
      if constexpr (X3) {
        sacc[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bfrag_lo[i >> 1], sacc[i & 1], 0, 0, 0);
        sacc[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rd_a_lo(0, i), bfrag[i >> 1], sacc[i & 1], 0, 0, 0);
      }
    }
  };
  auto half_max = [&](const f32x16* sacc) {
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < 32; k += 2)
      m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m, sacc[k >> 4][k & 15]),
                                        sacc[(k + 1) >> 4][(k + 1) & 15]);
    return __builtin_elementwise_maximum(m, __shfl_xor(m, 32, kWave));
  };

  // The positive pair is left out of the MFMA sums (the combines add it in
  // fp32, exactly): in a tile holding some of this wave's positives (at most
  // two tiles per wave and split; a wave-uniform test) its score becomes -inf,
  // so p = 0.  Score k of a lane is streamed row 32(k>>4) + 8((k&15)>>2) + 4h + (k&3).
  const int64_t wave_row0 = static_cast<int64_t>(blockIdx.x) * kRowsPerWG + wave * kRowsPerWave;
  // (the test is on wave-uniform scalars; a lane holds its positive in at
  // most one register, found from the row's digits: no 64-bit lane math)
  // The tiles [td_lo, td_hi] of the split that hold them (empty: td_lo > td_hi).
  const int64_t dlo = wave_row0 + a.diag_off - s_begin;  // first positive, as a column of the split
  const int64_t dhi = dlo + kRowsPerWave - 1, send = static_cast<int64_t>(ntiles) * kTile;
  const bool dnone = dhi < 0 || dlo >= send;
  const int td_lo = dnone ? 1 : static_cast<int>(max(dlo, int64_t{0}) / kTile);
  const int td_hi = dnone ? 0 : static_cast<int>(min(dhi, send - 1) / kTile);
  auto mask_diag = [&](f32x16* sacc, int tile) {
    if (tile < td_lo || tile > td_hi) return;
    const int64_t lo = dlo - static_cast<int64_t>(tile) * kTile;
    const int d = static_cast<int>(lo) + l32;  // this lane's positive, as a row of the tile
    const bool mine = d >= 0 && d < kTile && ((d >> 2) & 1) == h;
    const int kd = mine ? 16 * (d >> 5) + 4 * ((d >> 3) & 3) + (d & 3) : -1;  // its register
#pragma unroll
    for (int k = 0; k < 32; ++k)
      sacc[k >> 4][k & 15] = kd == k ? -INFINITY : sacc[k >> 4][k & 15];
  };

  const int pre = ntiles < kRingStages ? ntiles : kRingStages;
  for (int t = 0; t < pre; ++t) issue(t);
  f32x16 sa[2], sb[2];
  float mx = -INFINITY;  // max of the scores waiting in sc (rows pass)
  if (ntiles > 0) {
    wait_tiles(pre - 1);  // tile 0 landed
    __builtin_amdgcn_s_barrier();
    scores_plain(sa);
    mask_diag(sa, 0);
    if constexpr (MODE == 0) mx = half_max(sa);
  }

  constexpr int NS = 2 * G::KS;  // score steps per tile (one MFMA each; three in X3)
  constexpr int NSR = IMG * NS;  // score fragment reads per tile (X3: hi and lo)
  constexpr int NP = 4 * G::DT;  // P.V MFMAs per tile
#ifndef TT_IB_AHEAD
#define TT_IB_AHEAD 3
#endif
  constexpr int AHEAD = TT_IB_AHEAD;  // fragment reads in flight
  constexpr int EPS = 32 / NS;   // scores exponentiated per score step
  constexpr int EPP = 32 / NP;   // row-sum terms per P.V step
  constexpr int MX0 = NP / 2;    // P.V steps from which the next max runs
  constexpr int EMX = 32 / (NP - MX0);

  // One tile: sc holds S(tile), sn receives S(tile+1); STG = tile % 4.
  auto step = [&](auto stg, int tile, f32x16* sc, f32x16* sn) {
    constexpr int STG = decltype(stg)::value;
    constexpr int NXT = (STG + 1) % kRingStages;
    if constexpr (MODE == 0) {
      // m_run: an integer in log2 units, so every rescale factor is an exact
      // power of two and bf16(p) does not depend on when m moved
      const float mx2 = mx * kLog2e;
      if (__any(mx2 > m_run + kLazyRescale)) {
        const float m_new = __builtin_ceilf(__builtin_elementwise_maximum(m_run, mx2));
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
    // (after the last tile the look-ahead reads a stale stage: harmless, unused)
    constexpr int FR = AHEAD + IMG;  // fragment ring: X3 consumes two reads per score step
    bf16x8 fr[FR];
    auto prefetch = [&](int idx) {  // idx over the tile's NSR + IMG * NP fragment reads
      if (idx < NSR) {
        if constexpr (X3) fr[idx % FR] = (idx & 1) ? rd_a_lo(NXT, idx >> 1) : rd_a(NXT, idx >> 1);
        else fr[idx % FR] = rd_a(NXT, idx);
      } else if (idx < NSR + IMG * NP) {
        const int k = idx - NSR;
        if constexpr (X3) fr[idx % FR] = (k & 1) ? rd_t_lo(STG, k >> 1) : rd_t(STG, k >> 1);
        else fr[idx % FR] = rd_t(STG, k);
      }
    };
    rd_bias(NXT, sn);
#pragma unroll
    for (int i = 0; i < AHEAD; ++i) prefetch(i);
    const float mb = (MODE == 0) ? m_run : 0.0f;
    bf16x8 pf[4];
    bf16x8 pf_lo[X3 ? 4 : 1];  // X3: P's residual plane (P.V as bf16x3 too)
    __builtin_amdgcn_sched_barrier(0);

    // Region A: S(tile+1) MFMAs || p = exp2(s log2e - m log2e), bf16 pack.
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      prefetch(IMG * i + AHEAD);
      if constexpr (X3) prefetch(IMG * i + 1 + AHEAD);
      sn[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[(IMG * i) % FR], bfrag[i >> 1], sn[i & 1], 0, 0, 0);
      if constexpr (X3) {
        sn[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[(IMG * i) % FR], bfrag_lo[i >> 1], sn[i & 1], 0, 0, 0);
        sn[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[(IMG * i + 1) % FR], bfrag[i >> 1], sn[i & 1], 0, 0, 0);
      }
#pragma unroll
      for (int k = i * EPS; k < (i + 1) * EPS; ++k) {
        sc[k >> 4][k & 15] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[k >> 4][k & 15], kLog2e, -mb));
        if ((k & 7) == 7) {
          const int g = k >> 3, t = g >> 1, b = 8 * (g & 1);
          u32x4 pk;
          pk.x = pack_bf16x2(sc[t][b + 0], sc[t][b + 1]);
          pk.y = pack_bf16x2(sc[t][b + 2], sc[t][b + 3]);
          pk.z = pack_bf16x2(sc[t][b + 4], sc[t][b + 5]);
          pk.w = pack_bf16x2(sc[t][b + 6], sc[t][b + 7]);
          pf[g] = __builtin_bit_cast(bf16x8, pk);
          if constexpr (X3) {
            float e[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) e[u] = sc[t][b + u] - static_cast<float>(static_cast<__bf16>(sc[t][b + u]));
            u32x4 pl;
            pl.x = pack_bf16x2(e[0], e[1]);
            pl.y = pack_bf16x2(e[2], e[3]);
            pl.z = pack_bf16x2(e[4], e[5]);
            pl.w = pack_bf16x2(e[6], e[7]);
            pf_lo[g] = __builtin_bit_cast(bf16x8, pl);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // Region B: O^T += X^T . P^T of this tile || row sums, next tile's max.
    float mxa = -INFINITY;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      prefetch(NSR + IMG * j + AHEAD);
      if constexpr (X3) prefetch(NSR + IMG * j + 1 + AHEAD);
      o[j % G::DT] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[(NSR + IMG * j) % FR], pf[j / G::DT], o[j % G::DT],
                                                              0, 0, 0);
      if constexpr (X3) {
        o[j % G::DT] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[(NSR + IMG * j) % FR], pf_lo[j / G::DT],
                                                                o[j % G::DT], 0, 0, 0);
        o[j % G::DT] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[(NSR + IMG * j + 1) % FR], pf[j / G::DT],
                                                                o[j % G::DT], 0, 0, 0);
      }
      // S(tile+1)'s positives out, half way through: its MFMAs have landed
      // by now (masked right after region A the wave waited for them: +4 %
      // per pass), and the next max below reads them after
      if (j == MX0) mask_diag(sn, tile + 1);
      if constexpr (MODE == 0) {
#pragma unroll
        for (int k = j * EPP; k < (j + 1) * EPP; ++k) l_run += sc[k >> 4][k & 15];
        asm volatile("" : "+v"(l_run));  // keep the adds here (else sunk past the loop)
        if (j >= MX0) {
#pragma unroll
          for (int k = (j - MX0) * EMX; k < (j - MX0 + 1) * EMX; k += 2)
            mxa = __builtin_elementwise_maximum(__builtin_elementwise_maximum(mxa, sn[k >> 4][k & 15]),
                                                sn[(k + 1) >> 4][(k + 1) & 15]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (MODE == 0) mx = __builtin_elementwise_maximum(mxa, __shfl_xor(mxa, 32, kWave));

    // Ring: tile+2 resident for the next step, this tile's stage free.
    if (tile + 2 < ntiles) {
#ifndef TT_IB_PROBE_NOVMWAIT
      wait_tiles(tile + 3 < ntiles ? 1 : 0);
#endif
#ifndef TT_IB_PROBE_NOBARRIER
      __builtin_amdgcn_s_barrier();
#endif
      if (tile + kRingStages < ntiles) issue(tile + kRingStages);
    }
  };
  // Unrolled by the ring period: every LDS offset is a compile-time constant.
  for (int tile = 0; tile < ntiles; tile += 4) {
    step(std::integral_constant<int, 0>(), tile, sa, sb);
    if (tile + 1 < ntiles) step(std::integral_constant<int, 1>(), tile + 1, sb, sa);
    if (tile + 2 < ntiles) step(std::integral_constant<int, 2>(), tile + 2, sa, sb);
    if (tile + 3 < ntiles) step(std::integral_constant<int, 3>(), tile + 3, sb, sa);
  }

  const int64_t prow = static_cast<int64_t>(split) * a.n_stat_pad + stat_row;
  if constexpr (MODE == 0) {
    const float l_tot = l_run + __shfl_xor(l_run, 32, kWave);
    if (h == 0) {
      a.part_m[prow] = m_run;
      a.part_l[prow] = l_tot;
    }
  }
  float* po = a.part_o + prow * D;
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      f32x4 v;
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = o[dt][4 * r4 + u];
      *reinterpret_cast<f32x4*>(po + 32 * dt + 8 * r4 + 4 * h) = v;
    }
}

// Split combines: D/4 lanes per row (float4 partials), 1024/D rows per block.
//
// The passes leave the positive pair out of their sums; the combines add it
// in fp32 from the fp32 operands.  Rows: with the off-diagonal partials
// merged to (M, L, O) (M in log2 units), a = M ln2 + log L = lse over the
// negatives and pos = q_i . c_pos - logq_pos:
//   row loss  = softplus(a - pos)            (= lse - pos, without cancellation)
//   lse       = pos + row loss
//   dq        = sigmoid(a - pos) (O / L - c_pos)
// (1 - P_pos = sigmoid(a - pos) and P_ij = sigmoid(a - pos) p_ij / L, so
// dq = sum_j P_ij c_j - (1 - P_pos) c_pos: a mean of the negatives' rows minus
// the positive's, weighted by the exact 1 - P_pos, with no P - I cancellation.)
__device__ __forceinline__ float softplus_f(float x) {
  return x > 0.0f ? x + log1pf(expf(-x)) : log1pf(expf(x));
}

template <int D>
__device__ __forceinline__ void combine_row_finish(int64_t i, int sub, float M, float L, const f32x4& o,
                                                   const float (&ce)[4], const float (&qe)[4], float lq, int dim,
                                                   float* __restrict__ lse_out, float* __restrict__ loss_out,
                                                   float* __restrict__ dq, float* __restrict__ neg_lse_bias) {
  constexpr int LPR = D / 4;
  float dot = 0.0f;
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (4 * sub + u < dim) dot = __builtin_fmaf(qe[u], ce[u], dot);
#pragma unroll
  for (int m = LPR / 2; m >= 1; m >>= 1) dot += __shfl_xor(dot, m, LPR);
  const float pos = dot - lq;
  // no negative with p > 0 (a single column, or every other score -inf): P_pos = 1
  const bool none = !(L > 0.0f);
  const float a = none ? -INFINITY : M * kLn2 + logf(L);
  const float loss = none ? 0.0f : softplus_f(a - pos);
  const float g = none ? 0.0f : 1.0f / (1.0f + expf(pos - a));  // sigmoid(a - pos) = 1 - P_pos
  const float inv = none ? 0.0f : 1.0f / L;
  if (dq) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = 4 * sub + u;
      if (e < dim) dq[i * dim + e] = g * (o[u] * inv - ce[u]);
    }
  }
  if (sub == 0) {
    const float lse = pos + loss;
    lse_out[i] = lse;
    loss_out[i] = loss;
    if (neg_lse_bias) neg_lse_bias[i] = -lse;
  }
}

template <int D>
__global__ void __launch_bounds__(256) combine_rows_kernel(
    const float* __restrict__ part_m, const float* __restrict__ part_l, const float* __restrict__ part_o,
    int nsplit, int64_t n_stat_pad, const float* __restrict__ q, int64_t ldq, const float* __restrict__ c,
    int64_t ldc, const float* __restrict__ logq, int64_t n_rows, int dim, int64_t pos_offset,
    float* __restrict__ lse_out, float* __restrict__ loss_out, float* __restrict__ dq,
    float* __restrict__ neg_lse_bias) {
  constexpr int LPR = D / 4;  // lanes per row
  const int64_t i = blockIdx.x * (256ll / LPR) + threadIdx.x / LPR;
  const int sub = threadIdx.x % LPR;
  if (i >= n_rows) return;
  const int64_t pos = i + pos_offset;
  // the positive's operands, loaded with the partials (one round of loads
  // when nsplit <= 4; columns past dim read a clamped one and are dropped)
  float ce[4], qe[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = min(4 * sub + u, dim - 1);
    ce[u] = c[pos * ldc + e];
    qe[u] = q[i * ldq + e];
  }
  const float lq = logq ? logq[pos] : 0.0f;
  // splits in groups of 4 whose loads are all issued before any is used
  // (index clamped, weight 0 past nsplit); splits added in order.  The split
  // maxima are integers in log2 units: every weight is an exact power of two.
  float M = -1.0e30f;
  if (nsplit <= 4) {  // one pass: M from the same loads
    float m[4], l[4];
    f32x4 ps[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t sr = min(u, nsplit - 1) * n_stat_pad + i;
      m[u] = part_m[sr];
      l[u] = part_l[sr];
      ps[u] = *reinterpret_cast<const f32x4*>(part_o + sr * D + 4 * sub);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) M = fmaxf(M, m[u]);
    float L = 0.0f;
    f32x4 o = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u < nsplit) {
        const float w = exp2f(m[u] - M);
        L += l[u] * w;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] += ps[u][e] * w;
      }
    }
    combine_row_finish<D>(i, sub, M, L, o, ce, qe, lq, dim, lse_out, loss_out, dq, neg_lse_bias);
    return;
  }
  for (int s0 = 0; s0 < nsplit; s0 += 4) {
    float m[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) m[u] = part_m[min(s0 + u, nsplit - 1) * n_stat_pad + i];
#pragma unroll
    for (int u = 0; u < 4; ++u) M = fmaxf(M, m[u]);
  }
  float L = 0.0f;
  f32x4 o = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int s0 = 0; s0 < nsplit; s0 += 4) {
    float m[4], l[4];
    f32x4 ps[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t sr = min(s0 + u, nsplit - 1) * n_stat_pad + i;
      m[u] = part_m[sr];
      l[u] = part_l[sr];
      ps[u] = *reinterpret_cast<const f32x4*>(part_o + sr * D + 4 * sub);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (s0 + u < nsplit) {
        const float w = exp2f(m[u] - M);
        L += l[u] * w;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] += ps[u][e] * w;
      }
    }
  }
  combine_row_finish<D>(i, sub, M, L, o, ce, qe, lq, dim, lse_out, loss_out, dq, neg_lse_bias);
}

// Cols: dc_j = exp(-logq_j) * sum_s O_s[j] - (1 - P_pos) q_pos, the pass's
// sums holding every row but the positive i = j + pos_offset, and
// 1 - P_pos = -expm1(-row_loss_i) (exact; from lse_i when row_loss is NULL:
// -expm1(pos - lse_i), pos = q_i . c_j - logq_j).
// The loss = scale * sum(row_loss) by one 256-thread block in exactly
// tt_sum's order (its 1024 threads' strided sums and LDS tree, 4 virtual
// threads per thread), so the value is bit-identical to a tt_sum launch.
struct LossSum {
  const float* x;  // NULL: no loss block
  int64_t n;
  float scale;
  float* out;
};

__device__ __forceinline__ void loss_sum_block(const LossSum& L) {
  __shared__ float red[1024];
  for (int v = threadIdx.x; v < 1024; v += 256) {
    float acc = 0.0f;
    int64_t i = v;
    for (; i + 3 * 1024 < L.n; i += 4 * 1024) {
      const float a = L.x[i], b = L.x[i + 1024], c = L.x[i + 2048], d = L.x[i + 3072];
      acc = ((acc + a) + b) + c;
      acc = acc + d;
    }
    for (; i < L.n; i += 1024) acc += L.x[i];
    red[v] = acc;
  }
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    for (int v = threadIdx.x; v < w; v += 256) red[v] += red[v + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) L.out[0] = red[0] * L.scale;
}

template <int D>
__global__ void __launch_bounds__(256) combine_cols_kernel(const float* __restrict__ part_o, int nsplit,
                                                           int64_t n_stat_pad, const float* __restrict__ q,
                                                           int64_t ldq, const float* __restrict__ c, int64_t ldc,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ row_loss,
                                                           const float* __restrict__ logq, int64_t n_cols, int dim,
                                                           int64_t pos_offset, float* __restrict__ dc,
                                                           const LossSum loss) {
  if (loss.x && blockIdx.x == gridDim.x - 1) {  // the extra last block: the loss (row_loss is complete)
    loss_sum_block(loss);
    return;
  }
  constexpr int LPR = D / 4;
  const int64_t j = blockIdx.x * (256ll / LPR) + threadIdx.x / LPR;
  const int sub = threadIdx.x % LPR;
  if (j >= n_cols) return;
  const float lq = logq ? logq[j] : 0.0f;
  const float scale = logq ? expf(-lq) : 1.0f;
  const int64_t pos = j + pos_offset;
  float qe[4];  // q_pos, loaded with the first partials (clamped past dim, dropped)
#pragma unroll
  for (int u = 0; u < 4; ++u) qe[u] = q[pos * ldq + min(4 * sub + u, dim - 1)];
  float omp;  // 1 - P_pos
  if (row_loss) {
    omp = -expm1f(-row_loss[pos]);
  } else {
    float dot = 0.0f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (4 * sub + u < dim) dot = __builtin_fmaf(qe[u], c[j * ldc + 4 * sub + u], dot);
#pragma unroll
    for (int m = LPR / 2; m >= 1; m >>= 1) dot += __shfl_xor(dot, m, LPR);
    omp = -expm1f(fminf(dot - lq - lse[pos], 0.0f));
  }
  f32x4 o = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int s0 = 0; s0 < nsplit; s0 += 4) {  // 4 splits' loads in flight, added in order
    f32x4 ps[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      ps[u] = *reinterpret_cast<const f32x4*>(part_o + (min(s0 + u, nsplit - 1) * n_stat_pad + j) * D + 4 * sub);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (s0 + u < nsplit) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] += ps[u][e];
      }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = 4 * sub + u;
    if (e < dim) dc[j * dim + e] = o[u] * scale - omp * qe[u];
  }
}

int pick_dpad(int dim) {
  if (dim <= 32) return 32;
  if (dim <= 64) return 64;
  if (dim <= 128) return 128;
  return 0;
}

// Splits of the streamed extent so that the grid has >= 512 workgroups: two
// rounds over the 256 CUs (the pass holds 426 registers per lane, so one
// workgroup per CU).  At the C3 batch (B = 16384, 128 stationary blocks)
// S = 4 beat S = 2 — one round, fewer split partials — by 19-24 us per train
// step (same box, 3 interleaved pairs; rows pass 116 vs 129 us, cols 104 vs
// 118 us: the second round evens out the workgroups' finishing times).
// TT_INBATCH_WGS overrides the target.
int wg_target() {
  static const int v = [] {
    const char* e = std::getenv("TT_INBATCH_WGS");
    const int x = e ? std::atoi(e) : 0;
    return x > 0 ? x : 512;
  }();
  return v;
}
int pick_split(int64_t n_stat_pad, int64_t n_strm_pad) {
  const int64_t wgs = n_stat_pad / kRowsPerWG;
  int64_t s = ceil_div(wg_target(), wgs);
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
  float* bias;
  float* part_m;
  float* part_l;
  float* part_o;
};

PassWs carve_pass(Carver& cv, const Plan& p) {
  PassWs w;
  w.stat = cv.take<__bf16>(p.stat_pad * p.D);
  w.strm = cv.take<__bf16>(p.strm_pad * p.D);
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

PrepJob prep_job(const float* src, int64_t ld, int64_t n, int dim, __bf16* dst, const float* bv = nullptr,
                 float* bias = nullptr, float* bias2 = nullptr) {
  const int vec = (reinterpret_cast<uintptr_t>(src) % 16 == 0 && ld % 4 == 0 && dim % 4 == 0) ? 1 : 0;
  return PrepJob{src, ld, n, dst, bv, -1.0f, bias, bias2, vec};
}

// Preps one or two matrices padded to n_pad rows (j1.src == NULL: one).
int prep(int D, const PrepJob& j0, const PrepJob& j1, int dim, int64_t n_pad, hipStream_t st) {
  const dim3 grid(static_cast<unsigned>(n_pad / 32), j1.src ? 2u : 1u);
  switch (D) {
    case 32: hipLaunchKernelGGL(prep_kernel<32>, grid, dim3(256), 0, st, j0, j1, dim); break;
    case 64: hipLaunchKernelGGL(prep_kernel<64>, grid, dim3(256), 0, st, j0, j1, dim); break;
    default: hipLaunchKernelGGL(prep_kernel<128>, grid, dim3(256), 0, st, j0, j1, dim); break;
  }
  TT_CHECK_LAUNCH();
  return TT_OK;
}

template <int D>
void launch_combine_rows(dim3 grid, hipStream_t st, const float* pm, const float* pl, const float* po, int nsplit,
                         int64_t n_stat_pad, const float* q, int64_t ldq, const float* c, int64_t ldc,
                         const float* logq, int64_t n, int dim, int64_t pos_offset, float* lse, float* loss,
                         float* dq, float* neg_lse) {
  hipLaunchKernelGGL(combine_rows_kernel<D>, grid, dim3(256), 0, st, pm, pl, po, nsplit, n_stat_pad, q, ldq, c, ldc,
                     logq, n, dim, pos_offset, lse, loss, dq, neg_lse);
}

int combine_rows(int D, hipStream_t st, const float* pm, const float* pl, const float* po, int nsplit,
                 int64_t n_stat_pad, const float* q, int64_t ldq, const float* c, int64_t ldc, const float* logq,
                 int64_t n, int dim, int64_t pos_offset, float* lse, float* loss, float* dq, float* neg_lse) {
  const dim3 grid(static_cast<unsigned>(ceil_div(n, 1024 / D)));
  switch (D) {
    case 32: launch_combine_rows<32>(grid, st, pm, pl, po, nsplit, n_stat_pad, q, ldq, c, ldc, logq, n, dim,
                                     pos_offset, lse, loss, dq, neg_lse); break;
    case 64: launch_combine_rows<64>(grid, st, pm, pl, po, nsplit, n_stat_pad, q, ldq, c, ldc, logq, n, dim,
                                     pos_offset, lse, loss, dq, neg_lse); break;
    default: launch_combine_rows<128>(grid, st, pm, pl, po, nsplit, n_stat_pad, q, ldq, c, ldc, logq, n, dim,
                                      pos_offset, lse, loss, dq, neg_lse); break;
  }
  TT_CHECK_LAUNCH();
  return TT_OK;
}

int combine_cols(int D, hipStream_t st, const float* po, int nsplit, int64_t n_stat_pad, const float* q,
                 int64_t ldq, const float* c, int64_t ldc, const float* lse, const float* row_loss,
                 const float* logq, int64_t n, int dim, int64_t pos_offset, float* dc,
                 const LossSum& loss = LossSum{}) {
  const dim3 grid(static_cast<unsigned>(ceil_div(n, 1024 / D) + (loss.x ? 1 : 0)));
  switch (D) {
    case 32: hipLaunchKernelGGL(combine_cols_kernel<32>, grid, dim3(256), 0, st, po, nsplit, n_stat_pad, q, ldq, c,
                                ldc, lse, row_loss, logq, n, dim, pos_offset, dc, loss); break;
    case 64: hipLaunchKernelGGL(combine_cols_kernel<64>, grid, dim3(256), 0, st, po, nsplit, n_stat_pad, q, ldq, c,
                                ldc, lse, row_loss, logq, n, dim, pos_offset, dc, loss); break;
    default: hipLaunchKernelGGL(combine_cols_kernel<128>, grid, dim3(256), 0, st, po, nsplit, n_stat_pad, q, ldq, c,
                                ldc, lse, row_loss, logq, n, dim, pos_offset, dc, loss); break;
  }
  TT_CHECK_LAUNCH();
  return TT_OK;
}

template <int D, int MODE, bool X3>
int launch_pass_d(dim3 grid, const PassArgs& a, hipStream_t st) {
  constexpr int shm = Geo<D>::LDS_BYTES + (X3 ? kRingStages * Geo<D>::A_BYTES : 0);
  if (shm > 65536) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(inbatch_pass_kernel<D, MODE, X3>), hipFuncAttributeMaxDynamicSharedMemorySize, shm);
    TT_CHECK_HIP(attr);
  }
  const int probe = MODE == 0 ? TT_PROBE_INBATCH_ROWS : TT_PROBE_INBATCH_COLS;
  const int reps = probe_reps(probe);  // > 1 only for a repeat probe (the pass is idempotent)
  probe_begin(probe, st);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((inbatch_pass_kernel<D, MODE, X3>), grid, dim3(kThreads), shm, st, a);
  probe_end(MODE == 0 ? TT_PROBE_INBATCH_ROWS : TT_PROBE_INBATCH_COLS, st);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

template <int MODE, bool X3 = false>
int launch_pass(const Plan& p, const PassArgs& a, hipStream_t st) {
  // buffer descriptors address the bf16 images with 32-bit byte offsets
  if (p.strm_pad * p.D * 2 >= (1ll << 31))
    return fail(TT_ERR_UNSUPPORTED, "inbatch: %lld x %d streamed batch too large", (long long)p.strm_pad, p.D);
  dim3 grid(static_cast<unsigned>(p.stat_pad / kRowsPerWG), static_cast<unsigned>(p.split));
  switch (p.D) {
    case 32: return launch_pass_d<32, MODE, X3>(grid, a, st);
    case 64: return launch_pass_d<64, MODE, X3>(grid, a, st);
    default: return launch_pass_d<128, MODE, X3>(grid, a, st);
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
  const PrepJob none{};
  if ((rc = prep(p.D, prep_job(q, ldq, n_rows, dim, w.stat), none, dim, p.stat_pad, st))) return rc;
  if ((rc = prep(p.D, prep_job(c, ldc, n_cols, dim, w.strm, logq, w.bias), none, dim, p.strm_pad, st))) return rc;
  PassArgs a{w.stat, w.strm, w.bias, p.stat_pad, p.strm_pad, p.per_split, pos_offset, w.part_m, w.part_l, w.part_o};
  if ((rc = launch_pass<0>(p, a, st))) return rc;
  return combine_rows(p.D, st, w.part_m, w.part_l, w.part_o, p.split, p.stat_pad, q, ldq, c, ldc, logq, n_rows, dim,
                      pos_offset, lse, row_loss, dq, nullptr);
}

extern "C" int tt_inbatch_xent_cols(const float* q, int64_t ldq, int64_t n_rows, const float* lse,
                                    const float* row_loss, const float* c, int64_t ldc, int64_t n_cols, int32_t dim,
                                    const float* logq, int64_t pos_offset, float* dc, void* workspace,
                                    size_t workspace_bytes, tt_stream_t stream) {
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
  const PrepJob none{};
  if ((rc = prep(p.D, prep_job(c, ldc, n_cols, dim, w.stat), none, dim, p.stat_pad, st))) return rc;
  if ((rc = prep(p.D, prep_job(q, ldq, n_rows, dim, w.strm, lse, w.bias), none, dim, p.strm_pad, st))) return rc;
  PassArgs a{w.stat, w.strm, w.bias, p.stat_pad, p.strm_pad, p.per_split, pos_offset, nullptr, nullptr, w.part_o};
  if ((rc = launch_pass<1>(p, a, st))) return rc;
  return combine_cols(p.D, st, w.part_o, p.split, p.stat_pad, q, ldq, c, ldc, lse, row_loss, logq, n_cols, dim,
                      pos_offset, dc);
}

// ---------------------------------------------------------------------------
// Single-device fused loss: rows and cols passes share one bf16 preparation of
// q and c (one row-major image each), the cols pass's -lse bias is
// written by the rows combine.  5 launches in total.
namespace tt {
namespace {
struct FusedWs {
  __bf16 *qb, *cb;
  __bf16 *qb_lo, *cb_lo;  // x3 mode only
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
FusedWs carve_fused(Carver& cv, const FusedPlan& p, bool x3 = false) {
  FusedWs w;
  w.qb = cv.take<__bf16>(p.n_pad * p.D);
  w.cb = cv.take<__bf16>(p.n_pad * p.D);
  w.qb_lo = x3 ? cv.take<__bf16>(p.n_pad * p.D) : nullptr;
  w.cb_lo = x3 ? cv.take<__bf16>(p.n_pad * p.D) : nullptr;
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

namespace tt {
namespace {
// The fused entry's body; prepped: the bf16 copies and bias vectors are
// already in the workspace (tt_inbatch_prep of q and of c on the same
// workspace, ordered before this call).
int softmax_xent(const float* q, int64_t ldq, const float* c, int64_t ldc, int64_t n, int32_t dim, const float* logq,
                 float* lse, float* row_loss, float* dq, float* dc, void* workspace, size_t workspace_bytes,
                 tt_stream_t stream, bool prepped, float loss_scale = 1.0f, float* loss = nullptr, bool x3 = false) {
  int rc = check_common(q, ldq, n, c, ldc, n, dim);
  if (rc) return rc;
  TT_REQUIRE(lse && row_loss && dq && dc, "tt_inbatch_softmax_xent: NULL output");
  const FusedPlan p = fused_plan(n, dim);
  Carver cv(workspace, workspace_bytes);
  FusedWs w = carve_fused(cv, p, x3);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_inbatch_softmax_xent: workspace %zu < required %zu", workspace_bytes,
                cv.used());
  hipStream_t st = to_stream(stream);
  // one prep launch for both matrices; c's job also writes both bias vectors
  PrepJob jq = prep_job(q, ldq, n, dim, w.qb), jc = prep_job(c, ldc, n, dim, w.cb, logq, w.bias_logq, w.bias_lse);
  jq.dst_lo = w.qb_lo;
  jc.dst_lo = w.cb_lo;
  if (!prepped && (rc = prep(p.D, jq, jc, dim, p.n_pad, st))) return rc;
  const Plan pl{p.D, p.n_pad, p.n_pad, p.split, p.per_split};
  PassArgs ar{w.qb, w.cb, w.bias_logq, p.n_pad, p.n_pad, p.per_split, 0, w.part_m, w.part_l, w.part_o_rows,
              w.qb_lo, w.cb_lo};
  if ((rc = x3 ? launch_pass<0, true>(pl, ar, st) : launch_pass<0>(pl, ar, st))) return rc;
  if ((rc = combine_rows(p.D, st, w.part_m, w.part_l, w.part_o_rows, p.split, p.n_pad, q, ldq, c, ldc, logq, n, dim,
                         0, lse, row_loss, dq, w.bias_lse)))
    return rc;
  PassArgs ac{w.cb, w.qb, w.bias_lse, p.n_pad, p.n_pad, p.per_split, 0, nullptr, nullptr, w.part_o_cols,
              w.cb_lo, w.qb_lo};
  if ((rc = x3 ? launch_pass<1, true>(pl, ac, st) : launch_pass<1>(pl, ac, st))) return rc;
  return combine_cols(p.D, st, w.part_o_cols, p.split, p.n_pad, q, ldq, c, ldc, lse, row_loss, logq, n, dim, 0, dc,
                      loss ? LossSum{row_loss, n, loss_scale, loss} : LossSum{});
}
}  // namespace
}  // namespace tt

extern "C" int tt_inbatch_softmax_xent(const float* q, int64_t ldq, const float* c, int64_t ldc, int64_t n,
                                       int32_t dim, const float* logq, float* lse, float* row_loss, float* dq,
                                       float* dc, void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  using namespace tt;
  clear_error();
  return softmax_xent(q, ldq, c, ldc, n, dim, logq, lse, row_loss, dq, dc, workspace, workspace_bytes, stream, false);
}

extern "C" int tt_inbatch_softmax_xent_prepped(const float* q, int64_t ldq, const float* c, int64_t ldc, int64_t n,
                                               int32_t dim, const float* logq, float* lse, float* row_loss,
                                               float* dq, float* dc, void* workspace, size_t workspace_bytes,
                                               tt_stream_t stream) {
  using namespace tt;
  clear_error();
  return softmax_xent(q, ldq, c, ldc, n, dim, logq, lse, row_loss, dq, dc, workspace, workspace_bytes, stream, true);
}

extern "C" int tt_inbatch_softmax_xent_loss(const float* q, int64_t ldq, const float* c, int64_t ldc, int64_t n,
                                            int32_t dim, const float* logq, float* lse, float* row_loss, float* dq,
                                            float* dc, float loss_scale, float* loss, int32_t prepped,
                                            void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  using namespace tt;
  clear_error();
  TT_REQUIRE(loss, "tt_inbatch_softmax_xent_loss: NULL loss");
  return softmax_xent(q, ldq, c, ldc, n, dim, logq, lse, row_loss, dq, dc, workspace, workspace_bytes, stream,
                      prepped != 0, loss_scale, loss);
}

extern "C" int tt_inbatch_prep(const float* x, int64_t ldx, int64_t n, int32_t dim, int32_t operand,
                               const float* logq, void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  using namespace tt;
  clear_error();
  int rc = check_common(x, ldx, n, x, ldx, n, dim);
  if (rc) return rc;
  TT_REQUIRE(operand == 0 || operand == 1, "tt_inbatch_prep: operand %d is not 0 (q) or 1 (c)", operand);
  const FusedPlan p = fused_plan(n, dim);
  Carver cv(workspace, workspace_bytes);
  FusedWs w = carve_fused(cv, p);
  if (!workspace || cv.used() > workspace_bytes)
    return fail(TT_ERR_WORKSPACE, "tt_inbatch_prep: workspace %zu < required %zu", workspace_bytes, cv.used());
  const PrepJob none{};
  return prep(p.D, operand == 0 ? prep_job(x, ldx, n, dim, w.qb) : prep_job(x, ldx, n, dim, w.cb, logq, w.bias_logq,
                                                                              w.bias_lse),
              none, dim, p.n_pad, to_stream(stream));
}

// Opt-in fp32-faithful products (X3): the fused loss with S = Q.C^T and the
// softmax-weighted sums P.V both from bf16x3 products (hi.hi + hi.lo + lo.hi
// of split operands) in both passes — the reference's fp32 logits and
// gradients to ~2^-16 relative, so softmax weights at trained score
// magnitudes (|S| ~ 100) keep their fp32 values.  Three MFMAs where the
// default issues one, one workgroup per CU: ~3x the passes' time.
extern "C" size_t tt_inbatch_fused_x3_workspace_size(int64_t n, int32_t dim) {
  if (n < 1 || pick_dpad(dim) == 0) return 0;
  Carver cv(nullptr, 0);
  carve_fused(cv, fused_plan(n, dim), true);
  return cv.used();
}

extern "C" int tt_inbatch_softmax_xent_x3(const float* q, int64_t ldq, const float* c, int64_t ldc, int64_t n,
                                          int32_t dim, const float* logq, float* lse, float* row_loss, float* dq,
                                          float* dc, float loss_scale, float* loss, void* workspace,
                                          size_t workspace_bytes, tt_stream_t stream) {
  using namespace tt;
  clear_error();
  return softmax_xent(q, ldq, c, ldc, n, dim, logq, lse, row_loss, dq, dc, workspace, workspace_bytes, stream, false,
                      loss_scale, loss, true);
}
