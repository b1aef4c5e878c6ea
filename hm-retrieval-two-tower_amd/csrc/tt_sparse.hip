// K8+K9 (+K10): duplicate-id dedup, segmented gradient sum and the optimizer
// apply for embedding tables; dense optimizers for the tower MLP weights.
//
// Reference semantics (legacy Keras optimizer reached from
// /root/reference/pkg/modelling/models/two_tower_model.py:124 with
// /root/reference/pkg/modelling/optimizer_factory.py:15-18):
//   _resource_apply_sparse_duplicate_indices -> tf.unique + UnsortedSegmentSum
//   (per distinct id, rows summed in increasing batch position, starting from
//   0), then ResourceSparseApplyAdagradV2 per distinct row:
//       acc += g*g;  w -= lr*g / (sqrt(acc) + eps)
//
// MI355X design:
//  1. sort   — one 1024-thread workgroup per table: stable LSD radix sort of
//     (id, position) with 8-bit digits (ceil(bits(num_rows)/8) passes).  Each
//     wave owns a contiguous slice and ranks its elements with 8 ballots per
//     64-element group (wave-private LDS digit counters), so the sort is
//     stable and deterministic.  Then segment heads, per-id chunk layout.
//  2. chunk_sum — one (sub-)wave per chunk of <= kChunk consecutive rows of a
//     segment: sequential fp32 sum in position order, lanes over columns, so
//     every global read is a coalesced row slice.  Zipf heavy hitters (ids
//     repeated thousands of times in one batch) are split into chunks that run
//     in parallel instead of one long serial chain.
//  3. apply — one (sub-)wave per distinct id: chunk partials summed in chunk
//     order (bitwise reproducible; identical to TF's flat order whenever an id
//     occurs <= kChunk times in the batch, within 1e-6 rel otherwise), then the
//     optimizer update of that row.  HBM-bound: per distinct row
//     param r/w + slot r/w = 16*dim bytes.
// All arithmetic goes through ieee_op<> (one correctly rounded IEEE operation
// each; the file is built with -ffp-contract=off and HIP's default correctly
// rounded fp32 divide/sqrt) so results match the CPU restatement bit for bit.
// (HIP's __fsqrt_rn maps to the approximate native sqrt on this toolchain.)
#include "tt_common.h"

namespace tt {
namespace {

template <char OP>
__device__ __forceinline__ float ieee_op(float a, float b) {
  if constexpr (OP == '+') return a + b;
  if constexpr (OP == '-') return a - b;
  if constexpr (OP == '*') return a * b;
  return a / b;
}

constexpr int kSortThreads = 1024;
constexpr int kSortWaves = kSortThreads / kWave;
constexpr int kChunk = 32;
constexpr int kTablesPerLaunch = 16;
constexpr int kApplyThreads = 256;

// Per-table workspace layout (device and host agree on it).
struct TableWs {
  uint32_t* keys0;
  uint32_t* vals0;
  uint32_t* keys1;
  uint32_t* vals1;
  int32_t* uniq;      // [n+1] distinct ids, ascending
  int32_t* seg;       // [n+1] segment starts (seg[U] = n)
  int32_t* cbase;     // [n+1] first chunk of each distinct id (cbase[U] = #chunks)
  int32_t* cseg;      // [max_chunks] owning distinct id of each chunk
  int32_t* counts;    // [0] = U, [1] = #chunks
  float* partial;     // [max_chunks, dim] chunk sums
};

__host__ __device__ inline int64_t max_chunks(int64_t n) { return n + (n + kChunk - 1) / kChunk + 1; }

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

__host__ __device__ inline size_t table_ws_bytes(int64_t n, int32_t dim) {
  size_t b = 0;
  b += 4 * align256(sizeof(uint32_t) * n);
  b += 3 * align256(sizeof(int32_t) * (n + 1));
  b += align256(sizeof(int32_t) * max_chunks(n));
  b += align256(sizeof(int32_t) * 4);
  b += align256(sizeof(float) * max_chunks(n) * dim);
  return b;
}

__host__ __device__ inline TableWs carve_table(char* base, int64_t n, int32_t dim) {
  TableWs w;
  size_t o = 0;
  auto take = [&](size_t bytes) { char* p = base + o; o += align256(bytes); return p; };
  w.keys0 = reinterpret_cast<uint32_t*>(take(sizeof(uint32_t) * n));
  w.vals0 = reinterpret_cast<uint32_t*>(take(sizeof(uint32_t) * n));
  w.keys1 = reinterpret_cast<uint32_t*>(take(sizeof(uint32_t) * n));
  w.vals1 = reinterpret_cast<uint32_t*>(take(sizeof(uint32_t) * n));
  w.uniq = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (n + 1)));
  w.seg = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (n + 1)));
  w.cbase = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (n + 1)));
  w.cseg = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * max_chunks(n)));
  w.counts = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 4));
  w.partial = reinterpret_cast<float*>(take(sizeof(float) * max_chunks(n) * dim));
  return w;
}

struct TableJob {
  char* ws;
  const int32_t* ids[TT_MAX_SOURCES];
  int32_t goff[TT_MAX_SOURCES];
  float* table;
  float* slot0;
  float* slot1;
  int64_t num_rows;
  int32_t n;          // num_sources * batch
  int32_t dim;
  int32_t num_sources;
  int32_t passes;     // radix passes
  int32_t lanes_per_slot;  // P: lanes per chunk/id slot (pow2 <= 64)
  int32_t wave_begin_chunk; // first global wave of this table in chunk_sum
  int32_t wave_begin_apply; // first global wave of this table in apply
};

struct JobList {
  TableJob job[kTablesPerLaunch];
  int32_t num_jobs;
  int64_t batch;
  const float* grad;
  int64_t grad_stride;
};

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return (l == 0) ? 0ull : (~0ull >> (64 - l));
}

// Lanes (among `active`) holding the same 8-bit digit as this lane.
__device__ __forceinline__ uint64_t match_digit(unsigned d, uint64_t active) {
  uint64_t peers = active;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  return peers;
}

// Exclusive scan of one int per thread over the 1024-thread block; returns
// the prefix, writes the block total to *total.  Uses LDS scratch[>=16].
__device__ int block_exclusive_scan(int v, int* scratch, int* total) {
  const int lane = lane_id();
  const int w = threadIdx.x / kWave;
  int x = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int y = __shfl_up(x, off, kWave);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) scratch[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int i = 0; i < kSortWaves; ++i) {
      const int t = scratch[i];
      scratch[i] = run;
      run += t;
    }
    scratch[kSortWaves] = run;
  }
  __syncthreads();
  const int r = scratch[w] + x - v;
  *total = scratch[kSortWaves];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(kSortThreads) sort_segments_kernel(const JobList jl) {
  const TableJob& J = jl.job[blockIdx.x];
  const int64_t n = J.n;
  TableWs W = carve_table(J.ws, n, J.dim);
  __shared__ unsigned cnt[kSortWaves][256];
  __shared__ unsigned digit_base[256];
  __shared__ int scratch[kSortWaves + 1];

  // Step 0: keys = ids (out-of-range -> num_rows, sorted last and skipped),
  // vals = position in the concatenated source list.
  const uint32_t invalid_key = static_cast<uint32_t>(J.num_rows);
  for (int64_t p = threadIdx.x; p < n; p += kSortThreads) {
    const int s = static_cast<int>(p / jl.batch);
    const int64_t b = p - static_cast<int64_t>(s) * jl.batch;
    const int32_t id = J.ids[s][b];
    W.keys0[p] = (id >= 0 && id < J.num_rows) ? static_cast<uint32_t>(id) : invalid_key;
    W.vals0[p] = static_cast<uint32_t>(p);
  }
  __syncthreads();

  const int w = threadIdx.x / kWave;
  const int lane = lane_id();
  const int64_t chunk = ((n + kSortWaves - 1) / kSortWaves + kWave - 1) / kWave * kWave;
  const int64_t beg = w * chunk;
  const int64_t end = (beg + chunk < n) ? beg + chunk : n;

  uint32_t* sk = W.keys0;
  uint32_t* sv = W.vals0;
  uint32_t* dk = W.keys1;
  uint32_t* dv = W.vals1;
  for (int pass = 0; pass < J.passes; ++pass) {
    const int shift = 8 * pass;
    for (int i = threadIdx.x; i < kSortWaves * 256; i += kSortThreads) (&cnt[0][0])[i] = 0;
    __syncthreads();
    // Count digits per wave slice.
    for (int64_t g = beg; g < end; g += kWave) {
      const int64_t p = g + lane;
      const bool valid = p < end;
      const unsigned d = valid ? ((sk[p] >> shift) & 255u) : 0u;
      const uint64_t act = __ballot(valid);
      const uint64_t peers = match_digit(d, act);
      if (valid && (__ffsll(static_cast<long long>(peers)) - 1) == lane)
        cnt[w][d] += static_cast<unsigned>(__popcll(peers));
    }
    __syncthreads();
    if (threadIdx.x < 256) {
      const int d = threadIdx.x;
      unsigned run = 0;
      for (int ww = 0; ww < kSortWaves; ++ww) {
        const unsigned c = cnt[ww][d];
        cnt[ww][d] = run;
        run += c;
      }
      digit_base[d] = run;
    }
    __syncthreads();
    if (threadIdx.x < kWave) {  // exclusive scan of the 256 digit totals
      unsigned v0 = digit_base[4 * lane + 0], v1 = digit_base[4 * lane + 1];
      unsigned v2 = digit_base[4 * lane + 2], v3 = digit_base[4 * lane + 3];
      unsigned s = v0 + v1 + v2 + v3, x = s;
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) {
        const unsigned y = __shfl_up(x, off, kWave);
        if (lane >= off) x += y;
      }
      unsigned e = x - s;
      digit_base[4 * lane + 0] = e;
      digit_base[4 * lane + 1] = e + v0;
      digit_base[4 * lane + 2] = e + v0 + v1;
      digit_base[4 * lane + 3] = e + v0 + v1 + v2;
    }
    __syncthreads();
    // Stable scatter.
    for (int64_t g = beg; g < end; g += kWave) {
      const int64_t p = g + lane;
      const bool valid = p < end;
      const uint32_t k = valid ? sk[p] : 0u;
      const uint32_t v = valid ? sv[p] : 0u;
      const unsigned d = (k >> shift) & 255u;
      const uint64_t act = __ballot(valid);
      const uint64_t peers = match_digit(d, act);
      const unsigned base = cnt[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid) {
        const unsigned pos = digit_base[d] + base + static_cast<unsigned>(__popcll(peers & lanemask_lt()));
        dk[pos] = k;
        dv[pos] = v;
        if ((__ffsll(static_cast<long long>(peers)) - 1) == lane)
          cnt[w][d] = base + static_cast<unsigned>(__popcll(peers));
      }
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    uint32_t* t0 = sk; sk = dk; dk = t0;
    uint32_t* t1 = sv; sv = dv; dv = t1;
  }

  // Segment heads -> distinct ids and segment starts.
  const int64_t per = (n + kSortThreads - 1) / kSortThreads;
  const int64_t r0 = threadIdx.x * per;
  const int64_t r1 = (r0 + per < n) ? r0 + per : n;
  int heads = 0;
  for (int64_t i = r0; i < r1; ++i) heads += (i == 0 || sk[i] != sk[i - 1]) ? 1 : 0;
  int total_u = 0;
  int u = block_exclusive_scan(heads, scratch, &total_u);
  for (int64_t i = r0; i < r1; ++i) {
    if (i == 0 || sk[i] != sk[i - 1]) {
      W.uniq[u] = static_cast<int32_t>(sk[i]);
      W.seg[u] = static_cast<int32_t>(i);
      ++u;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    W.seg[total_u] = static_cast<int32_t>(n);
    W.counts[0] = total_u;
  }
  __syncthreads();
  // Chunk layout: ceil(len / kChunk) chunks per distinct id.
  const int64_t uper = (total_u + kSortThreads - 1) / kSortThreads;
  const int64_t u0 = threadIdx.x * uper;
  const int64_t u1 = (u0 + uper < total_u) ? u0 + uper : total_u;
  int nch = 0;
  for (int64_t q = u0; q < u1; ++q) nch += (W.seg[q + 1] - W.seg[q] + kChunk - 1) / kChunk;
  int total_c = 0;
  int c = block_exclusive_scan(nch, scratch, &total_c);
  for (int64_t q = u0; q < u1; ++q) {
    W.cbase[q] = c;
    const int k = (W.seg[q + 1] - W.seg[q] + kChunk - 1) / kChunk;
    for (int j = 0; j < k; ++j) W.cseg[c + j] = static_cast<int32_t>(q);
    c += k;
  }
  if (threadIdx.x == 0) {
    W.cbase[total_u] = total_c;
    W.counts[1] = total_c;
  }
}

// The sorted (id, position) arrays live in buffer 0 or 1 by pass parity.
__device__ __forceinline__ const uint32_t* sorted_vals(const TableWs& W, int passes) {
  return (passes & 1) ? W.vals1 : W.vals0;
}

__device__ __forceinline__ int find_job(const JobList& jl, int gw, bool apply) {
  int t = 0;
#pragma unroll 1
  for (int i = 1; i < jl.num_jobs; ++i) {
    const int b = apply ? jl.job[i].wave_begin_apply : jl.job[i].wave_begin_chunk;
    if (gw >= b) t = i;
  }
  return t;
}

__global__ void __launch_bounds__(kApplyThreads) chunk_sum_kernel(const JobList jl) {
  const int gw = blockIdx.x * (kApplyThreads / kWave) + threadIdx.x / kWave;
  const int t = find_job(jl, gw, false);
  const TableJob& J = jl.job[t];
  const TableWs W = carve_table(J.ws, J.n, J.dim);
  const int P = J.lanes_per_slot;
  const int lane = lane_id();
  const int c = (gw - J.wave_begin_chunk) * (kWave / P) + lane / P;
  if (c >= W.counts[1]) return;
  const int col0 = lane % P;
  const int q = W.cseg[c];
  const int r0 = W.seg[q] + (c - W.cbase[q]) * kChunk;
  const int r1 = min(r0 + kChunk, W.seg[q + 1]);
  const uint32_t* sv = sorted_vals(W, J.passes);
  for (int col = col0; col < J.dim; col += P) {
    float acc = 0.0f;
    for (int r = r0; r < r1; ++r) {
      const uint32_t p = sv[r];
      const int s = static_cast<int>(p / static_cast<uint32_t>(jl.batch));
      const int64_t b = static_cast<int64_t>(p) - static_cast<int64_t>(s) * jl.batch;
      acc = ieee_op<'+'>(acc, jl.grad[b * jl.grad_stride + J.goff[s] + col]);
    }
    W.partial[static_cast<int64_t>(c) * J.dim + col] = acc;
  }
}

enum ApplyOp { kWriteSum = 0, kAdagrad = 1, kAdamScatter = 2 };

struct ApplyParams {
  float lr;
  float eps;
  float one_minus_beta1;
  float one_minus_beta2;
  int32_t* out_uniq;   // kWriteSum
  float* out_sum;      // kWriteSum
  int32_t* out_count;  // kWriteSum
};

template <int OP>
__global__ void __launch_bounds__(kApplyThreads) apply_kernel(const JobList jl, const ApplyParams ap) {
  const int gw = blockIdx.x * (kApplyThreads / kWave) + threadIdx.x / kWave;
  const int t = find_job(jl, gw, true);
  const TableJob& J = jl.job[t];
  const TableWs W = carve_table(J.ws, J.n, J.dim);
  const int P = J.lanes_per_slot;
  const int lane = lane_id();
  const int q = (gw - J.wave_begin_apply) * (kWave / P) + lane / P;
  const int U = W.counts[0];
  if (OP == kWriteSum && gw == 0 && lane == 0) *ap.out_count = U;
  if (q >= U) return;
  const int32_t row = W.uniq[q];
  if (OP == kWriteSum && lane % P == 0) ap.out_uniq[q] = row;
  if (OP != kWriteSum && (row < 0 || row >= J.num_rows)) return;  // out-of-range ids
  const int c0 = W.cbase[q];
  const int c1 = W.cbase[q + 1];
  for (int col = lane % P; col < J.dim; col += P) {
    float g = 0.0f;
    for (int c = c0; c < c1; ++c) g = ieee_op<'+'>(g, W.partial[static_cast<int64_t>(c) * J.dim + col]);
    if (OP == kWriteSum) {
      ap.out_sum[static_cast<int64_t>(q) * J.dim + col] = g;
    } else if (OP == kAdagrad) {
      const int64_t o = static_cast<int64_t>(row) * J.dim + col;
      const float a = ieee_op<'+'>(J.slot0[o], ieee_op<'*'>(g, g));
      J.slot0[o] = a;
      J.table[o] = ieee_op<'-'>(J.table[o], ieee_op<'/'>(ieee_op<'*'>(ap.lr, g), ieee_op<'+'>(sqrtf(a), ap.eps)));
    } else {  // Adam: scatter-add of the scaled distinct-id gradient into the decayed slots
      const int64_t o = static_cast<int64_t>(row) * J.dim + col;
      J.slot0[o] = ieee_op<'+'>(J.slot0[o], ieee_op<'*'>(g, ap.one_minus_beta1));
      J.slot1[o] = ieee_op<'+'>(J.slot1[o], ieee_op<'*'>(ieee_op<'*'>(g, g), ap.one_minus_beta2));
    }
  }
}

// Dense elementwise passes (grid-stride).
__global__ void scale2_kernel(float* a, float sa, float* b, float sb, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    a[i] = ieee_op<'*'>(a[i], sa);
    b[i] = ieee_op<'*'>(b[i], sb);
  }
}

// Legacy Adam sparse path, final dense step: var -= lr*m / (sqrt(v) + eps).
__global__ void adam_var_kernel(float* var, const float* m, const float* v, float lr, float eps, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    var[i] = ieee_op<'-'>(var[i], ieee_op<'/'>(ieee_op<'*'>(lr, m[i]), ieee_op<'+'>(sqrtf(v[i]), eps)));
}

// ResourceApplyAdagradV2: accum += g^2; var -= g*lr / (sqrt(accum) + eps).
__global__ void dense_adagrad_kernel(float* p, float* acc, const float* g, int64_t n, float lr, float eps) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float a = ieee_op<'+'>(acc[i], ieee_op<'*'>(gi, gi));
    acc[i] = a;
    p[i] = ieee_op<'-'>(p[i], ieee_op<'/'>(ieee_op<'*'>(gi, lr), ieee_op<'+'>(sqrtf(a), eps)));
  }
}

// ResourceApplyAdam (use_nesterov=false):
//   m += (g - m)*(1-b1); v += (g*g - v)*(1-b2); var -= m*alpha / (sqrt(v) + eps)
__global__ void dense_adam_kernel(float* p, float* m, float* v, const float* g, int64_t n, float alpha,
                                  float omb1, float omb2, float eps) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float mi = ieee_op<'+'>(m[i], ieee_op<'*'>(ieee_op<'-'>(gi, m[i]), omb1));
    const float vi = ieee_op<'+'>(v[i], ieee_op<'*'>(ieee_op<'-'>(ieee_op<'*'>(gi, gi), v[i]), omb2));
    m[i] = mi;
    v[i] = vi;
    p[i] = ieee_op<'-'>(p[i], ieee_op<'/'>(ieee_op<'*'>(mi, alpha), ieee_op<'+'>(sqrtf(vi), eps)));
  }
}

int bits_for(int64_t x) {  // bits needed to represent values in [0, x]
  int b = 1;
  while ((int64_t(1) << b) <= x) ++b;
  return b;
}

int lanes_per_slot(int dim) {
  int p = 1;
  while (p < dim && p < kWave) p <<= 1;
  return p;
}

size_t tables_ws_bytes(const tt_sparse_table* tables, int32_t num_tables, int64_t batch) {
  size_t b = 0;
  for (int i = 0; i < num_tables; ++i)
    b += align256(table_ws_bytes(tables[i].num_sources * batch, tables[i].dim));
  return b;
}

int validate_tables(const tt_sparse_table* tables, int32_t num_tables, int64_t batch, bool adam) {
  TT_REQUIRE(tables != nullptr && num_tables >= 1, "sparse: no tables");
  TT_REQUIRE(batch >= 0, "sparse: negative batch");
  for (int i = 0; i < num_tables; ++i) {
    const tt_sparse_table& t = tables[i];
    TT_REQUIRE(t.table && t.slot0, "sparse: table %d has NULL parameter/slot pointer", i);
    TT_REQUIRE(!adam || t.slot1, "sparse: table %d needs slot1 for Adam", i);
    TT_REQUIRE(t.num_rows >= 1 && t.num_rows < (int64_t(1) << 31) - 1, "sparse: table %d num_rows out of range", i);
    TT_REQUIRE(t.dim >= 1 && t.dim <= 4096, "sparse: table %d dim=%d out of range", i, t.dim);
    TT_REQUIRE(t.num_sources >= 1 && t.num_sources <= TT_MAX_SOURCES, "sparse: table %d num_sources=%d", i, t.num_sources);
    TT_REQUIRE(t.num_sources * batch <= 65536 * 4, "sparse: table %d has %lld lookups (max %d)", i,
               static_cast<long long>(t.num_sources * batch), 65536 * 4);
    for (int s = 0; s < t.num_sources; ++s) TT_REQUIRE(t.ids[s] || batch == 0, "sparse: table %d source %d ids NULL", i, s);
  }
  return TT_OK;
}

// Runs sort -> chunk_sum -> apply<OP> over all tables, kTablesPerLaunch at a time.
template <int OP>
int run_sparse(const tt_sparse_table* tables, int32_t num_tables, int64_t batch, const float* grad,
               int64_t grad_stride, const ApplyParams& ap, void* workspace, hipStream_t st) {
  char* ws = static_cast<char*>(workspace);
  for (int first = 0; first < num_tables; first += kTablesPerLaunch) {
    const int cnt = (num_tables - first < kTablesPerLaunch) ? num_tables - first : kTablesPerLaunch;
    JobList jl{};
    jl.num_jobs = cnt;
    jl.batch = batch;
    jl.grad = grad;
    jl.grad_stride = grad_stride;
    int waves_c = 0, waves_a = 0;
    for (int i = 0; i < cnt; ++i) {
      const tt_sparse_table& t = tables[first + i];
      TableJob& J = jl.job[i];
      const int64_t n = t.num_sources * batch;
      J.ws = ws;
      ws += align256(table_ws_bytes(n, t.dim));
      for (int s = 0; s < TT_MAX_SOURCES; ++s) {
        J.ids[s] = (s < t.num_sources) ? t.ids[s] : nullptr;
        J.goff[s] = (s < t.num_sources) ? t.grad_col_offset[s] : 0;
      }
      J.table = t.table;
      J.slot0 = t.slot0;
      J.slot1 = t.slot1;
      J.num_rows = t.num_rows;
      J.n = static_cast<int32_t>(n);
      J.dim = t.dim;
      J.num_sources = t.num_sources;
      J.passes = (bits_for(t.num_rows) + 7) / 8;
      J.lanes_per_slot = lanes_per_slot(t.dim);
      J.wave_begin_chunk = waves_c;
      J.wave_begin_apply = waves_a;
      const int spw = kWave / J.lanes_per_slot;
      waves_c += static_cast<int>(ceil_div(max_chunks(n), spw));
      waves_a += static_cast<int>(ceil_div(n + 1, spw));
    }
    hipLaunchKernelGGL(sort_segments_kernel, dim3(cnt), dim3(kSortThreads), 0, st, jl);
    TT_CHECK_LAUNCH();
    const int wpb = kApplyThreads / kWave;
    hipLaunchKernelGGL(chunk_sum_kernel, dim3(ceil_div(waves_c, wpb)), dim3(kApplyThreads), 0, st, jl);
    TT_CHECK_LAUNCH();
    hipLaunchKernelGGL(apply_kernel<OP>, dim3(ceil_div(waves_a, wpb)), dim3(kApplyThreads), 0, st, jl, ap);
    TT_CHECK_LAUNCH();
  }
  return TT_OK;
}

dim3 stride_grid(int64_t n) {
  int64_t b = ceil_div(n, 256);
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return dim3(static_cast<unsigned>(b));
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" size_t tt_sparse_workspace_size(const tt_sparse_table* tables, int32_t num_tables, int64_t batch) {
  if (!tables || num_tables < 1 || batch < 0) return 0;
  return tables_ws_bytes(tables, num_tables, batch);
}

extern "C" int tt_sparse_adagrad(const tt_sparse_table* tables, int32_t num_tables, int64_t batch,
                                 const float* grad, int64_t grad_stride, float lr, float epsilon,
                                 void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  int rc = validate_tables(tables, num_tables, batch, false);
  if (rc) return rc;
  if (batch == 0) return TT_OK;
  TT_REQUIRE(grad != nullptr, "tt_sparse_adagrad: grad is NULL");
  const size_t need = tables_ws_bytes(tables, num_tables, batch);
  if (!workspace || workspace_bytes < need)
    return fail(TT_ERR_WORKSPACE, "tt_sparse_adagrad: workspace %zu < required %zu", workspace_bytes, need);
  ApplyParams ap{};
  ap.lr = lr;
  ap.eps = epsilon;
  return run_sparse<kAdagrad>(tables, num_tables, batch, grad, grad_stride, ap, workspace, to_stream(stream));
}

extern "C" int tt_sparse_adam(const tt_sparse_table* tables, int32_t num_tables, int64_t batch,
                              const float* grad, int64_t grad_stride, float lr, float beta1, float beta2,
                              float epsilon, int64_t step, void* workspace, size_t workspace_bytes,
                              tt_stream_t stream) {
  clear_error();
  int rc = validate_tables(tables, num_tables, batch, true);
  if (rc) return rc;
  TT_REQUIRE(step >= 1, "tt_sparse_adam: step must be >= 1");
  TT_REQUIRE(batch == 0 || grad != nullptr, "tt_sparse_adam: grad is NULL");
  const size_t need = tables_ws_bytes(tables, num_tables, batch);
  if (batch > 0 && (!workspace || workspace_bytes < need))
    return fail(TT_ERR_WORKSPACE, "tt_sparse_adam: workspace %zu < required %zu", workspace_bytes, need);
  hipStream_t st = to_stream(stream);
  // Coefficients exactly as legacy Adam._prepare_local computes them in fp32.
  const float b1 = beta1, b2 = beta2;
  const float b1p = powf(b1, static_cast<float>(step));
  const float b2p = powf(b2, static_cast<float>(step));
  const float lr_t = lr * (sqrtf(1.0f - b2p) / (1.0f - b1p));
  for (int i = 0; i < num_tables; ++i) {
    const int64_t n = tables[i].num_rows * tables[i].dim;
    hipLaunchKernelGGL(scale2_kernel, stride_grid(n), dim3(256), 0, st, tables[i].slot0, b1, tables[i].slot1, b2, n);
    TT_CHECK_LAUNCH();
  }
  if (batch > 0) {
    ApplyParams ap{};
    ap.one_minus_beta1 = 1.0f - b1;
    ap.one_minus_beta2 = 1.0f - b2;
    rc = run_sparse<kAdamScatter>(tables, num_tables, batch, grad, grad_stride, ap, workspace, st);
    if (rc) return rc;
  }
  for (int i = 0; i < num_tables; ++i) {
    const int64_t n = tables[i].num_rows * tables[i].dim;
    hipLaunchKernelGGL(adam_var_kernel, stride_grid(n), dim3(256), 0, st, tables[i].table, tables[i].slot0,
                       tables[i].slot1, lr_t, epsilon, n);
    TT_CHECK_LAUNCH();
  }
  return TT_OK;
}

extern "C" size_t tt_dedup_workspace_size(int64_t n, int32_t dim) {
  if (n < 0 || dim < 1) return 0;
  return align256(table_ws_bytes(n, dim));
}

extern "C" int tt_dedup_sum(const int32_t* ids, int64_t n, int64_t num_rows, const float* grad,
                            int64_t grad_stride, int32_t dim, int32_t* unique_ids, float* summed,
                            int32_t* num_unique, void* workspace, size_t workspace_bytes, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(ids && grad && unique_ids && summed && num_unique, "tt_dedup_sum: NULL pointer");
  TT_REQUIRE(n >= 1 && n <= 65536 * 4, "tt_dedup_sum: n=%lld out of range", static_cast<long long>(n));
  tt_sparse_table t{};
  t.table = summed;  // not written by kWriteSum
  t.slot0 = summed;
  t.num_rows = num_rows;
  t.dim = dim;
  t.num_sources = 1;
  t.ids[0] = ids;
  t.grad_col_offset[0] = 0;
  int rc = validate_tables(&t, 1, n, false);
  if (rc) return rc;
  const size_t need = tables_ws_bytes(&t, 1, n);
  if (!workspace || workspace_bytes < need)
    return fail(TT_ERR_WORKSPACE, "tt_dedup_sum: workspace %zu < required %zu", workspace_bytes, need);
  ApplyParams ap{};
  ap.out_uniq = unique_ids;
  ap.out_sum = summed;
  ap.out_count = num_unique;
  return run_sparse<kWriteSum>(&t, 1, n, grad, grad_stride, ap, workspace, to_stream(stream));
}

extern "C" int tt_dense_adagrad(float* param, float* accum, const float* grad, int64_t n, float lr,
                                float epsilon, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(n >= 0, "tt_dense_adagrad: negative n");
  if (n == 0) return TT_OK;
  TT_REQUIRE(param && accum && grad, "tt_dense_adagrad: NULL pointer");
  hipLaunchKernelGGL(dense_adagrad_kernel, stride_grid(n), dim3(256), 0, to_stream(stream), param, accum, grad, n,
                     lr, epsilon);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

extern "C" int tt_dense_adam(float* param, float* m, float* v, const float* grad, int64_t n, float lr,
                             float beta1, float beta2, float epsilon, int64_t step, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(n >= 0 && step >= 1, "tt_dense_adam: bad n/step");
  if (n == 0) return TT_OK;
  TT_REQUIRE(param && m && v && grad, "tt_dense_adam: NULL pointer");
  const float b1p = powf(beta1, static_cast<float>(step));
  const float b2p = powf(beta2, static_cast<float>(step));
  // TF ApplyAdamOp: alpha = lr * sqrt(1 - beta2_power) / (1 - beta1_power).
  const float alpha = (lr * sqrtf(1.0f - b2p)) / (1.0f - b1p);
  hipLaunchKernelGGL(dense_adam_kernel, stride_grid(n), dim3(256), 0, to_stream(stream), param, m, v, grad, n,
                     alpha, 1.0f - beta1, 1.0f - beta2, epsilon);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
