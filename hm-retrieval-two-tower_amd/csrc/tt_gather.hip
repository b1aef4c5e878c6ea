// K2+K3: grouped embedding gather + concat (InputLayer.call,
// /root/reference/pkg/modelling/layers/input_layer.py:45-69).
//
// One launch covers every feature: the flattened grid is partitioned into
// per-segment block ranges (prefix in the kernel argument block), and each
// segment copies whole table rows into its column range of the concatenated
// output.  Rows are moved with the widest vector (16/8/4 B per lane) the
// segment's dim, column offset and the output stride allow; `threads per row`
// lanes cover one row so a 128-float row is one 512-B coalesced read by 32
// lanes.  tt_gather_multi puts several calls (both towers) in one launch.
// The op is HBM-bound (algorithmic bytes per row: 2*dim*4 + 4).
#include "tt_common.h"
#include "tt_mlp_pack.h"

namespace tt {
namespace {

#ifndef TT_GATHER_THREADS
#define TT_GATHER_THREADS 256
#endif
constexpr int kGatherThreads = TT_GATHER_THREADS;
#ifndef TT_GATHER_ITERS
#define TT_GATHER_ITERS 2
#endif
constexpr int kGatherIters = TT_GATHER_ITERS;  // row passes per block (rows in flight per lane)

struct GatherSeg {
  const float* table;
  const int32_t* ids;
  float* out;            // this segment's columns: out + col_offset
  int64_t out_stride;
  int64_t num_rows;
  int32_t dim;
  int32_t vec;           // floats per lane loaded: 4, 2 or 1
  int32_t split_store;   // vec == 4 into an 8-byte aligned column: two float2 stores
  int32_t tpr;           // threads per row = dim / vec
  int32_t rows_per_pass; // kGatherThreads / tpr
  int32_t block_begin;   // first block of this segment in the flat grid
};

struct GatherArgs {
  GatherSeg seg[TT_MAX_SEGMENTS];
  int32_t num_segs;
  int64_t batch;
};

template <int VEC>
struct VecT;
template <>
struct VecT<4> {
  using type = float4;
};
template <>
struct VecT<2> {
  using type = float2;
};
template <>
struct VecT<1> {
  using type = float;
};

// All ids of the block's row passes are loaded first, then all rows, then
// all stores: kGatherIters independent row reads in flight per lane instead
// of a dependent id -> row chain per pass.
template <int VEC>
__device__ __forceinline__ void gather_segment(const GatherArgs& a, const GatherSeg& s, int local_block) {
  using V = typename VecT<VEC>::type;
  const int t = threadIdx.x;
  const int row_in_pass = t / s.tpr;
  const int lane_in_row = t - row_in_pass * s.tpr;
  if (row_in_pass >= s.rows_per_pass) return;
  const int64_t row0 = static_cast<int64_t>(local_block) * s.rows_per_pass * kGatherIters;
  const int col = lane_in_row * VEC;
  int64_t rr[kGatherIters];
#pragma unroll
  for (int it = 0; it < kGatherIters; ++it) {
    const int64_t b = row0 + static_cast<int64_t>(it) * s.rows_per_pass + row_in_pass;
    if (s.ids) {
      const int64_t r = b < a.batch ? s.ids[b] : -1;
      rr[it] = (r >= 0 && r < s.num_rows) ? r : -1;  // out-of-range id -> zero row
    } else {  // numeric pass-through column: table is the [batch] value vector
      rr[it] = b < a.batch ? b : -1;
    }
  }
  V v[kGatherIters];
#pragma unroll
  for (int it = 0; it < kGatherIters; ++it) {
    if (rr[it] >= 0) {
      v[it] = *reinterpret_cast<const V*>(s.table + rr[it] * static_cast<int64_t>(s.dim) + col);
    } else {
      if constexpr (VEC == 4) v[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      else if constexpr (VEC == 2) v[it] = make_float2(0.f, 0.f);
      else v[it] = 0.f;
    }
  }
#pragma unroll
  for (int it = 0; it < kGatherIters; ++it) {
    const int64_t b = row0 + static_cast<int64_t>(it) * s.rows_per_pass + row_in_pass;
    if (b >= a.batch) continue;
    float* dst = s.out + b * s.out_stride + col;
    if constexpr (VEC == 4) {
      if (s.split_store) {
        reinterpret_cast<float2*>(dst)[0] = make_float2(v[it].x, v[it].y);
        reinterpret_cast<float2*>(dst)[1] = make_float2(v[it].z, v[it].w);
        continue;
      }
    }
    *reinterpret_cast<V*>(dst) = v[it];
  }
}

// Blocks [0, gather_blocks) gather; the rest (tt_gather_multi_pack) pack the
// towers' MLP weight images for the step's forward (independent work in the
// same launch: no pack launch, no cross-queue fork in front of the forward).
__global__ void __launch_bounds__(kGatherThreads) gather_grouped_kernel(const GatherArgs a, const pack::PackJobs pj,
                                                                        int64_t pack_total, int32_t gather_blocks) {
  if (static_cast<int32_t>(blockIdx.x) >= gather_blocks) {
    const int64_t t = static_cast<int64_t>(blockIdx.x - gather_blocks) * kGatherThreads + threadIdx.x;
    if (t < pack_total) pack::pack_many_thread(pj, t);
    return;
  }
  // Locate this block's segment (<= 32 segments; scalar loop).
  int si = 0;
#pragma unroll 1
  for (int i = 1; i < a.num_segs; ++i)
    if (static_cast<int>(blockIdx.x) >= a.seg[i].block_begin) si = i;
  const GatherSeg& s = a.seg[si];
  const int local_block = blockIdx.x - s.block_begin;
  if (s.vec == 4)
    gather_segment<4>(a, s, local_block);
  else if (s.vec == 2)
    gather_segment<2>(a, s, local_block);
  else
    gather_segment<1>(a, s, local_block);
}

// Load width: 16/8/4 B by the table's alignment and dim.  A 16-B load into
// a column only 8-B aligned (e.g. a 128-float segment after a 2-float one)
// is stored as two float2.
int pick_vec(const tt_gather_segment& s, const float* out, int64_t out_stride, int* split) {
  const int dim = s.ids ? s.dim : 1;
  *split = 0;
  for (int v = 4; v > 1; v >>= 1) {
    if (dim % v) continue;
    if (reinterpret_cast<uintptr_t>(s.table) % (4 * v)) continue;
    const bool aligned = (s.col_offset % v == 0) && (out_stride % v == 0) &&
                         (reinterpret_cast<uintptr_t>(out) % (4 * v) == 0);
    if (aligned) return v;
    if (v == 4 && s.col_offset % 2 == 0 && out_stride % 2 == 0 && reinterpret_cast<uintptr_t>(out) % 8 == 0) {
      *split = 1;
      return 4;
    }
  }
  return 1;
}

constexpr int kMaxTagged = 16;
struct TaggedArgs {
  const float* table[kMaxTagged];
  int64_t num_rows[kMaxTagged];
  int32_t num_tables;
  int32_t dim;
  const int32_t* tags;
  const int32_t* rows;
  int64_t n;
  float* out;
  int64_t out_stride;
};

// One (sub-)wave of dim/4 lanes per request row, float4 moves.
__global__ void __launch_bounds__(256) gather_tagged_kernel(const TaggedArgs a) {
  const int tpr = a.dim / 4;
  const int rpb = 256 / tpr;
  const int64_t j = static_cast<int64_t>(blockIdx.x) * rpb + threadIdx.x / tpr;
  const int lane = threadIdx.x % tpr;
  if (j >= a.n || threadIdx.x / tpr >= rpb) return;
  const int t = a.tags[j];
  const int64_t r = a.rows[j];
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t >= 0 && t < a.num_tables && r >= 0 && r < a.num_rows[t])
    v = reinterpret_cast<const float4*>(a.table[t] + r * a.dim)[lane];
  reinterpret_cast<float4*>(a.out + j * a.out_stride)[lane] = v;
}

int add_call(GatherArgs& a, int32_t& blocks, const tt_gather_segment* segs, int32_t num_segs, float* out,
             int64_t out_stride) {
  TT_REQUIRE(segs != nullptr, "tt_gather: segs is NULL");
  TT_REQUIRE(num_segs >= 1 && a.num_segs + num_segs <= TT_MAX_SEGMENTS,
             "tt_gather: %d segments exceed the limit of %d", a.num_segs + num_segs, TT_MAX_SEGMENTS);
  TT_REQUIRE(out != nullptr, "tt_gather: out is NULL");
  for (int i = 0; i < num_segs; ++i) {
    const tt_gather_segment& s = segs[i];
    TT_REQUIRE(s.table != nullptr, "tt_gather: segment %d table is NULL", i);
    const int dim = s.ids ? s.dim : 1;
    TT_REQUIRE(dim >= 1 && dim <= 4 * kGatherThreads, "tt_gather: segment %d dim=%d outside [1,%d]", i, s.dim,
               4 * kGatherThreads);
    TT_REQUIRE(s.ids == nullptr || s.num_rows >= 1, "tt_gather: segment %d has an empty table", i);
    TT_REQUIRE(s.col_offset >= 0 && s.col_offset + dim <= out_stride,
               "tt_gather: segment %d columns [%d,%d) exceed out_stride %lld", i, s.col_offset, s.col_offset + dim,
               static_cast<long long>(out_stride));
    int split = 0;
    const int vec = pick_vec(s, out, out_stride, &split);
    const int tpr = dim / vec;
    TT_REQUIRE(tpr <= kGatherThreads, "tt_gather: segment %d dim too wide for vector %d", i, vec);
    GatherSeg& g = a.seg[a.num_segs++];
    g.table = s.table;
    g.ids = s.ids;
    g.out = out + s.col_offset;
    g.out_stride = out_stride;
    g.num_rows = s.num_rows;
    g.dim = dim;
    g.vec = vec;
    g.split_store = split;
    g.tpr = tpr;
    g.rows_per_pass = kGatherThreads / tpr;
    g.block_begin = blocks;
    const int64_t rows_per_block = static_cast<int64_t>(g.rows_per_pass) * kGatherIters;
    const int64_t nb = ceil_div(a.batch, rows_per_block);
    TT_REQUIRE(blocks + nb < (1ll << 31), "tt_gather: grid too large");
    blocks += static_cast<int32_t>(nb);
  }
  return TT_OK;
}

int launch(const GatherArgs& a, int32_t blocks, tt_stream_t stream, const pack::PackJobs* pj = nullptr,
           int64_t pack_total = 0) {
  static_assert(kGatherThreads == 256, "the pack blocks are 256-thread blocks");
  const int64_t pack_blocks = pj ? ceil_div(pack_total, kGatherThreads) : 0;
  const pack::PackJobs none{};
  hipLaunchKernelGGL(gather_grouped_kernel, dim3(static_cast<unsigned>(blocks + pack_blocks)), dim3(kGatherThreads), 0,
                     to_stream(stream), a, pj ? *pj : none, pj ? pack_total : int64_t(0), blocks);
  TT_CHECK_LAUNCH();
  return TT_OK;
}

}  // namespace
}  // namespace tt

extern "C" int tt_gather_grouped(const tt_gather_segment* segs, int32_t num_segs, int64_t batch, float* out,
                                 int64_t out_stride, tt_stream_t stream) {
  using namespace tt;
  clear_error();
  TT_REQUIRE(segs != nullptr, "tt_gather_grouped: segs is NULL");
  TT_REQUIRE(num_segs >= 1 && num_segs <= TT_MAX_SEGMENTS, "tt_gather_grouped: num_segs=%d outside [1,%d]",
             num_segs, TT_MAX_SEGMENTS);
  TT_REQUIRE(batch >= 0, "tt_gather_grouped: negative batch");
  TT_REQUIRE(out != nullptr || batch == 0, "tt_gather_grouped: out is NULL");
  if (batch == 0) return TT_OK;
  GatherArgs a{};
  a.batch = batch;
  int32_t blocks = 0;
  int rc = add_call(a, blocks, segs, num_segs, out, out_stride);
  if (rc) return rc;
  return launch(a, blocks, stream);
}

extern "C" int tt_gather_multi(const tt_gather_call* calls, int32_t num_calls, int64_t batch, tt_stream_t stream) {
  using namespace tt;
  clear_error();
  TT_REQUIRE(calls != nullptr && num_calls >= 1, "tt_gather_multi: no calls");
  TT_REQUIRE(batch >= 0, "tt_gather_multi: negative batch");
  if (batch == 0) return TT_OK;
  GatherArgs a{};
  a.batch = batch;
  int32_t blocks = 0;
  for (int c = 0; c < num_calls; ++c) {
    int rc = add_call(a, blocks, calls[c].segs, calls[c].num_segs, calls[c].out, calls[c].out_stride);
    if (rc) return rc;
  }
  return launch(a, blocks, stream);
}

extern "C" int tt_gather_multi_pack(const tt_gather_call* calls, int32_t num_calls, int64_t batch,
                                    const tt_mlp_pack_job* jobs, int32_t num_jobs, tt_stream_t stream) {
  using namespace tt;
  clear_error();
  TT_REQUIRE(calls != nullptr && num_calls >= 1, "tt_gather_multi_pack: no calls");
  TT_REQUIRE(batch >= 1, "tt_gather_multi_pack: batch must be >= 1");
  pack::PackJobs pj;
  int64_t total = 0;
  if (int rc = pack::make_pack_jobs(jobs, num_jobs, &pj, &total, "tt_gather_multi_pack")) return rc;
  GatherArgs a{};
  a.batch = batch;
  int32_t blocks = 0;
  for (int c = 0; c < num_calls; ++c) {
    int rc = add_call(a, blocks, calls[c].segs, calls[c].num_segs, calls[c].out, calls[c].out_stride);
    if (rc) return rc;
  }
  return launch(a, blocks, stream, &pj, total);
}

extern "C" int tt_gather_tagged(const tt_row_table* tables, int32_t num_tables, int32_t dim, const int32_t* tags,
                                const int32_t* rows, int64_t n, float* out, int64_t out_stride,
                                tt_stream_t stream) {
  using namespace tt;
  clear_error();
  TT_REQUIRE(tables && num_tables >= 1 && num_tables <= kMaxTagged, "tt_gather_tagged: 1..%d tables", kMaxTagged);
  TT_REQUIRE(dim >= 4 && dim % 4 == 0 && dim <= 1024, "tt_gather_tagged: dim=%d must be a multiple of 4 in [4,1024]",
             dim);
  TT_REQUIRE(n >= 0, "tt_gather_tagged: negative n");
  if (n == 0) return TT_OK;
  TT_REQUIRE(tags && rows && out, "tt_gather_tagged: NULL pointer");
  TT_REQUIRE(out_stride >= dim && out_stride % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0,
             "tt_gather_tagged: out must be 16-byte aligned rows");
  TaggedArgs a{};
  for (int i = 0; i < num_tables; ++i) {
    TT_REQUIRE(tables[i].table && reinterpret_cast<uintptr_t>(tables[i].table) % 16 == 0,
               "tt_gather_tagged: table %d must be 16-byte aligned", i);
    a.table[i] = tables[i].table;
    a.num_rows[i] = tables[i].num_rows;
  }
  a.num_tables = num_tables;
  a.dim = dim;
  a.tags = tags;
  a.rows = rows;
  a.n = n;
  a.out = out;
  a.out_stride = out_stride;
  const int rpb = 256 / (dim / 4);
  hipLaunchKernelGGL(gather_tagged_kernel, dim3(ceil_div(n, rpb)), dim3(256), 0, to_stream(stream), a);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
