// K2+K3: grouped embedding gather + concat (InputLayer.call,
// /root/reference/pkg/modelling/layers/input_layer.py:45-69).
//
// One launch covers every feature: the flattened grid is partitioned into
// per-segment block ranges (prefix in the kernel argument block), and each
// segment copies whole table rows into its column range of the concatenated
// output.  Rows are moved with the widest vector (16/8/4 B per lane) the
// segment's dim, column offset and the output stride allow; `threads per row`
// lanes cover one row so a 128-float row is one 512-B coalesced read by 32
// lanes.  The op is HBM-bound (algorithmic bytes per row: 2*dim*4 + 4).
#include "tt_common.h"

namespace tt {
namespace {

constexpr int kGatherThreads = 256;
constexpr int kGatherIters = 4;  // row passes per block

struct GatherSeg {
  const float* table;
  const int32_t* ids;
  int64_t num_rows;
  int32_t dim;
  int32_t col_offset;
  int32_t vec;           // floats per lane: 4, 2 or 1
  int32_t tpr;           // threads per row = dim / vec
  int32_t rows_per_pass; // kGatherThreads / tpr
  int32_t block_begin;   // first block of this segment in the flat grid
};

struct GatherArgs {
  GatherSeg seg[TT_MAX_SEGMENTS];
  int32_t num_segs;
  int64_t batch;
  float* out;
  int64_t out_stride;
};

template <int VEC>
__device__ __forceinline__ void copy_vec(float* dst, const float* src, bool valid) {
  if constexpr (VEC == 4) {
    float4 v = valid ? *reinterpret_cast<const float4*>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(dst) = v;
  } else if constexpr (VEC == 2) {
    float2 v = valid ? *reinterpret_cast<const float2*>(src) : make_float2(0.f, 0.f);
    *reinterpret_cast<float2*>(dst) = v;
  } else {
    *dst = valid ? *src : 0.f;
  }
}

template <int VEC>
__device__ __forceinline__ void gather_segment(const GatherArgs& a, const GatherSeg& s, int local_block) {
  const int t = threadIdx.x;
  const int row_in_pass = t / s.tpr;
  const int lane_in_row = t - row_in_pass * s.tpr;
  if (row_in_pass >= s.rows_per_pass) return;
  const int64_t row0 = static_cast<int64_t>(local_block) * s.rows_per_pass * kGatherIters;
#pragma unroll
  for (int it = 0; it < kGatherIters; ++it) {
    const int64_t b = row0 + static_cast<int64_t>(it) * s.rows_per_pass + row_in_pass;
    if (b >= a.batch) return;
    int64_t r;
    bool valid;
    if (s.ids) {
      r = s.ids[b];
      valid = (r >= 0) && (r < s.num_rows);
    } else {  // numeric pass-through column: table is the [batch] value vector
      r = b;
      valid = true;
    }
    const int col = lane_in_row * VEC;
    const float* src = s.table + (valid ? r : 0) * static_cast<int64_t>(s.dim) + col;
    float* dst = a.out + b * a.out_stride + s.col_offset + col;
    copy_vec<VEC>(dst, src, valid);
  }
}

__global__ void __launch_bounds__(kGatherThreads) gather_grouped_kernel(const GatherArgs a) {
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

int pick_vec(const tt_gather_segment& s, const float* out, int64_t out_stride) {
  const int dim = s.ids ? s.dim : 1;
  for (int v = 4; v > 1; v >>= 1) {
    if (dim % v) continue;
    if (s.col_offset % v) continue;
    if (out_stride % v) continue;
    if (reinterpret_cast<uintptr_t>(out) % (4 * v)) continue;
    if (reinterpret_cast<uintptr_t>(s.table) % (4 * v)) continue;
    return v;
  }
  return 1;
}

}  // namespace
}  // namespace tt

extern "C" int tt_gather_grouped(const tt_gather_segment* segs, int32_t num_segs,
                                 int64_t batch, float* out, int64_t out_stride,
                                 tt_stream_t stream) {
  using namespace tt;
  clear_error();
  TT_REQUIRE(segs != nullptr, "tt_gather_grouped: segs is NULL");
  TT_REQUIRE(num_segs >= 1 && num_segs <= TT_MAX_SEGMENTS,
             "tt_gather_grouped: num_segs=%d outside [1,%d]", num_segs, TT_MAX_SEGMENTS);
  TT_REQUIRE(batch >= 0, "tt_gather_grouped: negative batch");
  TT_REQUIRE(out != nullptr || batch == 0, "tt_gather_grouped: out is NULL");
  if (batch == 0) return TT_OK;
  GatherArgs a{};
  a.num_segs = num_segs;
  a.batch = batch;
  a.out = out;
  a.out_stride = out_stride;
  int32_t blocks = 0;
  for (int i = 0; i < num_segs; ++i) {
    const tt_gather_segment& s = segs[i];
    TT_REQUIRE(s.table != nullptr, "tt_gather_grouped: segment %d table is NULL", i);
    const int dim = s.ids ? s.dim : 1;
    TT_REQUIRE(dim >= 1 && dim <= 4 * kGatherThreads,
               "tt_gather_grouped: segment %d dim=%d outside [1,%d]", i, s.dim, 4 * kGatherThreads);
    TT_REQUIRE(s.ids == nullptr || s.num_rows >= 1,
               "tt_gather_grouped: segment %d has an empty table", i);
    TT_REQUIRE(s.col_offset >= 0 && s.col_offset + dim <= out_stride,
               "tt_gather_grouped: segment %d columns [%d,%d) exceed out_stride %lld", i,
               s.col_offset, s.col_offset + dim, static_cast<long long>(out_stride));
    const int vec = pick_vec(s, out, out_stride);
    const int tpr = dim / vec;
    TT_REQUIRE(tpr <= kGatherThreads, "tt_gather_grouped: segment %d dim too wide for vector %d", i, vec);
    GatherSeg& g = a.seg[i];
    g.table = s.table;
    g.ids = s.ids;
    g.num_rows = s.num_rows;
    g.dim = dim;
    g.col_offset = s.col_offset;
    g.vec = vec;
    g.tpr = tpr;
    g.rows_per_pass = kGatherThreads / tpr;
    g.block_begin = blocks;
    const int64_t rows_per_block = static_cast<int64_t>(g.rows_per_pass) * kGatherIters;
    const int64_t nb = ceil_div(batch, rows_per_block);
    TT_REQUIRE(blocks + nb < (1ll << 31), "tt_gather_grouped: grid too large");
    blocks += static_cast<int32_t>(nb);
  }
  hipLaunchKernelGGL(gather_grouped_kernel, dim3(blocks), dim3(kGatherThreads), 0,
                     to_stream(stream), a);
  TT_CHECK_LAUNCH();
  return TT_OK;
}
