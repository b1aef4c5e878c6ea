// Input pipeline on the device: batches assembled from a
// dataset resident in HBM.
//
// Reference: /root/reference/pkg/modelling/tfrecord_dataset.py:59-98 reads
// TFRecord shards, shuffles with a buffer of shuffle_size and batches
// (drop_remainder=False); the StringLookup then runs per batch inside the
// model (input_layer.py:33-36).  Here the encoded columns (int32 rows /
// float32 values, one 32-bit word per example and column) live in HBM for the
// whole run — H&M's ~31M transactions x 12 columns are ~1.5 GB of the 288 GB
// — and a step's batch is one gather by the epoch's permutation:
//   dst[c, b] = src[c, perm[*cursor + b]],   then *cursor += batch.
// The position lives in device memory, so the take can sit inside the
// replayed train-step graph: an epoch is nothing but graph replays.
#include "tt_common.h"

namespace tt {
namespace {

constexpr int kTakeThreads = 256;

// One thread per example: its permutation entry is read once, then every
// column's word; the writes of a wave are 256 contiguous bytes per column.
__global__ void __launch_bounds__(kTakeThreads)
    batch_take_kernel(const uint32_t* __restrict__ src, int64_t src_ld, int32_t ncols,
                      const int64_t* __restrict__ perm, int64_t n_rows, const int64_t* __restrict__ cursor,
                      int64_t batch, uint32_t* __restrict__ dst, int64_t dst_ld, int32_t* __restrict__ status) {
  const int64_t b = blockIdx.x * static_cast<int64_t>(kTakeThreads) + threadIdx.x;
  if (b >= batch) return;
  const int64_t pos = *cursor + b;
  int64_t r = (pos >= 0 && pos < n_rows) ? perm[pos] : -1;
  if (r < 0 || r >= n_rows) {
    // past the dataset (or a corrupt permutation): zero words and a flag the
    // host reads back (tt_batch_status); never a silent wrap-around
    if (status) atomicOr(status, 1);
    for (int32_t c = 0; c < ncols; ++c) dst[c * dst_ld + b] = 0u;
    return;
  }
  for (int32_t c = 0; c < ncols; ++c) dst[c * dst_ld + b] = src[c * src_ld + r];
}

__global__ void cursor_advance_kernel(int64_t* cursor, int64_t step) { *cursor += step; }

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" int tt_batch_take(const void* src, int64_t src_ld, int32_t ncols, const int64_t* perm, int64_t n_rows,
                             int64_t* cursor, int64_t batch, int32_t advance, void* dst, int64_t dst_ld,
                             int32_t* status, tt_stream_t stream) {
  clear_error();
  TT_REQUIRE(ncols >= 1, "tt_batch_take: ncols=%d < 1", ncols);
  TT_REQUIRE(batch >= 1 && n_rows >= 0, "tt_batch_take: bad batch / n_rows");
  TT_REQUIRE(src_ld >= n_rows && dst_ld >= batch, "tt_batch_take: leading dimensions too small");
  TT_REQUIRE(src && perm && cursor && dst, "tt_batch_take: NULL pointer");
  hipStream_t st = to_stream(stream);
  hipLaunchKernelGGL(batch_take_kernel, dim3(ceil_div(batch, kTakeThreads)), dim3(kTakeThreads), 0, st,
                     static_cast<const uint32_t*>(src), src_ld, ncols, perm, n_rows, cursor, batch,
                     static_cast<uint32_t*>(dst), dst_ld, status);
  TT_CHECK_LAUNCH();
  if (advance) {
    hipLaunchKernelGGL(cursor_advance_kernel, dim3(1), dim3(1), 0, st, cursor, batch);
    TT_CHECK_LAUNCH();
  }
  return TT_OK;
}
