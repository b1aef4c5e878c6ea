// Weight-image packing of the tower MLP GEMMs (tt_mlp_pack / _pack_many),
// shared by tt_mlp.hip and by tt_gather.hip's gather + pack launch
// (tt_gather_multi_pack): the images the step's forward reads, packed in the
// same launch as the towers' input gather.
#pragma once
#include "tt_common.h"

namespace tt {
namespace pack {

__device__ __forceinline__ unsigned bf16_bits(float v) {
  return static_cast<unsigned>(__builtin_bit_cast(unsigned short, static_cast<__bf16>(v)));
}
__device__ __forceinline__ float bf16_val(unsigned bits) { return __uint_as_float(bits << 16); }

// One thread per (k-step, column block, lane): 8 hi + 8 lo bf16 of
// B[k = 16 ks + 8 (lane >> 5) + j][n = 32 cb + (lane & 31)], j < 8, zero padded.
// trans: B = W^T with W [N, K] row-major (B[k][n] = W[n * ldw + k]).
// One lane's 8 consecutive k of column n, as bf16 hi and lo, into the image
// (fragment (ks, cb) of the B image, planes hi / lo).  All 8 loads are issued
// before any is used (branch-free: out-of-range elements read w[0], become 0).
__device__ __forceinline__ void pack_fragment(const float* __restrict__ w, int64_t ldw, int K, int N, int trans,
                                              int ks, int cb, int NB, int lane, __bf16* __restrict__ img) {
  const int n = 32 * cb + (lane & 31);
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 16 * ks + 8 * (lane >> 5) + j;
    const bool ok = k < K && n < N;
    const int64_t at = trans ? static_cast<int64_t>(n) * ldw + k : static_cast<int64_t>(k) * ldw + n;
    x[j] = w[ok ? at : 0];
  }
  unsigned hb[8], lb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 16 * ks + 8 * (lane >> 5) + j;
    const float v = (k < K && n < N) ? x[j] : 0.0f;
    hb[j] = bf16_bits(v);
    lb[j] = bf16_bits(v - bf16_val(hb[j]));
  }
  u32x4 hv, lv;
  hv.x = hb[0] | (hb[1] << 16); hv.y = hb[2] | (hb[3] << 16); hv.z = hb[4] | (hb[5] << 16); hv.w = hb[6] | (hb[7] << 16);
  lv.x = lb[0] | (lb[1] << 16); lv.y = lb[2] | (lb[3] << 16); lv.z = lb[4] | (lb[5] << 16); lv.w = lb[6] | (lb[7] << 16);
  const int64_t base = ((static_cast<int64_t>(ks) * NB + cb) * 2) * 64 + lane;
  reinterpret_cast<u32x4*>(img)[base] = hv;        // plane 0: hi
  reinterpret_cast<u32x4*>(img)[base + 64] = lv;   // plane 1: lo
}

// image k-steps padded to whole 64-deep stages, column blocks to 4 per wave row
struct PackJob {
  const float* w;
  int64_t ldw;
  int K, N, trans, KS, NB;
  __bf16* img;
  int64_t first;  // first thread of this job
};
constexpr int kMaxPackJobs = 8;
struct PackJobs {
  PackJob j[kMaxPackJobs];
  int n;
};

// The pack thread t of a PackJobs launch (t < total).
__device__ __forceinline__ void pack_many_thread(const PackJobs& jobs, int64_t t) {
  // jobs start on multiples of 64 threads: the job is wave-uniform (scalar search)
  const int64_t tw = (static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(t >> 6)))) << 6;
  int q = 0;
  while (q + 1 < jobs.n && tw >= jobs.j[q + 1].first) ++q;
  const PackJob& J = jobs.j[q];
  const int64_t u = t - J.first;
  const int lane = static_cast<int>(u & 63);
  const int cb = static_cast<int>((u >> 6) % J.NB);
  const int ks = static_cast<int>((u >> 6) / J.NB);
  pack_fragment(J.w, J.ldw, J.K, J.N, J.trans, ks, cb, J.NB, lane, J.img);
}

__host__ __device__ inline int mlp_ks(int K) { return (K + 63) / 64 * 4; }
__host__ __device__ inline int mlp_nb(int N) { return (N + 127) / 128 * 4; }

// Validated pack jobs of one call (the host side of tt_mlp_pack_many); TT_OK or
// an error code with the message set.  *total = the launch's threads.
inline int make_pack_jobs(const tt_mlp_pack_job* jobs, int32_t num_jobs, PackJobs* pj, int64_t* total,
                          const char* fn) {
  TT_REQUIRE(jobs && num_jobs >= 1 && num_jobs <= kMaxPackJobs, "%s: 1..%d jobs", fn, kMaxPackJobs);
  *pj = PackJobs{};
  pj->n = num_jobs;
  int64_t t = 0;
  for (int i = 0; i < num_jobs; ++i) {
    const tt_mlp_pack_job& j = jobs[i];
    TT_REQUIRE(j.w && j.img && j.K >= 1 && j.N >= 1, "%s: job %d: bad w/img/K/N", fn, i);
    TT_REQUIRE(j.ldw >= (j.trans ? j.K : j.N), "%s: job %d: ldw too small", fn, i);
    TT_REQUIRE(j.img_bytes >= static_cast<size_t>(mlp_ks(j.K)) * mlp_nb(j.N) * 2 * 64 * 8 * sizeof(__bf16),
               "%s: job %d: image too small", fn, i);
    PackJob& J = pj->j[i];
    J.w = j.w;
    J.ldw = j.ldw;
    J.K = j.K;
    J.N = j.N;
    J.trans = j.trans ? 1 : 0;
    J.KS = mlp_ks(j.K);
    J.NB = mlp_nb(j.N);
    J.img = static_cast<__bf16*>(j.img);
    J.first = t;
    t += static_cast<int64_t>(J.KS) * J.NB * 64;
  }
  *total = t;
  return TT_OK;
}

}  // namespace pack
}  // namespace tt
