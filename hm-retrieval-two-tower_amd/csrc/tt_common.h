// Shared helpers for libtt (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>

#include "tt.h"

namespace tt {

// ---- host-side error plumbing -------------------------------------------
int fail(int code, const char* fmt, ...);
void clear_error();
// Timing probes armed by tt_probe_arm (no-ops unless armed).
void probe_begin(int kernel, hipStream_t st);
void probe_end(int kernel, hipStream_t st);
int probe_reps(int kernel);  // launches to issue between the armed events (1 unless armed with reps)

#define TT_REQUIRE(cond, ...)                                  \
  do {                                                         \
    if (!(cond)) return ::tt::fail(TT_ERR_BAD_ARG, __VA_ARGS__); \
  } while (0)

#define TT_CHECK_HIP(expr)                                                   \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess)                                                    \
      return ::tt::fail(TT_ERR_HIP, "%s failed: %s", #expr,                 \
                        hipGetErrorString(e_));                              \
  } while (0)

#define TT_CHECK_LAUNCH() TT_CHECK_HIP(hipGetLastError())

inline hipStream_t to_stream(tt_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// Bump allocator over a caller-provided workspace; 256-B aligned carves.
struct Carver {
  char* base;
  size_t cap;
  size_t off = 0;
  Carver(void* p, size_t c) : base(static_cast<char*>(p)), cap(c) {}
  template <typename T>
  T* take(int64_t count) {
    size_t bytes = static_cast<size_t>(count) * sizeof(T);
    size_t start = (off + 255) & ~size_t(255);
    off = start + bytes;
    return base ? reinterpret_cast<T*>(base + start) : nullptr;
  }
  size_t used() const { return (off + 255) & ~size_t(255); }
};

// rocPRIM radix sorts of the sparse / routing paths.  Below the merge limit
// rocPRIM sorts with block sort + ~8 merge passes (our id sorts are 10^5-10^6
// keys); a limit of 0 forces onesweep (histogram + one pass per 8-bit digit).
// Measured at C3 (180k keys): the train step takes 0.614 ms with the merge
// path, 0.667 ms with onesweep, so rocPRIM's default limit stays.
#ifndef TT_SORT_MERGE_LIMIT
#define TT_SORT_MERGE_LIMIT (1024 * 1024)
#endif
#if defined(ROCPRIM_VERSION)
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, TT_SORT_MERGE_LIMIT>;
#endif

// ---- device-side helpers -------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  bf16x2 v = {static_cast<__bf16>(lo), static_cast<__bf16>(hi)};
  return __builtin_bit_cast(unsigned, v);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Workgroup barrier for LDS hand-offs only: this wave's LDS operations are
// complete (lgkmcnt(0)), global loads stay in flight.  __syncthreads() also
// waits vmcnt(0), which drains every prefetch a pipelined loop has issued.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt(63) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
}

// Sum over the 64 lanes of a wave (every lane receives the total).
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  return v;
}
__device__ __forceinline__ float wave_max_f32(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, kWave));
  return v;
}

// Order-preserving map float -> uint32 (larger float -> larger uint).
// -0.0 is canonicalised to +0.0 first so that it ties with +0.0, as float
// comparison (and tf.math.top_k) treats them.
__device__ __forceinline__ unsigned float_order_key(float f) {
  f = f + 0.0f;
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float order_key_float(unsigned k) {
  unsigned u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

}  // namespace tt
