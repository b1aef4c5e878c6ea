// Version string and thread-local error reporting for the libtt C ABI.
#include <cstdio>
#include <cstring>

#include "tt_common.h"

namespace tt {

static thread_local char g_last_error[1024] = {0};

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return code;
}

void clear_error() { g_last_error[0] = 0; }

// One-shot kernel timing probes (tt_probe_arm): the next launch of the armed
// kernel on this thread is bracketed by the caller's events.
static thread_local hipEvent_t g_probe[TT_PROBE_COUNT][2] = {};
static thread_local int g_probe_reps[TT_PROBE_COUNT] = {};

int probe_reps(int kernel) { return g_probe[kernel][0] && g_probe_reps[kernel] > 1 ? g_probe_reps[kernel] : 1; }

void probe_begin(int kernel, hipStream_t st) {
  if (g_probe[kernel][0]) (void)hipEventRecord(g_probe[kernel][0], st);
}

void probe_end(int kernel, hipStream_t st) {
  if (g_probe[kernel][1]) (void)hipEventRecord(g_probe[kernel][1], st);
  g_probe[kernel][0] = g_probe[kernel][1] = nullptr;
  g_probe_reps[kernel] = 0;
}

}  // namespace tt

extern "C" const char* tt_version(void) { return "tt 0.1.0 gfx950"; }

extern "C" const char* tt_last_error(void) { return tt::g_last_error; }

extern "C" int tt_probe_arm(int32_t kernel, void* ev_start, void* ev_stop) {
  tt::clear_error();
  TT_REQUIRE(kernel >= 0 && kernel < TT_PROBE_COUNT, "tt_probe_arm: unknown kernel %d", kernel);
  tt::g_probe[kernel][0] = static_cast<hipEvent_t>(ev_start);
  tt::g_probe[kernel][1] = static_cast<hipEvent_t>(ev_stop);
  tt::g_probe_reps[kernel] = 1;
  return TT_OK;
}

extern "C" int tt_probe_arm_repeat(int32_t kernel, void* ev_start, void* ev_stop, int32_t reps) {
  tt::clear_error();
  TT_REQUIRE(kernel >= 0 && kernel < TT_PROBE_COUNT, "tt_probe_arm_repeat: unknown kernel %d", kernel);
  TT_REQUIRE(reps >= 1 && reps <= 1000, "tt_probe_arm_repeat: reps %d outside [1, 1000]", reps);
  tt::g_probe[kernel][0] = static_cast<hipEvent_t>(ev_start);
  tt::g_probe[kernel][1] = static_cast<hipEvent_t>(ev_stop);
  tt::g_probe_reps[kernel] = reps;
  return TT_OK;
}
