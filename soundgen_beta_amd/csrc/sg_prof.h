// sg_prof.h — planner section timers (host). Enabled by SG_PLAN_PROF=1 in the
// environment: sg_plan_batch prints the accumulated seconds per section to
// stderr. Off by default (one relaxed load per scope).
#pragma once
#include <atomic>
#include <chrono>
#include <cstdint>

namespace sg {

enum ProfId { PF_HARM, PF_ROLLOFF, PF_CONTOUR, PF_ENVELOPE, PF_NOISE, PF_FILTER, PF_FINALIZE, PF_SPEC, PF_FRY, PF_XFADE,
              PF_EMIT, PF_TASKS, PF_TILES, PF_SOUNDGEN, PF_ENV_UPS, PF_ENV_STOCH, PF_ENV_TERMS, PF_N };
extern std::atomic<int64_t> g_prof_ns[PF_N];
extern bool g_prof_on;

struct ProfScope {
  int id;
  std::chrono::steady_clock::time_point t0;
  explicit ProfScope(int i) : id(i) {
    if (g_prof_on) t0 = std::chrono::steady_clock::now();
  }
  ~ProfScope() {
    if (g_prof_on)
      g_prof_ns[id].fetch_add(
          std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count(),
          std::memory_order_relaxed);
  }
};

}  // namespace sg
