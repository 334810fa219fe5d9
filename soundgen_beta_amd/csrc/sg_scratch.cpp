// sg_scratch.cpp — the planner's per-thread scratch pool (sg_rmath.h) and the
// huge-page bulk allocation (NoInitAlloc, sg_plan.h).
// Blocks of 32 KB and up are rounded to a power of two and parked on the
// freeing thread's free list (up to SCRATCH_CAP bytes per thread) instead of
// going back to glibc, which maps and unmaps blocks that large: with 16
// planning threads the unmaps' TLB shootdowns and the refaults of fresh zero
// pages were a quarter of planning time. The pool is released when its thread
// ends (planner worker threads live for one sg_plan_batch) or by
// scratch_trim() (the calling thread, at the end of sg_plan_batch).
#include <sys/mman.h>

#include <cstdlib>
#include <new>
#include <vector>

#include "sg_rmath.h"

namespace sg {
namespace {

constexpr size_t SCRATCH_MIN = size_t(1) << 15;
constexpr size_t SCRATCH_CAP = size_t(1) << 30;
constexpr int NCLASS = 48;

struct Pool {
  std::vector<void*> bins[NCLASS];
  size_t held = 0;
  void clear() noexcept {
    for (auto& b : bins) {
      for (void* p : b) std::free(p);
      b.clear();
    }
    held = 0;
  }
  ~Pool() { clear(); }
};

struct PoolSlot {
  Pool* p = nullptr;
  bool dead = false;  // thread-exit destruction done: later frees go to glibc
  ~PoolSlot() {
    delete p;
    p = nullptr;
    dead = true;
  }
};
thread_local PoolSlot slot;

inline int size_class(size_t bytes) {
  int c = 0;
  while ((size_t(1) << c) < bytes) ++c;
  return c;
}

}  // namespace

void* scratch_alloc(size_t bytes) {
  if (bytes < SCRATCH_MIN) {
    void* q = std::malloc(bytes ? bytes : 1);
    if (!q) throw std::bad_alloc();
    return q;
  }
  const int c = size_class(bytes);
  if (!slot.dead) {
    if (!slot.p) slot.p = new Pool();
    auto& b = slot.p->bins[c];
    if (!b.empty()) {
      void* q = b.back();
      b.pop_back();
      slot.p->held -= size_t(1) << c;
      return q;
    }
  }
  void* q = std::malloc(size_t(1) << c);
  if (!q) throw std::bad_alloc();
  return q;
}

void scratch_free(void* q, size_t bytes) noexcept {
  if (!q) return;
  if (bytes < SCRATCH_MIN || slot.dead) {
    std::free(q);
    return;
  }
  const int c = size_class(bytes);
  if (!slot.p || slot.p->held + (size_t(1) << c) > SCRATCH_CAP) {
    std::free(q);
    return;
  }
  try {
    slot.p->bins[c].push_back(q);
    slot.p->held += size_t(1) << c;
  } catch (...) {
    std::free(q);
  }
}

void* bulk_alloc(size_t bytes) {
  constexpr size_t HUGE = size_t(2) << 20;
  const size_t sz = (bytes + HUGE - 1) / HUGE * HUGE;
  void* q = std::aligned_alloc(HUGE, sz);
  if (!q) throw std::bad_alloc();
  static const bool no_thp = std::getenv("SG_NO_THP") != nullptr;  // experiment knob
  if (!no_thp) (void)madvise(q, sz, MADV_HUGEPAGE);  // advisory: 4 KB pages when THP is off
  return q;
}

void bulk_free(void* q, size_t) noexcept { std::free(q); }

void scratch_trim() noexcept {
  if (slot.p) slot.p->clear();
}

}  // namespace sg
