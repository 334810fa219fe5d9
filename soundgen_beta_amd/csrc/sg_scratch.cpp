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
#include <map>
#include <mutex>
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

// Freed bulk blocks are kept for the next plan (up to SG_HOST_CACHE_MB, default
// 8192 / LOCAL_WORLD_SIZE: one rank per GPU shares the node's memory; at least
// 1024; sg_host_cache_trim() returns them): a plan's host arrays are GBs, freed once uploaded, and the next plan
// of a batch asks for blocks of about the same sizes; reusing resident pages
// skips the page faults and the kernel's zeroing of fresh ones. Blocks are
// sized in classes of 1/16 of a power of two (<= 6.25 % slack), so a freed
// block serves any request of its class.
namespace {
constexpr size_t HUGE_PAGE = size_t(2) << 20;
size_t bulk_class(size_t bytes) {
  size_t sz = (bytes + HUGE_PAGE - 1) / HUGE_PAGE * HUGE_PAGE;
  int top = 63 - __builtin_clzll(sz);
  const size_t step = top > 4 ? size_t(1) << (top - 4) : 1;
  sz = (sz + step - 1) / step * step;
  return (sz + HUGE_PAGE - 1) / HUGE_PAGE * HUGE_PAGE;
}
struct BulkCache {
  std::mutex mu;
  std::multimap<size_t, void*> blocks;
  size_t bytes = 0;
  const size_t cap = [] {
    const char* e = std::getenv("SG_HOST_CACHE_MB");
    if (e) return (size_t)std::atoll(e) << 20;
    const char* w = std::getenv("LOCAL_WORLD_SIZE");
    const long long ranks = w ? std::max(1LL, std::atoll(w)) : 1;
    return (size_t)std::max(1024LL, 8192LL / ranks) << 20;
  }();
  ~BulkCache() {
    for (auto& b : blocks) std::free(b.second);
  }
};
BulkCache& bulk_cache() {
  static BulkCache* c = new BulkCache();  // never destroyed: frees may run on detached threads at exit
  return *c;
}
}  // namespace

void* bulk_alloc(size_t bytes) {
  const size_t sz = bulk_class(bytes);
  {
    BulkCache& c = bulk_cache();
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.blocks.find(sz);
    if (it != c.blocks.end()) {
      void* q = it->second;
      c.blocks.erase(it);
      c.bytes -= sz;
      return q;
    }
  }
  void* q = std::aligned_alloc(HUGE_PAGE, sz);
  if (!q) throw std::bad_alloc();
  (void)madvise(q, sz, MADV_HUGEPAGE);  // advisory: 4 KB pages when THP is off
  return q;
}

void bulk_free(void* q, size_t bytes) noexcept {
  if (!q) return;
  const size_t sz = bulk_class(bytes);
  BulkCache& c = bulk_cache();
  {
    std::lock_guard<std::mutex> g(c.mu);
    if (c.bytes + sz <= c.cap) {
      try {
        c.blocks.emplace(sz, q);
        c.bytes += sz;
        return;
      } catch (...) {
      }
    }
  }
  std::free(q);
}

size_t bulk_trim() noexcept {
  BulkCache& c = bulk_cache();
  std::multimap<size_t, void*> blocks;
  size_t held = 0;
  {
    std::lock_guard<std::mutex> g(c.mu);
    blocks.swap(c.blocks);
    held = c.bytes;
    c.bytes = 0;
  }
  for (auto& b : blocks) std::free(b.second);
  return held;
}

void scratch_trim() noexcept {
  if (slot.p) slot.p->clear();
}

}  // namespace sg
