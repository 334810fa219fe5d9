// Host-to-device upload of planner-sized host blocks: pageable vs registered
// (hipHostRegister) vs hipHostMalloc, and what pinning costs. Development probe
// for the plan upload.
//   hipcc -O2 --offload-arch=gfx950 tools/ubench/pin_probe.cpp -o tools/ubench/pin_probe
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t GB = size_t(1) << 30;
  const size_t n = (argc > 1 ? std::atoll(argv[1]) : 2) * GB;
  void* d = nullptr;
  CK(hipMalloc(&d, n));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto h2d = [&](const void* h, const char* what) {
    double best = 1e9;
    for (int r = 0; r < 3; ++r) {
      const double t = now();
      CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      best = std::min(best, now() - t);
    }
    std::printf("%-34s %7.3f s  %6.1f GB/s\n", what, best, n / best / 1e9);
  };
  // pageable, huge-page advised (the planner's bulk blocks)
  double t = now();
  void* h = std::aligned_alloc(size_t(2) << 20, n);
  (void)madvise(h, n, MADV_HUGEPAGE);
  std::memset(h, 1, n);
  std::printf("%-34s %7.3f s\n", "aligned_alloc + first touch", now() - t);
  h2d(h, "H2D pageable");
  t = now();
  CK(hipHostRegister(h, n, hipHostRegisterDefault));
  std::printf("%-34s %7.3f s\n", "hipHostRegister", now() - t);
  h2d(h, "H2D registered");
  t = now();
  CK(hipHostUnregister(h));
  std::printf("%-34s %7.3f s\n", "hipHostUnregister", now() - t);
  h2d(h, "H2D pageable again");
  std::free(h);
  // pinned from the allocator
  void* p = nullptr;
  t = now();
  CK(hipHostMalloc(&p, n, hipHostMallocDefault));
  std::printf("%-34s %7.3f s\n", "hipHostMalloc", now() - t);
  t = now();
  std::memset(p, 2, n);
  std::printf("%-34s %7.3f s\n", "hipHostMalloc first touch", now() - t);
  t = now();
  std::memset(p, 3, n);
  std::printf("%-34s %7.3f s\n", "second touch", now() - t);
  h2d(p, "H2D hipHostMalloc");
  t = now();
  CK(hipHostFree(p));
  std::printf("%-34s %7.3f s\n", "hipHostFree", now() - t);
  CK(hipFree(d));
  return 0;
}
