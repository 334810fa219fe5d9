// fetch_calib.hip — calibration of rocprofv3's FETCH_SIZE on gfx950 for the access
// patterns of the sine-bank kernels (MI355X_MICROARCH.md: "other access widths are
// uncalibrated"). Each kernel reads a known number of distinct bytes once; the
// output line gives the bytes, and the FETCH_SIZE of the same dispatch (rocprofv3
// --pmc FETCH_SIZE) divided by them is the counter's factor for the pattern.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d out -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

struct Desc {  // a 128-B wave-uniform descriptor (SgWTask's size)
  double v[16];
};

// 1. 16 B per lane, coalesced streaming (the guide's calibrated case)
__global__ void k_stream16(const float4* __restrict__ in, float* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float4 v = i < n ? in[i] : make_float4(0, 0, 0, 0);
  if (v.x + v.y + v.z + v.w == 12345.f) out[0] = v.x;
}
// 2. one 128-B descriptor per wave through a wave-uniform pointer (scalar loads)
__global__ void k_desc128(const Desc* __restrict__ d, float* __restrict__ out, size_t nw) {
  const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w >= nw) return;
  const Desc D = d[w];
  double s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += D.v[k];
  if (s == 12345.0 && (threadIdx.x & 63) == 0) out[0] = (float)s;
}
// 3. R contiguous floats per wave, 4 B per lane (a staged amplitude column), columns
//    at a stride of R floats (every byte read once)
template <int R>
__global__ void k_rows4(const float* __restrict__ a, float* __restrict__ out, size_t nw) {
  const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w >= nw) return;
  const int lane = threadIdx.x & 63;
  float s = 0.f;
  for (int r = lane; r < R; r += 64) s += a[w * R + r];
  if (s == 12345.f) out[0] = s;
}

template <class F>
static void run(const char* name, F launch, double bytes) {
  launch();
  if (hipDeviceSynchronize() != hipSuccess) { std::printf("%s failed\n", name); std::exit(1); }
  std::printf("%s bytes %.0f\n", name, bytes);
}

int main() {
  const size_t N = (size_t)256 << 20;  // 256 MiB per buffer (> the 256 MiB L3 with the others)
  char *a, *b;
  float* out;
  if (hipMalloc(&a, N) != hipSuccess || hipMalloc(&b, N) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(a, 0, N);
  hipMemset(b, 0, N);
  // flush: stream the other buffer between runs so nothing is L3-resident
  auto flush = [&]() { k_stream16<<<(unsigned)(N / 16 / 256), 256>>>((const float4*)b, out, N / 16); hipDeviceSynchronize(); };
  for (int rep = 0; rep < 2; ++rep) {
    flush();
    run("stream16", [&]() { k_stream16<<<(unsigned)(N / 16 / 256), 256>>>((const float4*)a, out, N / 16); }, (double)N);
    flush();
    const size_t nd = N / sizeof(Desc);
    run("desc128", [&]() { k_desc128<<<(unsigned)((nd + 3) / 4), 256>>>((const Desc*)a, out, nd); }, (double)nd * 128);
    flush();
    const size_t n60 = N / (60 * 4);
    run("rows4_R60", [&]() { k_rows4<60><<<(unsigned)((n60 + 3) / 4), 256>>>((const float*)a, out, n60); }, (double)n60 * 240);
    flush();
    const size_t n96 = N / (96 * 4);
    run("rows4_R96", [&]() { k_rows4<96><<<(unsigned)((n96 + 3) / 4), 256>>>((const float*)a, out, n96); }, (double)n96 * 384);
    flush();
    const size_t n32 = N / (32 * 4);
    run("rows4_R32", [&]() { k_rows4<32><<<(unsigned)((n32 + 3) / 4), 256>>>((const float*)a, out, n32); }, (double)n32 * 128);
  }
  hipFree(a);
  hipFree(b);
  hipFree(out);
  return 0;
}
