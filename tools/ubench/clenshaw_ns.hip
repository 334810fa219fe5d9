// Micro-benchmark (not product code): Clenshaw rows with LDS-broadcast amplitude
// rows (ds_read_b128, 8 rows per iteration, as sg_sine_bank) for NS = 2/4/8
// independent chains per lane, at the occupancy the VGPR count allows.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ROWS = 32, TASKS = 16;

template <int NS>
__global__ __launch_bounds__(256) void k(const float* __restrict__ A, const float* __restrict__ X, float* __restrict__ Y) {
  __shared__ __attribute__((aligned(16))) float rows[4][ROWS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* la = rows[w];
  float acc = 0.f;
  for (int task = 0; task < TASKS; ++task) {
    if (lane < ROWS) la[lane] = A[(task * 7 + lane) & 1023];
    float al[NS], b1[NS], b2[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) { al[s] = X[(blockIdx.x * 256 + threadIdx.x + 64 * s) & 4095]; b1[s] = b2[s] = 0.f; }
#pragma unroll 1
    for (int r = ROWS - 8; r >= 0; r -= 8) {
      const float4 a4 = *reinterpret_cast<const float4*>(la + r + 4);
      const float4 a0 = *reinterpret_cast<const float4*>(la + r);
#define RW(a) _Pragma("unroll") for (int s = 0; s < NS; ++s) { const float b = fmaf(al[s], b1[s], (a) - b2[s]); b2[s] = b1[s]; b1[s] = b; }
      RW(a4.w) RW(a4.z) RW(a4.y) RW(a4.x) RW(a0.w) RW(a0.z) RW(a0.y) RW(a0.x)
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) acc += b1[s];
  }
  Y[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const int blocks = 256 * 4 * 16;
  float *A, *X, *Y;
  hipMalloc(&A, 4096 * 4); hipMalloc(&X, 4096 * 4); hipMalloc(&Y, (size_t)blocks * 256 * 4);
  hipMemset(A, 0, 4096 * 4); hipMemset(X, 0, 4096 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int ns : {2, 4, 8}) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      if (ns == 2) k<2><<<blocks, 256>>>(A, X, Y);
      if (ns == 4) k<4><<<blocks, 256>>>(A, X, Y);
      if (ns == 8) k<8><<<blocks, 256>>>(A, X, Y);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    const double terms = (double)blocks * 256 * ns * ROWS * TASKS;
    printf("lds-bcast NS=%d  %.3f ms  %.2f T terms/s  %.2f lane-instr/term at peak\n", ns, best, terms / best / 1e9,
           78.6e12 / (terms / best * 1e3));
  }
  return 0;
}
