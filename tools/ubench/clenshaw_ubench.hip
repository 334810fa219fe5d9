// Micro-benchmark of the sine-bank inner loop forms on gfx950 (not product code):
// Clenshaw rows b = A_r + al*b1 - b2 with the row amplitude broadcast by
//  (0) DPP row_newbcast folded into v_sub_f32_dpp, (1) an SGPR operand,
//  (2) packed v_pk_fma/v_pk_add with SGPR splat, (3) plain VGPR (upper bound),
// and the accuracy of the hardware v_sin_f32 / v_cos_f32 against fp64.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
#define BC(v, K) __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, (v)), 0x150 + (K), 0xf, 0xf, true))

constexpr int ROWS = 64, ITERS = 64, NS = 2;

template <int MODE>
__global__ __launch_bounds__(256) void k(const float* __restrict__ A, const float* __restrict__ X, float* __restrict__ Y) {
  const int lane = threadIdx.x & 63;
  const int gid = blockIdx.x * 256 + threadIdx.x;
  float al[NS], b1[NS], b2[NS];
  for (int s = 0; s < NS; ++s) { al[s] = X[(gid * NS + s) & 4095]; b1[s] = b2[s] = 0.f; }
  float va[8];
  for (int g = 0; g < 8; ++g) va[g] = A[8 * g + (lane & 7)];
  for (int it = 0; it < ITERS; ++it) {
    if (MODE == 0) {
#define R0(g, K) for (int s = 0; s < NS; ++s) { const float b = fmaf(al[s], b1[s], BC(va[g], K) - b2[s]); b2[s] = b1[s]; b1[s] = b; }
#define G0(g) R0(g,7) R0(g,6) R0(g,5) R0(g,4) R0(g,3) R0(g,2) R0(g,1) R0(g,0)
      G0(7) G0(6) G0(5) G0(4) G0(3) G0(2) G0(1) G0(0)
    } else if (MODE == 1) {
#pragma unroll
      for (int r = ROWS - 1; r >= 0; --r) {
        const float a = A[r + (it & 1)];  // wave-uniform: SGPR
        for (int s = 0; s < NS; ++s) { const float b = fmaf(al[s], b1[s], a - b2[s]); b2[s] = b1[s]; b1[s] = b; }
      }
    } else if (MODE == 2) {
      f2 al2 = {al[0], al[1]}, c1 = {b1[0], b1[1]}, c2 = {b2[0], b2[1]};
#pragma unroll
      for (int r = ROWS - 1; r >= 0; --r) {
        const float a = A[r + (it & 1)];
        const f2 aa = {a, a};
        const f2 b = __builtin_elementwise_fma(al2, c1, aa - c2); c2 = c1; c1 = b;
      }
      b1[0] = c1.x; b1[1] = c1.y; b2[0] = c2.x; b2[1] = c2.y;
    } else {
#pragma unroll
      for (int r = ROWS - 1; r >= 0; --r) {
        const float a = va[r & 7];
        for (int s = 0; s < NS; ++s) { const float b = fmaf(al[s], b1[s], a - b2[s]); b2[s] = b1[s]; b1[s] = b; }
      }
    }
  }
  float y = 0.f;
  for (int s = 0; s < NS; ++s) y += b1[s] + b2[s];
  Y[gid] = y;
}

__global__ void k_sin(const float* __restrict__ X, float* __restrict__ S, float* __restrict__ Cc, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  S[i] = __builtin_amdgcn_sinf(X[i]);
  Cc[i] = __builtin_amdgcn_cosf(X[i]);
}

int main() {
  const int blocks = 256 * 8 * 4;
  float *A, *X, *Y;
  hipMalloc(&A, 4096 * 4); hipMalloc(&X, 4096 * 4); hipMalloc(&Y, (size_t)blocks * 256 * 4);
  std::vector<float> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = 1.9f * std::cos(0.001f * i);
  hipMemcpy(A, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  hipMemcpy(X, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[4] = {"dpp-fold", "sgpr", "packed-sgpr", "vgpr"};
  for (int mode = 0; mode < 4; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) k<0><<<blocks, 256>>>(A, X, Y);
      if (mode == 1) k<1><<<blocks, 256>>>(A, X, Y);
      if (mode == 2) k<2><<<blocks, 256>>>(A, X, Y);
      if (mode == 3) k<3><<<blocks, 256>>>(A, X, Y);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
    }
    const double terms = (double)blocks * 256 * NS * ROWS * ITERS;  // (sample, row) terms
    printf("%-12s %.3f ms  %.2f T sample-rows/s  (%.2f lane-instr/term at the 78.6 T lane-op/s peak)\n", names[mode], best,
           terms / best / 1e9, 78.6e12 / (terms / best * 1e3));
  }
  // hardware sin/cos accuracy (input in revolutions)
  const int n = 1 << 20;
  std::vector<float> x(n), s(n), c(n);
  for (int i = 0; i < n; ++i) x[i] = -0.5f + (float)i / n;
  float *dX, *dS, *dC; hipMalloc(&dX, n * 4); hipMalloc(&dS, n * 4); hipMalloc(&dC, n * 4);
  hipMemcpy(dX, x.data(), n * 4, hipMemcpyHostToDevice);
  k_sin<<<(n + 255) / 256, 256>>>(dX, dS, dC, n);
  hipMemcpy(s.data(), dS, n * 4, hipMemcpyDeviceToHost); hipMemcpy(c.data(), dC, n * 4, hipMemcpyDeviceToHost);
  double es = 0, ec = 0, rs = 0;
  for (int i = 0; i < n; ++i) {
    const double t = 2 * M_PI * (double)x[i];
    es = std::fmax(es, std::fabs(s[i] - std::sin(t)));
    ec = std::fmax(ec, std::fabs(c[i] - std::cos(t)));
    rs += (s[i] - std::sin(t)) * (s[i] - std::sin(t));
  }
  printf("v_sin_f32 max abs err %.3g (rms %.3g), v_cos_f32 max abs err %.3g\n", es, std::sqrt(rs / n), ec);
  return 0;
}
