// sg_wav.hip — the output writer of soundgen(savePath = ...) and morph(savePath = ...)
// (R/soundgen.R:854-856, R/morph.R:203-206): seewave::savewav(wave, f)
// (seewave_2.0.5.tar.gz::seewave/R/seewave.r:5192-5229) builds a 16-bit Wave and
// calls tuneR::normalize(unit = "16", level = max(wave) if <= 1 else 1)
// (tuneR_1.3.2.tar.gz::tuneR/R/normalize.R:5-64):
//   x <- x - mean(x); m <- max(abs(range(x)));
//   if (m > all.equal's 1.5e-8) x <- level * x / m;  x <- round(x * 32767)
// then tuneR::writeWave (tuneR/R/writeWave.R) writes the WAVE_FORMAT_EXTENSIBLE
// file. With savewav(rescale = c(lower, upper)) seewave::rescale
// ((x - min) * nrange / (max - min) - nrange / 2) replaces normalize and
// writeWave's as.integer truncates.
//
// Device part, per call of a batch: sg_pcm_stats (one workgroup per call: one
// pass for the sum as a double-double, min and max; mean and the scale follow
// in fp64 exactly as R rounds them), then sg_pcm_convert (tiles of 4096
// samples: read fp32 or fp64, R's per-sample fp64 arithmetic, round half to
// even, write int16 — half the bytes of the fp32 waveform cross PCIe).
// HBM-bound: 2 reads + 1 write of 2 B per sample.
#include <hip/hip_runtime.h>

#include "sg_dev.h"

namespace {

__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}

struct DD {
  double hi, lo;
};
__device__ __forceinline__ DD dd_add(DD x, DD y) {
  double s, e;
  two_sum(x.hi, y.hi, s, e);
  e += x.lo + y.lo;
  DD r;
  two_sum(s, e, r.hi, r.lo);
  return r;
}

template <class T>
__device__ void pcm_stats(const T* __restrict__ in, int64_t off, int64_t n, int mode, double nrange,
                          SgPcmStat* __restrict__ out) {
  DD acc{0.0, 0.0};
  double mn = INFINITY, mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const double x = (double)in[off + i];
    double s, e;
    two_sum(acc.hi, x, s, e);
    acc.hi = s;
    acc.lo += e;
    mn = fmin(mn, x);
    mx = fmax(mx, x);
  }
  __shared__ double sh[3][256];
  __shared__ double shl[256];
  sh[0][threadIdx.x] = acc.hi;
  shl[threadIdx.x] = acc.lo;
  sh[1][threadIdx.x] = mn;
  sh[2][threadIdx.x] = mx;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const DD r = dd_add(DD{sh[0][threadIdx.x], shl[threadIdx.x]}, DD{sh[0][threadIdx.x + w], shl[threadIdx.x + w]});
      sh[0][threadIdx.x] = r.hi;
      shl[threadIdx.x] = r.lo;
      sh[1][threadIdx.x] = fmin(sh[1][threadIdx.x], sh[1][threadIdx.x + w]);
      sh[2][threadIdx.x] = fmax(sh[2][threadIdx.x], sh[2][threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  SgPcmStat S{};
  S.min = sh[1][0];
  S.max = sh[2][0];
  if (mode == SG_PCM_NORMALIZE) {
    // mean(x): R sums in long double and corrects once; the exact sum in a
    // double-double rounds to the same double
    const double mean = n > 0 ? (sh[0][0] + shl[0]) / (double)n : 0.0;
    S.mean = mean;
    S.level = S.max <= 1 ? S.max : 1.0;  // savewav: max(wave@left), signed
    // max(abs(range(x - mean))): subtraction is monotone, so the extremes stay extremes
    S.m = fmax(fabs(S.max - mean), fabs(S.min - mean));
    S.scale = S.m > 1.5e-8 ? 1 : 0;  // !isTRUE(all.equal(m, 0))
  } else {
    S.m = S.max - S.min;
    S.level = nrange;
  }
  *out = S;
}

}  // namespace

extern "C" __global__ __launch_bounds__(256) void sg_pcm_stats_f32(const float* __restrict__ in,
                                                                   const SgPcmCall* __restrict__ calls, int mode,
                                                                   double nrange, SgPcmStat* __restrict__ stats) {
  const SgPcmCall C = calls[blockIdx.x];
  pcm_stats(in, C.off, C.len, mode, nrange, stats + blockIdx.x);
}
extern "C" __global__ __launch_bounds__(256) void sg_pcm_stats_f64(const double* __restrict__ in,
                                                                   const SgPcmCall* __restrict__ calls, int mode,
                                                                   double nrange, SgPcmStat* __restrict__ stats) {
  const SgPcmCall C = calls[blockIdx.x];
  pcm_stats(in, C.off, C.len, mode, nrange, stats + blockIdx.x);
}

template <class T>
__device__ void pcm_convert(const T* __restrict__ in, const SgPcmCall* __restrict__ calls,
                            const SgPcmTile* __restrict__ tiles, const SgPcmStat* __restrict__ stats, int mode,
                            int16_t* __restrict__ out) {
  const SgPcmTile t = tiles[blockIdx.x];
  const SgPcmCall C = calls[t.call];
  const SgPcmStat S = stats[t.call];
  const int64_t end = t.k0 + SG_PCM_TILE < C.len ? t.k0 + SG_PCM_TILE : C.len;
#pragma unroll 4
  for (int64_t k = t.k0 + threadIdx.x; k < end; k += 256) {
    const double x = (double)in[C.off + k];
    double v;
    if (mode == SG_PCM_NORMALIZE) {
      v = x - S.mean;
      if (S.scale) v = S.level * v / S.m;
      v = rint(v * 32767.0);  // round(): half to even
    } else {  // seewave::rescale, then writeWave's as.integer
      v = trunc((x - S.min) * S.level / S.m - S.level / 2);
    }
    out[C.off + k] = (int16_t)fmin(32767.0, fmax(-32768.0, v));
  }
}

extern "C" __global__ __launch_bounds__(256) void sg_pcm_convert_f32(const float* __restrict__ in,
                                                                     const SgPcmCall* __restrict__ calls,
                                                                     const SgPcmTile* __restrict__ tiles,
                                                                     const SgPcmStat* __restrict__ stats, int mode,
                                                                     int16_t* __restrict__ out) {
  pcm_convert(in, calls, tiles, stats, mode, out);
}
extern "C" __global__ __launch_bounds__(256) void sg_pcm_convert_f64(const double* __restrict__ in,
                                                                     const SgPcmCall* __restrict__ calls,
                                                                     const SgPcmTile* __restrict__ tiles,
                                                                     const SgPcmStat* __restrict__ stats, int mode,
                                                                     int16_t* __restrict__ out) {
  pcm_convert(in, calls, tiles, stats, mode, out);
}

#include <string>

#include "sg_exec.h"

namespace sg {

#define HIPCHK_W(x)                                                                                        \
  do {                                                                                                     \
    const hipError_t _e = (x);                                                                             \
    if (_e != hipSuccess) throw SgError(SG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e));   \
  } while (0)

void PcmJob::free() {
  if (buf) (void)hipFree(buf);
  *this = PcmJob{};
}

void PcmJob::prepare(const int64_t* off, const int64_t* len, int64_t n_calls, hipStream_t s) {
  std::vector<SgPcmCall> calls((size_t)n_calls);
  std::vector<SgPcmTile> tiles;
  for (int64_t c = 0; c < n_calls; ++c) {
    calls[c] = SgPcmCall{off[c], len[c]};
    for (int64_t k0 = 0; k0 < len[c]; k0 += SG_PCM_TILE) tiles.push_back(SgPcmTile{(int32_t)c, 0, k0});
  }
  free();
  n = n_calls;
  ntiles = (int64_t)tiles.size();
  const size_t bc = (size_t)n * sizeof(SgPcmCall), bt = (size_t)ntiles * sizeof(SgPcmTile),
               bs = (size_t)n * sizeof(SgPcmStat);
  const size_t up = 256;
  const size_t oc = 0, ot = (bc + up - 1) / up * up, os = ot + (bt + up - 1) / up * up;
  HIPCHK_W(hipMalloc(&buf, os + bs + up));
  this->calls = (SgPcmCall*)(buf + oc);
  this->tiles = (SgPcmTile*)(buf + ot);
  stats = (SgPcmStat*)(buf + os);
  if (bc) HIPCHK_W(hipMemcpyAsync(this->calls, calls.data(), bc, hipMemcpyHostToDevice, s));
  if (bt) HIPCHK_W(hipMemcpyAsync(this->tiles, tiles.data(), bt, hipMemcpyHostToDevice, s));
  HIPCHK_W(hipStreamSynchronize(s));
}

void PcmJob::run(const void* in, bool f64, int mode, double nrange, int16_t* out, hipStream_t s) const {
  if (n <= 0) return;
  if (f64) {
    hipLaunchKernelGGL(sg_pcm_stats_f64, dim3((unsigned)n), dim3(256), 0, s, (const double*)in, calls, mode, nrange,
                       stats);
  } else {
    hipLaunchKernelGGL(sg_pcm_stats_f32, dim3((unsigned)n), dim3(256), 0, s, (const float*)in, calls, mode, nrange,
                       stats);
  }
  HIPCHK_W(hipGetLastError());
  if (ntiles <= 0) return;
  if (f64) {
    hipLaunchKernelGGL(sg_pcm_convert_f64, dim3((unsigned)ntiles), dim3(256), 0, s, (const double*)in, calls, tiles,
                       stats, mode, out);
  } else {
    hipLaunchKernelGGL(sg_pcm_convert_f32, dim3((unsigned)ntiles), dim3(256), 0, s, (const float*)in, calls, tiles,
                       stats, mode, out);
  }
  HIPCHK_W(hipGetLastError());
}

}  // namespace sg
