// sg_mel.hip — compareSounds() on the device (R/matchPars.R:313-416), the
// similarity metric of matchPars(): getMelSpec()
// (R/matchPars.R:510-560 = tuneR 1.3.2 melfcc(spec_out = TRUE)$aspectrum:
// tuneR/R/melfcc.R, powspec.R, audspec.R, fft2melmx.R, hz2mel.R, mel2hz.R;
// signal 0.7-6 specgram.R, hamming.R) of a batch of candidates and the
// per-column cor / cosine / pixel / dtw against one target spectrum.
//
//   sg_mel_frames   one workgroup per frame: pre-emphasis 0.97 on the fly,
//                   hamming(winpts), zero-padded real nfft-point FFT (complex
//                   nfft/2 radix-2 Stockham in LDS + untangling; nfft <= 4096), |X|^2 of the
//                   first nfft/2 bins, the Slaney mel bands (sparse triangles),
//                   and the column's mean (soundgen's frame stripping)
//   sg_mel_cand     one workgroup per candidate: kept columns (colMeans >
//                   2^(throwaway/10)) compacted in order, their min and max (log01)
//   sg_mel_compare  one wavefront per (candidate, output column): matchColumns'
//                   central NA padding of the shorter spectrum, then cor,
//                   cosine, pixel and the dtw package's symmetric2 distance
//                   (anti-diagonal wavefront in LDS)
//   sg_mel_out      the normalised kept columns of one spectrum (getMelSpec's value)
// Everything is fp64: R computes in doubles, and the log01 spectra of weak
// bins amplify an fp32 FFT's absolute error past the 1e-6 parity bar.
// HBM-light: each candidate sample is read ~2x (50 % overlap), the work is the
// nfft log nfft FFT per frame and 200^2 DTW cells per column.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "sg_mel.h"
#include "sg_rmath.h"

namespace {

struct MelFrame {
  int64_t base;  // candidate sample 0 in the input buffer
  int32_t o;     // frame start within the candidate
  int32_t seg;   // samples of the frame inside the candidate (<= winpts)
};

struct MelBand {
  int32_t k0, n;  // first bin and count of the band's non-zero weights
  int32_t w0;     // offset of its weights
  int32_t pad;
};

struct MelCand {
  int32_t f0, nf;  // frames [f0, f0 + nf)
  int32_t job0;    // first column job
  int32_t pad;
};

template <typename T>
__global__ __launch_bounds__(256) void sg_mel_frames(const T* __restrict__ x, const MelFrame* __restrict__ frames,
                                                     const double* __restrict__ ham, const double2* __restrict__ tw,
                                                     const double2* __restrict__ twN, const MelBand* __restrict__ bands,
                                                     const double* __restrict__ wts, int winpts, int M, int logM,
                                                     int nb, double* __restrict__ spec,
                                                     double* __restrict__ colmean) {
  extern __shared__ double2 lds[];
  double2* A = lds;
  double2* B = lds + M;
  __shared__ double red[256];
  const MelFrame F = frames[blockIdx.x];
  const T* xc = x + F.base;
  // windowed, pre-emphasised frame packed as z[n] = xw[2n] + i xw[2n+1]
  for (int n = threadIdx.x; n < M; n += blockDim.x) {
    double v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = 2 * n + h;
      double s = 0;
      if (i < F.seg && i < winpts) {
        const int q = F.o + i;  // filter(x, c(1, -0.97), sides = 1): y[1] = x[1]
        s = (double)xc[q];
        if (q > 0) s -= 0.97 * (double)xc[q - 1];
        s *= ham[i];
      }
      v[h] = s;
    }
    A[n] = make_double2(v[0], v[1]);
  }
  __syncthreads();
  // radix-2 Stockham, forward (e^{-2 pi i / M}): Y[b 2Ns + k] = a + w b', Y[.. + Ns] = a - w b'
  double2* X = A;
  double2* Y = B;
  for (int s = 0, Ns = 1; s < logM; ++s, Ns <<= 1) {
    for (int j = threadIdx.x; j < M / 2; j += blockDim.x) {
      const int k = j & (Ns - 1);
      const double2 w = tw[k * (M / (2 * Ns))];
      const double2 a = X[j], b0 = X[j + M / 2];
      const double2 b = make_double2(b0.x * w.x - b0.y * w.y, b0.x * w.y + b0.y * w.x);
      const int o = (j - k) * 2 + k;
      Y[o] = make_double2(a.x + b.x, a.y + b.y);
      Y[o + Ns] = make_double2(a.x - b.x, a.y - b.y);
    }
    __syncthreads();
    double2* t = X;
    X = Y;
    Y = t;
  }
  // untangle: X_k = E_k + e^{-2 pi i k / N} O_k, E = (Z_k + conj Z_{M-k}) / 2,
  // O = -i (Z_k - conj Z_{M-k}) / 2; power |X_k|^2 into Y (as .x)
  double* P = reinterpret_cast<double*>(Y);
  for (int k = threadIdx.x; k < M; k += blockDim.x) {
    const double2 z = X[k], zc = X[(M - k) & (M - 1)];
    const double ex = 0.5 * (z.x + zc.x), ey = 0.5 * (z.y - zc.y);
    const double ox = 0.5 * (z.y + zc.y), oy = -0.5 * (z.x - zc.x);
    const double2 w = twN[k];
    const double re = ex + (w.x * ox - w.y * oy), im = ey + (w.x * oy + w.y * ox);
    P[k] = re * re + im * im;
  }
  __syncthreads();
  double part = 0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const MelBand bd = bands[b];
    double acc = 0;
    for (int i = 0; i < bd.n; ++i) acc += wts[bd.w0 + i] * P[bd.k0 + i];
    spec[(int64_t)blockIdx.x * nb + b] = acc;
    part += acc;
  }
  red[threadIdx.x] = part;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) colmean[blockIdx.x] = red[0] / nb;
}

// kept columns in frame order (colMeans(spec) > thr) and their min / max
__global__ __launch_bounds__(256) void sg_mel_cand(const MelCand* __restrict__ cands, const double* __restrict__ spec,
                                                   const double* __restrict__ colmean, double thr, int nb,
                                                   int32_t* __restrict__ kept, int32_t* __restrict__ nkept,
                                                   double* __restrict__ mn, double* __restrict__ mx) {
  __shared__ int32_t sc[256];
  __shared__ double rmn[256], rmx[256];
  const MelCand C = cands[blockIdx.x];
  int32_t run = 0;
  for (int c0 = 0; c0 < C.nf; c0 += 256) {
    const int f = c0 + threadIdx.x;
    const int flag = f < C.nf && colmean[C.f0 + f] > thr;
    sc[threadIdx.x] = flag;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive scan
      const int v = threadIdx.x >= o ? sc[threadIdx.x - o] : 0;
      __syncthreads();
      sc[threadIdx.x] += v;
      __syncthreads();
    }
    if (flag) kept[C.f0 + run + sc[threadIdx.x] - 1] = C.f0 + f;
    run += sc[255];
    __syncthreads();
  }
  double lo = INFINITY, hi = -INFINITY;
  for (int64_t e = threadIdx.x; e < (int64_t)run * nb; e += 256) {
    const double v = spec[(int64_t)kept[C.f0 + e / nb] * nb + e % nb];
    lo = fmin(lo, v);
    hi = fmax(hi, v);
  }
  rmn[threadIdx.x] = lo;
  rmx[threadIdx.x] = hi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      rmn[threadIdx.x] = fmin(rmn[threadIdx.x], rmn[threadIdx.x + o]);
      rmx[threadIdx.x] = fmax(rmx[threadIdx.x], rmx[threadIdx.x + o]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    nkept[blockIdx.x] = run;
    mn[blockIdx.x] = rmn[0];
    mx[blockIdx.x] = rmx[0];
  }
}

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// log01 of one kept column (melfcc + soundgen's log01: log(v - min + 1) / log(max - min + 1))
__device__ __forceinline__ double log01(double v, double lo, double den) { return log(v - lo + 1.0) / den; }

// central NA padding of matchColumns(m, ncol) (matchLengths 'central'): output
// column j shows column j + off of the short matrix, NA outside [0, mcols)
__device__ __forceinline__ int pad_off(int ncol, int mcols) { return (ncol + mcols + 2) / 2 - 1 - ncol; }

// One wavefront per (candidate, output column): methods cor, cosine, pixel, dtw
__global__ __launch_bounds__(64) void sg_mel_compare(const int32_t* __restrict__ job_cand,
                                                     const int32_t* __restrict__ job_col,
                                                     const double* __restrict__ tspec, int ncT, int nb,
                                                     const double* __restrict__ spec, const int32_t* __restrict__ kept,
                                                     const MelCand* __restrict__ cands,
                                                     const int32_t* __restrict__ nkept, const double* __restrict__ mn,
                                                     const double* __restrict__ mx, int do_dtw,
                                                     double* __restrict__ sims) {
  extern __shared__ double sh[];
  double* t = sh;
  double* d = sh + nb;
  double* D0 = sh + 2 * nb;
  double* D1 = D0 + nb;
  double* D2 = D1 + nb;
  const int c = job_cand[blockIdx.x], j = job_col[blockIdx.x];
  const int nk = nkept[c];
  const int ncol = nk > ncT ? nk : ncT;
  if (j >= ncol) return;
  double* out = sims + (int64_t)blockIdx.x * 4;
  int tj = j, cj = j;
  if (ncT < ncol) tj = j + pad_off(ncol, ncT);
  if (nk < ncol) cj = j + pad_off(ncol, nk);
  const double lo = mn[c], den = log(mx[c] - lo + 1.0);
  if (tj < 0 || tj >= ncT || cj < 0 || cj >= nk || !(den > 0)) {
    if (threadIdx.x < 4) out[threadIdx.x] = NAN;
    return;
  }
  const double* tc = tspec + (int64_t)tj * nb;
  const double* sc = spec + (int64_t)kept[cands[c].f0 + cj] * nb;
  double st = 0, sd = 0;
  for (int b = threadIdx.x; b < nb; b += 64) {
    const double tv = tc[b], dv = log01(sc[b], lo, den);
    t[b] = tv;
    d[b] = dv;
    st += tv;
    sd += dv;
  }
  st = wsum(st);
  sd = wsum(sd);
  const double mt = st / nb, md = sd / nb;
  double ab = 0, aa = 0, bb = 0, td = 0, tt = 0, dd = 0, ad = 0;
  for (int b = threadIdx.x; b < nb; b += 64) {
    const double a = t[b] - mt, e = d[b] - md;
    ab += a * e;
    aa += a * a;
    bb += e * e;
    td += t[b] * d[b];
    tt += t[b] * t[b];
    dd += d[b] * d[b];
    ad += fabs(t[b] - d[b]);
  }
  ab = wsum(ab);
  aa = wsum(aa);
  bb = wsum(bb);
  td = wsum(td);
  tt = wsum(tt);
  dd = wsum(dd);
  ad = wsum(ad);
  double dtw = NAN;
  if (do_dtw) {
    // symmetric2 DP (dtw package default; the host restatement is sg_dtw_symmetric2):
    // g(i, j) = min(g(i-1, j-1) + 2 d, g(i-1, j) + d, g(i, j-1) + d), d = |t_i - d_j|;
    // anti-diagonal a = i + j, entries indexed by i (D1: a - 1, D2: a - 2)
    __syncthreads();
    for (int a = 0; a <= 2 * nb - 2; ++a) {
      const int i0 = a - (nb - 1) > 0 ? a - (nb - 1) : 0, i1 = a < nb - 1 ? a : nb - 1;
      for (int i = i0 + threadIdx.x; i <= i1; i += 64) {
        const int jj = a - i;
        const double dist = fabs(t[i] - d[jj]);
        double g;
        if (a == 0) {
          g = dist;
        } else {
          g = INFINITY;
          if (i > 0 && jj > 0) g = fmin(g, D2[i - 1] + 2 * dist);
          if (i > 0) g = fmin(g, D1[i - 1] + dist);
          if (jj > 0) g = fmin(g, D1[i] + dist);
        }
        D0[i] = g;
      }
      __syncthreads();
      double* r = D2;
      D2 = D1;
      D1 = D0;
      D0 = r;
    }
    dtw = 1.0 - D1[nb - 1] / (double)(2 * nb);
  }
  if (threadIdx.x == 0) {
    const double cden = sqrt(aa * bb);
    out[0] = cden > 0 ? ab / cden : NAN;
    out[1] = td / sqrt(tt * dd);
    out[2] = 1.0 - ad / nb;
    out[3] = dtw;
  }
}

// getMelSpec's value: the kept columns, log01-normalised, nb x nk column-major
__global__ __launch_bounds__(256) void sg_mel_out(const double* __restrict__ spec, const int32_t* __restrict__ kept,
                                                  int nk, int nb, const double* __restrict__ mn,
                                                  const double* __restrict__ mx, double* __restrict__ out) {
  const double lo = mn[0], den = log(mx[0] - lo + 1.0);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < (int64_t)nk * nb; e += (int64_t)gridDim.x * 256)
    out[e] = log01(spec[(int64_t)kept[e / nb] * nb + e % nb], lo, den);
}

#define MELCHK(x)                                                                                        \
  do {                                                                                                   \
    hipError_t _e = (x);                                                                                 \
    if (_e != hipSuccess) throw sg::SgError(SG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

// Slaney mel scale (tuneR hz2mel / mel2hz, htk = FALSE)
double hz2mel(double f) {
  const double f_sp = 200.0 / 3, brkfrq = 1000.0, brkpt = brkfrq / f_sp, logstep = std::exp(std::log(6.4) / 27);
  return f < brkfrq ? f / f_sp : brkpt + std::log(std::max(f, 1e-300) / brkfrq) / std::log(logstep);
}
double mel2hz(double z) {
  const double f_sp = 200.0 / 3, brkfrq = 1000.0, brkpt = brkfrq / f_sp, logstep = std::exp(std::log(6.4) / 27);
  return z < brkpt ? f_sp * z : brkfrq * std::exp(std::log(logstep) * (z - brkpt));
}

// Device buffers of one compareSounds / getMelSpec launch sequence
// Device buffers of one mel run, and the host copies their uploads read: an
// async H2D copy from pageable memory may still be pending when the caller's
// vector goes away, so upload() stages the bytes in memory this object owns.
// The destructor frees the device buffers first (hipFree waits for the device),
// then the staged host bytes.
struct DevBuf {
  std::vector<void*> p;
  std::vector<std::vector<char>> host;
  template <class T>
  T* get(size_t n) {
    void* q = nullptr;
    MELCHK(hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)));
    p.push_back(q);
    return static_cast<T*>(q);
  }
  ~DevBuf() {
    for (void* q : p) (void)hipFree(q);
  }
};

template <class T>
T* upload(DevBuf& db, const std::vector<T>& v, hipStream_t s) {
  T* d = db.get<T>(v.size());
  if (!v.empty()) {
    const char* src = reinterpret_cast<const char*>(v.data());
    db.host.emplace_back(src, src + v.size() * sizeof(T));
    MELCHK(hipMemcpyAsync(d, db.host.back().data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  }
  return d;
}

}  // namespace

namespace sg {

MelGeom mel_geom(const sg_mel_params& p) {
  MelGeom g;
  const double sr = p.samplingRate;
  if (!(sr > 0) || !(p.windowLength > 0)) throw SgError(SG_E_ARG, "getMelSpec: samplingRate and windowLength must be > 0");
  const double step = std::isnan(p.step) ? p.windowLength * (1 - p.overlap / 100) : p.step;
  if (!(step > 0)) throw SgError(SG_E_ARG, "getMelSpec: step must be > 0");
  // tuneR powspec: winpts = round(wintime sr), steppts = round(steptime sr), nfft = 2^ceil(log2(winpts))
  g.winpts = (int)r_round(p.windowLength / 1000 * sr);
  g.steppts = (int)r_round(step / 1000 * sr);
  if (g.winpts < 2 || g.steppts < 1) throw SgError(SG_E_ARG, "getMelSpec: window shorter than 2 samples");
  g.nfft = (int)std::pow(2.0, std::ceil(std::log((double)g.winpts) / std::log(2.0)));
  if (g.nfft > 4096) throw SgError(SG_E_UNSUPPORTED, "getMelSpec: windows above 4096 points are not supported");
  g.nfreqs = g.nfft / 2;
  g.nb = (int)(100 * p.windowLength / 20);  // melfcc(nbands = 100 * windowLength / 20)
  if (g.nb < 1) throw SgError(SG_E_ARG, "getMelSpec: no mel bands");
  g.thr = std::pow(2.0, p.throwaway / 10);
  g.ham.resize(g.winpts);
  for (int i = 0; i < g.winpts; ++i) g.ham[i] = 0.54 - 0.46 * std::cos(2 * M_PI * i / (g.winpts - 1));
  // fft2melmx((nfreqs - 1) * 2, sr, nbands, 1, 0, maxFreq)[, 1:nfreqs] (audspec's nfft quirk)
  const int nfft2 = (g.nfreqs - 1) * 2;
  const double maxf = std::isnan(p.maxFreq) ? sr / 2 : p.maxFreq;
  const double minmel = hz2mel(0.0), maxmel = hz2mel(maxf);
  std::vector<double> binf(g.nb + 2);
  for (int i = 0; i < g.nb + 2; ++i) binf[i] = mel2hz(minmel + (double)i / (g.nb + 1) * (maxmel - minmel));
  for (int b = 0; b < g.nb; ++b) {
    // fs = fs[2] + width (fs - fs[2]) with width = 1, in R's (and numpy's) rounding
    const double f1 = binf[b + 1], f0 = f1 + 1.0 * (binf[b] - f1), f2 = f1 + 1.0 * (binf[b + 2] - f1);
    const double sc = 2 / (binf[b + 2] - binf[b]);
    int k0 = -1, n = 0;
    const int w0 = (int)g.w.size();
    for (int k = 0; k < g.nfreqs; ++k) {
      const double f = (double)k / nfft2 * sr;
      const double lo = (f - f0) / (f1 - f0), hi = (f2 - f) / (f2 - f1);
      const double w = sc * std::max(0.0, std::min(lo, hi));
      if (w > 0) {
        if (k0 < 0) k0 = k;
        // weights are contiguous in k (a triangle); zeros between would break the band
        while (k0 + n < k) { g.w.push_back(0.0); ++n; }
        g.w.push_back(w);
        ++n;
      }
    }
    g.band_k0.push_back(k0 < 0 ? 0 : k0);
    g.band_n.push_back(n);
    g.band_w0.push_back(w0);
  }
  const int M = g.nfreqs;  // complex points of the real nfft transform
  g.tw.resize(std::max(1, M / 2) * 2);
  for (int t = 0; t < M / 2; ++t) {
    g.tw[2 * t] = std::cos(2 * M_PI * t / M);
    g.tw[2 * t + 1] = -std::sin(2 * M_PI * t / M);
  }
  g.twN.resize(2 * M);
  for (int k = 0; k < M; ++k) {
    g.twN[2 * k] = std::cos(2 * M_PI * k / g.nfft);
    g.twN[2 * k + 1] = -std::sin(2 * M_PI * k / g.nfft);
  }
  return g;
}

// frames of a candidate of `len` samples (tuneR powspec via signal::specgram):
// starts 0, steppts, ..., nn steppts with nn = (len - winpts - 1) %/% steppts
int mel_frames(const MelGeom& g, int64_t len) {
  if (len > g.winpts) return (int)((double)(len - g.winpts - 1) / g.steppts + 1e-10) + 1;
  return 1;
}

namespace {

struct MelRun {
  int F = 0;
  DevBuf db;
  double* spec = nullptr;
  int32_t* kept = nullptr;
  int32_t* nkept = nullptr;
  double *mn = nullptr, *mx = nullptr;
  MelCand* cands = nullptr;
  std::vector<MelCand> hc;
};

template <typename T>
void mel_run(MelRun& r, const MelGeom& g, const T* d_x, const int64_t* offsets, const int64_t* lengths, int64_t n,
             hipStream_t s) {
  std::vector<MelFrame> fr;
  r.hc.resize(n);
  for (int64_t c = 0; c < n; ++c) {
    MelCand& C = r.hc[c];
    C.f0 = (int32_t)fr.size();
    C.nf = 0;
    if (lengths[c] <= 0) continue;
    const int nf = mel_frames(g, lengths[c]);
    for (int f = 0; f < nf; ++f) {
      const int64_t o = (int64_t)f * g.steppts;
      fr.push_back(MelFrame{offsets[c], (int32_t)o, (int32_t)std::min<int64_t>(g.winpts, lengths[c] - o)});
    }
    C.nf = nf;
  }
  r.F = (int)fr.size();
  std::vector<MelBand> bands(g.nb);
  for (int b = 0; b < g.nb; ++b) bands[b] = MelBand{g.band_k0[b], g.band_n[b], g.band_w0[b], 0};
  const MelFrame* d_fr = upload(r.db, fr, s);
  const double* d_ham = upload(r.db, g.ham, s);
  const double2* d_tw = reinterpret_cast<const double2*>(upload(r.db, g.tw, s));
  const double2* d_twN = reinterpret_cast<const double2*>(upload(r.db, g.twN, s));
  const MelBand* d_bands = upload(r.db, bands, s);
  const double* d_w = upload(r.db, g.w, s);
  r.cands = upload(r.db, r.hc, s);
  r.spec = r.db.get<double>((size_t)std::max(r.F, 1) * g.nb);
  double* colmean = r.db.get<double>(std::max(r.F, 1));
  r.kept = r.db.get<int32_t>(std::max(r.F, 1));
  r.nkept = r.db.get<int32_t>(n);
  r.mn = r.db.get<double>(n);
  r.mx = r.db.get<double>(n);
  const int M = g.nfreqs;
  int logM = 0;
  while ((1 << logM) < M) ++logM;
  if (r.F > 0) {
    hipLaunchKernelGGL(sg_mel_frames<T>, dim3((unsigned)r.F), dim3(256), (size_t)2 * M * sizeof(double2), s, d_x, d_fr,
                       d_ham, d_tw, d_twN, d_bands, d_w, g.winpts, M, logM, g.nb, r.spec, colmean);
    MELCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(sg_mel_cand, dim3((unsigned)n), dim3(256), 0, s, r.cands, r.spec, colmean, g.thr, g.nb, r.kept,
                     r.nkept, r.mn, r.mx);
  MELCHK(hipGetLastError());
}

}  // namespace

void mel_spec_device(const MelGeom& g, const double* d_x, int64_t len, std::vector<double>& out, int* nk_out,
                     hipStream_t s) {
  MelRun r;
  const int64_t off = 0;
  mel_run<double>(r, g, d_x, &off, &len, 1, s);
  int32_t nk = 0;
  MELCHK(hipMemcpyAsync(&nk, r.nkept, sizeof nk, hipMemcpyDeviceToHost, s));
  MELCHK(hipStreamSynchronize(s));
  *nk_out = nk;
  out.assign((size_t)nk * g.nb, 0.0);
  if (nk == 0) return;
  double* d_out = r.db.get<double>((size_t)nk * g.nb);
  const int64_t tot = (int64_t)nk * g.nb;
  hipLaunchKernelGGL(sg_mel_out, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 4096)), dim3(256), 0, s, r.spec,
                     r.kept, nk, g.nb, r.mn, r.mx, d_out);
  MELCHK(hipGetLastError());
  MELCHK(hipMemcpyAsync(out.data(), d_out, (size_t)tot * sizeof(double), hipMemcpyDeviceToHost, s));
  MELCHK(hipStreamSynchronize(s));
}

void compare_sounds_device(const MelGeom& g, const double* tspec, int ncT, const float* d_x, const int64_t* offsets,
                           const int64_t* lengths, int64_t n, int methods, int penalize, double* out, double* summary,
                           hipStream_t s) {
  MelRun r;
  mel_run<float>(r, g, d_x, offsets, lengths, n, s);
  // column jobs: candidate c may need up to max(ncT, its frames) output columns
  std::vector<int32_t> jc, jj;
  for (int64_t c = 0; c < n; ++c) {
    r.hc[c].job0 = (int32_t)jc.size();
    const int ub = lengths[c] > 0 ? std::max(ncT, r.hc[c].nf) : 0;
    for (int j = 0; j < ub; ++j) {
      jc.push_back((int32_t)c);
      jj.push_back(j);
    }
  }
  const int32_t* d_jc = upload(r.db, jc, s);
  const int32_t* d_jj = upload(r.db, jj, s);
  const double* d_t = upload(r.db, std::vector<double>(tspec, tspec + (size_t)ncT * g.nb), s);
  const int64_t J = (int64_t)jc.size();
  double* d_sims = r.db.get<double>((size_t)std::max<int64_t>(J, 1) * 4);
  if (J > 0) {
    hipLaunchKernelGGL(sg_mel_compare, dim3((unsigned)J), dim3(64), (size_t)5 * g.nb * sizeof(double), s, d_jc, d_jj,
                       d_t, ncT, g.nb, r.spec, r.kept, r.cands, r.nkept, r.mn, r.mx, (methods & 8) ? 1 : 0, d_sims);
    MELCHK(hipGetLastError());
  }
  std::vector<double> sims((size_t)J * 4);
  std::vector<int32_t> nk(n);
  if (J) MELCHK(hipMemcpyAsync(sims.data(), d_sims, sims.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  MELCHK(hipMemcpyAsync(nk.data(), r.nkept, nk.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  MELCHK(hipStreamSynchronize(s));
  // compareSounds' reduction (R/matchPars.R:378-416): per method the column
  // values' sum with NAs dropped over the column count (penalizeLengthDif), else
  // their mean; the summary is the mean over the methods that are not NA
  for (int64_t c = 0; c < n; ++c) {
    double* o = out + 4 * c;
    if (lengths[c] <= 0) {
      for (int m = 0; m < 4; ++m) o[m] = NAN;
      if (summary) summary[c] = NAN;
      continue;
    }
    const int ncol = std::max(ncT, (int)nk[c]);
    for (int m = 0; m < 4; ++m) {
      if (!(methods & (1 << m))) {
        o[m] = NAN;
        continue;
      }
      double sm = 0;
      int cnt = 0;
      for (int j = 0; j < ncol; ++j) {
        const double v = sims[((size_t)r.hc[c].job0 + j) * 4 + m];
        if (!std::isnan(v)) {
          sm += v;
          ++cnt;
        }
      }
      o[m] = penalize ? sm / ncol : (cnt ? sm / cnt : NAN);
    }
    if (summary) {
      double sm = 0;
      int cnt = 0;
      for (int m = 0; m < 4; ++m)
        if ((methods & (1 << m)) && !std::isnan(o[m])) {
          sm += o[m];
          ++cnt;
        }
      summary[c] = cnt ? sm / cnt : NAN;
    }
  }
}

}  // namespace sg
