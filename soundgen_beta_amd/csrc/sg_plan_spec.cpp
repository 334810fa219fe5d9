// sg_plan_spec.cpp — host planner of the spectral part: FFT geometries,
// noise (generateNoise(), R/source.R:57-138), formant filter
// (R/soundgen.R:743-807, seewave stft/istft), getSpectralEnvelope()
// (R/sourceSpectrum.R:261-566) and getSigmoid() (R/utilities_math.R:639-653).
// Lengths, frame starts and trims are integers computed here in fp64 with
// R's operation order; per-sample work runs in sg_fft.hip.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "sg_plan.h"
#include "sg_prof.h"

#ifndef SG_SEG_SORT
#define SG_SEG_SORT 1
#endif
#ifndef SG_ENV_SORT
#define SG_ENV_SORT 1
#endif

namespace sg {

namespace {
// Stage order of a transform: the largest odd primes first, then 4s and a 2. The
// first Stockham stage (Ns = 1) needs no twiddles, and it saves the most twiddle
// products on the largest radix ((R - 1) M / R of them); for M = 1102 = 29 x 19 x 2
// it makes the radix-29 stage the first, where sg_stft_ola runs it on the matrix
// pipe (sg_fft.hip stage29_mfma).
constexpr int kRadices[] = {31, 29, 23, 19, 17, 13, 11, 7, 5, 3, 4, 2};

// The fp64 trig tables of a transform depend on its length alone: each is
// computed once per process (every batch part plans its own geometries, so
// without this each part would redo them) and copied into the part's fl.
// kind: 0 windows (wl), 1 twiddles (wl), 2 stage twiddles (wl), 3 Bluestein chirp (n), 4 its DFT (n)
template <class Make>
std::shared_ptr<const vec> trig_table(int kind, int n, Make&& make) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, std::shared_ptr<const vec>> memo;
  const std::pair<int, int> key(kind, n);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
  }
  auto t = std::make_shared<const vec>(make());
  std::lock_guard<std::mutex> lk(mu);
  if (memo.size() >= 4096) memo.clear();  // bounded: windows of every length would otherwise accumulate
  return memo.emplace(key, t).first->second;
}
constexpr int kFftSlots = 8192;  // complex points per FFT workgroup (sg_fft.hip SG_FFT_SLOTS)
}  // namespace
// 0: noise uniforms copied into fl per item by the planner (the pre-round-3
// path); 1 (default) gathered on
// the device at upload. sg_set_uniform_gather changes it (tests compare the two).
std::atomic<int> g_ugather{-1};
bool ugather_on() {
  int v = g_ugather.load();
  if (v < 0) {
    v = 1;
    g_ugather.store(v);
  }
  return v == 1;
}

int64_t fs_alloc(Batch& B, int64_t n) {
  const int64_t o = B.fs_total;
  B.fs_total += (n + 63) / 64 * 64;
  return o;
}

int64_t fl_push(Batch& B, const double* v, int64_t n) {
  const int64_t o = bulk_size(B.fl_x, B.fl);
  B.fl.resize(B.fl.size() + (size_t)((n + 3) / 4 * 4));  // 16-B aligned blocks
  float* d = B.fl.data() + (o - B.fl_x.n);
  for (int64_t i = 0; i < n; ++i) d[i] = (float)v[i];
  for (int64_t i = n; i < (n + 3) / 4 * 4; ++i) d[i] = 0.f;
  return o;
}

// seewave ftwindow: hamming.w (seewave.r:7431-7437), hanning.w (:7444-7450)
static int64_t push_windows(Batch& B, int wl) {
  const auto win = trig_table(0, wl, [wl] {
    vec w(2 * (size_t)wl);
    for (int i = 0; i < wl; ++i) {
      w[i] = 0.54 - 0.46 * std::cos(2 * M_PI * (double)i / (double)(wl - 1));
      w[wl + i] = 0.5 - 0.5 * std::cos(2 * M_PI * (double)i / (double)(wl - 1));
    }
    return w;
  });
  return fl_push(B, win->data(), (int64_t)win->size());
}

// ---- complex DFTs of any length for sg_fft_frames (SgCdft, sg_dev.h)
static bool smooth31(int n) {
  for (int r : kRadices)
    while (n % r == 0) n /= r;
  return n == 1;
}
// n-point DFT in fp64 (n 5-smooth), recursive decimation in time; exponents reduced mod n exactly
static void dft_smooth(const std::vector<std::complex<double>>& x, std::vector<std::complex<double>>& y) {
  const int n = (int)x.size();
  y.assign((size_t)n, 0.0);
  if (n == 1) {
    y[0] = x[0];
    return;
  }
  int p = 2;
  while (n % p) ++p;
  const int m = n / p;
  std::vector<std::vector<std::complex<double>>> sub((size_t)p);
  for (int r = 0; r < p; ++r) {
    std::vector<std::complex<double>> xs((size_t)m);
    for (int j = 0; j < m; ++j) xs[j] = x[(size_t)j * p + r];
    dft_smooth(xs, sub[r]);
  }
  for (int k = 0; k < n; ++k) {
    std::complex<double> acc = 0.0;
    for (int r = 0; r < p; ++r) {
      const double a = -2.0 * M_PI * (double)(((int64_t)r * k) % n) / (double)n;
      acc += std::complex<double>(std::cos(a), std::sin(a)) * sub[r][k % m];
    }
    y[k] = acc;
  }
}
static SgCdft make_cdft(Batch& B, int n) {
  SgCdft c{};
  c.n = n;
  if (smooth31(n)) {
    c.geom = geometry(B, 2 * n);  // its M = n: radices, magic numbers, W_n table
    return c;
  }
  int L = 2 * n - 1;
  for (;; ++L) {
    int m = L;
    for (int r : {2, 3, 5})
      while (m % r == 0) m /= r;
    if (m == 1) break;
  }
  if (L > kFftSlots) throw SgError(SG_E_UNSUPPORTED, "FFT: Bluestein length " + std::to_string(L) + " exceeds LDS");
  c.L = L;
  c.geom = geometry(B, 2 * L);
  const auto ch = trig_table(3, n, [n] {
    vec h(2 * (size_t)n);
    for (int m = 0; m < n; ++m) {
      const double a = -M_PI * (double)(((int64_t)m * m) % (2 * (int64_t)n)) / (double)n;
      h[2 * m] = std::cos(a);
      h[2 * m + 1] = std::sin(a);
    }
    return h;
  });
  const auto bv = trig_table(4, n, [n, L, &ch] {
    std::vector<std::complex<double>> b((size_t)L, 0.0), bf;
    for (int m = 0; m < n; ++m) {
      b[m] = std::complex<double>((*ch)[2 * m], -(*ch)[2 * m + 1]);
      if (m > 0) b[L - m] = b[m];
    }
    dft_smooth(b, bf);
    vec v(2 * (size_t)L);
    for (int k = 0; k < L; ++k) {
      v[2 * k] = bf[k].real() / L;
      v[2 * k + 1] = bf[k].imag() / L;
    }
    return v;
  });
  c.chirp = fl_push(B, ch->data(), (int64_t)ch->size());
  c.bf = fl_push(B, bv->data(), (int64_t)bv->size());
  return c;
}
static int cdft_size(const SgCdft& c) { return c.L ? c.L : c.n; }

// odd window length (SG_FFT_ODD, sg_dev.h): forward wl-point and inverse
// (wl - 1)-point complex DFTs
static int geometry_odd(Batch& B, int wl) {
  SgFftGeom g{};
  g.wl = wl;
  g.M = wl / 2;
  g.kind = SG_FFT_ODD;
  g.fb = 1;
  g.cd[0] = make_cdft(B, wl);
  g.cd[1] = make_cdft(B, 2 * g.M);
  // the wl-point frame buffer, the Bluestein work buffer and the FFT twiddle table
  const int T = std::max(cdft_size(g.cd[0]), cdft_size(g.cd[1]));
  g.lds_bytes = (int32_t)(((int64_t)wl + 2 * (int64_t)T) * 8);
  if (g.lds_bytes > 160 * 1024) throw SgError(SG_E_UNSUPPORTED, "FFT: odd window length exceeds the LDS budget");
  g.win = push_windows(B, wl);
  for (size_t i = 0; i < B.geoms.size(); ++i)  // the sub-geometries were pushed first
    if (B.geoms[i].wl == wl) return (int)i;
  B.geoms.push_back(g);
  return (int)B.geoms.size() - 1;
}

int geometry(Batch& B, int wl) {
  for (size_t i = 0; i < B.geoms.size(); ++i)
    if (B.geoms[i].wl == wl) return (int)i;
  if (wl < 3) throw SgError(SG_E_UNSUPPORTED, "FFT: window length must be >= 3");
  if (wl % 2) return geometry_odd(B, wl);
  SgFftGeom g{};
  g.wl = wl;
  g.M = wl / 2;
  int m = g.M;
  for (int r : kRadices) {
    while (m % r == 0) {
      if (g.nstages >= SG_FFT_MAX_STAGES) throw SgError(SG_E_UNSUPPORTED, "FFT: too many stages");
      g.radix[g.nstages++] = r;
      m /= r;
    }
  }
  // a prime factor > 31 (windowLength_points shrinks to floor(L / 2) for short
  // sounds, R/soundgen.R:743, so any length occurs): direct DFT, one frame per workgroup
  const bool dft = m != 1;
  if (dft) {
    g.nstages = 0;
    g.cd[0] = make_cdft(B, g.M);  // Bluestein (pushes its L-point sub-geometry first)
    for (size_t i = 0; i < B.geoms.size(); ++i)
      if (B.geoms[i].wl == wl) return (int)i;
  }
  // twiddles W_M^t (t < M), W_N^k (k < M), fp64 -> fp32
  const int M = g.M;
  const auto tw = trig_table(1, wl, [M, wl] {
    vec w(4 * (size_t)M);
    for (int t = 0; t < M; ++t) {
      const double a = -2.0 * M_PI * (double)t / (double)M;
      w[2 * t] = std::cos(a);
      w[2 * t + 1] = std::sin(a);
      const double b = -2.0 * M_PI * (double)t / (double)wl;
      w[2 * M + 2 * t] = std::cos(b);
      w[2 * M + 2 * t + 1] = std::sin(b);
    }
    return w;
  });
  g.tw = fl_push(B, tw->data(), (int64_t)tw->size());
  {
    const SgFftGeom& gc = g;  // the stage radices are a function of wl
    const auto ts = trig_table(2, wl, [&gc] {
      vec t(2 * (size_t)std::max(1, gc.M - 1), 0.0);
      int ns = 1;
      for (int s = 0; s < gc.nstages; ++s) {
        const int r = gc.radix[s];
        for (int q = 1; q < r; ++q)
          for (int jm = 0; jm < ns; ++jm) {
            const size_t e = (size_t)(ns - 1 + (q - 1) * ns + jm);
            const double a = -2.0 * M_PI * (double)q * (double)jm / ((double)ns * r);
            t[2 * e] = std::cos(a);
            t[2 * e + 1] = std::sin(a);
          }
        ns *= r;
      }
      return t;
    });
    g.tws = fl_push(B, ts->data(), (int64_t)ts->size());
  }
  g.win = push_windows(B, wl);
  // frames per workgroup: one in-place LDS buffer of fb * M complex points,
  // fb * M <= 8192 (64 KB: two workgroups per CU; sg_fft.hip SG_FFT_SLOTS)
  // wavefront-per-frame kernel when every stage's butterflies fit the
  // register state of one wavefront: ceil(M / R / 64) <= max(1, SG_WAVE_STATE / R)
  g.kind = dft ? SG_FFT_DFT : SG_FFT_WAVE;
  for (int s = 0; s < g.nstages && !dft; ++s) {
    const int r = g.radix[s], nb = (g.M / r + 63) / 64;
    if (nb > std::max(1, SG_WAVE_STATE / r)) g.kind = SG_FFT_WG;
  }
  // sg_stft_ola: the next frame's inputs fit the prefetch registers, and the
  // LDS tables (twiddles, W_N^k, hamming, hanning) + SG_FFT_WAVES frame
  // slices, M pairs each, fit the 160 KB of a CU
  if (!dft && (g.M > 64 * SG_PF_SRC || g.M / 2 + 1 > 64 * SG_PF_PAIR)) g.kind = SG_FFT_WG;
  if (!dft && (int64_t)(SG_FFT_WAVES + 4) * g.M * 8 > 160 * 1024) g.kind = SG_FFT_WG;
  if (g.kind == SG_FFT_WAVE) {
    g.fb = SG_FFT_WAVES;
    g.lds_bytes = (SG_FFT_WAVES + 4) * g.M * 8;
  } else if (g.kind == SG_FFT_DFT) {
    g.fb = 1;
    g.lds_bytes = (g.M + 2 * g.cd[0].L) * 8;  // frame, Bluestein work buffer, W_L table
    if (g.lds_bytes > 160 * 1024) throw SgError(SG_E_UNSUPPORTED, "FFT: Bluestein frame exceeds the LDS budget");
  } else {
    g.fb = std::max(1, std::min(16, kFftSlots / g.M));
    if (g.fb * g.M > kFftSlots) throw SgError(SG_E_UNSUPPORTED, "FFT: window too long for LDS (wl > 16384)");
    g.lds_bytes = (g.fb + 1) * g.M * 8;  // + the W_M twiddle table
  }
  auto magic = [](int d) -> uint32_t { return d <= 1 ? 0u : (uint32_t)(((1ull << 32) + (uint64_t)d - 1) / (uint64_t)d); };
  int ns = 1;
  for (int s = 0; s < g.nstages; ++s) {
    g.mr_magic[s] = magic(g.M / g.radix[s]);
    g.ns_magic[s] = magic(ns);
    ns *= g.radix[s];
  }
  g.m_magic = magic(g.M);
  g.hp_magic = magic(g.M / 2 + 1);
  B.geoms.push_back(g);
  return (int)B.geoms.size() - 1;
}

// istft() frame bookkeeping shared by noise and filter: hop, xlen, W0 scale
struct IstftGeom {
  double h;
  int64_t xlen;
  float scale;
};
static IstftGeom istft_geom(int wl, int64_t nc, double ovlp) {
  IstftGeom g;
  g.h = (double)wl * (100 - ovlp) / 100;
  g.xlen = (int64_t)((double)wl + (double)(nc - 1) * g.h);  // numeric(xlen) truncates
  // sum(hanning(wl)^2) depends on wl alone: once per window length and thread
  thread_local std::vector<std::pair<int, double>> w0_memo;
  double W0d = -1;
  for (const auto& e : w0_memo)
    if (e.first == wl) { W0d = e.second; break; }
  if (W0d < 0) {
    long double W0 = 0;
    for (int i = 0; i < wl; ++i) {
      const double w = 0.5 - 0.5 * std::cos(2 * M_PI * (double)i / (double)(wl - 1));
      W0 += w * w;
    }
    W0d = (double)W0;
    if (w0_memo.size() >= 64) w0_memo.erase(w0_memo.begin());
    w0_memo.emplace_back(wl, W0d);
  }
  g.scale = (float)(g.h / W0d);
  return g;
}

// sg_stft_ola handles the OLA when its geometry runs one wavefront per frame
// and the overlap carried between frames fits the carry registers
static bool fusable(const SgFftGeom& g, double hop) {
  return g.kind == SG_FFT_WAVE && hop >= 1 && (double)g.wl - std::floor(hop) <= 128.0 * SG_CARRY_PAIRS;
}

static int push_ola(Batch& B, int phase, int64_t frames, int64_t nframes, int wl, const IstftGeom& ig, int64_t first,
                    int64_t len, int64_t out, bool fused, bool f64 = false) {
  if (fused && ig.xlen >= (int64_t)1 << 31) throw SgError(SG_E_UNSUPPORTED, "istft: output longer than 2^31 samples");
  SgOla o{};
  // fp64 frames (B.frames64) have no SgFrame: fidx -1 (unfused, sg_ola reads the frame scratch)
  o.fidx = f64 ? -1 : (int32_t)((int64_t)B.frames[phase].size() - nframes);
  o.fused = fused ? 1 : 0;
  o.frames = frames;
  o.out = out;
  o.first = first;
  o.len = len;
  o.xlen = ig.xlen;
  o.h = ig.h;
  o.nframes = (int32_t)nframes;
  o.wl = wl;
  o.scale = ig.scale;
  o.hi = (ig.h == std::floor(ig.h) && ig.h >= 1 && ig.h < 2147483647.0) ? (int32_t)ig.h : 0;
  B.olas[phase].push_back(o);
  return (int)B.olas[phase].size() - 1;
}

int plan_filter(Batch& B, int64_t sound, int64_t L, int wl, double overlap, int64_t env, int64_t env_nc,
                int64_t* out_len, int64_t* out_fs, bool hp) {
  ProfScope ps(PF_FILTER);
  const int gi = geometry(B, wl);
  const int64_t nr = wl / 2;
  // step = seq(1, max(1, L - wl), by = wl - overlap * wl / 100)   R/soundgen.R:744-748
  const double by = (double)wl - overlap * (double)wl / 100;
  const vec step = r_seq_by(1, (double)std::max<int64_t>(1, L - wl), by);
  const int64_t nc = (int64_t)step.size();
  if (env_nc != 1 && env_nc != nc) throw SgError(SG_E_ARG, "formant filter: envelope columns != frames");
  for (double x0 : step)
    if ((int64_t)x0 - 1 + wl > L) throw SgError(SG_E_DOMAIN, "stft: frame beyond the sound");
  const bool fused = !hp && fusable(B.geoms[gi], (double)wl * (100 - overlap) / 100);
  const int64_t fr = fused ? 0 : fs_alloc(B, nc * wl);  // frame scratch only for the unfused path
  if (hp) {  // fp64 forward transforms (sg_fft_frames64), then the fp32 overlap-add (sg_ola)
    for (int64_t c = 0; c < nc; ++c) {
      SgFrame64 f{};
      f.src = sound + (int64_t)step[c] - 1;
      const int64_t col = env_nc == 1 ? 0 : c * nr;
      f.env = env < 0 ? env - col : env + col;
      f.dst = fr + c * wl;
      f.wl = wl;
      B.frames64.push_back(f);
    }
    const IstftGeom ig = istft_geom(wl, nc, overlap);
    const int64_t out = fs_alloc(B, ig.xlen);
    B.fft_frames += nc;
    B.fft_flops += 2 * 5.0 * wl * std::log2((double)wl) * (double)nc;
    *out_len = ig.xlen;
    *out_fs = out;
    return push_ola(B, 1, fr, nc, wl, ig, 0, ig.xlen, out, false, true);
  }
  for (int64_t c = 0; c < nc; ++c) {
    SgFrame f{};
    f.src = sound + (int64_t)step[c] - 1;  // wave[x:(x + wl - 1)], x truncated
    const int64_t col = env_nc == 1 ? 0 : c * nr;
    f.env = env < 0 ? env - col : env + col;  // envelope area (encoded) or fl
    f.dst = fused ? -1 : fr + c * wl;
    B.frames[1].push_back(f);
    B.frame_geom[1].push_back(gi);
  }
  const IstftGeom ig = istft_geom(wl, nc, overlap);
  const int64_t out = fs_alloc(B, ig.xlen);
  B.fft_frames += nc;
  B.fft_flops += 2 * 5.0 * wl * std::log2((double)wl) * (double)nc;
  *out_len = ig.xlen;
  *out_fs = out;
  return push_ola(B, 1, fr, nc, wl, ig, 0, ig.xlen, out, fused);
}

bool plan_noise(Batch& B, Rng& R, int64_t len, const sg_anchors& noiseAnchors, double rolloffNoise,
                double attackLen, int wl, double sr, double overlap, const double* filterNoise, int64_t fnc,
                SgNoiseItem* item, int64_t filt_env) {
  ProfScope ps(PF_NOISE);
  // breathingStrength = getSmoothContour(noiseAnchors, len, valueFloor = -120, valueCeiling = 40)
  //   R/source.R:70-81 (NA when len == 0 or anchors NA)
  if (noiseAnchors.n <= 0 || len <= 0) return false;
  SgContour strength = contour_desc(B, noiseAnchors, len, true, -120, true, 40, true, sr);
  // step = seq(1, len + wl, by = hop); nr = wl / 2; nc = length(step)   R/source.R:88-94
  const int gi = geometry(B, wl);
  const double hop = (double)wl - overlap * (double)wl / 100;
  const int64_t nc = (int64_t)r_seq_by(1, (double)(len + wl), hop).size();
  const int64_t nr = wl / 2;
  // filter = [filterNoise or 1] * 2^(rolloffNoise / 10 * log2(1:nr)); column index per frame
  //   round(seq(1, ncol(filter), length.out = nc))   R/source.R:95-114
  const bool dev = filt_env < 0;  // device envelope job, rolloff included
  const int64_t ncolF = filterNoise || dev ? fnc : 1;
  int64_t filt_off = filt_env;
  if (!dev && !B.draws_only) {
    vec filt((size_t)(nr * ncolF));
    for (int64_t c = 0; c < ncolF; ++c)
      for (int64_t k = 0; k < nr; ++k)
        filt[c * nr + k] = (filterNoise ? filterNoise[c * nr + k] : 1.0) *
                           std::pow(2.0, rolloffNoise / 10 * std::log2((double)(k + 1)));
    filt_off = fl_push(B, filt.data(), (int64_t)filt.size());
  }
  vec fri((size_t)nc, 1.0);
  if ((filterNoise || dev) && !B.draws_only) {
    const vec s = r_seq_len(1, (double)ncolF, nc);
    for (int64_t c = 0; c < nc; ++c) fri[c] = r_round(s[c]);
  }
  // z1 = complex(real = runif(nr * nc)), column-major: bin fastest   R/source.R:111
  // (nr = wl / 2 is x.5 for an odd wl: floor(nr * nc) draws, matrix(nrow = nr)
  // keeps as.integer(nr) rows of them)
  const int64_t ndraw = (int64_t)((double)wl / 2 * (double)nc);
  const int64_t nu = std::min<int64_t>(ndraw, nr * nc);
  if (B.draws_only) {  // the item's length is all the caller's bout needs
    R.unif_f32(ndraw, nullptr);
    *item = SgNoiseItem{};
    item->len = len;
    item->ola = -1;
    return true;
  }
  int64_t u_off;
  if (ugather_on() && R.s && R.s->uniforms && R.iu + ndraw <= R.s->n_uniforms) {
    // every draw from the injected array: recorded, expanded on the device at upload
    const int64_t at = B.fu_total;
    B.fu_total += (nr * nc + 63) / 64 * 64;
    B.ugath.push_back(Batch::UGather{R.s->uniforms + R.iu, nu, at, (nr * nc + 3) / 4 * 4});
    R.iu += ndraw;
    u_off = -(at + 1);  // frame c: -(at + c nr + 1)
  } else {
    u_off = bulk_size(B.fl_x, B.fl);
    const int64_t u_loc = (int64_t)B.fl.size();
    B.fl.resize((size_t)(u_loc + (nr * nc + 3) / 4 * 4));  // the draws, then zeros to the 16-B pad
    R.unif_f32(nu, B.fl.data() + u_loc);
    std::fill(B.fl.begin() + u_loc + nu, B.fl.end(), 0.f);
    if (ndraw > nr * nc) R.unif_f32(ndraw - nr * nc, nullptr);
  }
  const bool fused = fusable(B.geoms[gi], (double)wl * (100 - overlap) / 100);
  const int64_t fr = fused ? 0 : fs_alloc(B, nc * wl);
  for (int64_t c = 0; c < nc; ++c) {
    SgFrame f{};
    f.src = u_off < 0 ? u_off - c * nr : u_off + c * nr;
    const int64_t col = ((int64_t)fri[c] - 1) * nr;
    f.env = dev ? filt_off - col : filt_off + col;
    f.dst = fused ? -1 : fr + c * wl;
    B.frames[0].push_back(f);
    B.frame_geom[0].push_back(gi);
  }
  // istft, then matchLengths(breathing, len, 'central')   R/utilities_math.R:413-444
  const IstftGeom ig = istft_geom(wl, nc, overlap);
  int64_t first = 0;
  if (ig.xlen != len) {
    const int64_t padded = ig.xlen < len ? ig.xlen + 2 * len : ig.xlen;
    const double halflen = (double)len / 2, center = (1 + (double)padded) / 2;
    const int64_t start = (int64_t)std::ceil(center - halflen);  // 1-based in the padded vector
    first = start - 1 - (ig.xlen < len ? len : 0);
  }
  const int64_t raw = fs_alloc(B, len);
  const int ola = push_ola(B, 0, fr, nc, wl, ig, first, len, raw, fused);
  B.fft_frames += nc;
  B.fft_flops += 1 * 5.0 * wl * std::log2((double)wl) * (double)nc;
  item->raw = raw;
  item->len = len;
  item->off = 0;
  item->ola = ola;  // phase-0 index == device index (noise OLAs come first)
  const double lf = std::floor(attackLen * sr / 1000);
  item->fade = (int32_t)(lf >= 2 ? std::min<double>(lf, (double)len) : 0);
  item->strength = strength;
  return true;
}

bool noise_to_fp64(Batch& B, const std::vector<int>& olas) {
  std::vector<SgFrame>& F = B.frames[0];
  int64_t first = (int64_t)F.size(), nf = 0;
  for (int o : olas) {
    const SgOla& O = B.olas[0][o];
    const int wl = O.wl;
    if (O.fidx < 0 || wl % 2 || wl > 4096 || !smooth31(wl / 2)) return false;  // sg_fft_frames64: M <= 2048, 31-smooth
    first = std::min<int64_t>(first, O.fidx);
    nf += O.nframes;
  }
  if (first + nf != (int64_t)F.size()) return false;  // not the tail of the frame list
  for (int o : olas) {
    SgOla& O = B.olas[0][o];
    if (O.fused) O.frames = fs_alloc(B, (int64_t)O.nframes * O.wl);  // frame scratch for sg_ola
    for (int32_t c = 0; c < O.nframes; ++c) {
      const SgFrame& f = F[(size_t)(O.fidx + c)];
      SgFrame64 g{};
      g.src = f.src;
      g.env = f.env;
      g.dst = O.frames + (int64_t)c * O.wl;
      g.wl = O.wl;
      g.mode = SG_F64_NOISE;
      B.frames64.push_back(g);
    }
    O.fidx = -1;
    O.fused = 0;
  }
  F.resize((size_t)first);
  B.frame_geom[0].resize((size_t)first);
  return true;
}

vec sigmoid_half(double sr, double freq, double shape, double spikiness) {
  // getSigmoid(), R/utilities_math.R:639-653: seq(from, to, length.out = sr / freq / 2)
  // (length.out rounded up), logistic, zeroOne
  const double from = -std::exp(-shape * spikiness), to = std::exp(shape * spikiness);
  const double slope = std::exp(std::fabs(shape)) * 5;
  const int64_t lo = (int64_t)std::ceil(sr / freq / 2);
  vec a = r_seq_len(from, to, lo);
  for (auto& v : a) v = 1 / (1 + std::exp(-v * slope));
  const double mn = r_min(a);
  for (auto& v : a) v -= mn;
  const double mx = r_max(a);
  for (auto& v : a) v /= mx;
  return a;
}

// ------------------------------------------------------------ envelope
namespace {
struct Track {
  vec time, freq, amp, width;
};
vec col_upsample(const double* t, const double* y, int64_t np, int64_t nPoints, double slf, int64_t nc) {
  // spline(approx(y, n = nPoints + 2^slf, x = time)$y, n = nc)   R/sourceSpectrum.R:326-335
  if (np <= 1) return vec((size_t)nc, y[0]);
  const vec xt(t, t + np), yt(y, y + np);
  const vec a = r_approx_n(xt, yt, (int64_t)((double)nPoints + std::pow(2.0, slf)));
  vec xs(a.size());
  for (size_t i = 0; i < xs.size(); ++i) xs[i] = (double)(i + 1);
  return r_spline(xs, a, nc);
}
}  // namespace

int64_t plan_envelope(Batch& B, Rng& R, double nrd, int64_t nc, const sg_formants* F, double formantDep,
                      double rolloffLip, const sg_anchors& mouthAnchors, double mouthOpenThres, double openMouthBoost,
                      double vocalTract, double temperature, double formDrift, double formDisp,
                      double formantDepStoch, double slf, double sr, double speedSound, double slope) {
  ProfScope ps(PF_ENVELOPE);
  const int64_t nr = (int64_t)nrd;  // matrix(nrow = nr): as.integer; bin_width keeps nrd
  int nF = F ? F->n_formants : 0;
  bool vtNull = std::isnan(vocalTract);
  double VT = vocalTract;
  std::vector<int32_t> np;
  vec t0, f0, a0, w0;  // concatenated input formants
  int f1_index = F ? F->f1_index : -1;
  if (nF > 0) {
    int64_t tot = 0;
    for (int f = 0; f < nF; ++f) { np.push_back(F->n_points[f]); tot += F->n_points[f]; }
    t0.assign(F->time, F->time + tot);
    f0.assign(F->freq, F->freq + tot);
    a0.assign(F->amp, F->amp + tot);
    w0.assign(F->width, F->width + tot);
  }
  // vocalTract guessed from formant dispersion when NULL   R/sourceSpectrum.R:293-307
  if (vtNull && nF > 0) {
    double fd = NAN;
    if (f0.size() >= 2) {
      vec d(f0.size() - 1);
      for (size_t i = 0; i + 1 < f0.size(); ++i) d[i] = f0[i + 1] - f0[i];
      fd = r_mean(d);
    }
    VT = speedSound / 2 / fd;
    vtNull = false;
  }
  // schwa from vocalTract when formants are NA   R/sourceSpectrum.R:309-322
  if (nF == 0 && !vtNull) {
    const double fr = speedSound / 4 / VT;
    np = {1};
    t0 = {0};
    f0 = {fr};
    a0 = {30};
    w0 = {50 * (1 + fr * fr / 6 / 1e6)};
    nF = 1;
    f1_index = 0;
  }
  vec mouth((size_t)nc, 0.5), mbin((size_t)nc, 1.0);
  SgEnvJob job{};
  job.nr = (int32_t)nr;
  job.nc = (int32_t)nc;
  job.slope = (float)slope;
  job.term0 = (int64_t)B.eterms.size();
  if (nF > 0) {
    int64_t nPoints = 0;
    for (int f = 0; f < nF; ++f) nPoints = std::max<int64_t>(nPoints, np[f]);
    std::vector<Track> fu(nF);
    int64_t off = 0;
    for (int f = 0; f < nF; ++f) {
      ProfScope pu(PF_ENV_UPS);
      // draws_only: the stochastic formants read the last track's frequencies alone
      if (!B.draws_only || f == nF - 1) fu[f].freq = col_upsample(&t0[off], &f0[off], np[f], nPoints, slf, nc);
      if (!B.draws_only) {
        fu[f].time = col_upsample(&t0[off], &t0[off], np[f], nPoints, slf, nc);
        fu[f].amp = col_upsample(&t0[off], &a0[off], np[f], nPoints, slf, nc);
        fu[f].width = col_upsample(&t0[off], &w0[off], np[f], nPoints, slf, nc);
      }
      off += np[f];
    }
    if (temperature > 0) {  // stochastic formants   R/sourceSpectrum.R:347-415
      ProfScope pst(PF_ENV_STOCH);
      double fdisp;
      if (vtNull && nF > 1) {
        vec c2(nF);
        int64_t o2 = 0;
        for (int f = 0; f < nF; ++f) { c2[f] = f0[o2] - (f ? f0[o2 - np[f - 1]] : 0); o2 += np[f]; }
        fdisp = r_mean(c2);
      } else if (!vtNull) {
        fdisp = 2 * speedSound / (4 * VT);
      } else {
        fdisp = NAN;
      }
      const double sdG = fdisp * temperature * formDisp;
      double fmax = r_max(fu.back().freq);
      if (!std::isnan(sdG) && formantDepStoch > 0) {
        while (fmax < (sr / 2 - 1000)) {
          vec rw = get_random_walk(R, nc, temperature * formDrift, 0, 1, vec{0.0}, false);
          if (rw.size() > 1) { const double m = r_mean(rw); for (auto& v : rw) v = v - m + 1; }
          const double g1 = R.rgamma(fdisp * fdisp / (sdG * sdG), fdisp / (sdG * sdG));
          Track t;
          if (!B.draws_only) t.time = fu[0].time;
          t.freq.resize(nc);
          for (int64_t c = 0; c < nc; ++c) t.freq[c] = fu.back().freq[c] + r_round(g1 * rw[rw.size() > 1 ? c : 0]);
          const double sh = (formantDep / temperature) * (formantDep / temperature);
          const double rt = formantDepStoch * formantDep / ((formantDepStoch * temperature) * (formantDepStoch * temperature));
          const double g2 = R.rgamma(sh, rt);
          t.amp.resize(nc);
          t.width.resize(nc);
          for (int64_t c = 0; c < nc && !B.draws_only; ++c) {
            t.amp[c] = r_round(g2 * rw[rw.size() > 1 ? c : 0]);
            t.width[c] = 50 + (std::log2(t.freq[c]) - 5) * 20;
          }
          fu.push_back(t);
          fmax = r_max(fu.back().freq);
        }
      }
      for (auto& tr : fu)
        for (int cc = 0; cc < 3; ++cc) {
          vec rw = get_random_walk(R, nc, temperature * formDrift, 0.3, 1, vec{}, true, B.draws_only);
          if (B.draws_only) continue;
          if (rw.size() > 1) { const double m = r_mean(rw); for (auto& v : rw) v = v - m + 1; }
          vec& col = cc == 0 ? tr.freq : cc == 1 ? tr.amp : tr.width;
          for (int64_t c = 0; c < nc; ++c) col[c] *= rw[rw.size() > 1 ? c : 0];
        }
    }
    // mouth opening   R/sourceSpectrum.R:426-456 (no draws: computed ahead of the bins, whose
    // shift below reads it)
    bool mouthNA = mouthAnchors.n < 1;
    for (int i = 0; i < mouthAnchors.n; ++i)
      if (std::isnan(mouthAnchors.value[i]) || std::isnan(mouthAnchors.time[i])) mouthNA = true;
    if (!mouthNA) {
      vec mo;
      if (!smooth_contour(mouthAnchors, nc, false, 0, true, 0, true, 1, mo)) mo.assign(nc, 0.5);
      for (int64_t c = 0; c < nc; ++c) {
        double v = mo[c];
        if (v < mouthOpenThres) v = 0;
        mouth[c] = v;
        mbin[c] = v > 0 ? 1 : 0;
      }
    }
    bool anyClosed = false;
    for (int64_t c = 0; c < nc; ++c) if (mbin[c] == 0) anyClosed = true;
    if (B.draws_only) {  // the envelope's last draw is behind; its one later error (the track count) in place
      if (fu.size() + (anyClosed && f1_index >= 0 ? 2 : 0) > 2 * 64)
        throw SgError(SG_E_UNSUPPORTED, "spectral envelope: more than 128 formant tracks");
      return 0;
    }
    // Hz -> bins   R/sourceSpectrum.R:417-424
    const double bw = sr / 2 / nrd;
    for (auto& tr : fu)
      for (int64_t c = 0; c < nc; ++c) {
        tr.freq[c] = (tr.freq[c] - bw / 2) / bw + 1;
        tr.width[c] = tr.width[c] / bw;
      }
    const bool adj = !vtNull && std::isfinite(VT);
    for (auto& tr : fu)
      for (int64_t c = 0; c < nc; ++c) {
        double ab = 0;
        if (adj) {
          const double ah = (mouth[c] - 0.5) * speedSound / (4 * VT);
          ab = (ah - bw / 2) / bw + 1;
        }
        tr.freq[c] += ab;
        if (tr.freq[c] < 1) tr.freq[c] = 1;
      }
    // nasalization when the mouth is closed   R/sourceSpectrum.R:469-504
    if (anyClosed && f1_index >= 0) {
      Track p = fu[f1_index], z = fu[f1_index];
      Track& f1 = fu[f1_index];
      for (int64_t c = 0; c < nc; ++c) {
        p.amp[c] = 0;
        if (mbin[c] == 0) {
          p.amp[c] = f1.amp[c] * 2 / 3;
          p.width[c] = f1.width[c] * 2 / 3;
          p.freq[c] = (f1.freq[c] > 550 / bw) ? f1.freq[c] - 250 / bw : f1.freq[c] + 250 / bw;
        }
      }
      for (int64_t c = 0; c < nc; ++c) {
        z.amp[c] = 0;
        if (mbin[c] == 0) {
          z.amp[c] = -f1.amp[c] * 2 / 3;
          z.freq[c] = (p.freq[c] + f1.freq[c]) / 2;
          z.width[c] = p.width[c];
        }
      }
      for (int64_t c = 0; c < nc; ++c)
        if (mbin[c] == 0) { f1.amp[c] = f1.amp[c] * 4 / 5; f1.width[c] = f1.width[c] * 5 / 4; }
      fu.push_back(p);
      fu.push_back(z);
    }
    // dgamma(1:nr, shape = mu^2/sd^2, rate = mu/sd^2), normalised by its column max,
    // times amp, summed over formants, times formantDep   R/sourceSpectrum.R:507-526
    // (terms emitted for sg_spec_env; the log-density max over the integer bins is
    // at floor or ceil of the mode (shape - 1) / rate, or at bin 1 for shape <= 1)
    const double L2E = 1.4426950408889634;  // 1 / ln 2
    // sg_spec_env holds two tracks per lane: more than 128 refuses THIS call (inside
    // plan_range's per-call try), not the whole batch at finalize_spec
    if (fu.size() > 2 * 64) throw SgError(SG_E_UNSUPPORTED, "spectral envelope: more than 128 formant tracks");
    job.ntr = (int32_t)fu.size();
    ProfScope pte(PF_ENV_TERMS);
    B.eterms.resize(B.eterms.size() + (size_t)(nc * job.ntr));
    SgEnvTerm* tm = &B.eterms[job.term0];
    for (int64_t c = 0; c < nc; ++c)
      for (size_t t = 0; t < fu.size(); ++t) {
        const Track& tr = fu[t];
        const double mg = tr.freq[c];
        double sdg = tr.width[c];
        if (sdg == 0) sdg = 1;
        const double shape = mg * mg / (sdg * sdg), rate = mg / (sdg * sdg);
        SgEnvTerm& e = tm[c * job.ntr + t];
        e = SgEnvTerm{};
        e.A = shape - 1;
        e.Rr = rate * L2E;
        // log2 density (+ const) at the integer bins k0, k1, as the device
        auto l2 = [&](double x) { return e.A * log2_int((int64_t)x) - e.Rr * x; };
        double kmax = 1;
        if (e.A > 0 && rate > 0) kmax = std::min((double)nr, std::max(1.0, e.A / rate));
        const double k0 = std::floor(kmax), k1 = std::min((double)nr, std::ceil(kmax));
        e.Lm = std::max(l2(k0), l2(k1));
        e.amp = tr.amp[c] * formantDep;
        e.ampf = (float)e.amp;
        // bins where the term is within 2^-SG_ENV_CUT of its column max (sg_dev.h): superset
        // from ln u - u + 1 <= -(u-1)^2/(2 max(u, 1))
        e.klo = 1;
        e.khi = (int32_t)nr;
        if (e.A > 0 && rate > 0) {
          const double xs = e.A / rate;
          const double lc = (e.A * std::log(xs) - rate * xs) - e.Lm / L2E;  // continuous max - integer max (>= 0)
          const double q = (SG_ENV_CUT / L2E + std::max(0.0, lc)) / e.A * (1 + 1e-6) + 1e-9;
          const double xlo = xs * (1 - std::sqrt(2 * q)), xhi = xs * (1 + q + std::sqrt(q * q + 2 * q));
          if (std::isfinite(xlo) && xlo > 2) e.klo = (int32_t)std::min<double>((double)nr + 1, std::floor(xlo) - 1);
          if (std::isfinite(xhi) && xhi < (double)nr - 1) e.khi = (int32_t)std::max(0.0, std::ceil(xhi) + 1);
        } else if (rate > 0) {
          const double xhi = 1 + SG_ENV_CUT / L2E / rate * (1 + 1e-6);
          if (std::isfinite(xhi) && xhi < (double)nr - 1) e.khi = (int32_t)std::ceil(xhi) + 1;
        }
        if (!std::isfinite(e.A) || !std::isfinite(e.Rr) || !std::isfinite(e.Lm)) {  // NaN track: no term passes the cut
          e.klo = 1;
          e.khi = 0;
        }
      }
  }
  if (B.draws_only) return 0;  // no formants: no draws
  // lip radiation, open-mouth boost, dB -> linear (2^(x/10))   R/sourceSpectrum.R:524-541
  job.col0 = (int64_t)B.ecols.size();
  for (int64_t c = 0; c < nc; ++c)
    B.ecols.push_back(SgEnvCol{(float)(rolloffLip * mbin[c]), (float)std::pow(2.0, mouth[c] * openMouthBoost / 10)});
  job.out = B.fe_total;
  B.fe_total += (nr * nc + 63) / 64 * 64;
  B.envjobs.push_back(job);
  return -(job.out + 1);
}

// ------------------------------------------------------------ finalize
void finalize_spec(Batch& B) {
  // envelope area after the uploaded floats: decode frame envelope offsets;
  // sg_spec_env wave tasks of SG_ENV_COLS columns
  B.fe_base = (bulk_size(B.fl_x, B.fl) + 63) / 64 * 64;
  B.fu_base = B.fe_base + (B.fe_total + 63) / 64 * 64;
  for (int ph = 0; ph < 2; ++ph)
    for (SgFrame& f : B.frames[ph]) {
      if (f.env < 0) f.env = B.fe_base + (-f.env - 1);
      if (ph == 0 && f.src < 0) f.src = B.fu_base + (-f.src - 1);
    }
  // gathered noise uniforms: the union of the callers' draw ranges, once, as floats
  // (C5: every call reads a window of one stream); one device job per item
  B.ustream.clear();
  B.ujobs.assign(B.ugath.size(), SgUJob{});
  if (!B.ugath.empty()) {
    std::vector<int64_t> ord(B.ugath.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = (int64_t)i;
    auto lo = [&](int64_t i) { return (uintptr_t)B.ugath[i].src; };
    std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return lo(a) < lo(b); });
    size_t k = 0;
    while (k < ord.size()) {
      const double* r0 = B.ugath[ord[k]].src;
      uintptr_t end = lo(ord[k]) + 8 * (uintptr_t)B.ugath[ord[k]].n;
      size_t k1 = k + 1;
      while (k1 < ord.size() && lo(ord[k1]) <= end) {
        end = std::max<uintptr_t>(end, lo(ord[k1]) + 8 * (uintptr_t)B.ugath[ord[k1]].n);
        ++k1;
      }
      const int64_t base = (int64_t)B.ustream.size(), n = (int64_t)((end - (uintptr_t)r0) / 8);
      B.ustream.resize((size_t)(base + n));
      for (int64_t j = 0; j < n; ++j) B.ustream[(size_t)(base + j)] = (float)r0[j];
      for (size_t q = k; q < k1; ++q) {
        const Batch::UGather& g = B.ugath[ord[q]];
        B.ujobs[ord[q]] = SgUJob{base + (g.src - r0), B.fu_base + g.dst, g.n, g.ntot};
      }
      k = k1;
    }
  }
  B.ugath.clear();
  B.ugath.shrink_to_fit();
  // fp64 frames: one root table W_N^t per window length (sg_roots64)
  B.roots64_wl.clear();
  B.roots64_off.clear();
  B.frames64_tab.clear();
  B.roots64_total = 0;
  B.frames64_maxwl = 0;
  // noise frames first (launched in phase 0, before the noise OLAs), then the filter frames;
  // OLAs address the frames' scratch outputs, not their order
  B.frames64_noise = std::stable_partition(B.frames64.begin(), B.frames64.end(),
                                           [](const SgFrame64& f) { return f.mode == SG_F64_NOISE; }) -
                     B.frames64.begin();
  // within each phase, the wl = 2204 frames first (sg_fft_frames64w, a frame per wavefront)
  {
    auto w = [](const SgFrame64& f) { return f.wl == 2 * SG_F64W_M_HOST; };
    const auto mid = B.frames64.begin() + B.frames64_noise;
    B.frames64_w[0] = std::stable_partition(B.frames64.begin(), mid, w) - B.frames64.begin();
    B.frames64_w[1] = std::stable_partition(mid, B.frames64.end(), w) - mid;
  }
  for (SgFrame64& f : B.frames64) {
    if (f.env < 0) f.env = B.fe_base + (-f.env - 1);
    if (f.mode == SG_F64_NOISE && f.src < 0) f.src = B.fu_base + (-f.src - 1);
    size_t w = 0;
    while (w < B.roots64_wl.size() && B.roots64_wl[w] != f.wl) ++w;
    if (w == B.roots64_wl.size()) {
      B.roots64_wl.push_back(f.wl);
      B.roots64_off.push_back(B.roots64_total);
      B.roots64_total += 2 * (int64_t)f.wl;  // W_N^t (N), then the fp64 hamming and hanning pairs (M each)
    }
    B.frames64_tab.push_back(B.roots64_off[w]);
    B.frames64_maxwl = std::max(B.frames64_maxwl, f.wl);
  }
  int32_t maxnr = 0;
  for (const SgEnvJob& j : B.envjobs) {
    maxnr = std::max(maxnr, j.nr);
    if (j.ntr > 2 * 64) throw SgError(SG_E_DEVICE, "spectral envelope: more than 128 formant tracks (planner check)");
  }
  // log2(k) for k = 1.. (padded to whole 64-bin chunks): spectral envelopes' bins and
  // the device amplitude formula's rolloff rows (sg_amp.h)
  B.elog2.resize((size_t)std::max<int64_t>(maxnr, B.amp_lg_rows) + 64);
  for (size_t k = 0; k < B.elog2.size(); ++k) B.elog2[k] = std::log2((double)(k + 1));
  B.envtasks.clear();
  for (size_t j = 0; j < B.envjobs.size(); ++j)
    for (int32_t c0 = 0; c0 < B.envjobs[j].nc; c0 += SG_ENV_COLS) B.envtasks.push_back(SgEnvTask{(int32_t)j, c0});
  auto cost = [&](const SgEnvTask& t) {  // sg_spec_env work of a task ~ columns x 128-bin chunks x tracks
    const SgEnvJob& J = B.envjobs[t.job];
    return (double)std::min<int32_t>(SG_ENV_COLS, J.nc - t.c0) * (double)((J.nr + 127) / 128) * (double)J.ntr;
  };
  // the costliest tasks first, so each workgroup's four waves carry about the same work
  // (in job order a workgroup mixed a job's last, partial task with the next job's)
  if (SG_ENV_SORT)
    std::stable_sort(B.envtasks.begin(), B.envtasks.end(),
                     [&](const SgEnvTask& a, const SgEnvTask& b) { return cost(a) > cost(b); });
  if (std::getenv("SG_DEBUG_PLAN")) {  // sg_spec_env workgroup balance
    double wmax = 0, wsum = 0;
    for (size_t i = 0; i < B.envtasks.size(); i += 4) {
      double mx = 0;
      for (size_t w = i; w < i + 4 && w < B.envtasks.size(); ++w) { mx = std::max(mx, cost(B.envtasks[w])); wsum += cost(B.envtasks[w]); }
      wmax += 4 * mx;
    }
    std::fprintf(stderr, "sg plan: envelope tasks %zu, workgroup cost %.3g, used %.3g (%.1f%% idle)\n", B.envtasks.size(), wmax,
                 wsum, wmax > 0 ? 100.0 * (wmax - wsum) / wmax : 0.0);
  }
  // frames: per phase, sorted by (kernel, geometry), stable so that the
  // frames of one OLA stay consecutive; groups for the workgroup kernel only
  B.fgroups.clear();
  std::vector<int64_t> pos[2];
  for (int ph = 0; ph < 2; ++ph) {
    // a stable counting sort over the geometries (few keys; 2.8 M frames per 16,384 C5
    // calls: a comparison sort was 90 % of finalize_spec)
    const size_t ng = B.geoms.size();
    std::vector<int64_t> rank(ng), start(ng + 1, 0);
    {
      std::vector<int32_t> og(ng);
      for (size_t g = 0; g < ng; ++g) og[g] = (int32_t)g;
      std::stable_sort(og.begin(), og.end(), [&](int32_t a, int32_t b) {
        const int ka = B.geoms[a].kind == SG_FFT_WAVE ? 0 : 1, kb = B.geoms[b].kind == SG_FFT_WAVE ? 0 : 1;
        return ka != kb ? ka < kb : a < b;
      });
      for (size_t r = 0; r < ng; ++r) rank[og[r]] = (int64_t)r;
    }
    for (int32_t gi : B.frame_geom[ph]) ++start[rank[gi] + 1];
    for (size_t r = 0; r < ng; ++r) start[r + 1] += start[r];
    std::vector<int64_t> idx(B.frames[ph].size());
    for (size_t i = 0; i < idx.size(); ++i) idx[start[rank[B.frame_geom[ph][i]]]++] = (int64_t)i;
    std::vector<SgFrame> fr(idx.size());
    std::vector<int32_t> fg(idx.size());
    pos[ph].assign(idx.size(), 0);
    for (size_t i = 0; i < idx.size(); ++i) {
      fr[i] = B.frames[ph][idx[i]];
      fg[i] = B.frame_geom[ph][idx[i]];
      pos[ph][idx[i]] = (int64_t)i;
    }
    B.frames[ph] = fr;
    B.frame_geom[ph] = fg;
    const int32_t base = ph == 0 ? 0 : (int32_t)B.frames[0].size();
    B.fgroup_lds[ph][0] = B.fgroup_lds[ph][1] = 0;
    B.fgroup_range[ph][0] = B.fgroup_range[ph][1] = (int64_t)B.fgroups.size();
    for (size_t i = 0; i < fr.size();) {
      const int gi = fg[i];
      const SgFftGeom& g = B.geoms[gi];
      if (g.kind == SG_FFT_WAVE) {  // transformed inside sg_stft_ola
        // + the radix-29 fragment table of the specialised M = 1102 path (sg_fft.hip SG_MAT29_BYTES)
        B.fgroup_lds[ph][0] = std::max(B.fgroup_lds[ph][0], (sg_fft_waves(ph) + 4) * g.M * 8 + (g.M == 1102 ? 2048 : 0));
        ++i;
        continue;
      }
      size_t j = i;
      while (j < fr.size() && fg[j] == gi && (int)(j - i) < g.fb) ++j;
      B.fgroups.push_back(SgFrameGroup{gi, ph == 0 ? SG_FRAME_NOISE : SG_FRAME_FILTER, base + (int32_t)i,
                                       (int32_t)(j - i)});
      B.fgroup_lds[ph][1] = std::max(B.fgroup_lds[ph][1], g.lds_bytes);
      i = j;
    }
    B.fgroup_range[ph][2] = (int64_t)B.fgroups.size();
  }
  // OLAs: device table [noise..., filter...]; unfused ones get sg_ola tiles
  // (slots [0, #tiles)), fused ones sg_stft_ola segments (slots after them)
  B.olas_dev.clear();
  B.olatiles.clear();
  B.olasegs.clear();
  B.ola_split = (int64_t)B.olas[0].size();
  for (int ph = 0; ph < 2; ++ph) {
    if (ph == 1) B.olatile_split = (int64_t)B.olatiles.size();
    const int32_t base = ph == 0 ? 0 : (int32_t)B.frames[0].size();
    for (const SgOla& o0 : B.olas[ph]) {
      SgOla o = o0;
      if (o0.fidx >= 0) o.fidx = base + (int32_t)pos[ph][o0.fidx];
      const int32_t oi = (int32_t)B.olas_dev.size();
      if (!o.fused) {
        o.tile0 = (int32_t)B.olatiles.size();
        for (int64_t q0 = 0; q0 < o.len; q0 += SG_OLA_TILE) B.olatiles.push_back(SgOlaTile{oi, 0, q0});
        o.nslot = (int32_t)B.olatiles.size() - o.tile0;
      }
      B.olas_dev.push_back(o);
    }
  }
  const int32_t nt = (int32_t)B.olatiles.size();
  int32_t nslots = 0;  // real segments so far (slots nt + nslots)
  B.stft_bytes = B.stft_samples = 0;
  B.stft_flops = 0;
  for (int ph = 0; ph < 2; ++ph) {
    B.seg_range[ph][0] = (int64_t)B.olasegs.size();
    const size_t o_lo = ph == 0 ? 0 : (size_t)B.ola_split, o_hi = ph == 0 ? (size_t)B.ola_split : B.olas_dev.size();
    const int32_t fbase = ph == 0 ? 0 : (int32_t)B.frames[0].size();
    const int WPH = sg_fft_waves(ph);
    // fused OLAs of the phase ordered by geometry; a workgroup's WPH (sg_fft_waves)
    // segments share one geometry (padding segments have nf = 0)
    std::vector<size_t> order;
    for (size_t oi = o_lo; oi < o_hi; ++oi)
      if (B.olas_dev[oi].fused) order.push_back(oi);
    auto geom_of = [&](size_t oi) { return B.frame_geom[ph][B.olas_dev[oi].fidx - fbase]; };
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return geom_of(a) < geom_of(b); });
    // Segment length: sg_seg_frames(ph) frames would leave a partial last round of
    // workgroups (one per CU), so pick the length that packs the segments into
    // whole rounds of sg_resident_waves(ph) (the fewest rounds sg_seg_frames(ph) needs).
    const int64_t SEG = sg_seg_frames(ph);
    int64_t seg_frames = SEG;
    {
      auto segs_at = [&](int64_t S) {
        int64_t tot = 0, run = 0;
        int prev = -2;
        for (size_t oi : order) {
          const int g = geom_of(oi);
          if (g != prev) {
            tot += (WPH - run % WPH) % WPH;  // padding of the previous geometry
            run = 0;
            prev = g;
          }
          const int64_t k = std::max<int64_t>(1, (B.olas_dev[oi].nframes + S - 1) / S);
          tot += k;
          run += k;
        }
        return tot + (WPH - run % WPH) % WPH;
      };
      const int64_t base = segs_at(SEG);
      const int64_t rounds = (base + sg_resident_waves(ph) - 1) / sg_resident_waves(ph);
      int64_t S = SG_SEG_MIN_FRAMES;
      while (S < SEG && segs_at(S) > rounds * sg_resident_waves(ph)) S = std::max(S + 1, S * 9 / 8);
      seg_frames = std::min<int64_t>(S, SEG);
    }
    int cur_geom = -1;
    size_t group0 = B.olasegs.size();  // first segment of the current geometry
    auto pad = [&]() {
      // a workgroup lasts as long as its longest segment: the geometry's segments go
      // longest first, so each workgroup's WPH segments have about the same length
      // (in OLA order the idle share was 10 % of the filter and 16 % of the noise
      // workgroups' wave-frames at C5). A segment's outputs and max slot are its own,
      // so the order changes no value.
      if (SG_SEG_SORT)
        std::stable_sort(B.olasegs.begin() + (std::ptrdiff_t)group0, B.olasegs.end(),
                         [](const SgSegment& a, const SgSegment& b) { return a.nf > b.nf; });
      while (((int64_t)B.olasegs.size() - B.seg_range[ph][0]) % WPH) {
        SgSegment d{};
        d.geom = cur_geom;
        B.olasegs.push_back(d);
      }
    };
    for (size_t oi : order) {
      SgOla& o = B.olas_dev[oi];
      const int gi = geom_of(oi);
      if (gi != cur_geom) {
        pad();
        cur_geom = gi;
        group0 = B.olasegs.size();
      }
      auto bstart = [&](int64_t f) -> int64_t {
        return o.hi > 0 ? f * o.hi : (int64_t)std::floor((double)f * o.h);
      };
      const int64_t n = o.nframes;
      const int64_t nseg = std::max<int64_t>(1, (n + seg_frames - 1) / seg_frames);
      {  // algorithmic bytes / flops of this OLA in sg_stft_ola (bench roofline)
        const int64_t nr = o.wl / 2;
        int64_t ncol = 0, prev = -1;
        for (int64_t f = 0; f < n; ++f) {
          const int64_t e = B.frames[ph][o.fidx - fbase + f].env;
          if (e != prev) ++ncol;
          prev = e;
        }
        const double fft = 5.0 * o.wl * std::log2((double)o.wl);
        if (ph == 0) {  // noise: uniforms nr per frame + filter columns + trimmed output
          B.stft_bytes += 4 * (nr * n + nr * ncol + o.len);
          B.stft_flops += fft * n;
        } else {  // filter: the sound under the frames + envelope columns + trimmed output
          B.stft_bytes += 4 * (std::min<int64_t>(o.xlen, o.wl + (int64_t)std::ceil((n - 1) * o.h)) + nr * ncol + o.len);
          B.stft_flops += 2 * fft * n;
        }
        B.stft_samples += o.len;
      }
      o.tile0 = nt + nslots;
      o.nslot = (int32_t)nseg;
      for (int64_t k = 0; k < nseg; ++k) {
        const int64_t F0 = k * n / nseg, F1 = (k + 1) * n / nseg;
        SgSegment sg{};
        sg.ola = (int32_t)oi;
        sg.geom = gi;
        sg.mode = ph == 0 ? SG_FRAME_NOISE : SG_FRAME_FILTER;
        sg.pa = k == 0 ? 0 : (int32_t)bstart(F0);
        sg.pb = k == nseg - 1 ? (int32_t)o.xlen : (int32_t)bstart(F1);
        int64_t f0 = F0;
        while (f0 > 0 && bstart(f0 - 1) + o.wl > sg.pa) --f0;  // frames overlapping the first owned sample
        sg.f0 = (int32_t)f0;
        sg.nf = (int32_t)(F1 - f0);
        sg.fdev = o.fidx + (int32_t)f0;
        sg.slot = nt + nslots++;
        sg.flags = (k == 0 ? SG_SEG_FIRST : 0) | (k == nseg - 1 ? SG_SEG_LAST : 0);
        B.olasegs.push_back(sg);
      }
    }
    pad();
    B.seg_range[ph][1] = (int64_t)B.olasegs.size();
  }
  B.n_segslots = nslots;
  if (std::getenv("SG_DEBUG_PLAN")) {
    int64_t owned = 0, run = 0, real = 0;
    for (const SgSegment& sg : B.olasegs) {
      if (sg.nf <= 0) continue;
      ++real;
      run += sg.nf;
    }
    for (const SgOla& o : B.olas_dev) if (o.fused) owned += o.nframes;
    for (int ph = 0; ph < 2; ++ph) {
      int64_t fr = 0, sgs = 0;
      for (int64_t i = B.seg_range[ph][0]; i < B.seg_range[ph][1]; ++i)
        if (B.olasegs[i].nf > 0) { fr += B.olasegs[i].nf; ++sgs; }
      std::fprintf(stderr, "sg plan: phase %d: %lld frames computed in %lld segments (%zu frames, %zu unfused groups)\n", ph,
                   (long long)fr, (long long)sgs, B.frames[ph].size(), (size_t)(B.fgroup_range[ph][2] - B.fgroup_range[ph][1]));
      // workgroup balance: a workgroup lasts as long as its longest segment
      const int WPH = sg_fft_waves(ph);
      int64_t wmax = 0, wsum = 0;
      for (int64_t i = B.seg_range[ph][0]; i < B.seg_range[ph][1]; i += WPH) {
        int64_t mx = 0;
        for (int w = 0; w < WPH && i + w < B.seg_range[ph][1]; ++w) mx = std::max<int64_t>(mx, B.olasegs[i + w].nf);
        wmax += mx * WPH;
        for (int w = 0; w < WPH && i + w < B.seg_range[ph][1]; ++w) wsum += std::max<int32_t>(0, B.olasegs[i + w].nf);
      }
      std::fprintf(stderr, "sg plan: phase %d: workgroup wave-frames %lld, used %lld (%.1f%% idle)\n", ph, (long long)wmax,
                   (long long)wsum, wmax ? 100.0 * (double)(wmax - wsum) / (double)wmax : 0.0);
    }
    std::map<int32_t, int64_t> gfr;  // fused frames per geometry
    for (const SgSegment& sg : B.olasegs)
      if (sg.nf > 0) gfr[sg.geom] += sg.nf;
    std::vector<std::pair<int64_t, int32_t>> gs;
    for (const auto& kv : gfr) gs.push_back({kv.second, kv.first});
    std::sort(gs.rbegin(), gs.rend());
    for (size_t i = 0; i < gs.size() && i < 16; ++i) {
      const SgFftGeom& g = B.geoms[gs[i].second];
      std::string rs;
      for (int s = 0; s < g.nstages; ++s) rs += (s ? "x" : "") + std::to_string(g.radix[s]);
      std::fprintf(stderr, "sg plan: geom wl=%d M=%d radices %s: %lld frames\n", g.wl, g.M, rs.c_str(),
                   (long long)gs[i].first);
    }
    std::map<int32_t, int64_t> gun;  // unfused (sg_fft_frames) frames per geometry
    for (const SgFrameGroup& fg : B.fgroups) gun[fg.geom] += fg.nf;
    for (const auto& kv : gun) {
      const SgFftGeom& g = B.geoms[kv.first];
      std::string rs;
      for (int s = 0; s < g.nstages; ++s) rs += (s ? "x" : "") + std::to_string(g.radix[s]);
      std::fprintf(stderr, "sg plan: unfused geom wl=%d M=%d kind %d radices %s: %lld frames\n", g.wl, g.M, g.kind,
                   rs.c_str(), (long long)kv.second);
    }
    std::fprintf(stderr, "sg plan: %lld fused segments (%lld slots incl. padding), %lld frames owned, %lld computed (%.1f%% recomputed)\n",
                 (long long)real, (long long)B.olasegs.size(), (long long)owned, (long long)run,
                 owned ? 100.0 * (double)(run - owned) / (double)owned : 0.0);
  }
  // items and mixes referring to filter-phase OLAs: device index = ola_split + i
  for (SgNoiseItem& it : B.items)
    if (it.flags & SG_ITEM_FILTER_OLA) {
      it.ola += (int32_t)B.ola_split;
      it.flags &= ~SG_ITEM_FILTER_OLA;
    }
  // mixes: [pre-filter..., final...]
  B.mixes_dev.clear();
  B.mixtiles.clear();
  // mixes: [pre-filter fp32..., pre-filter fp64 (to fh)..., final...]
  for (int pass = 0; pass < 3; ++pass) {
    const int ph = pass == 2 ? 1 : 0;
    if (pass == 1) B.mixtile_hp = (int64_t)B.mixtiles.size();
    if (pass == 2) B.mixtile_split = (int64_t)B.mixtiles.size();
    for (const SgMix& m0 : B.mixes[ph]) {
      if (ph == 0 && (m0.to_fs == 2) != (pass == 1)) continue;
      const int32_t mi = (int32_t)B.mixes_dev.size();
      for (int64_t k0 = 0; k0 < m0.len; k0 += SG_MIX_TILE) B.mixtiles.push_back(SgMixTile{mi, 0, k0});
      SgMix m = m0;
      if (m.base_kind == SG_BASE_NORM) m.base_ola += (int32_t)B.ola_split;
      B.mixes_dev.push_back(m);
    }
  }
}

}  // namespace sg

extern "C" int sg_set_uniform_gather(int32_t on) {
  if (on < 0 || on > 1) return SG_E_ARG;
  sg::g_ugather.store(on);
  return SG_OK;
}
