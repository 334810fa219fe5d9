// sg_plan_soundgen.cpp — host planner of soundgen() (R/soundgen.R:208-862):
// argument checks and hyper-parameters, stochastic syllable segmentation,
// per-syllable wiggling, the voiced part (plan_harmonics), the noise
// (plan_noise), the addVectors() layout, the formant filter (plan_filter)
// and the bout assembly. Every random draw happens here in the reference's
// order; every length is an integer computed in fp64 like R does. The
// per-sample work is emitted as device descriptors (syllables, noise frames,
// filter frames, OLAs, mixes) executed by sg_exec.cpp.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <optional>

#include "sg_plan.h"

namespace sg {

namespace {

// permittedValues rows 1..'rolloffNoise' (R/presets.R:22-56): default, low, high
constexpr int kNPV = 33;
const char* const kPVNames[kNPV] = {
    "repeatBout", "nSyl", "sylLen", "pauseLen", "temperature", "maleFemale", "creakyBreathy", "nonlinBalance",
    "nonlinDep", "jitterDep", "jitterLen", "vibratoFreq", "vibratoDep", "shimmerDep", "attackLen", "rolloff",
    "rolloffOct", "rolloffParab", "rolloffParabHarm", "rolloffKHz", "rolloffLip", "formantDep", "formantDepStoch",
    "vocalTract", "subFreq", "subDep", "shortestEpoch", "amDep", "amFreq", "amShape", "samplingRate",
    "windowLength", "rolloffNoise"};
const double kPV[kNPV][3] = {
    {1, 1, 20}, {1, 1, 10}, {300, 20, 5000}, {200, 20, 1000}, {.025, 0, 1}, {0, -1, 1}, {0, -1, 1},
    {0, 0, 100}, {50, 0, 100}, {3, 0, 24}, {1, 1, 100}, {5, 3, 10}, {0, 0, 3}, {0, 0, 100},
    {50, 0, 200}, {-12, -60, 0}, {-12, -30, 10}, {0, -50, 50}, {3, 1, 20}, {-6, -20, 0},
    {6, 0, 20}, {1, 0, 5}, {30, 0, 60}, {15.5, 2, 100}, {100, 10, 1000}, {100, 0, 500},
    {300, 50, 500}, {0, 0, 100}, {30, 10, 100}, {0, -1, 1}, {16000, 8000, 44100}, {40, 5, 100},
    {-14, -20, 20}};
constexpr double kSylLow = 20, kSylHigh = 5000, kPauseLow = 20, kPauseHigh = 1000;

double* slot(sg_soundgen_args& a, int i) {
  double* s[kNPV] = {&a.repeatBout, &a.nSyl, &a.sylLen, &a.pauseLen, &a.temperature, &a.maleFemale,
                     &a.creakyBreathy, &a.nonlinBalance, &a.nonlinDep, &a.jitterDep, &a.jitterLen,
                     &a.vibratoFreq, &a.vibratoDep, &a.shimmerDep, &a.attackLen, &a.rolloff, &a.rolloffOct,
                     &a.rolloffParab, &a.rolloffParabHarm, &a.rolloffKHz, &a.rolloffLip, &a.formantDep,
                     &a.formantDepStoch, &a.vocalTract, &a.subFreq, &a.subDep, &a.shortestEpoch, &a.amDep,
                     &a.amFreq, &a.amShape, &a.samplingRate, &a.windowLength, &a.rolloffNoise};
  return s[i];
}

// anchors with owned storage
struct Anc {
  vec t, v;
  sg_anchors view() const { return sg_anchors{(int32_t)t.size(), t.data(), v.data()}; }
  int64_t n() const { return (int64_t)t.size(); }
};
Anc anc(const sg_anchors& a) {
  Anc r;
  if (a.n > 0) { r.t.assign(a.time, a.time + a.n); r.v.assign(a.value, a.value + a.n); }
  return r;
}

// rbinom(1, 1, p) — R's inversion algorithm for size 1 (nmath/rbinom.c):
// no draw when p == 0; else u = unif_rand(), outcome (u >= 1 - p) for p <= .5,
// (u < p) for p > .5
double rbinom1(Rng& R, double p) {
  if (p == 0) return 0;
  if (p == 1) return 1;
  const double u = R.unif();
  return p <= 0.5 ? (u >= 1 - p ? 1 : 0) : (u < p ? 1 : 0);
}

// rnorm_bounded(), R/utilities_math.R:187-231
vec rnorm_bounded(Rng& R, int64_t n, const vec& mean_in, const vec& sd_in, const vec* low, const vec* high,
                  bool roundToInteger) {
  vec mean((size_t)n), sd((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    mean[i] = mean_in[mean_in.size() >= (size_t)n ? i : 0];
    sd[i] = sd_in[sd_in.size() >= (size_t)n ? i : 0];
  }
  auto lo = [&](int64_t i) { return low ? (*low)[low->size() > 1 ? i : 0] : -INFINITY; };
  auto hi = [&](int64_t i) { return high ? (*high)[high->size() > 1 ? i : 0] : INFINITY; };
  for (int64_t i = 0; i < n; ++i) {
    if (mean[i] < lo(i)) mean[i] = lo(i);
    if (mean[i] > hi(i)) mean[i] = hi(i);
  }
  bool anysd = false;
  for (double s : sd) if (s != 0) anysd = true;
  vec out(mean);
  if (!anysd) {
    if (roundToInteger) for (auto& v : out) v = r_round(v);
    return out;
  }
  for (int64_t i = 0; i < n; ++i) out[i] = R.rnorm(mean[i], sd[i]);
  if (roundToInteger) for (auto& v : out) v = r_round(v);
  if (!low && !high) return out;
  for (int64_t i = 0; i < n; ++i) {
    int guard = 0;
    while (out[i] < lo(i) || out[i] > hi(i)) {
      out[i] = R.rnorm(mean[i], sd[i]);
      if (roundToInteger) for (auto& v : out) v = r_round(v);
      if (++guard > 100000) throw SgError(SG_E_RANDOM, "rnorm_bounded: rejection loop too long");
    }
  }
  return out;
}
double rnorm_bounded1(Rng& R, double mean, double sd, double low, double high, bool rnd) {
  vec lo{low}, hi{high};
  return rnorm_bounded(R, 1, vec{mean}, vec{sd}, &lo, &hi, rnd)[0];
}

// sample(x, 1, prob) without replacement, R < 3.6 (ProbSampleNoReplace with revsort)
int sample_prob1(Rng& R, const double* prob, int n) {
  std::vector<double> p(n);
  std::vector<int> perm(n);
  double tot = 0;
  for (int i = 0; i < n; ++i) tot += prob[i];
  for (int i = 0; i < n; ++i) { p[i] = prob[i] / tot; perm[i] = i + 1; }
  // revsort (sort.c): heap sort into decreasing order carrying the index
  auto a = [&](int k) -> double& { return p[k - 1]; };
  auto ib = [&](int k) -> int& { return perm[k - 1]; };
  if (n > 1) {
    int l = (n >> 1) + 1, ir = n;
    for (;;) {
      double ra;
      int ii;
      if (l > 1) { l = l - 1; ra = a(l); ii = ib(l); }
      else {
        ra = a(ir); ii = ib(ir); a(ir) = a(1); ib(ir) = ib(1);
        if (--ir == 1) { a(1) = ra; ib(1) = ii; break; }
      }
      int i = l, j = l << 1;
      while (j <= ir) {
        if (j < ir && a(j) > a(j + 1)) ++j;
        if (ra > a(j)) { a(i) = a(j); ib(i) = ib(j); j += (i = j); }
        else j = ir + 1;
      }
      a(i) = ra;
      ib(i) = ii;
    }
  }
  const double rT = R.unif();
  double mass = 0;
  int j = 0;
  for (j = 0; j < n - 1; j++) { mass += p[j]; if (rT <= mass) break; }
  return perm[j];
}
int64_t unif_index(Rng& R, double dn) { return (int64_t)std::floor(dn * R.unif()); }  // R < 3.6 "Rounding"

// wiggleAnchors() for (time, value) anchors, R/utilities_soundgen.R:634-735
void wiggle_anchors(Rng& R, Anc& df, double T, double coef, const double low[2], const double high[2], bool allRows) {
  if (df.n() < 1) return;
  for (int64_t i = 0; i < df.n(); ++i) if (std::isnan(df.t[i]) || std::isnan(df.v[i])) return;
  const double prob[3] = {1 - T, T / 2, T / 2};
  const int action = sample_prob1(R, prob, 3);
  if (action == 3) {  // add
    if (df.n() == 1) {
      const double m = df.v[0], sd = df.v[0] * T * coef;
      const double na = rnorm_bounded1(R, m, sd, low[1], high[1], false);
      df.t = {0, 1};
      df.v = {df.v[0], na};
    } else {
      const int64_t a1 = unif_index(R, (double)df.n()) + 1;
      const int64_t dir = unif_index(R, 2.0) == 0 ? -1 : 1;
      const int64_t a2 = (a1 + dir < 1 || a1 + dir > df.n()) ? a1 - dir : a1 + dir;
      const int64_t i1 = std::min(a1, a2), i2 = std::max(a1, a2);
      long double st = 0, sv = 0;
      for (int64_t k = i1; k <= i2; ++k) { st += df.t[k - 1]; sv += df.v[k - 1]; }
      const double nt = (double)(st / (i2 - i1 + 1)), nv = (double)(sv / (i2 - i1 + 1));
      Anc o;
      for (int64_t k = 1; k <= i1; ++k) { o.t.push_back(df.t[k - 1]); o.v.push_back(df.v[k - 1]); }
      o.t.push_back(nt);
      o.v.push_back(nv);
      for (int64_t k = i2; k <= df.n(); ++k) { o.t.push_back(df.t[k - 1]); o.v.push_back(df.v[k - 1]); }
      df = o;
    }
  } else if (action == 2) {  // remove
    int64_t idx = 0;
    if (allRows) idx = unif_index(R, (double)df.n()) + 1;
    else if (df.n() > 2) idx = unif_index(R, (double)(df.n() - 2)) + 2;
    if (idx) { df.t.erase(df.t.begin() + idx - 1); df.v.erase(df.v.begin() + idx - 1); }
  }
  const double orig0 = df.t.front(), orig1 = df.t.back();
  double rng_[2];
  if (df.n() == 1) { rng_[0] = df.t[0]; rng_[1] = df.v[0]; }
  else {
    rng_[0] = std::fabs(r_max(df.t) - r_min(df.t));
    rng_[1] = std::fabs(r_max(df.v) - r_min(df.v));
    if (rng_[0] == 0) rng_[0] = std::fabs(df.t[0]);
    if (rng_[1] == 0) rng_[1] = std::fabs(df.v[0]);
  }
  vec* cols[2] = {&df.t, &df.v};
  for (int i = 0; i < 2; ++i) {
    vec lo{low[i]}, hi{high[i]};
    *cols[i] = rnorm_bounded(R, df.n(), *cols[i], vec{rng_[i] * T * coef}, &lo, &hi, false);
  }
  if (!allRows) { df.t.front() = orig0; df.t.back() = orig1; }
}

// divideIntoSyllables(), R/utilities_soundgen.R:515-566
void divide_into_syllables(Rng& R, int64_t nSyl, double sylLen, double pauseLen, double T, vec& st, vec& en) {
  st.assign(nSyl, 0);
  en.assign(nSyl, 0);
  if (nSyl == 1) { st[0] = 0; en[0] = sylLen; return; }
  double c = 0;
  for (int64_t s = 0; s < nSyl; ++s) {
    const double d = rnorm_bounded1(R, sylLen, sylLen * T, kSylLow, kSylHigh, false);
    const double p = rnorm_bounded1(R, pauseLen, pauseLen * T, kPauseLow, kPauseHigh, false);
    st[s] = 1 + c;
    en[s] = st[s] + d;
    c = en[s] + p;
  }
}

bool formants_moving(const sg_formants& F) {
  for (int f = 0; f < F.n_formants; ++f) if (F.n_points[f] > 1) return true;
  return false;
}

// addVectors(v1, v2, insertionPoint) layout, R/utilities_math.R:500-526:
// items are placed at offsets of the growing vector; a left pad shifts all.
struct Layout {
  int64_t len = 0;
  std::vector<SgNoiseItem> items;
  void add(SgNoiseItem it, double ip) {
    if (ip > 1) it.off = (int64_t)ip;  // v2 = c(rep(0, insertionPoint), v2)
    else if (ip < 1) {
      const int64_t pad = (int64_t)(1 - ip);
      for (auto& x : items) x.off += pad;
      len += pad;
      it.off = 0;
    } else it.off = 0;
    items.push_back(it);
    len = std::max(len, it.off + it.len);
  }
};

SgNoiseItem raw_item(int64_t fs_off, int64_t len, int64_t off) {
  SgNoiseItem it{};
  it.raw = fs_off;
  it.len = len;
  it.off = off;
  it.ola = -1;  // raw samples: no normalisation, envelope or fade
  it.strength.kind = 0;
  return it;
}

// ---- conditioning of the formant filter in fp32 ---------------------------
// The filter output's fp32 round-off is white source noise (the sine bank's and
// the forward STFT's, relative to the local source level) passed through the
// envelope, against the source's own harmonics passed through it. Per sampled
// glottal cycle, with its harmonic amplitudes a_h at bins k_h and the envelope
// column of the frame over it:
//   rho = rms_k env(k) / sqrt(sum_h a_h^2 env(k_h)^2 / sum_h a_h^2)
// Measured on C5's presets (tools/precision_study.py): the fp32 error of the
// normalised output is ~7e-9 rho; Misc$Cow reaches rho ~1e3-2e3 (1-3e-5 RMS on
// the GPU), every other preset stays below ~250. Bouts above SG_HP_RHO run
// the fp64 source and forward transform (DESIGN.md §5 "fp64 path").
double env_db_at(const Batch& B, const SgEnvJob& J, int64_t c, int64_t k) {
  const SgEnvTerm* tm = B.eterms.data() + J.term0 + c * J.ntr;
  const SgEnvCol& C = B.ecols[J.col0 + c];
  const double lk = log2_int(k);
  double acc = 0;
  for (int32_t t = 0; t < J.ntr; ++t) {
    const SgEnvTerm& e = tm[t];
    if (k < e.klo || k > e.khi) continue;
    const double d = e.A * lk - e.Rr * (double)k - e.Lm;
    if (d > -SG_ENV_CUT) acc += e.amp * std::exp2(d);
  }
  return (acc + C.lip * lk) * C.boost + J.slope * lk;
}

// env^2 of a bout's envelope on the bins 1, 1 + st, .. nr (st = nr / 256), per
// column asked for, computed once for both estimates below
struct EnvGrid {
  const Batch& B;
  const SgEnvJob& J;
  int64_t st;
  std::vector<std::pair<int64_t, vec>> cols;
  EnvGrid(const Batch& b, const SgEnvJob& j) : B(b), J(j), st(std::max<int64_t>(1, j.nr / 256)) {}
  const vec& col(int64_t c) {
    for (const auto& p : cols)
      if (p.first == c) return p.second;
    vec v;
    for (int64_t k = 1; k <= J.nr; k += st) v.push_back(std::exp2(env_db_at(B, J, c, k) / 5));
    cols.emplace_back(c, std::move(v));
    return cols.back().second;
  }
};

struct ProbeAt {
  int64_t pos;  // sample of the bout's pre-filter sound
  const HarmProbe* p;
};

double filter_conditioning(EnvGrid& G, const std::vector<ProbeAt>& probes, double hop, int wl, double sr) {
  const Batch& B = G.B;
  const SgEnvJob& J = G.J;
  double worst = 0;
  const int64_t nr = J.nr;
  for (const ProbeAt& pa : probes) {
    int64_t c = 0;
    if (J.nc > 1) {
      c = (int64_t)std::llround(((double)pa.pos - wl / 2.0) / hop);
      c = std::min<int64_t>(std::max<int64_t>(c, 0), J.nc - 1);
    }
    const vec& e2 = G.col(c);
    double n2 = 0;
    for (double v : e2) n2 += v;  // env^2
    const int64_t nk = (int64_t)e2.size();
    double s2 = 0, a2 = 0;
    const HarmProbe& hp = *pa.p;
    for (size_t h = 0; h < hp.amp.size(); ++h) {
      const double a = hp.amp[h];
      if (!(a > 0)) continue;
      const int64_t k = (int64_t)std::llround((double)(h + 1) * hp.f0 * wl / sr) + 1;
      if (k > nr) break;
      s2 += a * a * std::exp2(env_db_at(B, J, c, k) / 5);
      a2 += a * a;
    }
    if (a2 <= 0 || s2 <= 0 || nk == 0) continue;
    worst = std::max(worst, std::sqrt(n2 / (double)nk) / std::sqrt(s2 / a2));
  }
  return worst;
}

// The same rho for the pre-filter noise, whose fp32 round-off (its inverse
// STFT, ~eps x the noise level, white) meets the envelope against the noise's
// own spectrum: generateNoise's rolloffNoise filter (R/source.R:97-105), at the
// filter's bins (k x wl_noise / wl), over up to 4 envelope columns.
double noise_conditioning(EnvGrid& G, double rolloffNoise, int wl_noise, int wl) {
  const SgEnvJob& J = G.J;
  double worst = 0;
  const int64_t ncol = std::min<int64_t>(4, J.nc);
  for (int64_t q = 0; q < ncol; ++q) {
    const int64_t c = (2 * q + 1) * J.nc / (2 * ncol);
    const vec& e2 = G.col(c);
    double n2 = 0, s2 = 0, w2 = 0;
    int64_t i = 0;
    for (int64_t k = 1; k <= J.nr; k += G.st, ++i) {
      const double lk = wl_noise == wl ? log2_int(k) : std::log2((double)k * wl_noise / wl);
      const double p2 = std::exp2(rolloffNoise / 5 * lk);  // filter^2
      n2 += e2[(size_t)i];
      s2 += p2 * e2[(size_t)i];
      w2 += p2;
    }
    if (i == 0 || s2 <= 0 || w2 <= 0) continue;
    worst = std::max(worst, std::sqrt(n2 / (double)i) / std::sqrt(s2 / w2));
  }
  return worst;
}

bool smooth31(int64_t n) {
  for (int p : {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31})
    while (n > 1 && n % p == 0) n /= p;
  return n == 1;
}

// 0: never, 1: above the threshold (default), 2: every filtered bout (tests);
// defaults from SG_HP / SG_HP_RHO, changed by sg_set_fp64_policy
std::atomic<int> g_hp_mode{-1};
std::atomic<double> g_hp_rho{-1.0};
int hp_mode() {
  int m = g_hp_mode.load();
  if (m < 0) {
    m = 1;  // sg_set_fp64_policy changes it
    g_hp_mode.store(m);
  }
  return m;
}
// the pre-filter noise's fp64 threshold: measured with every noise in fp32
// (tools/noise_selector_study.py, profiles/r04x_noise_selector_study.json): the
// smallest noise estimate of a call over 1e-5 was 255 (1,280 C3 + C5 calls; every
// call at <= 200 within 6.2e-6), so 150 (round 3: 30, unmeasured)
double hp_rho_noise() {
  static const double r = [] {
    const char* e = std::getenv("SG_HP_RHO_NOISE");
    return e ? std::atof(e) : 150.0;
  }();
  return r;
}
double hp_rho() {
  double r = g_hp_rho.load();
  if (r < 0) {
    const char* e = std::getenv("SG_HP_RHO");
    r = e ? std::atof(e) : 100.0;  // measured: tools/selector_study.py (profiles/r04b_selector_study.json)
    g_hp_rho.store(r);
  }
  return r;
}

}  // namespace

int64_t plan_soundgen(Batch& B, const sg_soundgen_args& a_in, Rng& R, int64_t out_off, int first_syl) {
  (void)first_syl;
  sg_soundgen_args A = a_in;
  // range checks (R/soundgen.R:279-302)
  for (int i = 0; i < kNPV; ++i) {
    double* s = slot(A, i);
    if (std::isnan(*s) || *s < kPV[i][1] || *s > kPV[i][2]) {
      if (A.invalidArgAction == 1)
        throw SgError(SG_E_ARG, std::string(kPVNames[i]) + " must be between " + std::to_string(kPV[i][1]) +
                                    " and " + std::to_string(kPV[i][2]));
      if (A.invalidArgAction == 0) *s = kPV[i][0];
    }
  }
  const double sr = A.samplingRate;
  double wlp = std::floor(A.windowLength / 1000 * sr / 2) * 2;  // windowLength_points (R/soundgen.R:317)
  Anc pitchA = anc(A.pitchAnchors), pitchG = anc(A.pitchAnchorsGlobal), noiseA = anc(A.noiseAnchors);
  Anc amplA = anc(A.amplAnchors), amplG = anc(A.amplAnchorsGlobal), mouthA = anc(A.mouthAnchors);
  // hyper-parameters (R/soundgen.R:337-379)
  if (A.creakyBreathy < 0) {
    A.nonlinBalance = std::min(100.0, A.nonlinBalance - A.creakyBreathy * 50);
    A.jitterDep = std::max(0.0, A.jitterDep - A.creakyBreathy / 2);
    A.shimmerDep = std::max(0.0, A.shimmerDep - A.creakyBreathy * 5);
    A.subDep = A.subDep * std::pow(2.0, -A.creakyBreathy);
  } else if (A.creakyBreathy > 0) {
    noiseA.t = {0, A.sylLen + 100};
    noiseA.v.assign(2, std::min(40.0, -120 + A.creakyBreathy * 160));
  }
  A.rolloff = A.rolloff - A.creakyBreathy * 10;
  A.rolloffOct = A.rolloffOct - A.creakyBreathy * 5;
  A.subFreq = 2 * (A.subFreq - 50) / (1 + std::exp(-.1 * (50 - A.nonlinDep))) + 50;
  A.jitterDep = 2 * A.jitterDep / (1 + std::exp(.1 * (50 - A.nonlinDep)));
  // formants scaled along maleFemale (owned copy of the frequencies)
  const sg_formants& F0 = A.formants;
  int64_t totF = 0;
  for (int f = 0; f < F0.n_formants; ++f) totF += F0.n_points[f];
  vec ffreq(F0.freq ? F0.freq : nullptr, F0.freq ? F0.freq + totF : nullptr);
  if (A.maleFemale != 0) {
    for (auto& v : pitchA.v) v *= std::pow(2.0, A.maleFemale);
    for (auto& v : ffreq) v *= std::pow(1.25, A.maleFemale);
    A.vocalTract = A.vocalTract * (1 - .25 * A.maleFemale);
  }
  sg_formants Fm = A.formants;
  Fm.freq = ffreq.empty() ? nullptr : ffreq.data();
  // stochastic rounding of nSyl / repeatBout: rbinom(1, 1, p)
  const double nSyl = std::floor(A.nSyl) + rbinom1(R, A.nSyl - std::floor(A.nSyl));
  const double repeatBout = std::floor(A.repeatBout) + rbinom1(R, A.repeatBout - std::floor(A.repeatBout));
  const int64_t nS = (int64_t)nSyl, nB = (int64_t)repeatBout;
  vec pitchDeltas((size_t)std::max<int64_t>(nS, 1), 1.0);
  {
    bool anyNZ = false;
    for (double v : pitchG.v) if (v != 0) anyNZ = true;
    if (pitchG.n() > 0 && anyNZ && nS > 1) {
      vec pd;
      smooth_contour(pitchG.view(), nS, false, 1, false, 0, false, 0, pd);
      for (int64_t s = 0; s < nS; ++s) pitchDeltas[s] = std::pow(2.0, pd[s] / 12);
    }
  }
  if (pitchA.n() > 0) {
    const double mn = r_min(pitchA.t);
    if (mn < 0) for (auto& v : pitchA.t) v -= mn;
    const double mx = r_max(pitchA.t);
    if (mx > 1) for (auto& v : pitchA.t) v /= mx;
  }
  const double T = A.temperature;
  bool noiseAbove = false, amplBelow = false;
  for (double v : noiseA.v) if (v > A.throwaway) noiseAbove = true;
  for (double v : amplA.v) if (v < -A.throwaway) amplBelow = true;
  const bool wiggleNoise = T > 0 && noiseA.n() > 0 && noiseAbove;
  const bool wiggleAmpl = T > 0 && amplA.n() > 0 && amplBelow;
  sg_harm_params HP;
  sg_default_harm_params(&HP);
  HP.attackLen = A.attackLen; HP.jitterDep = A.jitterDep; HP.jitterLen = A.jitterLen;
  HP.vibratoFreq = A.vibratoFreq; HP.vibratoDep = A.vibratoDep; HP.shimmerDep = A.shimmerDep;
  HP.creakyBreathy = A.creakyBreathy; HP.rolloff = A.rolloff; HP.rolloffOct = A.rolloffOct;
  HP.rolloffKHz = A.rolloffKHz; HP.rolloffParab = A.rolloffParab; HP.rolloffParabHarm = A.rolloffParabHarm;
  HP.temperature = T; HP.pitchDriftDep = A.tempEffects[3]; HP.pitchDriftFreq = A.tempEffects[4];
  HP.shortestEpoch = A.shortestEpoch; HP.subFreq = A.subFreq; HP.subDep = A.subDep; HP.rolloffLip = A.rolloffLip;
  HP.amDep = A.amDep; HP.amFreq = A.amFreq; HP.nonlinBalance = A.nonlinBalance; HP.nonlinDep = A.nonlinDep;
  HP.pitchFloor = A.pitchFloor; HP.pitchCeiling = A.pitchCeiling; HP.pitchSamplingRate = A.pitchSamplingRate;
  HP.throwaway = A.throwaway; HP.samplingRate = sr; HP.overlap = A.overlap;
  static const double PV_VARY[9][2] = {{0, 100}, {0, 200}, {0, 24}, {0, 100}, {-60, 0},
                                       {-30, 10}, {50, 500}, {10, 1000}, {0, 500}};
  const bool postNoise = A.formantsNoise.n_formants > 0;  // separately filtered noise
  std::vector<size_t> final_mixes;  // phase-1 mixes of this call, in output order
  std::vector<int64_t> final_lens;
  int64_t total = 0;

  for (int64_t b = 0; b < nB; ++b) {
    // syllable segmentation (R/soundgen.R:482-531)
    double sylDur;
    if (A.sylLen >= kSylLow && A.sylLen <= kSylHigh)
      sylDur = rnorm_bounded1(R, A.sylLen, (kSylHigh - kSylLow) * T * A.tempEffects[0], kSylLow, kSylHigh, false);
    else sylDur = A.sylLen;
    const double pauseDur =
        rnorm_bounded1(R, A.pauseLen, (kPauseHigh - kPauseLow) * T * A.tempEffects[0], kPauseLow, kPauseHigh, false);
    vec sst, sen;
    divide_into_syllables(R, nS, sylDur, pauseDur, T * A.tempEffects[0], sst, sen);
    vec ssi((size_t)nS);
    for (int64_t s = 0; s < nS; ++s) ssi[s] = r_round(sst[s] * sr / 1000);
    ssi[0] = 1;
    if (noiseA.n() > 0 && noiseA.t[0] != 0) {
      const double shift = -r_round(noiseA.t[0] * sr / 1000);
      if (noiseA.t[0] < 0) ssi[0] = ssi[0] - shift;
      else for (auto& v : ssi) v -= shift;
    }
    // syllables: voiced items (syllable buffers + zero pauses) and noise items
    Layout voiced;
    std::vector<SgNoiseItem> noises;
    std::vector<double> noiseIp;
    std::vector<HarmProbe> probes;   // spectra of sampled glottal cycles (filter conditioning)
    std::vector<int64_t> probe_pos;  // their bout samples
    std::vector<int> bout_syls;      // syllables planned to fs in this bout
    sg_harm_params HPs = HP;
    for (int64_t s = 0; s < nS; ++s) {
      Anc pA = pitchA, aA = amplA;
      if (T > 0) {
        double* slots[9] = {&HPs.nonlinDep, &HPs.attackLen, &HPs.jitterDep, &HPs.shimmerDep, &HPs.rolloff,
                            &HPs.rolloffOct, &HPs.shortestEpoch, &HPs.subFreq, &HPs.subDep};
        const double base[9] = {HP.nonlinDep, HP.attackLen, HP.jitterDep, HP.shimmerDep, HP.rolloff,
                                HP.rolloffOct, HP.shortestEpoch, HP.subFreq, HP.subDep};
        const bool rnd[9] = {false, true, false, false, false, false, false, true, true};
        for (int p = 0; p < 9; ++p) {
          const double l = PV_VARY[p][0], h = PV_VARY[p][1];
          *slots[p] = rnorm_bounded1(R, base[p], (h - l) * T / 10, l, h, rnd[p]);
        }
        if (pA.n() > 0) {
          const double lo[2] = {0, 25}, hi[2] = {1, 3500};
          wiggle_anchors(R, pA, T, A.tempEffects[5], lo, hi, false);
        }
        if (wiggleNoise) {  // drawn, then discarded: the reference overwrites noiseAnchors_syl[[s]]
          Anc tmp = noiseA;
          const double lo[2] = {-INFINITY, -120}, hi[2] = {INFINITY, 40};
          wiggle_anchors(R, tmp, T, A.tempEffects[6], lo, hi, true);
        }
        if (wiggleAmpl) {
          const double lo[2] = {0, 0}, hi[2] = {1, -A.throwaway};
          wiggle_anchors(R, aA, T, A.tempEffects[7], lo, hi, false);
        }
      }
      const double dur = sen[s] - sst[s];
      vec pc;
      if (pA.n() > 0) {
        smooth_contour(pA.view(), (int64_t)r_round(dur * A.pitchSamplingRate / 1000), true, 0, true, A.pitchFloor,
                       true, A.pitchCeiling, pc, A.pitchSamplingRate);
        for (auto& v : pc) v *= pitchDeltas[s];
      }
      double minNoise = INFINITY;
      for (double v : noiseA.v) minNoise = std::min(minNoise, v);
      int64_t sylLen;
      if (dur < kSylLow || (noiseA.n() > 0 && minNoise >= 40) || pA.n() == 0) {
        sylLen = (int64_t)r_round(dur * sr / 1000);  // zeros: no item
      } else {
        int64_t fs_off = 0;
        const size_t np0 = probes.size();
        // the slot keeps the residue of the syllable's offset in the bout (a placed bout, below)
        sylLen = plan_harmonics(B, pc.data(), (int64_t)pc.size(), HPs, aA.view(), R, voiced.len & 3, B.draws_only, true,
                                &fs_off, &probes);
        for (size_t q = np0; q < probes.size(); ++q) probe_pos.push_back(voiced.len + probes[q].t);
        if (!B.draws_only) bout_syls.push_back((int)B.syls.size() - 1);
        SgNoiseItem it = raw_item(fs_off, sylLen, voiced.len);
        voiced.items.push_back(it);
      }
      voiced.len += sylLen;
      if (s < nS - 1) voiced.len += (int64_t)std::floor((sst[s + 1] - sen[s]) * sr / 1000);  // pause zeros
      // unvoiced part (R/soundgen.R:643-698)
      if (noiseA.n() > 0 && noiseAbove) {
        Anc ns = noiseA;
        for (auto& t : ns.t) if (t > 0) t = t * dur / A.sylLen;
        const int64_t uvDur = (int64_t)r_round((r_max(ns.t) - r_min(ns.t)) * sr / 1000);
        int64_t envN = 0, nInt = 0;
        if (postNoise) {
          // R/soundgen.R:662-663: max(lengths(formantsNoise)) > 1 | mouth moves;
          // a list of formant lists always has 4 fields, so it counts as moving
          bool moving = A.formantsNoise_rlen == 0 || A.formantsNoise_rlen > 1;
          bool mouthMoves = false;
          for (double v : mouthA.v) if (v != .5) mouthMoves = true;
          if (mouthMoves) moving = true;
          nInt = moving ? (int64_t)r_round((r_max(ns.t) - r_min(ns.t)) / 10) : 1;
          // the noise filter's rolloffNoise slope (R/source.R:103-105) is applied by the same job
          envN = plan_envelope(B, R, wlp / 2, nInt, &A.formantsNoise, A.formantDep, A.rolloffLip, mouthA.view(), 0,
                               0, A.vocalTract, T, A.tempEffects[1], A.tempEffects[2], A.formantDepStoch, 1, sr,
                               35400, A.rolloffNoise);
        }
        SgNoiseItem it{};
        if (!plan_noise(B, R, uvDur, ns.view(), A.rolloffNoise, HPs.attackLen, (int)wlp, sr, A.overlap, nullptr,
                        nInt, &it, nInt > 0 ? envN : 0)) {  // an empty filter is NA in R (filterNoise[1])
          it = raw_item(0, uvDur, 0);  // NA contour: generateNoise returns rep(0, len)
          it.flags = SG_ITEM_ZERO;
        }
        noises.push_back(it);
        noiseIp.push_back(ssi[s]);
      }
    }
    // sound = addVectors(voiced, unvoiced[[s]], ssi[s]) for breathing noise (R/soundgen.R:699-714)
    auto emit = [&](const Layout& L, int32_t& item0) {
      item0 = (int32_t)B.items.size();
      int32_t n = 0;
      for (const auto& it : L.items)
        if (!(it.flags & SG_ITEM_ZERO) && it.len > 0) { B.items.push_back(it); ++n; }
      return n;
    };
    Layout sound = voiced;
    if (!postNoise)
      for (size_t s = 0; s < noises.size(); ++s) sound.add(noises[s], noiseIp[s]);
    const int64_t Ls = sound.len;
    int32_t ncontent = 0;
    for (const auto& it : sound.items)
      if (!(it.flags & SG_ITEM_ZERO) && it.len > 0) ++ncontent;
    // the formant filter's envelope (R/soundgen.R:762-775; no draw between here
    // and there in R) and, from it, the bout's precision path
    int wl = 0;
    int64_t filt_env = 0, nInt = 1;
    bool hp = false;
    std::optional<EnvGrid> grid;  // env^2 samples of the bout's filter envelope (conditioning estimates)
    if (ncontent > 0) {
      const double fl2 = std::floor((double)Ls / 2);
      if (fl2 < wlp) wlp = fl2;  // persists into later bouts and their noise
      wl = (int)wlp;
      const vec step = r_seq_by(1, (double)std::max<int64_t>(1, Ls - wl), (double)wl - A.overlap * wl / 100);
      const int64_t nc = (int64_t)step.size();
      bool moving = formants_moving(Fm);
      bool mouthMoves = false;
      for (double v : mouthA.v) if (v != .5) mouthMoves = true;
      if (mouthA.n() > 0 && mouthMoves) moving = true;
      nInt = moving ? nc : 1;
      filt_env = plan_envelope(B, R, (double)wl / 2, nInt, &Fm, A.formantDep, A.rolloffLip, mouthA.view(), 0, 0,
                               A.vocalTract, T, A.tempEffects[1], A.tempEffects[2], A.formantDepStoch, 1, sr, 35400);
      // draws_only: the bout's last draw is behind; what may still fail before the next
      // bout's draws (the filter's FFT geometry; the global envelope's contour, below)
      // runs, the rest does not
      if (B.draws_only) geometry(B, wl);
      else grid.emplace(B, B.envjobs.back());
      const int mode = B.draws_only ? 0 : hp_mode();
      // the fp64 frame kernel takes even windows with a 31-smooth half M <= 2048
      if (mode > 0 && !bout_syls.empty() && wl % 2 == 0 && wl <= 4096 && smooth31(wl / 2)) {  // M <= 2048
        if (mode == 2) {
          hp = true;
        } else {
          std::vector<ProbeAt> pa;
          for (size_t q = 0; q < probes.size(); ++q) pa.push_back(ProbeAt{probe_pos[q], &probes[q]});
          const double rho = filter_conditioning(*grid, pa, (double)wl - A.overlap * wl / 100, wl, sr);
          B.rho_cur = std::max(B.rho_cur, rho);
          hp = rho > hp_rho();
        }
      }
    }
    // the pre-filter noise of an ill-conditioned bout: fp64 inverse transforms
    if (!postNoise && grid && hp_mode() > 0) {
      std::vector<int> nolas;
      for (const SgNoiseItem& it : noises)
        if (it.ola >= 0 && !(it.flags & SG_ITEM_ZERO)) nolas.push_back(it.ola);
      if (!nolas.empty()) {
        const double rn = noise_conditioning(*grid, A.rolloffNoise, B.olas[0][nolas[0]].wl, wl);
        B.rho_noise_cur = std::max(B.rho_noise_cur, rn);
        if ((hp_mode() == 2 || rn > hp_rho_noise()) && noise_to_fp64(B, nolas)) ++B.hp_noise_bouts;
      }
    }
    if (hp) {  // voiced syllables to the fp64 path; their items read fh
      ++B.hp_bouts;
      for (int si : bout_syls) {
        const int64_t old_off = B.syls[si].out_off;
        const int64_t fh_off = syllable_to_fp64(B, si);
        for (auto& it : sound.items)
          if (it.ola < 0 && !(it.flags & SG_ITEM_F64) && it.raw == old_off) {
            it.raw = fh_off;
            it.flags |= SG_ITEM_F64;
            break;
          }
      }
    }
    SgContour mult{};  // amplAnchorsGlobal (R/soundgen.R:715-733)
    mult.kind = 0;
    {
      bool below = false;
      for (double v : amplG.v) if (v < -A.throwaway) below = true;
      if (amplG.n() > 0 && below) {
        Anc g2 = amplG;
        for (auto& v : g2.v) v = std::pow(2.0, v / 10);
        mult = contour_desc(B, g2.view(), Ls, true, 0, true, -A.throwaway, false, sr);
      }
    }
    if (B.draws_only) continue;
    // The pre-filter mix writes the bout's sound: its voiced syllables, the breathing
    // noise and the global envelope (addVectors and `sound * amplEnvelope`). A bout
    // whose sound is its voiced syllables alone (noise filtered separately, or none;
    // fp32 path) is placed instead of mixed: each syllable's finalize writes its samples
    // straight into the sound buffer at the syllable's offset, times the global envelope
    // at that offset if there is one (the mix's own product), and mixes write only the
    // zeros between the syllables (zero under any envelope). Each syllable's slot
    // was allocated with the residue (mod 4 floats) of its offset, and the sound buffer
    // starts 16-B aligned, so a syllable keeps its residue when it moves (its W scratch
    // was aligned against it for sg_harm_copy's float4 runs, sg_plan_harm.cpp); one that
    // does not (none, by construction) is copied by a one-item mix.
    const bool place = !hp && (postNoise || noises.empty()) && !sound.items.empty() &&
                       sound.items.size() == bout_syls.size();
    int64_t sound_fs;
    if (place) {
      sound_fs = fs_alloc(B, std::max<int64_t>(Ls, 1));
      auto zero_mix = [&](int64_t a, int64_t n) {
        if (n <= 0) return;
        SgMix z{};
        z.dst = sound_fs + a;
        z.len = n;
        z.to_fs = 1;
        z.base_kind = SG_BASE_NONE;
        z.item0 = (int32_t)B.items.size();
        z.mult.kind = 0;
        B.mixes[0].push_back(z);
      };
      int64_t at = 0;
      ncontent = 0;
      for (size_t i = 0; i < sound.items.size(); ++i) {
        const SgNoiseItem& it = sound.items[i];
        zero_mix(at, it.off - at);
        at = std::max(at, it.off + it.len);
        if (it.len <= 0) continue;
        ++ncontent;
        SgSyllable& sy = B.syls[(size_t)bout_syls[i]];
        if ((sound_fs + it.off) % 4 == sy.out_off % 4) {
          sy.out_off = sound_fs + it.off;
          sy.genv = mult;  // the global envelope, applied by the finalize (kind 0: none)
          sy.genv_off = it.off;
          sy.genv_len = Ls;
          continue;
        }
        SgMix c{};
        c.dst = sound_fs + it.off;
        c.len = it.len;
        c.to_fs = 1;
        c.base_kind = SG_BASE_NONE;
        c.item0 = (int32_t)B.items.size();
        c.nitems = 1;
        c.mult = mult;
        SgNoiseItem ci = it;
        ci.off = 0;
        B.items.push_back(ci);
        B.mixes[0].push_back(c);
      }
      zero_mix(at, Ls - at);
    } else {
      sound_fs = hp ? fh_alloc(B, std::max<int64_t>(Ls, 1)) : fs_alloc(B, std::max<int64_t>(Ls, 1));
      SgMix pre{};
      pre.dst = sound_fs;
      pre.len = Ls;
      pre.to_fs = hp ? 2 : 1;
      pre.base_kind = SG_BASE_NONE;
      ncontent = emit(sound, pre.item0);
      pre.nitems = ncontent;
      pre.mult = mult;
      B.mixes[0].push_back(pre);
    }
    // formant filter (R/soundgen.R:736-807); skipped when sum(sound) == 0,
    // which here means: nothing synthesized (no syllable, no noise content)
    Layout post;
    if (ncontent == 0) {
      post.items.push_back(raw_item(sound_fs, Ls, 0));
      post.len = Ls;
    } else {
      int64_t filt_fs = 0, Lf = 0;
      const int ola = plan_filter(B, sound_fs, Ls, wl, A.overlap, filt_env, nInt, &Lf, &filt_fs, hp);
      SgNoiseItem fi = raw_item(filt_fs, Lf, 0);  // soundFiltered / max(soundFiltered)
      fi.ola = ola;
      fi.flags = SG_ITEM_FILTER_OLA;
      post.items.push_back(fi);
      post.len = Lf;
    }
    // separately filtered noise is added after the filter (R/soundgen.R:811-817)
    if (postNoise)
      for (size_t s = 0; s < noises.size(); ++s) post.add(noises[s], noiseIp[s]);
    SgMix fin{};
    fin.to_fs = 0;
    fin.base_kind = SG_BASE_NONE;
    fin.len = post.len;
    fin.nitems = emit(post, fin.item0);
    fin.mult.kind = 0;
    if (A.amDep > 0) {  // AM trill (R/soundgen.R:820-833)
      const vec half = sigmoid_half(sr, A.amFreq, A.amShape, 1);
      fin.am_tab = fl_push(B, half.data(), (int64_t)half.size());
      fin.am_lo = (int32_t)half.size();
      fin.am_dep = (float)A.amDep;
    }
    if (b > 0) {  // bout pause: rep(0, pauseLen * sr / 1000)
      const int64_t np = (int64_t)(A.pauseLen * sr / 1000);
      SgMix z{};
      z.len = np;
      z.base_kind = SG_BASE_NONE;
      final_mixes.push_back(B.mixes[1].size());
      final_lens.push_back(np);
      B.mixes[1].push_back(z);
      total += np;
    }
    final_mixes.push_back(B.mixes[1].size());
    final_lens.push_back(fin.len);
    B.mixes[1].push_back(fin);
    total += fin.len;
  }
  // addSilence: round(sr / 1000 * addSilence) zeros on both ends (R/soundgen.R:846-849)
  int64_t nsil = 0;
  if (!std::isnan(A.addSilence)) nsil = (int64_t)r_round(sr / 1000 * A.addSilence);
  int64_t pos = out_off;
  auto zeros = [&](int64_t n) {
    if (n <= 0) return;
    SgMix z{};
    z.dst = pos;
    z.len = n;
    z.base_kind = SG_BASE_NONE;
    B.mixes[1].push_back(z);
    pos += n;
  };
  zeros(nsil);
  for (size_t i = 0; i < final_mixes.size(); ++i) {
    B.mixes[1][final_mixes[i]].dst = pos;
    pos += final_lens[i];
  }
  zeros(nsil);
  return total + 2 * nsil;
}

void restore_soundgen_tail(Batch&, int) {}

}  // namespace sg

extern "C" int sg_set_fp64_policy(int32_t mode, double rho) {
  if (mode < 0 || mode > 2 || !(rho >= 0)) return SG_E_ARG;
  sg::g_hp_mode.store(mode);
  sg::g_hp_rho.store(rho);
  return SG_OK;
}

extern "C" int sg_permitted_value(int32_t i, const char** name, double* def_low_high) {
  if (i < 0 || i >= sg::kNPV) return SG_E_ARG;
  *name = sg::kPVNames[i];
  for (int j = 0; j < 3; ++j) def_low_high[j] = sg::kPV[i][j];
  return SG_OK;
}

extern "C" double sg_noise_threshold(int32_t which, double nonlinBalance) {
  return sg::noise_threshold(which, nonlinBalance);
}

extern "C" void sg_default_soundgen_args(sg_soundgen_args* a) {
  // formals of soundgen(), R/soundgen.R:208-277 (anchors and formants NA:
  // the caller supplies them, as the R wrapper does)
  std::memset(a, 0, sizeof *a);
  a->repeatBout = 1; a->nSyl = 1; a->sylLen = 300; a->pauseLen = 200; a->temperature = 0.025;
  const double te[8] = {.02, .3, .2, .5, .125, .05, .1, .1};
  std::memcpy(a->tempEffects, te, sizeof te);
  a->maleFemale = 0; a->creakyBreathy = 0; a->nonlinBalance = 0; a->nonlinDep = 50; a->jitterLen = 1;
  a->jitterDep = 3; a->vibratoFreq = 5; a->vibratoDep = 0; a->shimmerDep = 0; a->attackLen = 50;
  a->rolloff = -12; a->rolloffOct = -12; a->rolloffKHz = -6; a->rolloffParab = 0; a->rolloffParabHarm = 3;
  a->rolloffLip = 6; a->formantDep = 1; a->formantDepStoch = 30; a->vocalTract = 15.5; a->subFreq = 100;
  a->subDep = 100; a->shortestEpoch = 300; a->amDep = 0; a->amFreq = 30; a->amShape = 0; a->rolloffNoise = -14;
  a->samplingRate = 16000; a->windowLength = 50; a->overlap = 75; a->addSilence = 100; a->pitchFloor = 50;
  a->pitchCeiling = 3500; a->pitchSamplingRate = 3500; a->throwaway = -120; a->invalidArgAction = 0;
  a->formants.f1_index = -1;
  a->formantsNoise.f1_index = -1;
}
