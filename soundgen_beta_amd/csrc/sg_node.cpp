// sg_node.cpp — one process driving several devices (SURVEY.md §8e, §5 "comm
// backend": the one-process whole-node context). A batch of independent calls
// is split by calls with no data-path collective (every normalisation is per
// call, R/source.R:449, R/soundgen.R:807): each device plans, uploads and
// synthesizes its shard on its own stream, and copies its samples over its own
// PCIe link into the caller's host buffer at the call's offset of the
// whole-batch layout, so nothing is gathered through one device and the node's
// links run at once. The callers this serves are the batch loops the R API
// keeps: soundgen_batch(), morph() (R/morph.R:200-208) and matchPars()
// (R/matchPars.R:168-202).
//
// Assignment: LPT (largest first, onto the least-loaded device) over an
// analytic cost per call from its arguments alone -- the model of
// soundgen_beta_amd/dist.py (call_cost), restated here so that R reaches it:
// sine-bank (sample x kept rows x (1 + sidebands)), STFT frames x 5 wl log2 wl,
// per-sample assembly, with the weights measured on C5.
//
// Draws: injected arrays are per call, so shards plan independently (and in
// parallel on host threads). Callbacks (R's RNG through the shim) are ONE
// sequential stream in call order: the node first runs every call in order in
// the planner's draws-only mode (Batch::draws_only: the draws R would make, in
// R's order, and the errors that precede a call's last draw, but none of the
// per-sample work after it; a failing call stops the stream as lapply would),
// recording each call's draws, then plans the shards from the recorded draws,
// each call replaying its own -- the second pass runs on host threads and yields
// exactly the plans the stream would have. Runs of uniforms (generateNoise's
// runif(nr * nc)) come through the bulk callback when the caller has one.
//
// Execution: each shard is planned in chunks of consecutive calls; chunk c's
// samples cross the device's link while later chunks compute and host threads
// scatter chunk c - 1 to its whole-batch offsets (widened to double for R).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <numeric>
#include <queue>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "sg_plan.h"
#include "soundgen_hip.h"

struct sg_node {
  std::vector<int32_t> devices;
  // per device of the node, created on first execution (planning needs no device)
  struct Dev {
    sg_ctx* ctx = nullptr;
    hipStream_t run = nullptr, copy = nullptr;  // kernels; D2H copies
    float* d_out = nullptr;                     // the shard's packed samples, kept across executes
    size_t d_bytes = 0;
    void* pin[2] = {nullptr, nullptr};          // pinned staging ring, one chunk each
    size_t pin_bytes = 0;
    std::vector<hipEvent_t> ev;                 // per chunk: executed, copied
  };
  std::vector<Dev> dev;
  std::string err;
  std::mutex mu;
};

namespace {

// ---- per-call draw logs (callback batches) ----------------------------------
struct DrawLog {
  const sg_random* src = nullptr;  // the caller's draw source (arrays first, then callbacks)
  int64_t ni = 0, ui = 0;          // cursors into src's arrays
  std::vector<double> normals, uniforms, gammas;
  // runs of uniforms drawn through the bulk callback: their only consumer (the
  // planner's Rng::unif_f32, generateNoise's runif(nr * nc)) keeps them as floats, so
  // they are recorded as floats (half the bytes of the largest log)
  std::vector<float> runs;
  size_t gn = 0, gu = 0, gr = 0, gi = 0;  // replay cursors
};
double rec_norm(void* u) {
  auto* L = static_cast<DrawLog*>(u);
  const sg_random& s = *L->src;
  double v;
  if (s.normals && L->ni < s.n_normals) v = s.normals[L->ni++];
  else if (s.norm_cb) v = s.norm_cb(s.user);
  else throw sg::SgError(SG_E_RANDOM, "normal draws exhausted");
  L->normals.push_back(v);
  return v;
}
double rec_unif(void* u) {
  auto* L = static_cast<DrawLog*>(u);
  const sg_random& s = *L->src;
  double v;
  if (s.uniforms && L->ui < s.n_uniforms) v = s.uniforms[L->ui++];
  else if (s.unif_cb) v = s.unif_cb(s.user);
  else throw sg::SgError(SG_E_RANDOM, "uniform draws exhausted");
  L->uniforms.push_back(v);
  return v;
}
void rec_unif_n(void* u, double* out, int64_t n) {
  auto* L = static_cast<DrawLog*>(u);
  const sg_random& s = *L->src;
  int64_t k = 0;
  for (; k < n && s.uniforms && L->ui < s.n_uniforms; ++k) out[k] = s.uniforms[L->ui++];
  if (k < n) {
    if (s.unif_n_cb) s.unif_n_cb(s.user, out + k, n - k);
    else if (s.unif_cb)
      for (; k < n; ++k) out[k] = s.unif_cb(s.user);
    else throw sg::SgError(SG_E_RANDOM, "uniform draws exhausted");
  }
  const size_t at = L->runs.size();
  L->runs.resize(at + (size_t)n);
  for (int64_t q = 0; q < n; ++q) L->runs[at + (size_t)q] = (float)out[q];
}
double rec_gamma(void* u, double shape, double rate) {
  auto* L = static_cast<DrawLog*>(u);
  const sg_random& s = *L->src;
  const double v = s.gamma_cb(s.user, shape, rate);
  L->gammas.push_back(v);
  return v;
}
double replay_gamma(void* u, double, double) {
  auto* L = static_cast<DrawLog*>(u);
  if (L->gi >= L->gammas.size()) throw sg::SgError(SG_E_RANDOM, "replayed gamma draws exhausted");
  return L->gammas[L->gi++];
}
double replay_norm(void* u) {
  auto* L = static_cast<DrawLog*>(u);
  if (L->gn >= L->normals.size()) throw sg::SgError(SG_E_RANDOM, "replayed normal draws exhausted");
  return L->normals[L->gn++];
}
double replay_unif(void* u) {
  auto* L = static_cast<DrawLog*>(u);
  if (L->gu >= L->uniforms.size()) throw sg::SgError(SG_E_RANDOM, "replayed uniform draws exhausted");
  return L->uniforms[L->gu++];
}
void replay_unif_n(void* u, double* out, int64_t n) {
  auto* L = static_cast<DrawLog*>(u);
  if (L->gr + (size_t)n > L->runs.size()) throw sg::SgError(SG_E_RANDOM, "replayed uniform runs exhausted");
  for (int64_t q = 0; q < n; ++q) out[q] = (double)L->runs[L->gr + (size_t)q];
  L->gr += (size_t)n;
}
bool has_callbacks(const sg_random& r) { return r.norm_cb || r.unif_cb || r.gamma_cb; }

// ---- cost model (soundgen_beta_amd/dist.py call_cost) -------------------------
constexpr double W_ROW = 0.0035, W_FLOP = 0.00004, W_SAMPLE = 0.05;  // ns of one MI355X per unit

// rows getRolloff keeps at f0: harmonics below Nyquist whose dB level stays above
// throwaway (R/sourceSpectrum.R:86-101)
double harmonic_rows(double f0, double sr, double rolloff, double rolloffOct, double rolloffKHz, double throwaway) {
  f0 = std::max(f0, 1.0);
  const int64_t nH = (int64_t)std::ceil((sr / 2 - f0) / f0);
  const double slope = rolloff + rolloffKHz * (f0 - 200) / 1000;
  int64_t n = 1;
  for (int64_t h = 2; h <= std::max<int64_t>(nH, 1); ++h) {
    const double db = slope * std::log2((double)h) + rolloffOct * (f0 * (double)h - 200) / 1000;
    if (db < throwaway) break;
    n = h;
  }
  return (double)n;
}

// samples a call will produce, from its arguments (chunk sizing only)
double call_samples(const sg_call_desc& d) {
  if (d.kind == SG_CALL_HARMONICS)
    return d.harm ? (double)d.pitch_len / d.harm->pitchSamplingRate * d.harm->samplingRate : 0.0;
  if (!d.args) return 0;
  const sg_soundgen_args& a = *d.args;
  const double nSyl = std::max(1.0, std::floor(a.nSyl)), rep = std::max(1.0, std::floor(a.repeatBout));
  const double sil = std::isnan(a.addSilence) ? 0.0 : 2 * a.addSilence;
  return (a.sylLen * nSyl * rep + a.pauseLen * (nSyl * rep) + sil) / 1000.0 * a.samplingRate;
}

double call_cost(const sg_call_desc& d) {
  if (d.kind == SG_CALL_HARMONICS) {
    if (!d.harm || !d.pitch) return 0;
    const sg_harm_params& p = *d.harm;
    const double n = (double)d.pitch_len / p.pitchSamplingRate * p.samplingRate;
    std::vector<double> v;
    for (int64_t i = 0; i < d.pitch_len; ++i)
      if (std::isfinite(d.pitch[i])) v.push_back(d.pitch[i]);
    double rows = 0;
    if (!v.empty()) {
      std::sort(v.begin(), v.end());
      const size_t m = v.size();
      const double med = m % 2 ? v[m / 2] : 0.5 * (v[m / 2 - 1] + v[m / 2]);
      rows = harmonic_rows(med, p.samplingRate, p.rolloff, p.rolloffOct, p.rolloffKHz, p.throwaway);
    }
    return n * (rows * W_ROW + W_SAMPLE);
  }
  if (!d.args) return 0;
  const sg_soundgen_args& a = *d.args;
  const double sr = a.samplingRate;
  const double nSyl = std::max(1.0, std::floor(a.nSyl)), rep = std::max(1.0, std::floor(a.repeatBout));
  const double dur = a.sylLen * nSyl * rep + a.pauseLen * (nSyl - 1) * rep;
  const double n = dur / 1000.0 * sr;
  double rows = 0;
  double lsum = 0;
  int64_t nv = 0;
  for (int32_t i = 0; i < a.pitchAnchors.n; ++i) {
    const double v = a.pitchAnchors.value[i];
    if (std::isfinite(v)) {
      lsum += std::log(std::max(v, 1.0));
      ++nv;
    }
  }
  if (nv) {
    const double f0 = std::exp(lsum / (double)nv);
    rows = harmonic_rows(f0, sr, a.rolloff, a.rolloffOct, a.rolloffKHz, a.throwaway);
    if (a.subDep > 0 && a.nonlinBalance > 0) {
      const double nsub = std::max(0.0, std::nearbyint(f0 / std::max(a.subFreq, 1.0)) - 1);
      const double share = std::min(1.0, a.nonlinBalance / 100);
      rows *= 1 + nsub * share;
    }
  }
  const double wl = std::max(4.0, 2 * std::floor(a.windowLength * sr / 1000 / 2));
  const double hop = wl * (1 - a.overlap / 100);
  const double frames = n / std::max(hop, 1.0);
  // a noise phase exists when some noise anchor is above throwaway (R's default
  // noiseAnchors are -120 dB: no breathing)
  bool has_noise = false;
  for (int32_t i = 0; i < a.noiseAnchors.n; ++i) has_noise |= a.noiseAnchors.value[i] > a.throwaway;
  const double noise = 1.0 + (has_noise ? 1.0 : 0.0);
  const double fft = 2 * 5 * wl * std::log2(wl) * frames * noise;
  return n * (rows * W_ROW + W_SAMPLE) + fft * W_FLOP;
}

// device index of each call: largest cost first onto the least-loaded device
// (ties: lowest device, then call order) -- dist.py lpt_assign
std::vector<int32_t> lpt(const std::vector<double>& cost, int32_t k) {
  std::vector<int64_t> order(cost.size());
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return cost[x] > cost[y]; });
  using E = std::pair<double, int32_t>;
  std::priority_queue<E, std::vector<E>, std::greater<E>> heap;
  for (int32_t r = 0; r < k; ++r) heap.push({0.0, r});
  std::vector<int32_t> owner(cost.size(), 0);
  for (int64_t i : order) {
    const E e = heap.top();
    heap.pop();
    owner[i] = e.second;
    heap.push({e.first + cost[i], e.second});
  }
  return owner;
}

int node_err(sg_node* node, int code, const std::string& m) {
  if (node) {
    std::lock_guard<std::mutex> lk(node->mu);
    node->err = m;
  }
  return code;
}

template <class F>
int node_guarded(sg_node* node, F&& f) {
  try {
    return f();
  } catch (const sg::SgError& e) {
    return node_err(node, e.code, e.what());
  } catch (const std::bad_alloc&) {
    return node_err(node, SG_E_NOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return node_err(node, SG_E_ARG, e.what());
  }
}

}  // namespace

struct sg_node_plan {
  int64_t n = 0;
  int32_t k = 0;
  std::vector<int32_t> owner;            // device index (into the node) of each call
  std::vector<double> cost;              // the analytic cost the assignment used (ns of one MI355X)
  // per shard: its calls (ascending) in chunks of consecutive shard calls, each planned
  // as one sg_plan; a chunk's packed samples sit at dev_off of the shard's device output
  struct Chunk {
    int64_t j0, j1;      // shard-local call range
    sg_plan* plan = nullptr;
    int64_t dev_off = 0, samples = 0;
    std::vector<int64_t> keep;  // while planning: the chunk's planned calls
    bool uploaded = false;       // uploaded, host copies released (sg_plan_release_host)
  };
  std::vector<std::vector<int64_t>> idx;
  std::vector<std::vector<Chunk>> chunks;
  std::vector<int64_t> len, off;         // whole batch, call order, single-device layout
  std::vector<int32_t> status;
  std::vector<std::string> msg;
  int64_t total = 0;
  bool diverged = false;                 // a replayed call failed where its recording did not
  ~sg_node_plan() {
    for (auto& cs : chunks)
      for (Chunk& c : cs) sg_plan_destroy(c.plan);
  }
};

int sg_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int sg_node_create(const int32_t* devices, int32_t n, sg_node** out) {
  if (!out) return SG_E_ARG;
  *out = nullptr;
  std::vector<int32_t> dv;
  if (devices) {
    if (n <= 0) return SG_E_ARG;
    dv.assign(devices, devices + n);
  } else {
    const int c = n > 0 ? n : sg_device_count();
    if (c <= 0) return SG_E_DEVICE;
    for (int i = 0; i < c; ++i) dv.push_back(i);
  }
  for (int32_t d : dv)
    if (d < 0) return SG_E_ARG;
  auto* node = new (std::nothrow) sg_node();
  if (!node) return SG_E_NOMEM;
  node->devices = dv;
  node->dev.resize(dv.size());
  *out = node;
  return SG_OK;
}

void sg_node_destroy(sg_node* node) {
  if (!node) return;
  int cur = -1;
  const bool have = hipGetDevice(&cur) == hipSuccess;  // the caller's device, restored below
  for (size_t k = 0; k < node->devices.size(); ++k) {
    sg_node::Dev& d = node->dev[k];
    if (!d.ctx && !d.run && !d.copy) continue;
    (void)hipSetDevice(node->devices[k]);
    for (hipEvent_t e : d.ev) (void)hipEventDestroy(e);
    if (d.run) (void)hipStreamDestroy(d.run);
    if (d.copy) (void)hipStreamDestroy(d.copy);
    if (d.d_out) (void)hipFree(d.d_out);
    for (void* p : d.pin)
      if (p) (void)hipHostFree(p);
    sg_ctx_destroy(d.ctx);
  }
  if (have) (void)hipSetDevice(cur);
  delete node;
}

int32_t sg_node_size(const sg_node* node) { return node ? (int32_t)node->devices.size() : 0; }
const char* sg_node_last_error(const sg_node* node) { return node ? node->err.c_str() : ""; }

namespace {
// calls per chunk plan of a shard: SG_NODE_CHUNK (default 4096), and at most ~2^27
// estimated samples (512 MB of fp32 per staging slot)
int64_t chunk_calls() {
  static const int64_t v = [] {
    const char* e = std::getenv("SG_NODE_CHUNK");
    const long long c = e ? std::atoll(e) : 0;
    return (int64_t)(c > 0 ? c : 4096);
  }();
  return v;
}
constexpr double kChunkSamples = 134217728.0;
}  // namespace

int sg_node_plan_batch(sg_node* node, const sg_call_desc* calls, int64_t n_calls, sg_node_plan** out) {
  if (!node || !out || (n_calls > 0 && !calls) || n_calls < 0) return SG_E_ARG;
  *out = nullptr;
  return node_guarded(node, [&]() {
    auto P = std::make_unique<sg_node_plan>();
    const int32_t K = (int32_t)node->devices.size();
    P->n = n_calls;
    P->k = K;
    std::vector<double> cost((size_t)n_calls);
    for (int64_t i = 0; i < n_calls; ++i) cost[i] = call_cost(calls[i]);
    P->owner = lpt(cost, K);
    P->cost = cost;
    P->idx.assign(K, {});
    for (int64_t i = 0; i < n_calls; ++i) P->idx[P->owner[i]].push_back(i);
    P->len.assign(n_calls, 0);
    P->off.assign(n_calls, 0);
    P->status.assign(n_calls, 0);
    P->msg.assign(n_calls, "");

    // chunks: consecutive calls of a shard, <= chunk_calls() calls and ~kChunkSamples
    // samples (estimated from the arguments, so fixed before any call is planned)
    P->chunks.assign(K, {});
    for (int32_t k = 0; k < K; ++k) {
      const std::vector<int64_t>& ix = P->idx[k];
      const int64_t m = (int64_t)ix.size();
      for (int64_t j = 0; j < m;) {
        int64_t j1 = j;
        double smp = 0;
        while (j1 < m && j1 - j < chunk_calls() && (j1 == j || smp + call_samples(calls[ix[j1]]) <= kChunkSamples))
          smp += call_samples(calls[ix[j1++]]);
        sg_node_plan::Chunk c;
        c.j0 = j;
        c.j1 = j1;
        P->chunks[k].push_back(c);
        j = j1;
      }
    }
    // the calls each chunk plans: the caller's descriptors, or (callbacks) the replay
    // of the draws recorded in a first pass over the batch in call order
    std::vector<sg_call_desc> desc(calls, calls + n_calls);
    std::vector<char> planned((size_t)n_calls, 1);
    const bool any_cb = [&] {
      for (int64_t i = 0; i < n_calls; ++i)
        if (has_callbacks(calls[i].random)) return true;
      return false;
    }();
    const bool independent = any_cb;
    std::vector<DrawLog> logs(any_cb ? (size_t)n_calls : 0);
    // chunk planning: shard k's chunk c over its calls that were not stopped
    auto plan_chunk = [&](int32_t k, sg_node_plan::Chunk& c) {
      std::vector<sg_call_desc> sd;
      std::vector<int64_t> keep;
      for (int64_t j = c.j0; j < c.j1; ++j) {
        const int64_t i = P->idx[k][(size_t)j];
        if (!planned[i]) continue;
        if (any_cb && has_callbacks(calls[i].random)) {  // replay: the recorded draws, in order, by callback
          sg_random& r = desc[i].random;
          r = sg_random{};
          r.norm_cb = replay_norm;
          r.unif_cb = replay_unif;
          r.unif_n_cb = replay_unif_n;
          r.gamma_cb = calls[i].random.gamma_cb ? replay_gamma : nullptr;
          r.user = &logs[i];
          logs[i].gn = logs[i].gu = logs[i].gr = logs[i].gi = 0;
        }
        sd.push_back(desc[i]);
        keep.push_back(i);
      }
      c.keep = keep;
      if (sd.empty()) return;
      sg_plan* sp = nullptr;
      // beside the recording thread: one host thread fewer (the stream is the critical path)
      const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
      const int rc = sg::plan_batch_ex(nullptr, sd.data(), (int64_t)sd.size(), independent, &sp,
                                       any_cb ? std::max(1, std::min(16, hw) - 1) : 0);
      if (rc) throw sg::SgError(rc, "node planning: shard " + std::to_string(k) + " failed");
      c.plan = sp;
      c.samples = sg_plan_total_samples(sp);
      const int64_t n = (int64_t)sd.size();
      std::vector<int64_t> l((size_t)n), o((size_t)n);
      std::vector<int32_t> st((size_t)n);
      sg_plan_lengths(sp, l.data(), o.data());
      sg_plan_status(sp, st.data());
      for (int64_t q = 0; q < n; ++q) {
        const int64_t i = keep[(size_t)q];
        P->len[i] = l[q];
        P->status[i] = st[q];
        if (st[q]) P->msg[i] = sg_plan_call_message(sp, q);
      }
    };
    // chunks in the order their last call is reached in call order
    std::vector<std::pair<int64_t, std::pair<int32_t, size_t>>> order;
    for (int32_t k = 0; k < K; ++k)
      for (size_t c = 0; c < P->chunks[k].size(); ++c)
        order.push_back({P->idx[k][(size_t)(P->chunks[k][c].j1 - 1)], {k, c}});
    std::sort(order.begin(), order.end());
    if (!any_cb) {
      for (auto& o : order) plan_chunk(o.second.first, P->chunks[o.second.first][o.second.second]);
    } else {
      std::vector<sg_call_desc> rec(calls, calls + n_calls);
      for (int64_t i = 0; i < n_calls; ++i) {
        if (!has_callbacks(calls[i].random)) continue;  // injected arrays only: planned as given
        logs[i].src = &calls[i].random;
        // generateNoise's runif(nr * nc): ~2 uniforms per sample at 75 % overlap
        logs[i].runs.reserve((size_t)(2.2 * call_samples(calls[i])) + 1024);
        logs[i].normals.reserve(4096);
        logs[i].uniforms.reserve(256);
        sg_random& r = rec[i].random;
        r = sg_random{};
        r.norm_cb = rec_norm;
        r.unif_cb = rec_unif;
        r.unif_n_cb = rec_unif_n;
        // gammas are recorded only where the caller draws them by callback; otherwise the
        // planner draws them from normals and uniforms (sg_rmath.h Rng::rgamma), which the
        // other two record
        r.gamma_cb = calls[i].random.gamma_cb ? rec_gamma : nullptr;
        r.user = &logs[i];
      }
      // pass 1 on this thread, in call order: every call's draws (R's stream, R's order)
      // and the errors that precede its last draw, no device work (Batch::draws_only); a
      // failing callback call stops the stream. Pass 2 on a worker thread meanwhile:
      // each chunk is planned from the recorded draws as soon as its last call is
      // recorded (plan_batch_ex: host threads), so only the last chunks trail the stream.
      std::mutex mu;
      std::condition_variable cv;
      int64_t done = -1;  // calls [0, done] recorded
      std::exception_ptr werr;
      std::thread worker([&]() {
        try {
          for (auto& o : order) {
            {
              std::unique_lock<std::mutex> lk(mu);
              cv.wait(lk, [&] { return done >= o.first; });
            }
            plan_chunk(o.second.first, P->chunks[o.second.first][o.second.second]);
          }
        } catch (...) {
          werr = std::current_exception();
        }
      });
      std::vector<int32_t> st;
      std::vector<std::string> ms;
      const auto t0 = std::chrono::steady_clock::now();
      try {
        sg::record_draws(rec.data(), n_calls, st, ms, [&](int64_t i, int32_t status) {
          if (status) planned[i] = 0;  // read by the worker only after `done` passes i
          if ((i & 15) == 15 || i + 1 == n_calls) {
            {
              std::lock_guard<std::mutex> lk(mu);
              done = i;
            }
            cv.notify_one();
          }
        });
      } catch (...) {
        {
          std::lock_guard<std::mutex> lk(mu);
          done = n_calls;  // release the worker; its chunks plan what was recorded
        }
        cv.notify_one();
        worker.join();
        throw;
      }
      {
        std::lock_guard<std::mutex> lk(mu);
        done = n_calls;
      }
      cv.notify_one();
      if (std::getenv("SG_PLAN_PROF"))
        std::fprintf(stderr, "sg_node_prof record_draws (%lld calls) %.3f s\n", (long long)n_calls,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      worker.join();
      if (werr) std::rethrow_exception(werr);
      for (int64_t i = 0; i < n_calls; ++i)
        if (st[i]) {
          P->status[i] = st[i];
          P->msg[i] = ms[i];
        }
    }
    for (int32_t k = 0; k < K; ++k) {  // the shards' calls that were planned, chunk device offsets
      std::vector<int64_t> keep;
      int64_t dev_off = 0;
      for (auto& c : P->chunks[k]) {
        const int64_t j0 = (int64_t)keep.size();
        keep.insert(keep.end(), c.keep.begin(), c.keep.end());
        c.j0 = j0;
        c.j1 = (int64_t)keep.size();
        c.dev_off = dev_off;
        dev_off += c.samples;
        c.keep.clear();
      }
      P->idx[k] = keep;
      auto& cs = P->chunks[k];
      cs.erase(std::remove_if(cs.begin(), cs.end(), [](const sg_node_plan::Chunk& c) { return !c.plan; }), cs.end());
    }
    if (independent) {
      // A replayed call can fail only after its last draw (a failure before it is in
      // the recording): R's loop would have stopped there, so later callback calls are
      // marked unplanned as plan_range marks them (their draws were consumed by the
      // recording pass: sg_node_plan_batch's stream position is then past R's)
      int64_t first_fail = -1;
      for (int64_t i = 0; i < n_calls && first_fail < 0; ++i)
        if (P->status[i] && has_callbacks(calls[i].random)) first_fail = i;
      for (int64_t i = first_fail + 1; first_fail >= 0 && i < n_calls; ++i)
        if (has_callbacks(calls[i].random) && planned[i]) {
          if (P->status[i] == 0) P->diverged = true;
          P->status[i] = SG_E_ARG;
          P->msg[i] = "not planned: call " + std::to_string(first_fail + 1) +
                      " of the batch failed first (the RNG callback stream stops there)";
          P->len[i] = 0;
        }
    }
    // the whole batch's layout: 64-sample (256-B) aligned slots in call order, as one
    // device's plan lays them out (sg_api.cpp plan_range)
    int64_t off = 0;
    for (int64_t i = 0; i < n_calls; ++i) {
      P->off[i] = off;
      if (P->status[i] == 0) off += (P->len[i] + 63) / 64 * 64;
    }
    P->total = off;
    *out = P.release();
    return SG_OK;
  });
}

void sg_node_plan_destroy(sg_node_plan* p) { delete p; }
int64_t sg_node_plan_total_samples(const sg_node_plan* p) { return p ? p->total : 0; }
int64_t sg_node_plan_n_calls(const sg_node_plan* p) { return p ? p->n : 0; }

int sg_node_plan_lengths(const sg_node_plan* p, int64_t* out_len, int64_t* out_off) {
  if (!p) return SG_E_ARG;
  if (out_len) std::memcpy(out_len, p->len.data(), p->len.size() * sizeof(int64_t));
  if (out_off) std::memcpy(out_off, p->off.data(), p->off.size() * sizeof(int64_t));
  return SG_OK;
}
int sg_node_plan_status(const sg_node_plan* p, int32_t* out_status) {
  if (!p || !out_status) return SG_E_ARG;
  std::memcpy(out_status, p->status.data(), p->status.size() * sizeof(int32_t));
  return SG_OK;
}
const char* sg_node_plan_call_message(const sg_node_plan* p, int64_t i) {
  if (!p || i < 0 || i >= p->n) return "";
  return p->msg[i].c_str();
}
int sg_node_plan_owner(const sg_node_plan* p, int32_t* owner) {
  if (!p || !owner) return SG_E_ARG;
  std::memcpy(owner, p->owner.data(), p->owner.size() * sizeof(int32_t));
  return SG_OK;
}
int sg_node_plan_costs(const sg_node_plan* p, double* cost) {
  if (!p || !cost) return SG_E_ARG;
  std::memcpy(cost, p->cost.data(), p->cost.size() * sizeof(double));
  return SG_OK;
}
int64_t sg_node_plan_shard_samples(const sg_node_plan* p, int32_t k) {
  if (!p || k < 0 || k >= p->k) return 0;
  int64_t s = 0;
  for (const auto& c : p->chunks[k]) s += c.samples;
  return s;
}
int32_t sg_node_plan_chunks(const sg_node_plan* p, int32_t k) {
  return p && k >= 0 && k < p->k ? (int32_t)p->chunks[k].size() : 0;
}
int32_t sg_node_plan_diverged(const sg_node_plan* p) { return p && p->diverged ? 1 : 0; }
int sg_node_plan_call_work(const sg_node_plan* p, double* rows, double* fft_flops) {
  if (!p) return SG_E_ARG;
  for (int32_t k = 0; k < p->k; ++k)
    for (const auto& c : p->chunks[k]) {
      const int64_t n = c.j1 - c.j0;
      std::vector<double> r((size_t)n), f((size_t)n);
      sg_plan_call_work(c.plan, r.data(), f.data());
      for (int64_t q = 0; q < n; ++q) {
        const int64_t i = p->idx[k][(size_t)(c.j0 + q)];
        if (rows) rows[i] = r[q];
        if (fft_flops) fft_flops[i] = f[q];
      }
    }
  return SG_OK;
}

namespace {
#define NODE_HIPCHK(x)                                                                    \
  do {                                                                                    \
    hipError_t _e = (x);                                                                  \
    if (_e != hipSuccess)                                                                 \
      throw sg::SgError(SG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e));     \
  } while (0)

// f(a, b) over [0, n) split into at most `threads` ranges on host threads
template <class F>
void host_parallel(int64_t n, int threads, F&& f) {
  if (threads <= 1 || n < (1 << 16)) {
    f((int64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back([&, t]() { f(n * t / threads, n * (t + 1) / threads); });
  f((int64_t)0, n / threads);
  for (auto& x : th) x.join();
}

// Shard k on its device, pipelined by chunk: every chunk's kernels are queued on the
// run stream (uploading chunk plans on first use), then chunk c's packed samples go
// over the link into pinned staging slot c % 2 on the copy stream while host threads
// scatter chunk c - 1's calls to their whole-batch offsets (widened to double for R):
// the D2H of one chunk overlaps the compute of the later ones and the scatter of the
// earlier one. The device output and the staging stay allocated for the next execute
// (staging: two slots of the largest chunk, <= ~512 MB each).
template <typename T>
void run_shard(sg_node* node, sg_node_plan* p, int32_t k, T* out_host, int threads) {
  auto& cs = p->chunks[k];
  if (cs.empty()) return;
  sg_node::Dev& d = node->dev[k];
  const int dv = node->devices[k];
  NODE_HIPCHK(hipSetDevice(dv));
  if (!d.run) NODE_HIPCHK(hipStreamCreateWithFlags(&d.run, hipStreamNonBlocking));
  if (!d.copy) NODE_HIPCHK(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
  if (!d.ctx) {
    sg_ctx* c = nullptr;
    const int rc = sg_ctx_create(dv, &c);
    if (rc) throw sg::SgError(rc, "sg_ctx_create(" + std::to_string(dv) + ") failed");
    d.ctx = c;
  }
  const int64_t total = sg_node_plan_shard_samples(p, k);
  const size_t bytes = (size_t)std::max<int64_t>(total, 1) * sizeof(float);
  if (d.d_bytes < bytes) {
    if (d.d_out) NODE_HIPCHK(hipFree(d.d_out));
    d.d_out = nullptr;
    d.d_bytes = 0;
    NODE_HIPCHK(hipMalloc(&d.d_out, bytes));
    d.d_bytes = bytes;
  }
  size_t slot = 4;
  for (const auto& c : cs) slot = std::max(slot, (size_t)c.samples * sizeof(float));
  if (d.pin_bytes < slot) {
    for (void*& q : d.pin) {
      if (q) NODE_HIPCHK(hipHostFree(q));
      q = nullptr;
    }
    d.pin_bytes = 0;
    for (void*& q : d.pin) NODE_HIPCHK(hipHostMalloc(&q, slot, hipHostMallocDefault));
    d.pin_bytes = slot;
  }
  const size_t nc = cs.size();
  while (d.ev.size() < 2 * nc) {
    hipEvent_t e;
    NODE_HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    d.ev.push_back(e);
  }
  for (size_t c = 0; c < nc; ++c) {
    if (!cs[c].uploaded) {  // first execute: upload, then free the chunk's host copies (~0.7 MB per C5 call)
      int rc = sg_plan_upload(d.ctx, cs[c].plan);
      if (rc) throw sg::SgError(rc, std::string("shard upload: ") + sg_last_error(d.ctx));
      rc = sg_plan_release_host(cs[c].plan);
      if (rc) throw sg::SgError(rc, "shard upload: releasing host copies failed");
      cs[c].uploaded = true;
    }
    const int rc = sg_execute(d.ctx, cs[c].plan, d.d_out + cs[c].dev_off, d.run);
    if (rc) throw sg::SgError(rc, std::string("shard execute: ") + sg_last_error(d.ctx));
    NODE_HIPCHK(hipEventRecord(d.ev[2 * c], d.run));
  }
  const std::vector<int64_t>& idx = p->idx[k];
  // a chunk of consecutive calls of the batch (one device: every chunk) is one block
  // of the whole-batch layout: fp32 goes straight into the caller's buffer
  auto direct = [&](size_t c) {
    if (!std::is_same<T, float>::value || p->diverged) return false;  // diverged: calls unplanned after planning
    return idx[(size_t)(cs[c].j1 - 1)] - idx[(size_t)cs[c].j0] == cs[c].j1 - 1 - cs[c].j0;
  };
  auto copy = [&](size_t c) {
    NODE_HIPCHK(hipStreamWaitEvent(d.copy, d.ev[2 * c], 0));
    if (cs[c].samples)
      NODE_HIPCHK(hipMemcpyAsync(direct(c) ? (void*)(out_host + p->off[idx[(size_t)cs[c].j0]]) : d.pin[c % 2],
                                 d.d_out + cs[c].dev_off, (size_t)cs[c].samples * sizeof(float),
                                 hipMemcpyDeviceToHost, d.copy));
    NODE_HIPCHK(hipEventRecord(d.ev[2 * c + 1], d.copy));
  };
  auto scatter = [&](size_t c) {
    NODE_HIPCHK(hipEventSynchronize(d.ev[2 * c + 1]));
    if (direct(c)) return;
    const float* h = static_cast<const float*>(d.pin[c % 2]);
    const int64_t n = cs[c].j1 - cs[c].j0;
    std::vector<int64_t> l((size_t)n), o((size_t)n);
    sg_plan_lengths(cs[c].plan, l.data(), o.data());
    // calls in contiguous runs of the whole-batch layout move as one block
    host_parallel(cs[c].samples, threads, [&](int64_t a, int64_t b) {
      for (int64_t q = 0; q < n; ++q) {
        const int64_t i = idx[(size_t)(cs[c].j0 + q)];
        if (p->status[i]) continue;
        const int64_t s0 = std::max(a, o[q]), s1 = std::min(b, o[q] + l[q]);
        T* dst = out_host + p->off[i] - o[q];
        for (int64_t s = s0; s < s1; ++s) dst[s] = (T)h[s];
      }
    });
  };
  copy(0);
  for (size_t c = 1; c < nc; ++c) {
    copy(c);      // slot c % 2 was scattered at step c - 1
    scatter(c - 1);
  }
  scatter(nc - 1);
}

template <typename T>
int node_execute(sg_node* node, sg_node_plan* p, T* out_host) {
  if (!node || !p || (p->total > 0 && !out_host) || p->k != (int32_t)node->devices.size()) return SG_E_ARG;
  return node_guarded(node, [&]() {
    int cur = -1;
    const bool have = hipGetDevice(&cur) == hipSuccess;
    std::vector<std::exception_ptr> errs((size_t)p->k);
    std::vector<std::thread> th;
    int busy = 0;
    for (int32_t k = 0; k < p->k; ++k) busy += p->chunks[k].empty() ? 0 : 1;
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int threads = std::max(1, std::min(16, hw / std::max(1, busy)));
    for (int32_t k = 0; k < p->k; ++k)
      th.emplace_back([&, k]() {
        try {
          run_shard(node, p, k, out_host, threads);
        } catch (...) {
          errs[k] = std::current_exception();
        }
      });
    for (auto& t : th) t.join();
    if (have) (void)hipSetDevice(cur);
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
    return SG_OK;
  });
}
}  // namespace

int sg_node_execute_to_host(sg_node* node, sg_node_plan* p, double* out_host) {
  return node_execute(node, p, out_host);
}
int sg_node_execute_to_host_f32(sg_node* node, sg_node_plan* p, float* out_host) {
  return node_execute(node, p, out_host);
}
