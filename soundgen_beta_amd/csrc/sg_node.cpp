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
// sequential stream in call order: the node first plans every call in order
// with recording callbacks (the draws R would make, in R's order; a failing
// call stops the stream as lapply would), then plans the shards from the
// recorded draws, each call replaying its own -- the second pass runs on host
// threads and yields exactly the plans the stream would have.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <numeric>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "sg_plan.h"
#include "soundgen_hip.h"

struct sg_node {
  std::vector<int32_t> devices;
  std::vector<sg_ctx*> ctx;          // created on first upload/execute (planning needs no device)
  std::vector<hipStream_t> stream;   // one launch stream per shard
  std::vector<void*> pinned;         // per shard: pinned host staging of its packed samples
  std::vector<size_t> pinned_bytes;
  std::string err;
  std::mutex mu;
};

namespace {

// ---- per-call draw logs (callback batches) ----------------------------------
struct DrawLog {
  const sg_random* src = nullptr;  // the caller's draw source (arrays first, then callbacks)
  int64_t ni = 0, ui = 0;          // cursors into src's arrays
  std::vector<double> normals, uniforms, gammas;
  size_t gi = 0;                   // replay cursor of gammas
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
  std::vector<std::vector<int64_t>> idx; // per shard: its calls, ascending
  std::vector<sg_plan*> shard;           // per shard (nullptr: no calls)
  std::vector<int64_t> len, off;         // whole batch, call order, single-device layout
  std::vector<int32_t> status;
  std::vector<std::string> msg;
  int64_t total = 0;
  ~sg_node_plan() {
    for (sg_plan* p : shard) sg_plan_destroy(p);
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
  node->ctx.assign(dv.size(), nullptr);
  node->stream.assign(dv.size(), nullptr);
  node->pinned.assign(dv.size(), nullptr);
  node->pinned_bytes.assign(dv.size(), 0);
  *out = node;
  return SG_OK;
}

void sg_node_destroy(sg_node* node) {
  if (!node) return;
  for (size_t k = 0; k < node->devices.size(); ++k) {
    if (node->ctx[k]) {
      (void)hipSetDevice(node->devices[k]);
      if (node->stream[k]) (void)hipStreamDestroy(node->stream[k]);
      if (node->pinned[k]) (void)hipHostFree(node->pinned[k]);
      sg_ctx_destroy(node->ctx[k]);
    }
  }
  delete node;
}

int32_t sg_node_size(const sg_node* node) { return node ? (int32_t)node->devices.size() : 0; }
const char* sg_node_last_error(const sg_node* node) { return node ? node->err.c_str() : ""; }

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

    // the calls each shard plans: the caller's descriptors, or (callbacks) the
    // replay of the draws recorded in a first pass over the batch in call order
    std::vector<sg_call_desc> desc(calls, calls + n_calls);
    std::vector<char> planned((size_t)n_calls, 1);
    bool independent = false;
    std::vector<DrawLog> logs;
    bool any_cb = false;
    for (int64_t i = 0; i < n_calls && !any_cb; ++i) any_cb = has_callbacks(calls[i].random);
    if (any_cb) {
      logs.resize((size_t)n_calls);
      std::vector<sg_call_desc> rec(calls, calls + n_calls);
      for (int64_t i = 0; i < n_calls; ++i) {
        logs[i].src = &calls[i].random;
        sg_random& r = rec[i].random;
        r = sg_random{};
        r.norm_cb = rec_norm;
        r.unif_cb = rec_unif;
        // no gamma callback: the planner draws gammas from normals and uniforms
        // (sg_rmath.h Rng::gamma), which the other two record
        r.gamma_cb = calls[i].random.gamma_cb ? rec_gamma : nullptr;
        r.user = &logs[i];
      }
      // pass 1, in call order on this thread: the stream's draws per call (a failing
      // call stops it: plan_range plans no later callback call)
      sg_plan* whole = nullptr;
      int rc = sg::plan_batch_ex(nullptr, rec.data(), n_calls, false, &whole);
      if (rc) throw sg::SgError(rc, "node planning: recording pass failed");
      std::unique_ptr<sg_plan, void (*)(sg_plan*)> hold(whole, sg_plan_destroy);
      std::vector<int32_t> st((size_t)n_calls);
      sg_plan_status(whole, st.data());
      for (int64_t i = 0; i < n_calls; ++i)
        if (st[i]) {
          planned[i] = 0;
          P->status[i] = st[i];
          P->msg[i] = sg_plan_call_message(whole, i);
        }
      // pass 2 replays: normals and uniforms as injected arrays, gammas by callback
      for (int64_t i = 0; i < n_calls; ++i) {
        sg_random& r = desc[i].random;
        r = sg_random{};
        r.normals = logs[i].normals.data();
        r.n_normals = (int64_t)logs[i].normals.size();
        r.uniforms = logs[i].uniforms.data();
        r.n_uniforms = (int64_t)logs[i].uniforms.size();
        r.gamma_cb = calls[i].random.gamma_cb ? replay_gamma : nullptr;
        r.user = &logs[i];
        logs[i].gi = 0;
      }
      independent = true;
    }
    P->shard.assign(K, nullptr);
    for (int32_t k = 0; k < K; ++k) {
      std::vector<sg_call_desc> sd;
      std::vector<int64_t> keep;
      for (int64_t i : P->idx[k])
        if (planned[i]) {
          sd.push_back(desc[i]);
          keep.push_back(i);
        }
      P->idx[k] = keep;
      if (sd.empty()) continue;
      sg_plan* sp = nullptr;
      const int rc = sg::plan_batch_ex(nullptr, sd.data(), (int64_t)sd.size(), independent, &sp);
      if (rc) throw sg::SgError(rc, "node planning: shard " + std::to_string(k) + " failed");
      P->shard[k] = sp;
      const int64_t m = (int64_t)sd.size();
      std::vector<int64_t> l((size_t)m), o((size_t)m);
      std::vector<int32_t> st((size_t)m);
      sg_plan_lengths(sp, l.data(), o.data());
      sg_plan_status(sp, st.data());
      for (int64_t j = 0; j < m; ++j) {
        const int64_t i = keep[j];
        P->len[i] = l[j];
        P->status[i] = st[j];
        if (st[j]) P->msg[i] = sg_plan_call_message(sp, j);
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
  if (!p || k < 0 || k >= p->k || !p->shard[k]) return 0;
  return sg_plan_total_samples(p->shard[k]);
}

namespace {
#define NODE_HIPCHK(x)                                                                    \
  do {                                                                                    \
    hipError_t _e = (x);                                                                  \
    if (_e != hipSuccess)                                                                 \
      throw sg::SgError(SG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e));     \
  } while (0)

// Shard k on its device: upload, execute on the shard's stream, one D2H copy into
// the shard's pinned staging, then each call's samples to its whole-batch offset.
template <typename T>
void run_shard(sg_node* node, sg_node_plan* p, int32_t k, T* out_host) {
  sg_plan* sp = p->shard[k];
  if (!sp) return;
  const int dev = node->devices[k];
  NODE_HIPCHK(hipSetDevice(dev));
  if (!node->ctx[k]) {
    sg_ctx* c = nullptr;
    const int rc = sg_ctx_create(dev, &c);
    if (rc) throw sg::SgError(rc, "sg_ctx_create(" + std::to_string(dev) + ") failed");
    node->ctx[k] = c;
    NODE_HIPCHK(hipStreamCreateWithFlags(&node->stream[k], hipStreamNonBlocking));
  }
  sg_ctx* c = node->ctx[k];
  int rc = sg_plan_upload(c, sp);
  if (rc) throw sg::SgError(rc, std::string("shard upload: ") + sg_last_error(c));
  const int64_t T_ = sg_plan_total_samples(sp);
  const size_t bytes = (size_t)std::max<int64_t>(T_, 1) * sizeof(float);
  float* d_out = nullptr;
  NODE_HIPCHK(hipMalloc(&d_out, bytes));
  std::unique_ptr<void, hipError_t (*)(void*)> hold(d_out, hipFree);
  rc = sg_execute(c, sp, d_out, node->stream[k]);
  if (rc) throw sg::SgError(rc, std::string("shard execute: ") + sg_last_error(c));
  if (node->pinned_bytes[k] < bytes) {
    if (node->pinned[k]) NODE_HIPCHK(hipHostFree(node->pinned[k]));
    node->pinned[k] = nullptr;
    node->pinned_bytes[k] = 0;
    NODE_HIPCHK(hipHostMalloc(&node->pinned[k], bytes, hipHostMallocDefault));
    node->pinned_bytes[k] = bytes;
  }
  const float* h = static_cast<const float*>(node->pinned[k]);
  NODE_HIPCHK(hipMemcpyAsync(node->pinned[k], d_out, bytes, hipMemcpyDeviceToHost, node->stream[k]));
  NODE_HIPCHK(hipStreamSynchronize(node->stream[k]));
  const std::vector<int64_t>& idx = p->idx[k];
  std::vector<int64_t> l(idx.size()), o(idx.size());
  sg_plan_lengths(sp, l.data(), o.data());
  for (size_t j = 0; j < idx.size(); ++j) {
    const int64_t i = idx[j];
    if (p->status[i]) continue;
    T* dst = out_host + p->off[i];
    const float* src = h + o[j];
    for (int64_t q = 0; q < l[j]; ++q) dst[q] = (T)src[q];
  }
}

template <typename T>
int node_execute(sg_node* node, sg_node_plan* p, T* out_host) {
  if (!node || !p || (p->total > 0 && !out_host) || p->k != (int32_t)node->devices.size()) return SG_E_ARG;
  return node_guarded(node, [&]() {
    std::vector<std::exception_ptr> errs((size_t)p->k);
    std::vector<std::thread> th;
    for (int32_t k = 0; k < p->k; ++k)
      th.emplace_back([&, k]() {
        try {
          run_shard(node, p, k, out_host);
        } catch (...) {
          errs[k] = std::current_exception();
        }
      });
    for (auto& t : th) t.join();
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
