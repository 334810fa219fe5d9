// sg_api.cpp — C-ABI of libsoundgen_hip.so: context, batch plan/upload/
// execute, and the synchronous function-level entries mirroring the R API.
// No C++ exception crosses this boundary.
#include <hip/hip_runtime.h>

#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "sg_plan.h"
#include "sg_exec.h"
#include "sg_prof.h"

#include <cstdio>
#include <cstdlib>

struct sg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t aux = nullptr;  // finalize stream of the slice pipeline
  std::string err;
  bool profiling = false;
  std::vector<sg::SgProfEvent> prof_events;
};

struct sg_plan {
  sg::Batch B;
  sg::DevicePlan D;
};

namespace sg {
std::atomic<int64_t> g_prof_ns[PF_N];
bool g_prof_on = std::getenv("SG_PLAN_PROF") != nullptr;
}  // namespace sg

namespace {

int set_err(sg_ctx* ctx, int code, const std::string& m) {
  if (ctx) ctx->err = m;
  return code;
}

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t _e = (x);                                                                  \
    if (_e != hipSuccess)                                                                 \
      throw sg::SgError(SG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

template <class F>
int guarded(sg_ctx* ctx, F&& f) {
  try {
    return f();
  } catch (const sg::SgError& e) {
    return set_err(ctx, e.code, e.what());
  } catch (const std::bad_alloc&) {
    return set_err(ctx, SG_E_NOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return set_err(ctx, SG_E_ARG, e.what());
  }
}

// Rolls a Batch back to a checkpoint when planning one call fails.
struct Checkpoint {
  size_t segs, epochs, knots, amps, tasks, pieces, syls, syl_tiles, cknots, fl, items;
  size_t frames[2], olas[2], mixes[2], copies;
  int64_t w_total, harm_samples, harm_terms, harm_amp_bytes, fft_frames, fs_total;
  explicit Checkpoint(const sg::Batch& B)
      : segs(B.segs.size()), epochs(B.epochs.size()), knots(B.knots.size()), amps(B.amps.size()),
        tasks(B.tasks.size()), pieces(B.pieces.size()), syls(B.syls.size()), syl_tiles(B.syl_tiles.size()),
        cknots(B.cknots.size()), fl(B.fl.size()), items(B.items.size()), copies(B.copies.size()),
        w_total(B.w_total), harm_samples(B.harm_samples), harm_terms(B.harm_terms),
        harm_amp_bytes(B.harm_amp_bytes), fft_frames(B.fft_frames), fs_total(B.fs_total) {
    for (int p = 0; p < 2; ++p) { frames[p] = B.frames[p].size(); olas[p] = B.olas[p].size(); mixes[p] = B.mixes[p].size(); }
  }
  void restore(sg::Batch& B) const {
    B.segs.resize(segs); B.epochs.resize(epochs); B.knots.resize(knots); B.amps.resize(amps);
    B.tasks.resize(tasks); B.pieces.resize(pieces); B.syls.resize(syls); B.syl_tiles.resize(syl_tiles);
    B.cknots.resize(cknots); B.fl.resize(fl); B.items.resize(items); B.copies.resize(copies);
    for (int p = 0; p < 2; ++p) {
      B.frames[p].resize(frames[p]); B.frame_geom[p].resize(frames[p]);
      B.olas[p].resize(olas[p]); B.mixes[p].resize(mixes[p]);
    }
    B.w_total = w_total; B.harm_samples = harm_samples; B.harm_terms = harm_terms;
    B.harm_amp_bytes = harm_amp_bytes; B.fft_frames = fft_frames; B.fs_total = fs_total;
  }
};

}  // namespace

extern "C" {

int sg_abi_version(void) { return SG_ABI_VERSION; }

void sg_default_harm_params(sg_harm_params* p) {
  *p = sg_harm_params{50, 0, 0, 0, 1, 100, 0, 0, 0, -18, -2, -6, 0, 3, 6, 12, 0, .5, .125, .5, 300, 100,
                      0, 0, 30, 75, 16000, 75, 3500, 3500, -120};
}

int sg_ctx_create(int device, sg_ctx** out) {
  *out = nullptr;
  auto* c = new (std::nothrow) sg_ctx();
  if (!c) return SG_E_NOMEM;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SG_E_DEVICE;
  }
  *out = c;
  return SG_OK;
}

void sg_ctx_destroy(sg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  for (auto& ev : ctx->prof_events) { (void)hipEventDestroy(ev.e0); (void)hipEventDestroy(ev.e1); }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  delete ctx;
}

const char* sg_last_error(const sg_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

int sg_plan_batch(sg_ctx* ctx, const sg_call_desc* calls, int64_t n_calls, sg_plan** out) {
  return guarded(ctx, [&]() {
    auto P = std::make_unique<sg_plan>();
    sg::Batch& B = P->B;
    B.call_len.assign(n_calls, 0);
    B.call_off.assign(n_calls, 0);
    B.call_status.assign(n_calls, 0);
    B.call_msg.assign(n_calls, "");
    int64_t off = 0;
    for (int64_t c = 0; c < n_calls; ++c) {
      const sg_call_desc& d = calls[c];
      Checkpoint cp(B);
      const int first_syl = (int)B.syls.size();
      try {
        sg::Rng R;
        R.s = &d.random;
        int64_t L = 0;
        if (d.kind == SG_CALL_HARMONICS) {
          if (!d.pitch || !d.harm) throw sg::SgError(SG_E_ARG, "harmonics call without pitch/params");
          L = sg::plan_harmonics(B, d.pitch, d.pitch_len, *d.harm, d.amplAnchors, R, off, false);
          sg::tile_syllables(B, first_syl);
        } else if (d.kind == SG_CALL_SOUNDGEN) {
          if (!d.args) throw sg::SgError(SG_E_ARG, "soundgen call without args");
          L = sg::plan_soundgen(B, *d.args, R, off, first_syl);
          sg::tile_syllables(B, first_syl);
        } else {
          throw sg::SgError(SG_E_ARG, "unknown call kind");
        }
        B.call_off[c] = off;
        B.call_len[c] = L;
        off += (L + 63) / 64 * 64;  // 256-B aligned call slots
      } catch (const sg::SgError& e) {
        cp.restore(B);
        sg::restore_soundgen_tail(B, first_syl);
        B.call_status[c] = e.code;
        B.call_msg[c] = e.what();
        B.call_off[c] = off;
        B.call_len[c] = 0;
      }
    }
    B.total_out = off;
    {
      sg::ProfScope ps(sg::PF_FINALIZE);
      sg::finalize_plan(B);
    }
    {
      sg::ProfScope ps(sg::PF_SPEC);
      sg::finalize_spec(B);
    }
    if (sg::g_prof_on) {
      static const char* names[] = {"harmonics", "rolloff", "contour", "envelope", "noise", "filter", "finalize", "finalize_spec"};
      for (int i = 0; i < sg::PF_N; ++i)
        std::fprintf(stderr, "sg_plan_prof %-14s %.3f s\n", names[i], sg::g_prof_ns[i].exchange(0) * 1e-9);
    }
    *out = P.release();
    return SG_OK;
  });
}

void sg_plan_destroy(sg_plan* plan) {
  if (!plan) return;
  sg::device_free(plan->D);
  delete plan;
}

int64_t sg_plan_n_calls(const sg_plan* plan) { return plan ? (int64_t)plan->B.call_len.size() : 0; }
int64_t sg_plan_total_samples(const sg_plan* plan) { return plan ? plan->B.total_out : 0; }

int sg_plan_lengths(const sg_plan* plan, int64_t* out_len, int64_t* out_off) {
  if (!plan) return SG_E_ARG;
  const size_t n = plan->B.call_len.size();
  if (out_len) std::memcpy(out_len, plan->B.call_len.data(), n * sizeof(int64_t));
  if (out_off) std::memcpy(out_off, plan->B.call_off.data(), n * sizeof(int64_t));
  return SG_OK;
}

int sg_plan_status(const sg_plan* plan, int32_t* out_status) {
  if (!plan) return SG_E_ARG;
  std::memcpy(out_status, plan->B.call_status.data(), plan->B.call_status.size() * sizeof(int32_t));
  return SG_OK;
}

const char* sg_plan_call_message(const sg_plan* plan, int64_t i) {
  if (!plan || i < 0 || i >= (int64_t)plan->B.call_msg.size()) return "";
  return plan->B.call_msg[i].c_str();
}

int64_t sg_plan_device_bytes(const sg_plan* plan) { return plan ? sg::device_bytes(plan->B) : 0; }

int sg_plan_upload(sg_ctx* ctx, sg_plan* plan) {
  return guarded(ctx, [&]() {
    HIPCHK(hipSetDevice(ctx->device));
    sg::device_upload(plan->B, plan->D, ctx->stream);
    return SG_OK;
  });
}

int sg_execute(sg_ctx* ctx, sg_plan* plan, float* d_out, void* stream) {
  return guarded(ctx, [&]() {
    HIPCHK(hipSetDevice(ctx->device));
    if (!plan->D.uploaded) throw sg::SgError(SG_E_ARG, "sg_execute: plan not uploaded");
    // NULL is the null (default) stream, as for every HIP API: the kernels are
    // ordered after earlier null-stream work (e.g. torch's default stream)
    hipStream_t s = (hipStream_t)stream;
    sg::device_execute(plan->B, plan->D, d_out, s, ctx->aux, ctx->profiling ? &ctx->prof_events : nullptr);
    return SG_OK;
  });
}

int sg_set_profiling(sg_ctx* ctx, int on) {
  ctx->profiling = on != 0;
  return SG_OK;
}

// Average duration (ms) of one profiled kernel (SG_PROF_*) over the executes
// recorded since profiling was enabled (events are on the launch stream). Reading
// a kernel consumes its events; the others stay until read or destroyed.
int sg_profile_read_kernel(sg_ctx* ctx, int kernel, double* ms_avg, int64_t* n) {
  return guarded(ctx, [&]() {
    if (kernel != SG_PROF_SINE_BANK && kernel != SG_PROF_STFT_OLA)
      throw sg::SgError(SG_E_ARG, "sg_profile_read_kernel: unknown kernel id");
    double tot = 0;
    int64_t cnt = 0;
    std::vector<sg::SgProfEvent> keep;
    for (auto& ev : ctx->prof_events) {
      if (ev.kernel != kernel) {
        keep.push_back(ev);
        continue;
      }
      HIPCHK(hipEventSynchronize(ev.e1));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, ev.e0, ev.e1));
      tot += ms;
      ++cnt;
      (void)hipEventDestroy(ev.e0);
      (void)hipEventDestroy(ev.e1);
    }
    ctx->prof_events.swap(keep);
    *ms_avg = cnt ? tot / cnt : 0;
    *n = cnt;
    return SG_OK;
  });
}

int sg_profile_read(sg_ctx* ctx, double* sine_ms_avg, int64_t* n) {
  return sg_profile_read_kernel(ctx, SG_PROF_SINE_BANK, sine_ms_avg, n);
}

int sg_plan_kernel_stats(const sg_plan* plan, int64_t* harm_samples, int64_t* harm_terms, int64_t* harm_amp_bytes,
                         int64_t* fft_frames) {
  if (!plan) return SG_E_ARG;
  *harm_samples = plan->B.harm_samples;
  *harm_terms = plan->B.harm_terms;
  *harm_amp_bytes = plan->B.harm_amp_bytes;
  *fft_frames = plan->B.fft_frames;
  return SG_OK;
}

int sg_plan_stft_stats(const sg_plan* plan, int64_t* samples, int64_t* alg_bytes, double* flops) {
  if (!plan) return SG_E_ARG;
  *samples = plan->B.stft_samples;
  *alg_bytes = plan->B.stft_bytes;
  *flops = plan->B.stft_flops;
  return SG_OK;
}

int sg_synchronize(sg_ctx* ctx) {
  return guarded(ctx, [&]() {
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipStreamSynchronize(nullptr));  // sg_execute(..., NULL) work
    return SG_OK;
  });
}

int sg_execute_to_host(sg_ctx* ctx, sg_plan* plan, double* out_host) {
  return guarded(ctx, [&]() {
    HIPCHK(hipSetDevice(ctx->device));
    if (!plan->D.uploaded) sg::device_upload(plan->B, plan->D, ctx->stream);
    const int64_t T = plan->B.total_out;
    float* d_out = nullptr;
    HIPCHK(hipMalloc(&d_out, (size_t)std::max<int64_t>(T, 1) * sizeof(float)));
    std::unique_ptr<void, hipError_t (*)(void*)> hold_out(d_out, hipFree);
    sg::device_execute(plan->B, plan->D, d_out, ctx->stream, ctx->aux, nullptr);
    std::vector<float> h((size_t)T);
    if (T) HIPCHK(hipMemcpyAsync(h.data(), d_out, (size_t)T * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (size_t c = 0; c < plan->B.call_len.size(); ++c)
      for (int64_t i = 0; i < plan->B.call_len[c]; ++i)
        out_host[plan->B.call_off[c] + i] = h[plan->B.call_off[c] + i];
    return SG_OK;
  });
}

// ---- synchronous single-call helpers --------------------------------------
static int run_single(sg_ctx* ctx, const sg_call_desc& d, double* out, int64_t cap, int64_t* out_len) {
  sg_plan* plan = nullptr;
  int rc = sg_plan_batch(ctx, &d, 1, &plan);
  if (rc) return rc;
  std::unique_ptr<sg_plan, void (*)(sg_plan*)> hold(plan, sg_plan_destroy);
  if (plan->B.call_status[0]) return set_err(ctx, plan->B.call_status[0], plan->B.call_msg[0]);
  const int64_t L = plan->B.call_len[0];
  *out_len = L;
  if (L > cap) return set_err(ctx, SG_E_CAPACITY, "output buffer too small");
  return sg_execute_to_host(ctx, plan, out);  // single call: offset 0
}

int sg_generate_harmonics(sg_ctx* ctx, const double* pitch, int64_t len, const sg_harm_params* p,
                          sg_anchors amplAnchors, const sg_random* rnd, double* out, int64_t cap,
                          int64_t* out_len) {
  sg_call_desc d{};
  d.kind = SG_CALL_HARMONICS;
  d.pitch = pitch;
  d.pitch_len = len;
  d.harm = p;
  d.amplAnchors = amplAnchors;
  if (rnd) d.random = *rnd;
  return run_single(ctx, d, out, cap, out_len);
}

int sg_soundgen(sg_ctx* ctx, const sg_soundgen_args* a, const sg_random* rnd, double* out, int64_t cap,
                int64_t* out_len) {
  sg_call_desc d{};
  d.kind = SG_CALL_SOUNDGEN;
  d.args = a;
  if (rnd) d.random = *rnd;
  return run_single(ctx, d, out, cap, out_len);
}

// ---- function-level spectral entries (single-item batches) -----------------
static int run_plan_to_host(sg_ctx* ctx, sg_plan* P, double* out, int64_t n) {
  P->B.call_len.assign(1, n);
  P->B.call_off.assign(1, 0);
  P->B.call_status.assign(1, 0);
  P->B.call_msg.assign(1, "");
  P->B.total_out = n;
  sg::finalize_plan(P->B);
  sg::finalize_spec(P->B);
  return sg_execute_to_host(ctx, P, out);
}

// Test hook (not part of the reference surface): the wavefront FFT stages of
// sg_stft_ola on nframes frames of M = wl / 2 complex points (interleaved re, im).
int sg_debug_wave_fft(sg_ctx* ctx, int32_t wl, int32_t inverse, int32_t nframes, const float* in, float* out) {
  return guarded(ctx, [&]() {
    sg::Batch B;
    const int gi = sg::geometry(B, wl);
    const SgFftGeom g = B.geoms[gi];
    if (g.kind != SG_FFT_WAVE) throw sg::SgError(SG_E_UNSUPPORTED, "window length not on the wavefront FFT path");
    const size_t nd = (size_t)nframes * g.M * 2;
    void *dg = nullptr, *dfl = nullptr, *dd = nullptr;
    HIPCHK(hipMalloc(&dg, sizeof(SgFftGeom)));
    HIPCHK(hipMalloc(&dfl, B.fl.size() * sizeof(float)));
    HIPCHK(hipMalloc(&dd, nd * sizeof(float)));
    HIPCHK(hipMemcpy(dg, &g, sizeof(SgFftGeom), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dfl, B.fl.data(), B.fl.size() * sizeof(float), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dd, in, nd * sizeof(float), hipMemcpyHostToDevice));
    sg::launch_fft_probe((const SgFftGeom*)dg, (const float*)dfl, (float*)dd, g.M, nframes, inverse, ctx->stream);
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(out, dd, nd * sizeof(float), hipMemcpyDeviceToHost));
    (void)hipFree(dg);
    (void)hipFree(dfl);
    (void)hipFree(dd);
    return SG_OK;
  });
}

int sg_formant_filter(sg_ctx* ctx, const double* sound, int64_t len, const double* env, int32_t env_nc,
                      int32_t windowLength_points, double overlap, double* out, int64_t cap, int64_t* out_len) {
  return guarded(ctx, [&]() {
    auto P = std::make_unique<sg_plan>();
    sg::Batch& B = P->B;
    const int wl = windowLength_points;
    if (len < wl) throw sg::SgError(SG_E_ARG, "formant filter: sound shorter than the window");
    const int64_t src = sg::fl_push(B, sound, len);
    const int64_t snd = sg::fs_alloc(B, len);
    B.copies.push_back(sg::Batch::Copy{src, snd, len});
    const sg::vec e(env, env + (int64_t)(wl / 2) * env_nc);
    int64_t Lf = 0, filt = 0;
    const int ola = sg::plan_filter(B, snd, len, wl, overlap, e, env_nc, &Lf, &filt);
    *out_len = Lf;
    if (Lf > cap) throw sg::SgError(SG_E_CAPACITY, "output buffer too small");
    SgNoiseItem it{};
    it.raw = filt;
    it.len = Lf;
    it.ola = ola;
    it.flags = SG_ITEM_FILTER_OLA;
    B.items.push_back(it);
    SgMix m{};
    m.len = Lf;
    m.nitems = 1;
    B.mixes[1].push_back(m);
    return run_plan_to_host(ctx, P.get(), out, Lf);
  });
}

int sg_generate_noise(sg_ctx* ctx, int64_t len, sg_anchors noiseAnchors, double rolloffNoise, double attackLen,
                      int32_t windowLength_points, double samplingRate, double overlap, double throwaway,
                      const double* filterNoise, int32_t filter_nc, const sg_random* rnd, double* out) {
  (void)throwaway;
  return guarded(ctx, [&]() {
    auto P = std::make_unique<sg_plan>();
    sg::Batch& B = P->B;
    sg::Rng R;
    R.s = rnd;
    SgNoiseItem it{};
    SgMix m{};
    m.len = len;
    if (sg::plan_noise(B, R, len, noiseAnchors, rolloffNoise, attackLen, windowLength_points, samplingRate, overlap,
                       filterNoise, filter_nc, &it)) {
      B.items.push_back(it);
      m.nitems = 1;
    }
    B.mixes[1].push_back(m);
    return run_plan_to_host(ctx, P.get(), out, len);
  });
}

int sg_spectral_envelope(sg_ctx* ctx, int32_t nr, int32_t nc, const sg_formants* formants, double formantDep,
                         double rolloffLip, sg_anchors mouthAnchors, double mouthOpenThres, double openMouthBoost,
                         double vocalTract, double temperature, double formDrift, double formDisp,
                         double formantDepStoch, double smoothLinearFactor, double samplingRate, double speedSound,
                         const sg_random* rnd, double* out) {
  return guarded(ctx, [&]() {
    sg::Rng R;
    R.s = rnd;
    const sg::vec e = sg::spectral_envelope(R, nr, nc, formants, formantDep, rolloffLip, mouthAnchors, mouthOpenThres,
                                            openMouthBoost, vocalTract, temperature, formDrift, formDisp,
                                            formantDepStoch, smoothLinearFactor, samplingRate, speedSound);
    std::memcpy(out, e.data(), e.size() * sizeof(double));
    return SG_OK;
  });
}

int sg_get_rolloff(const double* pitch_per_gc, int32_t n_gc, int32_t nHarmonics, double rolloff, double rolloffOct,
                   double rolloffParab, double rolloffParabHarm, double rolloffKHz, double baseline,
                   double throwaway, double samplingRate, double* out, int32_t* out_rows) {
  return guarded(nullptr, [&]() {
    sg::vec p(pitch_per_gc, pitch_per_gc + n_gc);
    int64_t H = 0;
    sg::vec r = sg::get_rolloff(p, nHarmonics, sg::vec(n_gc, rolloff), sg::vec(n_gc, rolloffOct), rolloffParab,
                                rolloffParabHarm, sg::vec(n_gc, rolloffKHz), baseline, throwaway, samplingRate, H);
    std::memcpy(out, r.data(), r.size() * sizeof(double));
    *out_rows = (int32_t)H;
    return SG_OK;
  });
}

}  // extern "C"
