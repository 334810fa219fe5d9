// sg_api.cpp — C-ABI of libsoundgen_hip.so: context, batch plan/upload/
// execute, and the synchronous function-level entries mirroring the R API.
// No C++ exception crosses this boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <cstring>
#include <exception>
#include <memory>
#include <thread>
#include <string>
#include <vector>

#include "sg_plan.h"
#include "sg_exec.h"
#include "sg_amp.h"
#include "sg_prof.h"
#include "sg_mel.h"

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
  bool host_released = false;  // sg_plan_release_host: bulk host arrays freed, re-upload impossible
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
  size_t segs, epochs, knots, ampsrc, ampcols, ampjobs, tasks, pieces, syls, syl_tiles, cknots, fl, items;
  size_t frames[2], olas[2], mixes[2], copies, eterms, ecols, envjobs, frames64, ugath;
  int64_t amp_total, w_total, harm_samples, harm_terms, harm_amp_bytes, fft_frames, fs_total, fe_total, w64_total, fh_total,
      hp_bouts, hp_noise_bouts, fu_total;
  double fft_flops;
  explicit Checkpoint(const sg::Batch& B)
      : segs(B.segs.size()), epochs(B.epochs.size()), knots(B.knots.size()), ampsrc(B.ampsrc.size()),
        ampcols(B.ampcols.size()), ampjobs(B.ampjobs.size()),
        tasks(B.tasks.size()), pieces(B.pieces.size()), syls(B.syls.size()), syl_tiles(B.syl_tiles.size()),
        cknots(B.cknots.size()), fl(B.fl.size()), items(B.items.size()), copies(B.copies.size()),
        eterms(B.eterms.size()), ecols(B.ecols.size()), envjobs(B.envjobs.size()), amp_total(B.amp_total), w_total(B.w_total),
        harm_samples(B.harm_samples), harm_terms(B.harm_terms), harm_amp_bytes(B.harm_amp_bytes),
        fft_frames(B.fft_frames), fs_total(B.fs_total), fe_total(B.fe_total), w64_total(B.w64_total),
        fh_total(B.fh_total), hp_bouts(B.hp_bouts), hp_noise_bouts(B.hp_noise_bouts), fft_flops(B.fft_flops) {
    frames64 = B.frames64.size();
    ugath = B.ugath.size();
    fu_total = B.fu_total;
    for (int p = 0; p < 2; ++p) { frames[p] = B.frames[p].size(); olas[p] = B.olas[p].size(); mixes[p] = B.mixes[p].size(); }
  }
  void restore(sg::Batch& B) const {
    B.segs.resize(segs); B.epochs.resize(epochs); B.knots.resize(knots); B.ampsrc.resize(ampsrc);
    B.ampcols.resize(ampcols); B.ampjobs.resize(ampjobs); B.amp_total = amp_total;
    B.tasks.resize(tasks); B.pieces.resize(pieces); B.syls.resize(syls); B.syl_tiles.resize(syl_tiles);
    B.cknots.resize(cknots); B.fl.resize(fl); B.items.resize(items); B.copies.resize(copies);
    for (int p = 0; p < 2; ++p) {
      B.frames[p].resize(frames[p]); B.frame_geom[p].resize(frames[p]);
      B.olas[p].resize(olas[p]); B.mixes[p].resize(mixes[p]);
    }
    B.w_total = w_total; B.harm_samples = harm_samples; B.harm_terms = harm_terms;
    B.harm_amp_bytes = harm_amp_bytes; B.fft_frames = fft_frames; B.fs_total = fs_total;
    B.eterms.resize(eterms); B.ecols.resize(ecols); B.envjobs.resize(envjobs); B.fe_total = fe_total;
    B.frames64.resize(frames64); B.w64_total = w64_total; B.fh_total = fh_total; B.hp_bouts = hp_bouts;
    B.hp_noise_bouts = hp_noise_bouts;
    B.ugath.resize(ugath);
    B.fu_total = fu_total;
    B.fft_flops = fft_flops;
  }
};

// Plan calls [c0, c1) into B (empty), output slots from offset 0.
// Bulk-array elements per call over the calls planned so far in this process
// (g_growth): a part reserves its arrays up front (x1.25 of the running mean;
// reserve it never touches is never faulted in) instead of growing them by
// doubling, whose relocation copies and fresh-page faults were ~20 % of
// planning time. Only the first parts planned in a process grow.
struct GrowthEstimate {
  static constexpr int N = 17;
  std::atomic<int64_t> calls{0};
  std::atomic<int64_t> elems[N];
  GrowthEstimate() {
    for (auto& e : elems) e.store(0);
  }
  // one sample per part: keep the estimate a running mean over recent plans
  // (concurrent sg_plan_batch calls: the CAS lets one of them halve a given
  // count; each element is halved atomically)
  void decay() {
    int64_t c = calls.load();
    if (c < (int64_t(1) << 20)) return;
    if (!calls.compare_exchange_strong(c, c / 2)) return;  // another plan is decaying it
    for (auto& e : elems) {
      int64_t v = e.load();
      while (!e.compare_exchange_weak(v, v / 2)) {
      }
    }
  }
  template <class F>
  static void each(sg::Batch& B, F&& f) {
    f(0, B.segs); f(1, B.epochs); f(2, B.knots); f(3, B.ampsrc); f(4, B.tasks);
    f(5, B.pieces); f(6, B.syl_tiles); f(7, B.fl); f(8, B.cknots); f(9, B.eterms);
    f(10, B.frames[0]); f(11, B.frames[1]); f(12, B.frame_geom[0]); f(13, B.frame_geom[1]); f(14, B.syls);
    f(15, B.ecols); f(16, B.ampcols);
  }
  void reserve(sg::Batch& B, int64_t n_calls) const {
    const int64_t c = calls.load();
    if (c <= 0) return;
    each(B, [&](int i, auto& v) {
      v.reserve((size_t)(1.25 * (double)elems[i].load() / (double)c * (double)n_calls) + 256);
    });
  }
  void record(sg::Batch& B, int64_t n_calls) {
    each(B, [&](int i, auto& v) { elems[i] += (int64_t)v.size(); });
    calls += n_calls;
  }
};

GrowthEstimate g_growth;

// stream_stop: the calls' draw callbacks are one sequential stream (R's RNG), so a
// failing call ends the planning of later callback calls; false when every call's
// callbacks replay its own recorded draws (sg_node's second pass)
void plan_range(sg::Batch& B, const sg_call_desc* calls, int64_t c0, int64_t c1, bool stream_stop = true,
                const std::function<void(int64_t)>* on_done = nullptr) {
  const int64_t n = c1 - c0;
  B.call_len.assign(n, 0);
  B.call_off.assign(n, 0);
  B.call_status.assign(n, 0);
  B.call_fp64.assign(n, 0);
  B.call_rho.assign(n, 0.0);
  B.call_rho_noise.assign(n, 0.0);
  B.call_rows.assign(n, 0.0);
  B.call_flops.assign(n, 0.0);
  B.call_msg.assign(n, "");
  int64_t off = 0;
  // A call drawing from callbacks (R's RNG through the shim) that fails ends the
  // callback stream there: lapply(calls, soundgen) stops at that call's stop(),
  // so no later call may consume draws (.Random.seed stays where R leaves it).
  // Callback batches plan in one range on the calling thread (sg_plan_batch).
  int64_t cb_failed = -1;
  for (int64_t i = 0; i < n; ++i) {
    const sg_call_desc& d = calls[c0 + i];
    const bool cb = d.random.norm_cb || d.random.unif_cb || d.random.gamma_cb;
    if (cb && stream_stop && cb_failed >= 0) {
      B.call_status[i] = SG_E_ARG;
      B.call_msg[i] = "not planned: call " + std::to_string(c0 + cb_failed + 1) +
                      " of the batch failed first (the RNG callback stream stops there)";
      B.call_off[i] = off;
      B.call_len[i] = 0;
      continue;
    }
    Checkpoint cp(B);
    const int first_syl = (int)B.syls.size();
    const int64_t hp0 = B.hp_bouts, rows0 = B.harm_terms;
    const double fl0 = B.fft_flops;
    B.rho_cur = 0;
    B.rho_noise_cur = 0;
    try {
      sg::Rng R;
      R.s = &d.random;
      int64_t L = 0;
      if (d.kind == SG_CALL_HARMONICS) {
        if (!d.pitch || !d.harm) throw sg::SgError(SG_E_ARG, "harmonics call without pitch/params");
        L = sg::plan_harmonics(B, d.pitch, d.pitch_len, *d.harm, d.amplAnchors, R, off, B.draws_only);
        sg::ProfScope pt(sg::PF_TILES);
        if (!B.draws_only) sg::tile_syllables(B, first_syl);
      } else if (d.kind == SG_CALL_SOUNDGEN) {
        if (!d.args) throw sg::SgError(SG_E_ARG, "soundgen call without args");
        {
          sg::ProfScope pg(sg::PF_SOUNDGEN);
          L = sg::plan_soundgen(B, *d.args, R, off, first_syl);
        }
        sg::ProfScope pt(sg::PF_TILES);
        if (!B.draws_only) sg::tile_syllables(B, first_syl);
      } else {
        throw sg::SgError(SG_E_ARG, "unknown call kind");
      }
      B.call_off[i] = off;
      B.call_len[i] = L;
      B.call_fp64[i] = (int32_t)(B.hp_bouts - hp0);
      B.call_rho[i] = B.rho_cur;
      B.call_rho_noise[i] = B.rho_noise_cur;
      B.call_rows[i] = (double)(B.harm_terms - rows0);
      B.call_flops[i] = B.fft_flops - fl0;
      off += (L + 63) / 64 * 64;  // 256-B aligned call slots
    } catch (const sg::SgError& e) {
      cp.restore(B);
      sg::restore_soundgen_tail(B, first_syl);
      B.call_status[i] = e.code;
      B.call_msg[i] = e.what();
      B.call_off[i] = off;
      B.call_len[i] = 0;
      if (cb && cb_failed < 0) cb_failed = i;
    }
    if (on_done) (*on_done)(c0 + i);
  }
  B.total_out = off;
}

// Host threads for planning: SG_PLAN_THREADS, else the hardware threads capped
// at 16 (a GPU box's CPU share); one thread for small batches.
int plan_threads(int64_t n_calls) {
  int t = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
  if (const char* e = std::getenv("SG_PLAN_THREADS")) t = std::max(1, std::atoi(e));
  return (int)std::min<int64_t>(t, std::max<int64_t>(1, n_calls / 4));
}

// Where one part's arrays land in the merged batch.
struct PartBase {
  int64_t out, fs, fl, w, amp, asrc, acol, ajob, knot, ck, task, seg, syl, piece, st, item, copy, call, epoch, fe, term,
      col, job;
  int64_t w64, fh, fr64, fu, ug;
  int64_t fr[2], ola[2], mix[2];
};

// Concatenate per-chunk batches in call order, rebasing every cross-reference
// (scratch, arena and output offsets, table indices). Bases are prefix sums
// of the parts' sizes; geometries are matched by window length (a new one
// keeps its tables, which move with the part's fl). The parts are rebased and
// copied in parallel, each freed once copied.
void merge_parts(sg::Batch& D, std::vector<sg::Batch>& parts, int threads) {
  const size_t np = parts.size();
  std::vector<PartBase> base(np);
  std::vector<std::vector<int32_t>> gmap(np);
  PartBase c{};
  for (size_t k = 0; k < np; ++k) {
    sg::Batch& S = parts[k];
    base[k] = c;
    gmap[k].resize(S.geoms.size());
    for (size_t g = 0; g < S.geoms.size(); ++g) {
      int32_t j = 0;
      while (j < (int32_t)D.geoms.size() && D.geoms[j].wl != S.geoms[g].wl) ++j;
      if (j == (int32_t)D.geoms.size()) {
        SgFftGeom G = S.geoms[g];
        G.tw += c.fl; G.tws += c.fl; G.win += c.fl;
        for (SgCdft& cd : G.cd) {  // sub-geometries precede their users in the part
          if (cd.n == 0) continue;
          cd.geom = gmap[k][cd.geom];
          cd.chirp += c.fl; cd.bf += c.fl;
        }
        D.geoms.push_back(G);
      }
      gmap[k][g] = j;
    }
    c.out += S.total_out; c.fs += S.fs_total; c.fl += (int64_t)S.fl.size();
    c.w = (c.w + S.w_total + 3) / 4 * 4;  // keeps the parts' 16-B alignment of epoch waveforms
    c.amp += S.amp_total; c.asrc += (int64_t)S.ampsrc.size(); c.acol += (int64_t)S.ampcols.size();
    c.ajob += (int64_t)S.ampjobs.size();
    D.amp_lg_rows = std::max(D.amp_lg_rows, S.amp_lg_rows);
    c.knot += (int64_t)S.knots.size(); c.ck += (int64_t)S.cknots.size();
    c.task += (int64_t)S.tasks.size(); c.seg += (int64_t)S.segs.size(); c.syl += (int64_t)S.syls.size();
    c.piece += (int64_t)S.pieces.size(); c.st += (int64_t)S.syl_tiles.size(); c.item += (int64_t)S.items.size();
    c.copy += (int64_t)S.copies.size(); c.call += (int64_t)S.call_len.size(); c.epoch += (int64_t)S.epochs.size();
    c.fe += S.fe_total; c.term += (int64_t)S.eterms.size(); c.col += (int64_t)S.ecols.size();
    c.job += (int64_t)S.envjobs.size();
    c.w64 += S.w64_total; c.fh += S.fh_total; c.fr64 += (int64_t)S.frames64.size();
    c.fu += S.fu_total; c.ug += (int64_t)S.ugath.size();
    D.hp_bouts += S.hp_bouts;
    D.hp_noise_bouts += S.hp_noise_bouts;
    for (int ph = 0; ph < 2; ++ph) {
      c.fr[ph] += (int64_t)S.frames[ph].size(); c.ola[ph] += (int64_t)S.olas[ph].size();
      c.mix[ph] += (int64_t)S.mixes[ph].size();
    }
    D.harm_samples += S.harm_samples; D.harm_terms += S.harm_terms; D.harm_amp_bytes += S.harm_amp_bytes;
    D.fft_frames += S.fft_frames;
    D.fft_flops += S.fft_flops;
  }
  D.total_out = c.out; D.fs_total = c.fs; D.w_total = c.w; D.fe_total = c.fe;
  D.w64_total = c.w64; D.fh_total = c.fh; D.frames64.resize(c.fr64);
  D.fu_total = c.fu; D.ugath.resize(c.ug);
  D.ecols.resize(c.col); D.envjobs.resize(c.job);
  D.call_len.resize(c.call); D.call_off.resize(c.call); D.call_status.resize(c.call); D.call_msg.resize(c.call);
  D.call_fp64.resize(c.call); D.call_rho.resize(c.call); D.call_rho_noise.resize(c.call); D.call_rows.resize(c.call); D.call_flops.resize(c.call);
  D.epochs.resize(c.epoch); D.knots.resize(c.knot); D.pieces.resize(c.piece);
  D.amp_total = c.amp; D.ampsrc.resize(c.asrc); D.ampcols.resize(c.acol); D.ampjobs.resize(c.ajob); D.syls.resize(c.syl); D.syl_tiles.resize(c.st);
  D.cknots.resize(c.ck); D.items.resize(c.item);
  // the largest arrays stay in the parts' blocks (moved below, not copied)
  auto blocks = [&](auto& x, int64_t n) {
    x.blocks.resize(np);
    x.base.resize(np);
    x.n = n;
  };
  blocks(D.segs_x, c.seg); blocks(D.tasks_x, c.task); blocks(D.fl_x, c.fl);
  blocks(D.eterms_x, c.term); D.copies.resize(c.copy);
  for (int ph = 0; ph < 2; ++ph) {
    D.frames[ph].resize(c.fr[ph]); D.frame_geom[ph].resize(c.fr[ph]);
    D.olas[ph].resize(c.ola[ph]); D.mixes[ph].resize(c.mix[ph]);
  }
  auto put = [](auto& dst, auto& src, int64_t at) { std::copy(src.begin(), src.end(), dst.begin() + at); };
  auto one = [&](size_t k) {
    sg::Batch& S = parts[k];
    const PartBase& b = base[k];
    auto ck = [&](SgContour& x) { if (x.kind == 3) x.k_off += b.ck; };
    for (size_t i = 0; i < S.call_len.size(); ++i) {
      D.call_len[b.call + i] = S.call_len[i];
      D.call_off[b.call + i] = S.call_off[i] + b.out;
      D.call_status[b.call + i] = S.call_status[i];
      D.call_fp64[b.call + i] = S.call_fp64[i];
      D.call_rho[b.call + i] = S.call_rho[i];
      D.call_rho_noise[b.call + i] = S.call_rho_noise[i];
      D.call_rows[b.call + i] = S.call_rows[i];
      D.call_flops[b.call + i] = S.call_flops[i];
      D.call_msg[b.call + i] = std::move(S.call_msg[i]);
    }
    for (auto& e : S.epochs) {
      e.w_off += b.w; e.amp_off += b.amp; e.knot_off += b.knot;
      e.seg_off += (int32_t)b.seg; e.syl += (int32_t)b.syl;
    }
    for (auto& t : S.tasks) {
      t.w_off += (t.flags & SG_TASK_HP) ? b.w64 : b.w;
      t.a_off += b.amp; t.d_off += b.amp; t.syl += (int32_t)b.syl;
    }
    for (auto& s : S.syls)  // a syllable's pieces read W, or W64 for an fp64 syllable
      for (int32_t pi = s.piece0; pi < s.piece0 + s.npiece; ++pi) {
        SgPiece& p = S.pieces[pi];
        for (int q = 0; q < (p.nterms < 0 ? 1 : p.nterms); ++q) p.t[q].src += s.hp ? b.w64 : b.w;
      }
    for (auto& s : S.syls) {
      s.out_off += s.hp ? b.fh : (s.dst_fs ? b.fs : b.out);
      s.piece0 += (int32_t)b.piece; s.max_slot += (int32_t)b.syl; s.task0 += b.task;
      ck(s.env);
      ck(s.genv);
      if (s.drift.nk > 0) s.drift.k_off += b.ck;
    }
    for (auto& t : S.syl_tiles) {
      t.syl += (int32_t)b.syl; t.piece += (int32_t)b.piece;
      for (int w = 0; w < 4; ++w) t.wpiece[w] += (int32_t)b.piece;
    }
    for (int ph = 0; ph < 2; ++ph) {
      for (auto& f : S.frames[ph]) {
        // noise: uniforms in fl, or gathered (uniform area, encoded); filter: the sound in fs
        f.src = ph == 1 ? f.src + b.fs : (f.src < 0 ? f.src - b.fu : f.src + b.fl);
        f.env = f.env < 0 ? f.env - b.fe : f.env + b.fl;  // envelope area (encoded) or fl
        if (f.dst >= 0) f.dst += b.fs;
      }
      for (auto& g : S.frame_geom[ph]) g = gmap[k][g];
      for (auto& o : S.olas[ph]) {
        if (o.fidx >= 0) o.fidx += (int32_t)b.fr[ph];
        if (!o.fused) o.frames += b.fs;
        o.out += b.fs;
      }
      for (auto& m : S.mixes[ph]) {
        m.dst += m.to_fs == 2 ? b.fh : (m.to_fs ? b.fs : b.out);
        if (m.base_kind != SG_BASE_NONE) m.base += b.fs;
        if (m.base_kind == SG_BASE_NORM) m.base_ola += (int32_t)b.ola[1];
        m.item0 += (int32_t)b.item;
        if (m.am_lo > 0) m.am_tab += b.fl;
        ck(m.mult);
      }
    }
    for (auto& f : S.frames64) {
      // uniforms (fl, or the uniform area encoded) / pre-filter sound (fh)
      f.src = f.mode == SG_F64_NOISE ? (f.src < 0 ? f.src - b.fu : f.src + b.fl) : f.src + b.fh;
      f.env = f.env < 0 ? f.env - b.fe : f.env + b.fl;
      f.dst += b.fs;
    }
    for (auto& it : S.items) {
      it.raw += (it.flags & SG_ITEM_F64) ? b.fh : b.fs;
      if (it.flags & SG_ITEM_FILTER_OLA) it.ola += (int32_t)b.ola[1];
      else if (it.ola >= 0) it.ola += (int32_t)b.ola[0];
      ck(it.strength);
    }
    for (auto& x : S.copies) { x.fl_off += b.fl; x.fs_off += b.fs; }
    for (auto& j : S.envjobs) { j.out += b.fe; j.term0 += b.term; j.col0 += b.col; }
    for (auto& g : S.ugath) g.dst += b.fu;
    put(D.ugath, S.ugath, b.ug);
    auto move = [&](auto& x, auto& v, int64_t at) {
      x.blocks[k] = std::move(v);
      x.base[k] = at;
    };
    for (auto& j : S.ampjobs) {
      j.amp_off += b.amp;
      if (j.src_off >= 0) j.src_off += b.asrc;
      if (j.col0 >= 0) j.col0 += b.acol;
    }
    put(D.ampsrc, S.ampsrc, b.asrc); put(D.ampcols, S.ampcols, b.acol); put(D.ampjobs, S.ampjobs, b.ajob);
    move(D.eterms_x, S.eterms, b.term); move(D.segs_x, S.segs, b.seg);
    move(D.tasks_x, S.tasks, b.task); move(D.fl_x, S.fl, b.fl);
    put(D.ecols, S.ecols, b.col); put(D.envjobs, S.envjobs, b.job);
    put(D.epochs, S.epochs, b.epoch); put(D.knots, S.knots, b.knot); put(D.pieces, S.pieces, b.piece);
    put(D.syls, S.syls, b.syl); put(D.syl_tiles, S.syl_tiles, b.st); put(D.cknots, S.cknots, b.ck);
    put(D.items, S.items, b.item); put(D.copies, S.copies, b.copy);
    put(D.frames64, S.frames64, b.fr64);
    for (int ph = 0; ph < 2; ++ph) {
      put(D.frames[ph], S.frames[ph], b.fr[ph]); put(D.frame_geom[ph], S.frame_geom[ph], b.fr[ph]);
      put(D.olas[ph], S.olas[ph], b.ola[ph]); put(D.mixes[ph], S.mixes[ph], b.mix[ph]);
    }
  };
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < np;) one(k);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  // the parts (as large as the merged batch) are unmapped on a detached thread:
  // freeing them inside the copy loop serialised the merge threads' page faults
  auto* dead = new std::vector<sg::Batch>(std::move(parts));
  try {
    std::thread([dead]() { delete dead; }).detach();
  } catch (...) {
    delete dead;
  }
}
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
  int prev = -1;  // the caller's current device, restored afterwards
  const bool had = hipGetDevice(&prev) == hipSuccess;
  (void)hipSetDevice(ctx->device);
  for (auto& ev : ctx->prof_events) { (void)hipEventDestroy(ev.e0); (void)hipEventDestroy(ev.e1); }
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  delete ctx;
  if (had && prev >= 0) (void)hipSetDevice(prev);
}

const char* sg_last_error(const sg_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

int sg_plan_batch(sg_ctx* ctx, const sg_call_desc* calls, int64_t n_calls, sg_plan** out) {
  return sg::plan_batch_ex(ctx, calls, n_calls, false, out);
}
}  // extern "C"

namespace sg {
// The draws of every call in call order (one stream: a failing call ends it, as in
// plan_range), emitting nothing: Batch::draws_only. Per call status and message.
void record_draws(const sg_call_desc* calls, int64_t n_calls, std::vector<int32_t>& status,
                  std::vector<std::string>& msg, const std::function<void(int64_t, int32_t)>& on_call) {
  Batch B;
  B.draws_only = true;
  const std::function<void(int64_t)> done = [&](int64_t i) {
    if (on_call) on_call(i, B.call_status[(size_t)i]);
  };
  plan_range(B, calls, 0, n_calls, true, &done);
  if (sg::g_prof_on) {
    static const char* names[] = {"harmonics", "rolloff", "contour", "envelope", "noise", "filter", "finalize",
                                  "finalize_spec", "fry", "crossfade", "emit", "tasks", "tiles", "soundgen", "env_upsample", "env_stochastic", "env_terms"};
    for (int i = 0; i < sg::PF_N; ++i)
      std::fprintf(stderr, "sg_plan_prof record %-14s %.3f s\n", names[i], sg::g_prof_ns[i].exchange(0) * 1e-9);
  }
  status = std::move(B.call_status);
  msg = std::move(B.call_msg);
}

int plan_batch_ex(sg_ctx* ctx, const sg_call_desc* calls, int64_t n_calls, bool independent_draws, sg_plan** out,
                  int max_threads) {
  return guarded(ctx, [&]() {
    auto P = std::make_unique<sg_plan>();
    sg::Batch& B = P->B;
    // Calls are independent and each reads its own injected draws, so chunks of
    // calls are planned on host threads into private batches and concatenated in
    // call order (the result equals serial planning). Draw callbacks (R's RNG
    // through the shim, or one generator shared by the batch) are a single
    // sequential stream: such batches plan on the calling thread, unless every
    // call's callbacks replay its own recorded draws (independent_draws).
    bool callbacks = false;
    for (int64_t c = 0; c < n_calls && !callbacks; ++c)
      callbacks = calls[c].random.norm_cb || calls[c].random.unif_cb || calls[c].random.gamma_cb;
    const bool serial = callbacks && !independent_draws;
    const int threads = serial ? 1 : std::min(plan_threads(n_calls), max_threads > 0 ? max_threads : 1 << 30);
    g_growth.decay();
    if (threads <= 1) {
      g_growth.reserve(B, n_calls);
      plan_range(B, calls, 0, n_calls, !independent_draws);
      g_growth.record(B, n_calls);
    } else {
      constexpr int per_thread = 8;  // parts per thread (dynamic balance over uneven calls)
      const int64_t nchunk = std::min<int64_t>(n_calls, (int64_t)threads * per_thread);
      std::vector<sg::Batch> parts((size_t)nchunk);
      std::vector<std::exception_ptr> errs((size_t)nchunk);
      std::atomic<int64_t> next{0};
      auto work = [&]() {
        for (int64_t k; (k = next.fetch_add(1)) < nchunk;) {
          try {
            const int64_t c0 = k * n_calls / nchunk, c1 = (k + 1) * n_calls / nchunk;
            g_growth.reserve(parts[k], c1 - c0);
            plan_range(parts[k], calls, c0, c1, !independent_draws);
            g_growth.record(parts[k], c1 - c0);
          } catch (...) {
            errs[k] = std::current_exception();
          }
        }
      };
      const auto tp = std::chrono::steady_clock::now();
      std::vector<std::thread> pool;
      for (int t = 1; t < threads; ++t) pool.emplace_back(work);
      work();
      for (auto& t : pool) t.join();
      if (sg::g_prof_on)
        std::fprintf(stderr, "sg_plan_prof parts (%lld on %d threads) %.3f s\n", (long long)nchunk, threads,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - tp).count());
      for (auto& e : errs)
        if (e) std::rethrow_exception(e);
      const auto tm = std::chrono::steady_clock::now();
      merge_parts(B, parts, threads);
      if (sg::g_prof_on)
        std::fprintf(stderr, "sg_plan_prof merge (%d threads) %.3f s\n", threads,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - tm).count());
    }
    {
      sg::ProfScope ps(sg::PF_FINALIZE);
      sg::finalize_plan(B);
    }
    {
      sg::ProfScope ps(sg::PF_SPEC);
      sg::finalize_spec(B);
    }
    if (sg::g_prof_on) {
      static const char* names[] = {"harmonics", "rolloff", "contour", "envelope", "noise", "filter", "finalize",
                                    "finalize_spec", "fry", "crossfade", "emit", "tasks", "tiles", "soundgen", "env_upsample", "env_stochastic", "env_terms"};
      for (int i = 0; i < sg::PF_N; ++i)
        std::fprintf(stderr, "sg_plan_prof %-14s %.3f s\n", names[i], sg::g_prof_ns[i].exchange(0) * 1e-9);
      std::fprintf(stderr, "sg_plan_prof host MB: fl %.1f amps %.1f knots %.1f cknots %.1f tasks %.1f segs %.1f "
                   "frames %.1f pieces %.1f syl_tiles %.1f; scratch MB: fs %.1f w %.1f\n",
                   bulk_size(B.fl_x, B.fl) * 4e-6, B.amp_total * 4e-6, B.knots.size() * 8e-6,
                   B.cknots.size() * 8e-6, bulk_size(B.tasks_x, B.tasks) * sizeof(SgWTask) * 1e-6,
                   bulk_size(B.segs_x, B.segs) * sizeof(SgSeg) * 1e-6,
                   (B.frames[0].size() + B.frames[1].size()) * sizeof(SgFrame) * 1e-6,
                   B.pieces.size() * sizeof(SgPiece) * 1e-6, B.syl_tiles.size() * sizeof(SgSylTile) * 1e-6,
                   B.fs_total * 4e-6, B.w_total * 4e-6);
      std::fprintf(stderr, "sg_plan_prof fp64: filter bouts %lld, noise bouts %lld, frames %lld (noise %lld) of %lld\n",
                   (long long)B.hp_bouts, (long long)B.hp_noise_bouts, (long long)B.frames64.size(),
                   (long long)B.frames64_noise, (long long)(B.frames[0].size() + B.frames[1].size() + B.frames64.size()));
    }
    sg::scratch_trim();
    *out = P.release();
    return SG_OK;
  });
}
}  // namespace sg

extern "C" {

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

int64_t sg_plan_device_bytes(const sg_plan* plan) {
  if (!plan) return 0;
  return plan->host_released ? (int64_t)plan->D.arena_bytes : sg::device_bytes(plan->B);
}

int sg_plan_release_host(sg_plan* plan) {
  if (!plan) return SG_E_ARG;
  if (!plan->D.uploaded) return SG_E_ARG;
  sg::Batch& B = plan->B;
  auto drop = [](auto& v) { std::remove_reference_t<decltype(v)>().swap(v); };
  // The bulk arrays (~12 GB for a 16,384-call C5 plan) are returned to the OS on a
  // detached thread: unmapping them took ~1.2 s on the caller, which then plans
  // or uploads the next chunk meanwhile.
  struct Bulk {
    decltype(B.fl) fl;
    decltype(B.tasks) tasks;
    decltype(B.segs) segs;
    decltype(B.eterms) eterms;
    decltype(B.cknots) cknots;
    decltype(B.knots) knots;
    decltype(B.fl_x) fl_x;
    decltype(B.tasks_x) tasks_x;
    decltype(B.segs_x) segs_x;
    decltype(B.eterms_x) eterms_x;
  };
  auto* bulk = new Bulk{std::move(B.fl),     std::move(B.tasks),   std::move(B.segs), std::move(B.eterms),
                        std::move(B.cknots), std::move(B.knots),   std::move(B.fl_x), std::move(B.tasks_x),
                        std::move(B.segs_x), std::move(B.eterms_x)};
  B.fl_x = {}; B.tasks_x = {}; B.segs_x = {}; B.eterms_x = {};
  try {
    std::thread([bulk]() { delete bulk; }).detach();
  } catch (...) {
    delete bulk;  // no thread: free here
  }
  // what sg_execute reads from the host plan stays: slices, ranges and splits,
  // the table sizes it launches over, the copy list, the envelope area base
  drop(B.segs); drop(B.epochs); drop(B.knots); drop(B.ampsrc); drop(B.ampcols); drop(B.ampjobs); drop(B.tasks); drop(B.pieces); drop(B.syls);
  drop(B.syl_tiles); drop(B.fin_tiles); drop(B.copy_tiles); drop(B.ptiles); drop(B.cknots); drop(B.fl);
  drop(B.fgroups); drop(B.olasegs); drop(B.items); drop(B.mixes_dev); drop(B.eterms); drop(B.ecols); drop(B.envjobs);
  for (int ph = 0; ph < 2; ++ph) { drop(B.frames[ph]); drop(B.frame_geom[ph]); drop(B.olas[ph]); drop(B.mixes[ph]); }
  drop(B.ustream); drop(B.ujobs);
  plan->host_released = true;
  return SG_OK;
}

int sg_plan_upload(sg_ctx* ctx, sg_plan* plan) {
  return guarded(ctx, [&]() {
    if (plan->host_released) throw sg::SgError(SG_E_ARG, "sg_plan_upload: host arrays released");
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

int sg_execute_plans(sg_ctx* ctx, sg_plan* const* plans, float* const* d_outs, int n, void* stream) {
  return guarded(ctx, [&]() {
    HIPCHK(hipSetDevice(ctx->device));
    if (n < 0 || (n > 0 && (!plans || !d_outs))) throw sg::SgError(SG_E_ARG, "sg_execute_plans: bad plan list");
    std::vector<sg::PlanRun> runs;
    for (int i = 0; i < n; ++i) {
      if (!plans[i] || !plans[i]->D.uploaded) throw sg::SgError(SG_E_ARG, "sg_execute_plans: plan not uploaded");
      for (int j = 0; j < i; ++j)
        if (plans[j] == plans[i]) throw sg::SgError(SG_E_ARG, "sg_execute_plans: a plan listed twice");
      runs.push_back(sg::PlanRun{&plans[i]->B, &plans[i]->D, d_outs[i]});
    }
    if (runs.empty()) return SG_OK;
    sg::device_execute_many(runs, (hipStream_t)stream, ctx->aux, ctx->profiling ? &ctx->prof_events : nullptr);
    return SG_OK;
  });
}

int64_t sg_host_cache_trim(void) { return (int64_t)sg::bulk_trim(); }

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

int sg_plan_table_stats(const sg_plan* plan, int64_t* tables, int64_t* samples, int64_t* terms) {
  if (!plan || !tables || !samples || !terms) return SG_E_ARG;
  *tables = plan->D.uploaded ? (int64_t)plan->D.tabjobs_host.size() : 0;
  *samples = plan->D.uploaded ? plan->D.tab_samples : 0;
  *terms = plan->D.uploaded ? plan->D.tab_terms : 0;
  return SG_OK;
}

int sg_plan_stft_stats(const sg_plan* plan, int64_t* samples, int64_t* alg_bytes, double* flops) {
  if (!plan) return SG_E_ARG;
  *samples = plan->B.stft_samples;
  *alg_bytes = plan->B.stft_bytes;
  *flops = plan->B.stft_flops;
  return SG_OK;
}

int sg_plan_sine_tasks(const sg_plan* plan, int64_t* counts) {
  if (!plan || !counts) return SG_E_ARG;
  const sg::DevicePlan& D = plan->D;
  counts[0] = (int64_t)D.tlong_host.size();
  counts[1] = (int64_t)D.tshort_host.size();
  counts[2] = (int64_t)D.tall_host.size();
  counts[3] = (int64_t)D.tallp_host.size();
  counts[4] = (int64_t)D.thp_host.size();
  return SG_OK;
}

int64_t sg_plan_amp_count(const sg_plan* plan) { return plan && !plan->host_released ? plan->B.amp_total : 0; }

int sg_plan_debug_amps(const sg_plan* plan, float* out, int64_t n) {
  if (!plan || plan->host_released || !out || n < plan->B.amp_total) return SG_E_ARG;
  const sg::Batch& B = plan->B;
  std::vector<double> lg((size_t)B.amp_lg_rows + 1);
  for (size_t k = 0; k < lg.size(); ++k) lg[k] = std::log2((double)(k + 1));
  for (const SgAmpJob& J : B.ampjobs)  // sg_amp_build, one job after the other
    for (int32_t r = 0; r < J.Rp; ++r)
      for (int32_t g = 0; g < J.G; ++g) {
        float a;
        if (r >= J.R) a = 0.f;
        else if (J.src_off >= 0) a = B.ampsrc[J.src_off + (int64_t)g * J.Rp + r];
        else a = (float)sg::amp_value(B.ampcols.data() + J.col0, J, lg.data(), g, r);
        out[J.amp_off + (int64_t)g * J.Rp + r] = a;
      }
  return SG_OK;
}

int sg_plan_conditioning(const sg_plan* plan, double* rho) {
  if (!plan || !rho) return SG_E_ARG;
  const sg::Batch& B = plan->B;
  std::memcpy(rho, B.call_rho.data(), B.call_rho.size() * sizeof(double));
  return SG_OK;
}

int sg_plan_noise_conditioning(const sg_plan* plan, double* rho) {
  if (!plan || !rho) return SG_E_ARG;
  const sg::Batch& B = plan->B;
  std::memcpy(rho, B.call_rho_noise.data(), B.call_rho_noise.size() * sizeof(double));
  return SG_OK;
}

int sg_plan_precision(const sg_plan* plan, int32_t* call_fp64, int64_t* fp64_frames, int64_t* fp64_tasks) {
  if (!plan) return SG_E_ARG;
  const sg::Batch& B = plan->B;
  if (call_fp64) std::memcpy(call_fp64, B.call_fp64.data(), B.call_fp64.size() * sizeof(int32_t));
  if (fp64_frames) *fp64_frames = (int64_t)B.frames64.size();
  if (fp64_tasks) {
    int64_t n = 0;
    sg::bulk_each(B.tasks_x, B.tasks, [&](int64_t, const SgWTask* p, int64_t k) {
      for (int64_t i = 0; i < k; ++i) n += (p[i].flags & SG_TASK_HP) ? 1 : 0;
    });
    *fp64_tasks = n;
  }
  return SG_OK;
}

// dtw::dtw(x, y, distance.only = TRUE)$normalizedDistance with the package defaults:
// local distance |x_i - y_j| (Euclidean, 1-D), step pattern symmetric2
//   g(i, j) = min(g(i-1, j-1) + 2 d(i, j), g(i-1, j) + d(i, j), g(i, j-1) + d(i, j)),
// g(1, 1) = d(1, 1), normalised by n + m. Host code (compareSounds, R/matchPars.R:372-376).
int sg_mel_spec(sg_ctx* ctx, const double* wave, int64_t len, const sg_mel_params* p, double* out, int64_t cap,
                int32_t* nb, int32_t* nc) {
  return guarded(ctx, [&]() {
    if (!ctx || !p || !nb || !nc || len < 0 || (len > 0 && !wave)) throw sg::SgError(SG_E_ARG, "sg_mel_spec: bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    const sg::MelGeom g = sg::mel_geom(*p);
    if (len == 0) throw sg::SgError(SG_E_ARG, "getMelSpec: empty sound");
    double* d = nullptr;
    HIPCHK(hipMalloc(&d, (size_t)len * sizeof(double)));
    std::unique_ptr<double, void (*)(double*)> hold(d, [](double* q) { (void)hipFree(q); });
    HIPCHK(hipMemcpyAsync(d, wave, (size_t)len * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    std::vector<double> spec;
    int nk = 0;
    sg::mel_spec_device(g, d, len, spec, &nk, ctx->stream);
    *nb = g.nb;
    *nc = nk;
    if (out) {
      if ((int64_t)spec.size() > cap) throw sg::SgError(SG_E_CAPACITY, "sg_mel_spec: output capacity too small");
      std::memcpy(out, spec.data(), spec.size() * sizeof(double));
    }
    return SG_OK;
  });
}

int sg_compare_sounds_batch(sg_ctx* ctx, const double* target_spec, int32_t nb, int32_t nc_target,
                            const float* d_wave, const int64_t* offsets, const int64_t* lengths, int64_t n,
                            const sg_mel_params* p, int32_t methods, double* out, double* summary) {
  return guarded(ctx, [&]() {
    if (!ctx || !p || !out || n < 0 || (n > 0 && (!offsets || !lengths || !d_wave)) || nc_target < 0 ||
        (nc_target > 0 && !target_spec) || (methods & ~15) || methods == 0)
      throw sg::SgError(SG_E_ARG, "sg_compare_sounds_batch: bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    const sg::MelGeom g = sg::mel_geom(*p);
    if (nb != g.nb) throw sg::SgError(SG_E_ARG, "sg_compare_sounds_batch: target spectrum rows != mel bands");
    if (n == 0) return SG_OK;
    sg::compare_sounds_device(g, target_spec, nc_target, d_wave, offsets, lengths, n, methods,
                              p->penalizeLengthDif != 0, out, summary, ctx->stream);
    return SG_OK;
  });
}

int sg_dtw_symmetric2(const double* x, int64_t n, const double* y, int64_t m, double* out) {
  if (!x || !y || !out || n < 1 || m < 1) return SG_E_ARG;
  std::vector<double> prev((size_t)m), cur((size_t)m);
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t j = 0; j < m; ++j) {
      const double d = std::fabs(x[i] - y[j]);
      double g;
      if (i == 0 && j == 0) g = d;
      else {
        g = INFINITY;
        if (i > 0 && j > 0) g = std::min(g, prev[j - 1] + 2 * d);
        if (i > 0) g = std::min(g, prev[j] + d);
        if (j > 0) g = std::min(g, cur[j - 1] + d);
      }
      cur[j] = g;
    }
    std::swap(prev, cur);
  }
  *out = prev[m - 1] / (double)(n + m);
  return SG_OK;
}

int sg_plan_call_work(const sg_plan* plan, double* rows, double* fft_flops) {
  if (!plan) return SG_E_ARG;
  const sg::Batch& B = plan->B;
  if (rows) std::memcpy(rows, B.call_rows.data(), B.call_rows.size() * sizeof(double));
  if (fft_flops) std::memcpy(fft_flops, B.call_flops.data(), B.call_flops.size() * sizeof(double));
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
    const int64_t e = sg::fl_push(B, env, (int64_t)(wl / 2) * env_nc);
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
    if (!ctx) throw sg::SgError(SG_E_ARG, "sg_spectral_envelope: needs a device context (the matrix is computed on the GPU)");
    auto P = std::make_unique<sg_plan>();
    sg::Batch& B = P->B;
    sg::plan_envelope(B, R, nr, nc, formants, formantDep, rolloffLip, mouthAnchors, mouthOpenThres, openMouthBoost,
                      vocalTract, temperature, formDrift, formDisp, formantDepStoch, smoothLinearFactor, samplingRate,
                      speedSound);
    sg::finalize_spec(B);
    HIPCHK(hipSetDevice(ctx->device));
    sg::device_upload(B, P->D, ctx->stream);
    sg::launch_spec_env(P->D, B, ctx->stream);
    const size_t n = (size_t)nr * (size_t)nc;
    std::vector<float> h(n);
    if (n) HIPCHK(hipMemcpyAsync(h.data(), P->D.fl + B.fe_base + B.envjobs[0].out, n * sizeof(float),
                                 hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (size_t i = 0; i < n; ++i) out[i] = h[i];
    return SG_OK;
  });
}

// ---- output writer: seewave::savewav (R/soundgen.R:856, R/morph.R:205) -------
int sg_pcm16(sg_ctx* ctx, sg_plan* plan, const float* d_in, int16_t* d_out, void* stream) {
  return guarded(ctx, [&]() {
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    const sg::Batch& B = plan->B;
    const int64_t n = (int64_t)B.call_len.size();
    if (plan->D.pcm.n != n || !plan->D.pcm.buf) plan->D.pcm.prepare(B.call_off.data(), B.call_len.data(), n, s);
    plan->D.pcm.run(d_in, false, SG_PCM_NORMALIZE, 0.0, d_out, s);
    return SG_OK;
  });
}

int sg_savewav_pcm(sg_ctx* ctx, const double* wave, int64_t n, const double* rescale, int16_t* pcm_out) {
  return guarded(ctx, [&]() {
    if (rescale) {  // seewave.r:5200-5204
      if (rescale[0] >= 0) throw sg::SgError(SG_E_ARG, "The first value of 'rescale' should not be >=0");
      if (rescale[1] <= 0) throw sg::SgError(SG_E_ARG, "The first value of 'rescale' should not be <=0");
    }
    if (n <= 0) return SG_OK;
    HIPCHK(hipSetDevice(ctx->device));
    double* din = nullptr;
    int16_t* dout = nullptr;
    HIPCHK(hipMalloc(&din, (size_t)n * sizeof(double)));
    std::unique_ptr<void, hipError_t (*)(void*)> h1(din, hipFree);
    HIPCHK(hipMalloc(&dout, (size_t)n * sizeof(int16_t)));
    std::unique_ptr<void, hipError_t (*)(void*)> h2(dout, hipFree);
    HIPCHK(hipMemcpyAsync(din, wave, (size_t)n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    sg::PcmJob job;
    const int64_t off = 0;
    job.prepare(&off, &n, 1, ctx->stream);
    job.run(din, true, rescale ? SG_PCM_RESCALE : SG_PCM_NORMALIZE, rescale ? rescale[1] - rescale[0] : 0.0, dout,
            ctx->stream);
    HIPCHK(hipMemcpyAsync(pcm_out, dout, (size_t)n * sizeof(int16_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    job.free();
    return SG_OK;
  });
}

// tuneR::writeWave(object, filename, extensible = TRUE) of a mono 16-bit PCM
// Wave (tuneR_1.3.2.tar.gz::tuneR/R/writeWave.R): RIFF/WAVE, a 40-byte
// WAVE_FORMAT_EXTENSIBLE fmt chunk (channel mask 1 = front left, PCM subformat
// GUID), a fact chunk with the sample count, then the little-endian samples.
int sg_wav_write(const char* path, const int16_t* pcm, int64_t n, int32_t samplingRate) {
  if (!path || (n > 0 && !pcm) || n < 0 || n > (int64_t)0x7fffffff / 2 - 72) return SG_E_ARG;
  FILE* f = std::fopen(path, "wb");
  if (!f) return SG_E_ARG;
  auto u32 = [&](uint32_t v) { unsigned char b[4] = {(unsigned char)v, (unsigned char)(v >> 8), (unsigned char)(v >> 16), (unsigned char)(v >> 24)}; std::fwrite(b, 1, 4, f); };
  auto u16 = [&](uint16_t v) { unsigned char b[2] = {(unsigned char)v, (unsigned char)(v >> 8)}; std::fwrite(b, 1, 2, f); };
  const uint32_t bytes = (uint32_t)(n * 2);
  std::fwrite("RIFF", 1, 4, f);
  u32(bytes + 72);
  std::fwrite("WAVEfmt ", 1, 8, f);
  u32(40);
  u16(65534);                              // WAVE_FORMAT_EXTENSIBLE
  u16(1);                                  // channels
  u32((uint32_t)samplingRate);
  u32((uint32_t)samplingRate * 2);         // bytes per second
  u16(2);                                  // block align
  u16(16);                                 // bits per sample
  u16(22);                                 // cbSize
  u16(16);                                 // valid bits
  u32(1);                                  // channel mask: FL
  static const unsigned char guid[16] = {1, 0, 0, 0, 0, 0, 16, 0, 128, 0, 0, 170, 0, 56, 155, 113};  // PCM
  std::fwrite(guid, 1, 16, f);
  std::fwrite("fact", 1, 4, f);
  u32(4);
  u32((uint32_t)n);
  std::fwrite("data", 1, 4, f);
  u32(bytes);
  for (int64_t i = 0; i < n; ++i) u16((uint16_t)pcm[i]);
  const bool ok = std::ferror(f) == 0;
  return std::fclose(f) == 0 && ok ? SG_OK : SG_E_ARG;
}

int sg_get_smooth_contour(sg_anchors anchors, int64_t len, int32_t thisIsPitch, int32_t method, int32_t has_floor,
                          double valueFloor, int32_t has_ceil, double valueCeiling, double samplingRate, double* out,
                          int64_t* out_len) {
  return guarded(nullptr, [&]() {
    if (!out_len || len < -1 || (len != 0 && !out)) throw sg::SgError(SG_E_ARG, "sg_get_smooth_contour: arguments");
    sg::vec v;
    *out_len = 0;
    if (!sg::smooth_contour(anchors, len, thisIsPitch != 0, method, has_floor != 0, valueFloor, has_ceil != 0,
                            valueCeiling, v, samplingRate))
      return SG_OK;  // NA anchors or len 0: R returns NA
    std::memcpy(out, v.data(), v.size() * sizeof(double));
    *out_len = (int64_t)v.size();
    return SG_OK;
  });
}

int sg_get_rolloff(const double* pitch_per_gc, int32_t n_gc, int32_t nHarmonics, double rolloff, double rolloffOct,
                   double rolloffParab, double rolloffParabHarm, double rolloffParabCeiling, double rolloffKHz,
                   double baseline, double throwaway, double samplingRate, double* out, int32_t* out_rows) {
  return guarded(nullptr, [&]() {
    sg::vec p(pitch_per_gc, pitch_per_gc + n_gc);
    int64_t H = 0;
    sg::vec r = sg::get_rolloff(p, nHarmonics, sg::vec(n_gc, rolloff), sg::vec(n_gc, rolloffOct), rolloffParab,
                                rolloffParabHarm, sg::vec(n_gc, rolloffKHz), baseline, throwaway, samplingRate, H,
                                rolloffParabCeiling);
    std::memcpy(out, r.data(), r.size() * sizeof(double));
    *out_rows = (int32_t)H;
    return SG_OK;
  });
}

}  // extern "C"
