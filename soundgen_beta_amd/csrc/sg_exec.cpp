// sg_exec.cpp — HBM arena for a plan and the per-batch launch sequence.
#include "sg_exec.h"
#include "sg_amp.h"
#include "sg_prof.h"

#include <algorithm>
#include <chrono>
#include <exception>
#include <thread>
#include <cmath>
#include <climits>
#include <atomic>
#include <map>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>

namespace sg {

namespace {
#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t _e = (x);                                                                  \
    if (_e != hipSuccess)                                                                 \
      throw SgError(SG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e));     \
  } while (0)

constexpr size_t ALIGN = 256;
size_t up(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

struct Layout {
  size_t tall, tlong, tshort, tallp, srun, trun, thp, fin_tiles_hp, W64, fh, frames64, frames64_tab, roots64, roots64_wl,
      roots64_off;
  size_t segs, epochs, knots, amps, ampcols, ampjobs, ampsrc, tasks, pieces, syls, syl_tiles, copy_tiles, ptiles, cknots, W, taskmax, ptilemax, maxes, total;
  size_t geoms, frames, fgroups, olas, olatiles, olasegs, olatilemax, olamax, items, mixes, mixtiles, fl, fs;
  size_t eterms, ecols, envjobs, envtasks, elog2;
  explicit Layout(const Batch& B) {
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += up(bytes > 0 ? bytes : 1); return r; };
    const size_t ntask = (size_t)bulk_size(B.tasks_x, B.tasks);
    segs = take((size_t)bulk_size(B.segs_x, B.segs) * sizeof(SgSeg));
    epochs = take(B.epochs.size() * sizeof(SgEpoch));
    knots = take(B.knots.size() * sizeof(double));
    amps = take((size_t)B.amp_total * sizeof(float) + 64 * sizeof(float));
    ampcols = take(B.ampcols.size() * sizeof(SgAmpCol));
    ampjobs = take(B.ampjobs.size() * sizeof(SgAmpJob));
    ampsrc = take(B.ampsrc.size() * sizeof(float));
    tasks = take(ntask * sizeof(SgWTask));
    tall = take(ntask * sizeof(int32_t));
    tlong = take(ntask * sizeof(int32_t));
    tshort = take(ntask * sizeof(int32_t));
    tallp = take(ntask * sizeof(int32_t));
    srun = take((ntask + 1) * sizeof(int32_t));
    trun = take((ntask + 1) * sizeof(int32_t));
    thp = take(ntask * sizeof(int32_t));
    fin_tiles_hp = take(B.fin_tiles_hp.size() * sizeof(SgSylTile));
    W64 = take((size_t)B.w64_total * sizeof(double));
    fh = take((size_t)B.fh_total * sizeof(double));
    frames64 = take(B.frames64.size() * sizeof(SgFrame64));
    frames64_tab = take(B.frames64_tab.size() * sizeof(int64_t));
    roots64 = take((size_t)B.roots64_total * 2 * sizeof(double));
    roots64_wl = take(B.roots64_wl.size() * sizeof(int32_t));
    roots64_off = take(B.roots64_off.size() * sizeof(int64_t));
    pieces = take(B.pieces.size() * sizeof(SgPiece));
    syls = take(B.syls.size() * sizeof(SgSyllable));
    syl_tiles = take(B.fin_tiles.size() * sizeof(SgSylTile));
    copy_tiles = take(B.copy_tiles.size() * sizeof(SgCopyTile));
    ptiles = take(B.ptiles.size() * sizeof(SgSylTile));
    cknots = take(B.cknots.size() * sizeof(double));
    W = take((size_t)B.w_total * sizeof(float));
    taskmax = take(ntask * sizeof(float));
    ptilemax = take(B.ptiles.size() * sizeof(float));
    maxes = take(B.syls.size() * sizeof(float));
    geoms = take(B.geoms.size() * sizeof(SgFftGeom));
    frames = take((B.frames[0].size() + B.frames[1].size()) * sizeof(SgFrame));
    fgroups = take(B.fgroups.size() * sizeof(SgFrameGroup));
    olas = take(B.olas_dev.size() * sizeof(SgOla));
    olatiles = take(B.olatiles.size() * sizeof(SgOlaTile));
    olasegs = take(B.olasegs.size() * sizeof(SgSegment));
    olatilemax = take((B.olatiles.size() + (size_t)B.n_segslots) * sizeof(float));  // tile slots, then segment slots
    olamax = take(B.olas_dev.size() * sizeof(float));
    items = take(B.items.size() * sizeof(SgNoiseItem));
    mixes = take(B.mixes_dev.size() * sizeof(SgMix));
    mixtiles = take(B.mixtiles.size() * sizeof(SgMixTile));
    eterms = take((size_t)bulk_size(B.eterms_x, B.eterms) * sizeof(SgEnvTerm));
    ecols = take(B.ecols.size() * sizeof(SgEnvCol));
    envjobs = take(B.envjobs.size() * sizeof(SgEnvJob));
    envtasks = take(B.envtasks.size() * sizeof(SgEnvTask));
    elog2 = take(B.elog2.size() * sizeof(double));
    // uploaded floats, then the device-computed envelopes from fe_base on, then the
    // noise uniforms expanded at upload from fu_base on
    fl = take((size_t)std::max<int64_t>(std::max<int64_t>(bulk_size(B.fl_x, B.fl), B.fe_base + B.fe_total),
                                        B.fu_base + B.fu_total) * sizeof(float));
    fs = take((size_t)B.fs_total * sizeof(float) + 256);
    total = o;
  }
};
}  // namespace

// Split the 1024-sample finalize tiles of syllables without envelope or
// drift: the parts of a tile lying in direct or zero pieces go to the fast
// kernel (sg_harm_copy; aligned direct runs merged up to SG_COPY_TILE); tiles
// touching a crossfade (multi-term) piece, and every tile of a syllable with an
// envelope or drift, keep the general kernel.
static void split_finalize_tiles(Batch& B) {
  const int64_t copy_tile = SG_COPY_TILE;
  B.fin_tiles.clear();
  B.fin_tiles_hp.clear();
  B.copy_tiles.clear();
  for (const SgSylTile& t : B.syl_tiles) {
    const SgSyllable& sy = B.syls[t.syl];
    if (sy.hp) {  // fp64 syllable: sg_harm_finalize_hp
      B.fin_tiles_hp.push_back(t);
      continue;
    }
    const int64_t end = std::min<int64_t>(t.k0 + 1024, sy.L);
    const int pend = sy.piece0 + sy.npiece;
    bool ok = sy.env.kind == 0 && sy.drift.nk == 0 && sy.genv.kind == 0;
    for (int p = t.piece; ok && p < pend && B.pieces[p].start < end; ++p) ok = B.pieces[p].nterms <= 0;
    if (!ok) {
      B.fin_tiles.push_back(t);
      continue;
    }
    for (int p = t.piece; p < pend && B.pieces[p].start < end; ++p) {
      const SgPiece& pc = B.pieces[p];
      const int64_t a = std::max<int64_t>(t.k0, pc.start), b = std::min<int64_t>(end, pc.start + pc.len);
      if (b <= a) continue;
      SgCopyTile c{};
      const bool zero = pc.nterms == 0;
      c.src = zero ? 0 : pc.t[0].src + (a - pc.start);
      c.dst = sy.out_off + a;
      c.k0 = a;
      c.L = sy.L;
      c.n = (int32_t)(b - a);
      c.max_slot = sy.max_slot;
      c.fade = sy.fade;
      c.syl = t.syl;
      c.flags = (sy.dst_fs ? SG_COPY_FS : 0) | (zero ? SG_COPY_ZERO : 0) |
                (!zero && ((c.src - c.dst) & 3) == 0 ? SG_COPY_VEC : 0);
      if (!B.copy_tiles.empty()) {  // extend the previous aligned run
        SgCopyTile& q = B.copy_tiles.back();
        if ((q.flags & SG_COPY_VEC) && (c.flags & SG_COPY_VEC) && q.syl == c.syl && q.flags == c.flags &&
            q.k0 + q.n == c.k0 && q.src + q.n == c.src && q.n + c.n <= copy_tile) {
          q.n += c.n;
          continue;
        }
      }
      B.copy_tiles.push_back(c);
    }
  }
}

// direct-output table jobs: on by default; SG_TAB_DIRECT=0 keeps every span on W (experiment knob)
static bool direct_on() {  // read at each upload
  const char* e = std::getenv("SG_TAB_DIRECT");
  return !(e && e[0] == '0');
}

// Wavetable spans (SgTabJob, sg_dev.h): runs of consecutive constant-amplitude,
// linear-phase fp32 tasks of one syllable on one amplitude column whose
// interpolation-error bound admits a table of N <= 2^SG_TAB_LOGN_MAX points and
// with >= 4 N samples; each run one job per SG_TAB_TASKS tasks, in task order.
struct TabSpans {
  std::vector<SgTabJob> jobs;
  std::vector<uint8_t> in_tab;
  std::vector<uint8_t> direct_syl;  // per syllable: its samples go straight to the output (SG_TAB_DIRECT)
  int64_t tasks = 0, direct = 0;
  int64_t samples = 0, terms = 0;
};
// the column's amplitudes as sg_amp_build computes them (host restatement)
struct ColumnReader {
  const Batch& B;
  std::vector<std::pair<int64_t, int32_t>> by_off;  // (amp_off, job)
  std::vector<double> lg;
  explicit ColumnReader(const Batch& b) : B(b) {
    for (size_t j = 0; j < B.ampjobs.size(); ++j) by_off.push_back({B.ampjobs[j].amp_off, (int32_t)j});
    std::sort(by_off.begin(), by_off.end());
    lg.resize((size_t)B.amp_lg_rows + 2);
    for (size_t k = 0; k < lg.size(); ++k) lg[k] = std::log2((double)(k + 1));
  }
  // smallest log2 N with the bound <= SG_TAB_TOL sum |A_r|, 0 if none <= SG_TAB_LOGN_MAX
  int logn_max = SG_TAB_LOGN_MAX;
  int logn(int64_t a_off, int32_t Rn) const {
    auto it = std::upper_bound(by_off.begin(), by_off.end(), std::make_pair(a_off, INT32_MAX));
    if (it == by_off.begin()) return 0;
    const SgAmpJob& J = B.ampjobs[(size_t)std::prev(it)->second];
    const int64_t rel = a_off - J.amp_off;
    if (J.Rp <= 0 || rel % J.Rp != 0 || rel / J.Rp >= J.G || Rn > J.Rp) return 0;
    const int g = (int)(rel / J.Rp);
    double s0 = 0, s4 = 0;
    for (int r = 0; r < Rn; ++r) {
      double a = 0;
      if (r < J.R) a = J.src_off >= 0 ? (double)B.ampsrc[(size_t)(J.src_off + (int64_t)g * J.Rp + r)]
                                      : (double)(float)amp_value(B.ampcols.data() + J.col0, J, lg.data(), g, r);
      const double k = r + 1.0;
      s0 += std::fabs(a);
      s4 += std::fabs(a) * k * k * k * k;
    }
    if (!(s0 > 0)) return 0;
    const double two_pi4 = 1558.5454565440389;  // (2 pi)^4
    for (int b = SG_TAB_LOGN_MIN; b <= logn_max; ++b) {
      const double n4 = std::ldexp(1.0, 4 * b);
      if (two_pi4 * s4 / (384.0 * n4) <= SG_TAB_TOL * s0) return b;
    }
    return 0;
  }
};
// The batch's task blocks (Blocks<SgWTask>: one per planning part, then the
// batch's own vector). A syllable's tasks never straddle two blocks (a part plans
// whole calls), so the per-block passes below run on host threads independently.
struct TaskBlock {
  int64_t o;
  const SgWTask* p;
  int64_t n;
};
static std::vector<TaskBlock> task_blocks(const Batch& B) {
  std::vector<TaskBlock> tb;
  bulk_each(B.tasks_x, B.tasks, [&](int64_t o, const SgWTask* p, int64_t n) { tb.push_back(TaskBlock{o, p, n}); });
  return tb;
}
// f(i) for i in [0, n) on up to 16 host threads (the upload's per-block passes)
template <class F>
static void for_blocks(size_t n, F&& f) {
  const size_t nt = std::min<size_t>(n, std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
  if (nt <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::exception_ptr> errs(nt);
  auto work = [&](size_t t) {
    try {
      for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    } catch (...) {
      errs[t] = std::current_exception();
    }
  };
  std::vector<std::thread> pool;
  for (size_t t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}
// the runs of one block (jobs in task order; in_tab and direct_syl entries of the
// block's tasks and syllables, which no other block touches)
struct TabBlock {
  std::vector<SgTabJob> jobs;
  int64_t direct = 0, samples = 0, terms = 0;
};
static void group_block(const Batch& B, const ColumnReader& cols, const TaskBlock& blk, TabSpans& S, TabBlock& out) {
  auto tab_task = [](const SgWTask& t) {
    return t.flags == (SG_TASK_CONST | SG_TASK_LIN) && t.R <= SG_ROWS_F32 && t.Rn > 0;
  };
  // a whole syllable of direct (or zero) pieces without envelope or drift: the job
  // writes its final samples (sg_sine_bank_tab's direct mode)
  auto direct_ok = [&](const SgWTask& t, int64_t r0, int64_t r1) {
    if (t.syl < 0 || t.syl >= (int32_t)B.syls.size() || !direct_on()) return false;
    const SgSyllable& sy = B.syls[(size_t)t.syl];
    if (sy.hp || sy.env.kind != 0 || sy.genv.kind != 0 || sy.drift.nk != 0 || sy.nptile != 0) return false;
    if (r0 != sy.task0 || r1 != sy.task0 + sy.ntask || r1 - r0 > SG_TAB_TASKS) return false;
    for (int32_t p = sy.piece0; p < sy.piece0 + sy.npiece; ++p)
      if (B.pieces[(size_t)p].nterms > 0) return false;
    return true;
  };
  const int per_job = SG_TAB_TASKS;
  int64_t run0 = -1, run_samples = 0;
  SgWTask first{};
  auto close_run = [&](int64_t end) {  // tasks [run0, end)
    if (run0 < 0) return;
    const int logn = run_samples >= (int64_t(4) << SG_TAB_LOGN_MIN) ? cols.logn(first.a_off, first.Rn) : 0;
    if (logn && run_samples >= (int64_t(4) << logn)) {
      const bool dir = end - run0 <= per_job && direct_ok(first, run0, end);
      if (dir) {
        S.direct_syl[(size_t)first.syl] = 1;
        ++out.direct;
      }
      for (int64_t i = run0; i < end; i += per_job) {
        const int32_t n = (int32_t)std::min<int64_t>(per_job, end - i);
        out.jobs.push_back(SgTabJob{first.a_off, first.Rn, (int32_t)i, n, logn, first.syl, dir ? SG_TAB_DIRECT : 0});
        for (int64_t q = i; q < i + n; ++q) S.in_tab[(size_t)q] = 1;
      }
      out.samples += run_samples;
      out.terms += run_samples * first.Rn;
    }
    run0 = -1;
  };
  for (int64_t k = 0; k < blk.n; ++k) {
    const SgWTask& t = blk.p[k];
    const bool ok = tab_task(t);
    if (run0 >= 0 && !(ok && t.a_off == first.a_off && t.Rn == first.Rn && t.syl == first.syl)) close_run(blk.o + k);
    if (ok && run0 < 0) {
      run0 = blk.o + k;
      first = t;
      run_samples = 0;
    }
    if (ok) run_samples += t.len;
  }
  close_run(blk.o + blk.n);
}
// sine-bank task classes (each task's class depends on the task alone): fp64, tall
// (sg_sine_bank_tall, short ones two per wave in _tall_pairs), short fp32 (two per
// wave, sg_sine_bank_pairs), other fp32 (sg_sine_bank); tasks in a wavetable span
// have none
struct TaskClasses {
  std::vector<int32_t> tlong, tshort, tall, tallp, thp;
  std::vector<int32_t> srun, trun;  // run starts in tshort / tallp (block-local positions)
};
// a new run starts at a task of another syllable or after SG_RUN_TASKS tasks
static void run_start(std::vector<int32_t>& runs, const std::vector<int32_t>& list, int32_t& syl, const SgWTask& t) {
  const int32_t pos = (int32_t)list.size() - 1;
  if (runs.empty() || t.syl != syl || pos - runs.back() >= SG_RUN_TASKS) runs.push_back(pos);
  syl = t.syl;
}
static void classify_block(const TaskBlock& blk, const std::vector<uint8_t>& in_tab, TaskClasses& c) {
  int32_t ssyl = -1, tsyl = -1;
  for (int64_t k = 0; k < blk.n; ++k) {
    const SgWTask& t = blk.p[k];
    const int32_t i = (int32_t)(blk.o + k);
    const bool shrt = t.len <= 64 && !(t.flags & SG_TASK_ENV);
    if (!in_tab.empty() && in_tab[(size_t)i]) continue;
    if (t.flags & SG_TASK_HP) c.thp.push_back(i);
    else if (t.R > SG_ROWS_F32) {
      if (shrt) {
        c.tallp.push_back(i);
        run_start(c.trun, c.tallp, tsyl, t);
      } else {
        c.tall.push_back(i);
      }
    } else if (shrt) {
      c.tshort.push_back(i);
      run_start(c.srun, c.tshort, ssyl, t);
    } else {
      c.tlong.push_back(i);
    }
  }
}
// Wavetable spans and task classes of a batch, block by block on host threads;
// the result is what one pass over the tasks in order gives
static TabSpans group_tables(const Batch& B, bool tables, TaskClasses* classes) {
  TabSpans S;
  const std::vector<TaskBlock> tb = task_blocks(B);
  std::vector<TabBlock> tabs(tb.size());
  std::vector<TaskClasses> cls(classes ? tb.size() : 0);
  if (tables) {
    S.in_tab.assign((size_t)bulk_size(B.tasks_x, B.tasks), 0);
    S.direct_syl.assign(B.syls.size(), 0);
  }
  const ColumnReader cols(B);
  for_blocks(tb.size(), [&](size_t i) {
    if (tables) group_block(B, cols, tb[i], S, tabs[i]);
    if (classes) classify_block(tb[i], S.in_tab, cls[i]);
  });
  for (TabBlock& t : tabs) {
    S.jobs.insert(S.jobs.end(), t.jobs.begin(), t.jobs.end());
    S.direct += t.direct;
    S.samples += t.samples;
    S.terms += t.terms;
  }
  for (const SgTabJob& j : S.jobs) S.tasks += j.n;
  if (classes) {
    auto cat = [&](std::vector<int32_t> TaskClasses::*m) {
      std::vector<int32_t>& dst = classes->*m;
      dst.clear();
      size_t n = 0;
      for (const TaskClasses& c : cls) n += (c.*m).size();
      dst.reserve(n);
      for (const TaskClasses& c : cls) dst.insert(dst.end(), (c.*m).begin(), (c.*m).end());
    };
    // the runs of each block, rebased to the concatenated list, then the list's size
    auto runs = [&](std::vector<int32_t> TaskClasses::*r, std::vector<int32_t> TaskClasses::*m) {
      std::vector<int32_t>& dst = classes->*r;
      dst.clear();
      int32_t base = 0;
      for (const TaskClasses& c : cls) {
        for (int32_t x : c.*r) dst.push_back(base + x);
        base += (int32_t)(c.*m).size();
      }
      dst.push_back(base);
    };
    runs(&TaskClasses::srun, &TaskClasses::tshort);
    runs(&TaskClasses::trun, &TaskClasses::tallp);
    cat(&TaskClasses::tlong);
    cat(&TaskClasses::tshort);
    cat(&TaskClasses::tall);
    cat(&TaskClasses::tallp);
    cat(&TaskClasses::thp);
  }
  return S;
}

void finalize_plan(Batch& B) {
  split_finalize_tiles(B);
  if (std::getenv("SG_DEBUG_PLAN")) {
    std::fprintf(stderr, "sg plan: %zu sine tasks, %zu syllables, %zu copy tiles, %zu general finalize tiles\n",
                 (size_t)bulk_size(B.tasks_x, B.tasks), B.syls.size(), B.copy_tiles.size(), B.fin_tiles.size());
    {  // amplitude blocks of subharmonic (vocal-fry) epochs vs plain ones
      double fry = 0, plain = 0;
      int64_t nfry = 0;
      for (const SgEpoch& e : B.epochs) {
        const double b = (double)(2 * e.G - 1) * e.R * 4;
        if (e.invD < 1) { fry += b; ++nfry; } else plain += b;
      }
      std::fprintf(stderr, "sg plan: amplitude bytes: plain epochs %.3g, subharmonic epochs %.3g (%lld of %zu)\n", plain,
                   fry, (long long)nfry, B.epochs.size());
    }
    {
      const TabSpans T = group_tables(B, true, nullptr);
      int64_t cl = 0, cl_samples = 0;
      bulk_each(B.tasks_x, B.tasks, [&](int64_t, const SgWTask* p, int64_t n) {
        for (int64_t k = 0; k < n; ++k)
          if (p[k].flags == (SG_TASK_CONST | SG_TASK_LIN)) { ++cl; cl_samples += p[k].len; }
      });
      int64_t hist[13] = {0};
      for (const SgTabJob& j : T.jobs) ++hist[j.logn];
      std::fprintf(stderr, "sg plan: wavetable jobs %zu, %lld direct syllables (N = 256/512/1024/2048: %lld %lld %lld %lld; %zu tasks, %lld samples, %.3g terms); CONST|LIN tasks %lld (%lld samples)\n",
                   T.jobs.size(), (long long)T.direct, (long long)hist[8], (long long)hist[9], (long long)hist[10], (long long)hist[11],
                   (size_t)T.tasks, (long long)T.samples, (double)T.terms, (long long)cl,
                   (long long)cl_samples);
    }
    {  // pre-filter mixes that only place voiced syllables (raw items, no envelope, no noise)
      int64_t all = 0, ident = 0, ni = 0, ident_items = 0, noisy = 0, noisy_cov = 0, other = 0, env_only = 0, env_kind[4] = {0, 0, 0, 0};
      for (const SgMix& m : B.mixes[0]) {
        all += m.len;
        bool id = m.mult.kind == 0 && m.am_lo == 0 && m.to_fs == 1 && m.base_kind == SG_BASE_NONE;
        for (int32_t i = m.item0; i < m.item0 + m.nitems && id; ++i) {
          const SgNoiseItem& it = B.items[(size_t)i];
          id = it.ola < 0 && it.fade < 2 && it.strength.kind == 0 && !(it.flags & SG_ITEM_F64);
        }
        if (id) { ident += m.len; ident_items += m.nitems; }
        ni += m.nitems;
        if (!id && m.mult.kind == 0 && m.to_fs == 1) {  // noise-carrying mixes: samples under a noise item
          std::vector<std::pair<int64_t, int64_t>> iv;
          for (int32_t i = m.item0; i < m.item0 + m.nitems; ++i) {
            const SgNoiseItem& it = B.items[(size_t)i];
            if (it.ola >= 0) iv.push_back({std::max<int64_t>(0, it.off), std::min(m.len, it.off + it.len)});
          }
          std::sort(iv.begin(), iv.end());
          int64_t cov = 0, e = 0;
          for (auto& q : iv) { const int64_t a0 = std::max(q.first, e); if (q.second > a0) cov += q.second - a0; e = std::max(e, q.second); }
          noisy += m.len;
          noisy_cov += cov;
        } else if (!id) {
          other += m.len;
          bool vo = m.to_fs == 1;
          for (int32_t i = m.item0; i < m.item0 + m.nitems && vo; ++i) vo = B.items[(size_t)i].ola < 0;
          if (vo && m.mult.kind != 0) { env_only += m.len; env_kind[m.mult.kind & 3]++; }
        }
      }
      std::fprintf(stderr, "sg plan: pre-filter mixes %zu, %lld samples; voiced-only %lld samples (%lld of %lld items)\n",
                   B.mixes[0].size(), (long long)all, (long long)ident, (long long)ident_items, (long long)ni);
      std::fprintf(stderr, "sg plan: pre-filter mixes with noise %lld samples (%lld under noise), enveloped or fp64 %lld "
                   "(voiced-only with the global envelope %lld; contour kinds 1/2/3: %lld %lld %lld)\n",
                   (long long)noisy, (long long)noisy_cov, (long long)other, (long long)env_only, (long long)env_kind[1],
                   (long long)env_kind[2], (long long)env_kind[3]);
    }
    {  // spectral envelopes: jobs by column count, wave tasks, bins
      int64_t j1 = 0, jm = 0, cols = 0, bins = 0;
      for (const SgEnvJob& j : B.envjobs) {
        (j.nc == 1 ? j1 : jm)++;
        cols += j.nc;
        bins += (int64_t)j.nc * j.nr;
      }
      std::fprintf(stderr, "sg plan: envelope jobs %zu (%lld one-column), %lld columns, %lld bins, %zu wave tasks\n",
                   B.envjobs.size(), (long long)j1, (long long)cols, (long long)bins, B.envtasks.size());
    }
    std::vector<SgWTask> tasks;  // the merged task list (debug statistics only)
    bulk_each(B.tasks_x, B.tasks, [&](int64_t, const SgWTask* p, int64_t n) { tasks.insert(tasks.end(), p, p + n); });
    // sine-bank work: (sample, row) terms of the fp32 and the tall tasks, rows histogram of the tall ones
    double terms[2] = {0, 0};
    int64_t ntask[2] = {0, 0}, rmax = 0, samples[2] = {0, 0};
    std::map<int, int64_t> rh;
    int64_t nshort[2] = {0, 0}, lh[2][5] = {{0}};
    double sterms[2] = {0, 0};
    {  // fp64 (SG_TASK_HP) tasks
      int64_t nh = 0, sh = 0, lh64 = 0;
      double th = 0, rn = 0;
      for (const SgWTask& t : tasks)
        if (t.flags & SG_TASK_HP) {
          ++nh; sh += t.len; lh64 += t.len <= 64;
          th += (double)t.Rn * t.len * ((t.flags & SG_TASK_CONST) ? 1 : 2);
          rn += t.Rn;
        }
      std::fprintf(stderr, "sg plan: fp64 tasks %lld (%lld samples, %lld of <= 64 samples, %.3g chain terms, mean Rn %.1f)\n",
                   (long long)nh, (long long)sh, (long long)lh64, th, nh ? rn / nh : 0.0);
    }
    for (const SgWTask& t : tasks) {
      const int k = t.R > SG_ROWS_F32 ? 1 : 0;
      terms[k] += (double)t.R * t.len * ((t.flags & SG_TASK_CONST) ? 1 : 2);
      ++ntask[k];
      samples[k] += t.len;
      if (t.len <= 64) { ++nshort[k]; sterms[k] += (double)t.R * t.len * ((t.flags & SG_TASK_CONST) ? 1 : 2); }
      lh[k][t.len <= 64 ? 0 : t.len <= 128 ? 1 : t.len <= 256 ? 2 : t.len <= 512 ? 3 : 4]++;
      if (k) {
        rmax = std::max<int64_t>(rmax, t.R);
        rh[t.R < 256 ? 0 : t.R < 512 ? 1 : t.R < 1024 ? 2 : t.R < 2048 ? 3 : 4]++;
      }
    }
    std::fprintf(stderr, "sg plan: sine tasks fp32 %lld (%lld samples, %.3g chain terms), tall %lld (%lld samples, %.3g chain terms, max R %lld; R<256 %lld, <512 %lld, <1024 %lld, <2048 %lld, more %lld)\n",
                 (long long)ntask[0], (long long)samples[0], terms[0], (long long)ntask[1], (long long)samples[1], terms[1],
                 (long long)rmax, (long long)rh[0], (long long)rh[1], (long long)rh[2], (long long)rh[3], (long long)rh[4]);
    for (int k = 0; k < 2; ++k)
      std::fprintf(stderr, "sg plan: %s tasks <= 64 samples: %lld (%.3g chain terms); len <=64/128/256/512/more: %lld %lld %lld %lld %lld\n",
                   k ? "tall" : "fp32", (long long)nshort[k], sterms[k], (long long)lh[k][0], (long long)lh[k][1],
                   (long long)lh[k][2], (long long)lh[k][3], (long long)lh[k][4]);
  }
  // crossfade-piece tiles: fp32 syllables first, then the fp64 ones (sg_piece_max_hp)
  B.ptiles.clear();
  bool any_hp = false;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) B.ptile_hp = (int64_t)B.ptiles.size();
    for (size_t s = 0; s < B.syls.size(); ++s) {
      SgSyllable& sy = B.syls[s];
      if ((sy.hp != 0) != (pass == 1)) continue;
      any_hp |= sy.hp != 0;
      sy.ptile0 = (int32_t)B.ptiles.size();
      for (int32_t p = sy.piece0; p < sy.piece0 + sy.npiece; ++p)
        if (B.pieces[p].nterms > 0)
          for (int64_t q0 = 0; q0 < B.pieces[p].len; q0 += 256) B.ptiles.push_back(SgSylTile{(int32_t)s, p, q0});
      sy.nptile = (int32_t)B.ptiles.size() - sy.ptile0;
    }
  }
  // slices of whole syllables with about equal sample counts
  B.slices.clear();
  const int64_t nsyl = (int64_t)B.syls.size();
  if (nsyl == 0) return;
  int64_t total = 0;
  for (const SgSyllable& sy : B.syls) total += sy.L;
  int slices = SG_SLICES;
  if (any_hp) slices = 1;  // the fp64 syllables' tiles are listed after every fp32 one
  const int K = (int)std::min<int64_t>(slices, nsyl);
  int64_t acc = 0, ft = 0, ct = 0;
  int32_t s0 = 0;
  for (int32_t s = 0; s < nsyl; ++s) {
    acc += B.syls[s].L;
    const bool cut = s == nsyl - 1 || acc * K >= total * ((int64_t)B.slices.size() + 1);
    if (!cut) continue;
    Slice c{};
    c.s0 = s0; c.s1 = s + 1;
    c.t0 = B.syls[s0].task0;
    c.t1 = B.syls[s].task0 + B.syls[s].ntask;
    c.p0 = K == 1 ? 0 : B.syls[s0].ptile0;
    c.p1 = K == 1 ? B.ptile_hp : B.syls[s].ptile0 + B.syls[s].nptile;
    c.f0 = ft;
    while (ft < (int64_t)B.fin_tiles.size() && B.fin_tiles[ft].syl <= s) ++ft;
    c.f1 = ft;
    c.c0 = ct;
    while (ct < (int64_t)B.copy_tiles.size() && B.copy_tiles[ct].syl <= s) ++ct;
    c.c1 = ct;
    B.slices.push_back(c);
    s0 = s + 1;
  }
}

int64_t device_bytes(const Batch& B) { return (int64_t)Layout(B).total; }

void device_free(DevicePlan& D) {
  if (D.arena) (void)hipFree(D.arena);
  if (D.tabbuf) (void)hipFree(D.tabbuf);
  D.pcm.free();
  for (hipEvent_t e : D.ev_slice) (void)hipEventDestroy(e);
  if (D.ev_fork) (void)hipEventDestroy(D.ev_fork);
  if (D.ev_join) (void)hipEventDestroy(D.ev_join);
  D = DevicePlan{};
}

// wavetable path for long static spans (sg_sine_bank_tab): on by default;
// sg_set_sine_table(0) turns it off
static std::atomic<int> g_tab{-1};
static bool tab_on() {
  int v = g_tab.load();
  if (v < 0) {
    v = 1;  // sg_set_sine_table(0) turns the wavetable path off (tests)
    int expect = -1;
    g_tab.compare_exchange_strong(expect, v);
  }
  return v != 0;
}

}  // namespace sg
extern "C" int sg_set_sine_table(int32_t on) {
  if (on != 0 && on != 1) return SG_E_ARG;
  sg::g_tab.store(on);
  return SG_OK;
}
namespace sg {

void device_upload(const Batch& B, DevicePlan& D, hipStream_t s) {
  // SG_PLAN_PROF=1: seconds of each upload stage on stderr
  auto tprev = std::chrono::steady_clock::now();
  auto stage = [&](const char* what) {
    if (!g_prof_on) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "sg_upload_prof %-10s %.3f s\n", what, std::chrono::duration<double>(t - tprev).count());
    tprev = t;
  };
  Layout L(B);
  if (D.arena && D.arena_bytes < L.total) device_free(D);
  if (!D.arena) {
    HIPCHK(hipMalloc(&D.arena, L.total));
    D.arena_bytes = L.total;
  }
  stage("malloc");
  char* a = D.arena;
  D.segs = (SgSeg*)(a + L.segs);
  D.epochs = (SgEpoch*)(a + L.epochs);
  D.knots = (double*)(a + L.knots);
  D.amps = (float*)(a + L.amps);
  D.ampcols = (const SgAmpCol*)(a + L.ampcols);
  D.ampjobs = (const SgAmpJob*)(a + L.ampjobs);
  D.ampsrc = (const float*)(a + L.ampsrc);
  D.tasks = (SgWTask*)(a + L.tasks);
  D.tall = (int32_t*)(a + L.tall);
  D.tlong = (int32_t*)(a + L.tlong);
  D.tshort = (int32_t*)(a + L.tshort);
  D.tallp = (int32_t*)(a + L.tallp);
  D.srun = (int32_t*)(a + L.srun);
  D.trun = (int32_t*)(a + L.trun);
  D.thp = (int32_t*)(a + L.thp);
  D.fin_tiles_hp = (SgSylTile*)(a + L.fin_tiles_hp);
  D.W64 = (double*)(a + L.W64);
  D.fh = (double*)(a + L.fh);
  D.frames64 = (SgFrame64*)(a + L.frames64);
  D.frames64_tab = (int64_t*)(a + L.frames64_tab);
  D.roots64 = (double*)(a + L.roots64);
  D.roots64_wl = (int32_t*)(a + L.roots64_wl);
  D.roots64_off = (int64_t*)(a + L.roots64_off);
  D.pieces = (SgPiece*)(a + L.pieces);
  D.syls = (SgSyllable*)(a + L.syls);
  D.syl_tiles = (SgSylTile*)(a + L.syl_tiles);
  D.copy_tiles = (SgCopyTile*)(a + L.copy_tiles);
  D.ptiles = (SgSylTile*)(a + L.ptiles);
  D.cknots = (double*)(a + L.cknots);
  D.W = (float*)(a + L.W);
  D.taskmax = (float*)(a + L.taskmax);
  D.ptilemax = (float*)(a + L.ptilemax);
  D.maxes = (float*)(a + L.maxes);
  D.geoms = (SgFftGeom*)(a + L.geoms);
  D.frames = (SgFrame*)(a + L.frames);
  D.fgroups = (SgFrameGroup*)(a + L.fgroups);
  D.olas = (SgOla*)(a + L.olas);
  D.olatiles = (SgOlaTile*)(a + L.olatiles);
  D.olasegs = (SgSegment*)(a + L.olasegs);
  D.olatilemax = (float*)(a + L.olatilemax);
  D.olamax = (float*)(a + L.olamax);
  D.items = (SgNoiseItem*)(a + L.items);
  D.mixes = (SgMix*)(a + L.mixes);
  D.mixtiles = (SgMixTile*)(a + L.mixtiles);
  D.fl = (float*)(a + L.fl);
  D.fs = (float*)(a + L.fs);
  D.eterms = (SgEnvTerm*)(a + L.eterms);
  D.ecols = (SgEnvCol*)(a + L.ecols);
  D.envjobs = (SgEnvJob*)(a + L.envjobs);
  D.envtasks = (SgEnvTask*)(a + L.envtasks);
  D.elog2 = (double*)(a + L.elog2);
  auto cp = [&](void* dst, const void* src, size_t bytes) {
    if (bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
  };
  bulk_each(B.segs_x, B.segs, [&](int64_t o, const SgSeg* p, int64_t n) { cp(D.segs + o, p, n * sizeof(SgSeg)); });
  cp(D.epochs, B.epochs.data(), B.epochs.size() * sizeof(SgEpoch));
  cp(D.knots, B.knots.data(), B.knots.size() * sizeof(double));
  cp((void*)D.ampcols, B.ampcols.data(), B.ampcols.size() * sizeof(SgAmpCol));
  cp((void*)D.ampjobs, B.ampjobs.data(), B.ampjobs.size() * sizeof(SgAmpJob));
  cp((void*)D.ampsrc, B.ampsrc.data(), B.ampsrc.size() * sizeof(float));
  bulk_each(B.tasks_x, B.tasks, [&](int64_t o, const SgWTask* p, int64_t n) { cp(D.tasks + o, p, n * sizeof(SgWTask)); });
  stage("copy_tasks");
  // wavetable spans (SgTabJob, sg_dev.h) and the task classes, block by block
  TaskClasses C;
  TabSpans T = group_tables(B, tab_on(), &C);
  D.tlong_host.swap(C.tlong);
  D.tshort_host.swap(C.tshort);
  D.tall_host.swap(C.tall);
  D.tallp_host.swap(C.tallp);
  D.srun_host.swap(C.srun);
  D.trun_host.swap(C.trun);
  D.thp_host.swap(C.thp);
  D.tabjobs_host.swap(T.jobs);
  D.tab_samples = T.samples;
  D.tab_terms = T.terms;
  if (!D.tabjobs_host.empty()) {  // one allocation kept across uploads
    const size_t bj = D.tabjobs_host.size() * sizeof(SgTabJob);
    if (D.tabbuf && D.tabbuf_bytes < bj) {
      (void)hipFree(D.tabbuf);
      D.tabbuf = nullptr;
    }
    if (!D.tabbuf) {
      HIPCHK(hipMalloc(&D.tabbuf, bj));
      D.tabbuf_bytes = bj;
    }
    D.tabjobs = (SgTabJob*)D.tabbuf;
  }
  stage("classify");
  cp(D.tall, D.tall_host.data(), D.tall_host.size() * sizeof(int32_t));
  cp(D.tlong, D.tlong_host.data(), D.tlong_host.size() * sizeof(int32_t));
  cp(D.tshort, D.tshort_host.data(), D.tshort_host.size() * sizeof(int32_t));
  cp(D.tallp, D.tallp_host.data(), D.tallp_host.size() * sizeof(int32_t));
  cp(D.srun, D.srun_host.data(), D.srun_host.size() * sizeof(int32_t));
  cp(D.trun, D.trun_host.data(), D.trun_host.size() * sizeof(int32_t));
  cp(D.thp, D.thp_host.data(), D.thp_host.size() * sizeof(int32_t));
  if (!D.tabjobs_host.empty()) cp(D.tabjobs, D.tabjobs_host.data(), D.tabjobs_host.size() * sizeof(SgTabJob));
  cp(D.fin_tiles_hp, B.fin_tiles_hp.data(), B.fin_tiles_hp.size() * sizeof(SgSylTile));
  cp(D.frames64, B.frames64.data(), B.frames64.size() * sizeof(SgFrame64));
  cp(D.frames64_tab, B.frames64_tab.data(), B.frames64_tab.size() * sizeof(int64_t));
  cp(D.roots64_wl, B.roots64_wl.data(), B.roots64_wl.size() * sizeof(int32_t));
  cp(D.roots64_off, B.roots64_off.data(), B.roots64_off.size() * sizeof(int64_t));
  cp(D.pieces, B.pieces.data(), B.pieces.size() * sizeof(SgPiece));
  cp(D.syls, B.syls.data(), B.syls.size() * sizeof(SgSyllable));
  cp(D.syl_tiles, B.fin_tiles.data(), B.fin_tiles.size() * sizeof(SgSylTile));
  if (T.direct) {  // direct syllables: their W-reading copy tiles become empty (zero pieces stay)
    std::vector<SgCopyTile> ct(B.copy_tiles);
    for (SgCopyTile& c : ct)
      if (T.direct_syl[(size_t)c.syl] && !(c.flags & SG_COPY_ZERO)) c.n = 0;
    cp(D.copy_tiles, ct.data(), ct.size() * sizeof(SgCopyTile));
    HIPCHK(hipStreamSynchronize(s));  // ct is a temporary
  } else {
    cp(D.copy_tiles, B.copy_tiles.data(), B.copy_tiles.size() * sizeof(SgCopyTile));
  }
  cp(D.ptiles, B.ptiles.data(), B.ptiles.size() * sizeof(SgSylTile));
  cp(D.cknots, B.cknots.data(), B.cknots.size() * sizeof(double));
  cp(D.geoms, B.geoms.data(), B.geoms.size() * sizeof(SgFftGeom));
  cp(D.frames, B.frames[0].data(), B.frames[0].size() * sizeof(SgFrame));
  cp(D.frames + B.frames[0].size(), B.frames[1].data(), B.frames[1].size() * sizeof(SgFrame));
  cp(D.fgroups, B.fgroups.data(), B.fgroups.size() * sizeof(SgFrameGroup));
  cp(D.olas, B.olas_dev.data(), B.olas_dev.size() * sizeof(SgOla));
  cp(D.olatiles, B.olatiles.data(), B.olatiles.size() * sizeof(SgOlaTile));
  cp(D.olasegs, B.olasegs.data(), B.olasegs.size() * sizeof(SgSegment));
  cp(D.items, B.items.data(), B.items.size() * sizeof(SgNoiseItem));
  cp(D.mixes, B.mixes_dev.data(), B.mixes_dev.size() * sizeof(SgMix));
  cp(D.mixtiles, B.mixtiles.data(), B.mixtiles.size() * sizeof(SgMixTile));
  bulk_each(B.fl_x, B.fl, [&](int64_t o, const float* p, int64_t n) { cp(D.fl + o, p, n * sizeof(float)); });
  bulk_each(B.eterms_x, B.eterms,
            [&](int64_t o, const SgEnvTerm* p, int64_t n) { cp(D.eterms + o, p, n * sizeof(SgEnvTerm)); });
  cp(D.ecols, B.ecols.data(), B.ecols.size() * sizeof(SgEnvCol));
  cp(D.envjobs, B.envjobs.data(), B.envjobs.size() * sizeof(SgEnvJob));
  cp(D.envtasks, B.envtasks.data(), B.envtasks.size() * sizeof(SgEnvTask));
  cp(D.elog2, B.elog2.data(), B.elog2.size() * sizeof(double));
  stage("copy_rest");
  launch_amp_build(D, (int64_t)B.ampjobs.size(), s);  // the amplitude blocks, from the jobs just copied
  // gathered noise uniforms: the union of the draw ranges and the item jobs in a
  // temporary buffer, expanded into the uniform area
  void* ug = nullptr;
  if (!B.ujobs.empty()) {
    const size_t ub = up(B.ustream.size() * sizeof(float)), jb = B.ujobs.size() * sizeof(SgUJob);
    HIPCHK(hipMalloc(&ug, ub + jb));
    cp(ug, B.ustream.data(), B.ustream.size() * sizeof(float));
    cp((char*)ug + ub, B.ujobs.data(), jb);
    launch_ugather((const SgUJob*)((char*)ug + ub), (int64_t)B.ujobs.size(), (const float*)ug, D.fl, s);
  }
  HIPCHK(hipStreamSynchronize(s));
  stage("amps_sync");
  if (ug) (void)hipFree(ug);
  while (D.ev_slice.size() < B.slices.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    D.ev_slice.push_back(e);
  }
  if (!D.ev_fork) HIPCHK(hipEventCreateWithFlags(&D.ev_fork, hipEventDisableTiming));
  if (!D.ev_join) HIPCHK(hipEventCreateWithFlags(&D.ev_join, hipEventDisableTiming));
  D.uploaded = true;
}

// the harmonic chain of one plan on stream h: sine banks (four task classes),
// maxima, finalize
static void device_execute_harm(const Batch& B, DevicePlan& D, float* d_out, hipStream_t h,
                                std::vector<SgProfEvent>* prof) {
  // fp64 syllables: their sine-bank tasks and crossfade maxima first, so the
  // slices' per-syllable maxima include them; their finalize after the slices
  launch_sine_bank_hp(D, (int64_t)D.thp_host.size(), h);
  launch_piece_max_hp(D, B.ptile_hp, (int64_t)B.ptiles.size() - B.ptile_hp, h);
  for (size_t c = 0; c < B.slices.size(); ++c) {
    const Slice& sl = B.slices[c];
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof) {
      HIPCHK(hipEventCreate(&e0));
      HIPCHK(hipEventCreate(&e1));
      HIPCHK(hipEventRecord(e0, h));
    }
    {  // the slice's tasks of each class (ascending indices)
      auto range = [&](const std::vector<int32_t>& v, int64_t& k0) {
        const auto lo = std::lower_bound(v.begin(), v.end(), (int32_t)sl.t0);
        const auto hi = std::lower_bound(v.begin(), v.end(), (int32_t)sl.t1);
        k0 = lo - v.begin();
        return (int64_t)(hi - lo);
      };
      int64_t k0 = 0, n = 0;
      n = range(D.tlong_host, k0);
      launch_sine_bank(D, k0, n, h);
      // the runs of the slice's short tasks: [r0, r1) with starts inside [k0, k0 + n)
      auto runs = [&](const std::vector<int32_t>& rs, int64_t a, int64_t n, int64_t& r0) {
        const auto lo = std::lower_bound(rs.begin(), rs.end() - 1, (int32_t)a);
        const auto hi = std::lower_bound(lo, rs.end() - 1, (int32_t)(a + n));
        r0 = lo - rs.begin();
        return (int64_t)(hi - lo);
      };
      int64_t r0 = 0;
      n = range(D.tshort_host, k0);
      if (n > 0) {
        const int64_t nr = runs(D.srun_host, k0, n, r0);
        launch_sine_bank_pairs(D, r0, nr, h);
      }
      n = range(D.tall_host, k0);
      launch_sine_bank_tall(D, k0, n, h);
      n = range(D.tallp_host, k0);
      if (n > 0) {
        const int64_t nr = runs(D.trun_host, k0, n, r0);
        launch_sine_bank_tall_pairs(D, r0, nr, h);
      }
      if (!D.tabjobs_host.empty()) {  // the jobs whose first task lies in the slice, one launch
        const auto& J = D.tabjobs_host;
        const auto lo = std::partition_point(J.begin(), J.end(), [&](const SgTabJob& j) { return j.t0 < sl.t0; });
        const auto hi = std::partition_point(lo, J.end(), [&](const SgTabJob& j) { return j.t0 < sl.t1; });
        int logn = 0;
        for (auto it = lo; it != hi; ++it) logn = std::max<int>(logn, it->logn);
        launch_sine_bank_tab(D, logn, lo - J.begin(), hi - lo, d_out, h);
      }
    }
    if (prof) {
      HIPCHK(hipEventRecord(e1, h));
      prof->push_back({SG_PROF_SINE_BANK, e0, e1});
    }
    launch_piece_max(D, sl.p0, sl.p1 - sl.p0, h);
    launch_syl_max(D, sl.s0, sl.s1 - sl.s0, h);
    launch_harm_copy(D, sl.c0, sl.c1 - sl.c0, d_out, h);
    launch_harm_finalize(D, sl.f0, sl.f1 - sl.f0, d_out, h);
  }
  launch_harm_finalize_hp(D, (int64_t)B.fin_tiles_hp.size(), h);
}

// The harmonic source (sine banks -> maxima -> finalize) and the noise phase
// (envelopes -> noise STFT/OLA) read and write disjoint buffers, so they run
// concurrently: the harmonic chain on s2, the noise phase on s; the pre-filter
// mixes wait for both. SG_OVERLAP=0 runs everything on s (measurement knob).
static bool overlap_on() {
  static const bool on = [] {
    const char* e = std::getenv("SG_OVERLAP");
    return !(e && e[0] == '0');
  }();
  return on;
}

void device_execute(const Batch& B, DevicePlan& D, float* d_out, hipStream_t s, hipStream_t s2,
                    std::vector<SgProfEvent>* prof) {
  std::vector<PlanRun> one{PlanRun{&B, &D, d_out}};
  device_execute_many(one, s, s2, prof);
}

// Plans executed as one batch: one fork, every plan's harmonic chain queued on s2
// back to back, and on s per plan: envelopes, noise phase, wait for that plan's
// harmonic chain, pre-filter mixes, filter phase, final mixes. Plan p + 1's
// harmonic chain thus overlaps plan p's filter phase as well as its own noise
// phase. The plans own disjoint arenas and output slots. Profiling (per-kernel
// events) serialises everything on s.
void device_execute_many(const std::vector<PlanRun>& runs, hipStream_t s, hipStream_t s2,
                         std::vector<SgProfEvent>* prof) {
  const bool ovl = overlap_on() && prof == nullptr && s2 != nullptr && s2 != s;
  if (!ovl) {
    for (const PlanRun& r : runs) {
      device_execute_harm(*r.B, *r.D, r.out, s, prof);
      device_execute_spec(*r.B, *r.D, r.out, s, prof, false);
    }
    HIPCHK(hipGetLastError());
    return;
  }
  // fork: s2 starts after everything already queued on s
  DevicePlan& D0 = *runs[0].D;
  HIPCHK(hipEventRecord(D0.ev_fork, s));
  HIPCHK(hipStreamWaitEvent(s2, D0.ev_fork, 0));
  for (const PlanRun& r : runs) {
    device_execute_harm(*r.B, *r.D, r.out, s2, nullptr);
    HIPCHK(hipEventRecord(r.D->ev_join, s2));
  }
  for (const PlanRun& r : runs) device_execute_spec(*r.B, *r.D, r.out, s, nullptr, true, r.D->ev_join);
  HIPCHK(hipGetLastError());
}

// Spectral phases after the harmonic syllables: noise frames -> noise OLA,
// pre-filter mixes (sounds), filter frames -> filter OLA, final mixes.
void device_execute_spec(const Batch& B, const DevicePlan& D, float* d_out, hipStream_t s,
                         std::vector<SgProfEvent>* prof, bool join, hipEvent_t harm_done) {
  launch_spec_env(D, B, s);  // envelopes and noise filters read by both phases
  // phase: fused STFT/ISTFT/OLA segments, unfused frame groups + OLA tiles, per-OLA maxima
  auto phase = [&](int ph) {
    const int64_t* r = B.fgroup_range[ph];
    const int64_t nseg = B.seg_range[ph][1] - B.seg_range[ph][0];
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof && nseg > 0) {
      HIPCHK(hipEventCreate(&e0));
      HIPCHK(hipEventCreate(&e1));
      HIPCHK(hipEventRecord(e0, s));
    }
    launch_stft_ola(D, ph, B.seg_range[ph][0], nseg, B.fgroup_lds[ph][0], s);
    if (prof && nseg > 0) {
      HIPCHK(hipEventRecord(e1, s));
      prof->push_back({SG_PROF_STFT_OLA, e0, e1});
    }
    launch_fft_frames(D, r[1], r[2] - r[1], B.fgroup_lds[ph][1], s);
    launch_fft_frames64(D, B, ph, s);  // fp64 noise frames (phase 0), fp64 filter frames (phase 1)
    const int64_t t0 = ph == 0 ? 0 : B.olatile_split, t1 = ph == 0 ? B.olatile_split : (int64_t)B.olatiles.size();
    const int64_t o0 = ph == 0 ? 0 : B.ola_split, o1 = ph == 0 ? B.ola_split : (int64_t)B.olas_dev.size();
    launch_ola(D, t0, t1 - t0, s);
    launch_ola_max(D, o0, o1 - o0, s);
  };
  phase(0);
  for (const Batch::Copy& c : B.copies)
    HIPCHK(hipMemcpyAsync(D.fs + c.fs_off, D.fl + c.fl_off, (size_t)c.n * sizeof(float), hipMemcpyDeviceToDevice, s));
  if (join) HIPCHK(hipStreamWaitEvent(s, harm_done, 0));  // the harmonic syllables (fs, out) are final
  launch_mix(D, 0, B.mixtile_hp, d_out, s);
  launch_mix_hp(D, B.mixtile_hp, B.mixtile_split - B.mixtile_hp, s);
  phase(1);
  launch_mix(D, B.mixtile_split, (int64_t)B.mixtiles.size() - B.mixtile_split, d_out, s);
  HIPCHK(hipGetLastError());
}

}  // namespace sg
