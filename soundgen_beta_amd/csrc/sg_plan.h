// sg_plan.h — host planner: turns R-level calls into device descriptors.
// All integer bookkeeping (glottal cycles, gcLen, epochs, kept rows, zero-
// crossing trims, output lengths) is done here in fp64, bit-exact with R.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <utility>
#include <vector>

#include "sg_dev.h"
#include "sg_rmath.h"
#include "soundgen_hip.h"

namespace sg {

// Allocator whose resize() leaves new elements default-initialised (no zero
// fill): the planner's bulk arrays are always written after they grow, and the
// merged batch is filled by parallel copies (first touch on the copying thread).
// Blocks of SG_BULK_HUGE and up come from bulk_alloc (huge pages, sg_rmath.h).
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind { using other = NoInitAlloc<U>; };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  T* allocate(size_t n) {
    if (n * sizeof(T) < SG_BULK_HUGE) return std::allocator<T>::allocate(n);
    return static_cast<T*>(bulk_alloc(n * sizeof(T)));
  }
  void deallocate(T* p, size_t n) noexcept {
    if (n * sizeof(T) < SG_BULK_HUGE) std::allocator<T>::deallocate(p, n);
    else bulk_free(p, n * sizeof(T));
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
  template <class U>
  void construct(U* p) noexcept { ::new ((void*)p) U; }
};
template <class T>
using bulk = std::vector<T, NoInitAlloc<T>>;

// The largest bulk arrays of a merged batch stay in the planning parts' blocks
// (merge_parts moves them, no copy): blocks[i] holds elements [base[i],
// base[i] + blocks[i].size()) of the logical array, which continues with the
// Batch's own vector from n on. A batch planned in one piece has no blocks.
template <class T>
struct Blocks {
  std::vector<bulk<T>> blocks;
  std::vector<int64_t> base;
  int64_t n = 0;
};
template <class T>
inline int64_t bulk_size(const Blocks<T>& x, const bulk<T>& v) {
  return x.n + (int64_t)v.size();
}
// f(first element index, pointer, count) for every block, then the vector
template <class T, class F>
inline void bulk_each(const Blocks<T>& x, const bulk<T>& v, F&& f) {
  for (size_t i = 0; i < x.blocks.size(); ++i)
    if (!x.blocks[i].empty()) f(x.base[i], x.blocks[i].data(), (int64_t)x.blocks[i].size());
  if (!v.empty()) f(x.n, v.data(), (int64_t)v.size());
}
template <class T>
inline const T& bulk_at(const Blocks<T>& x, const bulk<T>& v, int64_t i) {  // debugging paths only
  if (i >= x.n) return v[(size_t)(i - x.n)];
  size_t lo = 0, hi = x.base.size() - 1;
  while (lo < hi) {
    const size_t m = (lo + hi + 1) / 2;
    if (x.base[m] <= i) lo = m; else hi = m - 1;
  }
  return x.blocks[lo][(size_t)(i - x.base[lo])];
}

struct DeviceArrays;  // sg_api.cpp

// FFT/OLA job of the noise source or the formant filter (seewave istft/stft)
struct SgFftJob;

// A slice of the batch (whole syllables) launched as one unit so that the
// HBM-bound finalize of slice c overlaps the VALU-bound sine bank of c+1.
struct Slice {
  int64_t t0, t1;    // sine-bank tasks
  int32_t p0, p1;    // crossfade-piece max tiles
  int32_t s0, s1;    // syllables
  int64_t f0, f1;    // finalize tiles (general path, fin_tiles)
  int64_t c0, c1;    // finalize tiles (fast path, copy_tiles)
};

struct Batch {
  // draws_only: a planning pass that only consumes each call's random draws in the
  // reference's order and raises the errors that precede its last draw, emitting
  // nothing (sg_node's recording pass over one R stream: the per-sample work after a
  // call's last draw -- amplitude columns, phase segments, wave tasks, envelope terms,
  // frames, mixes -- runs once, in the parallel replay)
  bool draws_only = false;
  // ---- harmonic source ----
  bulk<SgSeg> segs;
  bulk<SgEpoch> epochs;
  bulk<double> knots;
  // amplitude blocks: device-only (amp_total floats, sg_amp_build at upload) from
  // one SgAmpJob per epoch: the formula over ampcols, or a copy of ampsrc
  int64_t amp_total = 0;
  bulk<SgAmpCol> ampcols;
  std::vector<SgAmpJob> ampjobs;
  bulk<float> ampsrc;         // host-built [G][Rp] blocks (the fallback path)
  int64_t amp_lg_rows = 0;    // largest H: the log2 table the device formula reads
  bulk<SgWTask> tasks;
  bulk<SgPiece> pieces;
  std::vector<SgSyllable> syls;
  bulk<SgSylTile> syl_tiles;
  std::vector<SgSylTile> fin_tiles;    // derived (finalize_plan): syl_tiles the fast path does not take
  std::vector<SgCopyTile> copy_tiles;  // derived (finalize_plan): fast-path finalize tiles
  std::vector<SgSylTile> ptiles;   // tiles over multi-term (crossfade) pieces: [fp32 syllables..., fp64 syllables...]
  int64_t ptile_hp = 0;            // derived: first ptile of an fp64 syllable
  std::vector<SgSylTile> fin_tiles_hp;  // derived: finalize tiles of fp64 syllables (sg_harm_finalize_hp)
  std::vector<Slice> slices;
  // ---- spectral part (noise, formant filter, assembly) ----
  bulk<float> fl;                 // host-initialised floats (windows, twiddles, uniforms, envelopes, ...)
  int64_t fs_total = 0;                  // scratch floats (frames, sounds, raw noise)
  std::vector<SgFftGeom> geoms;
  std::vector<SgFrame> frames[2];        // [0] noise frames, [1] filter frames
  std::vector<int32_t> frame_geom[2];
  std::vector<SgOla> olas[2];            // [0] noise OLAs, [1] filter OLAs (device: [0] then [1])
  std::vector<SgFrame64> frames64;       // filter / noise frames of fp64 (ill-conditioned) bouts: sg_fft_frames64
  // derived (finalize_spec): the window lengths of the fp64 frames, their root tables
  // W_N^t (offsets in double2 units), each frame's table offset, the largest window
  std::vector<int32_t> roots64_wl;
  std::vector<int64_t> roots64_off, frames64_tab;
  int64_t roots64_total = 0;
  int32_t frames64_maxwl = 0;
  int64_t frames64_noise = 0;  // finalize_spec: frames64 holds the noise frames first
  // per phase: its leading frames of wl = 2204, one per wavefront in sg_fft_frames64w (the rest: sg_fft_frames64)
  int64_t frames64_w[2] = {0, 0};
  std::vector<SgNoiseItem> items;        // items[].ola indexes the device OLA table
  std::vector<SgMix> mixes[2];           // [0] pre-filter sounds (fs), [1] final output
  struct Copy { int64_t fl_off, fs_off, n; };
  std::vector<Copy> copies;              // fl -> fs before the filter phase
  // derived (finalize_spec)
  std::vector<SgFrameGroup> fgroups;
  // per phase (0 noise, 1 filter): groups [r1, r2) run sg_fft_frames ([r0, r1) empty: wavefront-kernel
  // geometries run fused in sg_stft_ola, fgroup_lds[ph][0] = its dynamic LDS)
  int64_t fgroup_range[2][3] = {{0, 0, 0}, {0, 0, 0}};
  int fgroup_lds[2][2] = {{0, 0}, {0, 0}};  // max dynamic LDS per phase and kernel
  std::vector<SgOla> olas_dev;
  std::vector<SgOlaTile> olatiles;
  int64_t olatile_split = 0, ola_split = 0;
  std::vector<SgSegment> olasegs;        // sg_stft_ola work units, SG_FFT_WAVES per workgroup
  int32_t n_segslots = 0;                // real (non-padding) segments: max slots after the tile slots
  int64_t seg_range[2][2] = {{0, 0}, {0, 0}};
  std::vector<SgMix> mixes_dev;
  std::vector<SgMixTile> mixtiles;
  int64_t mixtile_split = 0;
  int64_t mixtile_hp = 0;                // pre-filter tiles [mixtile_hp, mixtile_split) write fh (sg_mix_hp)
  bulk<double> cknots;   // contour / linear knot data
  int64_t w_total = 0;          // epoch-waveform scratch (floats)
  int64_t w64_total = 0;        // fp64 epoch-waveform scratch W64 (doubles; SG_TASK_HP tasks)
  int64_t fh_total = 0;         // fp64 sound scratch fh (doubles): voiced parts and sounds of fp64 bouts
  int64_t hp_bouts = 0;         // bouts whose formant filter runs the fp64 path
  int64_t hp_noise_bouts = 0;   // bouts whose pre-filter noise runs the fp64 frame kernel
  // device spectral envelopes (sg_spec_env): per-column/track terms, per-column
  // factors, jobs; outputs in the envelope area (fe_total floats after fe_base,
  // the end of the uploaded fl floats, fixed at finalize_spec). Until then a
  // frame's env < 0 encodes envelope-area offset -(env + 1).
  bulk<SgEnvTerm> eterms;
  // merged batch: the parts' blocks ahead of segs, tasks, fl, eterms (Blocks)
  Blocks<SgSeg> segs_x;
  Blocks<float> fl_x;
  Blocks<SgWTask> tasks_x;
  Blocks<SgEnvTerm> eterms_x;
  std::vector<SgEnvCol> ecols;
  std::vector<SgEnvJob> envjobs;
  int64_t fe_total = 0, fe_base = 0;
  std::vector<SgEnvTask> envtasks;  // derived (finalize_spec)
  // generateNoise()'s runif(nr * nc) read from an injected draw array are not
  // copied per item: the item records the caller's range and its offset in the
  // uniform area (fu_total floats after fu_base, device-only, after the envelope
  // area); finalize_spec copies the union of the ranges once (ustream, floats) and
  // sg_ugather expands the items at upload. Until then a noise frame's src < 0
  // encodes uniform-area offset -(src + 1).
  struct UGather {
    const double* src;
    int64_t n, dst, ntot;
  };
  std::vector<UGather> ugath;
  int64_t fu_total = 0, fu_base = 0;
  std::vector<float> ustream;  // derived (finalize_spec)
  std::vector<SgUJob> ujobs;   // derived (finalize_spec)
  std::vector<double> elog2;        // derived: log2(k), k = 1..max nr
  // ---- per call ----
  std::vector<int64_t> call_len, call_off;
  std::vector<int32_t> call_status;
  std::vector<int32_t> call_fp64;   // bouts of the call on the fp64 filter path
  std::vector<double> call_rho;     // the largest conditioning estimate over the call's filtered bouts
  double rho_cur = 0;               // (the call being planned)
  std::vector<double> call_rho_noise;  // the same for the pre-filter noise of its filtered bouts
  double rho_noise_cur = 0;
  std::vector<std::string> call_msg;
  int64_t total_out = 0;
  // ---- stats ----
  int64_t harm_samples = 0, harm_terms = 0, harm_amp_bytes = 0, fft_frames = 0;
  double fft_flops = 0;                      // nominal 5 wl log2 wl per transform, every frame path
  std::vector<double> call_rows, call_flops;  // per call: sine-bank (sample, row) terms, FFT flops
  int64_t stft_bytes = 0, stft_samples = 0;  // sg_stft_ola: algorithmic bytes, trimmed output samples
  double stft_flops = 0;                     // sg_stft_ola: nominal 5 wl log2 wl per transform
};

// Plan one generateHarmonics() call; the finalized syllable is written at
// `out_off` of the output buffer. Returns the syllable length.
// to_fs: the syllable goes to a fresh spectral-scratch region (*fs_off), the
// voiced part of a soundgen() bout, instead of the output buffer.
// A glottal cycle's harmonic spectrum sampled by the planner (formant-filter
// conditioning, sg_plan_soundgen.cpp): syllable sample, f0, row amplitudes (linear)
struct HarmProbe {
  int64_t t;
  double f0;
  std::vector<double> amp;
};
// With to_fs, out_off & 3 is the residue (mod 4 floats) of the fs slot allocated.
int64_t plan_harmonics(Batch& B, const double* pitch, int64_t len, const sg_harm_params& P,
                       const sg_anchors& amplAnchors, Rng& R, int64_t out_off, bool dry_run, bool to_fs = false,
                       int64_t* fs_off = nullptr, std::vector<HarmProbe>* probes = nullptr);
// Move syllable s (planned to fs) to the fp64 path: epochs' waveforms to W64,
// its tasks flagged SG_TASK_HP, output to a fresh fh region; returns that offset.
int64_t syllable_to_fp64(Batch& B, int s);
int64_t fh_alloc(Batch& B, int64_t n);

// getSmoothContour() for the lengths/values the planner needs on the host.
// method: 0 loess (default; 3-10 anchors -> sg_loess), 1 spline. sr is the
// call site's samplingRate (loess span depends on len / sr). Returns false
// for R's NA.
bool smooth_contour(const sg_anchors& an, int64_t len, bool thisIsPitch, int method, bool has_floor,
                    double vfloor, bool has_ceil, double vceil, vec& out, double sr = 16000);
// Device contour descriptor for getSmoothContour(len = L) (no host expansion;
// a loess contour becomes piecewise cubic knots at the k-d tree vertices)
SgContour contour_desc(Batch& B, const sg_anchors& an, int64_t L, bool has_floor, double vfloor,
                       bool has_ceil, double vceil, bool db, double sr);

void tile_syllables(Batch& B, int first_syl);

// Plan one soundgen() call (R/soundgen.R:208-862); returns the bout length.
int64_t plan_soundgen(Batch& B, const sg_soundgen_args& a, Rng& R, int64_t out_off, int first_syl);
// Roll back soundgen-specific batch state after a failed call.
void restore_soundgen_tail(Batch& B, int first_syl);
// Build derived tables (piece tiles) once all calls are planned.
void finalize_plan(Batch& B);
void finalize_spec(Batch& B);

// ---- spectral planning (sg_plan_spec.cpp) ----
// FFT geometry of window length wl (cached per wl); SG_E_UNSUPPORTED if
// wl/2 has a prime factor > 31.
int geometry(Batch& B, int wl);
int64_t fs_alloc(Batch& B, int64_t n);
int64_t fl_push(Batch& B, const double* v, int64_t n);
// STFT(hamming) x env -> ISTFT(hann) of the fs sound [sound, sound + L)
// (R/soundgen.R:743-806). env: nr x env_nc (column-major) at fl offset env
// (>= 0) or envelope-area offset -(env + 1) (< 0); returns the
// filter OLA index (phase 1); *out_len = istft length.
// hp: the sound is in fh (fp64) and the frames run sg_fft_frames64 (unfused)
int plan_filter(Batch& B, int64_t sound, int64_t L, int wl, double overlap, int64_t env, int64_t env_nc,
                int64_t* out_len, int64_t* out_fs, bool hp = false);
// generateNoise(), R/source.R:57-138: returns a noise item (off = 0);
// ok == false when the noise contour is NA (R returns zeros). filterNoise: host
// nr x fnc matrix; or filt_env < 0: a device envelope job (envelope-area
// offset -(filt_env + 1), fnc columns) that already includes the rolloffNoise slope.
bool plan_noise(Batch& B, Rng& R, int64_t len, const sg_anchors& noiseAnchors, double rolloffNoise,
                double attackLen, int wl, double sr, double overlap, const double* filterNoise, int64_t fnc,
                SgNoiseItem* item, int64_t filt_env = 0);
// The noise items of an ill-conditioned bout (their OLAs, phase 0, the last
// noises planned) on the fp64 frame kernel: the frames move from the phase-0
// list to frames64 (SG_F64_NOISE) and the OLAs read their scratch (sg_ola).
// False (nothing changed) when a window does not suit sg_fft_frames64.
bool noise_to_fp64(Batch& B, const std::vector<int>& olas);
// getSpectralEnvelope(), R/sourceSpectrum.R:261-566: the host part (tracks,
// draws) plus one sg_spec_env job computing the nr x nc matrix on the device;
// returns its envelope-area offset encoded as -(offset + 1). slope: dB per
// log2(bin) added after the boost (the noise rolloff, R/source.R:95-100).
// nrd = windowLength_points / 2 as R passes it (x.5 for an odd window: the
// matrix has as.integer(nrd) rows, bin_width uses nrd)
int64_t plan_envelope(Batch& B, Rng& R, double nrd, int64_t nc, const sg_formants* F, double formantDep,
                      double rolloffLip, const sg_anchors& mouthAnchors, double mouthOpenThres, double openMouthBoost,
                      double vocalTract, double temperature, double formDrift, double formDisp,
                      double formantDepStoch, double smoothLinearFactor, double sr, double speedSound,
                      double slope = 0);
vec sigmoid_half(double sr, double freq, double shape, double spikiness);

// getRolloff() with per-gc vector parameters (R/sourceSpectrum.R:71-186)
vec get_rolloff(const vec& pitch, int64_t nH, const vec& rolloff, const vec& rolloffOct, double rolloffParab,
                double rolloffParabHarm, const vec& rolloffKHz, double baseline, double throwaway, double sr,
                int64_t& H, double rolloffParabCeiling = NAN);  // NaN: NULL
vec get_random_walk(Rng& R, int64_t len, double rw_range, double rw_smoothing, int method, const vec& trend,
                    bool trend_lazy_rnorm, bool draws_only = false);
void clumper(vec& s, const vec& minLen);
double noise_threshold(int which, double nonlinBalance);

}  // namespace sg

namespace sg {
// sg_plan_batch with the draw-independence of the calls stated by the caller:
// independent_draws = every call's callbacks replay that call's own recorded
// draws (sg_node.cpp), so the batch may plan on host threads like injected draws
// max_threads > 0 caps the host threads (sg_node: one core records R's stream meanwhile)
int plan_batch_ex(sg_ctx* ctx, const sg_call_desc* calls, int64_t n_calls, bool independent_draws, sg_plan** out,
                  int max_threads = 0);
// The calls' draws in call order without planning their device work (Batch::draws_only):
// per call status (0 or SG_E_*) and message; a failing call ends a callback stream
// on_call(i, status) after each call (its draws recorded), on the calling thread
void record_draws(const sg_call_desc* calls, int64_t n_calls, std::vector<int32_t>& status,
                  std::vector<std::string>& msg, const std::function<void(int64_t, int32_t)>& on_call = {});
}  // namespace sg
