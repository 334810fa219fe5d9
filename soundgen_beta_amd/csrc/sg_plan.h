// sg_plan.h — host planner: turns R-level calls into device descriptors.
// All integer bookkeeping (glottal cycles, gcLen, epochs, kept rows, zero-
// crossing trims, output lengths) is done here in fp64, bit-exact with R.
#pragma once
#include <cstdint>
#include <vector>

#include "sg_dev.h"
#include "sg_rmath.h"
#include "soundgen_hip.h"

namespace sg {

struct DeviceArrays;  // sg_api.cpp

// FFT/OLA job of the noise source or the formant filter (seewave istft/stft)
struct SgFftJob;

// A slice of the batch (whole syllables) launched as one unit so that the
// HBM-bound finalize of slice c overlaps the VALU-bound sine bank of c+1.
struct Slice {
  int64_t t0, t1;    // sine-bank tasks
  int32_t p0, p1;    // crossfade-piece max tiles
  int32_t s0, s1;    // syllables
  int64_t f0, f1;    // finalize tiles
};

struct Batch {
  // ---- harmonic source ----
  std::vector<SgSeg> segs;
  std::vector<SgEpoch> epochs;
  std::vector<double> knots;
  std::vector<float> amps;
  std::vector<SgWTask> tasks;
  std::vector<SgPiece> pieces;
  std::vector<SgSyllable> syls;
  std::vector<SgSylTile> syl_tiles;
  std::vector<SgSylTile> ptiles;   // tiles over multi-term (crossfade) pieces
  std::vector<Slice> slices;
  std::vector<double> cknots;   // contour / linear knot data
  int64_t w_total = 0;          // epoch-waveform scratch (floats)
  // ---- per call ----
  std::vector<int64_t> call_len, call_off;
  std::vector<int32_t> call_status;
  std::vector<std::string> call_msg;
  int64_t total_out = 0;
  // ---- stats ----
  int64_t harm_samples = 0, harm_terms = 0, harm_amp_bytes = 0, fft_frames = 0;
};

// Plan one generateHarmonics() call; the finalized syllable is written at
// `out_off` of the output buffer. Returns the syllable length.
int64_t plan_harmonics(Batch& B, const double* pitch, int64_t len, const sg_harm_params& P,
                       const sg_anchors& amplAnchors, Rng& R, int64_t out_off, bool dry_run);

// getSmoothContour() for the lengths/values the planner needs on the host.
// method: 0 loess (default; only 1, 2 or >10 anchors supported), 1 spline.
// Returns false for R's NA.
bool smooth_contour(const sg_anchors& an, int64_t len, bool thisIsPitch, int method, bool has_floor,
                    double vfloor, bool has_ceil, double vceil, vec& out);
// Device contour descriptor for getSmoothContour(len = L) (no host expansion)
SgContour contour_desc(Batch& B, const sg_anchors& an, int64_t L, bool has_floor, double vfloor,
                       bool has_ceil, double vceil, bool db);

void tile_syllables(Batch& B, int first_syl);

// Plan one soundgen() call (R/soundgen.R:208-862); returns the bout length.
int64_t plan_soundgen(Batch& B, const sg_soundgen_args& a, Rng& R, int64_t out_off, int first_syl);
// Roll back soundgen-specific batch state after a failed call.
void restore_soundgen_tail(Batch& B, int first_syl);
// Build derived tables (piece tiles) once all calls are planned.
void finalize_plan(Batch& B);

// getRolloff() with per-gc vector parameters (R/sourceSpectrum.R:71-186)
vec get_rolloff(const vec& pitch, int64_t nH, const vec& rolloff, const vec& rolloffOct, double rolloffParab,
                double rolloffParabHarm, const vec& rolloffKHz, double baseline, double throwaway, double sr,
                int64_t& H);
vec get_random_walk(Rng& R, int64_t len, double rw_range, double rw_smoothing, int method, const vec& trend,
                    bool trend_lazy_rnorm);
void clumper(vec& s, const vec& minLen);

}  // namespace sg
