// sg_dev.h — plain-old-data descriptors shared by the host planner and the
// gfx950 kernels. Everything here lives in HBM after sg_plan_upload().
#pragma once
#include <stdint.h>

// Phase segment of a syllable: for u in (t0, t1] (1-based samples)
//   integr(u) = cumsum(pitch_up)[u] / samplingRate = c0 + m(c1 + m(c2 + m(c3 + m c4))),  m = u - t0
// i.e. the closed-form prefix sum of the FMM pitch spline piece y + dx(b + dx(c + dx d))
// (R's spline_eval keeps the left piece at an exact knot, R/utilities_soundgen.R:410 via
// stats splines.c; R/source.R:385 cumsum in long double). Coefficients are built in long
// double on the host, divided by samplingRate.
struct SgSeg {
  double t0;
  double c0, c1, c2, c3, c4;
};

// One subharmonic epoch of one syllable (R/source.R:389-427).
//   samples u = u0 + j, j in [0, n): W[j] = sum_r A_r(xo_j) * sin(2*pi*r*integr(u)/D)
//   xo_j = seq.int(x1, xG, length.out = n)[j]  (approx() compressed mapping)
//   A_r(x) = linear interpolation over knots[0..G) of column-major amps[G][R]
struct SgEpoch {
  int64_t w_off;     // scratch offset of W[0]
  int64_t amp_off;   // float offset of the [G][R] amplitude block
  int64_t knot_off;  // double offset of the G knots
  int32_t seg_off;   // first SgSeg of the syllable
  int32_t nseg;
  int32_t n;         // N_e samples
  int32_t G;         // knots / amplitude columns (>= 2)
  int32_t R;         // rows (multiple of SG_ROW_CHUNK, zero padded)
  int32_t u0;        // first sample, 1-based within the syllable
  double x1, xG;     // xout range
  double xby;        // (xG - x1) / (n - 1), as R's seq.int computes it
  double invD;       // 1 / D, D = nSubharm + 1
  // direct-copy window used for the fused max: W[j] lands at syllable
  // sample k = dk0 + j for j in [dj0, dj1) with weight 1.
  int32_t dj0, dj1;
  int64_t dk0;
  int32_t syl;       // syllable index
  int32_t pad;
};

constexpr int SG_ROW_CHUNK = 4;   // amplitude rows per ds_read_b128 (R padded to a multiple)

// One wave task of the sine bank: `len` (<= SG_TASK_MAX) consecutive samples
// j0.. of one epoch that lie in ONE phase segment and whose approx() xout all
// fall in one amplitude interval [knot i, knot i+1] (or in a run of intervals
// whose columns are equal, flag CONST). Everything the wave needs is in this
// record (wave-uniform scalar loads):
//   sample l = j - j0:  m = mbase + l,  integr/D = c0 + m(c1 + m(c2 + m(c3 + m c4)))  (1/D folded in)
//                       t = (tc0 + l * xby) * rdx   (approx() weight inside the interval)
constexpr int SG_TASK_CONST = 1;  // columns equal over the task: A chain only
constexpr int SG_TASK_ENV = 4;    // the syllable has an amplitude envelope (max taken after it)
// tasks with more rows than this (subharmonic sidebands) run in sg_sine_bank_tall:
// fp64 angle and recurrence (parity on the C5 presets with subFreq << f0)
constexpr int SG_ROWS_F32 = 96;
constexpr int SG_TASK_LIN = 2;    // phase segment linear (c2 = c3 = c4 = 0): one fp64 FMA per sample
// fp64 source of an ill-conditioned formant-filter call (planner: filter_conditioning,
// sg_plan_soundgen.cpp): fp64 angle and recurrence, w_off indexes the fp64 epoch scratch W64
constexpr int SG_TASK_HP = 8;
constexpr int SG_TASK_MAX = 1024;  // samples per task (16 slots of 64 lanes)
// short tasks (<= 64 samples) run in runs of consecutive tasks of one syllable, two per
// wave step, one wave per run (sg_sine_bank_pairs / _tall_pairs; round 6)
#ifndef SG_RUN_TASKS
#define SG_RUN_TASKS 8
#endif
struct SgWTask {
  int64_t w_off;       // W offset of epoch sample 0
  int64_t a_off;       // float offset of A[i][0..R)
  int64_t d_off;       // float offset of A[i+1][0..R): dA[i] = A[i+1] - A[i] is formed where the rows are staged
  int64_t dk0;         // syllable sample (0-based) of epoch sample 0
  double c0, c1, c2, c3, c4;  // phase segment (see SgSeg) times invD
  double invD;         // 1 / (nSubharm + 1)
  float rdx, tc0, xby;
  int32_t mbase;       // u(j0) - t0 of the segment
  int32_t R;           // rows (multiple of 16)
  int32_t j0, len;
  int32_t dj0, dj1;    // direct-copy window (fused max)
  int32_t syl;
  int32_t flags;
  int32_t Rn;          // rows the recurrence runs: R without the trailing rows whose A and dA are
                       // all zero (rounded up to 4; they add exact zeros); R keeps the class
};
static_assert(sizeof(SgWTask) == 128, "SgWTask layout");

// Wavetable path of a long span of constant-amplitude, linear-phase tasks (a static
// tone: SG_TASK_CONST | SG_TASK_LIN over thousands of samples, e.g. C2's tones).
// There W(j) = S(x_j) with S(x) = sum_r A_r sin(2 pi r x) a fixed 1-periodic function
// of the phase x_j in cycles. One workgroup per span (sg_sine_bank_tab) tabulates S
// and dS/dx at N = 2^b points per cycle into LDS (one fp32 inverse FFT; each
// interval's cubic Hermite coefficients), then every sample of the span's tasks is
// one table read and three FMAs at its phase, carried per lane as a 32-bit fixed
// point fraction of a cycle (one integer add per 64 samples; rounding <= 2^-33
// cycles per add). The interpolation error is at most
// (2 pi)^4 sum_r |A_r| r^4 / (384 N^4); the planner takes the smallest N in
// [2^8, 2^11] that holds it to SG_TAB_TOL sum_r |A_r| for the span's amplitude
// column (no table if none does), so a rolled-off spectrum gets a small table
// (tests/test_gpu_parity.py: the table path's error against the oracle stays at or
// below the fp32 recurrence's). The table is rebuilt every execute, by every
// workgroup of the span, and a span takes one only with >= 4 N samples.
struct SgTabJob {    // one workgroup: tasks [t0, t0 + n) (consecutive) on one amplitude column
  int64_t a_off;     // the column A[0..Rn)
  int32_t Rn, t0, n, logn;
  int32_t syl, flags;
};
constexpr int SG_TAB_DIRECT = 1;  // the job is a whole syllable of direct pieces: final samples to the output
constexpr int SG_TAB_LOGN_MIN = 8;
constexpr int SG_TAB_LOGN_MAX = 11;   // LDS 20 N bytes: 40 KB
constexpr double SG_TAB_TOL = 1e-7;
constexpr int SG_TAB_TASKS = 64;      // tasks per workgroup at most (a longer span: more workgroups)
// batch slices of the sine-bank / finalize pipeline; measured on MI355X (C2): 4 slices
// on two streams ran 0.41 ms/step against 0.32 for one (both kernels slowed when
// co-resident), so the default is a single slice
constexpr int SG_SLICES = 1;

// A piece of an assembled syllable (crossFade() chain, R/utilities_soundgen.R:328-375):
// value(k) = sum_t (w0 + w1*q + w2*q^2) * W[src_t + q], q = k - start.
constexpr int SG_MAX_TERMS = 4;
struct SgTerm {
  int64_t src;
  float w0, w1, w2, pad;
};
struct SgPiece {
  int64_t start;  // syllable-local sample
  int32_t len;
  int32_t nterms;
  SgTerm t[SG_MAX_TERMS];
};

// Finalize tile of the fast path (sg_harm_copy): `n` (<= SG_COPY_TILE_MAX) samples
// of a syllable without envelope / drift lying in ONE piece that is either a
// direct copy of the epoch waveform or zeros (crossFade's leading 0, 0):
//   out[dst + q] = W[src + q] / max * fade(k0 + q)    (zeros: 0)
// SG_COPY_VEC: source and destination share their 16-B residue (float4 path between
// scalar head and tail).
constexpr int SG_COPY_TILE = 2048;      // planner's merge target
constexpr int SG_COPY_TILE_MAX = 4096;  // kernel limit (16 float4 per lane)
constexpr int SG_COPY_FS = 1;     // destination is the spectral scratch fs
constexpr int SG_COPY_VEC = 2;
constexpr int SG_COPY_ZERO = 4;
struct SgCopyTile {
  int64_t src;       // W offset of the first sample
  int64_t dst;       // destination offset (output buffer, or fs with SG_COPY_FS)
  int64_t k0;        // syllable-local index of the first sample (fades)
  int64_t L;         // syllable length
  int32_t n;
  int32_t max_slot;
  int32_t fade;
  int32_t flags;
  int32_t syl;
  int32_t pad[3];
};
static_assert(sizeof(SgCopyTile) == 64, "SgCopyTile layout");

// Smooth contour over L samples (getSmoothContour(), R/smoothContours.R):
// kind 0 none(=1 after conversion), 1 flat, 2 seq(from,to), 3 fmm spline on
// xout = seq.int(x0, x1, L); then clamp, then optional 2^(v/10).
struct SgContour {
  int32_t kind;
  int32_t nk;        // spline knots
  int64_t k_off;     // offset (doubles) of x[nk], y, b, c, d arrays (5*nk)
  double a, b;       // flat value / seq from,to ; spline x0,x1
  double lo, hi;     // clamp (use -inf/inf when absent)
  double by;         // (b - a) / (L - 1) for the planned length L (device skips the division)
  int64_t L;
  int32_t db;        // 1: apply 2^(v/10)
  int32_t pad;
};

// Piecewise-linear approx() over knots (drift multiplier, R/source.R:459-467).
struct SgLinear {
  int32_t nk;        // 0 = none (multiplier 1)
  int32_t pad;
  int64_t k_off;     // x[nk], y[nk]
  double x0, x1;     // xout = seq.int(x0, x1, L)
};

struct SgSyllable {
  int64_t L;         // assembled length
  int64_t out_off;   // destination offset (final buffer or voiced scratch)
  int32_t piece0, npiece;
  int32_t fade;      // fade length (0/1 = none)
  int32_t max_slot;  // index into the per-syllable max array
  int32_t ntask;     // sine-bank tasks of the syllable: per-task max slots [task0, task0+ntask)
  int64_t task0;
  int32_t ptile0;    // crossfade-piece tiles: per-tile max slots [ptile0, ptile0+nptile)
  int32_t nptile;
  int32_t dst_fs;    // 1: out_off is in the spectral scratch (voiced part of a soundgen() bout)
  int32_t hp;        // 1: fp64 syllable: pieces read W64, out_off indexes the fp64 scratch fh
  SgContour env;     // amplEnvelope (kind 0 = none)
  SgLinear drift;
  // a syllable placed in its bout's sound buffer under the bout's global envelope
  // (amplAnchorsGlobal, R/soundgen.R:721-733): x *= genv at bout sample genv_off + k,
  // the bout genv_len long (kind 0 = none)
  SgContour genv;
  int64_t genv_off, genv_len;
};

// assemble/finalize tiles over syllable samples
struct SgSylTile {
  int32_t syl;
  int32_t piece;     // piece containing k0
  int64_t k0;
  // finalize tiles: per wavefront w (samples k0 + 256 w ...) the piece and the
  // drift-knot interval containing its first sample (planner; no device search)
  int32_t wpiece[4];
  int32_t wdrift[4];
};

// ------------------------------------------------------------------------
// Spectral part: seewave::stft / istft frames, OLA, noise, formant filter.
// Float data (inputs, windows, twiddles, envelopes) live in one fp32 arena
// `fl`; intermediate buffers (frame scratch, sound, raw noise) in `fs`.

constexpr int SG_FFT_MAX_STAGES = 12;
// One complex n-point DFT of sg_fft_frames (SG_FFT_DFT, SG_FFT_ODD geometries):
// a workgroup Stockham FFT when every prime factor of n is <= 31, else
// Bluestein's chirp-z form X_k = c_k sum_j (x_j c_j) conj(c_{k-j}), c_m = exp(-pi i m^2 / n),
// whose convolution runs as two L-point FFTs (L >= 2n - 1, 5-smooth).
struct SgCdft {
  int32_t n;      // points
  int32_t geom;   // geometry index of the FFT of size n (L == 0) or L (its M)
  int32_t L;      // Bluestein length, 0 = plain FFT
  int32_t pad;
  int64_t chirp;  // fl offset: n pairs c_m
  int64_t bf;     // fl offset: L pairs FFT_L(b) / L, b = conj(c) wrapped circularly
};
// FFT geometry of one window length wl = N (even), computed as a complex
// FFT of M = N/2 points (real-input / Hermitian-output packing).
struct SgFftGeom {
  SgCdft cd[2];                    // SG_FFT_DFT: cd[0] = the M-point transform; SG_FFT_ODD: cd[0] = wl points, cd[1] = wl - 1
  int32_t wl, M, nstages, fb;      // fb: frames per workgroup
  int32_t radix[SG_FFT_MAX_STAGES];
  int64_t tw;                      // fl offset: M pairs W_M^t, then M pairs W_N^k (interleaved re, im)
  int64_t win;                     // fl offset: hamming[wl] then hanning[wl] (seewave ftwindow)
  int32_t lds_bytes;
  int32_t kind;                    // SG_FFT_WAVE: one wavefront per frame (sg_fft_wave); SG_FFT_WG: sg_fft_frames
  // n / d == __umulhi(n, ceil(2^32 / d)) exactly for n * d < 2^32 (d > 1);
  // per stage s: d = M / radix[s] and d = Ns (product of the earlier radices)
  uint32_t mr_magic[SG_FFT_MAX_STAGES], ns_magic[SG_FFT_MAX_STAGES];
  uint32_t m_magic, hp_magic;      // d = M, d = M / 2 + 1
  int64_t tws;                     // fl offset: stage-ordered twiddles for sg_fft_wave, (M - 1) pairs:
                                   // stage s at Ns - 1, entry (r - 1) Ns + jm = W_M^(r jm M / (Ns R))
};

constexpr int SG_FFT_WG = 0;
constexpr int SG_FFT_WAVE = 1;
constexpr int SG_FFT_DFT = 2;   // M with a prime factor > 31: Bluestein (SgCdft) in sg_fft_frames
// odd wl (windowLength_points = floor(L / 2) for short sounds, R/soundgen.R:743):
// seewave's stft keeps wl %/% 2 = M rows, istft inverts 2M = wl - 1 points and
// recycles them against the wl-point window (seewave.r:3468-3479). Complex
// wl-point and 2M-point DFTs (cd[0], cd[1]), one frame per sg_fft_frames workgroup
constexpr int SG_FFT_ODD = 3;
constexpr int SG_WAVE_STATE = 24;  // complex butterfly points a lane holds per stage in sg_stft_ola
constexpr int SG_FFT_WAVES = 8;    // wavefronts (segments) per sg_stft_ola workgroup: one workgroup per CU

// sg_stft_ola_noise (no forward FFT: its specialised path fits 168 VGPRs, 3 waves per
// SIMD, and (12 + 4) M pairs of LDS fit 160 KB for every M <= 64 SG_PF_SRC)
#ifndef SG_NOISE_WAVES
#define SG_NOISE_WAVES 12
#endif
constexpr int SG_FFT_WAVES_NOISE = SG_NOISE_WAVES;
constexpr int sg_fft_waves(int phase) { return phase == 0 ? SG_FFT_WAVES_NOISE : SG_FFT_WAVES; }
constexpr int SG_PF_SRC = 20;      // sg_stft_ola register prefetch: sound pairs per lane (M <= 1280)
constexpr int SG_PF_PAIR = 10;     // bin pairs per lane (M / 2 + 1 <= 640)

constexpr int SG_FRAME_FILTER = 0;  // fs sound -> hamming -> FFT/wl -> x env -> ISTFT/wl -> x hann
constexpr int SG_FRAME_NOISE = 1;   // fl uniforms x fl filter (real spectrum)  -> ISTFT/wl -> x hann
struct SgFrame {
  int64_t src;  // FILTER: fs offset of the frame's first sound sample; NOISE: fl offset of nr uniforms
  int64_t env;  // fl offset of the nr envelope (FILTER) / filter (NOISE) values
  int64_t dst;  // fs offset of the wl windowed ISTFT outputs
};
// A formant-filter frame of an ill-conditioned call (sg_fft_frames64): the fp64
// sound fh[src .. src + wl) -> hamming -> fp64 DFT / wl -> x env (fp32 envelope
// area / fl) -> fp64 inverse DFT / 2M -> x hann -> fs[dst .. dst + wl) (fp32, for sg_ola)
// A noise frame of such a call (mode SG_F64_NOISE, generateNoise's istft): the
// real spectrum fl[src + k] x fl[env + k] -> fp64 inverse DFT / 2M -> x hann -> fs.
struct SgFrame64 {
  int64_t src;
  int64_t env;
  int64_t dst;
  int32_t wl;
  int32_t mode;  // SG_F64_FILTER, SG_F64_NOISE
};
constexpr int SG_F64W_M_HOST = 1102;  // sg_fft_frames64w's frame size (sg_fft.hip SG_F64W_M)
constexpr int32_t SG_F64_FILTER = 0;
constexpr int32_t SG_F64_NOISE = 1;
struct SgFrameGroup {  // frames of one workgroup: same geometry and mode
  int32_t geom, mode;
  int32_t f0, nf;
};

// Overlap-add of nframes windowed frames (seewave istft, seewave.r:3462-3484)
// into samples [first, first + len) of the full istft output of length xlen
// (samples outside [0, xlen) are the zero padding of matchLengths()).
struct SgOla {
  int64_t frames;  // fs offset of frame 0 (frames contiguous, wl floats each)
  int64_t out;     // fs offset of output sample `first`
  int64_t first, len, xlen;
  double h;        // hop wl * (100 - overlap) / 100
  int32_t nframes, wl;
  float scale;     // h / sum(hann^2)
  int32_t tile0;   // first per-tile max slot
  int32_t hi;      // h when it is a whole number of samples (integer gather path), else 0
  int32_t nslot;   // max slots [tile0, tile0 + nslot): sg_ola tiles or sg_stft_ola segments
  int32_t fidx;    // index of frame 0 (planner: within its phase; device: in the frame table)
  int32_t fused;   // 1: frames transformed and overlap-added by sg_stft_ola (no frame scratch)
};
constexpr int SG_OLA_TILE = 1024;

// sg_stft_ola work unit: frames [f0, f0 + nf) of one OLA (OLA-relative;
// f0 may start before the segment's own frames to rebuild the overlap
// carried in from earlier frames), owning istft samples [pa, pb).
struct SgSegment {
  int32_t ola, geom, mode;
  int32_t fdev;    // frame-table index of frame f0
  int32_t f0, nf;
  int32_t pa, pb;
  int32_t slot;    // per-segment max slot
  int32_t flags;   // SG_SEG_FIRST: writes the leading zero padding; SG_SEG_LAST: the trailing one
};
constexpr int SG_SEG_FIRST = 1;
constexpr int SG_SEG_LAST = 2;
// target frames owned per segment (one wavefront each), per phase. Shorter segments
// recompute more warm-up frames; round 5 (segments in OLA order) measured shorter ones
// faster because they balanced the workgroups (C5 per launch: noise 48 / 40 / 32 / 24
// frames 2.31 / 2.24 / 2.17 / 2.12 ms, filter 8.05 / 8.01 / 7.96 / 8.11 ms;
// profiles/r05zx_seg_ab.txt). With the segments sorted by length (round 6, SG_SEG_SORT)
// the balance no longer depends on it: noise 24 / 32 / 48 1.975 / 1.912 / 1.880 ms,
// filter 32 / 48 / 64 7.102 / 6.907 / 6.930 ms (profiles/r06za_seglen_ab_*.csv)
#ifndef SG_SEG_NOISE
#define SG_SEG_NOISE 48
#endif
#ifndef SG_SEG_FILTER
#define SG_SEG_FILTER 48
#endif
constexpr int sg_seg_frames(int phase) { return phase == 0 ? SG_SEG_NOISE : SG_SEG_FILTER; }
constexpr int SG_SEG_MIN_FRAMES = 8;  // shortest segment the planner picks (3 recomputed frames each)
constexpr int64_t SG_RESIDENT_WAVES = 256 * SG_FFT_WAVES;  // sg_stft_ola waves resident on a 256-CU MI355X
constexpr int64_t sg_resident_waves(int phase) { return 256 * (int64_t)sg_fft_waves(phase); }
constexpr int SG_CARRY_PAIRS = 16;  // sg_stft_ola carry registers: wl - floor(hop) <= 128 * 16 samples
struct SgOlaTile {
  int32_t ola, pad;
  int64_t q0;  // first sample of the tile (relative to `first`)
};

// Noise uniforms of one noise item copied on the device at upload (sg_ugather):
// fl[dst + j] = us[src + j] for j < n, 0 for n <= j < ntot (us: the union of the
// injected draw ranges the batch reads, as floats)
struct SgUJob {
  int64_t src, dst, n, ntot;
};

// Noise of one syllable, as generateNoise() returns it (R/source.R:124-131):
// matchLengths()-trimmed OLA output / its max * 2^(dB/10) contour, faded.
struct SgNoiseItem {
  int64_t raw;        // fs offset of the trimmed OLA output (len samples)
  int64_t len;
  int64_t off;        // insertion offset inside the mix (addVectors, R/utilities_math.R:500-526)
  int32_t ola;        // its OLA (max slot); < 0: raw samples (no normalisation)
  int32_t fade;       // fadeInOut length (0/1: none)
  int32_t flags;      // host bookkeeping: SG_ITEM_*
  int32_t pad;
  SgContour strength;
};
constexpr int SG_ITEM_FILTER_OLA = 1;  // ola indexes the filter-phase OLAs (shifted at finalize)
constexpr int SG_ITEM_ZERO = 2;        // all-zero content (R's rep(0, len)): layout only
constexpr int SG_ITEM_F64 = 4;         // raw indexes the fp64 scratch fh (voiced part of an fp64 bout)
// One output range: v = base + sum(noise items), * mult contour, * AM trill.
constexpr int SG_BASE_NONE = 0;  // zeros
constexpr int SG_BASE_RAW = 1;   // fs[base + k]
constexpr int SG_BASE_NORM = 2;  // fs[base + k] / olamax[base_ola]  (soundFiltered / max)
struct SgMix {
  int64_t dst;        // destination offset (fs when to_fs, else the output buffer)
  int64_t len;
  int64_t base, base_len;
  int32_t base_kind, base_ola;
  int32_t item0, nitems;
  int32_t to_fs;      // 0: output buffer, 1: fs, 2: fh (fp64 sound of an ill-conditioned filter call)
  int32_t am_lo;      // AM trill: half period of the sigmoid table (0: none)
  int64_t am_tab;     // fl offset of the sigmoid half period
  float am_dep, pad;
  SgContour mult;     // amplAnchorsGlobal envelope (kind 0: none)
};
constexpr int SG_MIX_TILE = 8192;  // samples per sg_mix workgroup (chunks of 2048: descriptors loaded once)
struct SgMixTile {
  int32_t mix, pad;
  int64_t k0;
};

// ------------------------------------------------------------------------
// getSpectralEnvelope() on the device (R/sourceSpectrum.R:507-541). The
// planner restates everything up to the formant tracks in bins (upsampling,
// stochastic formants, mouth opening, nasalization: sg_plan_spec.cpp); per
// column c and track t it emits the log2-density parameters of
//   dgamma(k, shape, rate) / max_k dgamma = 2^(A log2 k - Rr k - Lm),  k = 1..nr
// (A = shape - 1, Rr = rate / ln 2, Lm = the column max in the same units) and
// a bin range [klo, khi] (1-based) that contains every k where the term is
// within 2^-SG_ENV_CUT of the column max. sg_spec_env sums the terms in that range:
//   v(k, c) = (sum_t amp_t 2^(A log2 k - Rr k - Lm)) + lip_c log2 k) * boost_c + slope log2 k
//   env(k, c) = 2^(v / 10)        (fp32, column-major nr x nc)
// with amp_t = formant dB x formantDep, lip_c = rolloffLip x (mouth open),
// boost_c = 2^(mouth x openMouthBoost / 10) and slope = rolloffNoise for a noise
// filter (R/source.R:95-100), 0 for a formant filter.
struct SgEnvTerm {
  double A, Rr, Lm, amp;
  int32_t klo, khi;
  float ampf;  // (float)amp: sg_spec_env reads it as a scalar operand
  int32_t pad;
};
static_assert(sizeof(SgEnvTerm) == 48, "SgEnvTerm layout");
struct SgEnvCol {
  float lip, boost;
};
struct SgEnvJob {
  int64_t out;     // offset of the nr x nc output in the envelope area (fl + fe_base on the device)
  int64_t term0;   // SgEnvTerm of column c, track t: term0 + c * ntr + t
  int64_t col0;    // SgEnvCol of column c: col0 + c
  int32_t nr, nc, ntr;
  float slope;
};
constexpr int SG_ENV_COLS = 8;  // columns per wave task
// Terms below 2^-30 of their own column max are dropped: each changes the dB sum
// by <= |amp| 2^-30 (~6e-8 dB at 60 dB), far below the fp32 resolution of the sum;
// R adds them all (R/sourceSpectrum.R:507-522)
constexpr double SG_ENV_CUT = 30.0;
struct SgEnvTask {
  int32_t job, c0;
};

// ------------------------------------------------------------------------
// 16-bit PCM output (seewave::savewav -> tuneR::normalize -> writeWave), sg_wav.hip
constexpr int SG_PCM_NORMALIZE = 0;  // savewav(wave, f): center, level / max|x|, round(x * 32767)
constexpr int SG_PCM_RESCALE = 1;    // savewav(wave, f, rescale = c(lower, upper))
constexpr int SG_PCM_TILE = 4096;
struct SgPcmCall {
  int64_t off, len;  // the call's samples in the packed buffer (input and output)
};
struct SgPcmTile {
  int32_t call, pad;
  int64_t k0;
};
struct SgPcmStat {
  double mean, level, m, min, max;
  int32_t scale, pad;
};

// ------------------------------------------------------------------------
// Harmonic amplitude matrices built on the device at upload (sg_amp_build,
// SURVEY K3): getRolloff (R/sourceSpectrum.R:71-186), shimmer (R/source.R:
// 316-323) and getVocalFry_per_epoch (R/subharmonics.R:25-86) from per-glottal-
// cycle parameters. The host keeps every integer decision (kept rows, epochs,
// rows per task) and sends 80 B per cycle instead of the [G][R] matrices.
struct SgAmpCol {     // one glottal cycle
  double pitch;       // f0 (Hz) after jitter, drift and clamping
  double slope;       // rolloff + rolloffKHz (pitch - 200) / 1000 (dB/oct)
  double oct;         // rolloffOct (dB/oct per kHz above 200 Hz)
  double mx;          // column max of the thresholded dB (normalisation)
  double sh;          // shimmer factor (1 without shimmer)
  double rph;         // parabolic-rolloff harmonics (R's rounded value)
  double pa, pb, pc;  // parabola a k^2 + b k + c over harmonics k <= rph
  double sbw;         // subharmonic bandwidth subDep (Hz; vocal-fry epochs)
};
struct SgAmpJob {     // one epoch's [G][Rp] amplitude block A
  int64_t amp_off;          // destination in the device amplitude array
  int64_t src_off;          // >= 0: copy [G][Rp] floats from the uploaded source (host-built fallback)
  int64_t col0;             // SgAmpCol of the syllable's glottal cycle 0
  int32_t g0, G;            // the epoch's cycles [g0, g0 + G) of the syllable
  int32_t R, Rp;            // rows computed (ranks 1..R), row stride (padded)
  int32_t H, nsub;          // kept rolloff rows; subharmonics per harmonic (0: plain epoch)
  double thr, nyq, parab, t01, baseline;  // throwaway (dB), sr / 2, rolloffParab, 2^(throwaway / 10), 200 Hz
  int32_t any_oct, pad;
};
