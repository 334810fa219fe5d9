/*
 * soundgen_hip.h — C-ABI of libsoundgen_hip.so, the MI355X-native engine for
 * soundgen's additive-source + formant-filter hot path.
 *
 * Reference interfaces this ABI replaces (nemochina2008/soundgen_beta, R):
 *   soundgen()            R/soundgen.R:208-862   -> sg_soundgen / sg_plan_batch+sg_execute
 *   generateHarmonics()   R/source.R:173-471     -> sg_generate_harmonics
 *   generateNoise()       R/source.R:57-138      -> sg_generate_noise
 *   getSpectralEnvelope() R/sourceSpectrum.R:261-566 -> sg_spectral_envelope
 *   getRolloff()          R/sourceSpectrum.R:71-186  -> sg_get_rolloff (host helper)
 *   seewave::stft/istft + z*env (R/soundgen.R:779-806) -> sg_formant_filter
 *
 * Conventions (mirroring R's .Call world):
 *   - plain pointers + sizes, doubles on the host side (R numeric vectors);
 *   - every function returns 0 or a negative SG_E_* code; no C++ exception
 *     ever crosses this boundary; sg_last_error() gives the message;
 *   - random draws are INJECTED (R draws them in the reference's order and
 *     passes them in): standard normals and standard uniforms are consumed
 *     sequentially in R's draw order (see DESIGN.md "Randomness").
 *   - "NA" anchors/formants are encoded as n == 0; NULL scalars as NaN.
 */
#ifndef SOUNDGEN_HIP_H
#define SOUNDGEN_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_ABI_VERSION 5

enum {
  SG_OK = 0,
  SG_E_ARG = -1,         /* invalid argument (R: stop()) */
  SG_E_DOMAIN = -2,      /* R would error inside approx()/spline() etc. */
  SG_E_RANDOM = -3,      /* injected random stream exhausted */
  SG_E_UNSUPPORTED = -4, /* valid in R but not yet supported (e.g. loess) */
  SG_E_DEVICE = -5,      /* HIP runtime error */
  SG_E_CAPACITY = -6,    /* output buffer too small */
  SG_E_NOMEM = -7
};

/* A data.frame(time, value) of anchors. n == 0 encodes NA / NULL. */
typedef struct sg_anchors {
  int32_t n;
  const double* time;
  const double* value;
} sg_anchors;

/* A list of formants, each a data.frame(time, freq, amp, width) with
 * n_points[f] rows; arrays are concatenated over formants. n_formants == 0
 * encodes NA. f1_index is the position of the formant named "f1" (-1 if
 * absent; needed by the nasalization branch, R/sourceSpectrum.R:469-504). */
typedef struct sg_formants {
  int32_t n_formants;
  int32_t f1_index;
  const int32_t* n_points;
  const double* time;
  const double* freq;
  const double* amp;
  const double* width;
} sg_formants;

/* Random draws, consumed in the reference's draw order: standard normals
 * (rnorm), standard uniforms (runif) and gamma variates (rgamma). The arrays
 * are used first; once one is exhausted (or NULL) the matching callback is
 * called if set, else the call fails with SG_E_RANDOM. The R shim binds the
 * callbacks to R's own norm_rand()/unif_rand()/rgamma() so that draws follow
 * set.seed() exactly; tests inject arrays.
 * unif_n_cb (ABI 5, may be NULL): n consecutive uniforms into out, the same
 * values n unif_cb calls would return -- R: runif(n), i.e. unif_rand() in one C
 * loop. The planner takes generateNoise()'s runif(nr * nc) (R/source.R:111; ~8 k
 * draws per C5 call) through it in blocks instead of one callback per draw. */
typedef struct sg_random {
  const double* normals;
  int64_t n_normals;
  const double* uniforms;
  int64_t n_uniforms;
  double (*norm_cb)(void* user);
  double (*unif_cb)(void* user);
  double (*gamma_cb)(void* user, double shape, double rate);
  void* user;
  void (*unif_n_cb)(void* user, double* out, int64_t n);
} sg_random;

/* R's default random number generation (R 3.4.0: Mersenne-Twister,
 * Inversion normals), so that a seeded call draws what
 * `set.seed(seed); soundgen(...)` draws in R without R present. Replaces the
 * R runtime's unif_rand / norm_rand / exp_rand / rgamma (src/main/RNG.c,
 * src/nmath/{snorm,qnorm,sexp,rgamma}.c) reached by the reference through
 * runif/rnorm/rgamma calls, e.g. R/source.R:111, :278, :349,
 * R/utilities_math.R:212, :295, R/sourceSpectrum.R:384. sg_random_bind_rrng
 * points an sg_random's callbacks at one generator (one stream, so R's
 * interleaving of the draw kinds is kept). */
typedef struct sg_rrng sg_rrng;
int sg_rrng_create(int32_t seed, sg_rrng** out);  /* = set.seed(seed) */
void sg_rrng_destroy(sg_rrng* g);
void sg_rrng_set_seed(sg_rrng* g, int32_t seed);
double sg_rrng_unif(sg_rrng* g);                  /* runif(1) */
void sg_rrng_unif_n(sg_rrng* g, double* out, int64_t n); /* runif(n) (ABI 5) */
double sg_rrng_norm(sg_rrng* g);                  /* rnorm(1) */
double sg_rrng_exp(sg_rrng* g);                   /* rexp(1) */
double sg_rrng_gamma(sg_rrng* g, double shape, double scale); /* rgamma(1, shape, scale = scale) */
void sg_random_bind_rrng(sg_random* r, sg_rrng* g);

/* Formals of generateHarmonics(), R/source.R:173-205 (pitch and amplAnchors
 * are separate arguments). */
typedef struct sg_harm_params {
  double attackLen, nonlinBalance, nonlinDep, jitterDep, jitterLen;
  double vibratoFreq, vibratoDep, shimmerDep, creakyBreathy;
  double rolloff, rolloffOct, rolloffKHz, rolloffParab, rolloffParabHarm;
  double rolloffLip, rolloff_perAmpl, temperature, pitchDriftDep;
  double pitchDriftFreq, randomWalk_trendStrength, shortestEpoch, subFreq;
  double subDep, amDep, amFreq, overlap, samplingRate, pitchFloor;
  double pitchCeiling, pitchSamplingRate, throwaway;
} sg_harm_params;

/* Formals of soundgen(), R/soundgen.R:208-277. tempEffects is flattened in
 * the order sylLenDep, formDrift, formDisp, pitchDriftDep, pitchDriftFreq,
 * pitchAnchorsDep, noiseAnchorsDep, amplAnchorsDep. vocalTract NaN = NULL. */
typedef struct sg_soundgen_args {
  double repeatBout, nSyl, sylLen, pauseLen;
  sg_anchors pitchAnchors, pitchAnchorsGlobal;
  double temperature;
  double tempEffects[8];
  double maleFemale, creakyBreathy, nonlinBalance, nonlinDep;
  double jitterLen, jitterDep, vibratoFreq, vibratoDep, shimmerDep;
  double attackLen, rolloff, rolloffOct, rolloffKHz, rolloffParab;
  double rolloffParabHarm, rolloffLip;
  sg_formants formants;
  double formantDep, formantDepStoch, vocalTract;
  double subFreq, subDep, shortestEpoch, amDep, amFreq, amShape;
  sg_anchors noiseAnchors;
  sg_formants formantsNoise;
  double rolloffNoise;
  sg_anchors mouthAnchors, amplAnchors, amplAnchorsGlobal;
  double samplingRate, windowLength, overlap, addSilence;
  double pitchFloor, pitchCeiling, pitchSamplingRate, throwaway;
  int32_t invalidArgAction; /* 0 adjust, 1 abort, 2 ignore */
  /* max(unlist(lapply(formantsNoise, length))) evaluated on the caller's own
   * formantsNoise (R/soundgen.R:662-663): 1 for a vowel string, the number of
   * fields (4) for a list of formant lists. Noise formants are "moving" (one
   * envelope column per 10 ms) when it exceeds 1 or the mouth moves.
   * 0 = not supplied: treated as a list of formant lists (moving). */
  int32_t formantsNoise_rlen;
} sg_soundgen_args;

/* One call of a batch: either a whole soundgen() call or a bare
 * generateHarmonics() call on a given pitch contour. */
enum { SG_CALL_SOUNDGEN = 0, SG_CALL_HARMONICS = 1 };
typedef struct sg_call_desc {
  int32_t kind;
  /* SG_CALL_SOUNDGEN */
  const sg_soundgen_args* args;
  /* SG_CALL_HARMONICS */
  const double* pitch;
  int64_t pitch_len;
  const sg_harm_params* harm;
  sg_anchors amplAnchors;
  /* random draws for this call (both kinds) */
  sg_random random;
} sg_call_desc;

typedef struct sg_ctx sg_ctx;
typedef struct sg_plan sg_plan;

/* ---- context ---------------------------------------------------------- */
int sg_ctx_create(int device, sg_ctx** out);
void sg_ctx_destroy(sg_ctx* ctx);
const char* sg_last_error(const sg_ctx* ctx);
int sg_abi_version(void);
/* Fill the defaults of generateHarmonics()/soundgen() formals. */
void sg_default_harm_params(sg_harm_params* p);
void sg_default_soundgen_args(sg_soundgen_args* a);

/* ---- whole-node batch path: one process, several devices (ABI 3) --------
 * Replaces the single-device loop behind the R batch callers that north_star
 * keeps: soundgen_batch(), morph() (R/morph.R:200-208) and matchPars()
 * (R/matchPars.R:168-202), each a list of independent soundgen() calls.
 * A node is a list of device ordinals (a device may appear more than once;
 * NULL: 0 .. n - 1, and n <= 0 with NULL: every visible device). Planning needs
 * no device; each device's context is created on first execution. */
typedef struct sg_node sg_node;
typedef struct sg_node_plan sg_node_plan;
int sg_device_count(void);
int sg_node_create(const int32_t* devices, int32_t n, sg_node** out);
void sg_node_destroy(sg_node* node);
int32_t sg_node_size(const sg_node* node);
const char* sg_node_last_error(const sg_node* node);
/* Calls are assigned to the node's devices by LPT over an analytic cost per
 * call (samples x kept harmonic rows, STFT frames, per-sample assembly); each
 * device's shard is planned as one sg_plan. Lengths, offsets, statuses and
 * messages are those of the WHOLE batch in call order with sg_plan_batch's
 * layout, and every call's samples equal what sg_plan_batch of the whole batch
 * produces (a call's arithmetic does not depend on the batch around it). With
 * draw callbacks (R's RNG) the calls are first run in call order in a draws-only
 * pass that records each call's draws -- R's stream, R's order; a failing call ends
 * it as lapply() would -- and the shards are then planned, on host threads, from
 * the recorded draws (ABI 5: the recording pass no longer plans the device work).
 * Calls that carry only injected arrays are planned as given. */
int sg_node_plan_batch(sg_node* node, const sg_call_desc* calls, int64_t n_calls, sg_node_plan** out);
void sg_node_plan_destroy(sg_node_plan* plan);
int64_t sg_node_plan_n_calls(const sg_node_plan* plan);
int64_t sg_node_plan_total_samples(const sg_node_plan* plan);
int sg_node_plan_lengths(const sg_node_plan* plan, int64_t* out_len, int64_t* out_off);
int sg_node_plan_status(const sg_node_plan* plan, int32_t* out_status);
const char* sg_node_plan_call_message(const sg_node_plan* plan, int64_t i);
/* the node device index (0 .. size - 1) each call was assigned to */
int sg_node_plan_owner(const sg_node_plan* plan, int32_t* owner);
/* the analytic cost per call the assignment used (ns of one MI355X) */
int sg_node_plan_costs(const sg_node_plan* plan, double* cost);
int64_t sg_node_plan_shard_samples(const sg_node_plan* plan, int32_t k);
/* ABI 5: chunk plans of shard k (consecutive calls of the shard, <= SG_NODE_CHUNK
 * calls -- default 4096 -- and ~2^27 samples each: the unit of the execute pipeline) */
int32_t sg_node_plan_chunks(const sg_node_plan* plan, int32_t k);
/* ABI 5: 1 when a call failed in the shard planning after its recorded draws
 * succeeded (a failure behind a call's last draw that the draws-only recording pass
 * does not raise): later callback calls are then "not planned" as R's loop would
 * leave them, but their draws were consumed. 0 otherwise. */
int32_t sg_node_plan_diverged(const sg_node_plan* plan);
/* ABI 5: sg_plan_call_work per call of the whole batch (rows, flops: n_calls
 * doubles each, either may be NULL; unplanned calls are left untouched) */
int sg_node_plan_call_work(const sg_node_plan* plan, double* rows, double* fft_flops);
/* Synchronous: every device uploads, synthesizes its shard on its own streams
 * and copies it over its own link; each call's samples land in out_host at its
 * whole-batch offset (sg_node_plan_total_samples values in all). ABI 5: pipelined
 * by chunk (the D2H of a chunk overlaps the compute of the later ones and the host
 * scatter of the earlier one); the device output and two pinned staging slots of
 * the largest chunk stay allocated per device until sg_node_destroy. */
int sg_node_execute_to_host(sg_node* node, sg_node_plan* plan, double* out_host);
int sg_node_execute_to_host_f32(sg_node* node, sg_node_plan* plan, float* out_host);

/* ---- batch path (planned on host, executed on device) ------------------ */
/* All integer/length bookkeeping happens here, bit-exact with R. */
int sg_plan_batch(sg_ctx* ctx, const sg_call_desc* calls, int64_t n_calls,
                  sg_plan** out);
void sg_plan_destroy(sg_plan* plan);
int64_t sg_plan_n_calls(const sg_plan* plan);
int64_t sg_plan_total_samples(const sg_plan* plan);
/* per-call output length and offset into the packed output (int64 each) */
int sg_plan_lengths(const sg_plan* plan, int64_t* out_len, int64_t* out_off);
/* per-call status (0 ok or SG_E_*): a failed call marks its slot, the batch
 * does not abort (SURVEY §5 failure detection). */
int sg_plan_status(const sg_plan* plan, int32_t* out_status);
/* Bytes of device workspace the plan needs (descriptors + scratch). */
int64_t sg_plan_device_bytes(const sg_plan* plan);
/* Upload descriptors/inputs to HBM (outside any timed region). */
int sg_plan_upload(sg_ctx* ctx, sg_plan* plan);
/* After upload: free the plan's host copies of descriptors and inputs (a
 * 65,536-call preset batch holds ~0.7 MB per call on the host). Execution,
 * lengths, offsets, statuses and messages keep working; re-upload does not.
 * The bulk arrays are returned to the OS on a detached host thread, so the
 * call returns before their pages are unmapped.
 * No reference counterpart (R holds nothing between calls). */
int sg_plan_release_host(sg_plan* plan);
/* Run every kernel of the plan on `stream` (hipStream_t; NULL = the null
 * stream, ordered after earlier null-stream work such as torch's default stream)
 * writing fp32 samples into device buffer d_out (packed, offsets as above).
 * No host synchronisation inside; graph-capturable. */
int sg_execute(sg_ctx* ctx, sg_plan* plan, float* d_out, void* stream);
/* Several uploaded plans executed as ONE batch on `stream` (the outputs of
 * plan i go to d_outs[i], exactly as sg_execute(plans[i], d_outs[i]) would
 * write them): the harmonic chains of all plans run back to back on the
 * context's second stream, overlapping the spectral phases of the earlier
 * plans; everything is ordered after prior work on `stream` and joined back
 * to it. A plan may appear once. Replaces a loop of sg_execute over the 16k-call
 * chunks of one soundgen() batch (R/soundgen.R:208-862 per call). */
int sg_execute_plans(sg_ctx* ctx, sg_plan* const* plans, float* const* d_outs, int n, void* stream);
/* Profiling: when enabled, sg_execute brackets every sine-bank launch (one
 * per batch slice) and every sg_stft_ola launch with HIP events on the launch
 * stream; sg_profile_read
 * returns the average launch duration (ms) and the number of launches
 * recorded, and clears them. While profiling is on, the harmonic chain and
 * the noise phase (otherwise concurrent on the context's two streams) run one
 * after the other, so each recorded duration is the launch's own. */
int sg_set_profiling(sg_ctx* ctx, int on);
int sg_profile_read(sg_ctx* ctx, double* sine_ms_avg, int64_t* n);
/* Same for one kernel: SG_PROF_SINE_BANK (sg_sine_bank, generateHarmonics'
 * sine bank, R/source.R:389-419) or SG_PROF_STFT_OLA (sg_stft_ola, the fused
 * seewave stft/istft + overlap-add of R/soundgen.R:743-807 and R/source.R:88-131;
 * one event pair per phase launch). */
#define SG_PROF_SINE_BANK 0
#define SG_PROF_STFT_OLA 1
int sg_profile_read_kernel(sg_ctx* ctx, int kernel, double* ms_avg, int64_t* n);
int sg_synchronize(sg_ctx* ctx);
/* Synchronous convenience: upload (if needed), execute and copy the packed
 * output to host doubles: call i's samples land at out_host + offset[i]
 * (sg_plan_lengths), sg_plan_total_samples(plan) doubles in all. Random draws
 * happen only in sg_plan_batch, so a caller can size its buffer from the plan
 * before any sample is produced. */
int sg_execute_to_host(sg_ctx* ctx, sg_plan* plan, double* out_host);
/* Message of a failed call (status != 0). */
const char* sg_plan_call_message(const sg_plan* plan, int64_t i);
/* Per-kernel launch statistics of the last sg_execute (for roofline). */
int sg_plan_kernel_stats(const sg_plan* plan, int64_t* harm_samples,
                         int64_t* harm_terms, int64_t* harm_amp_bytes,
                         int64_t* fft_frames);
/* Wavetable spans of an uploaded plan (sg_set_sine_table): workgroups that
 * each build a table per execute, the samples they produce and the (sample, row) recurrence terms
 * those samples stand in for; zeros before upload. */
int sg_plan_table_stats(const sg_plan* plan, int64_t* tables, int64_t* samples, int64_t* terms);
/* sg_stft_ola work of the plan (fused seewave stft x envelope -> istft -> OLA,
 * R/soundgen.R:743-807, and generateNoise's istft, R/source.R:88-131): trimmed
 * output samples, algorithmic HBM bytes (source/uniforms + envelope columns +
 * output) and nominal flops (5 wl log2 wl per transform). */
int sg_plan_stft_stats(const sg_plan* plan, int64_t* samples, int64_t* alg_bytes, double* flops);
/* Sine-bank wave tasks of an uploaded plan by class (128-B descriptors, SgWTask):
 * counts[0] sg_sine_bank, [1] sg_sine_bank_pairs, [2] sg_sine_bank_tall,
 * [3] sg_sine_bank_tall_pairs, [4] sg_sine_bank_hp (zeros before upload). The
 * bench adds the descriptors to the kernels' algorithmic bytes. ABI 4. */
int sg_plan_sine_tasks(const sg_plan* plan, int64_t* counts);
/* Precision path of the plan (ABI 2): per call, the number of its bouts whose
 * formant filter runs in fp64 (source, pre-filter mix and forward STFT; the
 * planner's conditioning estimate of the fp32 round-off through the envelope
 * exceeded its threshold, env SG_HP_RHO, default 100; sg_set_fp64_policy: 0 never, 2 always);
 * totals of fp64 filter frames and sine-bank tasks. Any pointer may be NULL.
 * No reference counterpart: the R path is fp64 throughout. */
int sg_plan_precision(const sg_plan* plan, int32_t* call_fp64, int64_t* fp64_frames, int64_t* fp64_tasks);
/* Per call: the planner's conditioning estimate of the formant filter in fp32
 * (the largest over the call's filtered bouts; 0 when none was estimated):
 * bouts above the fp64 policy's threshold take the fp64 filter path. */
int sg_plan_conditioning(const sg_plan* plan, double* rho);
/* The same estimate for the pre-filter noise of each call's filtered bouts
 * (its fp32 inverse STFT's round-off against the formant envelope); above the
 * noise threshold those noise frames take the fp64 kernel. */
int sg_plan_noise_conditioning(const sg_plan* plan, double* rho);
/* Per-call device work the plan emits (ABI 2): sine-bank (sample, row) terms and
 * nominal FFT flops (5 wl log2 wl per transform), for load balancing across
 * GPUs (soundgen_beta_amd/dist.py). Either pointer may be NULL. */
int sg_plan_call_work(const sg_plan* plan, double* rows, double* fft_flops);
/* compareSounds() / getMelSpec() parameters (R/matchPars.R:313-325, :510-520
 * formals): windowLength and step in ms, overlap in %, throwaway in dB; step
 * NaN = windowLength * (1 - overlap / 100), maxFreq NaN = samplingRate / 2. */
typedef struct sg_mel_params {
  double samplingRate;
  double windowLength;
  double overlap;
  double step;
  double throwaway;
  double maxFreq;
  int32_t penalizeLengthDif;
  int32_t pad;
} sg_mel_params;
/* getMelSpec(s, ...) (R/matchPars.R:510-560: tuneR melfcc(spec_out = TRUE)
 * $aspectrum, frames with colMeans <= 2^(throwaway/10) dropped, log01) of one
 * host waveform, computed on the GPU in fp64: out (cap doubles) receives the
 * nb x nc matrix column-major; *nb and *nc are set (out may be NULL to size).
 * Windows of more than 4096 FFT points: SG_E_UNSUPPORTED. */
int sg_mel_spec(sg_ctx* ctx, const double* wave, int64_t len, const sg_mel_params* p, double* out, int64_t cap,
                int32_t* nb, int32_t* nc);
/* compareSounds(targetSpec = target, cand = candidate c, ...) for n candidates
 * in DEVICE memory (fp32, candidate c at d_wave + offsets[c], lengths[c]
 * samples; lengths[c] <= 0: skipped, NaN), against the host target spectrum
 * (nb x nc_target column-major, as sg_mel_spec returns it): out[4 c + m] for
 * m = cor, cosine, pixel, dtw (methods: bit m set = computed, else NaN; dtw is
 * the dtw package's symmetric2 normalizedDistance), summary[c] the mean of the
 * computed non-NA methods (compareSounds(summary = TRUE); may be NULL). One
 * launch sequence for the whole batch (R/matchPars.R:313-416, called per
 * candidate at :168, :202). */
int sg_compare_sounds_batch(sg_ctx* ctx, const double* target_spec, int32_t nb, int32_t nc_target,
                            const float* d_wave, const int64_t* offsets, const int64_t* lengths, int64_t n,
                            const sg_mel_params* p, int32_t methods, double* out, double* summary);
/* compareSounds' 'dtw' method (R/matchPars.R:372-376): dtw::dtw(x, y,
 * distance.only = TRUE)$normalizedDistance with the dtw package defaults
 * (|x_i - y_j|, symmetric2, / (n + m)). Host only (ABI 2). */
int sg_dtw_symmetric2(const double* x, int64_t n, const double* y, int64_t m, double* out);
/* Process-wide policy of the fp64 filter path for later sg_plan_batch calls:
 * mode 0 never, 1 when the conditioning estimate exceeds rho (default 100),
 * 2 every filtered bout. SG_E_ARG for an invalid mode or rho. */
int sg_set_fp64_policy(int32_t mode, double rho);
/* Process-wide source of the harmonic amplitude matrices for later
 * sg_plan_batch calls: 0 (default) built on the device at upload from
 * per-glottal-cycle parameters, 1 built on the host and uploaded (the
 * reference-order host restatement; tests compare the two). */
int sg_set_amp_policy(int32_t host_built);
/* Process-wide handling of generateNoise()'s uniforms read from injected draw
 * arrays, for later sg_plan_batch calls: 1 (default) the planner records each
 * noise item's range of the caller's array, copies the union of the ranges
 * once and the device expands the items at upload; 0 each item's draws are
 * copied into the plan (the same values either way; tests compare the two).
 * The arrays are read during sg_plan_batch only. */
int sg_set_uniform_gather(int32_t on);
/* Process-wide switch of the sine bank's wavetable path, for plans uploaded
 * later (sg_plan_upload, or the first sg_execute of a plan): 1 (default)
 * long runs of constant-amplitude, linear-phase tasks (static tones) sample a
 * per-span table of the harmonic sum by cubic Hermite interpolation
 * (sg_sine_bank_tab); 0 every task runs the row recurrence. */
int sg_set_sine_table(int32_t on);
/* Release the planner's process-wide cache of freed host blocks (kept for the
 * next plan, capped by SG_HOST_CACHE_MB or 8 GB / LOCAL_WORLD_SIZE). Returns
 * the bytes released. Safe at any time; later plans refill it. */
int64_t sg_host_cache_trim(void);
/* The amplitude blocks sg_amp_build writes at upload, evaluated on the host by
 * the same code (tests; no device needed): n = sg_plan_amp_count(plan) floats. */
int64_t sg_plan_amp_count(const sg_plan* plan);
int sg_plan_debug_amps(const sg_plan* plan, float* out, int64_t n);

/* ---- function-level entries mirroring the R API (synchronous) ---------- */
int sg_generate_harmonics(sg_ctx* ctx, const double* pitch, int64_t len,
                          const sg_harm_params* p, sg_anchors amplAnchors,
                          const sg_random* rnd, double* out, int64_t cap,
                          int64_t* out_len);
int sg_soundgen(sg_ctx* ctx, const sg_soundgen_args* a, const sg_random* rnd,
                double* out, int64_t cap, int64_t* out_len);
/* generateNoise(len, noiseAnchors, rolloffNoise, attackLen,
 * windowLength_points, samplingRate, overlap, throwaway, filterNoise);
 * filterNoise is nr x filter_nc column-major (NULL/0 = NA). */
int sg_generate_noise(sg_ctx* ctx, int64_t len, sg_anchors noiseAnchors,
                      double rolloffNoise, double attackLen,
                      int32_t windowLength_points, double samplingRate,
                      double overlap, double throwaway,
                      const double* filterNoise, int32_t filter_nc,
                      const sg_random* rnd, double* out);
/* getSpectralEnvelope(nr, nc, formants, formantDep, rolloffLip,
 * mouthAnchors, mouthOpenThres, openMouthBoost, vocalTract, temperature,
 * formDrift, formDisp, formantDepStoch, smoothLinearFactor, samplingRate,
 * speedSound) -> out[nr*nc] column-major. */
int sg_spectral_envelope(sg_ctx* ctx, int32_t nr, int32_t nc,
                         const sg_formants* formants, double formantDep,
                         double rolloffLip, sg_anchors mouthAnchors,
                         double mouthOpenThres, double openMouthBoost,
                         double vocalTract, double temperature,
                         double formDrift, double formDisp,
                         double formantDepStoch, double smoothLinearFactor,
                         double samplingRate, double speedSound,
                         const sg_random* rnd, double* out);
/* STFT(hamming) x envelope -> ISTFT(hann OLA) -> /max, R/soundgen.R:743-807.
 * env is nr x env_nc (env_nc == 1: stationary). out cap >= len. */
int sg_formant_filter(sg_ctx* ctx, const double* sound, int64_t len,
                      const double* env, int32_t env_nc,
                      int32_t windowLength_points, double overlap,
                      double* out, int64_t cap, int64_t* out_len);
/* getSmoothContour(anchors, len, thisIsPitch, method, valueFloor,
 * valueCeiling, samplingRate)  R/smoothContours.R:53-227 (exported,
 * NAMESPACE:10); method 0 = 'loess' (R's default), 1 = 'spline'. The
 * planner's own contour (host, fp64). out holds len doubles; *out_len = 0 when
 * R returns NA (no anchors, len 0). len = -1 is R's len = NULL: the anchor
 * times are in ms and len = floor(duration_ms * samplingRate / 1000) (out must
 * then hold that many doubles). */
int sg_get_smooth_contour(sg_anchors anchors, int64_t len, int32_t thisIsPitch, int32_t method, int32_t has_floor,
                          double valueFloor, int32_t has_ceil, double valueCeiling, double samplingRate, double* out,
                          int64_t* out_len);
/* getRolloff() (host helper; R returns H x nGC). out cap = nHarmonics*nGC.
 * rolloffParabCeiling NaN = NULL (R/sourceSpectrum.R:77, :105-107). */
int sg_get_rolloff(const double* pitch_per_gc, int32_t n_gc,
                   int32_t nHarmonics, double rolloff, double rolloffOct,
                   double rolloffParab, double rolloffParabHarm,
                   double rolloffParabCeiling, double rolloffKHz,
                   double baseline, double throwaway,
                   double samplingRate, double* out, int32_t* out_rows);

/* ---- output writer: seewave::savewav (R/soundgen.R:856, R/morph.R:205) --- */
/* 16-bit PCM of every call of an executed plan, as savewav(wave, f) converts a
 * waveform (tuneR::normalize(unit = "16", level = min(max(wave), 1)): center,
 * scale by level / max|x| unless that is ~0, round(x * 32767) half to even).
 * d_in: the plan's packed fp32 output; d_out: int16 at the same offsets. */
int sg_pcm16(sg_ctx* ctx, sg_plan* plan, const float* d_in, int16_t* d_out, void* stream);
/* The same conversion for one host waveform in R's fp64 arithmetic (on the
 * GPU); rescale NULL, or {lower, upper} for savewav(rescale = ...). */
int sg_savewav_pcm(sg_ctx* ctx, const double* wave, int64_t n, const double* rescale, int16_t* pcm_out);
/* The file tuneR::writeWave(extensible = TRUE) writes for a mono 16-bit Wave. */
int sg_wav_write(const char* path, const int16_t* pcm, int64_t n, int32_t samplingRate);

/* Reference data tables the planner restates (pinned by tests/test_rda_fixtures.py
 * against the decoded .rda files):
 *   permittedValues rows 1..33 (data/permittedValues.rda, R/presets.R:22-56):
 *     name, default, low, high of soundgen()'s range-checked arguments;
 *   noiseThresholdsDict$q1/$q2[nonlinBalance + 1] (R/sysdata.rda,
 *     data-raw/noiseThresholdsDict.R), which = 1 or 2. */
int sg_permitted_value(int32_t i, const char** name, double* def_low_high);
double sg_noise_threshold(int32_t which, double nonlinBalance);

/* Test hook, no reference counterpart: the wavefront FFT stages used inside
 * the fused STFT/ISTFT kernel, on nframes frames of wl/2 complex points
 * (interleaved re, im, in place semantics: out = DFT(in), unscaled; inverse
 * bit 0 uses exp(+2 pi i nk / M); bit 1, for wl = 2204 only, runs the radix-29
 * stage on the VALU as sg_stft_ola_noise does instead of on the matrix pipe).
 * SG_E_UNSUPPORTED if wl is not on that path. */
int sg_debug_wave_fft(sg_ctx* ctx, int32_t wl, int32_t inverse, int32_t nframes,
                      const float* in, float* out);

#ifdef __cplusplus
}
#endif
#endif /* SOUNDGEN_HIP_H */
