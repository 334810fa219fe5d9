/*
 * sg_r_shim.c — the thin .Call shim a maintainer adds to the reference R
 * package (nemochina2008/soundgen_beta, soundgen 1.0.0) so that its hot path
 * runs in libsoundgen_hip.so. Compiled only where R headers exist (R CMD
 * INSTALL with r/src/Makevars); it is not built in this repository's CI
 * (R is absent from the build image).
 *
 * Entry points (reference call sites they replace):
 *   C_sg_generate_harmonics  R/source.R:173-471     (do.call(generateHarmonics, ...) at R/soundgen.R:616-620)
 *   C_sg_soundgen            R/soundgen.R:208-862
 *   C_sg_generate_noise      R/source.R:57-138      (R/soundgen.R:686-696)
 *   C_sg_spectral_envelope   R/sourceSpectrum.R:261-566 (R/soundgen.R:668-680, :762-775)
 *   C_sg_formant_filter      R/soundgen.R:743-807   (seewave::stft x env -> seewave::istft)
 *   C_sg_soundgen_batch      a list of soundgen() calls planned as ONE batch
 *                            (the loops of R/morph.R:200-208, R/matchPars.R:176-190)
 *
 * Randomness: the sg_random callbacks are bound to R's own norm_rand(),
 * unif_rand() and rgamma() between GetRNGstate()/PutRNGstate(), so a
 * set.seed() before the call reproduces the reference's draws in its order.
 * Errors: a negative SG_E_* status becomes Rf_error(sg_last_error()) after
 * every device buffer of the call has been released (the library frees them
 * before returning); no C++ exception crosses the C ABI.
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Random.h>
#include <R_ext/Rdynload.h>
#include <Rmath.h>
#include <string.h>

#include "soundgen_hip.h"

static sg_ctx* g_ctx = NULL;

static sg_ctx* ctx(void) {
  if (!g_ctx && sg_ctx_create(0, &g_ctx) != SG_OK) Rf_error("soundgen_hip: no usable MI355X (sg_ctx_create failed)");
  return g_ctx;
}

/* The node of soundgen_batch: the devices of the last call's `devices`
 * (getOption("soundgen_hip.devices"); NULL = device 0, as ctx(); -1 = every
 * visible device), kept across calls while they stay the same. */
static sg_node* g_node = NULL;
static int32_t g_node_dev[64];
static int32_t g_node_n = -1;

static sg_node* node(SEXP devices) {
  int32_t dv[64];
  int32_t n = 0;
  if (Rf_isNull(devices)) {
    dv[n++] = 0;  /* the single device of the other entry points */
  } else if (TYPEOF(devices) == INTSXP && Rf_xlength(devices) == 1 && INTEGER(devices)[0] == -1) {
    n = 0;  /* opt-in fan-out: every visible device */
  } else {
    const R_xlen_t m = Rf_xlength(devices);
    if (TYPEOF(devices) != INTSXP || m < 1 || m > 64)
      Rf_error("soundgen_hip: devices must be an integer vector of 1 to 64 device ordinals");
    for (R_xlen_t i = 0; i < m; ++i) {
      const int v = INTEGER(devices)[i];
      if (v == NA_INTEGER || v < 0) Rf_error("soundgen_hip: device ordinals must be >= 0");
      dv[n++] = (int32_t)v;
    }
  }
  if (sg_device_count() <= 0) Rf_error("soundgen_hip: no usable MI355X (no HIP device)");
  if (g_node && n == g_node_n && (n == 0 || !memcmp(dv, g_node_dev, (size_t)n * sizeof(int32_t)))) return g_node;
  if (g_node) sg_node_destroy(g_node);
  g_node = NULL;
  if (sg_node_create(n ? dv : NULL, n, &g_node) != SG_OK) Rf_error("soundgen_hip: no usable MI355X (sg_node_create failed)");
  memcpy(g_node_dev, dv, (size_t)n * sizeof(int32_t));
  g_node_n = n;
  return g_node;
}

static double cb_norm(void* u) { (void)u; return norm_rand(); }
static double cb_unif(void* u) { (void)u; return unif_rand(); }
/* runif(n) in one C loop: generateNoise's runif(nr * nc) without a callback per draw */
static void cb_unif_n(void* u, double* out, int64_t n) {
  (void)u;
  for (int64_t i = 0; i < n; ++i) out[i] = unif_rand();
}
static double cb_gamma(void* u, double shape, double rate) { (void)u; return rgamma(shape, 1.0 / rate); }

static sg_random r_rng(void) {
  sg_random r;
  memset(&r, 0, sizeof r);
  r.norm_cb = cb_norm;
  r.unif_cb = cb_unif;
  r.gamma_cb = cb_gamma;
  r.unif_n_cb = cb_unif_n;
  return r;
}

static double num(SEXP list, const char* name, double dflt) {
  SEXP nms = Rf_getAttrib(list, R_NamesSymbol);
  for (R_xlen_t i = 0; i < Rf_xlength(list); ++i)
    if (!strcmp(CHAR(STRING_ELT(nms, i)), name)) {
      SEXP v = VECTOR_ELT(list, i);
      return (Rf_isNull(v) || Rf_xlength(v) < 1) ? NA_REAL : Rf_asReal(v);
    }
  return dflt;
}

/* data.frame(time, value) or NULL/NA -> sg_anchors (views into R memory) */
static sg_anchors anchors(SEXP df) {
  sg_anchors a = {0, NULL, NULL};
  if (!Rf_isNewList(df) || Rf_xlength(df) < 2) return a;
  SEXP t = VECTOR_ELT(df, 0), v = VECTOR_ELT(df, 1);
  if (TYPEOF(t) != REALSXP || TYPEOF(v) != REALSXP) Rf_error("anchors must be numeric data.frame(time, value)");
  a.n = (int32_t)Rf_xlength(t);
  a.time = REAL(t);
  a.value = REAL(v);
  return a;
}

static void check(int rc) {
  if (rc < 0) Rf_error("soundgen_hip: %s", sg_last_error(g_ctx));
}

/* plan (every random draw happens here, once, on R's RNG), size the R
 * vector from the plan, then run the device path */
static SEXP run_planned(const sg_call_desc* d) {
  sg_plan* plan = NULL;
  GetRNGstate();
  int rc = sg_plan_batch(ctx(), d, 1, &plan);
  PutRNGstate();
  check(rc);
  int32_t st = 0;
  sg_plan_status(plan, &st);
  if (st) {
    char msg[512];
    snprintf(msg, sizeof msg, "%s", sg_plan_call_message(plan, 0));
    sg_plan_destroy(plan);
    Rf_error("soundgen_hip: %s", msg);
  }
  int64_t len = 0, off = 0;
  sg_plan_lengths(plan, &len, &off);
  SEXP out = PROTECT(Rf_allocVector(REALSXP, sg_plan_total_samples(plan) > 0 ? sg_plan_total_samples(plan) : 1));
  rc = sg_execute_to_host(ctx(), plan, REAL(out));
  sg_plan_destroy(plan);
  check(rc);
  out = Rf_xlengthgets(out, len);
  UNPROTECT(1);
  return out;
}

/* generateHarmonics(pitch, <formals as a named list>, amplAnchors) */
SEXP C_sg_generate_harmonics(SEXP pitch, SEXP pars, SEXP amplAnchors) {
  if (TYPEOF(pitch) != REALSXP) Rf_error("pitch must be double");
  sg_harm_params p;
  sg_default_harm_params(&p);
#define F(nm) p.nm = num(pars, #nm, p.nm)
  F(attackLen); F(nonlinBalance); F(nonlinDep); F(jitterDep); F(jitterLen); F(vibratoFreq); F(vibratoDep);
  F(shimmerDep); F(creakyBreathy); F(rolloff); F(rolloffOct); F(rolloffKHz); F(rolloffParab);
  F(rolloffParabHarm); F(rolloffLip); F(rolloff_perAmpl); F(temperature); F(pitchDriftDep); F(pitchDriftFreq);
  F(randomWalk_trendStrength); F(shortestEpoch); F(subFreq); F(subDep); F(amDep); F(amFreq); F(overlap);
  F(samplingRate); F(pitchFloor); F(pitchCeiling); F(pitchSamplingRate); F(throwaway);
#undef F
  sg_call_desc d;
  memset(&d, 0, sizeof d);
  d.kind = SG_CALL_HARMONICS;
  d.pitch = REAL(pitch);
  d.pitch_len = Rf_xlength(pitch);
  d.harm = &p;
  d.amplAnchors = anchors(amplAnchors);
  d.random = r_rng();
  return run_planned(&d);
}

/* list(n_points = integer, f1_index = integer, time, freq, amp, width), as
 * .sg_flatten_formants() builds it, or NULL (NA formants) -> sg_formants
 * (views into R memory) */
static void flat_formants(SEXP v, sg_formants* f) {
  memset(f, 0, sizeof *f);
  f->f1_index = -1;
  if (Rf_isNull(v)) return;
  if (!Rf_isNewList(v) || Rf_xlength(v) != 6 || TYPEOF(VECTOR_ELT(v, 0)) != INTSXP)
    Rf_error("soundgen_hip: formants must be flattened by .sg_flatten_formants()");
  SEXP np = VECTOR_ELT(v, 0);
  R_xlen_t tot = 0;
  for (R_xlen_t k = 0; k < Rf_xlength(np); ++k) tot += INTEGER(np)[k];
  for (int j = 2; j < 6; ++j)
    if (TYPEOF(VECTOR_ELT(v, j)) != REALSXP || Rf_xlength(VECTOR_ELT(v, j)) != tot)
      Rf_error("soundgen_hip: formant time/freq/amp/width must be double, one value per row");
  f->n_formants = (int32_t)Rf_xlength(np);
  f->n_points = INTEGER(np);
  f->f1_index = Rf_asInteger(VECTOR_ELT(v, 1));
  f->time = REAL(VECTOR_ELT(v, 2));
  f->freq = REAL(VECTOR_ELT(v, 3));
  f->amp = REAL(VECTOR_ELT(v, 4));
  f->width = REAL(VECTOR_ELT(v, 5));
}

/* soundgen(...) with the formals of R/soundgen.R:208-277 already resolved by
 * the R wrapper (.sg_soundgen_args: anchors as data.frames, formants
 * flattened) -> sg_soundgen_args (views into R memory) */
static void soundgen_args(SEXP args, sg_soundgen_args* a) {
  if (!Rf_isNewList(args)) Rf_error("soundgen_hip: soundgen arguments must be a named list");
  sg_default_soundgen_args(a);
#define F(nm) a->nm = num(args, #nm, a->nm)
  F(repeatBout); F(nSyl); F(sylLen); F(pauseLen); F(temperature); F(maleFemale); F(creakyBreathy);
  F(nonlinBalance); F(nonlinDep); F(jitterLen); F(jitterDep); F(vibratoFreq); F(vibratoDep); F(shimmerDep);
  F(attackLen); F(rolloff); F(rolloffOct); F(rolloffKHz); F(rolloffParab); F(rolloffParabHarm); F(rolloffLip);
  F(formantDep); F(formantDepStoch); F(vocalTract); F(subFreq); F(subDep); F(shortestEpoch); F(amDep);
  F(amFreq); F(amShape); F(rolloffNoise); F(samplingRate); F(windowLength); F(overlap); F(addSilence);
  F(pitchFloor); F(pitchCeiling); F(pitchSamplingRate); F(throwaway);
#undef F
  SEXP nms = Rf_getAttrib(args, R_NamesSymbol);
  for (R_xlen_t i = 0; i < Rf_xlength(args); ++i) {
    const char* k = CHAR(STRING_ELT(nms, i));
    SEXP v = VECTOR_ELT(args, i);
    if (!strcmp(k, "pitchAnchors")) a->pitchAnchors = anchors(v);
    else if (!strcmp(k, "pitchAnchorsGlobal")) a->pitchAnchorsGlobal = anchors(v);
    else if (!strcmp(k, "noiseAnchors")) a->noiseAnchors = anchors(v);
    else if (!strcmp(k, "mouthAnchors")) a->mouthAnchors = anchors(v);
    else if (!strcmp(k, "amplAnchors")) a->amplAnchors = anchors(v);
    else if (!strcmp(k, "amplAnchorsGlobal")) a->amplAnchorsGlobal = anchors(v);
    else if (!strcmp(k, "formantsNoise_rlen")) a->formantsNoise_rlen = Rf_asInteger(v);
    else if (!strcmp(k, "invalidArgAction")) a->invalidArgAction = Rf_asInteger(v);
    else if (!strcmp(k, "tempEffects") && TYPEOF(v) == REALSXP && Rf_xlength(v) == 8)
      memcpy(a->tempEffects, REAL(v), sizeof a->tempEffects);
    else if (!strcmp(k, "formants_flat")) flat_formants(v, &a->formants);
    else if (!strcmp(k, "formantsNoise_flat")) flat_formants(v, &a->formantsNoise);
  }
}

SEXP C_sg_soundgen(SEXP args) {
  sg_soundgen_args a;
  soundgen_args(args, &a);
  sg_call_desc d;
  memset(&d, 0, sizeof d);
  d.kind = SG_CALL_SOUNDGEN;
  d.args = &a;
  d.random = r_rng();
  return run_planned(&d);
}

/* soundgen_batch(calls): a list of resolved soundgen() argument lists (as
 * .sg_soundgen_args builds each) planned as ONE sg_plan_batch and executed in
 * one pass over the node's devices (sg_node: LPT shards, each device on its own
 * stream and link; `devices` NULL = every visible device); returns the list of
 * waveforms in call order. R's RNG is drawn in
 * call order, each call's draws in the reference's order, so the result equals
 * lapply(calls, function(a) do.call(soundgen, a)) after the same set.seed().
 * A call R would stop() on stops the batch with that call's message, as the
 * loop would: its draws and those of the calls before it are consumed, and the
 * planner plans no later call once a callback-drawing call has failed
 * (plan_range in sg_api.cpp), so .Random.seed ends where the R loop leaves it. */
SEXP C_sg_soundgen_batch(SEXP calls, SEXP devices) {
  if (!Rf_isNewList(calls)) Rf_error("soundgen_hip: calls must be a list of argument lists");
  const R_xlen_t n = Rf_xlength(calls);
  SEXP res = PROTECT(Rf_allocVector(VECSXP, n));
  if (n == 0) {
    UNPROTECT(1);
    return res;
  }
  sg_soundgen_args* a = (sg_soundgen_args*)R_alloc((size_t)n, sizeof(sg_soundgen_args));
  sg_call_desc* d = (sg_call_desc*)R_alloc((size_t)n, sizeof(sg_call_desc));
  memset(d, 0, (size_t)n * sizeof(sg_call_desc));
  for (R_xlen_t i = 0; i < n; ++i) {
    soundgen_args(VECTOR_ELT(calls, i), &a[i]);
    d[i].kind = SG_CALL_SOUNDGEN;
    d[i].args = &a[i];
    d[i].random = r_rng();
  }
  sg_node* nd = node(devices);
  sg_node_plan* plan = NULL;
  GetRNGstate();
  int rc = sg_node_plan_batch(nd, d, (int64_t)n, &plan);
  PutRNGstate();
  if (rc) Rf_error("soundgen_hip: %s", sg_node_last_error(nd));
  int32_t* st = (int32_t*)R_alloc((size_t)n, sizeof(int32_t));
  int64_t* len = (int64_t*)R_alloc((size_t)n, sizeof(int64_t));
  int64_t* off = (int64_t*)R_alloc((size_t)n, sizeof(int64_t));
  sg_node_plan_status(plan, st);
  sg_node_plan_lengths(plan, len, off);
  for (R_xlen_t i = 0; i < n; ++i)
    if (st[i]) {
      char msg[512];
      snprintf(msg, sizeof msg, "call %ld: %s", (long)(i + 1), sg_node_plan_call_message(plan, (int64_t)i));
      sg_node_plan_destroy(plan);
      Rf_error("soundgen_hip: %s", msg);
    }
  const int64_t tot = sg_node_plan_total_samples(plan);
  SEXP all = PROTECT(Rf_allocVector(REALSXP, tot > 0 ? tot : 1));
  rc = sg_node_execute_to_host(nd, plan, REAL(all));
  sg_node_plan_destroy(plan);
  if (rc) Rf_error("soundgen_hip: %s", sg_node_last_error(nd));
  for (R_xlen_t i = 0; i < n; ++i) {
    SEXP y = Rf_allocVector(REALSXP, len[i]);
    SET_VECTOR_ELT(res, i, y);
    if (len[i]) memcpy(REAL(y), REAL(all) + off[i], (size_t)len[i] * sizeof(double));
  }
  UNPROTECT(2);
  return res;
}

/* generateNoise(len, noiseAnchors, <scalar formals as a named list>,
 * filterNoise): istft-based filtered noise, R/source.R:57-138. filterNoise is
 * NULL (NA) or an nr x nc double matrix, nr = windowLength_points / 2. */
SEXP C_sg_generate_noise(SEXP len, SEXP noiseAnchors, SEXP pars, SEXP filterNoise) {
  const double Ld = Rf_asReal(len);
  if (!(Ld >= 0)) Rf_error("soundgen_hip: len must be a non-negative number");
  const int64_t L = (int64_t)Ld;
  SEXP out = PROTECT(Rf_allocVector(REALSXP, L));
  const double* fn = NULL;
  int32_t fnc = 0;
  const int32_t wl = (int32_t)num(pars, "windowLength_points", 1024);
  if (!Rf_isNull(filterNoise)) {
    if (TYPEOF(filterNoise) != REALSXP || !Rf_isMatrix(filterNoise) || Rf_nrows(filterNoise) != wl / 2)
      Rf_error("soundgen_hip: filterNoise must be a double matrix with windowLength_points / 2 rows");
    fn = REAL(filterNoise);
    fnc = Rf_ncols(filterNoise);
  }
  sg_random rnd = r_rng();
  GetRNGstate();
  int rc = sg_generate_noise(ctx(), L, anchors(noiseAnchors), num(pars, "rolloffNoise", -6),
                             num(pars, "attackLen", 10), wl,
                             num(pars, "samplingRate", 16000), num(pars, "overlap", 75), num(pars, "throwaway", -120),
                             fn, fnc, &rnd, REAL(out));
  PutRNGstate();
  check(rc);
  UNPROTECT(1);
  return out;
}

/* getSpectralEnvelope(nr, nc, <formants flattened>, <scalar formals as a
 * named list>, mouthAnchors) -> the nr x nc double matrix R returns
 * (R/sourceSpectrum.R:261-566). vocalTract NULL travels as NA (NaN). The
 * tracks and stochastic formants are planned on the host with R's RNG; the
 * matrix is computed on the device. */
SEXP C_sg_spectral_envelope(SEXP nr, SEXP nc, SEXP formants, SEXP pars, SEXP mouthAnchors) {
  const int NR = Rf_asInteger(nr), NC = Rf_asInteger(nc);
  if (NR == NA_INTEGER || NC == NA_INTEGER || NR < 1 || NC < 1)
    Rf_error("soundgen_hip: nr and nc must be positive integers");
  sg_formants F;
  flat_formants(formants, &F);
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, NR, NC));
  sg_random rnd = r_rng();
  GetRNGstate();
  int rc = sg_spectral_envelope(ctx(), NR, NC, &F, num(pars, "formantDep", 1), num(pars, "rolloffLip", 6),
                                anchors(mouthAnchors), num(pars, "mouthOpenThres", 0),
                                num(pars, "openMouthBoost", 0), num(pars, "vocalTract", NA_REAL),
                                num(pars, "temperature", 0), num(pars, "formDrift", .3), num(pars, "formDisp", .2),
                                num(pars, "formantDepStoch", 30), num(pars, "smoothLinearFactor", 1),
                                num(pars, "samplingRate", 16000), num(pars, "speedSound", 35400), &rnd, REAL(out));
  PutRNGstate();
  check(rc);
  UNPROTECT(1);
  return out;
}

SEXP C_sg_formant_filter(SEXP sound, SEXP env, SEXP wl, SEXP overlap) {
  const int64_t L = Rf_xlength(sound);
  int64_t cap = L + 2 * (int64_t)Rf_asInteger(wl), n = 0;
  SEXP out = PROTECT(Rf_allocVector(REALSXP, cap));
  check(sg_formant_filter(ctx(), REAL(sound), L, REAL(env), Rf_isMatrix(env) ? Rf_ncols(env) : 1,
                          Rf_asInteger(wl), Rf_asReal(overlap), REAL(out), cap, &n));
  out = Rf_xlengthgets(out, n);
  UNPROTECT(1);
  return out;
}

static const R_CallMethodDef CALLS[] = {
    {"C_sg_generate_harmonics", (DL_FUNC)&C_sg_generate_harmonics, 3},
    {"C_sg_soundgen", (DL_FUNC)&C_sg_soundgen, 1},
    {"C_sg_generate_noise", (DL_FUNC)&C_sg_generate_noise, 4},
    {"C_sg_spectral_envelope", (DL_FUNC)&C_sg_spectral_envelope, 5},
    {"C_sg_formant_filter", (DL_FUNC)&C_sg_formant_filter, 4},
    {"C_sg_soundgen_batch", (DL_FUNC)&C_sg_soundgen_batch, 2},
    {NULL, NULL, 0}};

void R_init_soundgen(DllInfo* dll) {
  R_registerRoutines(dll, NULL, CALLS, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}

void R_unload_soundgen(DllInfo* dll) {
  (void)dll;
  if (g_ctx) sg_ctx_destroy(g_ctx);
  g_ctx = NULL;
  if (g_node) sg_node_destroy(g_node);
  g_node = NULL;
  g_node_n = -1;
}
