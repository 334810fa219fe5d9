# soundgen_hip.R — R-side wrappers a maintainer drops into the reference
# package (nemochina2008/soundgen_beta) to route its hot path through
# libsoundgen_hip.so. Formals and defaults are the reference's own; only the
# bodies change (see INTEGRATION.md). R is absent from this repository's
# image: tests/test_r_shim.py compiles r/src/sg_r_shim.c against a small mock of
# the R C API and drives each entry with the arguments these wrappers build.

# R/source.R:173-205
generateHarmonics = function(pitch, attackLen = 50, nonlinBalance = 0, nonlinDep = 0, jitterDep = 0,
                             jitterLen = 1, vibratoFreq = 100, vibratoDep = 0, shimmerDep = 0,
                             creakyBreathy = 0, rolloff = -18, rolloffOct = -2, rolloffKHz = -6,
                             rolloffParab = 0, rolloffParabHarm = 3, rolloffLip = 6, rolloff_perAmpl = 12,
                             temperature = 0, pitchDriftDep = .5, pitchDriftFreq = .125,
                             randomWalk_trendStrength = .5, shortestEpoch = 300, subFreq = 100,
                             subDep = 0, amDep = 0, amFreq = 30, amplAnchors = NA, overlap = 75,
                             samplingRate = 16000, pitchFloor = 75, pitchCeiling = 3500,
                             pitchSamplingRate = 3500, throwaway = -120) {
  pars = as.list(environment())
  pars$pitch = NULL
  pars$amplAnchors = NULL
  aa = if (is.data.frame(amplAnchors)) amplAnchors[, c('time', 'value')] else NULL
  .Call(C_sg_generate_harmonics, as.double(pitch), pars, aa)
}

# formants list(f1 = data.frame(time, freq, amp, width), ...) -> flat arrays
.sg_flatten_formants = function(formants) {
  if (!is.list(formants) || length(formants) == 0) return(NULL)
  fs = lapply(formants, as.data.frame)
  list(n_points = as.integer(sapply(fs, nrow)),
       f1_index = if ('f1' %in% names(fs)) match('f1', names(fs)) - 1L else -1L,
       time = as.double(unlist(lapply(fs, function(f) f$time))),
       freq = as.double(unlist(lapply(fs, function(f) f$freq))),
       amp = as.double(unlist(lapply(fs, function(f) f$amp))),
       width = as.double(unlist(lapply(fs, function(f) f$width))))
}

# R/soundgen.R:208-277: the reference's formals and defaults verbatim; the body
# keeps the reference's argument coercions (R/soundgen.R:305-315, :384-389) and
# hands the call to the device. Every formal is passed (as.list(environment())),
# so the default pitch contour, the vowel-'a' formants and the noise/mouth
# anchors reach the planner as R would use them.
soundgen_hip = function(repeatBout = 1, nSyl = 1, sylLen = 300, pauseLen = 200,
                        pitchAnchors = data.frame(time = c(0, .1, .9, 1), value = c(100, 150, 135, 100)),
                        pitchAnchorsGlobal = NA, temperature = 0.025,
                        tempEffects = list(sylLenDep = .02, formDrift = .3, formDisp = .2, pitchDriftDep = .5,
                                           pitchDriftFreq = .125, pitchAnchorsDep = .05, noiseAnchorsDep = .1,
                                           amplAnchorsDep = .1),
                        maleFemale = 0, creakyBreathy = 0, nonlinBalance = 0, nonlinDep = 50, jitterLen = 1,
                        jitterDep = 3, vibratoFreq = 5, vibratoDep = 0, shimmerDep = 0, attackLen = 50,
                        rolloff = -12, rolloffOct = -12, rolloffKHz = -6, rolloffParab = 0, rolloffParabHarm = 3,
                        rolloffLip = 6,
                        formants = list(f1 = list(time = 0, freq = 860, amp = 30, width = 120),
                                        f2 = list(time = 0, freq = 1280, amp = 40, width = 120),
                                        f3 = list(time = 0, freq = 2900, amp = 25, width = 200)),
                        formantDep = 1, formantDepStoch = 30, vocalTract = 15.5, subFreq = 100, subDep = 100,
                        shortestEpoch = 300, amDep = 0, amFreq = 30, amShape = 0,
                        noiseAnchors = data.frame(time = c(0, 300), value = c(-120, -120)),
                        formantsNoise = NA, rolloffNoise = -14,
                        mouthAnchors = data.frame(time = c(0, 1), value = c(.5, .5)),
                        amplAnchors = NA, amplAnchorsGlobal = NA, samplingRate = 16000, windowLength = 50,
                        overlap = 75, addSilence = 100, pitchFloor = 50, pitchCeiling = 3500,
                        pitchSamplingRate = 3500, throwaway = -120,
                        invalidArgAction = c('adjust', 'abort', 'ignore')[1],
                        plot = FALSE, play = FALSE, savePath = NA, ...) {
  a = as.list(environment())
  a$plot = a$play = a$savePath = NULL
  bout = .Call(C_sg_soundgen, .sg_soundgen_args(a))
  if (!is.na(savePath)) seewave::savewav(bout, filename = savePath, f = samplingRate)  # R/soundgen.R:854-856
  bout
}

# The argument coercions of R/soundgen.R:305-315, :384-389, applied to a named
# list holding EVERY soundgen() formal (as.list(environment()) of soundgen_hip,
# or its formals overridden by one call's arguments in soundgen_batch), so the
# default pitch contour, the vowel-'a' formants and the noise/mouth anchors
# reach the planner as R would use them.
.sg_soundgen_args = function(a) {
  # a tempEffects list naming only some effects keeps the others' defaults
  # (R/soundgen.R:458-470 reads them by name); flattened in the ABI's order
  te = list(sylLenDep = .02, formDrift = .3, formDisp = .2, pitchDriftDep = .5, pitchDriftFreq = .125,
            pitchAnchorsDep = .05, noiseAnchorsDep = .1, amplAnchorsDep = .1)
  te[names(a$tempEffects)] = a$tempEffects
  a$tempEffects = as.double(unlist(te[c('sylLenDep', 'formDrift', 'formDisp', 'pitchDriftDep', 'pitchDriftFreq',
                                        'pitchAnchorsDep', 'noiseAnchorsDep', 'amplAnchorsDep')]))
  a$invalidArgAction = match(a$invalidArgAction, c('adjust', 'abort', 'ignore')) - 1L
  if (is.character(a$formants)) a$formants = convertStringToFormants(a$formants)
  # R/soundgen.R:662: noise formants "move" when max(lengths(formantsNoise)) > 1,
  # evaluated on the caller's value (a string counts 1, a formant list its fields)
  a$formantsNoise_rlen = if (length(a$formantsNoise) && !is.na(a$formantsNoise[1]))
    as.integer(max(unlist(lapply(a$formantsNoise, length)))) else 0L
  if (is.character(a$formantsNoise)) a$formantsNoise = convertStringToFormants(a$formantsNoise)
  for (nm in c('pitchAnchors', 'pitchAnchorsGlobal', 'noiseAnchors', 'mouthAnchors', 'amplAnchors',
               'amplAnchorsGlobal')) {
    a[nm] = list(.sg_anchors(a[[nm]]))  # a[nm] = list(NULL) keeps the entry: NA travels as NULL
  }
  a$formants_flat = .sg_flatten_formants(a$formants)
  a$formantsNoise_flat = .sg_flatten_formants(a$formantsNoise)
  a$formants = a$formantsNoise = NULL
  a
}

# anchors -> data.frame(time, value) of doubles, or NULL for NA / NULL; a
# numeric vector spans time 0..1 (R/soundgen.R:305-311)
.sg_anchors = function(v) {
  if (is.numeric(v) && length(v) > 0) v = data.frame(time = seq(0, 1, length.out = length(v)), value = v)
  if (is.list(v) && length(v) >= 2)
    return(data.frame(time = as.double(v$time), value = as.double(v$value)))
  NULL
}

# soundgen() over a list of calls (each a list of soundgen() arguments; the
# others take soundgen's defaults), planned as ONE batch and executed in one
# device pass: the drop-in for R loops such as R/morph.R:200-208 and the
# population loop of matchPars (R/matchPars.R:176-190). R's RNG is drawn in call
# order, so after set.seed() it returns what
# lapply(calls, function(cl) do.call(soundgen, cl)) returns. The batch runs on
# the devices of `devices` (device ordinals; default: device 0, the device the
# other entry points use, so one R process per GPU stays on its GPU; "all": every
# visible MI355X), sharded by calls inside the library (sg_node), each device's
# shard over its own link.
soundgen_batch = function(calls, devices = getOption("soundgen_hip.devices", 0L)) {
  dflt = formals(soundgen_hip)
  dflt$... = dflt$plot = dflt$play = dflt$savePath = NULL
  dflt = lapply(dflt, eval)
  args = lapply(calls, function(cl) {
    a = dflt
    a[names(cl)] = cl
    .sg_soundgen_args(a)
  })
  .Call(C_sg_soundgen_batch, args, if (identical(devices, "all")) -1L else as.integer(devices))
}

# R/source.R:57-68: the reference's formals and defaults verbatim
generateNoise = function(len,
                         noiseAnchors = data.frame('time' = c(0, 300), 'value' = c(-120, -120)),
                         rolloffNoise = -6, attackLen = 10, windowLength_points = 1024, samplingRate = 16000,
                         overlap = 75, throwaway = -120, filterNoise = NA) {
  pars = list(rolloffNoise = rolloffNoise, attackLen = attackLen, windowLength_points = windowLength_points,
              samplingRate = samplingRate, overlap = overlap, throwaway = throwaway)
  fn = NULL
  if (!is.na(filterNoise[1])) {  # an nr x nc matrix (R/source.R:98-104); a vector is one column
    fn = as.matrix(filterNoise)
    storage.mode(fn) = 'double'
  }
  .Call(C_sg_generate_noise, as.double(len), .sg_anchors(noiseAnchors), pars, fn)
}

# R/sourceSpectrum.R:261-283: the reference's formals and defaults verbatim;
# the formants coercion of R/sourceSpectrum.R:284-293, the matrix from the
# device, the plot of R/sourceSpectrum.R:541-562
getSpectralEnvelope = function(nr, nc, formants = NA, formantDep = 1, rolloffLip = 6, mouthAnchors = NA,
                               mouthOpenThres = 0, openMouthBoost = 0, vocalTract = NULL, temperature = 0,
                               formDrift = .3, formDisp = .2, formantDepStoch = 30, smoothLinearFactor = 1,
                               samplingRate = 16000, speedSound = 35400, plot = FALSE, duration = NULL,
                               colorTheme = c('bw', 'seewave', '...')[1], nCols = 100, xlab = 'Time',
                               ylab = 'Frequency, kHz', ...) {
  if (is.character(formants)) {
    formants = convertStringToFormants(formants)
  } else if (is.list(formants)) {
    if (is.list(formants[[1]])) formants = lapply(formants, as.data.frame)
  } else if (!is.null(formants) && !is.na(formants)) {
    stop('If defined, formants must be a list or a string of characters
          from dictionary presets: a, o, i, e, u, 0 (schwa)')
  }
  pars = list(formantDep = formantDep, rolloffLip = rolloffLip, mouthOpenThres = mouthOpenThres,
              openMouthBoost = openMouthBoost, vocalTract = if (is.numeric(vocalTract)) vocalTract else NA_real_,
              temperature = temperature, formDrift = formDrift, formDisp = formDisp,
              formantDepStoch = formantDepStoch, smoothLinearFactor = smoothLinearFactor,
              samplingRate = samplingRate, speedSound = speedSound)
  # mouth anchors with any NA: the half-open mouth (R/sourceSpectrum.R:431-434)
  ma = if (length(mouthAnchors) < 1 || sum(is.na(mouthAnchors)) > 0) NULL else .sg_anchors(mouthAnchors)
  spectralEnvelope = .Call(C_sg_spectral_envelope, as.integer(nr), as.integer(nc),
                           .sg_flatten_formants(formants), pars, ma)
  if (plot) {
    x = if (is.numeric(duration)) seq(0, duration, length.out = nc) else seq(0, 1, length.out = nc)
    col = if (colorTheme == 'bw') gray(seq(from = 1, to = 0, length = nCols)) else
      if (colorTheme == 'seewave') seewave::spectro.colors(nCols) else rev(match.fun(colorTheme)(nCols))
    image(x = x, y = seq(0, samplingRate / 2, length.out = nr) / 1000, z = t(spectralEnvelope),
          xlab = xlab, ylab = ylab, col = col, ...)
  }
  spectralEnvelope
}
