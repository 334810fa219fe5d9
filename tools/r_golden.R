# tools/r_golden.R -- write R-derived golden vectors for the parity tests.
#
# R is absent from the build container, so the committed golden vectors
# (tests/golden/*.npz) come from the C restatement (oracle/). Anyone with R
# and the reference package (soundgen 1.0.0, seewave 2.0.5, tuneR) can run
#
#     Rscript tools/r_golden.R tests/golden/r
#
# to write the same deterministic cases from R itself as CSV files;
# tests/test_r_golden.py then checks the oracle (and through it the GPU path)
# against them, pinning the restatement -- loess contours included.
args <- commandArgs(trailingOnly = TRUE)
out <- if (length(args) > 0) args[1] else file.path("tests", "golden", "r")
dir.create(out, recursive = TRUE, showWarnings = FALSE)
suppressMessages(library(soundgen))
w <- function(name, x) {
  write.csv(data.frame(x = as.numeric(x)), file.path(out, paste0(name, ".csv")), row.names = FALSE)
}
gh <- soundgen:::generateHarmonics
gsc <- soundgen:::getSmoothContour

# generateHarmonics, deterministic (temperature = 0)
w("harm_roxygen", gh(pitch = seq(200, 300, length.out = 3500), samplingRate = 16000))
w("harm_tone_150_16k", gh(pitch = rep(150, 1750), samplingRate = 16000, rolloff = -12, rolloffOct = -12,
                          pitchFloor = 50))
w("harm_c2_237", gh(pitch = rep(237, 3500), samplingRate = 44100, pitchSamplingRate = 3500, temperature = 0,
                    nonlinBalance = 0, attackLen = 50, rolloff = -12, rolloffOct = -12, rolloffKHz = -6,
                    rolloffParab = 0, rolloffParabHarm = 3, pitchFloor = 50, pitchCeiling = 3500,
                    throwaway = -120))

# getSmoothContour: loess (3-10 anchors), the default method
w("contour_default_pitch", gsc(anchors = data.frame(time = c(0, .1, .9, 1), value = c(100, 150, 135, 100)),
                               len = 1050, thisIsPitch = TRUE, valueFloor = 50, valueCeiling = 3500,
                               samplingRate = 3500))
w("contour_ampl4", gsc(anchors = data.frame(time = c(0, .3, .6, 1), value = c(0, 40, 10, 20)), len = 5000,
                       valueFloor = 0, samplingRate = 16000))
w("contour_noise5", gsc(anchors = data.frame(time = c(0, 200, 500, 900, 1000),
                                             value = c(-30, -10, -40, -20, -25)),
                        len = 16000, valueFloor = -120, valueCeiling = 40, samplingRate = 16000))

# soundgen(), deterministic
w("soundgen_c1_pin", soundgen(sylLen = 1000, samplingRate = 16000, temperature = 0, addSilence = 0,
                              pitchAnchors = data.frame(time = c(0, 1), value = c(100, 150))))
w("soundgen_default_pitch", soundgen(sylLen = 300, samplingRate = 16000, temperature = 0, addSilence = 0))
cat("wrote golden vectors to", out, "\n")
