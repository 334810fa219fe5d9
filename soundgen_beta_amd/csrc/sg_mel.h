// sg_mel.h — compareSounds() / getMelSpec() on the device (sg_mel.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "soundgen_hip.h"

namespace sg {

// tuneR melfcc geometry of one parameter set (host, fp64, R's operation order)
struct MelGeom {
  int winpts = 0, steppts = 0, nfft = 0, nfreqs = 0, nb = 0;
  double thr = 0;                      // 2^(throwaway / 10)
  std::vector<double> ham;             // hamming(winpts)
  std::vector<int32_t> band_k0, band_n, band_w0;  // per mel band: its bins' weights
  std::vector<double> w;
  std::vector<double> tw, twN;         // e^{-2 pi i t / M} (t < M/2), e^{-2 pi i k / nfft} (k < M), (re, im)
};
MelGeom mel_geom(const sg_mel_params& p);
int mel_frames(const MelGeom& g, int64_t len);

// getMelSpec of one waveform already on the device: nb x nk column-major into out
void mel_spec_device(const MelGeom& g, const double* d_x, int64_t len, std::vector<double>& out, int* nk,
                     hipStream_t s);
// compareSounds(targetSpec = tspec (host, nb x ncT), cand = each candidate of
// d_x): out[4 c + m] per method (cor, cosine, pixel, dtw), summary[c]
void compare_sounds_device(const MelGeom& g, const double* tspec, int ncT, const float* d_x, const int64_t* offsets,
                           const int64_t* lengths, int64_t n, int methods, int penalize, double* out, double* summary,
                           hipStream_t s);

}  // namespace sg
