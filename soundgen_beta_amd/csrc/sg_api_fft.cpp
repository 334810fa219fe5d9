// sg_api_fft.cpp — function-level entries of the noise source, spectral
// envelope and formant filter (filled in by the FFT milestone).
#include "sg_plan.h"

extern "C" {

void sg_default_soundgen_args(sg_soundgen_args* a) { *a = sg_soundgen_args{}; }

int sg_generate_noise(sg_ctx*, int64_t, sg_anchors, double, double, int32_t, double, double, double,
                      const double*, int32_t, const sg_random*, double*) {
  return SG_E_UNSUPPORTED;
}

int sg_spectral_envelope(sg_ctx*, int32_t, int32_t, const sg_formants*, double, double, sg_anchors, double, double,
                         double, double, double, double, double, double, double, double, const sg_random*,
                         double*) {
  return SG_E_UNSUPPORTED;
}

int sg_formant_filter(sg_ctx*, const double*, int64_t, const double*, int32_t, int32_t, double, double*, int64_t,
                      int64_t*) {
  return SG_E_UNSUPPORTED;
}

}  // extern "C"
