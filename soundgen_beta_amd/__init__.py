"""soundgen_beta_amd — MI355X-native engine for soundgen's additive-source +
formant-filter hot path. The R-level API is mirrored in
`api` (soundgen, generateHarmonics, getRolloff, ...) and the batch path in
`batch`; all synthesis runs in libsoundgen_hip.so (HIP, gfx950)."""
from .api import (formantFilter, generateHarmonics, generateNoise, getRolloff,  # noqa: F401
                  getSpectralEnvelope, soundgen)
from .rargs import convertStringToFormants  # noqa: F401

__version__ = "0.1.0"
