"""R's default random number generator (R 3.4.0: Mersenne-Twister with
set.seed() scrambling, Inversion normals, Ahrens-Dieter exp/gamma), implemented
in the library (csrc/sg_rrng.cpp, include/soundgen_hip.h sg_rrng_*).

    rng = RRng(1)                 # set.seed(1)
    soundgen(temperature=0.1, rng=rng)   # draws what set.seed(1); soundgen(...) draws in R

Passed as `rng=` to soundgen()/generateHarmonics()/generateNoise()/
getSpectralEnvelope() (and to the oracle in tests), the generator is bound to
the planner's callbacks natively (sg_random_bind_rrng): one stream, R's order.
It also offers numpy-Generator-style methods (random, standard_normal,
standard_exponential, gamma) so code written for a numpy draw source works.
"""
import ctypes as C

from . import native


class RRng:
    def __init__(self, seed):
        L = native.lib()
        self._L = L
        self.ptr = C.c_void_p()
        native.check(L.sg_rrng_create(int(seed), C.byref(self.ptr)))

    def set_seed(self, seed):
        self._L.sg_rrng_set_seed(self.ptr, int(seed))

    def random(self, size=None):
        return self._many(self._L.sg_rrng_unif, size)

    def standard_normal(self, size=None):
        return self._many(self._L.sg_rrng_norm, size)

    def standard_exponential(self, size=None):
        return self._many(self._L.sg_rrng_exp, size)

    def gamma(self, shape, scale=1.0, size=None):
        f = lambda p: self._L.sg_rrng_gamma(p, float(shape), float(scale))  # noqa: E731
        return self._many(f, size)

    def _many(self, f, size):
        if size is None:
            return float(f(self.ptr))
        import numpy as np
        return np.array([f(self.ptr) for _ in range(int(size))])

    def bind(self, rnd):
        """Point an _abi.sg_random's callbacks at this generator."""
        self._L.sg_random_bind_rrng(C.byref(rnd), self.ptr)

    def __del__(self):
        try:
            if self.ptr:
                self._L.sg_rrng_destroy(self.ptr)
                self.ptr = C.c_void_p()
        except Exception:
            pass
