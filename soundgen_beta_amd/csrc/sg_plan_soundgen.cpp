// sg_plan_soundgen.cpp — host planner of the soundgen() orchestration
// (R/soundgen.R:208-862). Filled in by the noise/formant-filter milestone.
#include "sg_plan.h"

namespace sg {

int64_t plan_soundgen(Batch&, const sg_soundgen_args&, Rng&, int64_t, int) {
  throw SgError(SG_E_UNSUPPORTED, "soundgen() batch path not implemented yet");
}

void restore_soundgen_tail(Batch&, int) {}

}  // namespace sg
