// sg_exec.h — device-side plan (HBM arena) and kernel launch sequence.
#pragma once
#include <hip/hip_runtime.h>

#include "sg_plan.h"

namespace sg {

struct DevicePlan {
  bool uploaded = false;
  char* arena = nullptr;
  size_t arena_bytes = 0;
  SgSeg* segs = nullptr;
  SgEpoch* epochs = nullptr;
  double* knots = nullptr;
  float* amps = nullptr;
  SgTile* tiles = nullptr;
  SgPiece* pieces = nullptr;
  SgSyllable* syls = nullptr;
  SgSylTile* syl_tiles = nullptr;
  SgSylTile* ptiles = nullptr;
  double* cknots = nullptr;
  float* W = nullptr;
  unsigned* maxes = nullptr;
};

int64_t device_bytes(const Batch& B);
void device_upload(const Batch& B, DevicePlan& D, hipStream_t s);
void device_free(DevicePlan& D);
// e0/e1 (optional) bracket the sine-bank launch for profiling
void device_execute(const Batch& B, const DevicePlan& D, float* d_out, hipStream_t s, hipEvent_t e0, hipEvent_t e1);

// launchers (sg_harm.hip)
void launch_sine_bank(const DevicePlan& D, int64_t n_tiles, hipStream_t s);
void launch_piece_max(const DevicePlan& D, int64_t n_ptiles, hipStream_t s);
void launch_harm_finalize(const DevicePlan& D, int64_t n_stiles, float* out, hipStream_t s);

}  // namespace sg
