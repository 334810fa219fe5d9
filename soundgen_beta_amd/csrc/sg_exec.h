// sg_exec.h — device-side plan (HBM arena) and kernel launch sequence.
#pragma once
#include <hip/hip_runtime.h>

#include <utility>
#include <vector>

#include "sg_plan.h"

namespace sg {

// per-call 16-bit PCM conversion of a plan's output (sg_wav.hip); built on first use
struct PcmJob {
  char* buf = nullptr;
  SgPcmCall* calls = nullptr;
  SgPcmTile* tiles = nullptr;
  SgPcmStat* stats = nullptr;
  int64_t n = 0, ntiles = 0;
  void prepare(const int64_t* off, const int64_t* len, int64_t n_calls, hipStream_t s);
  void run(const void* in, bool f64, int mode, double nrange, int16_t* out, hipStream_t s) const;
  void free();
};

struct DevicePlan {
  bool uploaded = false;
  char* arena = nullptr;
  size_t arena_bytes = 0;
  SgSeg* segs = nullptr;
  SgEpoch* epochs = nullptr;
  double* knots = nullptr;
  float* amps = nullptr;
  const SgAmpCol* ampcols = nullptr;  // sg_amp_build inputs (read at upload)
  const SgAmpJob* ampjobs = nullptr;
  const float* ampsrc = nullptr;
  SgWTask* tasks = nullptr;
  int32_t* tall = nullptr;           // indices of tasks with R > SG_ROWS_F32 (sg_sine_bank_tall)
  std::vector<int32_t> tall_host;
  int32_t* tlong = nullptr;          // fp32 tasks run one per wave (sg_sine_bank)
  std::vector<int32_t> tlong_host;
  int32_t* tshort = nullptr;         // fp32 tasks of <= 64 samples, two per wave (sg_sine_bank_pairs)
  std::vector<int32_t> tshort_host;
  int32_t* tallp = nullptr;          // tall tasks of <= 64 samples, two per wave (sg_sine_bank_tall_pairs)
  std::vector<int32_t> tallp_host;
  // runs of the two short lists: consecutive entries of one syllable, <= SG_RUN_TASKS each,
  // one wave per run (positions in tshort / tallp where each run starts, then the list size)
  int32_t* srun = nullptr;
  std::vector<int32_t> srun_host;
  int32_t* trun = nullptr;
  std::vector<int32_t> trun_host;
  int32_t* thp = nullptr;            // SG_TASK_HP tasks (sg_sine_bank_hp)
  std::vector<int32_t> thp_host;
  // wavetable path (SgTabJob): tasks of long static-tone spans
  // (a separate allocation made at upload)
  char* tabbuf = nullptr;              // the wavetable spans' jobs (sg_sine_bank_tab)
  size_t tabbuf_bytes = 0;
  SgTabJob* tabjobs = nullptr;         // in task order
  std::vector<SgTabJob> tabjobs_host;
  int64_t tab_samples = 0, tab_terms = 0;  // samples and (sample, row) terms the tables stand in for
  SgSylTile* fin_tiles_hp = nullptr; // finalize tiles of fp64 syllables (sg_harm_finalize_hp)
  double* W64 = nullptr;             // fp64 epoch waveforms of SG_TASK_HP tasks
  double* fh = nullptr;              // fp64 sounds (voiced parts, pre-filter sounds) of fp64 bouts
  SgFrame64* frames64 = nullptr;     // their filter frames (sg_fft_frames64)
  int64_t* frames64_tab = nullptr;   // per frame: offset of its root table in roots64
  double* roots64 = nullptr;         // W_N^t tables (double2), one per window length (sg_roots64)
  int32_t* roots64_wl = nullptr;
  int64_t* roots64_off = nullptr;
  SgPiece* pieces = nullptr;
  SgSyllable* syls = nullptr;
  SgSylTile* syl_tiles = nullptr;    // general-path finalize tiles (Batch::fin_tiles)
  SgCopyTile* copy_tiles = nullptr;
  SgSylTile* ptiles = nullptr;
  double* cknots = nullptr;
  float* W = nullptr;
  float* taskmax = nullptr;
  float* ptilemax = nullptr;
  float* maxes = nullptr;
  SgFftGeom* geoms = nullptr;
  SgFrame* frames = nullptr;
  SgFrameGroup* fgroups = nullptr;
  SgOla* olas = nullptr;
  SgOlaTile* olatiles = nullptr;
  SgSegment* olasegs = nullptr;
  float* olatilemax = nullptr;
  float* olamax = nullptr;
  SgNoiseItem* items = nullptr;
  SgMix* mixes = nullptr;
  SgMixTile* mixtiles = nullptr;
  float* fl = nullptr;
  float* fs = nullptr;
  SgEnvTerm* eterms = nullptr;
  SgEnvCol* ecols = nullptr;
  SgEnvJob* envjobs = nullptr;
  SgEnvTask* envtasks = nullptr;
  double* elog2 = nullptr;
  PcmJob pcm;
  std::vector<hipEvent_t> ev_slice;  // slice c's maxes are ready (s -> s2)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

int64_t device_bytes(const Batch& B);
void device_upload(const Batch& B, DevicePlan& D, hipStream_t s);
void device_free(DevicePlan& D);
// HIP events bracketing one launch of a profiled kernel (SG_PROF_*), on its stream
struct SgProfEvent {
  int kernel;
  hipEvent_t e0, e1;
};
// Slice pipeline: sine bank + maxes of slice c on s, finalize of slice c on
// s2 (overlapping the sine bank of c+1); s waits for s2 at the end. prof
// (optional) receives one event pair per sine-bank and sg_stft_ola launch.
void device_execute(const Batch& B, DevicePlan& D, float* d_out, hipStream_t s, hipStream_t s2,
                    std::vector<SgProfEvent>* prof);
struct PlanRun {
  const Batch* B;
  DevicePlan* D;
  float* out;
};
void device_execute_many(const std::vector<PlanRun>& runs, hipStream_t s, hipStream_t s2,
                         std::vector<SgProfEvent>* prof);
void device_execute_spec(const Batch& B, const DevicePlan& D, float* d_out, hipStream_t s,
                         std::vector<SgProfEvent>* prof, bool join = false, hipEvent_t harm_done = nullptr);

// launchers (sg_harm.hip)
void launch_amp_build(const DevicePlan& D, int64_t n_jobs, hipStream_t s);
void launch_ugather(const SgUJob* jobs, int64_t n_jobs, const float* us, float* fl, hipStream_t s);
void launch_sine_bank(const DevicePlan& D, int64_t k0, int64_t n, hipStream_t s);
void launch_sine_bank_pairs(const DevicePlan& D, int64_t k0, int64_t n, hipStream_t s);
void launch_sine_bank_tall(const DevicePlan& D, int64_t k0, int64_t n, hipStream_t s);
void launch_sine_bank_tall_pairs(const DevicePlan& D, int64_t k0, int64_t n, hipStream_t s);
void launch_syl_max(const DevicePlan& D, int64_t s0, int64_t n_syls, hipStream_t s);
void launch_piece_max(const DevicePlan& D, int64_t p0, int64_t n_ptiles, hipStream_t s);
void launch_harm_finalize(const DevicePlan& D, int64_t f0, int64_t n_stiles, float* out, hipStream_t s);
void launch_harm_copy(const DevicePlan& D, int64_t c0, int64_t n_ctiles, float* out, hipStream_t s);
// the fp64 path of ill-conditioned formant-filter calls (SG_TASK_HP, SgSyllable::hp, sg_mix to fh, SgFrame64)
void launch_sine_bank_hp(const DevicePlan& D, int64_t n, hipStream_t s);
void launch_sine_bank_tab(const DevicePlan& D, int logn, int64_t j0, int64_t n, float* out, hipStream_t s);
void launch_piece_max_hp(const DevicePlan& D, int64_t p0, int64_t n_ptiles, hipStream_t s);
void launch_harm_finalize_hp(const DevicePlan& D, int64_t n_stiles, hipStream_t s);
void launch_mix_hp(const DevicePlan& D, int64_t t0, int64_t n_tiles, hipStream_t s);
void launch_fft_frames64(const DevicePlan& D, const Batch& B, int ph, hipStream_t s);
// sg_fft.hip
void launch_fft_frames(const DevicePlan& D, int64_t g0, int64_t n_groups, int lds_bytes, hipStream_t s);
void launch_stft_ola(const DevicePlan& D, int phase, int64_t s0, int64_t n_segs, int lds_bytes, hipStream_t s);
void launch_ola(const DevicePlan& D, int64_t t0, int64_t n_tiles, hipStream_t s);
void launch_ola_max(const DevicePlan& D, int64_t o0, int64_t n_olas, hipStream_t s);
void launch_fft_probe(const SgFftGeom* geom, const float* fl, float* data, int M, int nframes, int inverse,
                      hipStream_t s);
void launch_mix(const DevicePlan& D, int64_t t0, int64_t n_tiles, float* out, hipStream_t s);
// sg_env.hip: every spectral-envelope job of the plan (getSpectralEnvelope)
void launch_spec_env(const DevicePlan& D, const Batch& B, hipStream_t s);

}  // namespace sg
