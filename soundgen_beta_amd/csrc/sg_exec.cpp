// sg_exec.cpp — HBM arena for a plan and the per-batch launch sequence.
#include "sg_exec.h"

#include <cstring>
#include <string>

namespace sg {

namespace {
#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t _e = (x);                                                                  \
    if (_e != hipSuccess)                                                                 \
      throw SgError(SG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e));     \
  } while (0)

constexpr size_t ALIGN = 256;
size_t up(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

struct Layout {
  size_t segs, epochs, knots, amps, tiles, pieces, syls, syl_tiles, ptiles, cknots, W, maxes, total;
  explicit Layout(const Batch& B) {
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o += up(bytes > 0 ? bytes : 1); return r; };
    segs = take(B.segs.size() * sizeof(SgSeg));
    epochs = take(B.epochs.size() * sizeof(SgEpoch));
    knots = take(B.knots.size() * sizeof(double));
    amps = take(B.amps.size() * sizeof(float) + 64 * sizeof(float));
    tiles = take(B.tiles.size() * sizeof(SgTile));
    pieces = take(B.pieces.size() * sizeof(SgPiece));
    syls = take(B.syls.size() * sizeof(SgSyllable));
    syl_tiles = take(B.syl_tiles.size() * sizeof(SgSylTile));
    ptiles = take(B.ptiles.size() * sizeof(SgSylTile));
    cknots = take(B.cknots.size() * sizeof(double));
    W = take((size_t)B.w_total * sizeof(float));
    maxes = take(B.syls.size() * sizeof(unsigned));
    total = o;
  }
};
}  // namespace

void finalize_plan(Batch& B) {
  B.ptiles.clear();
  for (size_t s = 0; s < B.syls.size(); ++s) {
    const SgSyllable& sy = B.syls[s];
    for (int32_t p = sy.piece0; p < sy.piece0 + sy.npiece; ++p)
      if (B.pieces[p].nterms > 0)
        for (int64_t q0 = 0; q0 < B.pieces[p].len; q0 += 256) B.ptiles.push_back(SgSylTile{(int32_t)s, p, q0});
  }
}

int64_t device_bytes(const Batch& B) { return (int64_t)Layout(B).total; }

void device_free(DevicePlan& D) {
  if (D.arena) hipFree(D.arena);
  D = DevicePlan{};
}

void device_upload(const Batch& B, DevicePlan& D, hipStream_t s) {
  Layout L(B);
  if (D.arena && D.arena_bytes < L.total) device_free(D);
  if (!D.arena) {
    HIPCHK(hipMalloc(&D.arena, L.total));
    D.arena_bytes = L.total;
  }
  char* a = D.arena;
  D.segs = (SgSeg*)(a + L.segs);
  D.epochs = (SgEpoch*)(a + L.epochs);
  D.knots = (double*)(a + L.knots);
  D.amps = (float*)(a + L.amps);
  D.tiles = (SgTile*)(a + L.tiles);
  D.pieces = (SgPiece*)(a + L.pieces);
  D.syls = (SgSyllable*)(a + L.syls);
  D.syl_tiles = (SgSylTile*)(a + L.syl_tiles);
  D.ptiles = (SgSylTile*)(a + L.ptiles);
  D.cknots = (double*)(a + L.cknots);
  D.W = (float*)(a + L.W);
  D.maxes = (unsigned*)(a + L.maxes);
  auto cp = [&](void* dst, const void* src, size_t bytes) {
    if (bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
  };
  cp(D.segs, B.segs.data(), B.segs.size() * sizeof(SgSeg));
  cp(D.epochs, B.epochs.data(), B.epochs.size() * sizeof(SgEpoch));
  cp(D.knots, B.knots.data(), B.knots.size() * sizeof(double));
  cp(D.amps, B.amps.data(), B.amps.size() * sizeof(float));
  cp(D.tiles, B.tiles.data(), B.tiles.size() * sizeof(SgTile));
  cp(D.pieces, B.pieces.data(), B.pieces.size() * sizeof(SgPiece));
  cp(D.syls, B.syls.data(), B.syls.size() * sizeof(SgSyllable));
  cp(D.syl_tiles, B.syl_tiles.data(), B.syl_tiles.size() * sizeof(SgSylTile));
  cp(D.ptiles, B.ptiles.data(), B.ptiles.size() * sizeof(SgSylTile));
  cp(D.cknots, B.cknots.data(), B.cknots.size() * sizeof(double));
  HIPCHK(hipStreamSynchronize(s));
  D.uploaded = true;
}

void device_execute(const Batch& B, const DevicePlan& D, float* d_out, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  if (!B.syls.empty()) HIPCHK(hipMemsetAsync(D.maxes, 0, B.syls.size() * sizeof(unsigned), s));
  if (e0) HIPCHK(hipEventRecord(e0, s));
  launch_sine_bank(D, (int64_t)B.tiles.size(), s);
  if (e1) HIPCHK(hipEventRecord(e1, s));
  launch_piece_max(D, (int64_t)B.ptiles.size(), s);
  launch_harm_finalize(D, (int64_t)B.syl_tiles.size(), d_out, s);
  HIPCHK(hipGetLastError());
}

}  // namespace sg
