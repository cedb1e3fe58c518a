// Shared geometry of the PESQ front end (pesq.hip) and back end (pesq_back.hip): frames,
// segments and the band-major Bark layout of a row (PESQ.py:123-140, bark.py:189-204).
#pragma once
#include "fsem_common.h"

namespace fsem {
namespace pesq {

constexpr int NF = 48;            // frames per segment
constexpr int OWN = NF * 256;     // samples of band-pass power owned per segment
constexpr int NBARK = 49;
constexpr int PESQ_CH = FSEM_PESQ_CH;
constexpr int PESQ_TILE = 256 * PESQ_CH;  // 13312
constexpr int PESQ_WARM = 768;

// Bark bands are stored band-major per signal: bark[(s * NBARK + k) * bark_ld(F) + f], rows
// padded to a multiple of 32 frames: every row starts on a 128-byte line, so the back end's
// loads of one band over 64 consecutive frames (lane = frame) touch exactly two lines (a
// 4-frame padding left them straddling three: 1.25x the HBM reads), and the MFMA tiles' float4
// stores stay aligned.
__host__ __device__ inline int64_t bark_ld(int F) { return (F + 31) & ~31; }

__host__ __device__ inline int frames_of(int64_t L) {
  const int64_t Lp = L + (L % 256);  // PESQ.py:128-130: pad by L % 256 (sic)
  if (Lp < 512) return 0;
  return (int)(1 + (Lp - 512) / 256);
}

struct Geometry {
  int F, nfseg, npseg, nseg;
};

// Segment g owns band-pass power samples [g*OWN, (g+1)*OWN); the LAST segment owns
// [g*OWN, L), which its tile must cover: L - (nseg-1)*OWN <= PESQ_TILE - PESQ_WARM.  Every field is
// non-decreasing in L, so the geometry of the longest row bounds every shorter row's.
__host__ __device__ inline Geometry geometry(int64_t L) {
  Geometry g;
  g.F = frames_of(L);
  g.nfseg = (g.F + NF - 1) / NF;
  const int64_t span = PESQ_TILE - PESQ_WARM;
  g.npseg = L <= span ? 1 : (int)((L - span + OWN - 1) / OWN) + 1;
  g.nseg = g.nfseg > g.npseg ? g.nfseg : g.npseg;
  return g;
}

// Row length of utterance b: the per-row length when given (clamped to [0, L]), else L.
__device__ __forceinline__ int64_t row_length(const int32_t *__restrict__ lens, int64_t b, int64_t L) {
  if (!lens) return L;
  const int64_t n = lens[b];
  return n < 0 ? 0 : (n > L ? L : n);
}


// front workspace: per-segment power partials [2B, nseg, 4] float, then the segments' range
// shifts [2B, nseg] int (pesq_front's pexp)
inline size_t front_ppart_bytes(int64_t batch, int64_t length) {
  return align_up(sizeof(float) * (size_t)(2 * batch) * (size_t)geometry(length).nseg * 4, 256);
}

}  // namespace pesq
}  // namespace fsem
