// Resampling kernel descriptor shared by resample.hip and the fused STOI kernels.
#pragma once
#include "fsem_common.h"

#define FSEM_RS_MAX_COEF 512

namespace fsem {

struct ResampleKernel {
  int orig, nw, taps, width;  // reduced rates, taps = 2*width + orig
  float k[FSEM_RS_MAX_COEF];  // [nw][taps]
};

int make_resample_kernel(int32_t orig_freq, int32_t new_freq, ResampleKernel *rk);

// Polyphase resampler for any rate pair (resample.hip): rows r of `in` (row length n = lens[r]
// clamped to [0, n_in], or n_in) -> out + r * ld_out, ceil(n * nw / orig) samples; columns
// [ceil(n * nw / orig), zc) are zeroed (zc <= ceil(n_in * nw / orig); 0: none).
int launch_resample_tiled(const float *in, int64_t rows, int64_t n_in, int64_t ld_in, const int32_t *lens,
                          float *out, int64_t ld_out, int64_t zc, const ResampleKernel &rk, hipStream_t st);

// One output sample o of a row x[0..n): torchaudio's pad + strided conv1d.
__device__ __forceinline__ float resample_at(const float *__restrict__ x, int64_t n, int64_t o,
                                             const ResampleKernel &rk) {
  const int64_t m = o / rk.nw;
  const int j = (int)(o - m * rk.nw);
  const int64_t base = m * rk.orig - rk.width;
  const float *kj = rk.k + j * rk.taps;
  float acc = 0.f;
  if (base >= 0 && base + rk.taps <= n) {
    for (int t = 0; t < rk.taps; ++t) acc = fmaf(kj[t], x[base + t], acc);
  } else {
    for (int t = 0; t < rk.taps; ++t) {
      const int64_t i = base + t;
      const float v = (i >= 0 && i < n) ? x[i] : 0.f;
      acc = fmaf(kj[t], v, acc);
    }
  }
  return acc;
}

}  // namespace fsem
