// Resampling kernel descriptor shared by resample.hip and the fused STOI kernels.
#pragma once
#include <math.h>

#include "fsem_common.h"

#define FSEM_RS_MAX_COEF 512

namespace fsem {

// Largest filter (taps = 2 * width + orig) any rate pair may have: FSEM_ERATE beyond it.
#define RS_BIG_TAPS 8192

struct ResampleKernel {
  int orig, nw, taps, width;  // reduced rates, taps = 2*width + orig
  int big;                    // nw * taps > FSEM_RS_MAX_COEF: k unused, built on the device
  float k[FSEM_RS_MAX_COEF];  // [nw][taps]
};

// Coefficient (phase j, tap t) of torchaudio 2.8's _get_sinc_resample_kernel (sinc_interp_hann,
// lowpass_filter_width 6, rolloff 0.99; float64 build, float32 phase offsets, cast to float32)
// for the reduced rate pair orig -> nw.  Host and device evaluate the same float64 expression.
__host__ __device__ inline float sinc_coef(int j, int t, int orig, int nw, int width) {
  const double pi = 3.14159265358979323846;
  const double base = (double)(orig < nw ? orig : nw) * 0.99;
  const float ph32 = (float)(-j) / (float)nw;  // int arange / int -> float32 in torchaudio
  double tt = ((double)ph32 + (double)(t - width) / orig) * base;
  if (tt < -6.0) tt = -6.0;
  if (tt > 6.0) tt = 6.0;
  const double c = cos(tt * pi / 6.0 / 2.0);
  const double win = c * c;
  tt *= pi;
  const double s = (tt == 0.0) ? 1.0 : sin(tt) / tt;
  return (float)(s * (win * (base / orig)));
}

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
