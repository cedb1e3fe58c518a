// Polyphase windowed-sinc resampler = torchaudio.transforms.Resample (sinc_interp_hann,
// lowpass_filter_width 6, rolloff 0.99), the resampler of BaseMetric.prepare_audio
// (reference fast_se_metrics/base.py:13,19-20).
//
//   out[r, m*new + j] = sum_t K[j, t] * x[r, m*orig + t - width]     (x = 0 outside [0, n))
//   n_out = ceil(new * n / orig)
//
// The [new, taps] kernel is built on the host in float64 exactly like torchaudio's
// _get_sinc_resample_kernel (including its float32 phase offsets) and passed by value.
#include <math.h>

#include "fsem_resample.h"

namespace fsem {

int make_resample_kernel(int32_t orig_freq, int32_t new_freq, ResampleKernel *rk) {
  if (orig_freq <= 0 || new_freq <= 0) return FSEM_ERATE;
  int32_t a = orig_freq, b = new_freq;
  while (b) {
    int32_t t = a % b;
    a = b;
    b = t;
  }
  const int32_t g = a;
  const int orig = orig_freq / g, nw = new_freq / g;
  const double base = (double)(orig < nw ? orig : nw) * 0.99;
  const int width = (int)ceil(6.0 * orig / base);
  const int taps = 2 * width + orig;
  if ((int64_t)nw * taps > FSEM_RS_MAX_COEF) return FSEM_ERATE;
  rk->orig = orig;
  rk->nw = nw;
  rk->taps = taps;
  rk->width = width;
  const double pi = 3.14159265358979323846;
  for (int j = 0; j < nw; ++j) {
    const float ph32 = (float)(-j) / (float)nw;  // int arange / int -> float32 in torchaudio
    for (int t = 0; t < taps; ++t) {
      double tt = ((double)ph32 + (double)(t - width) / orig) * base;
      if (tt < -6.0) tt = -6.0;
      if (tt > 6.0) tt = 6.0;
      const double c = cos(tt * pi / 6.0 / 2.0);
      const double win = c * c;
      tt *= pi;
      const double s = (tt == 0.0) ? 1.0 : sin(tt) / tt;
      rk->k[j * taps + t] = (float)(s * (win * (base / orig)));
    }
  }
  return FSEM_OK;
}

__global__ void __launch_bounds__(256) resample_kernel(const float *__restrict__ in, int64_t n_in,
                                                       int64_t ld_in, float *__restrict__ out,
                                                       int64_t n_out, int64_t ld_out,
                                                       ResampleKernel rk) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = blockIdx.y;
  if (o >= n_out) return;
  out[r * ld_out + o] = resample_at(in + r * ld_in, n_in, o, rk);
}

}  // namespace fsem

extern "C" int64_t fsem_resample_length(int64_t n_in, int32_t orig_freq, int32_t new_freq) {
  fsem::ResampleKernel rk;
  if (orig_freq == new_freq) return n_in;
  if (fsem::make_resample_kernel(orig_freq, new_freq, &rk) != FSEM_OK) return -1;
  return (rk.nw * n_in + rk.orig - 1) / rk.orig;
}

extern "C" int fsem_resample_f32(const float *in, int64_t rows, int64_t n_in, int64_t ld_in,
                                 float *out, int64_t ld_out, int32_t orig_freq, int32_t new_freq,
                                 void *stream) {
  if (!in || !out || rows < 0 || n_in < 0 || ld_in < n_in) return FSEM_EINVAL;
  if (rows == 0 || n_in == 0) return FSEM_OK;
  fsem::ResampleKernel rk;
  int rc = fsem::make_resample_kernel(orig_freq, new_freq, &rk);
  if (rc != FSEM_OK) return rc;
  const int64_t n_out = (rk.nw * n_in + rk.orig - 1) / rk.orig;
  if (ld_out < n_out || rows > 65535) return FSEM_EINVAL;
  dim3 grid((unsigned)((n_out + 255) / 256), (unsigned)rows);
  hipLaunchKernelGGL(fsem::resample_kernel, grid, dim3(256), 0, (hipStream_t)stream, in, n_in,
                     ld_in, out, n_out, ld_out, rk);
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}
