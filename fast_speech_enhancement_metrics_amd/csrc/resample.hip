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

#include <mutex>

#include "fsem_resample.h"

namespace fsem {

static int build_resample_kernel(int32_t orig_freq, int32_t new_freq, ResampleKernel *rk) {
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
  if (taps > RS_BIG_TAPS) return FSEM_ERATE;  // reduced input rate too large (see fsem.h)
  rk->orig = orig;
  rk->nw = nw;
  rk->taps = taps;
  rk->width = width;
  rk->big = (int64_t)nw * taps > FSEM_RS_MAX_COEF;
  if (rk->big) return FSEM_OK;  // coefficients built on the device (resample_sinc_lds)
  for (int j = 0; j < nw; ++j)
    for (int t = 0; t < taps; ++t) rk->k[j * taps + t] = sinc_coef(j, t, orig, nw, width);
  return FSEM_OK;
}

// The kernels of the last few rate pairs, kept so a call does not re-evaluate ~nw * taps float64
// sinc / cos terms (16 -> 10 kHz: 140) on the host each time.
int make_resample_kernel(int32_t orig_freq, int32_t new_freq, ResampleKernel *rk) {
  constexpr int kSlots = 8;
  struct Slot {
    int32_t orig_freq, new_freq;
    ResampleKernel rk;
  };
  static std::mutex mu;
  static Slot slots[kSlots];
  static int used = 0, next = 0;
  {
    std::lock_guard<std::mutex> lock(mu);
    for (int i = 0; i < used; ++i)
      if (slots[i].orig_freq == orig_freq && slots[i].new_freq == new_freq) {
        *rk = slots[i].rk;
        return FSEM_OK;
      }
  }
  const int rc = build_resample_kernel(orig_freq, new_freq, rk);
  if (rc != FSEM_OK) return rc;
  std::lock_guard<std::mutex> lock(mu);
  slots[next] = Slot{orig_freq, new_freq, *rk};
  next = (next + 1) % kSlots;
  if (used < kSlots) ++used;
  return FSEM_OK;
}

// Tiled form: a workgroup owns gt consecutive polyphase groups m (group m = inputs
// x[m*orig - width, +taps) -> outputs [m*nw, +nw)).  The input window and the [nw, taps]
// coefficients are staged in LDS with coalesced loads (zeros outside the row: torchaudio's
// padding), each thread evaluates one group, and the outputs leave through LDS as coalesced
// stores.  Same tap order as resample_at (bitwise the same samples).
constexpr int RS_T = 256;
constexpr int RS_XS = 8192 + FSEM_RS_MAX_COEF;  // staged inputs: GT*orig + taps <= this
__global__ void __launch_bounds__(RS_T) resample_tiled(const float *__restrict__ in, int64_t n_in, int64_t ld_in,
                                                      const int32_t *__restrict__ lens, float *__restrict__ out,
                                                      int64_t ld_out, int64_t zc, int gt, int64_t r0, ResampleKernel rk) {
  __shared__ float xs[RS_XS];
  __shared__ float ks[FSEM_RS_MAX_COEF];
  __shared__ float ys[RS_T * 8];
  const int tid = threadIdx.x;
  const int64_t r = r0 + blockIdx.y;
  int64_t n = n_in;
  if (lens) {
    const int64_t v = lens[r];
    n = v < 0 ? 0 : (v > n_in ? n_in : v);
  }
  const int orig = rk.orig, nw = rk.nw, taps = rk.taps;
  const int64_t n_out = (n * nw + orig - 1) / orig;
  const int64_t m0 = (int64_t)blockIdx.x * gt;
  if (m0 * nw >= n_out) {  // past the row: only the zero tail [n_out, zc)
    for (int64_t i = m0 * nw + tid; i < min((m0 + gt) * nw, zc); i += RS_T) out[r * ld_out + i] = 0.f;
    return;
  }
  const float *__restrict__ x = in + r * ld_in;
  const int64_t base = m0 * orig - rk.width;
  const int nx = (gt - 1) * orig + taps;
  for (int i = tid; i < nx; i += RS_T) {
    const int64_t t = base + i;
    xs[i] = (t >= 0 && t < n) ? x[t] : 0.f;
  }
  for (int i = tid; i < nw * taps; i += RS_T) ks[i] = rk.k[i];
  __syncthreads();
  // groups in chunks whose outputs fit the staging buffer; thread tid evaluates groups
  // g0 + tid, g0 + tid + RS_T, ...; outputs leave as coalesced stores
  constexpr int YS = RS_T * 8;
  const int gc = YS / nw;  // groups per chunk (nw <= FSEM_RS_MAX_COEF / taps < YS)
  for (int g0 = 0; g0 < gt; g0 += gc) {
    const int g1 = min(gt, g0 + gc);
    if (g0) __syncthreads();
    for (int g = g0 + tid; g < g1; g += RS_T) {
      const float *xg = xs + g * orig;
      for (int j = 0; j < nw; ++j) {
        const float *kj = ks + j * taps;
        float acc = 0.f;
        for (int t = 0; t < taps; ++t) acc = fmaf(kj[t], xg[t], acc);
        ys[(g - g0) * nw + j] = acc;
      }
    }
    __syncthreads();
    const int nc = (g1 - g0) * nw;
    const int64_t ob = (m0 + g0) * nw;
    for (int i = tid; i < nc; i += RS_T) {
      if (ob + i < n_out)
        out[r * ld_out + ob + i] = ys[i];
      else if (ob + i < zc)
        out[r * ld_out + ob + i] = 0.f;
    }
  }
}

// Specialisation for the common rate pairs (8 -> 16 kHz, 8 -> 10 kHz, 48 -> 16 kHz): each lane
// keeps its group's taps in registers and takes the coefficients from the kernel argument
// block by scalar loads (compile-time indices), so the inner loop is NW*TAPS register FMAs.
template <int ORIG, int NW, int TAPS>
__global__ void __launch_bounds__(RS_T) resample_tiled_t(const float *__restrict__ in, int64_t n_in, int64_t ld_in,
                                                        const int32_t *__restrict__ lens, float *__restrict__ out,
                                                        int64_t ld_out, int64_t zc, int gt, int64_t r0, ResampleKernel rk) {
  __shared__ float xs[RS_XS];
  __shared__ float ys[RS_T * 8];
  const int tid = threadIdx.x;
  const int64_t r = r0 + blockIdx.y;
  int64_t n = n_in;
  if (lens) {
    const int64_t v = lens[r];
    n = v < 0 ? 0 : (v > n_in ? n_in : v);
  }
  const int64_t n_out = (n * NW + ORIG - 1) / ORIG;
  const int64_t m0 = (int64_t)blockIdx.x * gt;
  if (m0 * NW >= n_out) {  // past the row: only the zero tail [n_out, zc)
    for (int64_t i = m0 * NW + tid; i < min((m0 + gt) * NW, zc); i += RS_T) out[r * ld_out + i] = 0.f;
    return;
  }
  const float *__restrict__ x = in + r * ld_in;
  const int64_t base = m0 * ORIG - rk.width;
  const int nx = (gt - 1) * ORIG + TAPS;
  for (int i = tid; i < nx; i += RS_T) {
    const int64_t t = base + i;
    xs[i] = (t >= 0 && t < n) ? x[t] : 0.f;
  }
  __syncthreads();
  constexpr int GC = RS_T * 8 / NW / RS_T * RS_T;  // groups per chunk, a multiple of RS_T
  static_assert(GC >= RS_T, "chunk holds one group per thread");
  for (int g0 = 0; g0 < gt; g0 += GC) {
    const int g1 = min(gt, g0 + GC);
    if (g0) __syncthreads();
    for (int g = g0 + tid; g < g1; g += RS_T) {
      float v[TAPS];
#pragma unroll
      for (int t = 0; t < TAPS; ++t) v[t] = xs[g * ORIG + t];
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < TAPS; ++t) acc = fmaf(rk.k[j * TAPS + t], v[t], acc);
        ys[(g - g0) * NW + j] = acc;
      }
    }
    __syncthreads();
    const int nc = (g1 - g0) * NW;
    const int64_t ob = (m0 + g0) * NW;
    for (int i = tid; i < nc; i += RS_T) {
      if (ob + i < n_out)
        out[r * ld_out + ob + i] = ys[i];
      else if (ob + i < zc)
        out[r * ld_out + ob + i] = 0.f;
    }
  }
}

// Direct form for the common rate pairs when rows are float4-aligned (row pointers 16-byte
// aligned, leading dimensions multiples of 4): thread t owns the G consecutive polyphase groups
// [m0, m0 + G) (G*ORIG and G*NW multiples of 4), loads the aligned float4 chunks covering their
// taps straight from global memory -- every load of the thread in flight at once; the chunks it
// shares with its neighbours come from L1/L2 -- and stores its G*NW outputs as float4s.  No LDS
// and no barriers (the tiled form above serialises stage -> barrier -> compute -> barrier ->
// store and reached ~1.1 TB/s).  Same tap order as resample_at: bitwise the same samples.
template <int ORIG, int NW, int TAPS, int G>
__global__ void __launch_bounds__(RS_T) resample_direct_t(const float *__restrict__ in, int64_t n_in, int64_t ld_in,
                                                         const int32_t *__restrict__ lens, float *__restrict__ out,
                                                         int64_t ld_out, int64_t zc, int64_t r0, ResampleKernel rk) {
  constexpr int W = (TAPS - ORIG) / 2;                 // rk.width
  constexpr int W4 = (W + 3) & ~3;                     // first chunk starts W4 before the group
  constexpr int NCH = ((G - 1) * ORIG + TAPS + (W4 - W) + 3) / 4;
  constexpr int NO = G * NW;
  static_assert((G * ORIG) % 4 == 0 && NO % 4 == 0, "float4 granularity");
  const int64_t r = r0 + blockIdx.y;
  int64_t n = n_in;
  if (lens) {
    const int64_t v = lens[r];
    n = v < 0 ? 0 : (v > n_in ? n_in : v);
  }
  const int64_t n_out = (n * NW + ORIG - 1) / ORIG;
  const int64_t m0 = ((int64_t)blockIdx.x * RS_T + threadIdx.x) * G;
  const int64_t ob = m0 * NW;
  if (ob >= n_out) {  // past the row: only the zero tail [n_out, zc)
    float *__restrict__ y = out + r * ld_out + ob;
    if (ob + NO <= zc) {
#pragma unroll
      for (int c = 0; c < NO / 4; ++c) *reinterpret_cast<float4 *>(y + 4 * c) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int i = 0; i < NO && ob + i < zc; ++i) y[i] = 0.f;
    }
    return;
  }
  const float *__restrict__ x = in + r * ld_in;
  const int64_t lo = m0 * ORIG - W4;  // multiple of 4
  float v[NCH * 4];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int64_t t = lo + 4 * c;
    // a chunk starting inside [0, n) lies inside the row's ld_in (ld_in % 4 == 0)
    float4 q = (t >= 0 && t < n) ? *reinterpret_cast<const float4 *>(x + t) : make_float4(0.f, 0.f, 0.f, 0.f);
    v[4 * c + 0] = q.x;
    v[4 * c + 1] = t + 1 < n ? q.y : 0.f;
    v[4 * c + 2] = t + 2 < n ? q.z : 0.f;
    v[4 * c + 3] = t + 3 < n ? q.w : 0.f;
  }
  float o[NO];
#pragma unroll
  for (int j = 0; j < NW; ++j) {  // phase-major: the TAPS coefficients of phase j serve all G groups
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < TAPS; ++t) acc = fmaf(rk.k[j * TAPS + t], v[g * ORIG + (W4 - W) + t], acc);
      o[g * NW + j] = acc;
    }
  }
  float *__restrict__ y = out + r * ld_out + ob;
  if (ob + NO <= n_out) {
#pragma unroll
    for (int c = 0; c < NO / 4; ++c)
      *reinterpret_cast<float4 *>(y + 4 * c) = make_float4(o[4 * c], o[4 * c + 1], o[4 * c + 2], o[4 * c + 3]);
  } else {
#pragma unroll
    for (int i = 0; i < NO; ++i) {
      if (ob + i < n_out)
        y[i] = o[i];
      else if (ob + i < zc)
        y[i] = 0.f;
    }
  }
}

// Large coefficient tables (nw * taps > FSEM_RS_MAX_COEF: 44.1 kHz, 22.05 kHz, 11.025 kHz ... to
// 16 or 10 kHz).  A workgroup owns the phases [j0, j0 + J) of the polyphase groups [m0, m0 + GM):
// it builds those J coefficient rows in LDS with sinc_coef (the host formula, evaluated in float64
// on the device) and stages the GM groups' input window, then each thread evaluates outputs
// (group, phase) with the same k-ordered fmaf chain as resample_at.  Consecutive threads take
// consecutive phases of one group: coalesced stores of the interleaved output.
constexpr int RS_BIG_K = 8192;  // coefficient floats staged per workgroup
constexpr int RS_BIG_X = 8192;  // input floats staged per workgroup
__global__ void __launch_bounds__(RS_T) resample_sinc_lds(const float *__restrict__ in, int64_t n_in, int64_t ld_in,
                                                         const int32_t *__restrict__ lens, float *__restrict__ out,
                                                         int64_t ld_out, int64_t zc, int64_t r0, int njb, int J,
                                                         int GM, int orig, int nw, int taps, int width) {
  __shared__ float ks[RS_BIG_K];
  __shared__ float xs[RS_BIG_X];
  const int tid = threadIdx.x;
  const int64_t r = r0 + blockIdx.y;
  int64_t n = n_in;
  if (lens) {
    const int64_t v = lens[r];
    n = v < 0 ? 0 : (v > n_in ? n_in : v);
  }
  const int64_t n_out = (n * nw + orig - 1) / orig;
  const int jb = (int)(blockIdx.x % (unsigned)njb);
  const int64_t m0 = (int64_t)(blockIdx.x / (unsigned)njb) * GM;
  const int j0 = jb * J, nj = min(J, nw - j0);
  float *__restrict__ y = out + r * ld_out;
  if (m0 * nw >= n_out) {  // past the row: only the zero tail [n_out, zc)
    for (int i = tid; i < GM * nj; i += RS_T) {
      const int64_t o = (m0 + i / nj) * nw + j0 + i % nj;
      if (o < zc) y[o] = 0.f;
    }
    return;
  }
  for (int i = tid; i < nj * taps; i += RS_T) ks[i] = sinc_coef(j0 + i / taps, i % taps, orig, nw, width);
  const float *__restrict__ x = in + r * ld_in;
  const int64_t base = m0 * orig - width;
  const int nx = (GM - 1) * orig + taps;
  for (int i = tid; i < nx; i += RS_T) {
    const int64_t t = base + i;
    xs[i] = (t >= 0 && t < n) ? x[t] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < GM * nj; i += RS_T) {
    const int g = i / nj, jj = i % nj;
    const int64_t o = (m0 + g) * nw + j0 + jj;
    const float *__restrict__ kj = ks + jj * taps;
    const float *__restrict__ xg = xs + g * orig;
    float acc = 0.f;
    for (int t = 0; t < taps; ++t) acc = fmaf(kj[t], xg[t], acc);
    if (o < n_out)
      y[o] = acc;
    else if (o < zc)
      y[o] = 0.f;
  }
}
static_assert(RS_BIG_TAPS <= RS_BIG_K && RS_BIG_TAPS <= RS_BIG_X, "one phase row and one group window fit");

// One launch over rows [r0, r0 + nrows) (nrows <= kMaxGridY).
static int launch_resample_slice(const float *in, int64_t nrows, int64_t r0, int64_t n_in, int64_t ld_in,
                                 const int32_t *lens, float *out, int64_t ld_out, int64_t zc, const ResampleKernel &rk,
                                 hipStream_t st) {
  const int64_t rows = nrows;
  const int64_t groups = (n_in + rk.orig - 1) / rk.orig + 1;
  if (rk.big) {  // large coefficient tables (e.g. 44.1 kHz): built per workgroup in LDS
    const int J = std::min(rk.nw, std::max(1, RS_BIG_K / rk.taps));
    const int GM = std::max(1, (RS_BIG_X - rk.taps) / rk.orig + 1);
    const int64_t njb = (rk.nw + J - 1) / J, nmb = (groups + GM - 1) / GM;
    if ((double)njb * (double)nmb > 2147483647.0) return FSEM_EINVAL;
    hipLaunchKernelGGL(resample_sinc_lds, dim3((unsigned)(njb * nmb), (unsigned)rows), dim3(RS_T), 0, st, in, n_in,
                       ld_in, lens, out, ld_out, zc, r0, (int)njb, J, GM, rk.orig, rk.nw, rk.taps, rk.width);
    FSEM_CHECK_LAUNCH();
    return FSEM_OK;
  }
  const bool vec = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0) && ld_in % 4 == 0 && ld_out % 4 == 0;
#define FSEM_RS_DIRECT(O, N, T, G)                                                                           \
  if (vec && rk.orig == O && rk.nw == N && rk.taps == T) {                                                   \
    const dim3 grid_d((unsigned)((groups + RS_T * G - 1) / (RS_T * G)), (unsigned)rows);                    \
    hipLaunchKernelGGL((resample_direct_t<O, N, T, G>), grid_d, dim3(RS_T), 0, st, in, n_in, ld_in, lens, out, \
                       ld_out, zc, r0, rk);                                                                      \
    FSEM_CHECK_LAUNCH();                                                                                     \
    return FSEM_OK;                                                                                          \
  }
  FSEM_RS_DIRECT(1, 2, 15, 8)  // 8 -> 16 kHz (PESQ at 8 kHz)
  FSEM_RS_DIRECT(4, 5, 18, 4)  // 8 -> 10 kHz (STOI at 8 kHz)
  FSEM_RS_DIRECT(3, 1, 41, 4)  // 48 -> 16 kHz
#undef FSEM_RS_DIRECT
  const int gt = (RS_XS - rk.taps) / rk.orig + 1;  // groups per workgroup (inputs staged once)
  if (gt < 1 || rk.nw > RS_T * 8) return FSEM_ERATE;
  dim3 grid((unsigned)((groups + gt - 1) / gt), (unsigned)rows);
#define FSEM_RS_CASE(O, N, T)                                                                                \
  if (rk.orig == O && rk.nw == N && rk.taps == T) {                                                          \
    hipLaunchKernelGGL((resample_tiled_t<O, N, T>), grid, dim3(RS_T), 0, st, in, n_in, ld_in, lens, out, ld_out, \
                       zc, gt, r0, rk);                                                                           \
    FSEM_CHECK_LAUNCH();                                                                                      \
    return FSEM_OK;                                                                                           \
  }
  FSEM_RS_CASE(1, 2, 15)   // 8 -> 16 kHz (PESQ at 8 kHz)
  FSEM_RS_CASE(4, 5, 18)   // 8 -> 10 kHz (STOI at 8 kHz)
  FSEM_RS_CASE(3, 1, 41)   // 48 -> 16 kHz
#undef FSEM_RS_CASE
  hipLaunchKernelGGL(resample_tiled, grid, dim3(RS_T), 0, st, in, n_in, ld_in, lens, out, ld_out, zc, gt, r0, rk);
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}

int launch_resample_tiled(const float *in, int64_t rows, int64_t n_in, int64_t ld_in, const int32_t *lens,
                          float *out, int64_t ld_out, int64_t zc, const ResampleKernel &rk, hipStream_t st) {
  if (rows <= 0 || n_in <= 0) return FSEM_OK;
  for (int64_t r0 = 0; r0 < rows; r0 += kMaxGridY) {
    const int rc = launch_resample_slice(in, std::min(rows - r0, kMaxGridY), r0, n_in, ld_in, lens, out, ld_out, zc,
                                         rk, st);
    if (rc != FSEM_OK) return rc;
  }
  return FSEM_OK;
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
  if (!in || !out || rows < 0 || n_in < 0 || ld_in < n_in || n_in > fsem::kMaxLength) return FSEM_EINVAL;
  if (rows == 0 || n_in == 0) return FSEM_OK;
  fsem::ResampleKernel rk;
  int rc = fsem::make_resample_kernel(orig_freq, new_freq, &rk);
  if (rc != FSEM_OK) return rc;
  const int64_t n_out = (rk.nw * n_in + rk.orig - 1) / rk.orig;
  if (ld_out < n_out || n_out > fsem::kMaxLength) return FSEM_EINVAL;
  return fsem::launch_resample_tiled(in, rows, n_in, ld_in, nullptr, out, ld_out, 0, rk, (hipStream_t)stream);
}

extern "C" int fsem_resample_rows_f32(const float *in, int64_t rows, int64_t n_in, int64_t ld_in,
                                      const int32_t *lengths, float *out, int64_t ld_out, int32_t orig_freq,
                                      int32_t new_freq, void *stream) {
  if (!in || !out || !lengths || rows < 0 || n_in < 0 || ld_in < n_in || n_in > fsem::kMaxLength) return FSEM_EINVAL;
  if (orig_freq == new_freq) return FSEM_ERATE;  // nothing to resample: the caller keeps its rows
  if (rows == 0 || n_in == 0) return FSEM_OK;
  fsem::ResampleKernel rk;
  int rc = fsem::make_resample_kernel(orig_freq, new_freq, &rk);
  if (rc != FSEM_OK) return rc;
  const int64_t n_out = (rk.nw * n_in + rk.orig - 1) / rk.orig;
  if (ld_out < n_out || n_out > fsem::kMaxLength) return FSEM_EINVAL;
  return fsem::launch_resample_tiled(in, rows, n_in, ld_in, lengths, out, ld_out, n_out, rk, (hipStream_t)stream);
}
