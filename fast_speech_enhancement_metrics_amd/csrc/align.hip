// Opt-in time alignment of (clean, degraded) 16 kHz pairs before PESQ.
//
// Not part of the reference: its PESQ has no time alignment (fast_se_metrics/PESQ.py:19-22).
// The stages follow ITU-T P.862 section 10 as restated in oracle/align_oracle.py (test
// infrastructure; PARITY UNPINNED against P.862 implementations, none is importable here):
//   1. ta_energy + ta_envelope: 4 ms frame energies (64 samples), an iterated noise threshold
//      (P.862 apply_VAD), log envelope above it;
//   2. ta_crude: the envelope lag (|j| <= M frames) of the largest plain cross-correlation
//      (P.862 crude_align);
//   3. ta_fine_partial + ta_fine_pick: within +-383 samples of the crude delay, the lag of the
//      largest cross-correlation of the signals' first differences, over the whole row;
//   4. ta_shift: the aligned degraded row a[n] = deg[n + D] (0 <= n + D < L_row), else 0.
// Delay D > 0: the degraded row lags the clean one, deg[n] ~ ref[n - D].
//
// Cost is set by stage 3: 767 lags x L multiply-adds per row (about 123 M for 10 s), as
// register-blocked packed FMAs out of LDS (16 consecutive lags per lane sliding over the chunk);
// the other stages are O(L) or O(M * L / 64).
#include "fsem_common.h"

namespace fsem {
namespace align {

constexpr int FRAME = 64;            // envelope frame (4 ms at 16 kHz)
constexpr int VAD_ITERS = 12;
constexpr int FINE = 383;            // fine half-width in samples
constexpr int NLAG = 2 * FINE + 1;   // 767
constexpr int LG = 32;               // lags per lane
constexpr int NGRP = 24;             // lag groups (24 x 32 = 768 slots >= NLAG)
constexpr int NSL = 10;              // sample slices per chunk
constexpr int SL = 512;              // samples per slice
constexpr int CS = NSL * SL;         // samples per chunk (5120)
constexpr int WIN = CS + NGRP * LG;  // degraded window per chunk (5888)
static_assert(NGRP * LG >= NLAG && NGRP * NSL <= 256, "fine-stage thread map");
constexpr int ENV_LDS = 6144;        // envelope frames per signal kept in LDS by ta_crude

__device__ __forceinline__ int64_t row_len(const int32_t *lengths, int64_t b, int64_t L) {
  if (!lengths) return L;
  const int64_t n = lengths[b];
  return n < 0 ? 0 : (n > L ? L : n);
}

// LDS index of the degraded window's element m: a one-float skew every 32 so the 24 lag groups
// of a wave (32 floats apart) read distinct banks.
__device__ __forceinline__ int skew(int m) { return m + (m >> 5); }

// ---------------------------------------------------------------- stage 1: frame energies
// 16 lanes per frame (one float4 each), 4 frames per wave; frames of row s: k < L_row / 64.
__global__ void __launch_bounds__(256) ta_energy(const float *__restrict__ ref, const float *__restrict__ deg,
                                                 int64_t B, int64_t L, int64_t ld,
                                                 const int32_t *__restrict__ lengths, float *__restrict__ E,
                                                 int64_t nfr_cap) {
  const int64_t s = blockIdx.y + (int64_t)blockIdx.z * 65535;  // signal: 0..B-1 ref, B..2B-1 deg
  if (s >= 2 * B) return;
  const int64_t b = s < B ? s : s - B;
  const int64_t nfr = row_len(lengths, b, L) / FRAME;
  const int64_t k = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (k >= nfr_cap) return;
  const int q = threadIdx.x & 15;
  float acc = 0.f;
  if (k < nfr) {
    const float *x = (s < B ? ref : deg) + b * ld + k * FRAME + 4 * q;
    const float4 v = *reinterpret_cast<const float4 *>(x);
    acc = fmaf(v.w, v.w, fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x)));
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
  if (q == 0) E[s * nfr_cap + k] = acc;
}

// ---------------------------------------------------------------- stage 1b: envelopes
// One workgroup per signal: the noise threshold iterated VAD_ITERS times (sums in double, in a
// fixed order), then env = log(E / thr) above it, else 0, in place.
__global__ void __launch_bounds__(256) ta_envelope(int64_t B, int64_t L, const int32_t *__restrict__ lengths,
                                                   float *__restrict__ E, int64_t nfr_cap) {
  __shared__ double red[8];
  const int64_t s = blockIdx.x + (int64_t)blockIdx.y * 65535;
  if (s >= 2 * B) return;
  const int64_t b = s < B ? s : s - B;
  const int64_t nfr = row_len(lengths, b, L) / FRAME;
  float *__restrict__ e = E + s * nfr_cap;
  const int tid = threadIdx.x;
  auto bsum = [&](double v) {
    v = wave_sum_d(v);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
  };
  double t = 0.0;
  for (int64_t k = tid; k < nfr; k += 256) t += e[k];
  double thr = nfr > 0 ? bsum(t) / (double)nfr : 0.0;
  for (int it = 0; it < VAD_ITERS && nfr > 0; ++it) {
    double sm = 0.0, cnt = 0.0;
    for (int64_t k = tid; k < nfr; k += 256)
      if ((double)e[k] <= thr) {
        sm += e[k];
        cnt += 1.0;
      }
    sm = bsum(sm);
    cnt = bsum(cnt);
    if (cnt == 0.0) break;
    const double mu = sm / cnt;
    double sq = 0.0;
    for (int64_t k = tid; k < nfr; k += 256)
      if ((double)e[k] <= thr) sq += ((double)e[k] - mu) * ((double)e[k] - mu);
    sq = bsum(sq);
    thr = 1.001 * (mu + 2.0 * sqrt(sq / cnt));
  }
  __syncthreads();
  for (int64_t k = tid; k < nfr; k += 256) {
    const double v = e[k];
    e[k] = v > thr ? (float)log(v / thr) : 0.f;
  }
}

// ---------------------------------------------------------------- stage 2: crude delay
// One workgroup per row: lag j in [-M, M] per thread (strided), sum over k ascending in float;
// the first maximum (smallest j) above zero, else 0.  Envelopes in LDS when they fit.
__global__ void __launch_bounds__(256) ta_crude(int64_t B, int64_t L, const int32_t *__restrict__ lengths,
                                                const float *__restrict__ E, int64_t nfr_cap, int max_frames,
                                                int *__restrict__ crude) {
  __shared__ float er[ENV_LDS], ed[ENV_LDS];
  __shared__ float bv[256];
  __shared__ int bj[256];
  const int64_t b = blockIdx.x + (int64_t)blockIdx.y * 65535;
  if (b >= B) return;
  const int nfr = (int)(row_len(lengths, b, L) / FRAME);
  const int tid = threadIdx.x;
  const float *gr = E + b * nfr_cap, *gd = E + (B + b) * nfr_cap;
  const bool in_lds = nfr <= ENV_LDS;
  if (in_lds) {
    for (int k = tid; k < nfr; k += 256) {
      er[k] = gr[k];
      ed[k] = gd[k];
    }
  }
  __syncthreads();
  const float *r = in_lds ? er : gr;
  const float *d = in_lds ? ed : gd;
  const int M = nfr < 2 ? 0 : min(max_frames, nfr - 1);
  float best = 0.f;
  int arg = 0;
  for (int j = -M + tid; j <= M; j += 256) {
    const int k0 = j < 0 ? -j : 0, k1 = j < 0 ? nfr : nfr - j;
    float c = 0.f;
    for (int k = k0; k < k1; ++k) c = fmaf(r[k], d[k + j], c);
    if (c > best) {  // j ascending per thread: the first maximum is kept
      best = c;
      arg = j;
    }
  }
  bv[tid] = best;
  bj[tid] = (best > 0.f) ? arg : INT32_MAX;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      const float v2 = bv[tid + off];
      const int j2 = bj[tid + off];
      if (v2 > bv[tid] || (v2 == bv[tid] && j2 < bj[tid])) {
        bv[tid] = v2;
        bj[tid] = j2;
      }
    }
    __syncthreads();
  }
  if (tid == 0) crude[b] = (bj[0] == INT32_MAX) ? 0 : FRAME * bj[0];
}

// ---------------------------------------------------------------- stage 3: fine partials
// Workgroup (row b, chunk c): samples n in [c CS, (c+1) CS).  First differences in LDS:
// wr[n] (n >= 1, n < L_row), wd[m] for m = n + D over the window D in [D0 - FINE, D0 - FINE + 768).
// Thread (slice sl < NSL, group g < NGRP; 240 of the 256 lanes): LG = 32 lags
// D0 - FINE + LG g + i over its SL = 512 samples, the window wd[n + lag0 + i] held in registers
// as even- and odd-aligned pairs, two samples per step.  Partials per lag over the chunk: the
// NSL = 10 slices added in order, to part[b][c][768].
// Static LDS: wr (20 KB) + wd (24 KB) + ps (30 KB) = 74 KB per workgroup -- above the 64 KB
// of earlier CDNA parts; gfx950's 160 KB LDS per CU holds two such workgroups.
constexpr size_t kFineLds = sizeof(float) * (CS + (WIN + WIN / 32 + 64) + NSL * NGRP * LG);
static_assert(kFineLds <= 80 * 1024, "ta_fine_partial: two workgroups per CU in gfx950's 160 KB of LDS");
__global__ void __launch_bounds__(256) ta_fine_partial(const float *__restrict__ ref, const float *__restrict__ deg,
                                                       int64_t B, int64_t L, int64_t ld,
                                                       const int32_t *__restrict__ lengths,
                                                       const int *__restrict__ crude, int nchunk,
                                                       float *__restrict__ part) {
  __shared__ float wr[CS];
  __shared__ float wd[WIN + WIN / 32 + 64];
  __shared__ float ps[NSL][NGRP * LG];
  const int64_t blk = blockIdx.x;
  const int64_t b = blk / nchunk;
  const int c = (int)(blk % nchunk);
  if (b >= B) return;
  const int64_t Lr = row_len(lengths, b, L);
  const int64_t n0 = (int64_t)c * CS;
  const int64_t lag0 = (int64_t)crude[b] - FINE;
  const float *x = ref + b * ld, *y = deg + b * ld;
  const int tid = threadIdx.x;
  auto dif = [Lr](const float *z, int64_t i) {  // first difference, 0 outside [1, L_row)
    return (i >= 1 && i < Lr) ? z[i] - z[i - 1] : 0.f;
  };
  for (int i = tid; i < CS; i += 256) wr[i] = dif(x, n0 + i);
  for (int i = tid; i < WIN + 32; i += 256) wd[skew(i)] = dif(y, n0 + lag0 + i);  // +32: last slides
  __syncthreads();
  const int g = tid % NGRP, sl = tid / NGRP;
  if (sl < NSL) {
    // packed FP32 (v_pk_fma_f32: two lags per instruction).  W[i] = the window element of lag
    // LG g + i at the current sample; E[p] = (W[2p], W[2p+1]) serves the even sample of a
    // double step, O[p] = (W[2p+1], W[2p+2]) the odd one.  A double step retires the logical
    // pair 0 of both and appends the pairs (W[LG], W[LG+1]) / (W[LG+1], W[LG+2]): physical slot
    // (p + k) % (LG/2) holds logical pair p in double step k (unrolled: no moves but the
    // append).  Per double step: LG packed FMAs, two window reads, half a float4 of wr.
    typedef float f2 __attribute__((ext_vector_type(2)));
    constexpr int NP = LG / 2;
    f2 acc[NP], E[NP], O[NP];
    const int base = SL * sl + LG * g;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      acc[p] = (f2){0.f, 0.f};
      const float a = wd[skew(base + 2 * p)], b1 = wd[skew(base + 2 * p + 1)], b2 = wd[skew(base + 2 * p + 2)];
      E[p] = (f2){a, b1};
      O[p] = (f2){b1, b2};
    }
    const float4 *rr4 = reinterpret_cast<const float4 *>(wr + SL * sl);
    for (int n = 0; n < SL; n += LG) {
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int sm = n + 2 * k;
        const float4 xq = rr4[sm >> 2];  // the same float4 for two double steps (CSE)
        const float x0 = (k & 1) ? xq.z : xq.x, x1 = (k & 1) ? xq.w : xq.y;
#pragma unroll
        for (int p = 0; p < NP; ++p) acc[p] = __builtin_elementwise_fma((f2){x0, x0}, E[(p + k) % NP], acc[p]);
#pragma unroll
        for (int p = 0; p < NP; ++p) acc[p] = __builtin_elementwise_fma((f2){x1, x1}, O[(p + k) % NP], acc[p]);
        const float wa = wd[skew(base + sm + LG + 1)], wb = wd[skew(base + sm + LG + 2)];
        E[k] = (f2){O[(NP - 1 + k) % NP].y, wa};
        O[k] = (f2){wa, wb};
      }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      ps[sl][LG * g + 2 * p] = acc[p].x;
      ps[sl][LG * g + 2 * p + 1] = acc[p].y;
    }
  }
  __syncthreads();
  for (int j = tid; j < NGRP * LG; j += 256) {
    float t = ps[0][j];
#pragma unroll
    for (int q = 1; q < NSL; ++q) t += ps[q][j];
    part[(b * nchunk + c) * (NGRP * LG) + j] = t;
  }
}

// ---------------------------------------------------------------- stage 3b: fine delay
// One workgroup per row: per lag the chunk partials added in chunk order (double), the first
// maximum above zero (smallest lag), else the crude delay.
__global__ void __launch_bounds__(256) ta_fine_pick(int64_t B, const int *__restrict__ crude, int nchunk,
                                                    const float *__restrict__ part, int *__restrict__ delay) {
  __shared__ double bv[256];
  __shared__ int bj[256];
  const int64_t b = blockIdx.x + (int64_t)blockIdx.y * 65535;
  if (b >= B) return;
  const int tid = threadIdx.x;
  double best = 0.0;
  int arg = INT32_MAX;
  for (int j = tid; j < NLAG; j += 256) {
    double t = 0.0;
    for (int c = 0; c < nchunk; ++c) t += part[(b * nchunk + c) * (NGRP * LG) + j];
    if (t > best) {
      best = t;
      arg = j;
    }
  }
  bv[tid] = best;
  bj[tid] = arg;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      const double v2 = bv[tid + off];
      const int j2 = bj[tid + off];
      if (v2 > bv[tid] || (v2 == bv[tid] && j2 < bj[tid])) {
        bv[tid] = v2;
        bj[tid] = j2;
      }
    }
    __syncthreads();
  }
  if (tid == 0) delay[b] = (bj[0] == INT32_MAX) ? crude[b] : crude[b] - FINE + bj[0];
}

// ---------------------------------------------------------------- stage 4: shift
// Four outputs per thread (one float4 store; ld_out % 4 == 0), four scalar reads at n + D.
__global__ void __launch_bounds__(256) ta_shift(const float *__restrict__ deg, int64_t B, int64_t L, int64_t ld,
                                                const int32_t *__restrict__ lengths, const int *__restrict__ delay,
                                                float *__restrict__ out, int64_t ld_out) {
  const int64_t b = blockIdx.y + (int64_t)blockIdx.z * 65535;
  if (b >= B) return;
  const int64_t n = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (n >= L) return;
  const int64_t Lr = row_len(lengths, b, L);
  const int64_t D = delay[b];
  const float *y = deg + b * ld;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = n + i + D;
    v[i] = (n + i < Lr && m >= 0 && m < Lr) ? y[m] : 0.f;
  }
  if (n + 4 <= L) {
    *reinterpret_cast<float4 *>(out + b * ld_out + n) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int i = 0; i < 4 && n + i < L; ++i) out[b * ld_out + n + i] = v[i];
  }
}

inline int64_t frames_cap(int64_t L) { return L / FRAME; }
inline int64_t nchunks(int64_t L) { return (L + CS - 1) / CS; }

struct Ws {
  float *E;
  int *crude;
  float *part;
  int *delay;  // internal when the caller passes no delay array
};

inline size_t ws_bytes(int64_t B, int64_t L) {
  const size_t e = align_up((size_t)(2 * B * std::max<int64_t>(frames_cap(L), 1)) * 4, 256);
  const size_t cr = align_up((size_t)B * 4, 256);
  const size_t pt = align_up((size_t)(B * nchunks(L) * NGRP * LG) * 4, 256);
  return e + 2 * cr + pt;
}

inline Ws carve(void *ws, int64_t B, int64_t L) {
  char *p = static_cast<char *>(ws);
  Ws w;
  w.E = reinterpret_cast<float *>(p);
  p += align_up((size_t)(2 * B * std::max<int64_t>(frames_cap(L), 1)) * 4, 256);
  w.crude = reinterpret_cast<int *>(p);
  p += align_up((size_t)B * 4, 256);
  w.delay = reinterpret_cast<int *>(p);
  p += align_up((size_t)B * 4, 256);
  w.part = reinterpret_cast<float *>(p);
  return w;
}

}  // namespace align
}  // namespace fsem

using namespace fsem;

extern "C" size_t fsem_time_align_workspace_bytes(int64_t batch, int64_t length) {
  if (batch <= 0 || length <= 0) return 0;
  return align::ws_bytes(batch, length);
}

extern "C" int fsem_time_align_f32(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld,
                                   const int32_t *lengths, int32_t max_delay, int32_t *delay, float *deg_aligned,
                                   int64_t ld_out, void *ws, size_t ws_bytes, void *stream) {
  if (!ref || !deg || batch <= 0 || length <= 0 || ld < length || length > kMaxLength || max_delay < 0 ||
      (deg_aligned && (ld_out < length || ld_out % 4 != 0)) || (!delay && !deg_aligned) || (ld % 4) != 0)
    return FSEM_EINVAL;
  const int64_t nch = align::nchunks(length);
  if (batch * nch > INT32_MAX) return FSEM_EINVAL;
  if (!ws || ws_bytes < align::ws_bytes(batch, length)) return FSEM_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  align::Ws w = align::carve(ws, batch, length);
  int *dl = delay ? delay : w.delay;
  const int64_t nfr_cap = std::max<int64_t>(align::frames_cap(length), 1);
  const int64_t sig = 2 * batch;
  // 64-bit: max_delay may be INT32_MAX (alignment.py clamps to it), where the 32-bit sum would wrap
  const int max_frames =
      (int)std::min<int64_t>(((int64_t)max_delay + align::FRAME - 1) / align::FRAME, (int64_t)INT32_MAX);
  auto yz = [](int64_t n) { return dim3(1, (unsigned)std::min<int64_t>(n, 65535), (unsigned)((n + 65534) / 65535)); };
  {
    dim3 grid = yz(sig);
    grid.x = (unsigned)((nfr_cap + 15) / 16);
    align::ta_energy<<<grid, 256, 0, st>>>(ref, deg, batch, length, ld, lengths, w.E, nfr_cap);
    FSEM_CHECK_LAUNCH();
  }
  auto xy = [](int64_t n) { return dim3((unsigned)std::min<int64_t>(n, 65535), (unsigned)((n + 65534) / 65535)); };
  align::ta_envelope<<<xy(sig), 256, 0, st>>>(batch, length, lengths, w.E, nfr_cap);
  FSEM_CHECK_LAUNCH();
  align::ta_crude<<<xy(batch), 256, 0, st>>>(batch, length, lengths, w.E, nfr_cap, max_frames, w.crude);
  FSEM_CHECK_LAUNCH();
  align::ta_fine_partial<<<(unsigned)(batch * nch), 256, 0, st>>>(ref, deg, batch, length, ld, lengths, w.crude,
                                                                  (int)nch, w.part);
  FSEM_CHECK_LAUNCH();
  align::ta_fine_pick<<<xy(batch), 256, 0, st>>>(batch, w.crude, (int)nch, w.part, dl);
  FSEM_CHECK_LAUNCH();
  if (deg_aligned) {
    dim3 grid = yz(batch);
    grid.x = (unsigned)((length + 1023) / 1024);
    align::ta_shift<<<grid, 256, 0, st>>>(deg, batch, length, ld, lengths, dl, deg_aligned, ld_out);
    FSEM_CHECK_LAUNCH();
  }
  return FSEM_OK;
}
