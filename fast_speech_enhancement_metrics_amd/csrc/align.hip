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
// Utterance mode (fsem_time_align_utt_f32, P.862 sections 10.3-10.5 as restated in the oracle):
//   5. ta_utterances (a wave per row): the reference's utterances (speech runs >= 16 ms joined across gaps < 200 ms, at
//      least 200 ms long, at most 16), the regions they own (boundaries in the gaps' middles) and
//      the regions' 5120-sample pieces;
//   6. ta_crude_utt: each utterance's envelope lag over its search window (+-300 ms around it),
//      within +-75 frames of the row's crude lag;
//   7. ta_fine_partial (utterance pieces): the first-difference correlation per piece around the
//      utterance's crude delay;
//   8. ta_pick_utt: each region's fine delay, or two delays when splitting it at a piece boundary
//      raises the summed correlation peak by 20 % and the halves' delays differ by >= 16 samples;
//      ta_segments: the row's segments (equal neighbours merged) and its longest segment's delay;
//   9. ta_shift_seg: a[n] = deg[n + D_k] in segment k.
//
// P.862 mode (fsem_time_align_p862_f32, oracle/align_oracle.py steps 10-12; P.862 sections
// 10.5-10.6 restated on stage 7's 320 ms pieces): stages 5-7 as the utterance mode, then
//  10. ta_piece_peaks (a wave per piece): the piece's correlation peak and its lag;
//  11-12. ta_pick_p862 (workgroup per utterance): the pieces from 5 % of the utterance's largest
//      peak vote for their lags with weight peak^0.125 (P.862's histogram), the triangle-smoothed
//      histogram's first maximum is a range's delay and its share of the votes its confidence; a
//      range splits at the piece boundary whose two halves (two or more votes each, delays >= 1 ms
//      apart) are both more confident than the whole, the most confident pair first, and each
//      half once more (P.862 utterance_split, two levels: up to 4 segments per utterance);
//      ta_segments_p862: the row's segments as in stage 8, at most MAXSEG.
// Cost was set by stage 3: 767 lags x L multiply-adds per row (about 123 M for 10 s) as
// register-blocked packed FMAs out of LDS (ta_fine_partial); ta_fine_fft computes the same
// partials by fast correlation (per 1280-sample block, 2048-point transforms: ~12x less work).
// The other stages are O(L) or O(M * L / 64).
#include "fsem_common.h"
#include "fsem_fft.h"

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
// utterance mode (oracle/align_oracle.py steps 5-9; P.862 constant names)
constexpr int MINSPEECH = 4;         // frames: shorter speech runs are discarded (MINSPEECHLGTH)
constexpr int JOIN = 50;             // frames: shorter gaps join two speech runs (JOINSPEECHLGTH)
constexpr int MINUTT = 50;           // frames: shorter joined runs are not utterances
constexpr int SEARCHBUF = 75;        // frames: crude search window margin and lag range
constexpr int MAXU = 16;             // utterances per row
constexpr int MAXSEG = 2 * MAXU;     // segments per row (include/fsem.h FSEM_ALIGN_MAX_SEGMENTS)
constexpr int SPLIT_MIN = 16;        // samples: least delay difference of a split
constexpr double SPLIT_GAIN = 1.2;   // least gain of the summed correlation peaks of a split

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
  const int M = nfr < 2 ? 0 : min(max_frames, nfr - 1);
  float best = 0.f;
  int arg = 0;
  for (int j = -M + tid; j <= M; j += 256) {
    const int k0 = j < 0 ? -j : 0, k1 = j < 0 ? nfr : nfr - j;
    float c = 0.f;
    // two loops, not one over a selected pointer (flat loads), unrolled by 8: eight loads in
    // flight per wait, the chain of fmaf in the same order (as ta_crude_utt)
    if (in_lds) {
#pragma unroll 8
      for (int k = k0; k < k1; ++k) c = fmaf(er[k], ed[k + j], c);
    } else {
#pragma unroll 8
      for (int k = k0; k < k1; ++k) c = fmaf(gr[k], gd[k + j], c);
    }
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
// Utterance mode (utt != nullptr): slot c of row b is piece i of utterance u (pieces of u are
// slots [cs[u], cs[u+1])): samples [reg[u] + i CS, min(reg[u] + (i+1) CS, reg[u+1])) at lags
// around that utterance's crude delay (ucrude[u]).
// Bad-interval realignment (desc != nullptr): slot c < ndesc[b] of row b is desc[b][c] = {first
// sample, end sample, centre lag, interval}.
struct UttTables {
  const int *nutt;    // [B]
  const int *reg;     // [B][MAXU + 1] region starts (samples)
  const int *cs;      // [B][MAXU + 1] first piece slot per utterance
  const int *ucrude;  // [B][MAXU] crude delay (samples)
  const int4 *desc = nullptr;
  const int *ndesc = nullptr;  // [B]
};
// Workgroup blk's slot: row b, slot c, samples [n0, hi) correlated at lags lag0 + j (j < 768).
struct SlotRange {
  bool valid;
  int64_t b, Lr, n0, hi, lag0;
  int c;
};
__device__ __forceinline__ SlotRange slot_range(int64_t blk, int64_t B, int64_t L, const int32_t *lengths,
                                                const int *crude, int nchunk, const UttTables &ut) {
  SlotRange r;
  // slot descriptors (few active slots per row): rows fastest, so the active workgroups spread
  // over the XCDs instead of landing on the few that row-major slot ids map to
  r.b = ut.desc ? blk % B : blk / nchunk;
  r.c = (int)(ut.desc ? blk / B : blk % nchunk);
  r.valid = r.b < B;
  if (!r.valid) return r;
  r.Lr = row_len(lengths, r.b, L);
  r.n0 = (int64_t)r.c * CS;
  r.hi = r.n0 + CS;
  r.lag0 = crude ? (int64_t)crude[r.b] - FINE : 0;  // crude: NULL with slot descriptors
  if (ut.nutt) {
    const int U = ut.nutt[r.b];
    const int *cs = ut.cs + r.b * (MAXU + 1);
    if (r.c >= cs[U]) {  // past the row's pieces (uniform)
      r.valid = false;
      return r;
    }
    int u = 0;
    while (u + 1 < U && cs[u + 1] <= r.c) ++u;
    const int *reg = ut.reg + r.b * (MAXU + 1);
    r.n0 = (int64_t)reg[u] + (int64_t)(r.c - cs[u]) * CS;
    r.hi = std::min<int64_t>(r.n0 + CS, reg[u + 1]);
    r.lag0 = (int64_t)ut.ucrude[r.b * MAXU + u] - FINE;
  } else if (ut.desc) {
    if (r.c >= ut.ndesc[r.b]) {  // past the row's pieces (uniform)
      r.valid = false;
      return r;
    }
    const int4 d = ut.desc[r.b * nchunk + r.c];
    r.n0 = d.x;
    r.hi = d.y;
    r.lag0 = (int64_t)d.z - FINE;
  }
  return r;
}

__global__ void __launch_bounds__(256) ta_fine_partial(const float *__restrict__ ref, const float *__restrict__ deg,
                                                       int64_t B, int64_t L, int64_t ld,
                                                       const int32_t *__restrict__ lengths,
                                                       const int *__restrict__ crude, int nchunk,
                                                       float *__restrict__ part, UttTables ut) {
  __shared__ float wr[CS];
  __shared__ float wd[WIN + WIN / 32 + 64];
  __shared__ float ps[NSL][NGRP * LG];
  const SlotRange sr = slot_range(blockIdx.x, B, L, lengths, crude, nchunk, ut);
  if (!sr.valid) return;  // uniform
  const int64_t b = sr.b, Lr = sr.Lr, n0 = sr.n0, hi = sr.hi, lag0 = sr.lag0;
  const int c = sr.c;
  const float *x = ref + b * ld, *y = deg + b * ld;
  const int tid = threadIdx.x;
  auto dif = [Lr](const float *z, int64_t i) {  // first difference, 0 outside [1, L_row)
    return (i >= 1 && i < Lr) ? z[i] - z[i - 1] : 0.f;
  };
  for (int i = tid; i < CS; i += 256) wr[i] = (n0 + i < hi) ? dif(x, n0 + i) : 0.f;
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

// ---------------------------------------------------------------- stage 3, FFT form
// The same partials as ta_fine_partial by fast correlation (FSEM_FINE_FFT): wave q of the
// workgroup takes the slot's block q, x[i] = wr[n0 + 1280 q + i] (i < 1280 and below the slot's
// end, else 0) and y[i] = wd[n0 + 1280 q + lag0 + i] (i < 2048); its c_q[j] = sum_i x[i] y[i + j]
// (j < 768) is their circular correlation of length 2048 (no wrap: 1280 + 767 < 2048):
//   Z = FFT(x + i y) -- four 512-point transforms of the samples 4n + r (fft512_wave_x2) and a
//   radix-4 step -- then with A = Z[k] + conj Z[-k], B = Z[k] - conj Z[-k]:
//   X = A / 2, Y = B / 2i, and c = Re IFFT(conj(X) Y) = Re FFT(X conj(Y)) / 2048 with
//   X conj(Y) = i A conj(B) / 4 (one more four-transform FFT, after a transposition through the
//   wave's LDS area).  The four blocks' c_q are added in block order.  The values differ from the
//   direct sums by float32 rounding (both forms: ~1e-7 .. 1e-6 of |x| |y|); the work per slot is
//   ~12x smaller.
constexpr int FB = 1280;  // samples of x per block (wave)
constexpr int FN = 2048;  // transform length
static_assert(4 * FB == CS && FB + NGRP * LG - 1 <= FN, "four blocks per slot; no wrap");

__device__ __forceinline__ cf w2048(int t) {  // exp(-2 pi i t / 2048), 0 <= t < 2048
  // W_512^(t >> 2) from the 512-point table times W_2048^(t & 3)
  const float fr[4] = {1.0f, 0.9999953f, 0.99998116f, 0.9999576f};
  const float fi[4] = {-0.0f, -0.0030679568f, -0.0061358847f, -0.009203754f};
  const int f = t & 3;
  return cmul(cf{kTwRe[t >> 2], kTwIm[t >> 2]}, cf{fr[f], fi[f]});
}

__global__ void __launch_bounds__(256) ta_fine_fft(const float *__restrict__ ref, const float *__restrict__ deg,
                                                   int64_t B, int64_t L, int64_t ld,
                                                   const int32_t *__restrict__ lengths,
                                                   const int *__restrict__ crude, int nchunk,
                                                   float *__restrict__ part, UttTables ut) {
  __shared__ __attribute__((aligned(16))) float2 fbuf[4][FN];  // per wave: exchange + transposition
  const SlotRange sr = slot_range(blockIdx.x, B, L, lengths, crude, nchunk, ut);
  if (!sr.valid) return;  // uniform
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float2 *buf = fbuf[wave];
  const float *xr = ref + sr.b * ld, *yd = deg + sr.b * ld;
  const int64_t Lr = sr.Lr;
  const int64_t xb = sr.n0 + (int64_t)FB * wave;  // block start (x)
  const int64_t yb = xb + sr.lag0;                // window start (y)
  const int64_t xend = std::min<int64_t>(sr.hi, xb + FB);
  float cq[12];  // c_q at lags lane + 64 m
  if (xend > xb) {  // uniform
    cf tw1[8], tw2[8];
    fft512_twiddles(lane, tw1, tw2);
    // subsequence r's element n = lane + 64 s is z[4 n + r] = z[4 lane + 256 s + r]
    cf g[4][8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int i0 = 4 * lane + 256 * s;
      float xv[5], yv[5];  // samples i0 - 1 .. i0 + 3 of the block and the window
#pragma unroll
      for (int e = 0; e < 5; ++e) {
        const int64_t tx = xb + i0 - 1 + e, ty = yb + i0 - 1 + e;
        xv[e] = (tx >= 0 && tx < Lr) ? xr[tx] : 0.f;
        yv[e] = (ty >= 0 && ty < Lr) ? yd[ty] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t tx = xb + i0 + r, ty = yb + i0 + r;
        // first differences, 0 outside [1, L_row) (ta_fine_partial's dif), x also past the slot
        const float dx = (i0 + r < FB && tx < xend && tx >= 1 && tx < Lr) ? xv[r + 1] - xv[r] : 0.f;
        const float dy = (ty >= 1 && ty < Lr) ? yv[r + 1] - yv[r] : 0.f;
        g[r][s] = {dx, dy};
      }
    }
    cf t4[3][8];  // radix-4 twiddles W_2048^(r k0), k0 = lane + 64 j
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 1; r < 4; ++r) t4[r - 1][j] = w2048((r * (lane + 64 * j)) & (FN - 1));
    fft512_wave_x2(g[0], g[1], buf, lane, tw1, tw2);
    fft512_wave_x2(g[2], g[3], buf, lane, tw1, tw2);
    cf Z[32];  // Z[lane + 64 m]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const cf a0 = g[0][j], a1 = cmul(g[1][j], t4[0][j]), a2 = cmul(g[2][j], t4[1][j]),
               a3 = cmul(g[3][j], t4[2][j]);
      const cf s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = mul_mi(csub(a1, a3));
      Z[j] = cadd(s02, s13);
      Z[j + 8] = cadd(d02, d13);
      Z[j + 16] = csub(s02, s13);
      Z[j + 24] = csub(d02, d13);
    }
    // Q = i A conj(B): conj Z[-k] from lane 64 - lane, register 31 - m (lane 0: (32 - m) mod 32)
    const int plane = (64 - lane) & 63;
    cf Q[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) {
      float mr = __shfl(Z[31 - m].r, plane, 64);
      float mi = __shfl(Z[31 - m].i, plane, 64);
      if (lane == 0) {
        mr = Z[(32 - m) & 31].r;
        mi = Z[(32 - m) & 31].i;
      }
      const cf A = {Z[m].r + mr, Z[m].i - mi}, Bv = {Z[m].r - mr, Z[m].i + mi};
      const cf P = {fmaf(A.r, Bv.r, A.i * Bv.i), fmaf(A.i, Bv.r, -(A.r * Bv.i))};  // A conj(B)
      Q[m] = {-P.i, P.r};
    }
#pragma unroll
    for (int m = 0; m < 32; ++m) buf[lane + 64 * m] = make_float2(Q[m].r, Q[m].i);
    wave_lds_fence();
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float4 *q4 = reinterpret_cast<const float4 *>(buf + 4 * lane + 256 * s);
      const float4 u = q4[0], v = q4[1];
      g[0][s] = {u.x, u.y};
      g[1][s] = {u.z, u.w};
      g[2][s] = {v.x, v.y};
      g[3][s] = {v.z, v.w};
    }
    fft512_wave_x2(g[0], g[1], buf, lane, tw1, tw2);
    fft512_wave_x2(g[2], g[3], buf, lane, tw1, tw2);
    constexpr float kScale = 1.f / (4.f * FN);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const cf a0 = g[0][j], a1 = cmul(g[1][j], t4[0][j]), a2 = cmul(g[2][j], t4[1][j]),
               a3 = cmul(g[3][j], t4[2][j]);
      cq[j] = ((a0.r + a2.r) + (a1.r + a3.r)) * kScale;  // k0
      if (j < 4) cq[8 + j] = ((a0.r - a2.r) + (a1.i - a3.i)) * kScale;  // k0 + 512: Re(d02 - i d13)
    }
  } else {
#pragma unroll
    for (int m = 0; m < 12; ++m) cq[m] = 0.f;
  }
  wave_lds_fence();  // the last transform's reads of buf are done
  float *cb = reinterpret_cast<float *>(buf);
#pragma unroll
  for (int m = 0; m < 12; ++m) cb[lane + 64 * m] = cq[m];
  __syncthreads();
  const float *c0 = reinterpret_cast<const float *>(fbuf[0]), *c1 = reinterpret_cast<const float *>(fbuf[1]),
              *c2 = reinterpret_cast<const float *>(fbuf[2]), *c3 = reinterpret_cast<const float *>(fbuf[3]);
  for (int j = tid; j < NGRP * LG; j += 256)
    part[(sr.b * nchunk + sr.c) * (NGRP * LG) + j] = ((c0[j] + c1[j]) + c2[j]) + c3[j];
}

// the fine stage's partials of every slot: the FFT form (default), or the direct one
// (FSEM_FINE_FFT=0, kept for A/B): 4096 x 10 s PESQ with row / utterance / P.862-mode alignment
// 19.3 / 26.6 / 45.7 ms direct, 11.2 / 13.8 / 28.8 ms FFT, every synthetic delay recovered by both
// (profiles/r6_g/ab_fine_fft.txt)
#ifndef FSEM_FINE_FFT
#define FSEM_FINE_FFT 1
#endif
inline void launch_fine(unsigned grid, hipStream_t st, const float *ref, const float *deg, int64_t B, int64_t L,
                        int64_t ld, const int32_t *lengths, const int *crude, int nchunk, float *part,
                        const UttTables &ut) {
  if (FSEM_FINE_FFT)
    ta_fine_fft<<<grid, 256, 0, st>>>(ref, deg, B, L, ld, lengths, crude, nchunk, part, ut);
  else
    ta_fine_partial<<<grid, 256, 0, st>>>(ref, deg, B, L, ld, lengths, crude, nchunk, part, ut);
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

// ---------------------------------------------------------------- stage 5: utterances
// One wave per row: the reference envelope 64 frames at a time (one coalesced load, a ballot of
// the speech frames), the runs of each block walked with bit scans in wave-uniform (scalar)
// code -- speech runs of MINSPEECH frames or more, joined across gaps < JOIN frames, kept from
// MINUTT frames, at most MAXU (later ones join the last); then the regions (boundary: the
// middle of the gap, in whole frames) and their pieces.  No utterance: one covering the row
// (its crude window: every frame).
__global__ void __launch_bounds__(64) ta_utterances(int64_t B, int64_t L, const int32_t *__restrict__ lengths,
                                                    const float *__restrict__ E, int64_t nfr_cap,
                                                    int *__restrict__ nutt, int *__restrict__ utt,
                                                    int *__restrict__ reg, int *__restrict__ cs) {
  __shared__ int us[2 * MAXU];
  const int64_t b = blockIdx.x + (int64_t)blockIdx.y * 65535;
  if (b >= B) return;
  const int lane = threadIdx.x;
  const int64_t Lr = row_len(lengths, b, L);
  const int nfr = (int)(Lr / FRAME);
  const float *env = E + b * nfr_cap;
  int n = 0, s0 = -1, e0 = -1, rs = -1;  // utterances, joined run [s0, e0), open raw run from rs
  auto flush = [&]() {
    if (s0 >= 0 && e0 - s0 >= MINUTT) {
      if (n < MAXU) {
        if (lane == 0) {
          us[2 * n] = s0;
          us[2 * n + 1] = e0;
        }
        ++n;
      } else if (lane == 0) {
        us[2 * (MAXU - 1) + 1] = e0;
      }
    }
  };
  auto close_run = [&](int k) {  // the raw run [rs, k) ends
    if (k - rs >= MINSPEECH) {
      if (s0 >= 0 && rs - e0 < JOIN) {
        e0 = k;
      } else {
        flush();
        s0 = rs;
        e0 = k;
      }
    }
    rs = -1;
  };
  for (int k0 = 0; k0 < nfr; k0 += 64) {
    const int k = k0 + lane;
    const uint64_t m = __ballot(k < nfr && env[k] > 0.f);
    int pos = 0;
    while (pos < 64) {
      if (rs >= 0) {
        const uint64_t z = ~m >> pos;  // the open run ends at the next inactive frame
        if (z == 0) break;             // ... in a later block
        pos += __builtin_ctzll(z);
        close_run(k0 + pos);
      } else {
        const uint64_t o = m >> pos;
        if (o == 0) break;
        pos += __builtin_ctzll(o);
        rs = k0 + pos;
      }
    }
  }
  if (rs >= 0) close_run(nfr);
  flush();
  if (n == 0) {
    if (lane == 0) {
      us[0] = 0;
      us[1] = nfr;
    }
    n = 1;
  }
  __syncthreads();
  if (lane == 0) {
    int *uo = utt + b * (2 * MAXU);
    for (int i = 0; i < 2 * n; ++i) uo[i] = us[i];
    nutt[b] = n;
    int *rg = reg + b * (MAXU + 1);
    int *c = cs + b * (MAXU + 1);
    rg[0] = 0;
    for (int u = 1; u < n; ++u) rg[u] = FRAME * ((us[2 * u - 1] + us[2 * u]) / 2);
    rg[n] = (int)Lr;
    c[0] = 0;
    for (int u = 0; u < n; ++u) c[u + 1] = c[u] + std::max(1, (rg[u + 1] - rg[u] + CS - 1) / CS);
  }
}

// First-maximum argmax over a 256-thread workgroup: (v, j) with v > 0, or (0, INT32_MAX).
__device__ __forceinline__ void block_argmax(double &v, int &j, double *sv, int *sj) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double v2 = __shfl_xor(v, off, 64);
    const int j2 = __shfl_xor(j, off, 64);
    if (v2 > v || (v2 == v && j2 < j)) {
      v = v2;
      j = j2;
    }
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();  // the previous call's readers are done
  if ((threadIdx.x & 63) == 0) {
    sv[w] = v;
    sj[w] = j;
  }
  __syncthreads();
  v = sv[0];
  j = sj[0];
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if (sv[q] > v || (sv[q] == v && sj[q] < j)) {
      v = sv[q];
      j = sj[q];
    }
}

// ---------------------------------------------------------------- stage 6: per-utterance crude
// Workgroup (utterance u, row b): lag j = jrow - SEARCHBUF + tid (within |j| <= M), the envelope
// correlation over reference frames [start - SEARCHBUF, end + SEARCHBUF), k ascending in float.
// The window's frames of both envelopes are staged in LDS when they fit (UTT_LDS each; longer
// utterances read global memory): each lane's chain of fmaf then waits on LDS, not on HBM.
constexpr int UTT_LDS = 4096;
__global__ void __launch_bounds__(256) ta_crude_utt(int64_t B, int64_t L, const int32_t *__restrict__ lengths,
                                                    const float *__restrict__ E, int64_t nfr_cap, int max_frames,
                                                    const int *__restrict__ crude, const int *__restrict__ nutt,
                                                    const int *__restrict__ utt, int *__restrict__ ucrude) {
  __shared__ double sv[4];
  __shared__ int sj[4];
  __shared__ float sr[UTT_LDS], sd[UTT_LDS + 2 * SEARCHBUF + 1];
  const int u = blockIdx.y;  // rows fastest in the dispatch order: a row's active workgroups spread over the XCDs
  const int64_t b = blockIdx.x + (int64_t)blockIdx.z * 65535;
  if (b >= B || u >= nutt[b]) return;
  const int nfr = (int)(row_len(lengths, b, L) / FRAME);
  const int M = nfr < 2 ? 0 : min(max_frames, nfr - 1);
  const int jrow = crude[b] / FRAME;
  const int jlo = max(-M, jrow - SEARCHBUF), jhi = min(M, jrow + SEARCHBUF);
  const int k0 = max(0, utt[b * 2 * MAXU + 2 * u] - SEARCHBUF);
  const int k1 = min(nfr, utt[b * 2 * MAXU + 2 * u + 1] + SEARCHBUF);
  const float *gr = E + b * nfr_cap, *gd = E + (B + b) * nfr_cap;
  // LDS: sr[k - k0] = r[k] for k in [k0, k1); sd[m - k0 - jlo] = d[m] for m in [k0 + jlo, k1 + jhi)
  // (frames outside [0, nfr) are never read: ks / ke clip every lag's range)
  const bool in_lds = k1 - k0 <= UTT_LDS && jhi - jlo <= 2 * SEARCHBUF;
  if (in_lds) {
    for (int k = (int)threadIdx.x; k < k1 - k0; k += 256) sr[k] = gr[k0 + k];
    for (int k = (int)threadIdx.x; k < k1 - k0 + jhi - jlo; k += 256) {
      const int m = k0 + jlo + k;
      sd[k] = (m >= 0 && m < nfr) ? gd[m] : 0.f;
    }
  }
  __syncthreads();
  const int j = jlo + (int)threadIdx.x;
  double best = 0.0;
  int arg = INT32_MAX;
  if (j <= jhi) {
    const int ks = max(k0, -j), ke = min(k1, nfr - j);
    float c = 0.f;
    // two loops, not one over a selected pointer: a generic pointer turns the LDS reads into flat
    // loads (and one offset below the LDS aperture faults); index offsets, k ascending either way
    // (unrolled by 8: eight loads in flight per wait, the chain of fmaf in the same order)
    if (in_lds) {
#pragma unroll 8
      for (int k = ks; k < ke; ++k) c = fmaf(sr[k - k0], sd[k + j - k0 - jlo], c);
    } else {
#pragma unroll 8
      for (int k = ks; k < ke; ++k) c = fmaf(gr[k], gd[k + j], c);
    }
    if (c > 0.f) {
      best = c;
      arg = j;
    }
  }
  block_argmax(best, arg, sv, sj);
  if (threadIdx.x == 0) ucrude[b * MAXU + u] = FRAME * (arg == INT32_MAX ? jrow : arg);
}

// ---------------------------------------------------------------- stage 8: per-utterance pick
// Workgroup (utterance u, row b): lags l = tid + 256 q (q < 3, l < NLAG), the region's pieces
// added in piece order (double); the whole region's first peak, then every split s in
// [2, m - 2] (left = pieces < s, right = total - left) with two argmax reductions.
// useg[b][u] = {segments (1 or 2), split offset (samples), delay 1, delay 2}.
__global__ void __launch_bounds__(256) ta_pick_utt(int64_t B, const int *__restrict__ nutt, const int *__restrict__ cs,
                                                   const int *__restrict__ ucrude, int nslot,
                                                   const float *__restrict__ part, int *__restrict__ useg) {
  __shared__ double sv[4];
  __shared__ int sj[4];
  const int u = blockIdx.y;  // rows fastest in the dispatch order: a row's active workgroups spread over the XCDs
  const int64_t b = blockIdx.x + (int64_t)blockIdx.z * 65535;
  if (b >= B || u >= nutt[b]) return;
  const int tid = threadIdx.x;
  const int c0 = cs[b * (MAXU + 1) + u], m = cs[b * (MAXU + 1) + u + 1] - c0;
  const float *P = part + (b * nslot + c0) * (int64_t)(NGRP * LG);
  const int d0 = ucrude[b * MAXU + u];
  double tot[3], left[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < 3; ++q) tot[q] = 0.0;
  for (int i = 0; i < m; ++i)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int l = tid + 256 * q;
      if (l < NLAG) tot[q] += P[i * (NGRP * LG) + l];
    }
  // the thread's first peak (lags ascending) of an array given per q
  auto local_peak = [&](const double *a, double &v, int &j) {
    v = 0.0;
    j = INT32_MAX;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int l = tid + 256 * q;
      if (l < NLAG && a[q] > v) {
        v = a[q];
        j = l;
      }
    }
  };
  double vW;
  int iW;
  local_peak(tot, vW, iW);
  block_argmax(vW, iW, sv, sj);
  double bestT = -1.0, bvL = 0.0, bvR = 0.0;
  int bs = -1, biL = INT32_MAX, biR = INT32_MAX;
  for (int s = 1; s + 1 < m && m >= 4; ++s) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int l = tid + 256 * q;
      if (l < NLAG) left[q] += P[(s - 1) * (NGRP * LG) + l];
    }
    if (s < 2) continue;
    double right[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) right[q] = tot[q] - left[q];
    double vL, vR;
    int iL, iR;
    local_peak(left, vL, iL);
    local_peak(right, vR, iR);
    block_argmax(vL, iL, sv, sj);
    block_argmax(vR, iR, sv, sj);
    if (vL + vR > bestT) {  // uniform: every thread holds the reduced values
      bestT = vL + vR;
      bs = s;
      bvL = vL;
      bvR = vR;
      biL = iL;
      biR = iR;
    }
  }
  if (tid == 0) {
    int *o = useg + (b * MAXU + u) * 4;
    const bool split = bs > 0 && bvL > 0.0 && bvR > 0.0 && bestT > SPLIT_GAIN * vW &&
                       abs(biL - biR) >= SPLIT_MIN;
    o[0] = split ? 2 : 1;
    o[1] = split ? bs * CS : 0;
    o[2] = split ? d0 - FINE + biL : (iW == INT32_MAX ? d0 : d0 - FINE + iW);
    o[3] = split ? d0 - FINE + biR : o[2];
  }
}

// One thread per row: the segments in order (equal neighbours merged), the row's delay (its
// longest segment's, the first of equals).
__global__ void __launch_bounds__(64) ta_segments(int64_t B, int64_t L, const int32_t *__restrict__ lengths,
                                                  const int *__restrict__ nutt, const int *__restrict__ reg,
                                                  const int *__restrict__ useg, int *__restrict__ nseg,
                                                  int *__restrict__ seg_start, int *__restrict__ seg_delay,
                                                  int *__restrict__ delay) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  const int U = nutt[b];
  const int *rg = reg + b * (MAXU + 1);
  int *st = seg_start + b * (MAXSEG + 1), *dl = seg_delay + b * MAXSEG;
  int n = 0;
  auto add = [&](int start, int d) {
    if (n > 0 && dl[n - 1] == d) return;
    st[n] = start;
    dl[n] = d;
    ++n;
  };
  for (int u = 0; u < U; ++u) {
    const int *o = useg + (b * MAXU + u) * 4;
    add(rg[u], o[2]);
    if (o[0] == 2) add(rg[u] + o[1], o[3]);
  }
  st[n] = (int)row_len(lengths, b, L);
  int best = -1, d = 0;
  for (int k = 0; k < n; ++k)
    if (st[k + 1] - st[k] > best) {
      best = st[k + 1] - st[k];
      d = dl[k];
    }
  if (nseg) nseg[b] = n;
  if (delay) delay[b] = d;
}

// ---------------------------------------------------------------- stage 9: segment shift
__global__ void __launch_bounds__(256) ta_shift_seg(const float *__restrict__ deg, int64_t B, int64_t L, int64_t ld,
                                                    const int32_t *__restrict__ lengths, const int *__restrict__ nseg,
                                                    const int *__restrict__ seg_start,
                                                    const int *__restrict__ seg_delay, float *__restrict__ out,
                                                    int64_t ld_out) {
  __shared__ int st[MAXSEG + 1], dl[MAXSEG];
  const int64_t b = blockIdx.y + (int64_t)blockIdx.z * 65535;
  if (b >= B) return;
  const int n_s = nseg[b];
  if (threadIdx.x <= n_s) st[threadIdx.x] = seg_start[b * (MAXSEG + 1) + threadIdx.x];
  if (threadIdx.x < n_s) dl[threadIdx.x] = seg_delay[b * MAXSEG + threadIdx.x];
  __syncthreads();
  const int64_t n = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (n >= L) return;
  const int64_t Lr = row_len(lengths, b, L);
  const float *y = deg + b * ld;
  int k = 0;
  while (k + 1 < n_s && st[k + 1] <= n) ++k;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    while (k + 1 < n_s && st[k + 1] <= n + i) ++k;
    const int64_t m = n + i + dl[k];
    v[i] = (n + i < Lr && m >= 0 && m < Lr) ? y[m] : 0.f;
  }
  if (n + 4 <= L) {
    *reinterpret_cast<float4 *>(out + b * ld_out + n) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int i = 0; i < 4 && n + i < L; ++i) out[b * ld_out + n + i] = v[i];
  }
}

// ---------------------------------------------------------------- P.862 mode stages 10-12
constexpr int HIST_T = 8;            // lags: half-width of the histogram's triangle
constexpr double HIST_POW = 0.125;   // a piece's vote: its correlation peak to this power
constexpr double REL_MIN = 0.05;     // votes from this fraction of the utterance's largest peak
constexpr int USEG_P = 8;            // per utterance: {segments, 3 piece offsets, 4 delays}

// One wave per piece slot: the first maximum above zero of its NLAG partials, (value, lag index),
// or (0, -1).  Keys (value bits, ~lag) order positive floats as values, ties to the smaller lag.
__global__ void __launch_bounds__(256) ta_piece_peaks(int64_t nslot_total, const float *__restrict__ part,
                                                      float *__restrict__ pv, int *__restrict__ pl,
                                                      double *__restrict__ pw) {
  const int64_t slot = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= nslot_total) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const float *P = part + slot * (int64_t)(NGRP * LG);
  unsigned long long key = 0;
  for (int l = lane; l < NLAG; l += 64) {
    const float v = P[l];
    const unsigned long long k =
        v > 0.f ? ((unsigned long long)__float_as_uint(v) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)l) : 0ull;
    key = k > key ? k : key;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long k2 = __shfl_xor(key, off, 64);
    key = k2 > key ? k2 : key;
  }
  if (lane == 0) {
    pv[slot] = key ? __uint_as_float((unsigned)(key >> 32)) : 0.f;
    pl[slot] = key ? (int)(0xFFFFFFFFu - (unsigned)key) : -1;
    pw[slot] = key ? pow((double)__uint_as_float((unsigned)(key >> 32)), HIST_POW) : 0.0;  // its vote
  }
}

// Workgroup (utterance u, row b): its m pieces' peaks, the votes (REL_MIN of the largest), then
// up to three range evaluations' split searches (stage 12).  The votes (lag, peak^0.125) are
// computed once into LDS (utterances up to PCACHE pieces, 175 minutes at 16 kHz; longer ones
// recompute them from global memory per evaluation); a range's histogram is rebuilt from its
// pieces for every evaluation, each lag's votes and the total added in piece order (double).
constexpr int PCACHE = 2048;
__global__ void __launch_bounds__(256) ta_pick_p862(int64_t B, const int *__restrict__ nutt, const int *__restrict__ cs,
                                                    const int *__restrict__ ucrude, int nslot,
                                                    const float *__restrict__ pv, const int *__restrict__ pl,
                                                    const double *__restrict__ pwg, int *__restrict__ useg) {
  __shared__ double sv[4];
  __shared__ int sj[4];
  __shared__ double H[NGRP * LG + 2 * HIST_T];  // lag l at H[HIST_T + l]; zero margins
  __shared__ double pw[PCACHE];                 // a piece's vote, 0 if it does not vote
  __shared__ int pg[PCACHE];                    // its lag index, -1 if it does not vote
  const int u = blockIdx.y;  // rows fastest in the dispatch order: a row's active workgroups spread over the XCDs
  const int64_t b = blockIdx.x + (int64_t)blockIdx.z * 65535;
  if (b >= B || u >= nutt[b]) return;
  const int tid = threadIdx.x;
  const int c0 = cs[b * (MAXU + 1) + u], m = cs[b * (MAXU + 1) + u + 1] - c0;
  const float *v = pv + b * nslot + c0;
  const int *lg = pl + b * nslot + c0;
  const double *vw = pwg + b * nslot + c0;
  const int d0 = ucrude[b * MAXU + u];
  // the utterance's largest piece peak
  double vmax = 0.0;
  for (int i = tid; i < m; i += 256) vmax = fmax(vmax, (double)v[i]);
  {
    int dummy = 0;
    block_argmax(vmax, dummy, sv, sj);
  }
  const double vmin = REL_MIN * vmax;
  const bool cached = m <= PCACHE;
  auto vote = [&](int i, int &l, double &w) {  // piece i's lag index (-1: no vote) and weight
    if (cached) {
      l = pg[i];
      w = pw[i];
    } else {
      const bool ok = lg[i] >= 0 && (double)v[i] >= vmin;
      l = ok ? lg[i] : -1;
      w = ok ? vw[i] : 0.0;  // no pow here: a select would evaluate it for every piece
    }
  };
  if (cached)
    for (int i = tid; i < m; i += 256) {
      const bool ok = lg[i] >= 0 && (double)v[i] >= vmin;
      pg[i] = ok ? lg[i] : -1;
      pw[i] = ok ? vw[i] : 0.0;
    }
  for (int l = tid; l < NGRP * LG + 2 * HIST_T; l += 256)
    if (l < HIST_T || l >= HIST_T + NLAG) H[l] = 0.0;  // the margins, once: evaluations write every lag
  // (delay, confidence, votes) of pieces [a, e): every thread the same values
  auto eval = [&](int a, int e, int &D, double &conf, int &nv) {
    __syncthreads();  // the previous evaluation's readers of H (and the LDS fills above) are done
    int cnt = 0;
    double tot = 0.0, h[3] = {0.0, 0.0, 0.0};
#pragma unroll 4
    for (int i = a; i < e; ++i) {  // piece order; the thread's own lags only (branch-free: + 0.0)
      int l;
      double w;
      vote(i, l, w);
      cnt += l >= 0;
      tot += w;  // w = 0 for a piece that does not vote
      const double add = ((l & 255) == tid) ? w : 0.0;  // selects, not h[l >> 8]: no scratch array
      h[0] += (l >> 8) == 0 ? add : 0.0;
      h[1] += (l >> 8) == 1 ? add : 0.0;
      h[2] += (l >> 8) == 2 ? add : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (tid + 256 * q < NLAG) H[HIST_T + tid + 256 * q] = h[q];
    __syncthreads();
    double best = -1.0;
    int arg = INT32_MAX;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int l = tid + 256 * q;
      if (l >= NLAG) continue;
      double sm = 0.0;
#pragma unroll
      for (int k = -HIST_T; k <= HIST_T; ++k) sm += (double)(HIST_T + 1 - abs(k)) * H[HIST_T + l + k];
      if (sm > best) {
        best = sm;
        arg = l;
      }
    }
    block_argmax(best, arg, sv, sj);
    nv = cnt;
    if (cnt == 0) {
      D = d0;
      conf = 0.0;
    } else {
      D = d0 - FINE + arg;
      conf = best / ((HIST_T + 1) * tot);
    }
  };
  // the best split of [a, e) whose halves are both more confident than c: its boundary or -1.
  // One evaluation call site (left half at even t, right half at odd t): the evaluation is
  // inlined twice in the kernel, not once per use.
  auto best_split = [&](int a, int e, double c) {
    int bs = -1, dL = 0, nL = 0;
    double bsum = 0.0, cL = 0.0;
    const int ns = e - a >= 4 ? e - a - 3 : 0;  // s in [a + 2, e - 2]
    for (int t = 0; t < 2 * ns; ++t) {
      const int s = a + 2 + (t >> 1);
      const bool rt = t & 1;
      int dd, nn;
      double cc;
      eval(rt ? s : a, rt ? e : s, dd, cc, nn);
      if (!rt) {
        dL = dd;
        cL = cc;
        nL = nn;
      } else if (nL >= 2 && nn >= 2 && abs(dL - dd) >= SPLIT_MIN && cL > c && cc > c && (bs < 0 || cL + cc > bsum)) {
        bs = s;
        bsum = cL + cc;
      }
    }
    return bs;
  };
  // the ranges to evaluate, depth first and left first (segments come out in piece order): a
  // range splits at its best split below depth 2 (P.862 utterance_split, two levels), else it is
  // a segment
  int off[4] = {0, 0, 0, 0}, dl[4] = {0, 0, 0, 0}, n = 0;
  int sa[4] = {0, 0, 0, 0}, se[4] = {m, 0, 0, 0}, sdp[4] = {0, 0, 0, 0}, top = 1;
  while (top > 0) {
    --top;
    const int a = sa[top], e = se[top], dep = sdp[top];
    int D, nv;
    double c;
    eval(a, e, D, c, nv);
    const int sp = dep < 2 ? best_split(a, e, c) : -1;
    if (sp < 0) {
      off[n] = a;
      dl[n++] = D;
    } else {
      sa[top] = sp;
      se[top] = e;
      sdp[top++] = dep + 1;
      sa[top] = a;
      se[top] = sp;
      sdp[top++] = dep + 1;
    }
  }
  if (tid == 0) {
    int *o = useg + (b * MAXU + u) * USEG_P;
    o[0] = n;
    for (int k = 1; k < 4; ++k) o[k] = k < n ? off[k] : 0;
    for (int k = 0; k < 4; ++k) o[4 + k] = k < n ? dl[k] : dl[0];
  }
}

// One thread per row: the utterances' segments in order (equal neighbours merged, at most MAXSEG:
// later ones merge into the last), the row's delay (its longest segment's, the first of equals).
__global__ void __launch_bounds__(64) ta_segments_p862(int64_t B, int64_t L, const int32_t *__restrict__ lengths,
                                                       const int *__restrict__ nutt, const int *__restrict__ reg,
                                                       const int *__restrict__ useg, int *__restrict__ nseg,
                                                       int *__restrict__ seg_start, int *__restrict__ seg_delay,
                                                       int *__restrict__ delay) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  const int U = nutt[b];
  const int *rg = reg + b * (MAXU + 1);
  int *st = seg_start + b * (MAXSEG + 1), *dl = seg_delay + b * MAXSEG;
  int n = 0;
  for (int u = 0; u < U; ++u) {
    const int *o = useg + (b * MAXU + u) * USEG_P;
    for (int k = 0; k < o[0]; ++k) {
      const int d = o[4 + k];
      if ((n > 0 && dl[n - 1] == d) || n == MAXSEG) continue;
      st[n] = rg[u] + (k ? o[k] : 0) * CS;
      dl[n] = d;
      ++n;
    }
  }
  st[n] = (int)row_len(lengths, b, L);
  int best = -1, d = 0;
  for (int k = 0; k < n; ++k)
    if (st[k + 1] - st[k] > best) {
      best = st[k + 1] - st[k];
      d = dl[k];
    }
  if (nseg) nseg[b] = n;
  if (delay) delay[b] = d;
}

// ---------------------------------------------------------------- bad intervals (steps 13-15)
// P.862's realignment of bad intervals (section 10.7 as restated in oracle/align_oracle.py steps
// 13-15) on the per-frame disturbances of the aligned row (fsem_pesq_distances_f32's frames).
constexpr float BAD_THR = 30.f;  // THRESHOLD_BAD_FRAMES
constexpr int BAD_GAP = 4;       // frames: closer bad runs join
constexpr int BAD_MIN = 5;       // frames: shorter intervals are dropped
constexpr int MAXBAD = 16;       // intervals per row (include/fsem.h FSEM_PESQ_MAX_BAD)
constexpr int HOP = 256;         // samples per PESQ frame hop

// PESQ frames of a row (fsem_pesq_frames: PESQ.py:128-133 pads by L % 256, 512-sample frames)
__host__ __device__ inline int pesq_frames_of(int64_t L) {
  const int64_t Lp = L + (L % 256);
  return Lp < 512 ? 0 : (int)(1 + (Lp - 512) / 256);
}

// One wave per row: the symmetric disturbances 64 frames at a time (a ballot of the bad frames),
// the runs walked with bit scans in wave-uniform code as ta_utterances; then (lane 0) each
// interval's samples [256 f0, min(256 f1 + 256, L_row)), the delay of the segment holding its
// first sample, and its 5120-sample pieces as slot descriptors for ta_fine_partial.
__global__ void __launch_bounds__(64) ta_bad_find(int64_t B, int64_t L, const int32_t *__restrict__ lengths,
                                                  const float *__restrict__ frames, int64_t Fcap,
                                                  const int *__restrict__ nseg, const int *__restrict__ seg_start,
                                                  const int *__restrict__ seg_delay, int *__restrict__ n_bad,
                                                  int *__restrict__ bad, int4 *__restrict__ desc,
                                                  int *__restrict__ ndesc, int *__restrict__ cs_bad, int nslot) {
  __shared__ int iv[2 * MAXBAD];
  const int64_t b = blockIdx.x + (int64_t)blockIdx.y * 65535;
  if (b >= B) return;
  const int lane = threadIdx.x;
  const int64_t Lr = row_len(lengths, b, L);
  const int F = std::min<int64_t>(pesq_frames_of(Lr), Fcap);
  const float *sym = frames + 2 * b * Fcap;
  int n = 0, s0 = -1, e0 = -1, rs = -1;  // intervals, joined run [s0, e0), open raw run from rs
  auto flush = [&]() {
    if (s0 >= 0 && e0 - s0 >= BAD_MIN && n < MAXBAD) {
      if (lane == 0) {
        iv[2 * n] = s0;
        iv[2 * n + 1] = e0;
      }
      ++n;
    }
  };
  auto close_run = [&](int k) {  // the raw run [rs, k) ends
    if (s0 >= 0 && rs - e0 < BAD_GAP) {
      e0 = k;
    } else {
      flush();
      s0 = rs;
      e0 = k;
    }
    rs = -1;
  };
  for (int k0 = 0; k0 < (F >= 20 ? F : 0); k0 += 64) {
    const int k = k0 + lane;
    const uint64_t m = __ballot(k < F && sym[k] > BAD_THR);
    int pos = 0;
    while (pos < 64) {
      if (rs >= 0) {
        const uint64_t z = ~m >> pos;
        if (z == 0) break;
        pos += __builtin_ctzll(z);
        close_run(k0 + pos);
      } else {
        const uint64_t o = m >> pos;
        if (o == 0) break;
        pos += __builtin_ctzll(o);
        rs = k0 + pos;
      }
    }
  }
  if (rs >= 0) close_run(F);
  flush();
  __syncthreads();
  if (lane == 0) {
    const int ns = nseg[b];
    const int *st = seg_start + b * (MAXSEG + 1), *sd = seg_delay + b * MAXSEG;
    int *o = bad + b * (MAXBAD * 3);
    int *cb = cs_bad + b * (MAXBAD + 1);
    int c = 0;
    for (int i = 0; i < n; ++i) {
      const int f0 = iv[2 * i], f1 = iv[2 * i + 1];
      const int a = HOP * f0, e = (int)std::min<int64_t>((int64_t)HOP * f1 + HOP, Lr);
      int k = 0;
      while (k + 1 < ns && st[k + 1] <= a) ++k;
      const int d0 = sd[k];
      o[3 * i] = f0;
      o[3 * i + 1] = f1;
      o[3 * i + 2] = d0;
      cb[i] = c;
      for (int p = a; p < e && c < nslot; p += CS) desc[b * nslot + c++] = make_int4(p, std::min(p + CS, e), d0, i);
    }
    cb[n] = c;
    ndesc[b] = c;
    n_bad[b] = n;
  }
}

// Workgroup (interval i, row b): per lag the interval's pieces added in piece order (double), the
// first maximum above zero, else the segment delay (ta_fine_pick per interval).
__global__ void __launch_bounds__(256) ta_bad_pick(int64_t B, const int *__restrict__ n_bad,
                                                   const int *__restrict__ cs_bad, int nslot,
                                                   const float *__restrict__ part, int *__restrict__ bad) {
  __shared__ double sv[4];
  __shared__ int sj[4];
  const int i = blockIdx.y;  // rows fastest in the dispatch order: a row's active workgroups spread over the XCDs
  const int64_t b = blockIdx.x + (int64_t)blockIdx.z * 65535;
  if (b >= B || i >= n_bad[b]) return;
  const int tid = threadIdx.x;
  const int c0 = cs_bad[b * (MAXBAD + 1) + i], m = cs_bad[b * (MAXBAD + 1) + i + 1] - c0;
  const float *P = part + (b * nslot + c0) * (int64_t)(NGRP * LG);
  double v = 0.0;
  int j = INT32_MAX;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int l = tid + 256 * q;
    if (l >= NLAG) continue;
    double t = 0.0;
    for (int s = 0; s < m; ++s) t += P[s * (NGRP * LG) + l];
    if (t > v) {
      v = t;
      j = l;
    }
  }
  block_argmax(v, j, sv, sj);
  if (tid == 0 && j != INT32_MAX) {
    int *o = bad + (b * MAXBAD + i) * 3;
    o[2] = o[2] - FINE + j;
  }
}

// The second degraded row: a2[n] = deg[n + D_i] for n in interval i's samples (0 <= n + D_i <
// L_row), else the aligned row's a[n] (in place allowed: each element is read, then written, by
// one thread).
__global__ void __launch_bounds__(256) ta_bad_shift(const float *__restrict__ deg, const float *aligned, int64_t B,
                                                    int64_t L, int64_t ld, const int32_t *__restrict__ lengths,
                                                    const int *__restrict__ n_bad, const int *__restrict__ bad,
                                                    float *out, int64_t ld_out) {
  __shared__ int lo[MAXBAD], hi[MAXBAD], dl[MAXBAD];
  const int64_t b = blockIdx.y + (int64_t)blockIdx.z * 65535;
  if (b >= B) return;
  const int64_t Lr = row_len(lengths, b, L);
  const int nb = n_bad[b];
  if (threadIdx.x < nb) {
    const int *o = bad + (b * MAXBAD + threadIdx.x) * 3;
    lo[threadIdx.x] = HOP * o[0];
    hi[threadIdx.x] = (int)std::min<int64_t>((int64_t)HOP * o[1] + HOP, Lr);
    dl[threadIdx.x] = o[2];
  }
  __syncthreads();
  const int64_t n = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (n >= L) return;
  const float *y = deg + b * ld;
  float *r = out + b * ld_out;
  const float *a = aligned + b * ld_out;
  float v[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    int k = -1;
    for (int q = 0; q < nb; ++q)
      if (n + t >= lo[q] && n + t < hi[q]) k = q;
    if (k < 0) {
      v[t] = (n + t < L) ? a[n + t] : 0.f;
    } else {
      const int64_t m = n + t + dl[k];
      v[t] = (m >= 0 && m < Lr) ? y[m] : 0.f;
    }
  }
  if (n + 4 <= L) {
    *reinterpret_cast<float4 *>(r + n) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int t = 0; t < 4 && n + t < L; ++t) r[n + t] = v[t];
  }
}

// One wave per row: each interval takes the second row's frames when their symmetric sum is
// smaller (double, wave order), then PESQ.py:168-172's pooling and :240-243's mapping as
// pesq_back's pass 3 (windows lane-strided, wave sums in double).
__global__ void __launch_bounds__(64) ta_bad_pool(const float *__restrict__ frames, const float *__restrict__ frames2,
                                                  const float *__restrict__ dist, int64_t B, int64_t L,
                                                  int64_t Fcap, const int32_t *__restrict__ lengths,
                                                  const int *__restrict__ n_bad, const int *__restrict__ bad,
                                                  float *__restrict__ mos) {
  __shared__ int f0s[MAXBAD], f1s[MAXBAD];
  const int64_t b = blockIdx.x + (int64_t)blockIdx.y * 65535;
  if (b >= B) return;
  const int lane = threadIdx.x;
  const int64_t Lr = row_len(lengths, b, L);
  const int F = std::min<int64_t>(pesq_frames_of(Lr), Fcap);
  if (F < 20 || !__builtin_isfinite(dist[b])) {
    if (lane == 0) mos[b] = __builtin_nanf("");
    return;
  }
  const float *s1 = frames + 2 * b * Fcap, *a1 = s1 + Fcap;
  const float *s2 = frames2 + 2 * b * Fcap, *a2 = s2 + Fcap;
  const int nb = n_bad[b];
  int nu = 0;  // intervals that take the second row's frames (wave-uniform)
  for (int i = 0; i < nb; ++i) {
    const int f0 = bad[(b * MAXBAD + i) * 3], f1 = bad[(b * MAXBAD + i) * 3 + 1];
    double t1 = 0.0, t2 = 0.0;
    for (int f = f0 + lane; f < f1; f += 64) {
      t1 += s1[f];
      t2 += s2[f];
    }
    t1 = wave_sum_d(t1);
    t2 = wave_sum_d(t2);
    if (t2 < t1) {
      if (lane == 0) {
        f0s[nu] = f0;
        f1s[nu] = f1;
      }
      ++nu;
    }
  }
  __syncthreads();
  const int nw = (F - 20) / 10 + 1;
  double as_ = 0.0, aa_ = 0.0;
  for (int w = lane; w < nw; w += 64) {
    double s6 = 0.0, a6 = 0.0;
    for (int i = 0; i < 20; ++i) {
      const int f = 10 * w + i;
      bool second = false;
      for (int q = 0; q < nu; ++q) second |= (f >= f0s[q] && f < f1s[q]);
      const double x = second ? s2[f] : s1[f], y = second ? a2[f] : a1[f];
      const double x2 = x * x, y2 = y * y;
      s6 += x2 * x2 * x2;
      a6 += y2 * y2 * y2;
    }
    const double ps = pow(s6 / 20.0, 1.0 / 6.0), pa = pow(a6 / 20.0, 1.0 / 6.0);
    as_ += ps * ps;
    aa_ += pa * pa;
  }
  as_ = wave_sum_d(as_);
  aa_ = wave_sum_d(aa_);
  if (lane == 0) {
    const double ds = sqrt(as_ / nw), da = sqrt(aa_ / nw);
    double m = 4.5 - 0.1 * ds - 0.0309 * da;
    m = 0.999 + 4.0 / (1.0 + exp(-1.3669 * m + 3.8224));
    mos[b] = (float)m;
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

// utterance mode: the row-mode arrays (E, crude, internal delay; part with nslot pieces per row)
// plus the utterance tables and the internal segment outputs
inline int64_t nslots(int64_t L) { return nchunks(L) + MAXU; }
struct UttWs {
  float *E, *part;
  int *crude, *delay, *nutt, *utt, *reg, *cs, *ucrude, *useg, *nseg, *seg_start, *seg_delay;
};
inline size_t utt_ws_bytes(int64_t B, int64_t L) {
  auto ints = [B](int64_t per_row) { return align_up((size_t)(B * per_row) * 4, 256); };
  return align_up((size_t)(2 * B * std::max<int64_t>(frames_cap(L), 1)) * 4, 256) +
         align_up((size_t)(B * nslots(L) * NGRP * LG) * 4, 256) + ints(1) * 4 + ints(2 * MAXU) +
         2 * ints(MAXU + 1) + ints(MAXU) + ints(4 * MAXU) + ints(MAXSEG + 1) + ints(MAXSEG);
}
inline UttWs utt_carve(void *ws, int64_t B, int64_t L) {
  char *p = static_cast<char *>(ws);
  UttWs w;
  auto take = [&](size_t bytes) {
    char *q = p;
    p += align_up(bytes, 256);
    return q;
  };
  w.E = reinterpret_cast<float *>(take((size_t)(2 * B * std::max<int64_t>(frames_cap(L), 1)) * 4));
  w.part = reinterpret_cast<float *>(take((size_t)(B * nslots(L) * NGRP * LG) * 4));
  auto ti = [&](int64_t per_row) { return reinterpret_cast<int *>(take((size_t)(B * per_row) * 4)); };
  w.crude = ti(1);
  w.delay = ti(1);
  w.nutt = ti(1);
  w.nseg = ti(1);
  w.utt = ti(2 * MAXU);
  w.reg = ti(MAXU + 1);
  w.cs = ti(MAXU + 1);
  w.ucrude = ti(MAXU);
  w.useg = ti(4 * MAXU);
  w.seg_start = ti(MAXSEG + 1);
  w.seg_delay = ti(MAXSEG);
  return w;
}

// P.862 mode: the utterance-mode workspace, then the pieces' peaks and the wider segment table
struct P862Ws {
  float *pv;
  int *pl, *useg;
  double *pw;
};
inline size_t p862_ws_bytes(int64_t B, int64_t L) {
  return utt_ws_bytes(B, L) + 2 * align_up((size_t)(B * nslots(L)) * 4, 256) +
         align_up((size_t)(B * MAXU * USEG_P) * 4, 256) + align_up((size_t)(B * nslots(L)) * 8, 256);
}
inline P862Ws p862_carve(void *ws, int64_t B, int64_t L) {
  char *p = static_cast<char *>(ws) + utt_ws_bytes(B, L);
  P862Ws w;
  w.pv = reinterpret_cast<float *>(p);
  p += align_up((size_t)(B * nslots(L)) * 4, 256);
  w.pl = reinterpret_cast<int *>(p);
  p += align_up((size_t)(B * nslots(L)) * 4, 256);
  w.useg = reinterpret_cast<int *>(p);
  p += align_up((size_t)(B * MAXU * USEG_P) * 4, 256);
  w.pw = reinterpret_cast<double *>(p);
  return w;
}

// bad-interval workspace: the slot descriptors (an interval's pieces: at most nchunks + MAXBAD per
// row, the intervals being disjoint), their counts, the intervals' first slots, the partials
inline int64_t bad_nslots(int64_t L) { return nchunks(L) + MAXBAD; }
struct BadWs {
  int4 *desc;
  int *ndesc, *cs;
  float *part;
};
inline size_t bad_ws_bytes(int64_t B, int64_t L) {
  return align_up((size_t)(B * bad_nslots(L)) * sizeof(int4), 256) + align_up((size_t)B * 4, 256) +
         align_up((size_t)(B * (MAXBAD + 1)) * 4, 256) + align_up((size_t)(B * bad_nslots(L) * NGRP * LG) * 4, 256);
}
inline BadWs bad_carve(void *ws, int64_t B, int64_t L) {
  char *p = static_cast<char *>(ws);
  BadWs w;
  w.desc = reinterpret_cast<int4 *>(p);
  p += align_up((size_t)(B * bad_nslots(L)) * sizeof(int4), 256);
  w.ndesc = reinterpret_cast<int *>(p);
  p += align_up((size_t)B * 4, 256);
  w.cs = reinterpret_cast<int *>(p);
  p += align_up((size_t)(B * (MAXBAD + 1)) * 4, 256);
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
  align::launch_fine((unsigned)(batch * nch), st, ref, deg, batch, length, ld, lengths, w.crude, (int)nch, w.part,
                     align::UttTables{});
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

extern "C" size_t fsem_time_align_utt_workspace_bytes(int64_t batch, int64_t length) {
  if (batch <= 0 || length <= 0) return 0;
  return align::utt_ws_bytes(batch, length);
}

// the utterance and P.862 modes (stages 1-2, 5-7, then 8 or 10-12, then 9)
static int time_align_segmented(bool p862, const float *ref, const float *deg, int64_t batch, int64_t length,
                                int64_t ld, const int32_t *lengths, int32_t max_delay, int32_t *delay,
                                int32_t *n_seg, int32_t *seg_start, int32_t *seg_delay, float *deg_aligned,
                                int64_t ld_out, void *ws, size_t ws_bytes, void *stream) {
  if (!ref || !deg || batch <= 0 || length <= 0 || ld < length || length > kMaxLength || max_delay < 0 ||
      (deg_aligned && (ld_out < length || ld_out % 4 != 0)) || (ld % 4) != 0 ||
      (!delay && !n_seg && !deg_aligned) || ((n_seg != nullptr) != (seg_start != nullptr)) ||
      ((n_seg != nullptr) != (seg_delay != nullptr)))
    return FSEM_EINVAL;
  const int64_t nsl = align::nslots(length);
  if (batch * nsl > INT32_MAX) return FSEM_EINVAL;
  if (!ws || ws_bytes < (p862 ? align::p862_ws_bytes(batch, length) : align::utt_ws_bytes(batch, length)))
    return FSEM_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  align::UttWs w = align::utt_carve(ws, batch, length);
  int *dl = delay ? delay : w.delay;
  int *ns = n_seg ? n_seg : w.nseg;
  int *ss = seg_start ? seg_start : w.seg_start;
  int *sd = seg_delay ? seg_delay : w.seg_delay;
  const int64_t nfr_cap = std::max<int64_t>(align::frames_cap(length), 1);
  const int64_t sig = 2 * batch;
  const int max_frames =
      (int)std::min<int64_t>(((int64_t)max_delay + align::FRAME - 1) / align::FRAME, (int64_t)INT32_MAX);
  auto yz = [](int64_t n) { return dim3(1, (unsigned)std::min<int64_t>(n, 65535), (unsigned)((n + 65534) / 65535)); };
  auto xy = [](int64_t n) { return dim3((unsigned)std::min<int64_t>(n, 65535), (unsigned)((n + 65534) / 65535)); };
  {
    dim3 grid = yz(sig);
    grid.x = (unsigned)((nfr_cap + 15) / 16);
    align::ta_energy<<<grid, 256, 0, st>>>(ref, deg, batch, length, ld, lengths, w.E, nfr_cap);
    FSEM_CHECK_LAUNCH();
  }
  align::ta_envelope<<<xy(sig), 256, 0, st>>>(batch, length, lengths, w.E, nfr_cap);
  FSEM_CHECK_LAUNCH();
  align::ta_crude<<<xy(batch), 256, 0, st>>>(batch, length, lengths, w.E, nfr_cap, max_frames, w.crude);
  FSEM_CHECK_LAUNCH();
  align::ta_utterances<<<xy(batch), 64, 0, st>>>(batch, length, lengths, w.E, nfr_cap, w.nutt, w.utt, w.reg, w.cs);
  FSEM_CHECK_LAUNCH();
  {
    const dim3 grid((unsigned)std::min<int64_t>(batch, 65535), align::MAXU, (unsigned)((batch + 65534) / 65535));
    align::ta_crude_utt<<<grid, 256, 0, st>>>(batch, length, lengths, w.E, nfr_cap, max_frames, w.crude, w.nutt,
                                              w.utt, w.ucrude);
    FSEM_CHECK_LAUNCH();
  }
  align::launch_fine((unsigned)(batch * nsl), st, ref, deg, batch, length, ld, lengths, w.crude, (int)nsl, w.part,
                     align::UttTables{w.nutt, w.reg, w.cs, w.ucrude});
  FSEM_CHECK_LAUNCH();
  if (p862) {
    const align::P862Ws q = align::p862_carve(ws, batch, length);
    align::ta_piece_peaks<<<(unsigned)((batch * nsl + 3) / 4), 256, 0, st>>>(batch * nsl, w.part, q.pv, q.pl, q.pw);
    FSEM_CHECK_LAUNCH();
    const dim3 grid((unsigned)std::min<int64_t>(batch, 65535), align::MAXU, (unsigned)((batch + 65534) / 65535));
    align::ta_pick_p862<<<grid, 256, 0, st>>>(batch, w.nutt, w.cs, w.ucrude, (int)nsl, q.pv, q.pl, q.pw, q.useg);
    FSEM_CHECK_LAUNCH();
    align::ta_segments_p862<<<(unsigned)((batch + 63) / 64), 64, 0, st>>>(batch, length, lengths, w.nutt, w.reg,
                                                                          q.useg, ns, ss, sd, dl);
    FSEM_CHECK_LAUNCH();
  } else {
    const dim3 grid((unsigned)std::min<int64_t>(batch, 65535), align::MAXU, (unsigned)((batch + 65534) / 65535));
    align::ta_pick_utt<<<grid, 256, 0, st>>>(batch, w.nutt, w.cs, w.ucrude, (int)nsl, w.part, w.useg);
    FSEM_CHECK_LAUNCH();
    align::ta_segments<<<(unsigned)((batch + 63) / 64), 64, 0, st>>>(batch, length, lengths, w.nutt, w.reg, w.useg,
                                                                   ns, ss, sd, dl);
    FSEM_CHECK_LAUNCH();
  }
  if (deg_aligned) {
    dim3 grid = yz(batch);
    grid.x = (unsigned)((length + 1023) / 1024);
    align::ta_shift_seg<<<grid, 256, 0, st>>>(deg, batch, length, ld, lengths, ns, ss, sd, deg_aligned, ld_out);
    FSEM_CHECK_LAUNCH();
  }
  return FSEM_OK;
}

extern "C" int fsem_time_align_utt_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                                       int64_t ld, const int32_t *lengths, int32_t max_delay, int32_t *delay,
                                       int32_t *n_seg, int32_t *seg_start, int32_t *seg_delay,
                                       float *deg_aligned, int64_t ld_out, void *ws, size_t ws_bytes,
                                       void *stream) {
  return time_align_segmented(false, ref, deg, batch, length, ld, lengths, max_delay, delay, n_seg, seg_start,
                              seg_delay, deg_aligned, ld_out, ws, ws_bytes, stream);
}

extern "C" size_t fsem_time_align_p862_workspace_bytes(int64_t batch, int64_t length) {
  if (batch <= 0 || length <= 0) return 0;
  return align::p862_ws_bytes(batch, length);
}

extern "C" int fsem_time_align_p862_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                                        int64_t ld, const int32_t *lengths, int32_t max_delay, int32_t *delay,
                                        int32_t *n_seg, int32_t *seg_start, int32_t *seg_delay,
                                        float *deg_aligned, int64_t ld_out, void *ws, size_t ws_bytes,
                                        void *stream) {
  return time_align_segmented(true, ref, deg, batch, length, ld, lengths, max_delay, delay, n_seg, seg_start,
                              seg_delay, deg_aligned, ld_out, ws, ws_bytes, stream);
}

extern "C" size_t fsem_pesq_bad_intervals_workspace_bytes(int64_t batch, int64_t length) {
  if (batch <= 0 || length <= 0) return 0;
  return align::bad_ws_bytes(batch, length);
}

extern "C" int fsem_pesq_bad_intervals_f32(const float *ref, const float *deg, const float *deg_aligned,
                                           int64_t batch, int64_t length, int64_t ld, const int32_t *lengths,
                                           const float *frames, const int32_t *n_seg, const int32_t *seg_start,
                                           const int32_t *seg_delay, int32_t *n_bad, int32_t *bad,
                                           float *deg_second, int64_t ld_out, void *ws, size_t ws_bytes,
                                           void *stream) {
  if (!ref || !deg || !deg_aligned || !frames || !n_seg || !seg_start || !seg_delay || !n_bad || !bad ||
      !deg_second || batch <= 0 || length <= 0 || ld < length || length > kMaxLength || ld_out < length ||
      ld_out % 4 != 0 || ld % 4 != 0)
    return FSEM_EINVAL;
  const int64_t nsl = align::bad_nslots(length);
  if (batch * nsl > INT32_MAX) return FSEM_EINVAL;
  if (!ws || ws_bytes < align::bad_ws_bytes(batch, length)) return FSEM_EWORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const align::BadWs w = align::bad_carve(ws, batch, length);
  const int64_t Fcap = align::pesq_frames_of(length);
  auto yz = [](int64_t n) { return dim3(1, (unsigned)std::min<int64_t>(n, 65535), (unsigned)((n + 65534) / 65535)); };
  auto xy = [](int64_t n) { return dim3((unsigned)std::min<int64_t>(n, 65535), (unsigned)((n + 65534) / 65535)); };
  align::ta_bad_find<<<xy(batch), 64, 0, st>>>(batch, length, lengths, frames, Fcap, n_seg, seg_start, seg_delay,
                                               n_bad, bad, w.desc, w.ndesc, w.cs, (int)nsl);
  FSEM_CHECK_LAUNCH();
  align::UttTables ut{};
  ut.desc = w.desc;
  ut.ndesc = w.ndesc;
  align::launch_fine((unsigned)(batch * nsl), st, ref, deg, batch, length, ld, lengths, nullptr, (int)nsl, w.part,
                     ut);
  FSEM_CHECK_LAUNCH();
  {
    const dim3 grid((unsigned)std::min<int64_t>(batch, 65535), align::MAXBAD, (unsigned)((batch + 65534) / 65535));
    align::ta_bad_pick<<<grid, 256, 0, st>>>(batch, n_bad, w.cs, (int)nsl, w.part, bad);
    FSEM_CHECK_LAUNCH();
  }
  {
    dim3 grid = yz(batch);
    grid.x = (unsigned)((length + 1023) / 1024);
    align::ta_bad_shift<<<grid, 256, 0, st>>>(deg, deg_aligned, batch, length, ld, lengths, n_bad, bad, deg_second,
                                              ld_out);
    FSEM_CHECK_LAUNCH();
  }
  return FSEM_OK;
}

extern "C" int fsem_pesq_pool_f32(const float *frames, const float *frames2, const float *dist, int64_t batch,
                                  int64_t length, const int32_t *lengths, const int32_t *n_bad, const int32_t *bad,
                                  float *mos, void *stream) {
  if (!frames || !frames2 || !dist || !n_bad || !bad || !mos || batch <= 0 || length <= 0 || length > kMaxLength)
    return FSEM_EINVAL;
  const int64_t Fcap = align::pesq_frames_of(length);
  if (Fcap < 20 && !lengths) return FSEM_ESHORT;
  auto xy = [](int64_t n) { return dim3((unsigned)std::min<int64_t>(n, 65535), (unsigned)((n + 65534) / 65535)); };
  align::ta_bad_pool<<<xy(batch), 64, 0, (hipStream_t)stream>>>(frames, frames2, dist, batch, length, Fcap, lengths,
                                                                 n_bad, bad, mos);
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}
