// PESQ-wb engine for gfx950 (MI355X).
//
// Replaces the reference's per-utterance PyTorch pipeline
//   PESQ.get_disturbances / compute_metric     fast_se_metrics/PESQ.py:174-245
//   BarkFilterBank                             fast_se_metrics/utils/bark.py:100-204
//   Loudness                                   fast_se_metrics/utils/loudness.py:27-67
// with two kernels:
//
// pesq_front  one 256-thread workgroup per (signal, segment of 56 frames):
//   A  coalesced float4 load of a 15360-sample tile (768 warm-up + 56 hops + 1 hop) into LDS
//   B  level-alignment band-pass power (PESQ.py:92-98), time-parallel:
//        lane j owns chunk j (60 samples); end state of its zero-state response is a
//        linear functional of the chunk (table kBpG); a 4-level Hillis-Steele scan with the
//        chunk transition powers (kBpScan) gives every lane its true start state; lane then
//        re-runs the five-section cascade from that state and sums y^2 over the samples its
//        segment owns.  Filter state decays to <1e-14 within 16 chunks, so 4 levels suffice.
//   C  taper of the first / last 15 samples (PESQ.py:108-109)
//   D  pre-emphasis IIR (PESQ.py:111), same scan scheme (2 states), written back in place
//   E  Hann-512 frames, two frames per 512-point complex FFT (z = frame_a + i*frame_b,
//      radix-8 Stockham, one wave per FFT, LDS exchange), |X|^2 split, DC zeroed; the
//      spectra of 16 frames are parked in the already-consumed part of the tile and the
//      Bark contraction fbank[49x256] x spec runs on MFMA (v_mfma_f32_16x16x4_f32) over the
//      block-sparse K-steps of each 16-band tile.
//   Outputs per signal: Bark bands [F, 49] BEFORE the level scale (linear, applied in the
//   back end), and the partial band-pass power of the segment.  The reference's
//   equalize_ranges (PESQ.py:115-121) cancels exactly under the level alignment and is
//   therefore not computed.
//
// pesq_back   one 256-thread workgroup per utterance: level scale, silent frames, band and
//   frame equalisation, Zwicker loudness, symmetric / asymmetric disturbance, L6/L2 pooling
//   and the MOS mapping (PESQ.py:142-245), deterministic block reductions.
#include "fsem_fft.h"

namespace fsem {

namespace pesq {

constexpr int PT = 256;
constexpr int CH = FSEM_PESQ_CH;  // 60 samples per lane
constexpr int TILE = PT * CH;     // 15360
constexpr int WARM = 768;
constexpr int NF = 56;            // frames per segment
constexpr int OWN = NF * 256;     // samples of band-pass power owned per segment
constexpr int NBARK = 49;
constexpr int SCAN_LD = 11;       // floats per lane in the scan buffer
constexpr int XBUF = 4 * 1024;    // 4 waves x 512 complex
constexpr int SPEC_LD = 257;      // parked spectrum row stride (bank-conflict pad)
constexpr int NBP = 10;           // band-pass states (5 sections)
static_assert(WARM + 256 * (NF + 1) == TILE, "tile geometry");
static_assert(PT * SCAN_LD <= XBUF, "scan buffer fits the exchange buffer");
static_assert(SPEC_LD * 63 + 256 <= TILE + XBUF, "parked spectra stay in LDS");

__global__ void __launch_bounds__(PT, 2)
    pesq_front(const float *__restrict__ ref, const float *__restrict__ deg, int64_t B, int64_t L,
               int64_t ld, int F, int nseg, int npseg, float *__restrict__ bark,
               float *__restrict__ ppart) {
  __shared__ __attribute__((aligned(16))) float tile[TILE];
  __shared__ __attribute__((aligned(16))) float xbuf[XBUF];
  __shared__ float red[8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t s = blockIdx.x / nseg;
  const int g = (int)(blockIdx.x - s * nseg);
  const float *__restrict__ xrow = (s < B) ? ref + s * ld : deg + (s - B) * ld;
  const int64_t tstart = (int64_t)g * OWN - WARM;  // global sample index of tile[0]

  // ---------------------------------------------------------------- A: load tile
  {
    const bool al = ((reinterpret_cast<uintptr_t>(xrow) & 15) == 0);
    float4 *t4 = reinterpret_cast<float4 *>(tile);
    for (int v = tid; v < TILE / 4; v += PT) {
      const int64_t t = tstart + 4 * v;
      float4 val;
      if (al && t >= 0 && t + 3 < L) {
        val = *reinterpret_cast<const float4 *>(xrow + t);
      } else {
        val.x = (t >= 0 && t < L) ? xrow[t] : 0.f;
        val.y = (t + 1 >= 0 && t + 1 < L) ? xrow[t + 1] : 0.f;
        val.z = (t + 2 >= 0 && t + 2 < L) ? xrow[t + 2] : 0.f;
        val.w = (t + 3 >= 0 && t + 3 < L) ? xrow[t + 3] : 0.f;
      }
      t4[v] = val;
    }
  }
  __syncthreads();

  const float4 *__restrict__ my4 = reinterpret_cast<const float4 *>(tile + CH * tid);

  // ---------------------------------------------------------------- B: band-pass power
  {
    float e[NBP];
#pragma unroll
    for (int i = 0; i < NBP; ++i) e[i] = 0.f;
#pragma unroll
    for (int q = 0; q < CH / 4; ++q) {
      const float4 v = my4[q];
      const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int i = 0; i < NBP; ++i) e[i] = fmaf(kBpG[4 * q + c][i], xs[c], e[i]);
      }
    }
    // Hillis-Steele scan over the 256 chunks (truncated: state decays below 1e-14 in 16)
#pragma unroll
    for (int i = 0; i < NBP; ++i) xbuf[tid * SCAN_LD + i] = e[i];
    __syncthreads();
#pragma unroll
    for (int lv = 0; lv < 4; ++lv) {
      const int d = 1 << lv;
      float q[NBP];
#pragma unroll
      for (int i = 0; i < NBP; ++i) q[i] = (tid >= d) ? xbuf[(tid - d) * SCAN_LD + i] : 0.f;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NBP; ++i) {
        float acc = e[i];
#pragma unroll
        for (int k = 0; k < NBP; ++k) acc = fmaf(kBpScan[lv][i][k], q[k], acc);
        e[i] = acc;
      }
#pragma unroll
      for (int i = 0; i < NBP; ++i) xbuf[tid * SCAN_LD + i] = e[i];
      __syncthreads();
    }
    float z[NBP];
#pragma unroll
    for (int i = 0; i < NBP; ++i) z[i] = (tid >= 1) ? xbuf[(tid - 1) * SCAN_LD + i] : 0.f;

    // ownership window of this segment, in tile coordinates
    const int64_t own_len64 = (g < npseg) ? ((L - (int64_t)g * OWN) < OWN ? (L - (int64_t)g * OWN) : OWN) : 0;
    const int own_lo = WARM, own_hi = WARM + (int)own_len64;
    float acc = 0.f;
#pragma unroll 3
    for (int q = 0; q < CH / 4; ++q) {
      const float4 v = my4[q];
      const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float u = xs[c];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const float y = u + z[2 * k];
          z[2 * k] = fmaf(-kBpSecA[k][0], y, z[2 * k + 1]);
          z[2 * k + 1] = fmaf(-kBpSecA[k][1], y, -u);
          u = y;
        }
        const int li = CH * tid + 4 * q + c;
        acc = (li >= own_lo && li < own_hi) ? fmaf(u, u, acc) : acc;
      }
    }
    const float tot = block_sum_256(acc, red);
    if (tid == 0) ppart[s * nseg + g] = tot * (kBpGain * kBpGain);
    __syncthreads();
  }

  // ---------------------------------------------------------------- C: taper (PESQ.py:108-109)
  if (tid < 15) {
    const int64_t t = tid;  // head: x[t] *= (t+1)/16
    const int64_t li = t - tstart;
    if (li >= 0 && li < TILE) tile[li] *= (float)(tid + 1) / 16.f;
  } else if (tid >= 32 && tid < 47) {
    const int64_t t = L - 15 + (tid - 32);  // tail: x[L-15+i] *= (15-i)/16
    const int64_t li = t - tstart;
    if (t >= 0 && li >= 0 && li < TILE) tile[li] *= (float)(15 - (tid - 32)) / 16.f;
  }
  __syncthreads();

  // ---------------------------------------------------------------- D: pre-emphasis (PESQ.py:111)
  {
    float e0 = 0.f, e1 = 0.f;
#pragma unroll
    for (int q = 0; q < CH / 4; ++q) {
      const float4 v = my4[q];
      const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        e0 = fmaf(kPreG[4 * q + c][0], xs[c], e0);
        e1 = fmaf(kPreG[4 * q + c][1], xs[c], e1);
      }
    }
    xbuf[tid * SCAN_LD + 0] = e0;
    xbuf[tid * SCAN_LD + 1] = e1;
    __syncthreads();
#pragma unroll
    for (int lv = 0; lv < 4; ++lv) {
      const int d = 1 << lv;
      const float q0 = (tid >= d) ? xbuf[(tid - d) * SCAN_LD + 0] : 0.f;
      const float q1 = (tid >= d) ? xbuf[(tid - d) * SCAN_LD + 1] : 0.f;
      __syncthreads();
      e0 = fmaf(kPreScan[lv][0][0], q0, fmaf(kPreScan[lv][0][1], q1, e0));
      e1 = fmaf(kPreScan[lv][1][0], q0, fmaf(kPreScan[lv][1][1], q1, e1));
      xbuf[tid * SCAN_LD + 0] = e0;
      xbuf[tid * SCAN_LD + 1] = e1;
      __syncthreads();
    }
    float z0 = (tid >= 1) ? xbuf[(tid - 1) * SCAN_LD + 0] : 0.f;
    float z1 = (tid >= 1) ? xbuf[(tid - 1) * SCAN_LD + 1] : 0.f;
    const float b0 = kPreB[0], b1 = kPreB[1], b2 = kPreB[2], a1 = kPreA[1], a2 = kPreA[2];
    const int64_t lim = L - tstart;  // tile index of the first sample >= L
    float4 *w4 = reinterpret_cast<float4 *>(tile + CH * tid);
#pragma unroll 3
    for (int q = 0; q < CH / 4; ++q) {
      const float4 v = w4[q];
      float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float u = xs[c];
        const float y = fmaf(b0, u, z0);
        z0 = fmaf(b1, u, fmaf(-a1, y, z1));
        z1 = fmaf(b2, u, -a2 * y);
        const int li = CH * tid + 4 * q + c;
        xs[c] = (li < lim) ? y : 0.f;  // the reference zero-pads AFTER the filter (PESQ.py:128)
      }
      w4[q] = make_float4(xs[0], xs[1], xs[2], xs[3]);
    }
  }
  __syncthreads();

  // ---------------------------------------------------------------- E: FFT + Bark (MFMA)
  const int nfr = min(NF, F - g * NF);  // valid frames in this segment
  if (nfr <= 0) return;
  float win[8];
  cf tw1[8], tw2[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    win[r] = kHann512[lane + 64 * r];
    const int i1 = (8 * r * (lane & 7)) & 511;
    const int i2 = (r * lane) & 511;
    tw1[r] = {kTwRe[i1], kTwIm[i1]};
    tw2[r] = {kTwRe[i2], kTwIm[i2]};
  }
  float2 *wbuf = reinterpret_cast<float2 *>(xbuf) + wave * 512;
  const int nrounds = (nfr + 7) / 8;
  const int plane = (64 - lane) & 63;
  for (int rd = 0; rd < nrounds; ++rd) {
    const int fa = 2 * (4 * rd + wave);  // local frame index of z's real part
    float pa[4], pb[4];
    const bool active = fa < nfr;
    if (active) {
      cf v[8];
      const float *fra = tile + WARM + 256 * fa;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int n = lane + 64 * r;
        v[r] = {fra[n] * win[r], fra[256 + n] * win[r]};
      }
      fft512_wave(v, wbuf, lane, tw1, tw2);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float mr = __shfl(v[7 - r].r, plane, 64);
        float mi = __shfl(v[7 - r].i, plane, 64);
        if (lane == 0) {
          mr = v[(8 - r) & 7].r;
          mi = v[(8 - r) & 7].i;
        }
        const float zr = v[r].r, zi = v[r].i;
        pa[r] = 0.25f * ((zr + mr) * (zr + mr) + (zi - mi) * (zi - mi));
        pb[r] = 0.25f * ((zi + mi) * (zi + mi) + (zr - mr) * (zr - mr));
      }
      if (lane == 0) {  // spec[:, :, 0] = 0 (PESQ.py:136)
        pa[0] = 0.f;
        pb[0] = 0.f;
      }
    }
    __syncthreads();  // every wave is done reading the tile for this round
    if (active) {
      float *ra = tile + SPEC_LD * fa;
      float *rb = ra + SPEC_LD;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ra[lane + 64 * r] = pa[r];
        rb[lane + 64 * r] = pb[r];
      }
    }
    if ((rd & 1) || rd == nrounds - 1) {
      // ---- Bark contraction of the 16-frame group on MFMA: C[frame][band] += P x Fb
      __syncthreads();
      const int grp = rd >> 1;
      const int row = lane & 15, kq = lane >> 4;
      const int frow = min(16 * grp + row, nfr - 1);
      const float *srow = tile + SPEC_LD * frow;
      // wave -> (small tile, part of tile 2) ; tile ranges from kBarkTileK
      int tsmall, k0s, k1s, k02, k12;
      if (wave == 0) { tsmall = 0; k02 = 14; k12 = 25; }
      else if (wave == 1) { tsmall = 1; k02 = 25; k12 = 31; }
      else if (wave == 2) { tsmall = -1; k02 = 31; k12 = 47; }
      else { tsmall = 3; k02 = 47; k12 = 59; }
      typedef float f4 __attribute__((ext_vector_type(4)));
      f4 acc_s = {0.f, 0.f, 0.f, 0.f}, acc_2 = {0.f, 0.f, 0.f, 0.f};
      if (tsmall >= 0) {
        k0s = kBarkTileK[tsmall][0];
        k1s = kBarkTileK[tsmall][1];
        const int band = 16 * tsmall + row;
        for (int kk = k0s; kk < k1s; ++kk) {
          const int bin = 4 * kk + kq;
          const float a = srow[bin];
          const float bv = (band < NBARK && kBandOfBin[bin] == band) ? kBarkCorr[band] : 0.f;
          acc_s = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc_s, 0, 0, 0);
        }
      }
      {
        const int band = 32 + row;
        for (int kk = k02; kk < k12; ++kk) {
          const int bin = 4 * kk + kq;
          const float a = srow[bin];
          const float bv = (kBandOfBin[bin] == band) ? kBarkCorr[band] : 0.f;
          acc_2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc_2, 0, 0, 0);
        }
      }
      // C/D layout: col = lane & 15 (band in tile), row = (lane >> 4) * 4 + i (frame)
      float *part = xbuf + wave * 256;  // per-wave tile-2 partial (deterministic order)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[(kq * 4 + i) * 16 + row] = acc_2[i];
      if (tsmall >= 0) {
        const int band = 16 * tsmall + row;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int fl = 16 * grp + kq * 4 + i;
          if (band < NBARK && fl < nfr)
            bark[((int64_t)s * F + (int64_t)g * NF + fl) * NBARK + band] = acc_s[i];
        }
      }
      __syncthreads();
      {
        const int fr_ = tid >> 4, col = tid & 15;
        const float v = xbuf[tid] + xbuf[256 + tid] + xbuf[512 + tid] + xbuf[768 + tid];
        const int fl = 16 * grp + fr_;
        if (fl < nfr) bark[((int64_t)s * F + (int64_t)g * NF + fl) * NBARK + 32 + col] = v;
      }
      __syncthreads();
    }
  }
}

__global__ void __launch_bounds__(256) pesq_power_sum(const float *__restrict__ ppart, int nseg,
                                                      int64_t nsig, float *__restrict__ power) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsig) return;
  float acc = 0.f;
  for (int g = 0; g < nseg; ++g) acc += ppart[s * nseg + g];
  power[s] = acc;
}

// ------------------------------------------------------------------------------ back end
__device__ __forceinline__ float loud(float p, int b) {
  // loudness.py:64-65: (2T)^e ((0.5 + 0.5 P/T)^e - 1), 0 where P <= T; times Sl (folded)
  const float t = kThresh[b];
  if (!(p > t)) return 0.f;
  return kLoud2TE[b] * (powf(fmaf(0.5f, p / t, 0.5f), kLoudExp[b]) - 1.f);
}

__global__ void __launch_bounds__(256)
    pesq_back(const float *__restrict__ bark, const float *__restrict__ power, int64_t B, int64_t L,
              int F, float *__restrict__ scratch, float *__restrict__ mos) {
  __shared__ float ratio[NBARK];
  __shared__ double dred[8];
  __shared__ float fred[8];
  __shared__ float bsum[4][2][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = blockIdx.x;
  const float *__restrict__ bc = bark + (b * (int64_t)F) * NBARK;
  const float *__restrict__ bn = bark + ((b + B) * (int64_t)F) * NBARK;
  float *__restrict__ silent = scratch + b * (int64_t)F * 5;
  float *__restrict__ fr = silent + F;
  float *__restrict__ afpc = fr + F;
  float *__restrict__ sym = afpc + F;
  float *__restrict__ asym = sym + F;
  // PESQ.py:97-100 -- power = sum / (L + 5120) / 1.04684; bark scales by 1e7 / power
  const float pc = power[b] / (float)(L + 5120) / 1.04684f;
  const float pn = power[b + B] / (float)(L + 5120) / 1.04684f;
  const float sc = 1e7f / pc, sn = 1e7f / pn;

  // pass 1: silent frames (PESQ.py:146, loudness.py:48-53 with factor 1e2)
  for (int f = tid; f < F; f += 256) {
    float a = 0.f;
    for (int k = 0; k < NBARK; ++k) {
      const float c = bc[f * NBARK + k] * sc;
      a += (c > kThresh[k] * 100.f) ? c : 0.f;
    }
    silent[f] = (a < 1e7f) ? 1.f : 0.f;
  }
  __syncthreads();
  // pass 2: mean audible band power over all frames (loudness.py:55-60)
  {
    float mc = 0.f, mn = 0.f;
    if (lane < NBARK) {
      const float t100 = kThresh[lane] * 100.f;
      for (int f = wave; f < F; f += 4) {
        if (silent[f] != 0.f) continue;
        const float c = bc[f * NBARK + lane] * sc;
        const float n = bn[f * NBARK + lane] * sn;
        mc += (c > t100) ? c : 0.f;
        mn += (n > t100) ? n : 0.f;
      }
    }
    bsum[wave][0][lane] = mc;
    bsum[wave][1][lane] = mn;
    __syncthreads();
    if (tid < NBARK) {
      const float c = (bsum[0][0][tid] + bsum[1][0][tid] + bsum[2][0][tid] + bsum[3][0][tid]) / F;
      const float n = (bsum[0][1][tid] + bsum[1][1][tid] + bsum[2][1][tid] + bsum[3][1][tid]) / F;
      ratio[tid] = fminf(fmaxf((n + 1000.f) / (c + 1000.f), 0.01f), 100.f);  // PESQ.py:151-152
    }
    __syncthreads();
  }
  // pass 3: frame power ratio (PESQ.py:157-159)
  for (int f = tid; f < F; f += 256) {
    float ac = 0.f, an = 0.f;
    for (int k = 0; k < NBARK; ++k) {
      const float c = ratio[k] * (bc[f * NBARK + k] * sc);
      const float n = bn[f * NBARK + k] * sn;
      ac += (c > kThresh[k]) ? c : 0.f;
      an += (n > kThresh[k]) ? n : 0.f;
    }
    fr[f] = (ac + 5e3f) / (an + 5e3f);
    afpc[f] = ac;
  }
  __syncthreads();
  // pass 4: loudness, disturbances, weighting (PESQ.py:161-224)
  const float sqrt_tw = sqrtf((float)kTotalWidth);
  for (int f = tid; f < F; f += 256) {
    float r = (f >= 1) ? 0.8f * fr[f] + 0.2f * fr[f - 1] : fr[0];  // non-recursive (PESQ.py:161)
    r = fminf(fmaxf(r, 3e-4f), 5.f);
    float s2 = 0.f, as = 0.f;
    for (int k = 0; k < NBARK; ++k) {
      const float ec = ratio[k] * (bc[f * NBARK + k] * sc);
      const float en = r * (bn[f * NBARK + k] * sn);
      const float lc = loud(ec, k), ln = loud(en, k);
      float d = ln - lc;
      const float dz = 0.25f * fminf(lc, ln);
      d = copysignf(fmaxf(fabsf(d) - dz, 0.f), d);
      if (k >= 1) {
        const float wd = kWidthBark[k] * d;
        s2 = fmaf(wd, wd, s2);
        float a = powf((en + 50.f) / (ec + 50.f), 1.2f);
        a = (a < 3.f) ? 0.f : fminf(a, 12.f);
        as += fabsf(wd * a);
      }
    }
    float sy = fmaxf(sqrt_tw * sqrtf(s2), 1e-20f);
    float ay = fmaxf(as, 1e-20f);
    const float w = powf((afpc[f] + 1e5f) / 1e7f, 0.04f);
    sym[f] = fminf(sy / w, 45.f);
    asym[f] = fminf(ay / w, 45.f);
  }
  __syncthreads();
  // pass 5: L6 within 20-frame windows (hop 10), L2 across windows (PESQ.py:168-172)
  const int nw = (F - 20) / 10 + 1;
  double as_ = 0.0, aa_ = 0.0;
  for (int w = tid; w < nw; w += 256) {
    double s6 = 0.0, a6 = 0.0;
    for (int i = 0; i < 20; ++i) {
      const double x = sym[10 * w + i], y = asym[10 * w + i];
      const double x2 = x * x, y2 = y * y;
      s6 += x2 * x2 * x2;
      a6 += y2 * y2 * y2;
    }
    const double ps = pow(s6 / 20.0, 1.0 / 6.0), pa = pow(a6 / 20.0, 1.0 / 6.0);
    as_ += ps * ps;
    aa_ += pa * pa;
  }
  as_ = block_sum_256_d(as_, dred);
  __syncthreads();
  aa_ = block_sum_256_d(aa_, dred + 4);
  if (tid == 0) {
    const double ds = sqrt(as_ / nw), da = sqrt(aa_ / nw);
    double m = 4.5 - 0.1 * ds - 0.0309 * da;           // PESQ.py:240
    m = 0.999 + 4.0 / (1.0 + exp(-1.3669 * m + 3.8224));  // PESQ.py:243
    mos[b] = (float)m;
  }
  (void)fred;
}

inline int frames_of(int64_t L) {
  const int64_t Lp = L + (L % 256);  // PESQ.py:128-130: pad by L % 256 (sic)
  if (Lp < 512) return 0;
  return (int)(1 + (Lp - 512) / 256);
}

struct Geometry {
  int F, nfseg, npseg, nseg;
};

inline Geometry geometry(int64_t L) {
  Geometry g;
  g.F = frames_of(L);
  g.nfseg = (g.F + NF - 1) / NF;
  g.npseg = (int)((L + OWN - 1) / OWN);
  g.nseg = g.nfseg > g.npseg ? g.nfseg : g.npseg;
  return g;
}

}  // namespace pesq
}  // namespace fsem

using namespace fsem;

extern "C" int fsem_pesq_frames(int64_t length) { return pesq::frames_of(length); }

extern "C" size_t fsem_pesq_front_workspace_bytes(int64_t batch, int64_t length) {
  const pesq::Geometry g = pesq::geometry(length);
  return align_up(sizeof(float) * (size_t)(2 * batch) * (size_t)g.nseg, 256);
}

extern "C" size_t fsem_pesq_workspace_bytes(int64_t batch, int64_t length) {
  const pesq::Geometry g = pesq::geometry(length);
  size_t bytes = fsem_pesq_front_workspace_bytes(batch, length);
  bytes += align_up(sizeof(float) * (size_t)(2 * batch) * (size_t)g.F * pesq::NBARK, 256);  // bark
  bytes += align_up(sizeof(float) * (size_t)(2 * batch), 256);                               // power
  bytes += fsem_pesq_back_workspace_bytes(batch, length);                                     // back
  return bytes;
}

extern "C" int fsem_pesq_front_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                                   int64_t ld, float *bark, float *power, void *ws, size_t ws_bytes,
                                   void *stream) {
  if (!ref || !deg || !bark || !power || batch <= 0 || length <= 0 || ld < length) return FSEM_EINVAL;
  const pesq::Geometry g = pesq::geometry(length);
  if (g.F < 20) return FSEM_ESHORT;
  if (ws_bytes < fsem_pesq_front_workspace_bytes(batch, length) || !ws) return FSEM_EWORKSPACE;
  const int64_t nblk = 2 * batch * (int64_t)g.nseg;
  if (nblk > 0x7fffffff) return FSEM_EINVAL;
  float *ppart = static_cast<float *>(ws);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(pesq::pesq_front, dim3((unsigned)nblk), dim3(pesq::PT), 0, st, ref, deg, batch,
                     length, ld, g.F, g.nseg, g.npseg, bark, ppart);
  FSEM_CHECK_LAUNCH();
  hipLaunchKernelGGL(pesq::pesq_power_sum, dim3((unsigned)((2 * batch + 255) / 256)), dim3(256), 0, st,
                     ppart, g.nseg, 2 * batch, power);
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}

extern "C" size_t fsem_pesq_back_workspace_bytes(int64_t batch, int64_t length) {
  const pesq::Geometry g = pesq::geometry(length);
  return align_up(sizeof(float) * (size_t)batch * (size_t)g.F * 5, 256);
}

extern "C" int fsem_pesq_back_f32(const float *bark, const float *power, int64_t batch, int64_t length,
                                  float *mos, void *ws, size_t ws_bytes, void *stream) {
  if (!bark || !power || !mos || batch <= 0 || length <= 0) return FSEM_EINVAL;
  const pesq::Geometry g = pesq::geometry(length);
  if (g.F < 20) return FSEM_ESHORT;
  if (!ws || ws_bytes < fsem_pesq_back_workspace_bytes(batch, length)) return FSEM_EWORKSPACE;
  if (batch > 0x7fffffff) return FSEM_EINVAL;
  hipLaunchKernelGGL(pesq::pesq_back, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream, bark,
                     power, batch, length, g.F, static_cast<float *>(ws), mos);
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}

extern "C" int fsem_pesq_wb_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                                int64_t ld, float *mos, void *ws, size_t ws_bytes, void *stream) {
  if (!ref || !deg || !mos || batch <= 0 || length <= 0 || ld < length) return FSEM_EINVAL;
  const pesq::Geometry g = pesq::geometry(length);
  if (g.F < 20) return FSEM_ESHORT;
  if (!ws || ws_bytes < fsem_pesq_workspace_bytes(batch, length)) return FSEM_EWORKSPACE;
  char *p = static_cast<char *>(ws);
  const size_t front = fsem_pesq_front_workspace_bytes(batch, length);
  float *bark = reinterpret_cast<float *>(p + front);
  p += front + align_up(sizeof(float) * (size_t)(2 * batch) * (size_t)g.F * pesq::NBARK, 256);
  float *power = reinterpret_cast<float *>(p);
  p += align_up(sizeof(float) * (size_t)(2 * batch), 256);
  int rc = fsem_pesq_front_f32(ref, deg, batch, length, ld, bark, power, ws, front, stream);
  if (rc != FSEM_OK) return rc;
  return fsem_pesq_back_f32(bark, power, batch, length, mos, p,
                            fsem_pesq_back_workspace_bytes(batch, length), stream);
}
