// STOI / ESTOI engine for gfx950 (MI355X).
//
// Replaces the reference's STOI.compute_stoi / compute_metric
// (fast_se_metrics/STOI.py:153-205) and, for 16 kHz (any non-10 kHz) input, the
// BaseMetric resampler (base.py:19-20) -- the 16 -> 10 kHz polyphase resampling is fused
// into the kernels that consume the 10 kHz signal, so the resampled signal never exists
// in HBM.  Four kernels per call:
//
//  stoi_*vad*    resample the signals to 10 kHz (fused, or the joint PESQ front end does it) and
//                the clean rows' VAD quarter sums: energies of hann(257)[1:]-windowed 256-sample
//                frames, hop 128 (STOI.py:92-99), assembled from 64-sample blocks (fsem_vad.h).
//  stoi_select   per utterance: frame energies in dB, 40 dB voice-activity selection against the
//                loudest clean frame, stream compaction of the kept frame indices (STOI.py:101-108).
//  stoi_tob      per (utterance, 32 STFT frames): overlap-added signal built directly from
//                the kept frames (STOI.py:71-86, never materialised), 512-point FFTs of two
//                consecutive frames of one signal (one wave per frame pair), 15 one-third-octave
//                band envelopes (STOI.py:49-69, 121-125).
//  stoi_seg      per utterance: 30-frame segments -- equalisation + clipping, row / column
//                normalisation and correlations for STOI and ESTOI (STOI.py:113-198), one
//                lane per segment, band envelopes staged in LDS (no 30x materialisation).
#include <algorithm>

#include "fsem_fft.h"
#include "fsem_internal.h"
#include "fsem_resample.h"
#include "fsem_vad.h"

namespace fsem {
namespace stoi {

constexpr int NB = 15;     // one-third octave bands
constexpr int NSEG = 30;   // frames per segment
constexpr int VF = 64;     // VAD frames per workgroup
#ifndef FSEM_TOB_TF
#define FSEM_TOB_TF 32
#endif
constexpr int TF = FSEM_TOB_TF;  // STFT frames per workgroup
constexpr float kClip = 1.0f + 5.62341325190349f;  // 1 + 10^(-beta/20), beta = -15 (STOI.py:136-137)

// Per-row lengths: row b holds lens[b] input samples (clamped to [0, ncap]) when lens is
// given, else ncap.  Its 10 kHz length is that of the reference's resampler on the unpadded
// row, ceil(n * nw / orig) (torchaudio Resample, base.py:20), and its VAD frame count
// 1 + (L10 - 256) / 128 (STOI.py:92-94).
struct Rows {
  const int32_t *lens;
  int64_t ncap;
  int orig, nw;  // reduced rate pair (1, 1 for 10 kHz input)
  __device__ __forceinline__ int64_t n(int64_t b) const {
    if (!lens) return ncap;
    const int64_t v = lens[b];
    return v < 0 ? 0 : (v > ncap ? ncap : v);
  }
  __device__ __forceinline__ int64_t l10(int64_t b) const { return (n(b) * nw + orig - 1) / orig; }
  __device__ __forceinline__ int nv(int64_t b) const {
    const int64_t L10 = l10(b);
    return L10 >= 256 ? (int)((L10 - 256) / 128 + 1) : 0;
  }
};

struct Src {
  const float *x;  // input row base (clean or denoised)
  int64_t n;       // input length at the input rate
};

// 10 kHz sample o of a row: either the input itself (sr == 10 kHz) or the fused resampler.
__device__ __forceinline__ float sample10(const Src &s, int64_t o, int64_t L10, bool direct,
                                          const ResampleKernel &rk) {
  if (o < 0 || o >= L10) return 0.f;
  return direct ? s.x[o] : resample_at(s.x, s.n, o, rk);
}

// VAD quarter sums (fsem_vad.h) of the complete 64-sample blocks among the first n samples of
// a 4096-sample chunk y (16-byte aligned; LDS or global), chunk start a multiple of 128 (block
// parity = block index parity).  256 threads: 16 groups of 16 lanes, one block per group and pass
// (block j = 16 pass + group: parity of the group index).  wa, wb = vad_windows(lane,
// (tid >> 4) & 1), loaded by the caller up front (a load here would wait for its stores).
__device__ __forceinline__ void vad_chunk(const float *__restrict__ y, int n, float2 *__restrict__ vrow, int tid,
                                          float4 wa, float4 wb) {
  const int lane = tid & 63, grp = tid >> 4;
  const float4 *__restrict__ y4 = reinterpret_cast<const float4 *>(y);
  for (int j0 = 0; 64 * j0 < n; j0 += 16) {  // uniform trip count: whole groups shuffle together
    const int j = j0 + grp;
    const bool full = 64 * j + 64 <= n;
    const float4 v = full ? y4[16 * j + (lane & 15)] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float e = vad_quarter(v, wa, wb, lane);
    if ((lane & 14) == 0 && full) reinterpret_cast<float *>(vrow)[2 * j + (lane & 1)] = e;
  }
}

// Resample both signals of an utterance to 10 kHz once (written to the workspace, read back
// only for the kept frames by stoi_tob) and compute the clean frame energies (STOI.py:92-99).
// Persistent workgroups walk items (utterance, chunk, signal); the next item's 16 kHz input is
// in flight in registers (range-checked buffer loads) while the current one is resampled.
// 16 -> 10 kHz: each lane evaluates one polyphase group (8 inputs in, 5 outputs out) with the
// compile-time torchaudio kernel kRs16k10k (28 LDS reads, 140 uniform-coefficient FMAs).
constexpr int VF2 = 32;                        // VAD frames per chunk
constexpr int YT = VF2 * 128 + 128;            // 10 kHz samples produced per item (8320)
constexpr int NG = YT / 5 + 2;                 // polyphase groups per item
constexpr int XT4 = (8 * NG + 32) / 4;         // float4s of 16 kHz input staged per item
constexpr int XPF = (XT4 + 255) / 256;         // prefetch float4s per thread
__global__ void __launch_bounds__(256, 2)
    stoi_resample_vad16(const float *__restrict__ ref, const float *__restrict__ deg, Rows rows, int64_t ld,
                        int nchunk, int64_t nitems, float *__restrict__ y10, int64_t y_ld,
                        float2 *__restrict__ vad, int64_t v_ld) {
  __shared__ __attribute__((aligned(16))) float xin[XPF * 256 * 4 + 4];
  __shared__ __attribute__((aligned(16))) float ytile[YT + 8];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches)
  auto item_src = [&](int64_t item, int64_t &b, int &chunk, int &sig, int64_t &o0, int64_t &i0) {
    sig = (int)(item & 1);
    const int64_t bc = item >> 1;
    b = bc / nchunk;
    chunk = (int)(bc - b * nchunk);
    o0 = (int64_t)chunk * (VF2 * 128);
    i0 = 8 * (o0 / 5) - 12;  // 4-aligned base; group m reads x[8m - 10 + t] = xin[8(m - m0) + 4 + t]
  };
  auto prefetch = [&](int64_t item, float4 pre[XPF]) {
    int64_t b, o0, i0;
    int chunk, sig;
    item_src(item, b, chunk, sig, o0, i0);
    const int64_t n_in = rows.n(b);
    const uint32_t nbytes = (uint32_t)(((n_in + 3) & ~(int64_t)3) * 4);
    const float *row = (sig == 0 ? ref : deg) + b * ld;
    const uint64_t base = reinterpret_cast<uint64_t>(row);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    void *p = reinterpret_cast<void *>(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(p, 0, __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
#pragma unroll
    for (int k = 0; k < XPF; ++k) {
      const int64_t t = i0 + 4 * (tid + 256 * k);
      typedef float v4f __attribute__((ext_vector_type(4)));
      v4f v = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(t * 4), 0, 0));
      // zero-pad past the row end (torchaudio pads the input, base.py:20)
      if (t + 3 >= n_in) {
        v.x = (t < n_in) ? v.x : 0.f;
        v.y = (t + 1 < n_in) ? v.y : 0.f;
        v.z = (t + 2 < n_in) ? v.z : 0.f;
        v.w = 0.f;
      }
      pre[k] = make_float4(v.x, v.y, v.z, v.w);
    }
  };
  float4 vwa, vwb;
  vad_windows(lane, (tid >> 4) & 1, vwa, vwb);
  float4 pre[XPF];
  int64_t item = blockIdx.x;
  if (item < nitems) prefetch(item, pre);
  for (; item < nitems; item += gridDim.x) {
    int64_t b, o0, i0;
    int chunk, sig;
    item_src(item, b, chunk, sig, o0, i0);
    const int64_t L10 = rows.l10(b);
    if (o0 >= L10) {  // chunk past this row's end
      if (item + gridDim.x < nitems) prefetch(item + gridDim.x, pre);
      continue;
    }
    // staged at +2 floats: group m's 28 taps then start 16-byte aligned at xin[8(m - m0) + 4]
    float2 *x2 = reinterpret_cast<float2 *>(xin + 2);
#pragma unroll
    for (int k = 0; k < XPF; ++k) {
      x2[2 * (tid + 256 * k)] = make_float2(pre[k].x, pre[k].y);
      x2[2 * (tid + 256 * k) + 1] = make_float2(pre[k].z, pre[k].w);
    }
    lds_barrier();
    if (item + gridDim.x < nitems) prefetch(item + gridDim.x, pre);
    const int64_t o_end = min(o0 + (int64_t)YT, L10);
    const int64_t m0 = o0 / 5;
    const int64_t m1 = (o_end + 4) / 5;
    for (int64_t m = m0 + tid; m < m1; m += 256) {
      const float4 *xs4 = reinterpret_cast<const float4 *>(xin + 8 * (m - m0) + 4);
      float v[28];
#pragma unroll
      for (int t = 0; t < 7; ++t) {
        const float4 q = xs4[t];
        v[4 * t] = q.x;
        v[4 * t + 1] = q.y;
        v[4 * t + 2] = q.z;
        v[4 * t + 3] = q.w;
      }
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < 28; ++t) acc = fmaf(kRs16k10k[j][t], v[t], acc);
        const int64_t o = 5 * m + j;
        if (o >= o0 && o < o_end) ytile[o - o0] = acc;
      }
    }
    lds_barrier();
    // store this chunk's own 10 kHz samples (float4, coalesced; y_ld % 64 == 0, o0 % 4 == 0)
    const int nown = (int)min((int64_t)(VF2 * 128), L10 - o0);
    float *__restrict__ yr = y10 + (b * 2 + sig) * y_ld + o0;
    for (int k = tid; 4 * k < nown; k += 256) {
      if (4 * k + 3 < nown) {
        reinterpret_cast<float4 *>(yr)[k] = reinterpret_cast<const float4 *>(ytile)[k];
      } else {
        for (int c = 4 * k; c < nown; ++c) yr[c] = ytile[c];
      }
    }
    if (sig == 0) vad_chunk(ytile, nown, vad + b * v_ld + (o0 >> 6), tid, vwa, vwb);  // clean VAD quarter sums
    lds_barrier();
  }
}

// Generic rate pairs (and 10 kHz input): one output per thread through resample_at.
constexpr int VF3 = 32;
constexpr int YT3 = VF3 * 128 + 128;
__global__ void __launch_bounds__(256)
    stoi_resample_vad(const float *__restrict__ ref, const float *__restrict__ deg, Rows rows, int64_t ld,
                      int mode, ResampleKernel rk, float *__restrict__ y10, int64_t y_ld,
                      float2 *__restrict__ vad, int64_t v_ld, int64_t b0) {
  __shared__ __attribute__((aligned(16))) float ytile[YT3];
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t b = b0 + blockIdx.y;
  const int64_t o0 = (int64_t)blockIdx.x * (VF3 * 128);
  const int64_t n_in = rows.n(b), L10 = rows.l10(b);
  if (o0 >= L10) return;
  const int64_t o_end = min(o0 + (int64_t)YT3, L10);
  const int ny = (int)(o_end - o0);
  const int nw_own = (int)min((int64_t)(VF3 * 128), L10 - o0);
  float4 vwa, vwb;
  vad_windows(lane, (tid >> 4) & 1, vwa, vwb);
  for (int sig = 0; sig < 2; ++sig) {
    const Src src{(sig == 0 ? ref : deg) + b * ld, n_in};
    for (int k = tid; k < ny; k += 256) ytile[k] = sample10(src, o0 + k, L10, mode == 1, rk);
    lds_barrier();
    float *__restrict__ yr = y10 + (b * 2 + sig) * y_ld + o0;
    for (int k = tid; k < nw_own; k += 256) yr[k] = ytile[k];
    if (sig == 0) vad_chunk(ytile, nw_own, vad + b * v_ld + (o0 >> 6), tid, vwa, vwb);
    lds_barrier();
  }
}

// 10 kHz rows already in HBM (other-rate path: tiled resampler output): the clean rows' VAD
// quarter sums, 4096 samples per workgroup.
constexpr int VQ = 4096;
__global__ void __launch_bounds__(256)
    stoi_vad10(const float *__restrict__ y10, int64_t y_ld, Rows rows, float2 *__restrict__ vad, int64_t v_ld,
               int64_t b0) {
  const int64_t b = b0 + blockIdx.y;
  const int64_t o0 = (int64_t)blockIdx.x * VQ;
  const int64_t L10 = rows.l10(b);
  if (o0 >= L10) return;
  float4 vwa, vwb;
  vad_windows(threadIdx.x & 63, (threadIdx.x >> 4) & 1, vwa, vwb);
  vad_chunk(y10 + (2 * b) * y_ld + o0, (int)min((int64_t)VQ, L10 - o0), vad + b * v_ld + (o0 >> 6), threadIdx.x, vwa,
            vwb);
}

__global__ void __launch_bounds__(256)
    stoi_select(const float2 *__restrict__ vad, int64_t v_ld, int nv_ld, Rows rows, int *__restrict__ idx,
                int *__restrict__ kept) {
  __shared__ float red[8];
  __shared__ int wcount[4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches)
  const int64_t b = blockIdx.x;
  const int NV = rows.nv(b);
  const float2 *__restrict__ q = vad + b * v_ld;
  float m = -INFINITY;
  int nan_seen = 0;
  for (int i = tid; i < NV; i += 256) {
    const float e = vad_energy_db(q, i);
    m = fmaxf(m, e);
    nan_seen |= (e != e);
  }
  m = block_max_256(m, red);
  // a NaN energy (a NaN clean sample) makes torch's max NaN, so no frame passes the test and the
  // row has no segments (STOI NaN); fmaxf alone would skip it
  const float thr = __syncthreads_or(nan_seen) ? __builtin_nanf("") : m - 40.f;  // (max - dynamic_range - e) < 0  (STOI.py:102)
  int base = 0;
  for (int i0 = 0; i0 < NV; i0 += 256) {
    const int i = i0 + tid;
    const bool keep = (i < NV) && ((thr - vad_energy_db(q, i)) < 0.f);
    const unsigned long long bal = __ballot(keep);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wcount[wave] = __popcll(bal);
    lds_barrier();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wcount[w];
    if (keep) idx[b * nv_ld + off + pre] = i;
    base += wcount[0] + wcount[1] + wcount[2] + wcount[3];
    lds_barrier();
  }
  if (tid == 0) kept[b] = base;
}

#ifdef FSEM_STAMPS
// Diagnostic build only (tools/tob_stamps.py): s_memtime at stoi_tob phase boundaries.
constexpr int kTobStampBlocks = 131072;
__device__ unsigned long long g_tob_stamps[kTobStampBlocks][4];
#define TSTAMP(i)                                                                            \
  do {                                                                                       \
    const unsigned lin_ = blockIdx.y * gridDim.x + blockIdx.x;                               \
    if (threadIdx.x == 0 && lin_ < kTobStampBlocks) g_tob_stamps[lin_][i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define TSTAMP(i) \
  do {            \
  } while (0)
#endif

// Peak biased float exponents of a wave's clean and denoised samples (0: all zero or
// denormal), packed (clean << 16 | denoised): per-lane maxima, then a DPP reduction (row
// rotations, row broadcasts) with a packed 16-bit max -- both signals per instruction, no LDS --
// whose last lane holds the wave's maxima (uniform result).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t peak_exponents(float c0, float c1, float c2, float c3, float d0, float d1,
                                                   float d2, float d3) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  // exponent field of the largest magnitude: a float max over |x| (abs source modifiers, max3)
  auto mx4 = [](float a, float b, float c, float d) {
    return __float_as_uint(__builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(a), __builtin_fabsf(b)),
                                           __builtin_fmaxf(__builtin_fabsf(c), __builtin_fabsf(d))));
  };
  const uint32_t mc = mx4(c0, c1, c2, c3), md = mx4(d0, d1, d2, d3);
  uint32_t e = ((mc >> 7) & 0xffff0000u) | (md >> 23);
  auto pmax = [](uint32_t x, uint32_t y) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(us2, x), __builtin_bit_cast(us2, y)));
  };
  e = pmax(e, dpp_u<0x121>(e));  // row_ror:1
  e = pmax(e, dpp_u<0x122>(e));  // row_ror:2
  e = pmax(e, dpp_u<0x124>(e));  // row_ror:4
  e = pmax(e, dpp_u<0x128>(e));  // row_ror:8 -> every lane holds its row's maxima
  // rows 1 and 3 take rows 0 and 2 (row_bcast:15), rows 2 and 3 take lane 31 (row_bcast:31);
  // rows outside the mask read 0, the identity of the max
  e = pmax(e, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, 0x142, 0xA, 0xF, false));
  e = pmax(e, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, 0x143, 0xC, 0xF, false));
  return __builtin_amdgcn_readlane(e, 63);
}

// Powers of one transform in the wave's exchange area, bin k of frame a at tob_pw(k), of frame b
// at TOB_PB + tob_pw(k): bins from 128 on 3 words further, which makes the band sums' 12 piece
// reads (lane l reads its piece start + i) 2-way instead of 3-way bank conflicts in each 32-lane
// half (the piece starts of kObmPiece, gen_tables.py, never straddle bin 128; round 6, 24 fewer
// LDS cycles per transform of ~230); the stores stay lane-linear (64-bin rows, one offset each).
constexpr int TOB_PB = 264;
__device__ __forceinline__ constexpr int tob_pw(int k) { return k + (k >= 128 ? 3 : 0); }
constexpr bool tob_pieces_unsplit() {
  for (int l = 0; l < 64; ++l)
    if (kObmPiece[l][2] < 128 && kObmPiece[l][3] > 128) return false;
  return true;
}
static_assert(tob_pieces_unsplit() && 2 * TOB_PB <= 2 * kFftBuf - 12, "padded band-sum layout");

constexpr int TOB_WAVES = 4;  // 256-thread workgroups (8 waves x 66 KB measured no faster)
__global__ void __launch_bounds__(64 * TOB_WAVES)
    stoi_tob(const float *__restrict__ y10, int64_t y_ld, int64_t B, Rows rows, const int *__restrict__ idx,
             const int *__restrict__ kept, int nv_ld, float *__restrict__ tob, int64_t tmax, int64_t b0) {
  __shared__ __attribute__((aligned(16))) float blk[2][TF + 1][128];
  __shared__ __attribute__((aligned(16))) float xbuf[TOB_WAVES * 2 * kFftBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: kept indices by scalar loads
  const int64_t b = b0 + blockIdx.y;
  const int n = kept[b];
  const int T = n - 2;  // STFT frames of the overlap-added signal: 1 + ((n+1)*128 - 512)/128
  const int64_t L10 = rows.l10(b);
  const int k0 = blockIdx.x * TF;
  if (k0 >= T) return;
  TSTAMP(0);
  const int kend = min(k0 + TF, T);
  const int *kidx = idx + b * nv_ld;
  const float *__restrict__ yc = y10 + (b * 2) * y_ld;
  const float *__restrict__ yd = yc + y_ld;
  // range-checked raw buffer loads over each row's [0, L10): samples past the row end read as 0
  // without a branch per load (torchaudio's zero padding of the overlap-added signal)
  auto row_rsrc = [L10](const float *y) {
    const uint64_t base = reinterpret_cast<uint64_t>(y);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    void *p = reinterpret_cast<void *>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, __builtin_amdgcn_readfirstlane((uint32_t)(L10 * 4)), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rc = row_rsrc(yc), rd = row_rsrc(yd);
  auto at = [](__amdgpu_buffer_rsrc_t r, int64_t o) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(o * 4), 0, 0));
  };
  const float w_lo = kHann256s[lane], w_lo2 = kHann256s[lane + 64];
  const float w_hi = kHann256s[128 + lane], w_hi2 = kHann256s[128 + 64 + lane];

  // overlap-added blocks q = k0+1 .. kend+1:  block_q[t] = w[t] F_{i_q}[t] + w[128+t] F_{i_{q-1}}[128+t]
  const int nblk = kend - k0 + 1;
  // every block of the wave in flight at once (one memory latency round): blocks past nblk
  // re-read the last block (clamped kept index) and are not stored
  constexpr int NBW = (TF + 1 + TOB_WAVES - 1) / TOB_WAVES;  // blocks per wave
  float g[NBW][8];
#pragma unroll
  for (int u = 0; u < NBW; ++u) {
    const int j = min(wave + TOB_WAVES * u, nblk - 1);
    const int q = k0 + 1 + j;
    const int iq = kidx[q], ip = kidx[q - 1];
    const int64_t a0 = 128LL * iq, a1 = 128LL * ip + 128;
    g[u][0] = at(rc, a0 + lane);
    g[u][1] = at(rc, a1 + lane);
    g[u][2] = at(rc, a0 + 64 + lane);
    g[u][3] = at(rc, a1 + 64 + lane);
    g[u][4] = at(rd, a0 + lane);
    g[u][5] = at(rd, a1 + lane);
    g[u][6] = at(rd, a0 + 64 + lane);
    g[u][7] = at(rd, a1 + 64 + lane);
  }
#pragma unroll
  for (int u = 0; u < NBW; ++u) {
    const int j = wave + TOB_WAVES * u;
    if (j < nblk) {  // uniform
      // plain lane-ordered stores (one address VGPR, immediate offsets): no M0 juggling
      blk[0][j][lane] = w_lo * g[u][0] + w_hi * g[u][1];
      blk[0][j][64 + lane] = w_lo2 * g[u][2] + w_hi2 * g[u][3];
      blk[1][j][lane] = w_lo * g[u][4] + w_hi * g[u][5];
      blk[1][j][64 + lane] = w_lo2 * g[u][6] + w_hi2 * g[u][7];
    }
  }
  lds_stores_done();  // other waves read these blocks
  lds_barrier();
  TSTAMP(1);

  cf tw1[8], tw2[8];
  fft512_twiddles(lane, tw1, tw2);
  const float win[4] = {w_lo, w_lo2, w_hi, w_hi2};  // STFT window on the 256 centred samples
  float2 *wbuf = reinterpret_cast<float2 *>(xbuf) + wave * kFftBuf;
  float *pbuf = reinterpret_cast<float *>(wbuf);
  const int plane = (64 - lane) & 63;
  const int pc_sig = kObmPiece[lane][0], pc_band = kObmPiece[lane][1];
  const int pc_lo = kObmPiece[lane][2], pc_hi = kObmPiece[lane][3];
  // this lane's piece in the padded power layout (tob_pw): no piece crosses bin 128
  const int pc_at = TOB_PB * pc_sig + tob_pw(pc_lo);
  const int pc_gs = kObmPiece[lane][4];
  const bool pc_head = kObmPiece[lane][5] != 0;
  // Two consecutive STFT frames of ONE signal per complex FFT (z = frame a + i frame b): the
  // Hermitian split recovers each from Z[k] -/+ conj(Z[N-k]), whose rounding is relative to |Z|
  // in that bin, i.e. to the two frames' own spectra there.  (Pairing clean with denoised instead
  // let a loud clean band leak into a denoised band 100 dB below it -- tone-probe rows whose
  // denoised signal is a pure tone got 2-3x the float32 noise floor of a separate transform in
  // their off-tone bands, tools/tob_dump.py.)  Neighbouring frames share half their samples, so
  // their spectra are alike except at onsets, which the peak equalisation below covers.
  const int nfr = kend - k0;
  const int nfft = 2 * ((nfr + 1) >> 1);  // (signal, frame pair) transforms of this workgroup
  for (int f = wave; f < nfft; f += TOB_WAVES) {
    const int sg = f & 1;          // signal (wave-uniform: TOB_WAVES is even)
    const int ja = 2 * (f >> 1);   // frame a = k0 + ja = [block_{ja}, block_{ja+1}] * w, frame b = a + 1
    const bool has_b = ja + 1 < nfr;
    cf v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = lane + 64 * (r & 1);
      const float a = blk[sg][ja + (r >> 1)][t];
      const float bq = has_b ? blk[sg][ja + 1 + (r >> 1)][t] : 0.f;  // (uniform)
      v[r] = {a * win[r], bq * win[r]};
    }
#pragma unroll
    for (int r = 4; r < 8; ++r) v[r] = {0.f, 0.f};
    // An all-zero frame has an exactly zero spectrum, but the shared transform's rounding is not
    // exactly Hermitian: ~1e-7 of the other frame's spectrum would leak into it, and the segment
    // normalisation (STOI.py:113-119) would turn that leak into a correlation (an all-zero
    // denoised signal next to non-zero frames would score like noise, not 0).
    // The same rounding leaks ~1e-7 of the louder frame's spectrum into the quieter one's, so a
    // frame ~100 dB or more below its neighbour (an onset after silence) would lose its spectrum
    // to the leak.  Pairs with a gap of 2^7 or more in peak sample are equalised first: frame b
    // is scaled by 2^sh to frame a's peak exponent (exact in floating point), its power by 2^-2sh
    // after the FFT (exact again).
    const uint32_t pk = peak_exponents(v[0].r, v[1].r, v[2].r, v[3].r, v[0].i, v[1].i, v[2].i, v[3].i);
    const int ea = (int)(pk >> 16), eb = (int)(pk & 0xffffu);
    const bool a_zero = ea == 0 && !__any(v[0].r != 0.f || v[1].r != 0.f || v[2].r != 0.f || v[3].r != 0.f);
    const bool b_zero = eb == 0 && !__any(v[0].i != 0.f || v[1].i != 0.f || v[2].i != 0.f || v[3].i != 0.f);
    int sh = (ea > 0 && eb > 0) ? ea - eb : 0;
    sh = (sh >= 7 || sh <= -7) ? max(-60, min(60, sh)) : 0;
    if (sh != 0) {  // uniform
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r].i = __builtin_amdgcn_ldexpf(v[r].i, sh);
    }
    // wave-uniform factors, applied to the band envelopes after the square root (powers of two:
    // the same values as scaling every bin's power by 0.25 (x 2^-2sh for frame b's power),
    // short of under/overflow), or 0 for a zero frame.  Scaling after the root keeps the
    // hardware sqrt's input at the equalised level: v_sqrt_f32 loses accuracy on tiny and
    // denormal inputs, which a quiet frame scaled down first would feed it.
    const float a_scale = a_zero ? 0.f : 0.5f;
    const float b_scale = b_zero ? 0.f : __builtin_amdgcn_ldexpf(0.5f, -sh);
    fft512_wave<true>(v, wbuf, lane, tw1, tw2);  // v[4..7] = 0: the frame's zero-padded half
    float pa[4], pb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mr = __shfl(v[7 - r].r, plane, 64);
      float mi = __shfl(v[7 - r].i, plane, 64);
      if (lane == 0) {
        mr = v[(8 - r) & 7].r;
        mi = v[(8 - r) & 7].i;
      }
      // (pa, pb) = (|zr + mr|^2 + (zi - mi)^2, |zi + mi|^2 + (zr - mr)^2) in packed FP32:
      // the same per-element operations as the scalar form, half the instructions
      typedef float f2v __attribute__((ext_vector_type(2)));
      const f2v z = {v[r].r, v[r].i}, m = {mr, mi};
      const f2v sm = z + m;
      const f2v df = z.yx - m.yx;  // (zi - mi, zr - mr)
      const f2v pp = __builtin_elementwise_fma(sm, sm, df * df);
      pa[r] = pp.x;
      pb[r] = pp.y;
    }
    // plain lane-ordered stores: one address VGPR for the kernel, immediate offsets (paired
    // ds_write2st64_b32) -- no M0 save / set / hazard nop / restore per store (4 SALU each, 32
    // per transform: the kernel is issue bound, SQ_INSTS_SALU 45 % of its VALU count)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pbuf[tob_pw(64 * r) + lane] = pa[r];
      pbuf[TOB_PB + tob_pw(64 * r) + lane] = pb[r];
    }
    wave_lds_fence();
    {
      // band sums: one <=12-bin piece per lane (lanes of piece set 0: frame a, set 1: frame b),
      // segmented shuffle reduction per band
      const float *ps = pbuf + pc_at;
      float acc = (pc_lo < pc_hi) ? ps[0] : 0.f;
#pragma unroll
      for (int i = 1; i < 12; ++i) {  // unconditional reads (inside the frame's powers), masked adds
        const float x = ps[i];
        acc += (pc_lo + i < pc_hi) ? x : 0.f;
      }
      // each band's group (1, 2 or 4 lanes, aligned inside a 16-lane row): two in-row DPP steps
      // (row_shl k: lane l reads lane l + k), no LDS round trip
      {
        const float a1 = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, acc), 0x101, 0xF, 0xF, true));
        acc += (pc_gs >= 2) ? a1 : 0.f;
        const float a2 = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, acc), 0x102, 0xF, 0xF, true));
        acc += (pc_gs >= 4) ? a2 : 0.f;
      }
      // hardware square root (1 ulp; the correctly rounded sqrtf is a ~17-instruction sequence
      // that every lane of the wave issues)
      if (pc_head && (pc_sig == 0 || has_b))
        tob[((b + sg * B) * NB + pc_band) * tmax + k0 + ja + pc_sig] =
            __builtin_amdgcn_sqrtf(acc) * (pc_sig ? b_scale : a_scale);
    }
    wave_lds_fence();
  }
  TSTAMP(2);
}

// One lane per 30-frame segment m: x[j][t] = X[j][m + t], y likewise (STOI.py:121-198).
// SEG_T-lane workgroups, one per (utterance, block of SEG_T segments): grid (B, P), so a short
// batch still fills the chip; each writes its block's two correlation sums (double) to
// part[b][p], which stoi_seg_sum adds up in block order (batch-independent: SEG_T is fixed).
// SEG_T = 256 (4 waves, 34 KB of LDS): per-kernel trace A/B at 4096 x 10 s, 3 rounds,
// stoi_seg 0.970 vs 1.002 ms at 128 and the step 6.952 vs 7.001 ms; 384 and 512 lose 40 %
// (profiles/r5_t).  Clean and denoised envelopes interleaved in LDS as (x, y) pairs,
// so every clean/denoised pair of operations is one packed-FP32 instruction (v_pk_fma_f32 /
// v_pk_add_f32 / v_pk_mul_f32: twice the v_fma_f32 rate on gfx950).  The per-lane row
// statistics of the ESTOI time normalisation stay in registers (uniform-index writes from the
// rolled band loop).
#ifndef FSEM_SEG_T
#define FSEM_SEG_T 256
#endif
#ifndef FSEM_SEG_OCC
#define FSEM_SEG_OCC 3
#endif
constexpr int SEG_T = FSEM_SEG_T;
constexpr int SEG_WAVES = SEG_T / 64;
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(SEG_T, FSEM_SEG_OCC)
    stoi_seg(const float *__restrict__ tob, int64_t B, int64_t tmax, const int *__restrict__ kept,
             double *__restrict__ part, int P, int64_t b0) {
  constexpr int W = SEG_T + NSEG;  // frames per pass
  constexpr int LDX = W + 1;
  __shared__ f2 XY[NB][LDX];
  __shared__ double red[2 * SEG_WAVES];
  const int tid = threadIdx.x;
  const int64_t b = b0 + blockIdx.y;
  const int p = blockIdx.x;
  const int n = kept[b];
  const int S = n - 31;  // num_segments = (len - 512)//128 - 30 + 2 with len = (n+1)*128 (STOI.py:183-186)
  const int m0 = p * SEG_T;
  if (m0 >= S) return;  // past this row's segments (stoi_seg_sum reads blocks p < ceil(S / 128))
  const int T = n - 2;
  const float *xc = tob + (b * NB) * tmax;
  const float *xd = tob + ((b + B) * NB) * tmax;
  double st = 0.0, et = 0.0;
  constexpr float kInvN = 1.f / NSEG;
  {
    const int nf = min(W, T - m0);
    // all 2 x 15 x W loads of the pass in flight at once (one latency round), then the stores.
    // Frame indices clamped to the block's last frame instead of predicated loads (no branch per
    // load): the slots past nf hold copies no segment of this block reads (segment m = m0 + tid <
    // S reads frames tid .. tid + 29 < nf)
    {
      f2 va[NB], vb[NB];
      const int t2 = tid + SEG_T;
      const int ia = min(tid, nf - 1), ib = min(t2, nf - 1);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const float *xr = xc + j * tmax + m0, *dr = xd + j * tmax + m0;
        va[j] = (f2){xr[ia], dr[ia]};
        vb[j] = (f2){xr[ib], dr[ib]};
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        XY[j][tid] = va[j];
        if (t2 < W) XY[j][t2] = vb[j];
      }
    }
    lds_barrier();
    const int m = m0 + tid;
    if (m < S) {
      float s_acc = 0.f;
      // per-lane row statistics of the ESTOI time normalisation, kept in VGPRs: the band loop
      // stays rolled and writes them with its uniform index (register-indexed moves)
      f2 rxy[NB], nmr[NB];  // (1/|x - mu_x|, 1/|y - mu_y|), -(mu_x, mu_y) * rxy
      f2 nvar = {0.f, 0.f};  // sum over bands of rxy^2: the time normalisation's noise variance / 1e-24
#pragma unroll 1
      for (int j = 0; j < NB; ++j) {
        // the rows centred in place first: ||row||^2 = ||row - mu||^2 + N mu^2 (two non-negative
        // terms, ~1 ulp) replaces the separate sum of squares, and the clipped row is
        // fma(d, sc, sc mu) -- 30 packed instructions fewer per band
        f2 v[NSEG];
        f2 s1 = {0.f, 0.f};
#pragma unroll
        for (int t = 0; t < NSEG; ++t) {
          v[t] = XY[j][tid + t];
          s1 += v[t];
        }
        const f2 mu = s1 * kInvN;
        f2 dd = {0.f, 0.f};  // (sum dx^2, sum dy^2)
#pragma unroll
        for (int t = 0; t < NSEG; ++t) {
          v[t] = v[t] - mu;
          dd = __builtin_elementwise_fma(v[t], v[t], dd);
        }
        const f2 s2 = __builtin_elementwise_fma(mu * (float)NSEG, mu, dd);
        // equalize_clip (STOI.py:129-139).  Hardware sqrt / rcp / rsq (~1 ulp) instead of the
        // correctly rounded sequences: ~1e-7 relative per segment, far inside the tolerance.
        const float alpha = __builtin_amdgcn_sqrtf(s2.x) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(s2.y) + 1e-9f);
        const f2 sc = {kClip, alpha};  // (x * kClip, alpha * y)
        const f2 smu = sc * mu;
        static_assert(NSEG % 2 == 0, "frame pairs");
        f2 c[NSEG / 2];
        f2 syc2 = {0.f, 0.f};
#pragma unroll
        for (int u = 0; u < NSEG / 2; ++u) {
          const f2 q0 = __builtin_elementwise_fma(v[2 * u], sc, smu), q1 = __builtin_elementwise_fma(v[2 * u + 1], sc, smu);
          c[u] = (f2){fminf(q0.y, q0.x), fminf(q1.y, q1.x)};
          syc2 += c[u];
        }
        const float myc = (syc2.x + syc2.y) * kInvN;
        const f2 myc2 = {myc, myc};
        f2 dcc2 = {0.f, 0.f};
        float dxc = 0.f;
#pragma unroll
        for (int u = 0; u < NSEG / 2; ++u) {
          const f2 dc = c[u] - myc2;
          dcc2 = __builtin_elementwise_fma(dc, dc, dcc2);
          dxc = fmaf(v[2 * u].x, dc.x, dxc);
          dxc = fmaf(v[2 * u + 1].x, dc.y, dxc);
        }
        const float dcc = dcc2.x + dcc2.y;
        // normalize() (STOI.py:113-119) centres, adds 1e-12 * randn and divides by the norm: in
        // expectation the squared norm gains N * 1e-24 (N = 30 frames) and the noise itself
        // averages out of the correlation.  So 1 / sqrt(||row - mean||^2 + 30e-24): the same
        // value for every row with ||row - mean||^2 > 5e-16 (the addend is below its rounding),
        // 0 for a zero-variance row, ~0 for a row far below the noise (where the reference's
        // own result is that noise: inputs at 1e-15 scale score ~0 +- 1e-2 there), and NaN / Inf
        // rows propagate.
        constexpr float kReg30 = 30e-24f;
        const float rxn = __builtin_amdgcn_rsqf(dd.x + kReg30);
        const float ryn = __builtin_amdgcn_rsqf(dd.y + kReg30);
        const float rcn = __builtin_amdgcn_rsqf(dcc + kReg30);
        // torch.minimum (STOI.py:139) propagates a NaN of the scaled denoised row, fminf drops
        // it: a NaN / Inf denoised row (alpha non-finite) poisons the sum as in the reference.
        // (A select, not alpha - alpha: contracted into fma(a, b, -(a b)) that difference is the
        // product's rounding error, not 0.)
        s_acc = fmaf(dxc * rxn, rcn, s_acc) + (__builtin_isfinite(alpha) ? 0.f : __builtin_nanf(""));
        rxy[j] = (f2){rxn, ryn};
        nvar = __builtin_elementwise_fma(rxy[j], rxy[j], nvar);
        nmr[j] = -mu * rxy[j];
      }
      // ESTOI: time-normalised rows, then band (column) normalisation (STOI.py:178-181).  The
      // reference's time normalisation leaves noise of variance 1e-24 * rxy^2 in every element
      // (negligible unless a row is near the 1e-12 noise itself), which the band normalisation's
      // expected squared norm takes after centring (x 14/15), plus its own 15e-24.
      const f2 breg = __builtin_elementwise_fma(nvar, (f2){14e-24f / 15.f, 14e-24f / 15.f}, (f2){15e-24f, 15e-24f});
      float e_acc = 0.f;
      for (int t = 0; t < NSEG; ++t) {
        f2 a[NB];
        f2 ma = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          a[j] = __builtin_elementwise_fma(XY[j][tid + t], rxy[j], nmr[j]);
          ma += a[j];
        }
        ma *= 1.f / NB;
        f2 q = {0.f, 0.f};  // (sum da^2, sum dc^2)
        float ac = 0.f;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const f2 d = a[j] - ma;
          q = __builtin_elementwise_fma(d, d, q);
          ac = fmaf(d.x, d.y, ac);
        }
        const float ra = __builtin_amdgcn_rsqf(q.x + breg.x);
        const float rc = __builtin_amdgcn_rsqf(q.y + breg.y);
        e_acc = fmaf(ac * ra, rc, e_acc);
      }
      st += (double)s_acc;
      et += (double)e_acc;
    }
  }
  // deterministic reduction over the workgroup's waves, in wave order
  st = wave_sum_d(st);
  et = wave_sum_d(et);
  lds_barrier();
  if ((tid & 63) == 0) {
    red[(tid >> 6) * 2] = st;
    red[(tid >> 6) * 2 + 1] = et;
  }
  lds_barrier();
  if (tid == 0) {
    double a = red[0], e = red[1];
#pragma unroll
    for (int w = 1; w < SEG_WAVES; ++w) {
      a += red[2 * w];
      e += red[2 * w + 1];
    }
    part[(b * P + p) * 2] = a;
    part[(b * P + p) * 2 + 1] = e;
  }
}

// Per-utterance totals of stoi_seg's block sums, in block order: compute_correlation /
// num_segments (STOI.py:150,198); NaN without a full segment.
__global__ void __launch_bounds__(256)
    stoi_seg_sum(const double *__restrict__ part, int P, int64_t B, const int *__restrict__ kept,
                 float *__restrict__ stoi_out, float *__restrict__ estoi_out) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int S = kept[b] - 31;
  if (S <= 0) {
    stoi_out[b] = __builtin_nanf("");
    estoi_out[b] = __builtin_nanf("");
    return;
  }
  const int np = (S + SEG_T - 1) / SEG_T;
  const double *q = part + b * P * 2;
  double st = 0.0, et = 0.0;
  for (int p = 0; p < np; ++p) {
    st += q[2 * p];
    et += q[2 * p + 1];
  }
  stoi_out[b] = (float)(st / NB / S);
  estoi_out[b] = (float)(et / NSEG / S);
}

// segment blocks per row of a tob buffer with tmax frames (S <= tmax - 29)
inline int seg_blocks(int64_t tmax) { return tmax > 29 ? (int)((tmax - 29 + SEG_T - 1) / SEG_T) : 1; }

struct Geometry {
  int64_t L10;
  int NV, nv_ld, tmax;
  int64_t v_ld;  // VAD quarter sums per row (float2)
  int64_t y_ld;
  bool direct;
  int mode;
};

inline int make_geometry(int64_t length, int32_t sr, Geometry *g, ResampleKernel *rk) {
  g->direct = (sr == 10000);
  if (g->direct) {
    g->L10 = length;
    rk->orig = rk->nw = 1;
    rk->taps = 1;
    rk->width = 0;
  } else {
    const int rc = make_resample_kernel(sr, 10000, rk);
    if (rc != FSEM_OK) return rc;
    g->L10 = (rk->nw * length + rk->orig - 1) / rk->orig;
  }
  g->NV = g->L10 >= 256 ? (int)((g->L10 - 256) / 128 + 1) : 0;
  g->nv_ld = (int)align_up((size_t)(g->NV > 0 ? g->NV : 1), 64);
  g->v_ld = vad_ld(g->L10);
  g->tmax = g->NV > 2 ? g->NV - 2 : 1;
  g->y_ld = (int64_t)align_up((size_t)g->L10, 64);
  g->mode = g->direct ? 1 : ((sr == 16000) ? 0 : 2);
  return FSEM_OK;
}

inline size_t ws_bytes(int64_t B, const Geometry &g) {
  size_t s = 0;
  s += align_up(sizeof(float2) * (size_t)B * (size_t)g.v_ld, 256);        // VAD quarter sums
  s += align_up(sizeof(int) * (size_t)B * g.nv_ld, 256);                  // kept indices
  s += align_up(sizeof(int) * (size_t)B, 256);                            // kept counts
  s += align_up(sizeof(float) * (size_t)(2 * B) * NB * (size_t)g.tmax, 256);  // tob
  s += align_up(sizeof(double) * 2 * (size_t)B * (size_t)seg_blocks(g.tmax), 256);  // segment block sums
  s += align_up(sizeof(float) * (size_t)(2 * B) * (size_t)g.y_ld, 256);      // 10 kHz signals
  return s;
}

// Pointers into a STOI workspace laid out by ws_bytes().
struct Ws {
  float2 *vad;
  int *idx, *kept;
  float *tob, *y10;
  double *part;
};

inline Ws carve(void *ws, int64_t B, const Geometry &g) {
  Ws w;
  char *p = static_cast<char *>(ws);
  w.vad = reinterpret_cast<float2 *>(p);
  p += align_up(sizeof(float2) * (size_t)B * (size_t)g.v_ld, 256);
  w.idx = reinterpret_cast<int *>(p);
  p += align_up(sizeof(int) * (size_t)B * g.nv_ld, 256);
  w.kept = reinterpret_cast<int *>(p);
  p += align_up(sizeof(int) * (size_t)B, 256);
  w.tob = reinterpret_cast<float *>(p);
  p += align_up(sizeof(float) * (size_t)(2 * B) * NB * (size_t)g.tmax, 256);
  w.part = reinterpret_cast<double *>(p);
  w.y10 = reinterpret_cast<float *>(static_cast<char *>(ws) + ws_bytes(B, g) -
                                    align_up(sizeof(float) * (size_t)(2 * B) * (size_t)g.y_ld, 256));
  return w;
}

// Everything after the clean frame energies: selection, band envelopes, segments.
inline int run_seg(int64_t B, const float *tob, int64_t tmax, const int *kept, double *part, float *stoi_out,
                   float *estoi_out, hipStream_t st) {
  const int P = seg_blocks(tmax);
  for (int64_t b0 = 0; b0 < B; b0 += kMaxGridY) {
    hipLaunchKernelGGL(stoi_seg, dim3((unsigned)P, (unsigned)std::min(B - b0, kMaxGridY)), dim3(SEG_T), 0, st, tob,
                       B, tmax, kept, part, P, b0);
    FSEM_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(stoi_seg_sum, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, part, P, B, kept, stoi_out,
                     estoi_out);
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}

inline int run_tail(int64_t B, const Geometry &g, const Rows &rows, const float *y10, const float2 *vad, int *idx,
                    int *kept, float *tob, int64_t tmax, double *part, float *stoi_out, float *estoi_out,
                    hipStream_t st) {
  hipLaunchKernelGGL(stoi_select, dim3((unsigned)B), dim3(256), 0, st, vad, g.v_ld, g.nv_ld, rows, idx, kept);
  FSEM_CHECK_LAUNCH();
  for (int64_t b0 = 0; b0 < B; b0 += kMaxGridY) {
    hipLaunchKernelGGL(stoi_tob, dim3((unsigned)((g.tmax + TF - 1) / TF), (unsigned)std::min(B - b0, kMaxGridY)),
                       dim3(64 * TOB_WAVES), 0, st, y10, g.y_ld, B, rows, idx, kept, g.nv_ld, tob, tmax, b0);
    FSEM_CHECK_LAUNCH();
  }
  if (stoi_out) return run_seg(B, tob, tmax, kept, part, stoi_out, estoi_out, st);
  return FSEM_OK;
}

inline int run(const float *ref, const float *deg, int64_t B, int64_t length, int64_t ld,
               const int32_t *lengths, int32_t sr, float *stoi_out, float *estoi_out, int32_t *kept_out,
               float *tob_out, int64_t tob_ld, void *ws, size_t ws_size, hipStream_t st) {
  Geometry g;
  ResampleKernel rk;
  int rc = make_geometry(length, sr, &g, &rk);
  if (rc != FSEM_OK) return rc;
  if (g.NV <= 0 && !lengths) return FSEM_ESHORT;  // with lengths: NaN rows instead
  const Rows rows{lengths, length, rk.orig, rk.nw};
  if (!ws || ws_size < ws_bytes(B, g)) return FSEM_EWORKSPACE;
  Ws w = carve(ws, B, g);
  int64_t tmax = g.tmax;
  if (tob_out) {
    w.tob = tob_out;
    tmax = tob_ld;
  }
  if (kept_out) w.kept = kept_out;
  if (g.mode == 0) {
    const int nchunk = (int)((g.L10 + VF2 * 128 - 1) / (VF2 * 128));
    const int64_t nitems = B * (int64_t)nchunk * 2;
    const int ncu = cu_count();
    const int64_t grid = nitems < (int64_t)ncu * 3 ? nitems : (int64_t)ncu * 3;  // 3 resident per CU
    hipLaunchKernelGGL(stoi_resample_vad16, dim3((unsigned)grid), dim3(256), 0, st, ref, deg, rows, ld, nchunk,
                       nitems, w.y10, g.y_ld, w.vad, g.v_ld);
  } else if (g.mode == 2) {
    // other rates: tiled polyphase resampler into the 10 kHz rows, then the clean energies
    rc = launch_resample_tiled(ref, B, length, ld, lengths, w.y10, 2 * g.y_ld, 0, rk, st);
    if (rc != FSEM_OK) return rc;
    rc = launch_resample_tiled(deg, B, length, ld, lengths, w.y10 + g.y_ld, 2 * g.y_ld, 0, rk, st);
    if (rc != FSEM_OK) return rc;
    for (int64_t b0 = 0; b0 < B; b0 += kMaxGridY) {
      hipLaunchKernelGGL(stoi_vad10, dim3((unsigned)((g.L10 + VQ - 1) / VQ), (unsigned)std::min(B - b0, kMaxGridY)),
                         dim3(256), 0, st, w.y10, g.y_ld, rows, w.vad, g.v_ld, b0);
      FSEM_CHECK_LAUNCH();
    }
  } else {
    for (int64_t b0 = 0; b0 < B; b0 += kMaxGridY) {
      hipLaunchKernelGGL(stoi_resample_vad,
                         dim3((unsigned)((g.L10 + VF3 * 128 - 1) / (VF3 * 128)), (unsigned)std::min(B - b0, kMaxGridY)),
                         dim3(256), 0, st, ref, deg, rows, ld, g.mode, rk, w.y10, g.y_ld, w.vad, g.v_ld, b0);
      FSEM_CHECK_LAUNCH();
    }
  }
  FSEM_CHECK_LAUNCH();
  return run_tail(B, g, rows, w.y10, w.vad, w.idx, w.kept, w.tob, tmax, w.part, stoi_out, estoi_out, st);
}

}  // namespace stoi
}  // namespace fsem

using namespace fsem;

extern "C" size_t fsem_stoi_workspace_bytes(int64_t batch, int64_t length, int32_t sample_rate) {
  stoi::Geometry g;
  ResampleKernel rk;
  if (stoi::make_geometry(length, sample_rate, &g, &rk) != FSEM_OK) return 0;
  return stoi::ws_bytes(batch, g);
}

extern "C" int fsem_stoi_f32(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld,
                             const int32_t *lengths, int32_t sample_rate, float *stoi_out, float *estoi_out,
                             void *ws, size_t ws_bytes, void *stream) {
  if (!ref || !deg || !stoi_out || !estoi_out || batch <= 0 || length <= 0 || ld < length || length > kMaxLength)
    return FSEM_EINVAL;
  return stoi::run(ref, deg, batch, length, ld, lengths, sample_rate, stoi_out, estoi_out, nullptr, nullptr, 0,
                   ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int fsem_stoi_tob_f32(const float *ref10, const float *deg10, int64_t batch, int64_t length10,
                                 int64_t ld, int32_t *kept, float *tob, int64_t tmax, void *ws, size_t ws_bytes,
                                 void *stream) {
  if (!ref10 || !deg10 || !kept || !tob || batch <= 0 || length10 <= 0 || ld < length10 || length10 > kMaxLength)
    return FSEM_EINVAL;
  stoi::Geometry g;
  ResampleKernel rk;
  int rc = stoi::make_geometry(length10, 10000, &g, &rk);
  if (rc != FSEM_OK) return rc;
  if (tmax < g.tmax) return FSEM_EINVAL;
  return stoi::run(ref10, deg10, batch, length10, ld, nullptr, 10000, nullptr, nullptr, kept, tob, tmax, ws,
                   ws_bytes, (hipStream_t)stream);
}

extern "C" size_t fsem_pesq_stoi_workspace_bytes(int64_t batch, int64_t length) {
  return align_up(fsem_pesq_workspace_bytes(batch, length), 256) + fsem_stoi_workspace_bytes(batch, length, 16000);
}

extern "C" int fsem_pesq_stoi_f32(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld,
                                  const int32_t *lengths, float *mos, float *stoi_out, float *estoi_out, void *ws,
                                  size_t ws_bytes, void *stream) {
  if (!ref || !deg || !mos || !stoi_out || !estoi_out || batch <= 0 || length <= 0 || ld < length ||
      length > kMaxLength)
    return FSEM_EINVAL;
  stoi::Geometry g;
  ResampleKernel rk;
  int rc = stoi::make_geometry(length, 16000, &g, &rk);
  if (rc != FSEM_OK) return rc;
  if (!lengths && (g.NV <= 0 || fsem_pesq_frames(length) < 20)) return FSEM_ESHORT;
  if (!ws || ws_bytes < fsem_pesq_stoi_workspace_bytes(batch, length)) return FSEM_EWORKSPACE;
  const size_t pesq_bytes = align_up(fsem_pesq_workspace_bytes(batch, length), 256);
  stoi::Ws w = stoi::carve(static_cast<char *>(ws) + pesq_bytes, batch, g);
  const stoi::Rows rows{lengths, length, rk.orig, rk.nw};
  hipStream_t st = (hipStream_t)stream;
  // PESQ-wb with the 10 kHz rows emitted from the same input tiles; the PESQ back end runs on a
  // side stream concurrently with the STOI tail, and the caller's stream joins the side stream.
  // Large batches start the back end (one wave per pair) beside the STOI segment kernel (VALU
  // bound, where its latency-bound waves fit in better than beside the LDS-bound stoi_tob); small
  // batches (several waves per pair) start it as soon as the front end is done, beside
  // stoi_select / stoi_tob, since neither fills the chip.  Both only read what the front end wrote.
  const hipStream_t side = side_stream(st);
  const bool early = pesq::back_waves(batch, length) > 1;
  rc = pesq::run_wb_front(ref, deg, batch, length, ld, lengths, ws, pesq_bytes, w.y10, g.y_ld, w.vad, g.v_ld, st);
  if (rc != FSEM_OK) return rc;
  if (early) {
    rc = stream_wait(side, st);
    if (rc != FSEM_OK) return rc;
    rc = pesq::run_wb_back(batch, length, lengths, mos, ws, side);
    if (rc != FSEM_OK) return rc;
    rc = stoi::run_tail(batch, g, rows, w.y10, w.vad, w.idx, w.kept, w.tob, g.tmax, w.part, stoi_out, estoi_out,
                        st);
  } else {
    rc = stoi::run_tail(batch, g, rows, w.y10, w.vad, w.idx, w.kept, w.tob, g.tmax, w.part, nullptr, nullptr, st);
    if (rc != FSEM_OK) return rc;
    rc = stream_wait(side, st);
    if (rc != FSEM_OK) return rc;
    rc = pesq::run_wb_back(batch, length, lengths, mos, ws, side);
    if (rc != FSEM_OK) return rc;
    rc = stoi::run_seg(batch, w.tob, g.tmax, w.kept, w.part, stoi_out, estoi_out, st);
  }
  const int rj = stream_wait(st, side);
  return rc != FSEM_OK ? rc : rj;
}

#ifdef FSEM_STAMPS
// diagnostic build only (not part of include/fsem.h)
extern "C" int fsem_debug_read_tob_stamps(void *dst, size_t bytes) {
  if (hipDeviceSynchronize() != hipSuccess) return FSEM_ELAUNCH;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(stoi::g_tob_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? FSEM_OK : FSEM_ELAUNCH;
}
#endif

extern "C" const char *fsem_strerror(int code) {
  switch (code) {
    case FSEM_OK: return "ok";
    case FSEM_EINVAL: return "invalid argument";
    case FSEM_EWORKSPACE: return "workspace too small";
    case FSEM_ELAUNCH: return "HIP launch failed";
    case FSEM_ESHORT: return "input too short for the metric";
    case FSEM_ERATE: return "unsupported sample-rate pair";
    default: return "unknown error";
  }
}

extern "C" int fsem_version(void) { return 10; }  // 10: + fsem_pesq_wb_frames_f32; 9: + fsem_pesq_bad_intervals_*, fsem_pesq_pool_f32; 8: + fsem_time_align_p862_*; 7: + fsem_host_buffer_mapped; 6: + fsem_build_id; 5: + fsem_time_align_utt_*; 4: + fsem_pre_emphasize_f32; 3: + fsem_time_align_*, fsem_pesq_distances_*

// The build's content hash (_build.py passes -DFSEM_BUILD_ID); the marker prefix lets the host
// layer read the id from the file without loading it (_build.library_build_id).
#ifndef FSEM_BUILD_ID
#define FSEM_BUILD_ID "unknown"
#endif
static const char kBuildIdMarker[] = "FSEM_BUILD_ID:" FSEM_BUILD_ID;
extern "C" const char *fsem_build_id(void) { return kBuildIdMarker + 14; }
// The offload target, recorded apart from the content hash (_build.library_build_arch): a library
// built for another target is refused at load rather than rebuilt.
#ifndef FSEM_BUILD_ARCH
#define FSEM_BUILD_ARCH "unknown"
#endif
__attribute__((used)) static const char kBuildArchMarker[] = "FSEM_BUILD_ARCH:" FSEM_BUILD_ARCH;

// The drop-in call's scores go straight into its pinned host buffer when the runtime maps that
// buffer into the device address space at the same address (hipHostMalloc memory on ROCm).
extern "C" int fsem_host_buffer_mapped(const void *p) {
  if (!p) return 0;
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void *>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return d == p ? 1 : 0;
}
