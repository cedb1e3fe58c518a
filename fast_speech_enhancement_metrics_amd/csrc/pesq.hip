// PESQ-wb engine for gfx950 (MI355X).
//
// Replaces the reference's per-utterance PyTorch pipeline
//   PESQ.get_disturbances / compute_metric     fast_se_metrics/PESQ.py:174-245
//   BarkFilterBank                             fast_se_metrics/utils/bark.py:100-204
//   Loudness                                   fast_se_metrics/utils/loudness.py:27-67
// with two kernels:
//
// pesq_front  persistent 256-thread workgroups over items (signal, segment of 48 frames):
//   A  float4 buffer loads of a 13 312-sample tile (768 warm-up + 48 hops + 1 hop) into LDS
//      at the item's start (the other resident workgroup covers their latency)
//   J  (joint entry only) STOI's 16 -> 10 kHz resampler on the same tile, on MFMA, plus the
//      STOI VAD quarter sums of the clean rows (see resample_tile)
//   B  level-alignment band-pass power (PESQ.py:92-98), time-parallel:
//        lane j owns chunk j (52 samples); end state of its zero-state response is a
//        linear functional of the chunk (table kScanG); a 4-level Hillis-Steele scan with the
//        chunk transition powers (kBpScan) gives every lane its true start state; lane then
//        re-runs the five-section cascade from that state and sums y^2 over the samples its
//        segment owns.  Filter state decays to <1e-11 within 16 chunks, so 4 levels suffice.
//   C  taper of the first / last 15 samples (PESQ.py:108-109)
//   D  pre-emphasis IIR (PESQ.py:111), same scan scheme: FIR part first, then the all-pole
//      part on states y[n-1], y[n-2] (as the reference's lfilter), written back in place
//   E  Hann-512 frames, two frames per 512-point complex FFT (z = frame_a + i*frame_b,
//      radix-8 Stockham, one wave per FFT, LDS exchange), |X|^2 split, DC zeroed; the
//      spectra of the 48 frames are parked in the already-consumed part of the tile and the
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
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <type_traits>

#include "fsem_fft.h"
#include "fsem_internal.h"
#include "fsem_pesq.h"
#include "fsem_vad.h"

namespace fsem {

namespace pesq {

#ifdef FSEM_STAMPS
// Diagnostic build only (tools/stamps.py): s_memtime at phase boundaries of pesq_front.
constexpr int kStampBlocks = 65536;
__device__ unsigned long long g_stamps[kStampBlocks][16];
#define STAMP(i)                                                                                   \
  do {                                                                                             \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks) g_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

// Diagnostic builds only (tools/ab_front.py): FSEM_DOUBLE = k runs phase k
// of pesq_front twice per item (1 resampler, 2 IIR pass 1, 3 chunk scan, 4 FFTs, 5 IIR pass 2)
// -- the marginal wall time of a phase inside the full kernel; the outputs are not meaningful.
#ifndef FSEM_DOUBLE
#define FSEM_DOUBLE 0
#endif

constexpr int PT = 256;
constexpr int CH = FSEM_PESQ_CH;  // 52 samples per lane (stride 208 B: conflict-free b128)
constexpr int TILE = PT * CH;     // 13312
constexpr int WARM = 768;
constexpr int NS = 12;            // scan states: 10 band-pass (5 sections) + 2 pre-emphasis
// floats per lane in the scan buffer: 12, the states as three 16-byte words (ds_read_b128 /
// ds_write_b128, conflict-free at a 48-byte stride -- lanes l, l + 16 share banks, and the
// b128 lane groups hold distinct l mod 16; one LDS round trip per scan level instead of six
// ds_read2_b32 waited for one by one)
constexpr int SCAN_LD = 12;
// exchange buffer: 4 waves x 512 complex for the FFTs, the resampler's per-wave staging slices
// (4 x 960 floats, joint entry), or the two buffers of the double-buffered chunk scan.  Scan
// buffer A keeps wave w's states inside wave w's own staging slice (960 w + 13 lane: no wave
// writes into a slice another wave may still be reading, and no barrier is needed between the
// resampler and the scan); buffer B (first written after a barrier) is packed after A's last
// state.  With the tile, 81 568 B per workgroup: 2 fit a CU.
constexpr int SCAN_A_WAVE = 960;                               // = the resampler's RS_STAGE
constexpr int SCAN_B0 = 3 * SCAN_A_WAVE + 64 * SCAN_LD;        // just past buffer A
constexpr int XBUF = 3 * SCAN_A_WAVE + 64 * 13 + PT * 13;      // 7040 floats
static_assert(XBUF >= 4 * 2 * kFftBuf, "FFT exchange areas fit");
constexpr int SPEC_LD = 258;      // parked spectrum row stride: = 2 mod 32, MFMA A reads conflict-free
constexpr int NBP = 10;           // band-pass states
constexpr int PF = TILE / 4 / PT; // float4 per thread per tile
static_assert(WARM + 256 * (NF + 1) == TILE, "tile geometry");
static_assert(64 * SCAN_LD <= SCAN_A_WAVE && SCAN_B0 + PT * SCAN_LD <= XBUF && (SCAN_B0 * 4) % 16 == 0,
              "scan buffer A: a wave's states within its staging slice; B within the exchange buffer");
static_assert(SPEC_LD * (NF - 1) + 256 <= TILE, "parked spectra stay in the tile");
static_assert(TILE % (4 * PT) == 0, "tile load split");

// PESQ.py:90,108-109: first 15 samples x (t+1)/16, last 15 samples x (L-t)/16, else 1:
// w(t) = sat((t+1)/16) * sat((L-t)/16), exact in float32 for t, L < 2^24.
__device__ __forceinline__ float taper_w(float tf, float Lf) {
  return __saturatef((tf + 1.f) * 0.0625f) * __saturatef((Lf - tf) * 0.0625f);
}

// Range of a tile: float32 squares and |X|^2 of the band-pass / pre-emphasis outputs stay
// finite and normal for tile scales within [2^-40, 2^40] (the scale: the peak magnitude of the
// chunks' pass-1 end states, which bound both filters' outputs to within their gains, a factor
// ~100).  The main front-end pass only flags a signal with a tile outside that window (rare:
// a worklist of signals in the workspace); the SAFE instance then redoes the flagged signals'
// segments, each tile scaled by 2^sh (its scale to [1, 2); exact in floating point) from pass 2
// on: the segment's Bark bands and power partials carry 2^(2 sh), recorded per (signal, segment)
// in pexp and undone in the back end.  The reference divides both signals by their joint peak
// first (equalize_ranges, PESQ.py:115-121), which cancels under the level alignment except for
// this range: without the scaling, common scales of 1e-15 / 1e18 gave NaN / 4.64.
__device__ __forceinline__ bool out_of_range(float peak) {
  const int ex = (int)((__float_as_uint(peak) >> 23) & 0xff);
  return peak != 0.f && (ex < 127 - 40 || ex >= 127 + 40);  // denormal / tiny, huge or Inf
}
__device__ __forceinline__ int range_shift(float peak) {
  const uint32_t bits = __float_as_uint(peak);
  const int ex = (int)((bits >> 23) & 0xff);  // biased exponent: 0 = zero / denormal, 255 = inf / NaN
  if (ex == 0 || ex == 255 || (ex >= 127 - 40 && ex < 127 + 40)) return 0;
  return 127 - ex;  // peak * 2^sh in [1, 2)
}

// Wave maximum of non-negative floats (as integers: same order), uniform result: DPP row
// rotations, then row broadcasts (rows outside the mask read 0, the identity); lane 63 holds it.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_rot(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ float wave_max_pos(float v) {
  uint32_t e = __float_as_uint(v);
  e = max(e, dpp_rot<0x121>(e));  // row_ror:1
  e = max(e, dpp_rot<0x122>(e));  // row_ror:2
  e = max(e, dpp_rot<0x124>(e));  // row_ror:4
  e = max(e, dpp_rot<0x128>(e));  // row_ror:8
  e = max(e, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, 0x142, 0xA, 0xF, false));  // row_bcast:15
  e = max(e, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return __uint_as_float(__builtin_amdgcn_readlane(e, 63));
}

// Wave sum by DPP (row rotations 1, 2, 4, 8 -- every lane then holds its row's sum -- and two
// row broadcasts), read from lane 63: no LDS round trip (the butterfly of __shfl_xor is six
// ds_bpermute waited for one by one).  A fixed summation order, deterministic.
__device__ __forceinline__ float wave_sum_dpp(float v) {
  auto rot = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), decltype(ctrl)::value, 0xF, 0xF, false));
  };
  v += rot(v, std::integral_constant<int, 0x121>{});  // row_ror:1
  v += rot(v, std::integral_constant<int, 0x122>{});  // row_ror:2
  v += rot(v, std::integral_constant<int, 0x124>{});  // row_ror:4
  v += rot(v, std::integral_constant<int, 0x128>{});  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));  // row_bcast:15
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));  // row_bcast:31
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

struct Item {
  int64_t s;       // signal (0..B-1 ref, B..2B-1 deg)
  int g;           // segment
  int64_t tstart;  // global sample index of tile[0]
  const float *xrow;
  int64_t L;       // this row's length
};

__device__ __forceinline__ Item make_item(int64_t item, int nseg, int64_t B, int64_t ld, int64_t L,
                                          const int32_t *__restrict__ lens, const float *ref,
                                          const float *deg) {
  Item it;
  it.s = item / nseg;
  it.g = (int)(item - it.s * nseg);
  it.tstart = (int64_t)it.g * OWN - WARM;
  const int64_t b = (it.s < B) ? it.s : it.s - B;
  it.xrow = ((it.s < B) ? ref : deg) + b * ld;
  it.L = row_length(lens, b, L);
  return it;
}

// One tile straight into LDS: buffer loads with the LDS as destination (buffer_load_dwordx4 ...
// lds: 16 bytes per lane to the wave-uniform base in M0 + 16 lane), no VGPRs, no LDS stores.
// A wave-uniform descriptor over [0, ceil4(L)): out-of-range float4s (t < 0 wraps the 32-bit
// offset; t >= ceil4(L)) arrive as zeros from the hardware range check.  Samples in
// [L, ceil4(L)) may hold anything: both filters are causal and every output at t >= L is
// masked, so they cannot reach a PESQ result (rows must be readable up to ceil4(L),
// include/fsem.h); the joint resampler zeroes them (below).  The caller waits (vmcnt) and
// barriers before reading the tile.  Measured in round 3: loading the next item's tile into
// registers during the FFT / Bark phases (a prefetch, 52 VGPRs held across them) was slower
// than loading at the item's start (5.27 vs 5.21 ms): the second resident workgroup hides the
// latency, and the prefetch registers cost spills and scheduling.
__device__ __forceinline__ void load_tile_lds(const Item &it, int tid, float *tile) {
  const int64_t L = it.L;
  const uint64_t base = reinterpret_cast<uint64_t>(it.xrow);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  const uint32_t nbytes = __builtin_amdgcn_readfirstlane((uint32_t)(((L + 3) & ~(int64_t)3) * 4));
  void *p = reinterpret_cast<void *>(((uint64_t)hi << 32) | lo);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(p, 0, nbytes, 0x00020000);
  const int t0 = (int)it.tstart;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int t = t0 + 4 * (tid + PT * k);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsrc, (__attribute__((address_space(3))) void *)(tile + 4 * (64 * wave + PT * k)), 16, t * 4, 0, 0, 0);
  }
}

// Pre-emphasis FIR part (PESQ.py:111 via torchaudio's lfilter: FIR first, then the all-pole
// part).  The float32 numerator is exactly b0 (1, -2, 1) (b1 = -2 b0 and b2 = b0 in float32), so
// w = b0 (x[n] - 2 x[n-1] + x[n-2]) = b0 ((x[n] - x[n-1]) - (x[n-1] - x[n-2])): the second
// difference of the tapered input, formed from first differences (exact for neighbouring samples
// within a factor 2 of each other), so a DC offset cancels exactly and never enters the all-pole
// states.  b0 moves to the output (the FFT window carries it): the all-pole part runs on
// yh = y / b0 driven by the second difference.  h1 = x[n-1], d1 = x[n-1] - x[n-2].
__device__ __forceinline__ float pre_fir(float xp, float &h1, float &d1) {
  const float d = xp - h1;
  const float dd = d - d1;
  d1 = d;
  h1 = xp;
  return dd;
}

// Opaque first differences.  The IIR passes take the chunk's samples as first differences
// x[n] - x[n-1]; the SLP vectoriser pairs two of them as (x[n], x[n+1]) - (x[n-1], x[n]) and
// fetches the odd-aligned pair straight from LDS, splitting the chunk's float4 loads into b96 /
// read2_b32 pieces (more LDS instructions, 4-way bank conflicts at the 52-float chunk stride).
// An empty asm on the difference keeps it scalar: one v_sub per sample, ds_read_b128 loads.
// (Applied on the hot paths -- pass 1 without taper, the split pass 2; in the masked pass 2 it
// makes the compiler unroll the loop fully, +45 % VALU code.)
__device__ __forceinline__ float opaque_diff(float a, float b) {
  float d = a - b;
  asm("" : "+v"(d));
  return d;
}

// IIR pass 1: end states of this lane's chunk from zero state -- band-pass (states 0..9,
// untapered input) and pre-emphasis all-pole part (states 10..11, driven by the second
// difference of the tapered input) -- as functionals of the chunk's first differences
// (kScanG, gen_tables.py) plus the boundary terms of the samples before it: h1 = x[-1] and
// d1 = x[-1] - x[-2] (tapered).  Fully unrolled: the functionals (__constant__) come in by
// scalar loads as SGPR operands.  Edge chunks (TAPER) keep separate differences of the raw
// (band-pass) and tapered (pre-emphasis) input; samples past the row end (up to ceil4(L): any
// value) stay out of both, so out of the end states, which also decide the tile's range check.
template <bool TAPER>
__device__ __forceinline__ void iir_pass1(const float4 *__restrict__ my4, int64_t t_lane, int64_t L, float h1,
                                          float d1, float hr, float e[NS]) {
  const float tf0 = (float)t_lane, Lf = (float)L;
  // opaque table pointer: the rows stay memory operands (s_load) instead of folded literals.
  // (Measured in round 5: the rows from an LDS copy by broadcast ds_read_b128 instead -- no
  // SGPR streaming -- made the joint front end 13 % slower rolled, 27 % unrolled)
  uint64_t gaddr = reinterpret_cast<uint64_t>(&kScanG[0][0]);
  asm volatile("" : "+s"(gaddr));
  // the 12 functionals as six packed pairs (states 2j, 2j + 1): one v_pk_fma_f32 per pair and
  // sample with the pair's SGPR operand straight from the scalar loads, written out rather than
  // left to the SLP vectoriser (which pesq.hip is compiled without: it paired literal constants
  // into SGPRs with two s_mov_b32 each elsewhere, _build.SOURCE_FLAGS)
  typedef float pf2v __attribute__((ext_vector_type(2)));
  typedef const __attribute__((address_space(4))) pf2v crow2[NS / 2];
  crow2 *G = reinterpret_cast<crow2 *>(gaddr);
  pf2v ep[NS / 2];
#pragma unroll
  for (int j = 0; j < NBP / 2; ++j) ep[j] = (pf2v){kScanB[2 * j], kScanB[2 * j + 1]} * hr;  // S x[-1] (untapered)
  ep[NBP / 2] = (pf2v){kScanB[NBP], kScanB[NBP + 1]} * d1;                                // -G2[0] d[-1] (tapered)
  float xr = hr;  // previous raw sample (TAPER: the band-pass's own history)
#pragma unroll
  for (int q = 0; q < CH / 4; ++q) {
    const float4 v = my4[q];
    const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int n = 4 * q + c;
      float dp, db;
      if (TAPER) {
        const float xb = (t_lane + n >= L) ? 0.f : xs[c];
        const float xp = xs[c] * taper_w(tf0 + (float)n, Lf);  // 0 past the row end
        db = xb - xr;
        xr = xb;
        dp = xp - h1;
        h1 = xp;
      } else {
        db = dp = opaque_diff(xs[c], h1);
        h1 = xs[c];
      }
#pragma unroll
      for (int j = 0; j < NBP / 2; ++j) ep[j] = __builtin_elementwise_fma(G[n][j], (pf2v){db, db}, ep[j]);
      ep[NBP / 2] = __builtin_elementwise_fma(G[n][NBP / 2], (pf2v){dp, dp}, ep[NBP / 2]);
    }
  }
#pragma unroll
  for (int j = 0; j < NS / 2; ++j) {
    e[2 * j] = ep[j].x;
    e[2 * j + 1] = ep[j].y;
  }
}

// IIR pass 2 from the true start state z: band-pass cascade (power over owned samples) and
// pre-emphasis, whose output overwrites the chunk in place (zero from `lim` on).
// MASK: per-sample ownership / end-of-row masks (first / last segment of a row, edge waves).
// Without MASK every sample is owned-or-not by whole 4-sample groups: a non-final segment's
// owned range [WARM, WARM + OWN) cuts chunks only at chunk offsets P_LO = WARM % CH and
// P_HI = (WARM + OWN) % CH, so the band-pass power is summed in three accumulators --
// samples [0, P_HI), [P_HI, P_LO), [P_LO, CH) -- and each lane keeps the parts it owns.
constexpr int P_HI = (WARM + OWN) % CH, P_LO = WARM % CH;
static_assert(P_HI % 4 == 0 && P_LO % 4 == 0 && P_HI < P_LO, "pass-2 power split points");

// Pre-emphasis all-pole part of one sample: y = w - a1 y[n-1] - a2 y[n-2], states z[NBP] =
// y[n-1], z[NBP + 1] = y[n-2].
__device__ __forceinline__ float pre_ap(float w, float z[NS]) {
  const float y = fmaf(-kPreA[1], z[NBP], fmaf(-kPreA[2], z[NBP + 1], w));
  z[NBP + 1] = z[NBP];
  z[NBP] = y;
  return y;
}

// Pre-emphasis of one untapered sample, the split pass's (the same arithmetic as pre_fir + pre_ap).
__device__ __forceinline__ float pre_step(float xp, float z[NS], float &h1, float &h2) {
  const float d = opaque_diff(xp, h1);
  const float dd = d - h2;
  h2 = d;
  h1 = xp;
  return pre_ap(dd, z);
}

template <bool TAPER, bool MASK>
__device__ __forceinline__ void iir_pass2_group(float4 *__restrict__ w4, int q, float z[NS], float &acc, int own_lo,
                                                int own_hi, int lim, float tf0, float Lf, float &h1, float &h2) {
  const float4 v = w4[q];
  float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int n = 4 * q + c;
    float u = xs[c];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float y = u + z[2 * k];
      z[2 * k] = fmaf(-kBpSecA[k][0], y, z[2 * k + 1]);
      z[2 * k + 1] = fmaf(-kBpSecA[k][1], y, -u);
      u = y;
    }
    acc = (!MASK || (n >= own_lo && n < own_hi)) ? fmaf(u, u, acc) : acc;
    const float xp = TAPER ? xs[c] * taper_w(tf0 + (float)n, Lf) : xs[c];
    const float y = pre_ap(pre_fir(xp, h1, h2), z);
    xs[c] = (!MASK || n < lim) ? y : 0.f;  // the reference zero-pads AFTER the filter (PESQ.py:128)
  }
  w4[q] = make_float4(xs[0], xs[1], xs[2], xs[3]);
}

template <bool TAPER>
__device__ __forceinline__ float iir_pass2_masked(float4 *__restrict__ w4, float z[NS], int own_lo, int own_hi,
                                                  int lim, int64_t t_lane, int64_t L, float h1, float h2) {
  const float tf0 = (float)t_lane, Lf = (float)L;
  float acc = 0.f;
#pragma unroll 3
  for (int q = 0; q < CH / 4; ++q) iir_pass2_group<TAPER, true>(w4, q, z, acc, own_lo, own_hi, lim, tf0, Lf, h1, h2);
  return acc;
}

// Band-pass section k of iir_pass2_group, one sample (same operations, same order).
__device__ __forceinline__ float bp_section(int k, float u, float z[NS]) {
  const float y = u + z[2 * k];
  z[2 * k] = fmaf(-kBpSecA[k][0], y, z[2 * k + 1]);
  z[2 * k + 1] = fmaf(-kBpSecA[k][1], y, -u);
  return y;
}

// One time-skewed step of the cascade: section k (KLO <= k <= KHI) works on sample n - k, its
// input p[k] being section k-1's output of the previous step, so the five section updates of a
// step are independent (a lone wave runs a dependent v_fma chain at ~1.7x the time per
// instruction of independent ones, tools/micro/dep_chain.hip).  Section 4's output feeds acc.
template <int KLO, int KHI>
__device__ __forceinline__ void bp_step(float x, float p[5], float z[NS], float &acc) {
#pragma unroll
  for (int k = KHI; k >= KLO; --k) {  // descending: p[k+1] is read before section k rewrites it
    const float y = bp_section(k, k == 0 ? x : p[k], z);
    if (k < 4) p[k + 1] = y;
    else acc = fmaf(y, y, acc);
  }
}

// Packed steady state of the skewed cascade (sections 1-4 as two float2 pairs: one
// v_pk_add_f32 and two v_pk_fma_f32 per pair instead of three scalar instructions per section;
// section 0 and the pre-emphasis stay scalar).  Per element the same operations in the same
// order as bp_step<0, 4> + pre_step, so the outputs are bitwise those of the scalar form.
// The pairs are sections (1, 3) and (2, 4): the skewed cascade's next inputs are then (y0, y2)
// and (y1, y3) = the (1, 3) outputs themselves, so only y2 moves between register pairs (pairs
// (1, 2), (3, 4) needed three moves per sample; 182 vs 195 VALU per 12 samples, 7.172 vs 7.199
// ms per joint call, profiles/r4_fa/).
typedef float pf2 __attribute__((ext_vector_type(2)));
struct Pk {
  pf2 zaA, zbA, zaB, zbB;  // A = sections (1, 3): (z[2], z[6]), (z[3], z[7]); B = (2, 4): (z[4], z[8]), (z[5], z[9])
  pf2 pA, pB;              // section inputs (p[1], p[3]), (p[2], p[4])
};
__device__ __forceinline__ void pk_load(Pk &q, const float z[NS], const float p[5]) {
  q.zaA = (pf2){z[2], z[6]};
  q.zbA = (pf2){z[3], z[7]};
  q.zaB = (pf2){z[4], z[8]};
  q.zbB = (pf2){z[5], z[9]};
  q.pA = (pf2){p[1], p[3]};
  q.pB = (pf2){p[2], p[4]};
}
__device__ __forceinline__ void pk_store(const Pk &q, float z[NS], float p[5]) {
  z[2] = q.zaA.x; z[6] = q.zaA.y; z[3] = q.zbA.x; z[7] = q.zbA.y;
  z[4] = q.zaB.x; z[8] = q.zaB.y; z[5] = q.zbB.x; z[9] = q.zbB.y;
  p[1] = q.pA.x; p[3] = q.pA.y; p[2] = q.pB.x; p[4] = q.pB.y;
}
// one step: sections 4..1 on their (older) samples, section 0 on x; section 4's output to acc
__device__ __forceinline__ void pk_step(float x, Pk &q, float z[NS], float &acc) {
  const pf2 na0_B = (pf2){-kBpSecA[2][0], -kBpSecA[4][0]}, na1_B = (pf2){-kBpSecA[2][1], -kBpSecA[4][1]};
  const pf2 na0_A = (pf2){-kBpSecA[1][0], -kBpSecA[3][0]}, na1_A = (pf2){-kBpSecA[1][1], -kBpSecA[3][1]};
  const pf2 yB = q.pB + q.zaB;  // (y2, y4)
  q.zaB = __builtin_elementwise_fma(na0_B, yB, q.zbB);
  q.zbB = __builtin_elementwise_fma(na1_B, yB, -q.pB);
  acc = fmaf(yB.y, yB.y, acc);
  const pf2 yA = q.pA + q.zaA;  // (y1, y3)
  q.zaA = __builtin_elementwise_fma(na0_A, yA, q.zbA);
  q.zbA = __builtin_elementwise_fma(na1_A, yA, -q.pA);
  const float y0 = bp_section(0, x, z);
  q.pA = (pf2){y0, yB.x};
  q.pB = yA;
}
__device__ __forceinline__ void skew_group_pk(float4 *__restrict__ w4, int q4, Pk &q, float z[NS], float &acc,
                                              float &h1, float &h2) {
  const float4 v = w4[q4];
  float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    pk_step(xs[c], q, z, acc);
    xs[c] = pre_step(xs[c], z, h1, h2);
  }
  w4[q4] = make_float4(xs[0], xs[1], xs[2], xs[3]);
}

// Unmasked: the owned power of a lane whose range boundaries lie at 0, P_HI, P_LO or CH.
// The cascade runs time-skewed (bp_step): bitwise the per-sample arithmetic and summation order
// of iir_pass2_group<false, false>, with four fill steps in group 0 and four drain steps after
// group CH/4-1; the power of group r is summed while group r+1 is filtered.
static_assert(P_HI >= 4, "group 0 lies in the first power part");
__device__ __forceinline__ float iir_pass2_split(float4 *__restrict__ w4, float z[NS], int own_lo, int own_hi,
                                                float h1, float h2) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  float p[5];
  {
    const float4 v = w4[0];
    float xs[4] = {v.x, v.y, v.z, v.w};
    bp_step<0, 0>(xs[0], p, z, a0);
    xs[0] = pre_step(xs[0], z, h1, h2);
    bp_step<0, 1>(xs[1], p, z, a0);
    xs[1] = pre_step(xs[1], z, h1, h2);
    bp_step<0, 2>(xs[2], p, z, a0);
    xs[2] = pre_step(xs[2], z, h1, h2);
    bp_step<0, 3>(xs[3], p, z, a0);
    xs[3] = pre_step(xs[3], z, h1, h2);
    w4[0] = make_float4(xs[0], xs[1], xs[2], xs[3]);
  }
  {
    Pk pq;  // steady state in packed form (measured 2.605 -> 2.552 ms per 2048-row front-end launch)
    pk_load(pq, z, p);
#pragma unroll
    for (int q = 1; q < P_HI / 4 + 1; ++q) skew_group_pk(w4, q, pq, z, a0, h1, h2);
#pragma unroll 3
    for (int q = P_HI / 4 + 1; q < P_LO / 4 + 1; ++q) skew_group_pk(w4, q, pq, z, a1, h1, h2);
#pragma unroll
    for (int q = P_LO / 4 + 1; q < CH / 4; ++q) skew_group_pk(w4, q, pq, z, a2, h1, h2);
    pk_store(pq, z, p);
  }
  bp_step<1, 4>(0.f, p, z, a2);
  bp_step<2, 4>(0.f, p, z, a2);
  bp_step<3, 4>(0.f, p, z, a2);
  bp_step<4, 4>(0.f, p, z, a2);
  const bool lo_in = own_lo <= 0, hi_in = own_hi >= CH;
  return (lo_in && hi_in) ? (a0 + a1) + a2
       : (own_lo == P_LO && hi_in) ? a2
       : (lo_in && own_hi == P_HI) ? a0
       : 0.f;
}

// Joint mode (fsem_pesq_stoi_f32): STOI's 16 -> 10 kHz resampler (BaseMetric.prepare_audio,
// base.py:19-20) runs on the same LDS tile, so the input is read from HBM once for both
// metrics.  Segment g owns 10 kHz outputs [g*OWN10, (g+1)*OWN10) (the last: up to the row's
// 10 kHz length), i.e. polyphase groups m = g*OWN/8 + j whose 28 taps x[8m - 10 + t] sit at
// tile[WARM - 10 + 8j + t]; same tap order as stoi_resample_vad16, so bitwise the same y10.
constexpr int OWN10 = OWN / 8 * 5;  // 7680
constexpr int TILE_PAD = 32;        // zeros after the tile: the last segment's final taps
static_assert(OWN % 8 == 0, "segments start on polyphase-group boundaries");
static_assert((WARM - 12) % 4 == 0, "16-byte aligned tap reads");

// The polyphase resampler as a matrix product on MFMA (v_mfma_f32_16x16x4_f32).  Three
// consecutive polyphase groups form a super-group: 24 inputs -> 15 outputs over 44 taps,
//   y[15 s + p] = sum_{t<44} x[24 s - 10 + t] * R[t][p],
//   R[t][p] = kRs16k10k[p % 5][t - 8 (p / 5)] (zero outside the 28 taps),
// so a wave step multiplies A = the tile's Hankel rows of 64 super-groups (4 MFMA tiles of 16,
// one tap per lane per K-step, read straight from the tile) by the constant B = R (11 K-steps
// x 16 columns, column 15 zero; one VGPR per K-step, loaded once per kernel).  The f32 MFMA is
// bit-for-bit a k-ordered fmaf chain and the zero taps add exact zeros, so every output is the
// scalar resampler's fmaf chain over t = 0..27: the 10 kHz rows stay bitwise those of
// stoi_resample_vad16.  The VALU stays free for the other workgroup on the SIMD.  Outputs are
// staged output-major in the wave's slice of the (then idle) exchange buffer and leave as
// aligned float4 stores.
constexpr int RS_KS = 11;                  // K-steps (44 taps)
constexpr int RS_TILES = 4;                // 16-super-group MFMA tiles per wave step
constexpr int RS_STAGE = RS_TILES * 16 * 15;  // outputs per wave step (960)
static_assert(4 * RS_STAGE <= XBUF && RS_STAGE == SCAN_A_WAVE, "resampler staging slices = scan buffer A slices");
static_assert(OWN10 % RS_STAGE == 0 && OWN10 / RS_STAGE == 8, "two wave steps per wave and segment");
// the last segment owns up to (TILE - WARM) * 5 / 8 outputs; the taps of its last super-group
// (x 0 coefficients included: a NaN there would poison the row) stay in the zeroed pad.  Rows
// past the outputs only feed their own (unstored) output rows.
static_assert(WARM - 10 + 24 * (((TILE - WARM) * 5 / 8 + 14) / 15 - 1) + 4 * RS_KS <= TILE + TILE_PAD,
              "tap reads of stored outputs stay in the tile");
struct RsMfmaB {
  float b[RS_KS][64];
};
constexpr RsMfmaB make_rs_b() {
  RsMfmaB t{};
  for (int ks = 0; ks < RS_KS; ++ks)
    for (int l = 0; l < 64; ++l) {
      const int k = 4 * ks + (l >> 4), p = l & 15, q = k - 8 * (p / 5);
      t.b[ks][l] = (p < 15 && q >= 0 && q < 28) ? kRs16k10k[p % 5][q] : 0.f;
    }
  return t;
}
__constant__ static const RsMfmaB kRsMfmaB = make_rs_b();

// With vrow (clean rows of the joint entry), the staged outputs also give the STOI VAD quarter
// sums of every complete 64-sample block (fsem_vad.h), so no kernel re-reads the 10 kHz rows for
// the frame energies.
__device__ __forceinline__ void resample_tile(const float *__restrict__ tile, int64_t o_lo, int64_t o_hi,
                                              float *__restrict__ yrow, float2 *__restrict__ vrow,
                                              float4 wa, float4 wb, const float rb[RS_KS],
                                              float *__restrict__ stage, int lane, int wave) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int nsg = (int)((o_hi - o_lo + 14) / 15);  // super-groups holding outputs
  const int row = lane & 15, kq = lane >> 4;
  for (int st = 0;; ++st) {
    const int s0 = 16 * RS_TILES * (4 * st + wave);  // first super-group of this wave step (uniform)
    if (s0 >= nsg) break;
    // A operand: lane (row, kq) holds x[24 s - 10 + 4 ks + kq] of super-group s = s0 + 16 tl + row;
    // super-groups past nsg read tile samples (zeros past the row end) and are never stored
    const float *__restrict__ a = tile + (WARM - 10) + 24 * (s0 + row) + kq;
    f4 c[RS_TILES];
#pragma unroll
    for (int tl = 0; tl < RS_TILES; ++tl) c[tl] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < RS_KS; ++ks) {
      float av[RS_TILES];
#pragma unroll
      for (int tl = 0; tl < RS_TILES; ++tl) av[tl] = a[24 * 16 * tl + 4 * ks];
#pragma unroll
      for (int tl = 0; tl < RS_TILES; ++tl) c[tl] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[tl], rb[ks], c[tl], 0, 0, 0);
    }
    // D layout: lane holds rows 4 kq + i (super-groups), column row (output phase p < 15)
    if (row < 15) {
#pragma unroll
      for (int tl = 0; tl < RS_TILES; ++tl)
#pragma unroll
        for (int i = 0; i < 4; ++i) stage[15 * (16 * tl + 4 * kq + i) + row] = c[tl][i];
    }
    wave_lds_fence();
    const int64_t ob = o_lo + 15 * (int64_t)s0;  // multiple of 64: aligned float4 stores, whole blocks
    const int n = (int)min((int64_t)RS_STAGE, o_hi - ob);
    const float4 *__restrict__ s4 = reinterpret_cast<const float4 *>(stage);
    if (vrow) {  // uniform: every lane runs every pass (the quarter sums shuffle over 16 lanes)
      for (int q0 = 0; 4 * q0 < n; q0 += 64) {
        const int q = q0 + lane;
        // reads past n stay inside xbuf (4 * 256 floats from the last wave's slice) and only
        // feed blocks that are not stored
        const float4 v = s4[q];
        if (4 * q + 3 < n) {
          reinterpret_cast<float4 *>(yrow + ob)[q] = v;
        } else {
          for (int c = 4 * q; c < n; ++c) yrow[ob + c] = stage[c];
        }
        const float e = vad_quarter(v, wa, wb, lane);
        if ((lane & 14) == 0 && 4 * (q & ~15) + 64 <= n)
          reinterpret_cast<float *>(vrow)[2 * ((ob >> 6) + (q >> 4)) + (lane & 1)] = e;
      }
    } else {
      for (int q = lane; 4 * q < n; q += 64) {
        if (4 * q + 3 < n) {
          reinterpret_cast<float4 *>(yrow + ob)[q] = s4[q];
        } else {
          for (int c = 4 * q; c < n; ++c) yrow[ob + c] = stage[c];
        }
      }
    }
    wave_lds_fence();
  }
}

// Persistent: workgroup w starts at item (signal, segment) w and takes its further items from a
// queue (one atomic per item, claimed an item ahead);
// each item's tile goes straight into LDS at its start (load_tile_lds).
// rng: the range bookkeeping in the workspace -- pexp [2B * nseg] (per-segment shifts, zeroed
// before the main pass), count [1], flags [2B] (zeroed), worklist [2B] of flagged signals.
// SAFE (JOINT = false only): process the worklist's signals' segments with range shifts.
template <bool JOINT, bool VARLEN, bool SAFE = false>
__global__ void __launch_bounds__(PT, 2)
    pesq_front(const float *__restrict__ ref, const float *__restrict__ deg, int64_t B, int64_t Lcap,
               int64_t ld, const int32_t *__restrict__ lens_arg, int F, int npseg, int nseg, int64_t nitems,
               float *__restrict__ bark, float *__restrict__ ppart, int *__restrict__ rng,
               float *__restrict__ y10, int64_t y_ld, float2 *__restrict__ vad, int64_t v_ld) {
  static_assert(!(SAFE && JOINT), "the SAFE pass redoes PESQ only");
  __shared__ __attribute__((aligned(16))) float tile[TILE + TILE_PAD];
  __shared__ __attribute__((aligned(16))) float xbuf[XBUF];
  __shared__ float red[8];
  // the scan's source for chunks before the tile's first: 12 zero states (written once)
  __shared__ __attribute__((aligned(16))) float zrow[NS];
  __shared__ int64_t next_item;  // the workgroup's next item (from the queue)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches)
  const int32_t *__restrict__ lens = VARLEN ? lens_arg : nullptr;  // uniform batches: no per-row lookups
  if (JOINT && tid < TILE_PAD) tile[TILE + tid] = 0.f;  // never rewritten
  if (tid < NS) zrow[tid] = 0.f;                        // never rewritten (first item's barriers)
  // ---- per-lane constants, loaded once
  float win[8];
  cf tw1[8], tw2[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) win[r] = kHann512[lane + 64 * r] * kPreB[0];  // x b0: pre_fir
  fft512_twiddles(lane, tw1, tw2);
  const int plane = (64 - lane) & 63;
  // Bark MFMA (v_mfma_f32_16x16x4_f32): wave w owns frame rows 16w..16w+15 of the segment and
  // all four 16-band tiles; B operand = fbank x correction.  Per lane (band 16 t + lane % 16,
  // bins 4 k + lane / 16 of K-step k) one bit per K-step of the tile's range says whether the
  // bin lies in the band: tiles 0, 1, 3 (5 + 11 + 5 steps) share one word, tile 2 (45 steps)
  // takes two.  B of step k = bcor & -(bit k): one bit-field extract and one AND.
  constexpr int K0a = kBarkTileK[0][0], K0b = kBarkTileK[0][1];
  constexpr int K1a = kBarkTileK[1][0], K1b = kBarkTileK[1][1];
  constexpr int K2a = kBarkTileK[2][0], K2b = kBarkTileK[2][1];
  constexpr int K3a = kBarkTileK[3][0], K3b = kBarkTileK[3][1];
  static_assert((K0b - K0a) + (K1b - K1a) + (K3b - K3a) <= 32 && K2b - K2a <= 64, "Bark band masks");
  uint32_t bm013_c = 0, bm2lo_c = 0, bm2hi_c = 0;
  uint32_t bcor_c[4];
  {
    int blo[4], bhi[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int band = 16 * t + (lane & 15);
      blo[t] = band < NBARK ? kBandEdge[band] : 0;
      bhi[t] = band < NBARK ? kBandEdge[band + 1] : 0;
      // x 0.25: the Hermitian split's 1/4 (exact power of two, so the same products as scaling
      // every bin before the GEMM, short of underflow)
      bcor_c[t] = __float_as_uint(band < NBARK ? 0.25f * kBarkCorr[band] : 0.f);
    }
    auto in = [&](int t, int k) {
      const int bin = 4 * k + (lane >> 4);
      return bin >= blo[t] && bin < bhi[t];
    };
    for (int k = K0a; k < K0b; ++k) bm013_c |= (uint32_t)in(0, k) << (k - K0a);
    for (int k = K1a; k < K1b; ++k) bm013_c |= (uint32_t)in(1, k) << (k - K1a + (K0b - K0a));
    for (int k = K3a; k < K3b; ++k) bm013_c |= (uint32_t)in(3, k) << (k - K3a + (K0b - K0a) + (K1b - K1a));
    for (int k = K2a; k < K2b; ++k) {
      if (k - K2a < 32) bm2lo_c |= (uint32_t)in(2, k) << (k - K2a);
      else bm2hi_c |= (uint32_t)in(2, k) << (k - K2a - 32);
    }
  }

  // VAD window quarters (joint entry): a wave step's chunk starts at 10 kHz sample
  // g * OWN10 + 960 (4 st + wave), i.e. at quarter block 120 g + 15 (4 st + wave), so the block
  // parity of this lane's group is (wave + lane / 16) & 1 for every step.  Loaded once: a
  // load inside the step would wait (vmcnt) for the step's own y10 stores.
  static_assert(OWN10 % 128 == 0 && RS_STAGE % 64 == 0 && (RS_STAGE / 64) % 2 == 1, "VAD block parity");
  static_assert(RS_STAGE % 15 == 0, "wave steps start on super-group boundaries");
  float4 vwa, vwb;
  vad_windows(lane, (wave + (lane >> 4)) & 1, vwa, vwb);
  float rsb[RS_KS];  // resampler MFMA B operand (this lane's column of R per K-step)
#pragma unroll
  for (int ks = 0; ks < RS_KS; ++ks) rsb[ks] = JOINT ? kRsMfmaB.b[ks][lane] : 0.f;

  int *__restrict__ const pexp = rng;
  int *__restrict__ const rcount = rng + 2 * B * nseg;
  // items past the first gridDim.x come from a queue (counter zeroed with the range bookkeeping):
  // a workgroup that becomes resident late (other kernels on its CU) takes fewer items
  unsigned int *__restrict__ const qcount = reinterpret_cast<unsigned int *>(rcount + 1);
  int *__restrict__ const rflag = rcount + 2;
  int *__restrict__ const rlist = rflag + 2 * B;
  // SAFE: the worklist's items (signal rlist[i / nseg], segment i % nseg); usually none
  const int64_t n_items = SAFE ? (int64_t)__builtin_amdgcn_readfirstlane(*rcount) * nseg : nitems;
  auto item_at = [&](int64_t i) {
    return SAFE ? (int64_t)rlist[i / nseg] * nseg + i % nseg : i;
  };
  bool prefetched = false;  // this item's tile load went out during the previous item's Bark phase
  for (int64_t item = blockIdx.x, item_next; item < n_items; item = item_next) {
    // the item after this one: claimed now (lane 0 of wave 0), published to the workgroup before
    // the next tile load (next_tile) or at the item's end; the SAFE pass strides statically
    unsigned int claim = 0;
    if (!SAFE && tid == 0) claim = atomicAdd(qcount, 1u);
    item_next = -1;
    auto take_next = [&]() {  // every thread; a barrier between the write and the reads
      if (tid == 0) next_item = SAFE ? item + gridDim.x : (int64_t)gridDim.x + claim;
      lds_barrier();
      item_next = uniform_i64(next_item);
    };
    const Item it = make_item(item_at(item), nseg, B, ld, Lcap, lens, ref, deg);
    const int64_t L = it.L;
    Geometry rg;  // this row's geometry (the launch's for uniform batches)
    if (VARLEN) {
      rg = geometry(L);
    } else {
      rg.F = F;
      rg.npseg = npseg;
      rg.nseg = nseg;
    }
    if (VARLEN && it.g >= rg.nseg) {  // segment past this row's end: no samples, no frames
      if (tid < 4) ppart[(it.s * nseg + it.g) * 4 + tid] = 0.f;
      if (prefetched) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // its unused tile load (ordered before the next)
      prefetched = false;
      take_next();
      lds_barrier();  // every thread has read next_item before it is rewritten
      continue;
    }
    STAMP(0);
    if (!prefetched) load_tile_lds(it, tid, tile);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's tile loads have landed
    if (JOINT && (L & 3) && it.tstart + TILE > L) {
      // the row ends in this tile: the resampler sees zeros past it (torchaudio pads,
      // base.py:20); only the float4 at floor4(L) holds samples past L (the rest is range-checked)
      lds_barrier();
      const int r = (int)(L & 3), q = (int)((L & ~(int64_t)3) - it.tstart);
      if (tid < 4 && tid >= r && q >= 0) tile[q + tid] = 0.f;
    }
    lds_barrier();
    STAMP(14);
    if (JOINT) {
      const int64_t L10 = (5 * L + 7) / 8;
      const int64_t o_lo = (int64_t)it.g * OWN10;
      const int64_t o_hi = (it.g == rg.nseg - 1) ? L10 : min(L10, o_lo + OWN10);
      const int64_t b = it.s < B ? it.s : it.s - B;
      float2 *vrow = (vad && it.s < B) ? vad + b * v_ld : nullptr;  // clean rows only
      resample_tile(tile, o_lo, o_hi, y10 + (2 * b + (it.s < B ? 0 : 1)) * y_ld, vrow, vwa, vwb, rsb,
                    xbuf + RS_STAGE * wave, lane, wave);
      if (FSEM_DOUBLE == 1)
        resample_tile(tile, o_lo, o_hi, y10 + (2 * b + (it.s < B ? 0 : 1)) * y_ld, vrow, vwa, vwb, rsb,
                      xbuf + RS_STAGE * wave, lane, wave);
    }
    STAMP(1);
    const int g = it.g;
    const int64_t tstart = it.tstart;
    const float4 *__restrict__ my4 = reinterpret_cast<const float4 *>(tile + CH * tid);
    const int64_t t_lane = tstart + CH * tid;  // global index of this lane's first sample
    // lanes whose chunk meets the tapered edges (PESQ.py:108-109); wave-uniform fast path
    const bool edge = (t_lane < 15) || (t_lane + CH > L - 15 && t_lane < L);
    const bool wave_edge = __any(edge);

    // ---------------------------------------------------------------- IIR pass 1: end states
    // band-pass (untapered input, PESQ.py:94) and pre-emphasis (tapered, PESQ.py:108-111)
    // the two (tapered) samples before the chunk: the pre-emphasis FIR's history (zero at the
    // tile start, as the zero state there); read before pass 2 rewrites the tile in place
    float xm1 = 0.f, xm2 = 0.f, xr1 = 0.f;  // xr1: the raw x[-1] (the band-pass's history)
    if (tid > 0) {
      // an opaque index: the load vectoriser would otherwise chain this 8-byte load with the
      // chunk's float4 loads (passes 1 and 2) and split the chain at its 8-byte offset into
      // b96 / read2 pieces (more LDS instructions, 4-way bank conflicts)
      int hidx = CH * tid - 2;
      asm volatile("" : "+v"(hidx));
      const float2 hm = *reinterpret_cast<const float2 *>(tile + hidx);
      xm1 = xr1 = hm.y;
      xm2 = hm.x;
      if (__builtin_amdgcn_readfirstlane((int)wave_edge)) {
        xr1 = (t_lane - 1 >= L) ? 0.f : xr1;
        xm1 *= taper_w((float)(t_lane - 1), (float)L);
        xm2 *= taper_w((float)(t_lane - 2), (float)L);
      }
    }
    float e[NS];
    if (__builtin_amdgcn_readfirstlane((int)wave_edge))
      iir_pass1<true>(my4, t_lane, L, xm1, xm1 - xm2, xr1, e);
    else
      iir_pass1<false>(my4, t_lane, L, xm1, xm1 - xm2, xm1, e);
    if (FSEM_DOUBLE == 2) {
      const float4 *m2 = my4;
      asm volatile("" : "+v"(m2));
      float e2[NS];
      if (__builtin_amdgcn_readfirstlane((int)wave_edge))
        iir_pass1<true>(m2, t_lane, L, xm1, xm1 - xm2, xr1, e2);
      else
        iir_pass1<false>(m2, t_lane, L, xm1, xm1 - xm2, xm1, e2);
#pragma unroll
      for (int i = 0; i < NS; ++i) e[i] = (e[i] + e2[i]) * 0.5f;
    }
    // The tile's scale for its range shift (below): the peak magnitude of the chunks' end
    // states, which bound both filters' outputs -- the quantities squared from pass 2 on -- to
    // within the filters' gains (a factor ~100, far inside the shift's [2^-40, 2^40] window);
    // wave maxima, combined after the scan's first barrier.
    {
      float pk = 0.f;
#pragma unroll
      for (int i = 0; i < NS; ++i) pk = fmaxf(pk, fabsf(e[i]));
      pk = wave_max_pos(pk);
      if (SAFE) {
        if (lane == 0) red[wave] = pk;  // combined after the scan's first barrier
      } else if (lane == 0 && out_of_range(pk)) {
        // rare: put the signal on the SAFE pass's worklist (once)
        if (atomicExch(&rflag[it.s], 1) == 0) rlist[atomicAdd(rcount, 1)] = (int)it.s;
      }
    }
    STAMP(2);
    // ---------------------------------------------------------------- chunk scan (4 levels)
    // double-buffered (read one buffer, write the other): one barrier per level.  Buffer A at
    // 960 (tid / 64) + 13 (tid % 64) (inside the wave's own resampler staging slice), buffer B
    // at SCAN_B0 + 13 tid; levels 0..3 read A, B, A, B.
    auto scan_at = [&](bool in_b, int t) {
      return in_b ? xbuf + SCAN_B0 + t * SCAN_LD : xbuf + SCAN_A_WAVE * (t >> 6) + (t & 63) * SCAN_LD;
    };
    // the 12 states of a lane as three float4 words
    auto put_states = [&](float *dst) {
      float4 *d4 = reinterpret_cast<float4 *>(dst);
      d4[0] = make_float4(e[0], e[1], e[2], e[3]);
      d4[1] = make_float4(e[4], e[5], e[6], e[7]);
      d4[2] = make_float4(e[8], e[9], e[10], e[11]);
    };
    auto get_states = [&](const float *src, float q[NS]) {
      const float4 *s4 = reinterpret_cast<const float4 *>(src);
      const float4 a = s4[0], b = s4[1], c = s4[2];
      const float v[NS] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
      for (int i = 0; i < NS; ++i) q[i] = v[i];
    };
    put_states(scan_at(false, tid));
    lds_barrier();
#pragma unroll
    for (int lv8 = 0; lv8 < (FSEM_DOUBLE == 3 ? 8 : 4); ++lv8) {
      const int lv = lv8 & 3;
      const int d = 1 << lv;
      float q[NS];
      // lanes without a chunk d back read the zero row (an address select instead of 12
      // multiplications by a 0/1 flag)
      get_states(tid >= d ? scan_at(lv & 1, tid - d) : zrow, q);
#pragma unroll
      for (int i = 0; i < NBP; ++i) {
        float acc = e[i];
        // the cascade's transition is block lower-triangular: section i/2 sees sections <= i/2
#pragma unroll
        for (int k = 0; k < 2 * (i / 2) + 2; ++k) acc = fmaf(kBpScan[lv][i][k], q[k], acc);
        e[i] = acc;
      }
      {
        const float p0 = fmaf(kPreScan[lv][0][0], q[NBP], fmaf(kPreScan[lv][0][1], q[NBP + 1], e[NBP]));
        const float p1 = fmaf(kPreScan[lv][1][0], q[NBP], fmaf(kPreScan[lv][1][1], q[NBP + 1], e[NBP + 1]));
        e[NBP] = p0;
        e[NBP + 1] = p1;
      }
      put_states(scan_at(!(lv & 1), tid));
      lds_barrier();
    }
    // start state of chunk j = inclusive prefix of chunk j-1 (level 3 wrote buffer A)
    float z[NS];
    {
      get_states(tid >= 1 ? scan_at(false, tid - 1) : zrow, z);
      // pre-emphasis: scan basis (u, v) -> direct-form states (y[n-1], y[n-2]) (gen_tables.py)
      const float u = z[NBP], v = z[NBP + 1];
      z[NBP] = fmaf(kPreToY[0][0], u, kPreToY[0][1] * v);
      z[NBP + 1] = fmaf(kPreToY[1][0], u, kPreToY[1][1] * v);
    }
    // The tile's range shift (uniform, 0 for every tile whose peak lies in [2^-40, 2^40]).
    // Pass 1 and the scan are linear and range-safe; squares (the band-pass power, |X|^2) come
    // from pass 2 on, so a shifted tile scales its start states, the filters' history and its
    // own chunk here -- exact powers of two, no barrier (pass 2 reads only the lane's chunk).
    int sh = 0;
    if (SAFE) {
      sh = __builtin_amdgcn_readfirstlane(range_shift(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
      if (tid == 0) pexp[it.s * nseg + it.g] = sh;
    }
    if (SAFE && sh != 0) {
#pragma unroll
      for (int i = 0; i < NS; ++i) z[i] = __builtin_amdgcn_ldexpf(z[i], sh);
      xm1 = __builtin_amdgcn_ldexpf(xm1, sh);
      xm2 = __builtin_amdgcn_ldexpf(xm2, sh);
      float4 *c4 = reinterpret_cast<float4 *>(tile + CH * tid);
#pragma unroll 1
      for (int q = 0; q < CH / 4; ++q) {
        const float4 v = c4[q];
        c4[q] = make_float4(__builtin_amdgcn_ldexpf(v.x, sh), __builtin_amdgcn_ldexpf(v.y, sh),
                            __builtin_amdgcn_ldexpf(v.z, sh), __builtin_amdgcn_ldexpf(v.w, sh));
      }
    }
    STAMP(3);

    // ---------------------------------------------------------------- IIR pass 2
    {
      const int64_t own_len = (g == rg.nseg - 1) ? L - (int64_t)g * OWN : min((int64_t)OWN, L - (int64_t)g * OWN);
      const int own_lo = WARM - CH * tid, own_hi = WARM + (int)own_len - CH * tid;  // chunk-local
      const int lim = (int)min((int64_t)CH, max((int64_t)0, L - t_lane));       // y = 0 from here
      float4 *w4 = reinterpret_cast<float4 *>(tile + CH * tid);
      float acc;
      // per-sample masks only where a lane's owned range is cut elsewhere than at the split
      // points (a row's last segment) or the row ends inside the chunk
      const bool split_ok = (own_lo <= 0 || own_lo == P_LO || own_lo >= CH) &&
                            (own_hi >= CH || own_hi == P_HI || own_hi <= 0) && lim >= CH;
      if (__builtin_amdgcn_readfirstlane((int)wave_edge))
        acc = iir_pass2_masked<true>(w4, z, own_lo, own_hi, lim, t_lane, L, xm1, xm1 - xm2);
      else if (__builtin_amdgcn_readfirstlane((int)__all(split_ok)))
        acc = iir_pass2_split(w4, z, own_lo, own_hi, xm1, xm1 - xm2);
      else
        acc = iir_pass2_masked<false>(w4, z, own_lo, own_hi, lim, t_lane, L, xm1, xm1 - xm2);
      if (FSEM_DOUBLE == 5) {  // again over the (rewritten) chunk, from the same start state
        float z2[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) z2[i] = z[i] * 0.5f;
        acc += __builtin_amdgcn_readfirstlane((int)__all(split_ok)) && !__builtin_amdgcn_readfirstlane((int)wave_edge)
                   ? iir_pass2_split(w4, z2, own_lo, own_hi, xm1, xm1 - xm2)
                   : iir_pass2_masked<false>(w4, z2, own_lo, own_hi, lim, t_lane, L, xm1, xm1 - xm2);
      }
      // per-wave partials (no workgroup barrier); pesq_power_sum adds them in a fixed order
      const float tot = wave_sum_dpp(acc);
      if (lane == 0) ppart[(it.s * nseg + g) * 4 + wave] = tot * (kBpGain * kBpGain);
    }
    lds_barrier();
    STAMP(4);

    // ---------------------------------------------------------------- FFT rounds
    const int nfr = min(NF, rg.F - g * NF);  // valid frames in this segment
    float2 *wbuf = reinterpret_cast<float2 *>(xbuf) + wave * kFftBuf;
    const int nrounds = nfr > 0 ? (nfr + 7) / 8 : 0;
    // the 12 distinct tile samples of a frame pair (frame a: [0, 512), frame b: [256, 768))
    auto load_pair = [&](int fa, float o[12]) {
      const float *fra = tile + WARM + 256 * fa;  // in the tile for every fa < 2 (4 * 6)
#pragma unroll
      for (int r = 0; r < 12; ++r) o[r] = fra[lane + 64 * r];
    };
    auto power_split = [&](const cf v[8], float *qa, float *qb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float mr = __shfl(v[7 - r].r, plane, 64);
        float mi = __shfl(v[7 - r].i, plane, 64);
        if (lane == 0) {
          mr = v[(8 - r) & 7].r;
          mi = v[(8 - r) & 7].i;
        }
        typedef float f2v __attribute__((ext_vector_type(2)));
        const f2v z = {v[r].r, v[r].i}, m = {mr, mi};
        const f2v sm = z + m;
        const f2v df = z.yx - m.yx;
        const f2v pp = __builtin_elementwise_fma(sm, sm, df * df);
        qa[r] = pp.x;
        qb[r] = pp.y;
      }
      if (lane == 0) {
        qa[0] = 0.f;
        qb[0] = 0.f;
      }
    };
    auto window = [&](const float c[12], cf v[8]) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        typedef float f2v __attribute__((ext_vector_type(2)));
        const f2v w2 = (f2v){c[r], c[r + 4]} * (f2v){win[r], win[r]};
        v[r] = {w2.x, w2.y};
      }
    };
    // Rounds of 8 frames (one frame pair per wave) in chunks of two rounds: each wave transforms
    // its two pairs of a chunk together (fft512_wave_x2: one pair's butterflies beside the other's
    // LDS exchange, one exchange area), GR = 2 chunks per barrier.  Their spectra are held (16
    // values per lane) until every wave has read the tile for them, then parked in the consumed
    // part of the tile, below the next chunks' inputs.  (Round 6: the front end 4.389 -> 4.329 ms
    // against one pair at a time with the next pair's samples read ahead; reading the next chunk
    // ahead here spills VGPRs and loses 1.5 %, profiles/r6_g/.)
    constexpr int GR = 2;
    static_assert(SPEC_LD * 8 * 2 * GR <= WARM + 256 * 8 * 2 * GR, "parking below the next rounds' inputs");
    const int nchunk = (nrounds + 1) / 2;
    // chunks k < nchunk <= 3 read rounds <= 5, inside the tile (as the RPB = 3 plan's reads)
    static_assert(WARM + 256 * (2 * (4 * 5 + 3)) + 768 <= TILE + TILE_PAD && NF / 8 <= 6, "chunk reads in the tile");
    auto load_chunk = [&](int k, float (*c)[12]) {
#pragma unroll
      for (int h = 0; h < 2; ++h) load_pair(2 * (4 * (2 * k + h) + wave), c[h]);
    };
    for (int k0 = 0; k0 < nchunk; k0 += GR) {
      float pa[2 * GR][4], pb[2 * GR][4];
#pragma unroll
      for (int q = 0; q < GR; ++q) {
        const int k = k0 + q;
        if (k >= nchunk) break;  // wave-uniform
        const int f0 = 2 * (4 * (2 * k) + wave), f1 = 2 * (4 * (2 * k + 1) + wave);
        float cc[2][12];
        load_chunk(k, cc);
        cf v0[8], v1[8];
        window(cc[0], v0);
        window(cc[1], v1);
        if (f1 < nfr) {
          fft512_wave_x2(v0, v1, wbuf, lane, tw1, tw2);
          if (FSEM_DOUBLE == 4) fft512_wave_x2(v0, v1, wbuf, lane, tw1, tw2);
          power_split(v0, pa[2 * q], pb[2 * q]);
          power_split(v1, pa[2 * q + 1], pb[2 * q + 1]);
        } else if (f0 < nfr) {
          fft512_wave(v0, wbuf, lane, tw1, tw2);
          power_split(v0, pa[2 * q], pb[2 * q]);
        }
      }
      lds_barrier();  // every wave is done reading the tile for these rounds
      STAMP(6 + k0);
#pragma unroll
      for (int h = 0; h < 2 * GR; ++h) {
        const int fa = 2 * (4 * (2 * k0 + h) + wave);
        if (fa < nfr) {
          float *ra = tile + SPEC_LD * fa;
          float *rb = ra + SPEC_LD;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ra[lane + 64 * r] = pa[h][r];
            rb[lane + 64 * r] = pb[h][r];
          }
        }
      }
    }
    lds_barrier();
    STAMP(13);

    // ---------------------------------------------------------------- Bark bands on MFMA
    // Work split over the four waves (K-steps of v_mfma_f32_16x16x4_f32): waves 0-2 take frame
    // tile f = wave with band tiles 2 (45 steps) and 0 (5); wave 3 takes band tiles 1 (11) and
    // 3 (5) of all three frame tiles -- 50 / 48 MFMAs per wave instead of 66 on three waves.
    {
      typedef float f4 __attribute__((ext_vector_type(4)));
      const int row = lane & 15, kq = lane >> 4;
      // opaque copies: keep the B-operand extracts inside the item loop (else LICM hoists
      // them all into live VGPRs across the whole kernel)
      uint32_t bm013 = bm013_c, bm2lo = bm2lo_c, bm2hi = bm2hi_c, bcor[4];
      asm volatile("" : "+v"(bm013), "+v"(bm2lo), "+v"(bm2hi));
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bcor[t] = bcor_c[t];
        asm volatile("" : "+v"(bcor[t]));
      }
      // B operand of K-step bit `bit` of mask word w: bcor where the bit is set, else +0
      auto bop = [](uint32_t w, int bit, uint32_t cor) {
        return __uint_as_float(cor & (uint32_t)__builtin_amdgcn_sbfe((int)w, bit, 1));
      };
      // band-major output rows (bark_ld): lane (row, kq) of frame tile f holds frames
      // 16 f + 4 kq + i of one band -- one aligned float4 per band row
      const int64_t fld = bark_ld(F);
      float *__restrict__ bsig = bark + (int64_t)it.s * NBARK * fld + (int64_t)g * NF;
      auto put4 = [&](int band, int fl, f4 v) {
        float *o = bsig + band * fld + fl;
        if (fl + 3 < nfr) {
          *reinterpret_cast<f4 *>(o) = v;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (fl + i < nfr) o[i] = v[i];
        }
      };
      // The tile is free once every wave has read its last A operands: the next item's tile
      // load goes out then, before the last MFMA batch and the stores (which cover part of its
      // latency).  Waves 0-2 hold tile 2's last 29 K-steps across the barrier, wave 3 frame tile 2.
      auto next_tile = [&]() {
        take_next();  // (its barrier: every wave holds its remaining operands, the tile may be rewritten)
        prefetched = false;
        if (item_next < n_items) {
          const Item nit = make_item(item_at(item_next), nseg, B, ld, Lcap, lens, ref, deg);
          load_tile_lds(nit, tid, tile);
          prefetched = true;
        }
      };
      if (wave < 3) {
        constexpr int KB1 = 16, KR = (K2b - K2a) - KB1;  // tile 2: first batch, the rest
        const bool act = 16 * wave < nfr;
        // operands read and MFMAs run unconditionally (rows clamped into the tile; results of a
        // frame tile past nfr are not stored): no partially defined registers across the barrier
        const float *srow = tile + SPEC_LD * min(16 * wave + row, max(nfr, 1) - 1);
        f4 c0 = {0.f, 0.f, 0.f, 0.f}, c2a = c0, c2b = c0;
        auto mf2 = [&](int j, float a) {
          const float bv = j < 32 ? bop(bm2lo, j, bcor[2]) : bop(bm2hi, j - 32, bcor[2]);
          if (j & 1)
            c2b = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, c2b, 0, 0, 0);
          else
            c2a = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, c2a, 0, 0, 0);
        };
        float ar[KR];
        {
          // A operand: the wave's 16 spectrum rows, one bin per lane per K-step; a batch's LDS
          // reads are issued before its MFMA chain (the chain then never waits on LDS latency)
          float a0[K0b - K0a], a2[KB1];
#pragma unroll
          for (int k = 0; k < K0b - K0a; ++k) a0[k] = srow[4 * (K0a + k) + kq];
#pragma unroll
          for (int k = 0; k < KB1; ++k) a2[k] = srow[4 * (K2a + k) + kq];
#pragma unroll
          for (int k = 0; k < K0b - K0a; ++k)
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[k], bop(bm013, k, bcor[0]), c0, 0, 0, 0);
#pragma unroll
          for (int k = 0; k < KR; ++k) ar[k] = srow[4 * (K2a + KB1 + k) + kq];
#pragma unroll
          for (int k = 0; k < KB1; ++k) mf2(k, a2[k]);
        }
        next_tile();
#pragma unroll
        for (int k = 0; k < KR; ++k) mf2(KB1 + k, ar[k]);
        if (act) {
          put4(row, 16 * wave + 4 * kq, c0);
          put4(32 + row, 16 * wave + 4 * kq, c2a + c2b);
        }
      } else {
        f4 c1[3], c3[3];
#pragma unroll
        for (int f = 0; f < 3; ++f) {
          c1[f] = (f4){0.f, 0.f, 0.f, 0.f};
          c3[f] = c1[f];
        }
        // three frame tiles = three independent accumulator chains per band tile
        float a1[3][K1b - K1a], a3[3][K3b - K3a];
        auto rd = [&](int f) {
          const float *srow = tile + SPEC_LD * min(16 * f + row, max(nfr, 1) - 1);
#pragma unroll
          for (int k = 0; k < K1b - K1a; ++k) a1[f][k] = srow[4 * (K1a + k) + kq];
#pragma unroll
          for (int k = 0; k < K3b - K3a; ++k) a3[f][k] = srow[4 * (K3a + k) + kq];
        };
        auto mf = [&](int f) {
#pragma unroll
          for (int k = 0; k < K1b - K1a; ++k)
            c1[f] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[f][k], bop(bm013, k + (K0b - K0a), bcor[1]), c1[f], 0, 0, 0);
#pragma unroll
          for (int k = 0; k < K3b - K3a; ++k)
            c3[f] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                a3[f][k], bop(bm013, k + (K0b - K0a) + (K1b - K1a), bcor[3]), c3[f], 0, 0, 0);
        };
#pragma unroll
        for (int f = 0; f < 3; ++f) rd(f);
        mf(0);
        mf(1);
        next_tile();
        mf(2);
#pragma unroll
        for (int f = 0; f < 3; ++f) {
          if (16 * f < nfr) {
            put4(16 + row, 16 * f + 4 * kq, c1[f]);
            if (row == 0) put4(48, 16 * f + 4 * kq, c3[f]);
          }
        }
      }
    }
    STAMP(15);
    if (item_next < 0) {  // no Bark phase ran (uniform)
      take_next();
      lds_barrier();
    }
  }
}

// Stage entry (fsem_pesq_front_f32): per-signal power sums of the partials, each segment's
// range shift undone (an unrepresentable power becomes inf, as its true value would).
__global__ void __launch_bounds__(256) pesq_power_sum(const float *__restrict__ ppart, const int *__restrict__ pexp,
                                                      int nseg, int64_t nsig, float *__restrict__ power) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsig) return;
  float acc = 0.f;
  for (int g = 0; g < 4 * nseg; ++g) acc += __builtin_amdgcn_ldexpf(ppart[s * nseg * 4 + g], -2 * pexp[s * nseg + g / 4]);
  power[s] = acc;
}

// Stage entry: the Bark bands of range-shifted segments back to the input's scale: one thread
// per (signal, segment), which returns at once unless that segment was shifted (the common case:
// the launch costs a read of the shift array).
__global__ void __launch_bounds__(256) pesq_bark_unshift(float *__restrict__ bark, const int *__restrict__ pexp,
                                                         int nseg, int64_t nsig, int F) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsig * nseg) return;
  const int sh = pexp[i];
  if (sh == 0) return;
  const int64_t s = i / nseg;
  const int g = (int)(i - s * nseg);
  const int64_t fld = bark_ld(F);
  const int f0 = g * NF, f1 = min(F, f0 + NF);
  for (int k = 0; k < NBARK; ++k)
    for (int f = f0; f < f1; ++f) {
      float *p = bark + (s * NBARK + k) * fld + f;
      *p = __builtin_amdgcn_ldexpf(*p, -2 * sh);
    }
}

// Stage entry (fsem_pre_emphasize_f32): the pre-emphasis IIR of PESQ.pre_emphasize (PESQ.py:111)
// as torchaudio's lfilter evaluates it -- FIR part over the zero-padded input (taps oldest
// first), then the sequential all-pole loop acc = w - y[n-2] a2 - y[n-1] a1 -- with the
// roundings written out (no contraction), so each output is the torchaudio-order float32 value.
// One thread per row: a stage method off the scoring path (the scoring front end runs the same
// filter time-parallel, pesq_front pass 2).
__global__ void __launch_bounds__(64) pesq_pre_emphasis(const float *__restrict__ x, int64_t rows, int64_t L,
                                                        int64_t ld, float *__restrict__ y, int64_t ld_out) {
#pragma clang fp contract(off)  // every product rounded on its own, as the C loop
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float *__restrict__ xr = x + r * ld;
  float *__restrict__ yr = y + r * ld_out;
  const float b0 = kPreB[2], b1 = kPreB[1], b2 = kPreB[0];  // flipped taps: x[n-2], x[n-1], x[n]
  const float a2 = kPreA[2] / kPreA[0], a1 = kPreA[1] / kPreA[0];
  float x1 = 0.f, x2 = 0.f, y1 = 0.f, y2 = 0.f;
  for (int64_t n = 0; n < L; ++n) {
    const float x0 = xr[n];
    float w = b0 * x2;
    w = w + b1 * x1;
    w = w + b2 * x0;
    w = w / kPreA[0];
    float acc = w - y2 * a2;
    acc = acc - y1 * a1;  // (the loop's last term, the unwritten zero slot x a_flip[2] = 1, adds -0)
    yr[n] = acc;
    x2 = x1;
    x1 = x0;
    y2 = y1;
    y1 = acc;
  }
}

}  // namespace pesq
}  // namespace fsem

using namespace fsem;

extern "C" int fsem_pesq_frames(int64_t length) { return pesq::frames_of(length); }

extern "C" int fsem_pre_emphasize_f32(const float *x, int64_t rows, int64_t length, int64_t ld, float *y,
                                      int64_t ld_out, void *stream) {
  if (!x || !y || rows <= 0 || length <= 0 || ld < length || ld_out < length || length > kMaxLength) return FSEM_EINVAL;
  hipLaunchKernelGGL(pesq::pesq_pre_emphasis, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, (hipStream_t)stream, x,
                     rows, length, ld, y, ld_out);
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}

#ifdef FSEM_STAMPS
// diagnostic build only (not part of include/fsem.h)
extern "C" int fsem_debug_read_stamps(void *dst, size_t bytes) {
  if (hipDeviceSynchronize() != hipSuccess) return FSEM_ELAUNCH;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(pesq::g_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? FSEM_OK : FSEM_ELAUNCH;
}
#endif

// range bookkeeping after the partials: pexp [2B nseg], count, item queue, flags [2B], worklist [2B] (int)
static size_t front_rng_ints(int64_t batch, int64_t length) {
  return (size_t)(2 * batch) * (size_t)pesq::geometry(length).nseg + 2 + 4 * (size_t)batch;
}

extern "C" size_t fsem_pesq_front_workspace_bytes(int64_t batch, int64_t length) {
  return pesq::front_ppart_bytes(batch, length) + align_up(sizeof(int) * front_rng_ints(batch, length), 256);
}

extern "C" size_t fsem_pesq_workspace_bytes(int64_t batch, int64_t length) {
  const pesq::Geometry g = pesq::geometry(length);
  size_t bytes = fsem_pesq_front_workspace_bytes(batch, length);
  bytes += align_up(sizeof(float) * (size_t)(2 * batch) * pesq::NBARK * (size_t)pesq::bark_ld(g.F), 256);  // bark
  bytes += align_up(sizeof(float) * (size_t)(2 * batch), 256);                               // power
  bytes += fsem_pesq_back_workspace_bytes(batch, length);                                     // back
  return bytes;
}

int fsem::pesq::launch_front(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld,
                             const int32_t *lengths, float *bark, float *power, void *ws, size_t ws_bytes,
                             float *y10, int64_t y_ld, float2 *vad, int64_t v_ld, hipStream_t st,
                             bool power_sums) {
  if (!ref || !deg || !bark || (power_sums && !power) || batch <= 0 || length <= 0 || ld < length || length > kMaxLength)
    return FSEM_EINVAL;
  const pesq::Geometry g = pesq::geometry(length);
  if (g.F < 20 && !lengths) return FSEM_ESHORT;
  if (ws_bytes < fsem_pesq_front_workspace_bytes(batch, length) || !ws) return FSEM_EWORKSPACE;
  const int64_t nitems = 2 * batch * (int64_t)g.nseg;
  const int ncu = cu_count();
  // 2 resident workgroups per CU; FSEM_FRONT_WGS_PER_CU (diagnostics only) overrides
  static const int wgs_per_cu = [] {
    const char *e = getenv("FSEM_FRONT_WGS_PER_CU");
    const int v = e ? atoi(e) : 0;
    return (v >= 1 && v <= 2) ? v : 2;
  }();
  // FSEM_FRONT_CUS (diagnostics only: tools/ab_overlap.py's partitioned grid) caps the CUs the
  // persistent grid is sized for, leaving the rest to kernels on other streams
  static const int front_cus = [] {
    const char *e = getenv("FSEM_FRONT_CUS");
    return e ? atoi(e) : 0;
  }();
  const int64_t cus = (front_cus > 0 && front_cus < ncu) ? front_cus : ncu;
  const int64_t grid = std::min<int64_t>(nitems, cus * wgs_per_cu);
  float *ppart = static_cast<float *>(ws);
  int *rng = reinterpret_cast<int *>(static_cast<char *>(ws) + pesq::front_ppart_bytes(batch, length));
  int *pexp = rng;
  // shifts, worklist count, item queue and flags start at zero (the worklist itself is written
  // before read); the size rounded up to 16 bytes (inside the 256-aligned region) so the runtime
  // fills it with one kernel instead of an aligned body and a tail
  if (hipMemsetAsync(rng, 0, align_up(sizeof(int) * ((size_t)(2 * batch) * g.nseg + 2 + 2 * (size_t)batch), 16), st) !=
      hipSuccess)
    return FSEM_ELAUNCH;
#define FSEM_FRONT(J, V, S)                                                                                      \
  hipLaunchKernelGGL((pesq::pesq_front<J, V, S>), dim3((unsigned)grid), dim3(pesq::PT), 0, st, ref, deg, batch,  \
                     length, ld, lengths, g.F, g.npseg, g.nseg, nitems, bark, ppart, rng, y10, y_ld, vad, v_ld)
  if (y10) {
    if (lengths) FSEM_FRONT(true, true, false);
    else FSEM_FRONT(true, false, false);
  } else {
    if (lengths) FSEM_FRONT(false, true, false);
    else FSEM_FRONT(false, false, false);
  }
  FSEM_CHECK_LAUNCH();
  // the range-safe pass over the flagged signals (an empty worklist: every workgroup exits at once)
  if (lengths) FSEM_FRONT(false, true, true);
  else FSEM_FRONT(false, false, true);
#undef FSEM_FRONT
  FSEM_CHECK_LAUNCH();
  if (!power_sums) return FSEM_OK;  // the back end sums the partials itself
  // stage entry: the bands and powers at the input's own scale (include/fsem.h)
  hipLaunchKernelGGL(pesq::pesq_power_sum, dim3((unsigned)((2 * batch + 255) / 256)), dim3(256), 0, st,
                     ppart, pexp, g.nseg, 2 * batch, power);
  FSEM_CHECK_LAUNCH();
  const int64_t nb = 2 * batch * g.nseg;
  hipLaunchKernelGGL(pesq::pesq_bark_unshift, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st, bark, pexp,
                     g.nseg, 2 * batch, g.F);
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}

extern "C" int fsem_pesq_front_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                                   int64_t ld, const int32_t *lengths, float *bark, float *power, void *ws,
                                   size_t ws_bytes, void *stream) {
  return pesq::launch_front(ref, deg, batch, length, ld, lengths, bark, power, ws, ws_bytes, nullptr, 0, nullptr,
                            0, (hipStream_t)stream);
}

extern "C" int fsem_pesq_front_y10_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                                       int64_t ld, const int32_t *lengths, float *bark, float *power, float *y10,
                                       int64_t y_ld, float *vad, int64_t vad_ld, void *ws, size_t ws_bytes,
                                       void *stream) {
  if (!y10 || y_ld < (5 * length + 7) / 8 || (y_ld & 3)) return FSEM_EINVAL;
  if (vad && vad_ld < fsem::vad_ld((5 * length + 7) / 8)) return FSEM_EINVAL;
  return pesq::launch_front(ref, deg, batch, length, ld, lengths, bark, power, ws, ws_bytes, y10, y_ld,
                            reinterpret_cast<float2 *>(vad), vad_ld, (hipStream_t)stream);
}

hipStream_t fsem::side_stream(hipStream_t st) {
  constexpr int kMaxDev = 64;
  static std::mutex mu;
  static hipStream_t side[kMaxDev] = {};
  int cur = 0;
  hipDevice_t dev = 0;
  if (hipGetDevice(&cur) != hipSuccess || hipStreamGetDevice(st, &dev) != hipSuccess) return st;
  // created on the current device only; a stream of another device keeps its work on one stream
  if (dev != cur || dev < 0 || dev >= kMaxDev) return st;
  std::lock_guard<std::mutex> lock(mu);
  if (!side[dev] && hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking) != hipSuccess) {
    side[dev] = nullptr;
    return st;
  }
  return side[dev];
}

namespace {
// The join events of one host thread, one per device, released when the thread exits
// (errors ignored: at process exit the runtime may already be gone).
struct ThreadEvents {
  static constexpr int kMaxDev = 64;
  hipEvent_t ev[kMaxDev] = {};
  ~ThreadEvents() {
    for (hipEvent_t &e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};
}  // namespace

int fsem::stream_wait(hipStream_t waiter, hipStream_t producer) {
  if (waiter == producer) return FSEM_OK;
  // One event per (host thread, device), recorded anew for every edge.  This relies on the
  // HIP (as CUDA) snapshot semantics of hipStreamWaitEvent: a wait waits for the record that is
  // the event's most recent one WHEN THE WAIT IS ENQUEUED, so re-recording the event for the
  // next edge (possibly on another stream) does not move an earlier wait.  No other thread
  // records this event.
  thread_local ThreadEvents tev;
  hipEvent_t *ev = tev.ev;
  hipDevice_t dev = 0;
  if (hipStreamGetDevice(producer, &dev) != hipSuccess || dev < 0 || dev >= ThreadEvents::kMaxDev) return FSEM_ELAUNCH;
  if (!ev[dev]) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return FSEM_ELAUNCH;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return FSEM_ELAUNCH;
    const bool made = hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming) == hipSuccess;
    if (cur != dev) (void)hipSetDevice(cur);
    if (!made) {
      ev[dev] = nullptr;
      return FSEM_ELAUNCH;
    }
  }
  const bool ok = hipEventRecord(ev[dev], producer) == hipSuccess && hipStreamWaitEvent(waiter, ev[dev], 0) == hipSuccess;
  return ok ? FSEM_OK : FSEM_ELAUNCH;
}

int fsem::cu_count() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cache[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  n = 256;
  (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

// Workspace of the whole-metric entry: [front partials | bark | power | back scratch].
struct WbWs {
  size_t front;
  float *bark, *power;
  char *back;
};
static WbWs carve_wb(void *ws, int64_t batch, int64_t length) {
  const pesq::Geometry g = pesq::geometry(length);
  WbWs w;
  char *p = static_cast<char *>(ws);
  w.front = fsem_pesq_front_workspace_bytes(batch, length);
  w.bark = reinterpret_cast<float *>(p + w.front);
  p += w.front + align_up(sizeof(float) * (size_t)(2 * batch) * pesq::NBARK * (size_t)pesq::bark_ld(g.F), 256);
  w.power = reinterpret_cast<float *>(p);
  p += align_up(sizeof(float) * (size_t)(2 * batch), 256);
  w.back = p;
  return w;
}

int fsem::pesq::run_wb_front(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld,
                             const int32_t *lengths, void *ws, size_t ws_bytes, float *y10, int64_t y_ld,
                             float2 *vad, int64_t v_ld, hipStream_t stream) {
  if (!ref || !deg || batch <= 0 || length <= 0 || ld < length || length > kMaxLength) return FSEM_EINVAL;
  const pesq::Geometry g = pesq::geometry(length);
  if (g.F < 20 && !lengths) return FSEM_ESHORT;
  if (!ws || ws_bytes < fsem_pesq_workspace_bytes(batch, length)) return FSEM_EWORKSPACE;
  const WbWs w = carve_wb(ws, batch, length);
  return pesq::launch_front(ref, deg, batch, length, ld, lengths, w.bark, w.power, ws, w.front, y10, y_ld, vad,
                            v_ld, stream, /*power_sums=*/false);
}

int fsem::pesq::run_wb_back(int64_t batch, int64_t length, const int32_t *lengths, float *mos, void *ws,
                            hipStream_t back_st) {
  if (!mos) return FSEM_EINVAL;
  const WbWs w = carve_wb(ws, batch, length);
  // the front end's per-segment power partials sit at the start of the workspace (launch_front)
  return pesq::launch_back(w.bark, nullptr, static_cast<const float *>(ws), batch, length, lengths, mos, w.back,
                           fsem_pesq_back_workspace_bytes(batch, length), back_st);
}

int fsem::pesq::run_wb(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld,
                       const int32_t *lengths, float *mos, void *ws, size_t ws_bytes, float *y10, int64_t y_ld,
                       float2 *vad, int64_t v_ld, hipStream_t stream, hipStream_t back_st) {
  if (!mos) return FSEM_EINVAL;
  int rc = run_wb_front(ref, deg, batch, length, ld, lengths, ws, ws_bytes, y10, y_ld, vad, v_ld, stream);
  if (rc != FSEM_OK) return rc;
  rc = stream_wait(back_st, stream);
  if (rc != FSEM_OK) return rc;
  return run_wb_back(batch, length, lengths, mos, ws, back_st);
}

extern "C" int fsem_pesq_wb_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                                int64_t ld, const int32_t *lengths, float *mos, void *ws, size_t ws_bytes,
                                void *stream) {
  return pesq::run_wb(ref, deg, batch, length, ld, lengths, mos, ws, ws_bytes, nullptr, 0, nullptr, 0,
                       (hipStream_t)stream, (hipStream_t)stream);
}

// The whole-metric path with the back end's intermediates (ABI 10): the front end with its range
// handling (no host-side row scaling, which the stage entries need), then the back end's
// distances and per-frame disturbances beside the scores.
extern "C" int fsem_pesq_wb_frames_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                                       int64_t ld, const int32_t *lengths, float *mos, float *dist, float *frames,
                                       void *ws, size_t ws_bytes, void *stream) {
  if (!mos || !dist || !frames) return FSEM_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int rc = pesq::run_wb_front(ref, deg, batch, length, ld, lengths, ws, ws_bytes, nullptr, 0, nullptr, 0, st);
  if (rc != FSEM_OK) return rc;
  const WbWs w = carve_wb(ws, batch, length);
  return pesq::launch_back(w.bark, nullptr, static_cast<const float *>(ws), batch, length, lengths, mos, w.back,
                           fsem_pesq_back_workspace_bytes(batch, length), st, dist, frames);
}
