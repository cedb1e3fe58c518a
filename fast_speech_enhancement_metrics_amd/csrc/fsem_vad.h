// STOI voice-activity frame energies (STOI.py:92-99) from 64-sample quarter blocks.
//
// Frame i of a 10 kHz row y spans y[128 i, 128 i + 256) under W = hann(257)[1:]; its energy is
//   E(i) = ((Q(2i, 0) + Q(2i+1, 1)) + Q(2i+2, 2)) + Q(2i+3, 3),
//   Q(m, r) = sum_t (W[64 r + t] * y[64 m + t])^2,  t < 64,
// and the reference keeps frames with 20 log10(sqrt(E) + 1e-9) within 40 dB of the loudest.
// Each quarter block m serves two window quarters -- r = m & 1 (first half of frame m / 2 or
// (m - 1) / 2) and r = 2 + (m & 1) (second half) -- stored as vad[m] = {Q(m, m & 1),
// Q(m, 2 + (m & 1))}.  Q is evaluated in one fixed order everywhere: 16 lanes, lane k holding
// samples 4k .. 4k+3 (packed W^2 y^2 partial sums), then a fixed DPP butterfly over the 16
// lanes.  Every producer (the joint PESQ front end, the fused STOI resamplers, the 10 kHz
// path) goes through vad_quarter(),
// so the kept-frame decisions are bitwise the same on every path.  The reference sums a frame
// in torch's order; the difference is a few ulp of E, far below the 40 dB decision margin
// except for frames within ~1e-6 dB of the threshold.
#pragma once
#include "fsem_fft.h"

namespace fsem {

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Squared window quarters of the lane's 4 samples for a block of parity p:
// {W[64p + 4k + c]^2}, {W[128 + 64p + 4k + c]^2}, k = lane & 15.
__device__ __forceinline__ void vad_windows(int lane, int p, float4 &wa, float4 &wb) {
  const int k = 4 * (lane & 15) + 64 * p;
  wa = make_float4(kHann256s[k] * kHann256s[k], kHann256s[k + 1] * kHann256s[k + 1],
                   kHann256s[k + 2] * kHann256s[k + 2], kHann256s[k + 3] * kHann256s[k + 3]);
  wb = make_float4(kHann256s[k + 128] * kHann256s[k + 128], kHann256s[k + 129] * kHann256s[k + 129],
                   kHann256s[k + 130] * kHann256s[k + 130], kHann256s[k + 131] * kHann256s[k + 131]);
}

// Q of the block whose 64 samples sit as float4s on the 16 lanes of this lane's group (all 16
// active).  Lane k: packed {W^2 y^2} partial sums of its 4 samples; then the even lanes carry
// the first window quarter and the odd lanes the second through a DPP butterfly (lane ^ 1
// exchange, lane ^ 2, row rotations by 4 and 8).  Result: group lane 0 holds Q(m, m & 1),
// group lane 1 holds Q(m, 2 + (m & 1)); other lanes hold partial sums.
typedef float vad_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float vad_quarter(float4 y, float4 wa, float4 wb, int lane) {
  const vad_f2 ylo = {y.x, y.y}, yhi = {y.z, y.w};
  const vad_f2 y2lo = ylo * ylo, y2hi = yhi * yhi;
  const vad_f2 pa = __builtin_elementwise_fma((vad_f2){wa.x, wa.y}, y2lo, (vad_f2){wa.z, wa.w} * y2hi);
  const vad_f2 pb = __builtin_elementwise_fma((vad_f2){wb.x, wb.y}, y2lo, (vad_f2){wb.z, wb.w} * y2hi);
  const float sa = pa.x + pa.y, sb = pb.x + pb.y;
  const bool odd = lane & 1;
  float v = odd ? sb : sa;
  v += dpp_f32<0xB1>(odd ? sa : sb);  // quad_perm [1,0,3,2]: partner's value of my quarter
  v += dpp_f32<0x4E>(v);              // quad_perm [2,3,0,1]
  v += dpp_f32<0x124>(v);             // row_ror:4
  v += dpp_f32<0x128>(v);             // row_ror:8
  return v;
}

// Frame i's energy in dB from a row's quarter sums (STOI.py:92-99: 20 log10(||w frame|| + eps)).
__device__ __forceinline__ float vad_energy_db(const float2 *__restrict__ q, int i) {
  const float e = ((q[2 * i].x + q[2 * i + 1].x) + q[2 * i + 2].y) + q[2 * i + 3].y;
  return 20.f * log10f(sqrtf(e) + 1e-9f);
}

// Quarter blocks stored per row (row stride of the vad array, in float2): blocks 0 .. 2 NV + 1
// are the ones frames use, all inside the row's first L10 samples.
__host__ __device__ inline int64_t vad_ld(int64_t L10) { return ((L10 / 64 + 1) + 63) / 64 * 64; }

}  // namespace fsem
