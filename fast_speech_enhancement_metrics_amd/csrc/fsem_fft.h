// One-wave 512-point complex FFT (radix-8 Stockham) shared by the PESQ and STOI kernels.
#pragma once
#include "fsem_common.h"

namespace fsem {
#include "fsem_tables.inc"

struct cf {
  float r, i;
};
__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cf cmul(cf a, cf b) {
  return {fmaf(a.r, b.r, -a.i * b.i), fmaf(a.r, b.i, a.i * b.r)};
}
__device__ __forceinline__ cf mul_mi(cf a) { return {a.i, -a.r}; }  // a * (-i)

// In-register forward DFT of 8 points (radix-2 DIT, W8 = exp(-i pi/4)).
__device__ __forceinline__ void dft8(cf v[8]) {
  const float h = 0.70710678118654752f;
  cf a0 = cadd(v[0], v[4]), a1 = csub(v[0], v[4]);
  cf a2 = cadd(v[2], v[6]), a3 = mul_mi(csub(v[2], v[6]));
  cf a4 = cadd(v[1], v[5]), a5 = csub(v[1], v[5]);
  cf a6 = cadd(v[3], v[7]), a7 = mul_mi(csub(v[3], v[7]));
  cf b0 = cadd(a0, a2), b2 = csub(a0, a2), b1 = cadd(a1, a3), b3 = csub(a1, a3);
  cf c0 = cadd(a4, a6), c2 = csub(a4, a6), c1 = cadd(a5, a7), c3 = csub(a5, a7);
  cf w1c1 = {h * (c1.r + c1.i), h * (c1.i - c1.r)};    // c1 * (1 - i)/sqrt2
  cf w3c3 = {h * (c3.i - c3.r), -h * (c3.r + c3.i)};   // c3 * (-1 - i)/sqrt2
  cf mic2 = mul_mi(c2);
  v[0] = cadd(b0, c0);
  v[4] = csub(b0, c0);
  v[1] = cadd(b1, w1c1);
  v[5] = csub(b1, w1c1);
  v[2] = cadd(b2, mic2);
  v[6] = csub(b2, mic2);
  v[3] = cadd(b3, w3c3);
  v[7] = csub(b3, w3c3);
}

// LDS exchange area per wave: 512 float2, element i stored at fsw(i) = i ^ ((i >> 3) & 15).
// The XOR swizzle keeps all four access patterns bank-conflict-free under the gfx950 LDS
// lane-group rules (stage scatters 8*lane + r and o1 + 8r as ds_write_b64 in 16-lane groups,
// gathers lane + 64r as ds_read_b64 in 32-lane groups) without padding; the former i + i/8
// padding left 2-way conflicts on the gathers.
constexpr int kFftBuf = 512;
__device__ __forceinline__ int fpad(int i) { return i ^ ((i >> 3) & 15); }

// Packed-FP32 form of the butterflies: complex values as float2 vectors, so additions become
// v_pk_add_f32 and the multiplications by -i, (1-i)/sqrt2, (-1-i)/sqrt2 fold into v_pk_fma_f32
// with swapped operands (op_sel) -- on gfx950 one packed instruction costs the issue slot of
// one scalar one (tools/micro/valu_rate.hip: 2x the FP32 rate).  IEEE per element, so the
// arithmetic per element is that of the scalar form up to the fused multiply-adds.
typedef float f2 __attribute__((ext_vector_type(2)));
#define FSEM_FMA2 __builtin_elementwise_fma

__device__ __forceinline__ f2 cmul2(f2 a, f2 b) {  // a * b
  const f2 t = a.xx * b;
  return FSEM_FMA2(b.yx, (f2){-a.y, a.y}, t);
}

__device__ __forceinline__ void dft8v(f2 v[8]) {
  const f2 pm = {1.f, -1.f}, mp = {-1.f, 1.f};
  const float h = 0.70710678118654752f;
  const f2 hh = {h, h}, nh = {-h, -h};
  const f2 a0 = v[0] + v[4], a1 = v[0] - v[4];
  const f2 a2 = v[2] + v[6], d26 = v[2] - v[6];
  const f2 a4 = v[1] + v[5], a5 = v[1] - v[5];
  const f2 a6 = v[3] + v[7], d37 = v[3] - v[7];
  const f2 b0 = a0 + a2, b2 = a0 - a2;
  const f2 b1 = FSEM_FMA2(d26.yx, pm, a1), b3 = FSEM_FMA2(d26.yx, mp, a1);  // a1 -/+ i d26
  const f2 c0 = a4 + a6, c2 = a4 - a6;
  const f2 c1 = FSEM_FMA2(d37.yx, pm, a5), c3 = FSEM_FMA2(d37.yx, mp, a5);
  const f2 t1 = FSEM_FMA2(c1.yx, pm, c1);   // c1 (1 - i)
  const f2 t3 = FSEM_FMA2(c3.yx, pm, -c3);  // c3 (-1 - i)
  v[0] = b0 + c0;
  v[4] = b0 - c0;
  v[1] = FSEM_FMA2(t1, hh, b1);
  v[5] = FSEM_FMA2(t1, nh, b1);
  v[2] = FSEM_FMA2(c2.yx, pm, b2);  // b2 - i c2
  v[6] = FSEM_FMA2(c2.yx, mp, b2);
  v[3] = FSEM_FMA2(t3, hh, b3);
  v[7] = FSEM_FMA2(t3, nh, b3);
}

// dft8v for inputs whose upper half v[4..7] is zero (a frame zero-padded to twice its length,
// STOI's 256-sample window in a 512-point FFT): the first butterfly layer is the identity.
// Same values as dft8v except for the sign of exact zeros (v + 0 there).
__device__ __forceinline__ void dft8v_lo4(f2 v[8]) {
  const f2 pm = {1.f, -1.f}, mp = {-1.f, 1.f};
  const float h = 0.70710678118654752f;
  const f2 hh = {h, h}, nh = {-h, -h};
  const f2 b0 = v[0] + v[2], b2 = v[0] - v[2];
  const f2 b1 = FSEM_FMA2(v[2].yx, pm, v[0]), b3 = FSEM_FMA2(v[2].yx, mp, v[0]);
  const f2 c0 = v[1] + v[3], c2 = v[1] - v[3];
  const f2 c1 = FSEM_FMA2(v[3].yx, pm, v[1]), c3 = FSEM_FMA2(v[3].yx, mp, v[1]);
  const f2 t1 = FSEM_FMA2(c1.yx, pm, c1);
  const f2 t3 = FSEM_FMA2(c3.yx, pm, -c3);
  v[0] = b0 + c0;
  v[4] = b0 - c0;
  v[1] = FSEM_FMA2(t1, hh, b1);
  v[5] = FSEM_FMA2(t1, nh, b1);
  v[2] = FSEM_FMA2(c2.yx, pm, b2);
  v[6] = FSEM_FMA2(c2.yx, mp, b2);
  v[3] = FSEM_FMA2(t3, hh, b3);
  v[7] = FSEM_FMA2(t3, nh, b3);
}

// v[r] *= tw[r] for r = 1..7 as cmul2 in two sweeps: the seven products first, then the seven
// fused multiply-adds, so no v_pk_fma_f32 directly follows the v_pk_mul_f32 it reads (gfx950
// inserts a wait state between a packed-FP32 result and its packed reader: one s_nop per pair
// when the compiler keeps each pair together).  Same operations per element as cmul2.
__device__ __forceinline__ void twiddle7(f2 v[8], const cf tw[8]) {
  f2 t[8];
#pragma unroll
  for (int r = 1; r < 8; ++r) t[r] = v[r].xx * (f2){tw[r].r, tw[r].i};
#pragma unroll
  for (int r = 1; r < 8; ++r) v[r] = FSEM_FMA2((f2){tw[r].i, tw[r].r}, (f2){-v[r].y, v[r].y}, t[r]);
}

// 512-point complex FFT of one wave, radix-8 Stockham, natural-order result in
// v[r] = Z[lane + 64 r].  `buf` = this wave's kFftBuf-float2 LDS exchange area.
// LO4: Z[n] = 0 for n >= 256 (vc[4..7] are not read).
template <bool LO4 = false>
__device__ __forceinline__ void fft512_wave(cf vc[8], float2 *buf, int lane, const cf tw1[8],
                                            const cf tw2[8]) {
  f2 v[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = (f2){vc[r].r, vc[r].i};
  if (LO4)
    dft8v_lo4(v);
  else
    dft8v(v);
#pragma unroll
  for (int r = 0; r < 8; ++r) buf[fpad(8 * lane + r)] = make_float2(v[r].x, v[r].y);
  wave_lds_fence();
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    float2 t = buf[fpad(lane + 64 * r)];
    v[r] = (f2){t.x, t.y};
  }
  twiddle7(v, tw1);
  dft8v(v);
  wave_lds_fence();
  const int o1 = (lane >> 3) * 64 + (lane & 7);
#pragma unroll
  for (int r = 0; r < 8; ++r) buf[fpad(o1 + 8 * r)] = make_float2(v[r].x, v[r].y);
  wave_lds_fence();
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    float2 t = buf[fpad(lane + 64 * r)];
    v[r] = (f2){t.x, t.y};
  }
  twiddle7(v, tw2);
  dft8v(v);
  wave_lds_fence();
#pragma unroll
  for (int r = 0; r < 8; ++r) vc[r] = {v[r].x, v[r].y};
}


// Two 512-point FFTs of one wave through ONE exchange area, software-pipelined: each FFT's
// butterflies run while the other's exchange is in flight (one LDS round trip per exchange
// instead of two back-to-back FFTs' four each).  A wave's LDS operations execute in issue
// order, so a gather issued before the other FFT's scatter reads its data first (write after
// read within the wave); the fences wait for scatters before the gathers that read them.
// Results as two fft512_wave calls (the same operations per element, in the same order).
__device__ __forceinline__ void fft512_wave_x2(cf va[8], cf vb[8], float2 *buf, int lane, const cf tw1[8],
                                               const cf tw2[8]) {
  f2 a[8], b[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    a[r] = (f2){va[r].r, va[r].i};
    b[r] = (f2){vb[r].r, vb[r].i};
  }
  const int o1 = (lane >> 3) * 64 + (lane & 7);
  auto scatter1 = [&](const f2 *v) {
#pragma unroll
    for (int r = 0; r < 8; ++r) buf[fpad(8 * lane + r)] = make_float2(v[r].x, v[r].y);
  };
  auto scatter2 = [&](const f2 *v) {
#pragma unroll
    for (int r = 0; r < 8; ++r) buf[fpad(o1 + 8 * r)] = make_float2(v[r].x, v[r].y);
  };
  auto gather = [&](f2 *v) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float2 t = buf[fpad(lane + 64 * r)];
      v[r] = (f2){t.x, t.y};
    }
  };
  dft8v(a);
  scatter1(a);
  dft8v(b);  // beside A's first scatter
  wave_lds_fence();
  gather(a);
  scatter1(b);  // after A's gather in issue order
  twiddle7(a, tw1);
  dft8v(a);  // beside B's first scatter
  wave_lds_fence();
  gather(b);
  scatter2(a);
  twiddle7(b, tw1);
  dft8v(b);  // beside A's second scatter
  wave_lds_fence();
  gather(a);
  scatter2(b);
  twiddle7(a, tw2);
  dft8v(a);  // beside B's second scatter
  wave_lds_fence();
  gather(b);
  twiddle7(b, tw2);
  dft8v(b);
  wave_lds_fence();
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    va[r] = {a[r].x, a[r].y};
    vb[r] = {b[r].x, b[r].y};
  }
}

// Per-lane twiddles of stages 1 and 2: W512^(8 r (lane&7)) and W512^(r lane).
__device__ __forceinline__ void fft512_twiddles(int lane, cf tw1[8], cf tw2[8]) {
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int i1 = (8 * r * (lane & 7)) & 511;
    const int i2 = (r * lane) & 511;
    tw1[r] = {kTwRe[i1], kTwIm[i1]};
    tw2[r] = {kTwRe[i2], kTwIm[i2]};
  }
}

}  // namespace fsem
