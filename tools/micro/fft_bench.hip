// Microbenchmark: 512-point complex FFT forms on gfx950, frames read from an LDS tile, two real
// frames per complex FFT, power split, spectra parked in LDS (the pesq_front FFT round).
//   A  fft512_wave: one FFT per wave, 8 points per lane, radix-8 x 3, two LDS exchanges, mirror
//      shuffles for the power split (the engine's form)
//   B  16 lanes per FFT (4 per wave), 32 points per lane: DFT-32 in registers, twiddle, one LDS
//      exchange, two DFT-16 in registers; the lane holds bins k and -k (no mirror shuffles)
// Also checks B against A numerically.  Usage: ./fft_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../../fast_speech_enhancement_metrics_amd/csrc/fsem_fft.h"

using namespace fsem;

constexpr int TILEN = 768 + 17 * 256;  // 16 frames

template <int N>
__device__ __forceinline__ f2 wc(int m) {  // W_N^m
  const int i = ((512 / N) * m) & 511;
  return (f2){kTwRe[i], kTwIm[i]};
}

__device__ __forceinline__ void dft4v(f2 &x0, f2 &x1, f2 &x2, f2 &x3) {
  const f2 pm = {1.f, -1.f}, mp = {-1.f, 1.f};
  const f2 a = x0 + x2, b = x0 - x2, c = x1 + x3, d = x1 - x3;
  x0 = a + c;
  x2 = a - c;
  x1 = FSEM_FMA2(d.yx, pm, b);  // b - i d
  x3 = FSEM_FMA2(d.yx, mp, b);  // b + i d
}

__device__ __forceinline__ void dft16v(f2 v[16]) {
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) dft4v(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
#pragma unroll
  for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1) v[4 * k1 + n2] = cmul2(v[4 * k1 + n2], wc<16>(n2 * k1));
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) dft4v(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
  f2 o[16];
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) o[k1 + 4 * k2] = v[4 * k1 + k2];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = o[k];
}

__device__ __forceinline__ void dft32v(f2 v[32]) {
  f2 t[4][8];
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) t[n2][n1] = v[4 * n1 + n2];
    dft8v(t[n2]);
  }
#pragma unroll
  for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1) t[n2][k1] = cmul2(t[n2][k1], wc<32>(n2 * k1));
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1) dft4v(t[0][k1], t[1][k1], t[2][k1], t[3][k1]);
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1)
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) v[k1 + 8 * k2] = t[k2][k1];
}

constexpr int G16_LD = 17;                 // exchange row stride (float2): conflict-free reads
constexpr int G16_BUF = 16 * G16_LD;       // per group (two phases of 16 rows)
constexpr int G16_GRP = G16_BUF + 16;      // group stride; odd groups start 16 float2 later (banks)
constexpr int G16_WAVE = 4 * G16_GRP + 16;  // per wave

__device__ __forceinline__ void fft512_g16(f2 v[32], float2 *buf, int l, const f2 tw[32], f2 s0[16], f2 s1[16]) {
  dft32v(v);
#pragma unroll
  for (int k1 = 1; k1 < 32; ++k1) v[k1] = cmul2(v[k1], tw[k1]);
  const int k1a = l == 15 ? 0 : l + 1, k1b = l == 15 ? 16 : 31 - l;
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
#pragma unroll
    for (int k = 0; k < 16; ++k) buf[G16_LD * k + l] = make_float2(v[16 * ph + k].x, v[16 * ph + k].y);
    wave_lds_fence();
    const float2 *ra = buf + G16_LD * (ph ? k1b - 16 : k1a);
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) {
      const float2 p = ra[n2];
      if (ph) s1[n2] = (f2){p.x, p.y};
      else s0[n2] = (f2){p.x, p.y};
    }
    wave_lds_fence();
  }
  dft16v(s0);
  dft16v(s1);
}

template <int OCC>
__global__ void __launch_bounds__(256, OCC) kA(float *out, int iters, int check) {
  __shared__ __attribute__((aligned(16))) float tile[TILEN];
  __shared__ __attribute__((aligned(16))) float2 xb[4 * kFftBuf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < TILEN; i += 256) tile[i] = __sinf(0.01f * i + blockIdx.x) + 0.001f * (i % 7);
  __syncthreads();
  float win[8];
  cf tw1[8], tw2[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) win[r] = kHann512[lane + 64 * r];
  fft512_twiddles(lane, tw1, tw2);
  const int plane = (64 - lane) & 63;
  float2 *wbuf = xb + wave * kFftBuf;
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    const int fa = 2 * (4 * (it & 1) + wave);
    cf v[8];
    const float *fra = tile + 768 + 256 * fa;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int n = lane + 64 * r;
      v[r] = {fra[n] * win[r], fra[256 + n] * win[r]};
    }
    fft512_wave(v, wbuf, lane, tw1, tw2);
    float pa[4], pb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mr = __shfl(v[7 - r].r, plane, 64);
      float mi = __shfl(v[7 - r].i, plane, 64);
      if (lane == 0) {
        mr = v[(8 - r) & 7].r;
        mi = v[(8 - r) & 7].i;
      }
      const float zr = v[r].r, zi = v[r].i;
      pa[r] = 0.25f * fmaf(zr + mr, zr + mr, (zi - mi) * (zi - mi));
      pb[r] = 0.25f * fmaf(zi + mi, zi + mi, (zr - mr) * (zr - mr));
    }
    if (lane == 0) pa[0] = pb[0] = 0.f;
    __syncthreads();
    // park (row stride 258) in the consumed part of the tile
    float *ra = tile + 258 * (fa & 15), *rb = ra + 258;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ra[lane + 64 * r] = pa[r];
      rb[lane + 64 * r] = pb[r];
    }
    if (check && it == 0 && blockIdx.x == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        out[(2 * wave) * 256 + lane + 64 * r] = pa[r];
        out[(2 * wave + 1) * 256 + lane + 64 * r] = pb[r];
      }
    }
    acc += pa[0];
    __syncthreads();
  }
  if (!check) out[blockIdx.x * 256 + tid] = acc;
}

template <int OCC, int TWL, int WINL = 0>
__global__ void __launch_bounds__(256, OCC) kB(float *out, int iters, int check) {
  __shared__ __attribute__((aligned(16))) float tile[TILEN];
  __shared__ __attribute__((aligned(16))) float2 xb[4 * G16_WAVE];
  __shared__ float2 twl[16][32];
  __shared__ float hwin[512];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l = lane & 15, g = lane >> 4;
  for (int i = tid; i < TILEN; i += 256) tile[i] = __sinf(0.01f * i + blockIdx.x) + 0.001f * (i % 7);
  for (int i = tid; i < 512; i += 256) {
    const int ll = i >> 5, k = i & 31;
    twl[ll][k] = make_float2(kTwRe[(ll * k) & 511], kTwIm[(ll * k) & 511]);
    hwin[i] = kHann512[i];
  }
  __syncthreads();
  float win[32];
  f2 tw[32];
#pragma unroll
  for (int n1 = 0; n1 < 32; ++n1) {
    win[n1] = WINL ? 0.f : kHann512[16 * n1 + l];
    const int i = (l * n1) & 511;
    tw[n1] = TWL ? (f2){0.f, 0.f} : (f2){kTwRe[i], kTwIm[i]};
  }
  float2 *gbuf = xb + wave * G16_WAVE + g * G16_GRP + (g & 1) * 16;
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    // 4 FFTs per wave: frames 2 (4 wave + g) + {0, 1} of round it % 6 / 4 (same tile offsets as A over 4 iters)
    const int fa = 8 * (wave & 1) + 2 * g;
    f2 v[32];
    const float *fra = tile + 768 + 256 * fa;
#pragma unroll
    for (int n1 = 0; n1 < 32; ++n1) {
      const int n = 16 * n1 + l;
      const float w = WINL ? hwin[n] : win[n1];
      v[n1] = (f2){fra[n] * w, fra[256 + n] * w};
    }
    f2 s0[16], s1[16];
    if (TWL) {
      f2 twr[32];
#pragma unroll
      for (int k = 1; k < 32; ++k) {
        const float2 t = twl[l][k];
        twr[k] = (f2){t.x, t.y};
      }
      fft512_g16(v, gbuf, l, twr, s0, s1);
    } else {
      fft512_g16(v, gbuf, l, tw, s0, s1);
    }
    // power split: bin k = k1a + 32 j (slot 0, j) pairs with -k = (slot 1, 15 - j); lane 15:
    // slot 0 bins 32 j (pairs j, 16 - j), slot 1 bins 16 + 32 j (pairs j, 15 - j)
    const bool l15 = l == 15;
    const int k1a = l15 ? 0 : l + 1;
    float pa[16], pb[16];
    int bin[16];
    (void)bin;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      f2 z, m;
      if (j < 8) {
        z = s0[j];
        m = l15 ? s0[(16 - j) & 15] : s1[15 - j];
      } else {
        z = l15 ? s1[j - 8] : s0[j];
        m = l15 ? s1[15 - (j - 8)] : s1[15 - j];
      }
      pa[j] = 0.25f * fmaf(z.x + m.x, z.x + m.x, (z.y - m.y) * (z.y - m.y));
      pb[j] = 0.25f * fmaf(z.y + m.y, z.y + m.y, (z.x - m.x) * (z.x - m.x));
    }
    if (l15) pa[0] = pb[0] = 0.f;
    __syncthreads();
    float *ra = tile + 258 * fa, *rb = ra + 258;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int bj = j < 8 ? (l15 ? 32 * j : k1a + 32 * j) : (l15 ? 16 + 32 * (j - 8) : (31 - l) + 32 * (15 - j));
      ra[bj] = pa[j];
      rb[bj] = pb[j];
    }
    if (check && it == 0 && blockIdx.x == 0 && wave == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int bj = j < 8 ? (l15 ? 32 * j : k1a + 32 * j) : (l15 ? 16 + 32 * (j - 8) : (31 - l) + 32 * (15 - j));
        out[8192 + (2 * g) * 256 + bj] = pa[j];
        out[8192 + (2 * g + 1) * 256 + bj] = pb[j];
      }
    }
    acc += pa[3];
    __syncthreads();
  }
  if (!check) out[blockIdx.x * 256 + tid] = acc;
}

static size_t g_dyn = 0;
template <typename K>
static float run(K kern, int blocks, float *out, int iters) {
  hipFuncAttributes at;
  hipFuncGetAttributes(&at, (const void *)kern);
  const size_t dyn = g_dyn > at.sharedSizeBytes ? g_dyn - at.sharedSizeBytes : 0;
  hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
  printf("  [static LDS %zu B, dyn %zu B, VGPR-limited regs %d]\n", at.sharedSizeBytes, dyn, at.numRegs);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), dyn, 0, out, 4, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), dyn, 0, out, iters, 0);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float *out;
  hipMalloc(&out, sizeof(float) * 256 * ncu * 8 + 65536);
  // numerics: B's frames 0..7 of wave 0 (iteration 0) vs A's (frames 2 (4 w) + {0,1}, w = 0..3)
  hipMemset(out, 0, 65536 * 4);
  hipLaunchKernelGGL((kA<2>), dim3(1), dim3(256), 0, 0, out, 1, 1);
  hipLaunchKernelGGL((kB<2, 1, 1>), dim3(1), dim3(256), 0, 0, out, 1, 1);
  hipDeviceSynchronize();
  std::vector<float> h(65536);
  hipMemcpy(h.data(), out, 65536 * 4, hipMemcpyDeviceToHost);
  double md = 0, mx = 0;
  for (int f = 0; f < 8; ++f)
    for (int k = 0; k < 256; ++k) {
      md = fmax(md, fabs(h[f * 256 + k] - h[8192 + f * 256 + k]));
      mx = fmax(mx, fabs(h[f * 256 + k]));
    }
  printf("check: max |A - B| = %.3g (max |A| = %.3g)\n", md, mx);
  const int iters = 600;
  for (int per_cu : {2, 3, 4}) {
    g_dyn = per_cu == 2 ? 80 * 1024 : per_cu == 3 ? 53 * 1024 : 40 * 1024;
    const int blocks = ncu * per_cu * 4;
    const double ffts_a = (double)blocks * 4 * iters, ffts_b = (double)blocks * 16 * iters;
    float ta = run(kA<2>, blocks, out, iters);
    float tb = run(kB<2, 1, 0>, blocks, out, iters);
    float tc = run(kB<2, 1, 1>, blocks, out, iters);
    printf("blocks/CU %d: A %.3f ms = %.4f ns/FFT(chip)  B(lds tw) %.3f ms = %.4f ns/FFT  B(lds tw+win) %.3f ms = %.4f ns/FFT\n",
           per_cu, ta, ta * 1e6 / ffts_a, tb, tb * 1e6 / ffts_b, tc, tc * 1e6 / ffts_b);
  }
  return 0;
}
