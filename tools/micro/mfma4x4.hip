// Microbenchmark + layout probe: v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4, K = 1) on gfx950
// against v_mfma_f32_16x16x4_f32 -- the operand / result lane mapping, bitwise agreement with an
// fmaf chain, and the issue rate of independent chains (cycles per instruction per SIMD).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma4x4 tools/micro/mfma4x4.hip && /tmp/mfma4x4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

typedef float f4 __attribute__((ext_vector_type(4)));

// layout: A[l] = a(l), B[l] = b(l), C = 0 -> D[l][r] for every lane and register
__global__ void layout(const float *a, const float *b, float *d) {
  const int l = threadIdx.x;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[4 * l + r] = c[r];
}

// chain of K steps: C = mfma(A_k, B_k, C) vs fmaf(A_k, B_k, C) in the predicted lane mapping
__global__ void chain(const float *a, const float *b, int K, float *d) {
  const int l = threadIdx.x;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < K; ++k) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[64 * k + l], b[64 * k + l], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[4 * l + r] = c[r];
}

template <int MODE, int NCH>
__global__ void __launch_bounds__(256) rate(float *out, int iters, long long *cyc) {
  f4 c[NCH];
  const float s = threadIdx.x * 1e-7f;
  for (int i = 0; i < NCH; ++i) c[i] = (f4){s, s, s, s};
  float a = 1.0000001f + s, b = 0.9999999f;
  asm volatile("" : "+v"(a), "+v"(b));
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (MODE == 0)
        c[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[i], 0, 0, 0);
      else
        c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float r = 0.f;
  for (int i = 0; i < NCH; ++i) r += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float *a, *b, *d;
  hipMallocManaged(&a, sizeof(float) * 64 * 64);
  hipMallocManaged(&b, sizeof(float) * 64 * 64);
  hipMallocManaged(&d, sizeof(float) * 256);
  for (int l = 0; l < 64; ++l) {
    a[l] = (float)(l + 1);          // distinct small integers: products identify (A lane, B lane)
    b[l] = (float)(1000 * (l + 1));
  }
  hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, a, b, d);
  hipDeviceSynchronize();
  // predicted: lane l holds block q = l / 4, column j = l % 4, rows r: D = A[4q + r] * B[4q + j]
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int q = l / 4, j = l % 4;
      const float want = a[4 * q + r] * b[4 * q + j];
      if (d[4 * l + r] != want) {
        if (bad < 8) printf("layout: lane %d reg %d got %g want %g\n", l, r, d[4 * l + r], want);
        ++bad;
      }
    }
  printf("layout (lane l: block l/4, column l%%4, register r = row; A lane 4q+r, B lane 4q+j): %s\n",
         bad ? "MISMATCH" : "ok");
  // bitwise fmaf chain
  const int K = 64;
  unsigned s = 12345u;
  auto rnd = [&]() {
    s = s * 1664525u + 1013904223u;
    return (float)((s >> 8) & 0xffff) / 65536.f * ((s & 1) ? 1.f : 1e-3f);
  };
  for (int i = 0; i < 64 * K; ++i) {
    a[i] = rnd();
    b[i] = rnd();
  }
  hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, a, b, K, d);
  hipDeviceSynchronize();
  int nb = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int q = l / 4, j = l % 4;
      float c = 0.f;
      for (int k = 0; k < K; ++k) c = fmaf(a[64 * k + 4 * q + r], b[64 * k + 4 * q + j], c);
      if (d[4 * l + r] != c) ++nb;
    }
  printf("k-ordered fmaf chain (K = %d): %d of 256 results differ\n", K, nb);
  // rates
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float *out;
  long long *cyc;
  hipMalloc(&out, sizeof(float) * 256 * ncu);
  hipMallocManaged(&cyc, sizeof(long long));
  const int iters = 4000;
  auto run = [&](auto kern, const char *name, int nch, int per_iter_mfma) {
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(256), 0, 0, out, iters, cyc);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(256), 0, 0, out, iters, cyc);
    hipDeviceSynchronize();
    printf("%-22s chains %d: %.2f cycles per MFMA (one wave per SIMD)\n", name, nch,
           (double)*cyc / ((double)iters * per_iter_mfma));
  };
  run(rate<0, 1>, "4x4x1_16b f32", 1, 1);
  run(rate<0, 2>, "4x4x1_16b f32", 2, 2);
  run(rate<0, 4>, "4x4x1_16b f32", 4, 4);
  run(rate<1, 1>, "16x16x4 f32", 1, 1);
  run(rate<1, 4>, "16x16x4 f32", 4, 4);
  return 0;
}
