// Microbenchmark: issue rate of v_fma_f32 vs v_pk_fma_f32 on gfx950 (independent chains).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(256) k(float *out, int iters) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  float a[16];
  f2 p[8];
  const float s = threadIdx.x * 1e-7f;
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = s + i;
#pragma unroll
  for (int i = 0; i < 8; ++i) p[i] = (f2){s + i, s - i};
  const f2 m = (f2){1.0000001f, 0.9999999f};
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(1.0000001f), "v"(1e-9f));
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(m), "v"(m));
    }
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += a[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) r += p[i].x + p[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float *out;
  hipMalloc(&out, sizeof(float) * 256 * ncu * 16);
  const int iters = 20000;
  for (int wpsimd : {1, 2, 4}) {
    const int blocks = ncu * wpsimd;  // 256-thread blocks: one wave per SIMD each
    for (int mode = 0; mode < 2; ++mode) {
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 10);
      else hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 10);
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
      else hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      // per SIMD: wpsimd waves x iters x (16 instr) ; FMAs per lane: 16 per iter either way
      const double instr = (double)iters * (mode == 0 ? 16 : 8) * wpsimd;
      const double cyc = ms * 1e-3 * 2.4e9;
      const double flops = 2.0 * 16 * iters * 256.0 * blocks / (ms * 1e-3);
      printf("waves/SIMD %d %-11s: %.3f ms  %.2f cycles/instr/SIMD  %.1f TFLOP/s\n", wpsimd,
             mode == 0 ? "v_fma_f32" : "v_pk_fma_f32", ms, cyc / instr, flops / 1e12);
    }
  }
  return 0;
}
