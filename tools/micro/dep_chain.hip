// Microbenchmark: cycles per dependent v_fma_f32 on gfx950 for C independent chains per wave
// (C = 1 is a pure dependency chain), at 1 and 2 waves per SIMD.  Tells whether a serial
// recursion (the IIR sections of pesq_front) is bound by VALU latency or by issue.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int C>
__global__ void __launch_bounds__(256) k(float *out, int iters) {
  float a[C];
  const float s = threadIdx.x * 1e-7f;
#pragma unroll
  for (int i = 0; i < C; ++i) a[i] = s + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16 / C; ++r)
#pragma unroll
      for (int i = 0; i < C; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(1.0000001f), "v"(1e-9f));
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < C; ++i) r += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int C>
static void run(int ncu, float *out, int wpsimd) {
  const int iters = 20000, blocks = ncu * wpsimd;
  hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(256), 0, 0, out, 10);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double per_wave_instr = (double)iters * 16;
  printf("waves/SIMD %d chains %2d: %.3f ms  %.2f ns per instr per wave (%.2f cycles @2.4GHz)\n", wpsimd, C, ms,
         ms * 1e6 / per_wave_instr, ms * 1e-3 * 2.4e9 / per_wave_instr);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float *out;
  hipMalloc(&out, sizeof(float) * 256 * ncu * 4);
  for (int w : {1, 2}) {
    run<1>(ncu, out, w);
    run<2>(ncu, out, w);
    run<4>(ncu, out, w);
    run<8>(ncu, out, w);
    run<16>(ncu, out, w);
  }
  return 0;
}
