// Shared helpers of libfsem (gfx950 / CDNA4).  Wave size is 64 everywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fsem.h"

#define FSEM_WAVE 64

#define FSEM_CHECK_LAUNCH()                                    \
  do {                                                         \
    if (hipGetLastError() != hipSuccess) return FSEM_ELAUNCH;  \
  } while (0)

namespace fsem {

// Workgroup barrier that orders LDS only.  __syncthreads() also waits for every outstanding
// global load/store (vmcnt(0)), which would drain the next tile's prefetch at every barrier;
// kernels that communicate through LDS alone use this instead.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// A wave-uniform 64-bit value (e.g. read from LDS) moved to scalar registers.
__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// Sum over a 256-thread block (4 waves).  `scratch` >= 4 floats of LDS.  All threads get it.
__device__ __forceinline__ float block_sum_256(float v, float *scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  lds_barrier();
  if (lane == 0) scratch[w] = v;
  lds_barrier();
  return scratch[0] + scratch[1] + scratch[2] + scratch[3];
}

__device__ __forceinline__ double block_sum_256_d(double v, double *scratch) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  return scratch[0] + scratch[1] + scratch[2] + scratch[3];
}

__device__ __forceinline__ float block_max_256(float v, float *scratch) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(scratch[0], scratch[1]), fmaxf(scratch[2], scratch[3]));
}

// Compiler barrier for intra-wave LDS exchange (LDS ops of one wave complete in order).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wait for this wave's outstanding LDS stores (before other waves read the data).
__device__ __forceinline__ void lds_stores_done() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Longest row any entry accepts (input samples, and 10 / 16 kHz samples after resampling): the
// kernels address a row with 32-bit byte offsets (raw buffer loads, range-checked descriptors).
// 2^29 samples = 9.3 h at 16 kHz; longer rows give FSEM_EINVAL (include/fsem.h).
constexpr int64_t kMaxLength = int64_t(1) << 29;

// Launches that map rows (utterances) to grid.y cover at most kMaxGridY rows each; the host loops
// over slices [r0, r0 + kMaxGridY) and passes r0 (HIP's grid.y limit, hipDeviceProp maxGridSize[1]).
constexpr int64_t kMaxGridY = 65535;

}  // namespace fsem
