// ds_write_addtid_b32 addressing check: 4 waves, wave w stores w*100 + lane at base &buf[w][0].
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ void lds_store_lanes(float *base, float v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float *)base;
  uint32_t saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tds_write_addtid_b32 %1\n\ts_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(v), "s"(a) : "memory");
}
__global__ void k(float *out) {
  __shared__ float buf[8][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 512; i += 256) buf[i / 64][i % 64] = -1.f;
  __syncthreads();
  lds_store_lanes(&buf[wave][0], (float)(wave * 100 + lane));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the compiler does not track the asm store
  __syncthreads();
  for (int i = tid; i < 512; i += 256) out[i] = buf[i / 64][i % 64];
}
int main() {
  float *d, h[512];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 512; ++i) {
    const float want = i < 256 ? (float)((i / 64) * 100 + i % 64) : -1.f;
    if (h[i] != want) { if (bad < 8) printf("i=%d got %g want %g\n", i, h[i], want); ++bad; }
  }
  for (int r = 0; r < 8; ++r) printf("row %d: %g %g ... %g\n", r, h[64 * r], h[64 * r + 1], h[64 * r + 63]);
  printf("addtid: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
  return 0;
}
