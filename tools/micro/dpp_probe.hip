// Which source lane does each DPP control read?  out[c][lane] = source lane id.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL> __device__ int dpp(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }
__global__ void k(int *out) {
  const int lane = threadIdx.x;
  out[0 * 64 + lane] = dpp<0xB1>(lane);
  out[1 * 64 + lane] = dpp<0x4E>(lane);
  out[2 * 64 + lane] = dpp<0x124>(lane);
  out[3 * 64 + lane] = dpp<0x12C>(lane);
}
int main() {
  int h[256], *d;
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char *names[4] = {"quad_perm 0xB1", "quad_perm 0x4E", "row_ror 4", "row_ror 12"};
  for (int c = 0; c < 4; ++c) {
    printf("%-15s:", names[c]);
    for (int l = 0; l < 20; ++l) printf(" %d", h[c * 64 + l]);
    printf("\n");
  }
  return 0;
}
