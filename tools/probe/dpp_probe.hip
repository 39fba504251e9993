// Probe: lane sources of permlane32/16_swap and DPP row_shl on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  int l = threadIdx.x;
  auto a = __builtin_amdgcn_permlane32_swap(l, l, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(l, l, false, false);
  o[l] = a[0]; o[64 + l] = a[1]; o[128 + l] = b[0]; o[192 + l] = b[1];
  o[256 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x101, 0xF, 0xF, false);
  o[320 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x108, 0xF, 0xF, false);
}
int main() {
  int* d; hipMalloc(&d, 384 * 4); hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
  int h[384]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[6] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]", "shl1", "shl8"};
  for (int t = 0; t < 6; t++) { printf("%s:", nm[t]); for (int l = 0; l < 64; l++) printf(" %d", h[t * 64 + l]); printf("\n"); }
  return 0;
}
