// Which XCD runs which workgroup?  Prints the histogram of (blockIdx % 8) -> XCC_ID for a
// large grid, to check the round-robin dispatch assumption behind the XCD-sliced SpMV.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void probe(unsigned* out, int spin) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (threadIdx.x == 0) out[blockIdx.x] = xcc & 0xF;
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(1);
}
int main() {
  const int nb = 65536;
  unsigned* d;
  hipMalloc(&d, nb * 4);
  for (int spin : {0, 100}) {
    hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 0, 0, d, spin);
    std::vector<unsigned> h(nb);
    hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost);
    int tab[8][16] = {};
    for (int b = 0; b < nb; ++b) tab[b % 8][h[b]]++;
    printf("spin %d: rows = blockIdx%%8, cols = XCC_ID 0..7\n", spin);
    for (int r = 0; r < 8; ++r) {
      for (int c = 0; c < 8; ++c) printf("%7d", tab[r][c]);
      printf("\n");
    }
    printf("first 24 blocks:");
    for (int b = 0; b < 24; ++b) printf(" %u", h[b]);
    printf("\n");
  }
  return 0;
}
