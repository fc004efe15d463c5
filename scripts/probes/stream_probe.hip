// Micro-benchmark: streaming-read rate of a u32 array with the stream kernel's access shape
// (per lane: NQ consecutive 16-byte loads; waves stride over 1024*NQ/4-element tasks).
// build: hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NQ, int NT>
__global__ __launch_bounds__(1024) void rd(const uint32_t* __restrict__ a, uint64_t n, uint32_t* out) {
  const uint64_t per = 4 * NQ;
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t base = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * per; base < n; base += nth * per) {
    const u32x4* p = reinterpret_cast<const u32x4*>(a + base);
    u32x4 c[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) c[q] = NT ? __builtin_nontemporal_load(p + q) : p[q];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc += c[q][0] ^ c[q][1] ^ c[q][2] ^ c[q][3];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t n = 1ull << 30;  // 4 GiB
  uint32_t *a, *o;
  if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
  (void)hipMemset(a, 1, n * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](auto kern, int wg, const char* name) {
    float ms = 0;
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(256 * wg), dim3(1024), 0, 0, a, n, o);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
    }
    printf("%-28s wg/cu %d  %7.3f ms  %6.2f TB/s\n", name, wg, ms, n * 4.0 / ms / 1e9);
  };
  for (int wg : {1, 2}) {
    run(rd<4, 1>, wg, "4 x dwordx4 nt");
    run(rd<4, 0>, wg, "4 x dwordx4");
    run(rd<8, 1>, wg, "8 x dwordx4 nt");
    run(rd<8, 0>, wg, "8 x dwordx4");
    run(rd<2, 0>, wg, "2 x dwordx4");
  }
  return 0;
}
