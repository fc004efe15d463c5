// Micro-benchmark: does data a kernel has just WRITTEN come back faster than HBM when the next
// kernel reads it (is it held by the 256 MB memory-side cache)?  A writer kernel stores W
// bytes (plain or non-temporal 16-byte stores), a reader kernel then streams the same W bytes;
// the reader's rate for W well below / well above 256 MB tells.  Also: reading the same W bytes
// twice in a row (read-after-read).
// build: hipcc --offload-arch=gfx950 -O3 -o mall_probe mall_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NT>
__global__ __launch_bounds__(1024) void wr(uint32_t* __restrict__ a, uint64_t n) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += nth * 4) {
    u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(a + i));
    else *reinterpret_cast<u32x4*>(a + i) = v;
  }
}
__global__ __launch_bounds__(1024) void rd(const uint32_t* __restrict__ a, uint64_t n, uint32_t* out) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; i < n; i += nth * 16) {
    const u32x4* p = reinterpret_cast<const u32x4*>(a + i);
    u32x4 c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = p[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc += c[q][0] ^ c[q][1] ^ c[q][2] ^ c[q][3];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t cap = 1ull << 30;  // 4 GiB of u32
  uint32_t *a, *o;
  if (hipMalloc(&a, cap * 4) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
  (void)hipMemset(a, 1, cap * 4);
  hipEvent_t e0, e1, e2;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventCreate(&e2);
  for (uint64_t mb : {32ull, 64ull, 128ull, 192ull, 256ull, 384ull, 512ull, 1024ull, 2048ull, 4096ull}) {
    const uint64_t n = mb * (1ull << 20) / 4;
    for (int nt = 0; nt < 2; ++nt) {
      float w = 0, r = 0, r2 = 0;
      for (int rep = 0; rep < 3; ++rep) {
        // evict: stream the far end of the buffer first when the window is small
        if (n * 2 <= cap) hipLaunchKernelGGL(rd, dim3(256), dim3(1024), 0, 0, a + cap / 2, cap / 2, o);
        (void)hipEventRecord(e0);
        if (nt) hipLaunchKernelGGL(wr<1>, dim3(256), dim3(1024), 0, 0, a, n);
        else hipLaunchKernelGGL(wr<0>, dim3(256), dim3(1024), 0, 0, a, n);
        (void)hipEventRecord(e1);
        hipLaunchKernelGGL(rd, dim3(256), dim3(1024), 0, 0, a, n, o);
        (void)hipEventRecord(e2);
        (void)hipEventSynchronize(e2);
        (void)hipEventElapsedTime(&w, e0, e1);
        (void)hipEventElapsedTime(&r, e1, e2);
        (void)hipEventRecord(e1);
        hipLaunchKernelGGL(rd, dim3(256), dim3(1024), 0, 0, a, n, o);
        (void)hipEventRecord(e2);
        (void)hipEventSynchronize(e2);
        (void)hipEventElapsedTime(&r2, e1, e2);
      }
      printf("%5llu MB %s stores: write %6.2f TB/s | read right after %6.2f TB/s | read again %6.2f TB/s\n",
             (unsigned long long)mb, nt ? "non-temporal" : "plain       ", n * 4.0 / w / 1e9,
             n * 4.0 / r / 1e9, n * 4.0 / r2 / 1e9);
    }
  }
  return 0;
}
