// Placement probe 3: is device memory uniform?  Fills the device with 1-GB buffers and times a
// streaming read, a streaming write and a random 8-byte gather on each of them.
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/probes/region_probe scripts/probes/region_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, uint64_t n16, uint32_t* out) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += nth * 4) {
    u32x4 c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = i + q * nth < n16 ? a[i + q * nth] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) acc += c[q].x ^ c[q].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ a, uint64_t n16) {
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += nth)
    a[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}
__global__ __launch_bounds__(256) void k_gather(const double* __restrict__ a, uint64_t n8, uint32_t per, double* out) {
  uint64_t x = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B97F4A7C15ull + 12345;
  double s = 0;
  for (uint32_t k = 0; k < per; k += 8) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
      v[q] = a[x % n8];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  if (s == 1.2345) out[0] = s;
}
int main() {
  const size_t B = 1ull << 30;
  std::vector<void*> bufs;
  size_t fr = 0, tot = 0;
  while (true) {
    hipMemGetInfo(&fr, &tot);
    if (fr < (6ull << 30)) break;
    void* p = nullptr;
    if (hipMalloc(&p, B) != hipSuccess) break;
    bufs.push_back(p);
  }
  uint32_t* out;
  hipMalloc(&out, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("%zu buffers of 1 GB\n", bufs.size());
  auto best = [&](auto&& launch) {
    float b = 1e9f;
    for (int r = 0; r < 4; ++r) {
      hipEventRecord(e0, 0);
      launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (r) b = std::min(b, ms);
    }
    return b;
  };
  for (size_t i = 0; i < bufs.size(); ++i) {
    void* p = bufs[i];
    const float w = best([&] { hipLaunchKernelGGL(k_write, dim3(256 * 8), dim3(256), 0, 0, (u32x4*)p, B / 16); });
    const float r = best([&] { hipLaunchKernelGGL(k_read, dim3(256 * 8), dim3(256), 0, 0, (const u32x4*)p, B / 16, out); });
    const float g = best([&] { hipLaunchKernelGGL(k_gather, dim3(256 * 16), dim3(256), 0, 0, (const double*)p, B / 8, 64u, (double*)out); });
    printf("buffer %3zu at %p: write %6.0f GB/s  read %6.0f GB/s  gather %6.1f G/s\n", i, p, B / (w * 1e6), B / (r * 1e6),
           256.0 * 16 * 256 * 64 / (g * 1e6));
  }
  return 0;
}
