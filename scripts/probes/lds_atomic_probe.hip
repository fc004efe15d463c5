// Micro-benchmark: LDS f64 accumulation rate per CU (ds_add_f64 atomics vs plain RMW) with
// random row offsets inside a 4096-entry accumulator.
// build: hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics -o lds_atomic_probe lds_atomic_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(1024) void acc_kernel(const uint32_t* __restrict__ idx, int iters, double* out) {
  __shared__ double acc[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) acc[i] = 0.0;
  __syncthreads();
  uint32_t s = idx[(blockIdx.x * blockDim.x + threadIdx.x) & 65535];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s = s * 1664525u + 1013904223u;
      const uint32_t r = (s >> 8) & 4095;
      if (MODE == 0) atomicAdd(&acc[r], 1.0);
      else acc[r] += 1.0;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = acc[0];
}

int main() {
  uint32_t* d; double* o;
  if (hipMalloc(&d, 65536 * 4) != hipSuccess || hipMalloc(&o, 8 * 4096) != hipSuccess) return 1;
  (void)hipMemset(d, 7, 65536 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int iters = 2000;
  for (int mode = 0; mode < 2; ++mode) {
    for (int wg : {256, 512, 1024}) {
      float ms = 0;
      for (int r = 0; r < 2; ++r) {
        (void)hipEventRecord(a);
        if (mode == 0) hipLaunchKernelGGL(acc_kernel<0>, dim3(wg), dim3(1024), 0, 0, d, iters, o);
        else hipLaunchKernelGGL(acc_kernel<1>, dim3(wg), dim3(1024), 0, 0, d, iters, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
      }
      const double ops = 1024.0 * wg * iters * 8;
      printf("%s  wgs %4d: %7.3f ms  %8.1f G adds/s  %.2f lanes/clk/CU\n", mode ? "plain RMW " : "ds_add_f64", wg, ms,
             ops / ms / 1e6, ops / (ms * 1e-3) / 256 / 2.4e9);
    }
  }
  return 0;
}
