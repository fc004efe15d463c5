// Micro-benchmark: random 8-byte gathers per second on MI355X from L1 / L2 / MALL / HBM
// sized tables and from LDS, with the index stream itself as the baseline.
// build: hipcc --offload-arch=gfx950 -O3 -o gather_probe gather_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// MODE 0: index stream only; 1: global gathers; 2: LDS gathers (table <= 16K doubles)
template <int MODE>
__global__ __launch_bounds__(1024) void gather(const uint32_t* __restrict__ idx, uint64_t n,
                                               const double* __restrict__ tab, uint32_t tmask,
                                               double* out) {
  __shared__ double lds[16384];
  if (MODE == 2) {
    for (uint32_t i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = tab[i & tmask];
    __syncthreads();
  }
  const uint64_t per = 16;
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  double acc = 0.0;
  for (uint64_t base = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * per; base < n; base += nthreads * per) {
    const u32x4* p = reinterpret_cast<const u32x4*>(idx + base);
    u32x4 c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = __builtin_nontemporal_load(p + q);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t i = c[k >> 2][k & 3] & tmask;
      if (MODE == 0) acc += (double)i;
      else if (MODE == 1) acc += tab[i];
      else acc += lds[i];
    }
  }
  if (acc == -1.0) out[0] = acc;
}

int main() {
  const uint64_t n = 1ull << 28;  // 268M gathers
  std::vector<uint32_t> h(n);
  std::mt19937 rng(1);
  for (uint64_t i = 0; i < n; ++i) h[i] = rng();
  uint32_t* d_idx; double* d_tab; double* d_out;
  const uint64_t tabn = 1ull << 26;  // 512 MB
  CK(hipMalloc(&d_idx, n * 4));
  CK(hipMalloc(&d_tab, tabn * 8));
  CK(hipMalloc(&d_out, 8));
  CK(hipMemcpy(d_idx, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemset(d_tab, 0, tabn * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](int mode, uint32_t tmask, int wg_per_cu, int threads) -> float {
    dim3 gr(256 * wg_per_cu), bl(threads);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(gather<0>, gr, bl, 0, 0, d_idx, n, d_tab, tmask, d_out);
      else if (mode == 1) hipLaunchKernelGGL(gather<1>, gr, bl, 0, 0, d_idx, n, d_tab, tmask, d_out);
      else hipLaunchKernelGGL(gather<2>, gr, bl, 0, 0, d_idx, n, d_tab, tmask, d_out);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
  };
  printf("n = %llu gathers\n", (unsigned long long)n);
  const int cfg[][2] = {{1, 1024}, {2, 1024}};
  for (auto& c : cfg) {
    float ms = run(0, 0xFFFFFFFFu, c[0], c[1]);
    printf("wg/cu %d thr %d  index stream only          %7.3f ms  %7.1f G/s  %6.1f GB/s\n", c[0], c[1], ms, n / ms / 1e6, n * 4 / ms / 1e6);
    for (uint32_t bits : {0u, 8u, 11u, 14u, 17u, 19u, 21u, 23u, 25u, 26u}) {
      const uint32_t m = bits ? (1u << bits) - 1 : 0u;
      ms = run(1, m, c[0], c[1]);
      printf("wg/cu %d thr %d  global table %9.0f KB    %7.3f ms  %7.1f G/s  %.3f lanes/clk/CU\n", c[0], c[1], (m + 1) * 8.0 / 1024, ms, n / ms / 1e6, n / (ms * 1e-3) / 256 / 2.4e9);
    }
    for (uint32_t bits : {0u, 8u, 14u}) {
      const uint32_t m = bits ? (1u << bits) - 1 : 0u;
      ms = run(2, m, 1, 1024);
      printf("wg/cu 1 thr 1024  LDS table %9.0f KB       %7.3f ms  %7.1f G/s  %.3f lanes/clk/CU\n", (m + 1) * 8.0 / 1024, ms, n / ms / 1e6, n / (ms * 1e-3) / 256 / 2.4e9);
    }
  }
  return 0;
}
