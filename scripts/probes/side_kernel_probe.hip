// Micro-benchmark: how long a short scatter kernel (the shape of the sparse exchange's unpack:
// 2.7 M 8-byte values to scattered positions of a 22 MB array) takes on a second stream while
// the engine's round loop runs on the first -- i.e. beside a stream launch whose workgroups hold
// PR_STREAM_CUS of the 32 compute units of every XCD for its whole length.  Prints the scatter's
// duration alone and beside the loop, and the loop's round time with and without the side work.
// build (repo root): hipcc --offload-arch=gfx950 -O3 -Iinclude -o scripts/probes/side_kernel_probe \
//   scripts/probes/side_kernel_probe.hip -Lpage-rank-and-tfidf-using-apache-spark_amd/_build -lprmi355x \
//   -Wl,-rpath,'$ORIGIN/../../page-rank-and-tfidf-using-apache-spark_amd/_build' -lpthread
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include "prmi355x.h"

__global__ void k_scatter(double* dst, const uint32_t* pos, const double* val, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[pos[i]] = val[i];
}
__global__ void k_positions(uint32_t* pos, uint32_t n, uint32_t m) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // a sorted, gappy position list like the exchange's (entries a peer references, in x order)
  if (i < n) pos[i] = static_cast<uint32_t>((static_cast<uint64_t>(i) * m) / n);
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static void quant(const char* what, std::vector<float> v) {
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  printf("%s n %zu  p10 %.0f  p50 %.0f  p90 %.0f  max %.0f us\n", what, n, v[n / 10] * 1e3, v[n / 2] * 1e3,
         v[(9 * n) / 10] * 1e3, v[n - 1] * 1e3);
}

int main(int argc, char** argv) {
  const int scale = argc > 1 ? atoi(argv[1]) : 26;
  pr_opts o;
  pr_opts_default(&o);
  o.device = 0;
  pr_ctx* c = nullptr;
  if (pr_create(&c, &o) || pr_generate_rmat(c, scale, 16, 4)) { printf("engine: %s\n", c ? pr_last_error(c) : "create"); return 1; }
  pr_stats st{};
  pr_run(c, 2, 0.0, &st);
  pr_run(c, 10, 0.0, &st);
  const double base = st.ms_per_iter;
  const uint32_t n = 2700000, m = 2750000;
  double *dst, *val;
  uint32_t* pos;
  CK(hipMalloc(&dst, 8ull * m));
  CK(hipMalloc(&val, 8ull * n));
  CK(hipMalloc(&pos, 4ull * n));
  CK(hipMemset(val, 0, 8ull * n));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipLaunchKernelGGL(k_positions, dim3((n + 255) / 256), dim3(256), 0, s, pos, n, m);
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto sample = [&](int k, std::vector<float>* out) {
    for (int i = 0; i < k; ++i) {
      hipEventRecord(a, s);
      hipLaunchKernelGGL(k_scatter, dim3((n + 255) / 256), dim3(256), 0, s, dst, pos, val, n);
      hipEventRecord(b, s);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (out) out->push_back(ms);
      std::this_thread::sleep_for(std::chrono::microseconds(300));
    }
  };
  sample(20, nullptr);
  std::vector<float> alone, beside;
  sample(200, &alone);
  const char* cus = getenv("PR_STREAM_CUS");
  printf("stream launch: %s of 32 compute units per XCD\n", cus ? cus : "32");
  quant("scatter alone:        ", alone);
  pr_stats st2{};
  std::thread th([&] { pr_run(c, 150, 0.0, &st2); });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  sample(300, &beside);
  th.join();
  quant("scatter beside rounds:", beside);
  printf("round: %.3f ms alone, %.3f ms with the side scatters (300 scatters in 150 rounds)\n", base, st2.ms_per_iter);
  pr_destroy(c);
  return 0;
}
