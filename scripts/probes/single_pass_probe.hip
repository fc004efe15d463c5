// Baseline probe: the same SpMV c = A^T x in ONE pass over a plain CSR -- (a) a degree-binned pull
// kernel family (sub-wave groups of 1..32 lanes per row for the power-law tail, a wavefront per
// row for mid-degree rows, workgroups over 4096-edge segments with an fp64 atomic per segment
// for hub rows) and (b) rocSPARSE's CSR SpMV (adaptive / LRB / row-split) -- on the graph the
// engine runs, exported in the engine's own numbering (rows and columns ordered by in-degree, so
// hot sources sit together).  Prints GTEPS next to the engine's round.  Values are checked
// between the two baselines.  Timing context only: no product path uses this file.
// build (repo root): hipcc --offload-arch=gfx950 -O3 -Wno-deprecated-declarations -Iinclude \
//   -o scripts/probes/single_pass_probe scripts/probes/single_pass_probe.hip \
//   -Lpage-rank-and-tfidf-using-apache-spark_amd/_build -lprmi355x -lrocsparse \
//   -Wl,-rpath,'$ORIGIN/../../page-rank-and-tfidf-using-apache-spark_amd/_build'
#include <hip/hip_runtime.h>
#include <rocsparse/rocsparse.h>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "prmi355x.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
#define RK(x) do { rocsparse_status s_ = (x); if (s_ != rocsparse_status_success) { printf("%s: status %d\n", #x, (int)s_); return 1; } } while (0)

// G lanes per row (G divides 64): lanes stride over the row's columns, shuffle reduction
template <int G>
__global__ __launch_bounds__(256) void k_pull(const uint32_t* __restrict__ rows, uint32_t nrows,
                                              const int32_t* __restrict__ rp, const uint32_t* __restrict__ col,
                                              const double* __restrict__ x, double* __restrict__ y) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t r = t / G, l = t % G;
  if (r >= nrows) return;  // (whole groups leave together: G divides the wave)
  const uint32_t row = rows[r];
  const int32_t b = rp[row], e = rp[row + 1];
  double s = 0.0;
#pragma unroll 4
  for (int32_t i = b + (int32_t)l; i < e; i += G) s += x[col[i]];
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) s += __shfl_down(s, o, G);
  if (l == 0) y[row] = s;
}
// hub rows: one workgroup per 4096-edge segment, 16 edges per thread, one atomic per segment
struct Seg { uint32_t row; int32_t b, e; };
__global__ __launch_bounds__(256) void k_pull_seg(const Seg* __restrict__ segs, const uint32_t* __restrict__ col,
                                                  const double* __restrict__ x, double* __restrict__ y) {
  __shared__ double red[4];
  const Seg sg = segs[blockIdx.x];
  double s = 0.0;
#pragma unroll 16
  for (int32_t i = sg.b + (int32_t)threadIdx.x; i < sg.e; i += 256) s += x[col[i]];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(&y[sg.row], (red[0] + red[1]) + (red[2] + red[3]));
}
__global__ void k_zero_rows(const uint32_t* rows, uint32_t n, double* y) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[rows[i]] = 0.0;
}

int main(int argc, char** argv) {
  const int scale = argc > 1 ? atoi(argv[1]) : 26;
  const int reps = 5;
  pr_opts o;
  pr_opts_default(&o);
  o.device = 0;
  pr_ctx* c = nullptr;
  if (pr_create(&c, &o) || pr_generate_rmat(c, scale, 16, 4)) { printf("engine: %s\n", c ? pr_last_error(c) : "create"); return 1; }
  pr_stats st{};
  pr_run(c, 2, 0.0, &st);
  pr_run(c, 10, 0.0, &st);
  uint64_t n = 0, nnz = 0;
  if (pr_export_csr(c, nullptr, nullptr, nullptr, nullptr, &n, &nnz)) { printf("export: %s\n", pr_last_error(c)); return 1; }
  printf("R-MAT scale %d: n %llu nnz %llu | engine round %.3f ms = %.1f GTEPS (two launches, per-piece partial sums)\n",
         scale, (unsigned long long)n, (unsigned long long)nnz, st.ms_per_iter, st.gteps);
  if (nnz >= (1ull << 31)) { printf("nnz needs 64-bit row offsets: not in this probe\n"); return 1; }
  std::vector<uint64_t> rp64(n + 1);
  std::vector<uint32_t> col(nnz), outdeg(n), dw(n);
  if (pr_export_csr(c, rp64.data(), col.data(), outdeg.data(), dw.data(), &n, &nnz)) { printf("export: %s\n", pr_last_error(c)); return 1; }
  pr_destroy(c);  // (frees the engine's device memory)
  std::vector<int32_t> rp(n + 1);
  for (uint64_t i = 0; i <= n; ++i) rp[i] = (int32_t)rp64[i];
  std::vector<double> hx(n);
  for (uint64_t i = 0; i < n; ++i) hx[i] = 1.0 / (double)std::max(1u, outdeg[i]);
  // bins by in-degree: [1,2) G=1, [2,4) 2, [4,8) 4, [8,16) 8, [16,32) 16, [32,64) 32, [64,4096) 64, >= 4096 segments
  std::vector<uint32_t> bins[7];
  std::vector<uint32_t> hubs;
  std::vector<Seg> segs;
  for (uint32_t r = 0; r < n; ++r) {
    const uint32_t d = (uint32_t)(rp[r + 1] - rp[r]);
    if (!d) continue;
    if (d >= 4096) {
      hubs.push_back(r);
      for (int32_t b = rp[r]; b < rp[r + 1]; b += 4096) segs.push_back({r, b, std::min(b + 4096, rp[r + 1])});
    } else {
      int k = 0;
      while (k < 6 && (2u << k) <= d) ++k;
      bins[k].push_back(r);
    }
  }
  int32_t* d_rp; uint32_t* d_col; double *d_x, *d_y, *d_y2, *d_val; uint32_t* d_rows[7]; uint32_t* d_hubs; Seg* d_segs;
  CK(hipMalloc(&d_rp, 4ull * (n + 1)));
  CK(hipMalloc(&d_col, 4ull * nnz));
  CK(hipMalloc(&d_x, 8ull * n));
  CK(hipMalloc(&d_y, 8ull * n));
  CK(hipMalloc(&d_y2, 8ull * n));
  CK(hipMemcpy(d_rp, rp.data(), 4ull * (n + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_col, col.data(), 4ull * nnz, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_x, hx.data(), 8ull * n, hipMemcpyHostToDevice));
  CK(hipMemset(d_y, 0, 8ull * n));
  CK(hipMemset(d_y2, 0, 8ull * n));
  for (int k = 0; k < 7; ++k) {
    CK(hipMalloc(&d_rows[k], 4ull * std::max<size_t>(1, bins[k].size())));
    CK(hipMemcpy(d_rows[k], bins[k].data(), 4ull * bins[k].size(), hipMemcpyHostToDevice));
  }
  CK(hipMalloc(&d_hubs, 4ull * std::max<size_t>(1, hubs.size())));
  CK(hipMemcpy(d_hubs, hubs.data(), 4ull * hubs.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&d_segs, sizeof(Seg) * std::max<size_t>(1, segs.size())));
  CK(hipMemcpy(d_segs, segs.data(), sizeof(Seg) * segs.size(), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto grid = [](uint64_t threads) { return dim3((unsigned)((threads + 255) / 256)); };
  // ---- (a) degree-binned pull ----------------------------------------------------------
  double bin_ms[8] = {0};
  uint64_t bin_edges[8] = {0};
  for (int k = 0; k < 7; ++k)
    for (uint32_t r : bins[k]) bin_edges[k] += (uint64_t)(rp[r + 1] - rp[r]);
  for (uint32_t r : hubs) bin_edges[7] += (uint64_t)(rp[r + 1] - rp[r]);
  for (int rep = 0; rep <= reps; ++rep) {  // rep 0 = warm-up
    for (int k = 0; k < 8; ++k) {
      const uint32_t nr = k < 7 ? (uint32_t)bins[k].size() : (uint32_t)segs.size();
      if (!nr) continue;
      if (k == 7) hipLaunchKernelGGL(k_zero_rows, grid(hubs.size()), dim3(256), 0, 0, d_hubs, (uint32_t)hubs.size(), d_y);
      CK(hipEventRecord(e0, 0));
      switch (k) {
        case 0: hipLaunchKernelGGL(k_pull<1>, grid(nr), dim3(256), 0, 0, d_rows[k], nr, d_rp, d_col, d_x, d_y); break;
        case 1: hipLaunchKernelGGL(k_pull<2>, grid(2ull * nr), dim3(256), 0, 0, d_rows[k], nr, d_rp, d_col, d_x, d_y); break;
        case 2: hipLaunchKernelGGL(k_pull<4>, grid(4ull * nr), dim3(256), 0, 0, d_rows[k], nr, d_rp, d_col, d_x, d_y); break;
        case 3: hipLaunchKernelGGL(k_pull<8>, grid(8ull * nr), dim3(256), 0, 0, d_rows[k], nr, d_rp, d_col, d_x, d_y); break;
        case 4: hipLaunchKernelGGL(k_pull<16>, grid(16ull * nr), dim3(256), 0, 0, d_rows[k], nr, d_rp, d_col, d_x, d_y); break;
        case 5: hipLaunchKernelGGL(k_pull<32>, grid(32ull * nr), dim3(256), 0, 0, d_rows[k], nr, d_rp, d_col, d_x, d_y); break;
        case 6: hipLaunchKernelGGL(k_pull<64>, grid(64ull * nr), dim3(256), 0, 0, d_rows[k], nr, d_rp, d_col, d_x, d_y); break;
        default: hipLaunchKernelGGL(k_pull_seg, dim3(nr), dim3(256), 0, 0, d_segs, d_col, d_x, d_y); break;
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) bin_ms[k] += ms / reps;
    }
  }
  double tot = 0;
  const char* names[8] = {"in-degree 1 (1 lane/row)", "2-3 (2 lanes)", "4-7 (4 lanes)", "8-15 (8 lanes)", "16-31 (16 lanes)",
                          "32-63 (32 lanes)", "64-4095 (wavefront/row)", ">= 4096 (4096-edge segments)"};
  for (int k = 0; k < 8; ++k) {
    tot += bin_ms[k];
    printf("  pull bin %-30s edges %11llu  %8.3f ms  %7.1f GTEPS\n", names[k], (unsigned long long)bin_edges[k], bin_ms[k],
           bin_ms[k] > 0 ? bin_edges[k] / (bin_ms[k] * 1e6) : 0.0);
  }
  printf("degree-binned single-pass pull: %.3f ms per SpMV = %.1f GTEPS (%.2f GB of columns + offsets; x gathered at random)\n",
         tot, nnz / (tot * 1e6), (4.0 * nnz + 4.0 * n) / 1e9);
  // ---- (b) rocSPARSE ---------------------------------------------------------------------
  CK(hipMalloc(&d_val, 8ull * nnz));
  {
    std::vector<double> ones(1 << 20, 1.0);
    for (uint64_t off = 0; off < nnz; off += ones.size())
      CK(hipMemcpy(d_val + off, ones.data(), 8ull * std::min<uint64_t>(ones.size(), nnz - off), hipMemcpyHostToDevice));
  }
  rocsparse_handle h;
  RK(rocsparse_create_handle(&h));
  rocsparse_spmat_descr A;
  rocsparse_dnvec_descr X, Y;
  RK(rocsparse_create_csr_descr(&A, (int64_t)n, (int64_t)n, (int64_t)nnz, d_rp, d_col, d_val, rocsparse_indextype_i32,
                                rocsparse_indextype_i32, rocsparse_index_base_zero, rocsparse_datatype_f64_r));
  RK(rocsparse_create_dnvec_descr(&X, (int64_t)n, d_x, rocsparse_datatype_f64_r));
  RK(rocsparse_create_dnvec_descr(&Y, (int64_t)n, d_y2, rocsparse_datatype_f64_r));
  const double alpha = 1.0, beta = 0.0;
  const struct { rocsparse_spmv_alg alg; const char* name; } algs[] = {
      {rocsparse_spmv_alg_csr_adaptive, "csr_adaptive"}, {rocsparse_spmv_alg_csr_lrb, "csr_lrb"},
      {rocsparse_spmv_alg_csr_rowsplit, "csr_rowsplit"}};
  std::vector<double> y1(n), y2(n);
  CK(hipMemcpy(y1.data(), d_y, 8ull * n, hipMemcpyDeviceToHost));
  for (const auto& a : algs) {
    size_t bs = 0;
    CK(hipMemset(d_y2, 0x42, 8ull * n));  // (1.6e11 everywhere: an algorithm that returns without computing shows)
    RK(rocsparse_spmv(h, rocsparse_operation_none, &alpha, A, X, &beta, Y, rocsparse_datatype_f64_r, a.alg,
                      rocsparse_spmv_stage_buffer_size, &bs, nullptr));
    void* buf = nullptr;
    CK(hipMalloc(&buf, std::max<size_t>(bs, 8)));
    RK(rocsparse_spmv(h, rocsparse_operation_none, &alpha, A, X, &beta, Y, rocsparse_datatype_f64_r, a.alg,
                      rocsparse_spmv_stage_preprocess, &bs, buf));
    double ms_sum = 0;
    for (int rep = 0; rep <= reps; ++rep) {
      CK(hipEventRecord(e0, 0));
      RK(rocsparse_spmv(h, rocsparse_operation_none, &alpha, A, X, &beta, Y, rocsparse_datatype_f64_r, a.alg,
                        rocsparse_spmv_stage_compute, &bs, buf));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) ms_sum += ms / reps;
    }
    // the two baselines agree
    CK(hipMemcpy(y2.data(), d_y2, 8ull * n, hipMemcpyDeviceToHost));
    double worst = 0;
    for (uint64_t i = 0; i < n; ++i)
      worst = std::max(worst, std::fabs(y1[i] - y2[i]) / std::max(1e-300, std::max(std::fabs(y1[i]), std::fabs(y2[i]))));
    if (!(worst < 1e-9))
      printf("rocSPARSE %-13s returned success after %.3f ms without writing y (not a measurement)\n", a.name, ms_sum);
    else
      printf("rocSPARSE %-13s %.3f ms per SpMV = %.1f GTEPS (explicit fp64 values: %.2f GB of matrix per pass); "
             "worst relative difference to the binned pull %.2e\n", a.name, ms_sum, nnz / (ms_sum * 1e6),
             (12.0 * nnz + 4.0 * n) / 1e9, worst);
    CK(hipFree(buf));
  }
  return 0;
}
