// Placement probe 2: does the round time depend on how CONTIGUOUS the engine's arrays are in
// physical memory?  Before the engine allocates anything, fill the device with blocks of B MB,
// free every other one (the rest stay allocated as spacers), then build the bench graph -- its
// arrays can only be assembled from B-MB holes -- and time rounds.  B = 0: no spacers.
// build: hipcc --offload-arch=gfx950 -O2 -Iinclude -o scripts/probes/frag_probe scripts/probes/frag_probe.hip \
//   -Lpage-rank-and-tfidf-using-apache-spark_amd/_build -lprmi355x \
//   -Wl,-rpath,'$ORIGIN/../../page-rank-and-tfidf-using-apache-spark_amd/_build'
// usage: frag_probe B_MB [scale] [keep_every] [max_gb]   (keep_every = 1 with max_gb = G: a G-GB
//        ballast stays allocated below the engine's arrays)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "prmi355x.h"

int main(int argc, char** argv) {
  const size_t bmb = argc > 1 ? (size_t)atoll(argv[1]) : 64;
  const int scale = argc > 2 ? atoi(argv[2]) : 26;
  const int keep_every = argc > 3 ? atoi(argv[3]) : 2;
  const size_t max_gb = argc > 4 ? (size_t)atoll(argv[4]) : 100000;
  std::vector<void*> blocks;
  if (bmb) {
    size_t fr = 0, tot = 0;
    hipSetDevice(0);
    hipMemGetInfo(&fr, &tot);
    const size_t b = bmb << 20;
    while (true) {
      hipMemGetInfo(&fr, &tot);
      if (fr < (4ull << 30) + b || blocks.size() * b >= (max_gb << 30)) break;
      void* p = nullptr;
      if (hipMalloc(&p, b) != hipSuccess) break;
      blocks.push_back(p);
    }
    size_t kept = 0;
    for (size_t i = 0; i < blocks.size(); ++i)
      if (i % keep_every != 0) { hipFree(blocks[i]); blocks[i] = nullptr; } else ++kept;
    hipMemGetInfo(&fr, &tot);
    printf("spacers: %zu blocks of %zu MB allocated, %zu kept; free %.1f of %.1f GB\n", blocks.size(), bmb, kept, fr / 1e9, tot / 1e9);
  }
  pr_opts o;
  pr_opts_default(&o);
  o.device = 0;
  pr_ctx* c = nullptr;
  if (pr_create(&c, &o) || pr_generate_rmat(c, scale, 16, 4)) { printf("engine: %s\n", c ? pr_last_error(c) : "create"); return 1; }
  pr_stats st{};
  pr_run(c, 3, 0.0, &st);
  for (int r = 0; r < 3; ++r) {
    pr_run(c, 20, 0.0, &st);
    printf("  blocks of %zu MB: %.1f GTEPS  %.4f ms/round  SpMV kernels %.4f ms\n", bmb, st.gteps, st.ms_per_iter, st.ms_spmv_kernel);
  }
  pr_destroy(c);
  for (void* p : blocks) if (p) hipFree(p);
  return 0;
}
