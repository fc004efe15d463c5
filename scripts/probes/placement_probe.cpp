// Placement probe: does the round time depend on WHERE the round's arrays sit in device memory?
// Builds the bench graph, times rounds, then applies steps "G:names": allocate a ballast of G GB
// (1-GB blocks), move the named arrays (comma list, or "all") to fresh allocations
// (pr_debug_move_array: new buffer, device copy, old one freed), free the ballast, time again.
// build: hipcc -O2 -Iinclude -o scripts/probes/placement_probe -x hip scripts/probes/placement_probe.cpp \
//   -Lpage-rank-and-tfidf-using-apache-spark_amd/_build -lprmi355x \
//   -Wl,-rpath,'$ORIGIN/../../page-rank-and-tfidf-using-apache-spark_amd/_build'
// usage: placement_probe scale step...
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "prmi355x.h"


int main(int argc, char** argv) {
  const int scale = argc > 1 ? atoi(argv[1]) : 26;
  pr_opts o;
  pr_opts_default(&o);
  o.device = 0;
  pr_ctx* c = nullptr;
  if (pr_create(&c, &o) || pr_generate_rmat(c, scale, 16, 4)) { printf("engine: %s\n", c ? pr_last_error(c) : "create"); return 1; }
  pr_stats st{};
  pr_run(c, 3, 0.0, &st);
  auto timed = [&](const char* what) {
    pr_run(c, 20, 0.0, &st);
    const double a = st.gteps;
    pr_run(c, 20, 0.0, &st);
    printf("%-40s %.1f / %.1f GTEPS  SpMV kernels %.4f ms\n", what, a, st.gteps, st.ms_spmv_kernel);
    fflush(stdout);
  };
  timed("as built");
  const char* all[] = {"partial", "col16", "col", "bits", "roffL", "x", "maps", "meta"};
  for (int a = 2; a < argc; ++a) {
    const char* colon = strchr(argv[a], ':');
    if (!colon) continue;
    const int gb = atoi(argv[a]);
    std::vector<void*> ballast;
    for (int i = 0; i < gb; ++i) {
      void* p = nullptr;
      if (hipMalloc(&p, 1ull << 30) != hipSuccess) break;
      ballast.push_back(p);
    }
    std::string names = colon + 1;
    std::vector<std::string> list;
    if (names == "all") list.assign(all, all + 8);
    else {
      size_t pos = 0;
      while (pos <= names.size()) {
        const size_t q = names.find(',', pos);
        list.push_back(names.substr(pos, q == std::string::npos ? std::string::npos : q - pos));
        if (q == std::string::npos) break;
        pos = q + 1;
      }
    }
    for (const std::string& n : list)
      if (pr_debug_move_array(c, n.c_str())) { printf("move %s: %s\n", n.c_str(), pr_last_error(c)); return 1; }
    for (void* p : ballast) hipFree(p);
    timed(argv[a]);
  }
  pr_destroy(c);
  return 0;
}
