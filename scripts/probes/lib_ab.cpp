// Regression check between two builds of the engine library on one box: loads each library in a
// process of its own (dlopen by path), generates the bench graph, runs warm-up rounds and a
// timed run, prints GTEPS and the SpMV kernel time.  The caller interleaves the libraries.
// build: g++ -O2 -Iinclude -o scripts/probes/lib_ab scripts/probes/lib_ab.cpp -ldl
// usage: lib_ab LIB.so [scale] [steps] [repeats]
#include <dlfcn.h>
#include <cstdio>
#include <cstdlib>
#include "prmi355x.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int scale = argc > 2 ? atoi(argv[2]) : 26, steps = argc > 3 ? atoi(argv[3]) : 20;
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) { printf("dlopen: %s\n", dlerror()); return 1; }
#define SYM(name) auto f_##name = reinterpret_cast<decltype(&name)>(dlsym(h, #name)); if (!f_##name) { printf("missing %s\n", #name); return 1; }
  SYM(pr_opts_default) SYM(pr_create) SYM(pr_generate_rmat) SYM(pr_run) SYM(pr_last_error) SYM(pr_destroy) SYM(pr_build_id)
  pr_opts o;
  f_pr_opts_default(&o);
  o.device = 0;
  pr_ctx* c = nullptr;
  if (f_pr_create(&c, &o) || f_pr_generate_rmat(c, scale, 16, 4)) { printf("engine: %s\n", c ? f_pr_last_error(c) : "create"); return 1; }
  pr_stats st{};
  f_pr_run(c, 3, 0.0, &st);
  const int reps = argc > 4 ? atoi(argv[4]) : 1;  // > 1: the same timed run again and again (drift over time)
  for (int r = 1; r < reps; ++r) {
    f_pr_run(c, steps, 0.0, &st);
    printf("  run %3d: %.1f GTEPS  %.4f ms/round\n", r, st.gteps, st.ms_per_iter);
  }
  f_pr_run(c, steps, 0.0, &st);
  printf("%s | build %.8s | %.1f GTEPS  %.4f ms/round  SpMV kernels %.4f ms\n", argv[1], f_pr_build_id(), st.gteps, st.ms_per_iter, st.ms_spmv_kernel);
  f_pr_destroy(c);
  return 0;
}
