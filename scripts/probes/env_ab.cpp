// In-process A/B of run-time switches of the engine (the ones read at every launch, e.g.
// PR_DYNTAIL / PR_DYNG / PR_DYNL2): one graph, one placement, alternating settings.
// build: g++ -O2 -Iinclude -o scripts/probes/env_ab scripts/probes/env_ab.cpp \
//   -Lpage-rank-and-tfidf-using-apache-spark_amd/_build -lprmi355x \
//   -Wl,-rpath,'$ORIGIN/../../page-rank-and-tfidf-using-apache-spark_amd/_build'
// usage: env_ab scale reps "NAME=V NAME=V" "NAME=V ..."      (each argument one setting; "" = defaults)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "prmi355x.h"

static void apply(const std::string& set, bool on) {
  size_t pos = 0;
  while (pos < set.size()) {
    size_t q = set.find(' ', pos);
    if (q == std::string::npos) q = set.size();
    const std::string kv = set.substr(pos, q - pos);
    const size_t eq = kv.find('=');
    if (eq != std::string::npos) {
      if (on) setenv(kv.substr(0, eq).c_str(), kv.substr(eq + 1).c_str(), 1);
      else unsetenv(kv.substr(0, eq).c_str());
    }
    pos = q + 1;
  }
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const int scale = atoi(argv[1]), reps = atoi(argv[2]);
  pr_opts o;
  pr_opts_default(&o);
  o.device = 0;
  pr_ctx* c = nullptr;
  if (pr_create(&c, &o) || pr_generate_rmat(c, scale, 16, 4)) { printf("engine: %s\n", c ? pr_last_error(c) : "create"); return 1; }
  pr_stats st{};
  pr_run(c, 5, 0.0, &st);
  std::vector<double> sum(argc, 0.0);
  for (int r = 0; r < reps; ++r)
    for (int a = 3; a < argc; ++a) {
      apply(argv[a], true);
      pr_run(c, 3, 0.0, &st);
      if (pr_run(c, 20, 0.0, &st)) { printf("run: %s\n", pr_last_error(c)); return 1; }
      apply(argv[a], false);
      printf("rep %d | %-40s | %.1f GTEPS  SpMV kernels %.4f ms\n", r + 1, argv[a][0] ? argv[a] : "defaults", st.gteps, st.ms_spmv_kernel);
      fflush(stdout);
      sum[a] += st.gteps;
    }
  for (int a = 3; a < argc; ++a) printf("mean | %-40s | %.1f GTEPS\n", argv[a][0] ? argv[a] : "defaults", sum[a] / reps);
  pr_destroy(c);
  return 0;
}
