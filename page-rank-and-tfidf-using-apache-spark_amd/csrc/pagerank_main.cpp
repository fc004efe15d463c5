// `pagerank` -- the host entry point that stands in for PageRank.main (PageRank.java:21-206)
// where no JVM is available.  Same job, same file contract, engine behind the C ABI.
//
//   pagerank [ARCS MAPPING [ITERATIONS]] [--out PATH] [--topk K] [--tol X] [--verbose]
//            [--normalized] [--resume CKPT] [--checkpoint CKPT] [--dump PATH]
//
// --dump writes every ranked page by id (`id \t title \t rank`, pr_write_rank_dump): the
// full rank dump of SURVEY.md 8f #2 beside ./topPage.
// --normalized, --resume and --checkpoint are not in the reference:
// normalized ranks (r^0 = 1/N_tot, base 0.15/N_tot); continue from a checkpoint's ranks for
// ITERATIONS more rounds; write the final ranks as a checkpoint.
//
// No positional arguments: reads ./wikipedia_arcs and ./wikipedia_mapping (the basenames of
// the reference's hard-coded s3n inputs, :27,:30), runs 10 rounds (:92) and writes the top
// 100 (:189) `title\trank` lines to ./topPage (:192-197).
//
// Failure behaviour mirrors the reference job: a malformed input line or an empty dangling
// RDD kills the job (exit 1, Java exception name on stderr, no topPage written); an
// IOException while writing ./topPage is printed and swallowed (:201-204, exit 0).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "prmi355x.h"

static int die(pr_ctx* c, int rc) {
  fprintf(stderr, "Exception in thread \"main\" %s\n", c ? pr_last_error(c) : "pr_create failed");
  pr_destroy(c);
  return rc == PR_E_PARSE || rc == PR_E_EMPTY_DANGLING ? 1 : 2;
}

int main(int argc, char** argv) {
  std::string arcs = "./wikipedia_arcs", mapping = "./wikipedia_mapping", out = "./topPage";
  std::string resume, checkpoint, dump;
  int iterations = 10, npos = 0;
  double tol = 0.0;
  pr_opts o;
  pr_opts_default(&o);
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--out" && i + 1 < argc) out = argv[++i];
    else if (a == "--topk" && i + 1 < argc) o.topk = static_cast<uint32_t>(atoi(argv[++i]));
    else if (a == "--tol" && i + 1 < argc) tol = atof(argv[++i]);
    else if (a == "--verbose") o.flags |= PR_F_VERBOSE;
    else if (a == "--normalized") o.flags |= PR_F_NORMALIZED;
    else if (a == "--resume" && i + 1 < argc) resume = argv[++i];
    else if (a == "--checkpoint" && i + 1 < argc) checkpoint = argv[++i];
    else if (a == "--dump" && i + 1 < argc) dump = argv[++i];
    else if (a == "-h" || a == "--help") {
      printf("usage: %s [ARCS MAPPING [ITERATIONS]] [--out PATH] [--topk K] [--tol X] [--verbose]\n"
             "          [--normalized] [--resume CKPT] [--checkpoint CKPT] [--dump PATH]\n", argv[0]);
      return 0;
    } else {
      if (npos == 0) arcs = a;
      else if (npos == 1) mapping = a;
      else if (npos == 2) iterations = atoi(a.c_str());
      ++npos;
    }
  }
  pr_ctx* c = nullptr;
  int rc = pr_create(&c, &o);
  if (rc) return die(c, rc);
  rc = pr_ingest_files(c, arcs.c_str(), mapping.c_str());
  if (rc) return die(c, rc);
  if (!resume.empty()) {
    rc = pr_checkpoint_load(c, resume.c_str());
    if (rc) return die(c, rc);
  }
  pr_stats st;
  rc = pr_run(c, iterations, tol, &st);
  if (rc) return die(c, rc);
  if (!checkpoint.empty()) {
    rc = pr_checkpoint_save(c, checkpoint.c_str());
    if (rc) return die(c, rc);
  }
  if (o.flags & PR_F_VERBOSE)
    fprintf(stderr, "[prmi355x] %d rounds, %.3f ms/round, %.2f GTEPS, nnz=%llu\n", st.iterations,
            st.ms_per_iter, st.gteps, static_cast<unsigned long long>(st.nnz));
  if (!dump.empty()) {
    rc = pr_write_rank_dump(c, dump.c_str());
    if (rc) return die(c, rc);
  }
  rc = pr_write_top_page(c, out.c_str());
  if (rc == PR_E_IO) {
    fprintf(stderr, "%s\n", pr_last_error(c));  // e.printStackTrace(), job still succeeds
  } else if (rc) {
    return die(c, rc);
  }
  pr_destroy(c);
  return 0;
}
