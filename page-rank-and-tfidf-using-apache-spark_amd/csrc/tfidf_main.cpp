// `tfidf` -- the host entry point that stands in for Spark.main (Spark.java:22-173, the
// repository's TF-IDF job) where no JVM is available.  Same file contract, engine behind the
// C ABI.
//
//   tfidf [DUMP] [--word W] [--out PATH]
//
// No DUMP: reads ./data (the basename of the reference's hard-coded s3n input, :26).  Writes
// "total docs are N" and the top 100 `title\ttfidf` rows for "cloud" (:140) to ./output
// (:164-171).  A malformed line kills the job (exit 1, Java exception on stderr).
#include <cstdio>
#include <string>

#include "prmi355x.h"

int main(int argc, char** argv) {
  std::string dump = "./data", word = "cloud", out = "./output";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--word" && i + 1 < argc) word = argv[++i];
    else if (a == "--out" && i + 1 < argc) out = argv[++i];
    else if (a == "-h" || a == "--help") {
      printf("usage: %s [DUMP] [--word W] [--out PATH]\n", argv[0]);
      return 0;
    } else {
      dump = a;
    }
  }
  pr_opts o;
  pr_opts_default(&o);
  pr_ctx* c = nullptr;
  int rc = pr_create(&c, &o);
  if (!rc) rc = pr_tfidf_ingest_file(c, dump.c_str());
  if (!rc) rc = pr_tfidf_write_output(c, word.c_str(), out.c_str());
  if (rc) {
    fprintf(stderr, "Exception in thread \"main\" %s\n", c ? pr_last_error(c) : "pr_create failed");
    pr_destroy(c);
    return rc == PR_E_PARSE ? 1 : 2;
  }
  pr_destroy(c);
  return 0;
}
