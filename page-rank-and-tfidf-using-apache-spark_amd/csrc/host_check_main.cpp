// `prmi_host_check` -- drives the host-only side of the C ABI (PR_DEVICE_NONE contexts) over
// a directory of test cases, for the AddressSanitizer/UBSan build (`make asan`).  Everything
// it touches runs on the CPU: the text ingest of PageRank.java:26-60 (host parser), the
// graph info / id / pair accessors, Java Double.toString formatting, error paths and the
// PR_E_NODEV refusals of device calls.  tests/test_asan_host.py writes the cases, runs this
// under the sanitizers and checks every printed line against the oracle.
//
//   prmi_host_check CASEDIR NCASES
//     CASEDIR/<i>.arcs, CASEDIR/<i>.map   ingest inputs of case i
//     CASEDIR/doubles.bin                 raw little-endian doubles for pr_format_double
// Output lines (strings hex-encoded so any byte survives):
//   case <i> err <rc> <hex(message)>
//   case <i> info <n_vertices> <raw_edges> <n_tot> <n_pairs>
//   id <i> <v> <hex>          pair <i> <k> <id> <hex>          fmt <hex>
//   nodev <name> <rc>         done
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "prmi355x.h"

namespace {

bool slurp(const std::string& path, std::string* out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  out->clear();
  char buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) out->append(buf, k);
  fclose(f);
  return true;
}

std::string hex(const char* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    const unsigned char c = static_cast<unsigned char>(p[i]);
    s[2 * i] = d[c >> 4];
    s[2 * i + 1] = d[c & 15];
  }
  return s.empty() ? std::string("-") : s;
}

pr_ctx* host_ctx() {
  pr_opts o;
  pr_opts_default(&o);
  o.device = PR_DEVICE_NONE;
  pr_ctx* c = nullptr;
  if (pr_create(&c, &o) != PR_OK) {
    fprintf(stderr, "pr_create(PR_DEVICE_NONE) failed\n");
    exit(2);
  }
  return c;
}

// accessors read into exact-size buffers (a one-byte overrun would trip the sanitizer)
std::string id_string(pr_ctx* c, uint32_t v) {
  size_t len = 0;
  if (pr_id_string(c, v, nullptr, 0, &len) != PR_OK) return "?";
  std::vector<char> b(len ? len : 1);
  pr_id_string(c, v, b.data(), len, &len);
  return hex(b.data(), len);
}

void run_case(const std::string& dir, int i) {
  std::string a, m;
  const std::string base = dir + "/" + std::to_string(i);
  if (!slurp(base + ".arcs", &a) || !slurp(base + ".map", &m)) {
    printf("case %d err %d %s\n", i, PR_E_IO, hex("missing", 7).c_str());
    return;
  }
  pr_ctx* c = host_ctx();
  // heap copies of exactly the input size: the parser must never read past the end
  std::vector<char> ab(a.begin(), a.end()), mb(m.begin(), m.end());
  const int rc = pr_ingest_buffers(c, ab.empty() ? nullptr : ab.data(), ab.size(),
                                   mb.empty() ? nullptr : mb.data(), mb.size());
  if (rc != PR_OK) {
    const char* e = pr_last_error(c);
    printf("case %d err %d %s\n", i, rc, hex(e, strlen(e)).c_str());
    pr_destroy(c);
    return;
  }
  pr_graph_info gi;
  pr_graph_get_info(c, &gi);
  printf("case %d info %llu %llu %llu %llu\n", i, static_cast<unsigned long long>(gi.n_vertices),
         static_cast<unsigned long long>(gi.raw_edges), static_cast<unsigned long long>(gi.n_tot),
         static_cast<unsigned long long>(gi.n_pairs));
  for (uint32_t v = 0; v < gi.n_vertices; ++v) printf("id %d %u %s\n", i, v, id_string(c, v).c_str());
  for (uint64_t k = 0; k < gi.n_pairs; ++k) {
    uint32_t id = 0;
    size_t len = 0;
    pr_pair(c, k, &id, nullptr, 0, &len);
    std::vector<char> t(len ? len : 1);
    pr_pair(c, k, &id, t.data(), len, &len);
    printf("pair %d %llu %u %s\n", i, static_cast<unsigned long long>(k), id, hex(t.data(), len).c_str());
  }
  // out-of-range accessors refuse
  if (pr_id_string(c, gi.n_vertices, nullptr, 0, nullptr) != PR_E_ARG ||
      pr_pair(c, gi.n_pairs, nullptr, nullptr, 0, nullptr) != PR_E_ARG)
    printf("case %d accessor-range-not-refused\n", i);
  pr_destroy(c);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s CASEDIR NCASES\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int n = atoi(argv[2]);
  printf("version %s\n", pr_version());
  // device calls on a host-only context refuse with PR_E_NODEV
  {
    pr_ctx* c = host_ctx();
    printf("nodev generate_rmat %d\n", pr_generate_rmat(c, 4, 2, 1));
    const char arcs[] = "1\t2\n", map[] = "1\tA\n2\tB\n";
    pr_ingest_buffers(c, arcs, sizeof arcs - 1, map, sizeof map - 1);
    pr_stats st;
    printf("nodev run %d\n", pr_run(c, 1, 0.0, &st));
    uint32_t d[2];
    printf("nodev degrees %d\n", pr_get_degrees(c, d, d, d, 2));
    printf("nodev tfidf_ingest %d\n", pr_tfidf_ingest_buffer(c, "a\tb c\n", 6));
    pr_destroy(c);
  }
  for (int i = 0; i < n; ++i) run_case(dir, i);
  std::string dbl;
  if (slurp(dir + "/doubles.bin", &dbl)) {
    for (size_t k = 0; k + 8 <= dbl.size(); k += 8) {
      double v;
      std::memcpy(&v, dbl.data() + k, 8);
      char buf[64];
      const int len = pr_format_double(v, buf, sizeof buf);
      printf("fmt %s\n", len > 0 ? hex(buf, static_cast<size_t>(len)).c_str() : "-");
    }
  }
  printf("done\n");
  return 0;
}
