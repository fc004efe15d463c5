// Device text ingest: the reference's two input files -> dense ids, raw
// arcs and distinct mapping pairs (PageRank.java:26-60; line/field rules in SURVEY.md
// Appendix A.1 and at the top of host_graph.cpp).
//
// host_graph.cpp parses on the CPU for contexts without a device; a device context runs this
// path.  Both give identical results -- ids, arcs, pairs, N_tot, the first malformed line
// (tests/test_gpu_ingest.py):
//   1. both files go into one device buffer B = arcs || mapping;
//   2. byte i ends a line when B[i] == '\n', or B[i] == '\r' not followed by '\n'
//      (rocprim::select over byte positions); a final unterminated line counts;
//   3. one thread per line does s.split("\t") -> parts[0], parts[1] (:39-40, :47-49), or
//      records the line as malformed (the smallest such line wins: the reference dies at the
//      first one with ArrayIndexOutOfBoundsException);
//   4. dense ids: one open-addressing table over the id tokens (arc src, arc dst per line,
//      then the mapping ids) keyed by their bytes.  A slot keeps the smallest token index
//      holding its string (atomicMin), so "token t is its string's first appearance" flags
//      plus an exclusive scan number the ids in first-appearance order, like the host;
//   5. the same scheme keyed by (id, title) yields the distinct mapping pairs in order
//      (:43-51), and keyed by the whole line the distinct raw mapping lines N_tot (:60).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "engine.h"
#include "host_graph.h"
#include "text_device.h"

namespace prmi {
namespace {

// s.split("\t")[0], [1]: key [start, tab), value [tab+1, next tab or end); fewer than two
// fields (no tab, or nothing but tabs after the first) -> malformed
__global__ void k_split(const char* B, const uint64_t* E, uint64_t nE, uint64_t L, uint64_t b0,
                        uint64_t b1, uint64_t* koff, uint32_t* klen, uint64_t* voff,
                        uint32_t* vlen, uint64_t* loff, uint32_t* llen, unsigned long long* bad) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * IB + threadIdx.x;
  if (k >= L) return;
  uint64_t s, e;
  line_bounds(B, E, nE, b0, b1, k, &s, &e);
  if (loff) {
    loff[k] = s;
    llen[k] = static_cast<uint32_t>(e - s);
  }
  uint64_t t = s;
  while (t < e && B[t] != '\t') ++t;
  uint64_t j = t + 1;
  while (j < e && B[j] == '\t') ++j;
  if (t >= e || j >= e) {
    atomicMin(bad, static_cast<unsigned long long>(k));
    koff[k] = s;
    klen[k] = 0;
    voff[k] = s;
    vlen[k] = 0;
    return;
  }
  uint64_t q = t + 1;
  while (q < e && B[q] != '\t') ++q;
  koff[k] = s;
  klen[k] = static_cast<uint32_t>(t - s);
  voff[k] = t + 1;
  vlen[k] = static_cast<uint32_t>(q - (t + 1));
}

}  // namespace

int dev_ingest_text(const char* arcs, size_t alen, const char* map, size_t mlen, HostGraph* g,
                    ParseError* pe, hipStream_t s, std::string* err) {
  g->text = true;
  const uint64_t nb = static_cast<uint64_t>(alen) + mlen;
  DevBufs db;
  char* B = nullptr;
  ITRY(db.get(&B, nb + 1, err));
  if (alen) IHIP(hipMemcpyAsync(B, arcs, alen, hipMemcpyHostToDevice, s));
  if (mlen) IHIP(hipMemcpyAsync(B + alen, map, mlen, hipMemcpyHostToDevice, s));
  // lines of both regions
  uint64_t *Ea, *Em, nEa, nEm;
  ITRY(line_ends(B, 0, alen, db, &Ea, &nEa, s, err));
  ITRY(line_ends(B, alen, nb, db, &Em, &nEm, s, err));
  uint64_t lastA = 0, lastM = 0;
  if (nEa) IHIP(hipMemcpyAsync(&lastA, Ea + (nEa - 1), 8, hipMemcpyDeviceToHost, s));
  if (nEm) IHIP(hipMemcpyAsync(&lastM, Em + (nEm - 1), 8, hipMemcpyDeviceToHost, s));
  IHIP(hipStreamSynchronize(s));
  const uint64_t La = line_count(0, alen, nEa, lastA);
  const uint64_t Lm = line_count(alen, nb, nEm, lastM);
  const uint64_t T64 = 2 * La + Lm;
  // 32-bit token indices in the id table; PR_INGEST_MAX_TOKENS lowers the cap (tests force
  // the host fallback with it)
  uint64_t cap = 1ull << 30;
  if (const char* e = getenv("PR_INGEST_MAX_TOKENS")) cap = std::min<uint64_t>(cap, strtoull(e, nullptr, 0));
  if (T64 >= cap) {
    if (err) *err = "input too large for the device ingest (" + std::to_string(T64) + " id tokens)";
    return prmi::INGEST_NOFIT;
  }
  const uint32_t T = static_cast<uint32_t>(T64);
  // split every line; id tokens: [2k] src, [2k+1] dst of arc line k, [2La + k] mapping id
  uint64_t *ak, *av, *mk, *mv, *ml;
  uint32_t *akl, *avl, *mkl, *mvl, *mll;
  ITRY(db.get(&ak, La, err)); ITRY(db.get(&akl, La, err));
  ITRY(db.get(&av, La, err)); ITRY(db.get(&avl, La, err));
  ITRY(db.get(&mk, Lm, err)); ITRY(db.get(&mkl, Lm, err));
  ITRY(db.get(&mv, Lm, err)); ITRY(db.get(&mvl, Lm, err));
  ITRY(db.get(&ml, Lm, err)); ITRY(db.get(&mll, Lm, err));
  unsigned long long* bad = nullptr;
  ITRY(db.get(&bad, 2, err));
  IHIP(hipMemsetAsync(bad, 0xFF, 16, s));
  if (La) hipLaunchKernelGGL(k_split, dim3(blocks(La)), dim3(IB), 0, s, B, Ea, nEa, La, 0ull, static_cast<uint64_t>(alen), ak, akl, av, avl, nullptr, nullptr, bad);
  if (Lm) hipLaunchKernelGGL(k_split, dim3(blocks(Lm)), dim3(IB), 0, s, B, Em, nEm, Lm, static_cast<uint64_t>(alen), nb, mk, mkl, mv, mvl, ml, mll, bad + 1);
  IHIP(hipGetLastError());
  unsigned long long hbad[2];
  IHIP(hipMemcpyAsync(hbad, bad, 16, hipMemcpyDeviceToHost, s));
  IHIP(hipStreamSynchronize(s));
  // the arcs are parsed before the mapping pairs (:35-41 before :43-51): the arcs' first
  // malformed line wins
  for (int f = 0; f < 2; ++f) {
    if (hbad[f] == ~0ull) continue;
    const uint64_t k = hbad[f];
    const uint64_t* E = f ? Em : Ea;
    const uint64_t nE = f ? nEm : nEa, b0 = f ? alen : 0, b1 = f ? nb : alen;
    uint64_t e2[2] = {0, 0};  // E[k-1], E[k]
    if (k > 0) IHIP(hipMemcpyAsync(&e2[0], E + (k - 1), 8, hipMemcpyDeviceToHost, s));
    if (k < nE) IHIP(hipMemcpyAsync(&e2[1], E + k, 8, hipMemcpyDeviceToHost, s));
    IHIP(hipStreamSynchronize(s));
    auto H = [&](uint64_t o) { return f ? map + (o - alen) : arcs + o; };  // host byte of B[o]
    uint64_t st = k == 0 ? b0 : e2[0] + 1, en = b1;
    if (k < nE) {
      en = e2[1];
      if (*H(en) == '\n' && en > st && *H(en - 1) == '\r') --en;
    }
    pe->failed = true;
    pe->in_mapping = f == 1;
    pe->line = k + 1;
    pe->text.assign(H(st), std::min<uint64_t>(en - st, 200));
    return PR_E_PARSE;
  }
  // one token list for the id table
  uint64_t* toff;
  uint32_t* tlen;
  ITRY(db.get(&toff, T, err));
  ITRY(db.get(&tlen, T, err));
  if (La) {
    // interleave src/dst: strided 2-D copies
    IHIP(hipMemcpy2DAsync(toff, 16, ak, 8, 8, La, hipMemcpyDeviceToDevice, s));
    IHIP(hipMemcpy2DAsync(toff + 1, 16, av, 8, 8, La, hipMemcpyDeviceToDevice, s));
    IHIP(hipMemcpy2DAsync(tlen, 8, akl, 4, 4, La, hipMemcpyDeviceToDevice, s));
    IHIP(hipMemcpy2DAsync(tlen + 1, 8, avl, 4, 4, La, hipMemcpyDeviceToDevice, s));
  }
  if (Lm) {
    IHIP(hipMemcpyAsync(toff + 2 * La, mk, 8 * Lm, hipMemcpyDeviceToDevice, s));
    IHIP(hipMemcpyAsync(tlen + 2 * La, mkl, 4 * Lm, hipMemcpyDeviceToDevice, s));
  }
  uint32_t *id_of, n_ids;
  uint64_t* id_off;
  uint32_t* id_len;
  ITRY(dedupe(B, toff, tlen, nullptr, T, db, &id_of, &n_ids, &id_off, &id_len, nullptr, s, err));
  // :60 N_tot: distinct raw mapping lines
  uint32_t *line_no, n_lines;
  ITRY(dedupe(B, ml, mll, nullptr, static_cast<uint32_t>(Lm), db, &line_no, &n_lines, nullptr, nullptr, nullptr, s, err));
  // :43-51 distinct (id, title) pairs, in first-appearance order
  uint32_t *pair_no, n_pairs;
  uint64_t* p_off;
  uint32_t *p_len, *p_id;
  ITRY(dedupe(B, mv, mvl, id_of + 2 * La, static_cast<uint32_t>(Lm), db, &pair_no, &n_pairs, &p_off, &p_len, &p_id, s, err));
  // back to the host
  std::vector<uint32_t> ids;
  std::vector<uint64_t> ioff, poff;
  std::vector<uint32_t> ilen, plen;
  ITRY(to_host(&ids, id_of, 2 * La, s, err));
  ITRY(to_host(&ioff, id_off, n_ids, s, err));
  ITRY(to_host(&ilen, id_len, n_ids, s, err));
  ITRY(to_host(&g->pair_id, p_id, n_pairs, s, err));
  ITRY(to_host(&poff, p_off, n_pairs, s, err));
  ITRY(to_host(&plen, p_len, n_pairs, s, err));
  IHIP(hipStreamSynchronize(s));
  auto host_at = [&](uint64_t o) { return o < alen ? arcs + o : map + (o - alen); };
  g->n_tot = n_lines;
  g->m_raw = La;
  g->src.resize(La);
  g->dst.resize(La);
  for (uint64_t k = 0; k < La; ++k) {
    g->src[k] = ids[2 * k];
    g->dst[k] = ids[2 * k + 1];
  }
  {
    std::string arena;
    uint64_t bytes = 0;
    for (uint32_t l : ilen) bytes += l;
    arena.reserve(bytes);
    std::vector<uint64_t> off(n_ids);
    for (uint32_t i = 0; i < n_ids; ++i) {
      off[i] = arena.size();
      arena.append(host_at(ioff[i]), ilen[i]);
    }
    g->ids.adopt(std::move(arena), std::move(off), std::move(ilen));
  }
  g->pair_off.resize(n_pairs);
  g->pair_len = plen;
  g->titles.clear();
  for (uint32_t i = 0; i < n_pairs; ++i) {
    g->pair_off[i] = g->titles.size();
    g->titles.append(host_at(poff[i]), plen[i]);
  }
  g->n = n_ids;
  g->n_pairs = n_pairs;
  g->mapw.assign(g->n, 0);
  for (uint32_t id : g->pair_id) g->mapw[id]++;
  return PR_OK;
}

}  // namespace prmi
