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

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "host_graph.h"
#include "prmi355x.h"

namespace prmi {

#define IHIP(x)                                                                    \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      if (err) *err = std::string(#x) + ": " + hipGetErrorString(e_);              \
      return e_ == hipErrorOutOfMemory ? PR_E_OOM : PR_E_HIP;                      \
    }                                                                              \
  } while (0)

namespace {

constexpr int IB = 256;

struct LineEnd {
  const char* B;
  uint64_t b1;
  __device__ bool operator()(const uint64_t& i) const {
    const char c = B[i];
    return c == '\n' || (c == '\r' && !(i + 1 < b1 && B[i + 1] == '\n'));
  }
};

// content [start, end) of line k of a region [b0, b1) whose nE line ends are E[]
__host__ __device__ inline void line_bounds(const char* B, const uint64_t* E, uint64_t nE,
                                            uint64_t b0, uint64_t b1, uint64_t k,
                                            uint64_t* start, uint64_t* end) {
  const uint64_t s = k == 0 ? b0 : E[k - 1] + 1;
  uint64_t e = b1;
  if (k < nE) {
    e = E[k];
    if (B[e] == '\n' && e > s && B[e - 1] == '\r') --e;  // "\r\n" is one terminator
  }
  *start = s;
  *end = e;
}

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

__device__ inline uint64_t hash_span(const char* p, uint32_t n, uint64_t h) {
  h ^= 0xCBF29CE484222325ull ^ (static_cast<uint64_t>(n) * 0x9E3779B97F4A7C15ull);
  for (uint32_t i = 0; i < n; ++i) h = (h ^ static_cast<unsigned char>(p[i])) * 0x100000001B3ull;
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  return h;
}

__device__ inline bool same_span(const char* B, uint64_t a, uint32_t la, uint64_t b, uint32_t lb) {
  if (la != lb) return false;
  for (uint32_t i = 0; i < la; ++i)
    if (B[a + i] != B[b + i]) return false;
  return true;
}

// token t = bytes [off[t], off[t] + len[t]) (and tag[t] when tag != nullptr: pairs are keyed
// by (id, title)); slot_of[t] = its string's slot, first[slot] = smallest token index
__global__ void k_intern(const char* B, const uint64_t* off, const uint32_t* len,
                         const uint32_t* tag, uint32_t T, uint32_t* slots, uint32_t* first,
                         uint64_t mask, uint32_t* slot_of) {
  const uint32_t t = blockIdx.x * IB + threadIdx.x;
  if (t >= T) return;
  const uint64_t o = off[t];
  const uint32_t n = len[t];
  const uint32_t g = tag ? tag[t] : 0u;
  uint64_t h = hash_span(B + o, n, tag ? (static_cast<uint64_t>(g) + 1) * 0xD6E8FEB86659FD93ull : 0) & mask;
  for (;;) {
    uint32_t s = __hip_atomic_load(&slots[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 0) {
      s = atomicCAS(&slots[h], 0u, t + 1);
      if (s == 0) break;
    }
    const uint32_t u = s - 1;
    if ((!tag || tag[u] == g) && same_span(B, off[u], len[u], o, n)) break;
    h = (h + 1) & mask;
  }
  if (__hip_atomic_load(&first[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > t)
    atomicMin(&first[h], t);
  slot_of[t] = static_cast<uint32_t>(h);
}

__global__ void k_first_flag(const uint32_t* slot_of, const uint32_t* first, uint32_t T,
                             uint32_t* flag) {
  const uint32_t t = blockIdx.x * IB + threadIdx.x;
  if (t < T) flag[t] = first[slot_of[t]] == t ? 1u : 0u;
}

// number[t] = rank of t's first appearance among all first appearances
__global__ void k_number(const uint32_t* slot_of, const uint32_t* first, const uint32_t* rank,
                         uint32_t T, uint32_t* number) {
  const uint32_t t = blockIdx.x * IB + threadIdx.x;
  if (t < T) number[t] = rank[first[slot_of[t]]];
}

// per distinct string (in order): its first token's bytes
__global__ void k_firsts(const uint32_t* flag, const uint32_t* rank, const uint64_t* off,
                         const uint32_t* len, const uint32_t* tag, uint32_t T, uint64_t* o_off,
                         uint32_t* o_len, uint32_t* o_tag) {
  const uint32_t t = blockIdx.x * IB + threadIdx.x;
  if (t >= T || !flag[t]) return;
  const uint32_t r = rank[t];
  o_off[r] = off[t];
  o_len[r] = len[t];
  if (o_tag) o_tag[r] = tag[t];
}

inline uint32_t blocks(uint64_t n) { return static_cast<uint32_t>((n + IB - 1) / IB); }

struct DevBufs {
  std::vector<void*> v;
  ~DevBufs() {
    for (void* p : v)
      if (p) (void)hipFree(p);
  }
  template <class T>
  int get(T** p, uint64_t count, std::string* err) {
    *p = nullptr;
    IHIP(hipMalloc(reinterpret_cast<void**>(p), (count ? count : 1) * sizeof(T)));
    v.push_back(*p);
    return PR_OK;
  }
};

#define ITRY(x)                     \
  do {                              \
    int rc_ = (x);                  \
    if (rc_ != PR_OK) return rc_;   \
  } while (0)

// line ends of region [b0, b1) -> E (device), count
int line_ends(const char* B, uint64_t b0, uint64_t b1, DevBufs& db, uint64_t** E, uint64_t* nE,
              hipStream_t s, std::string* err) {
  const uint64_t n = b1 - b0;
  ITRY(db.get(E, n, err));
  uint64_t* d_cnt = nullptr;
  ITRY(db.get(&d_cnt, 1, err));
  *nE = 0;
  if (n == 0) return PR_OK;
  size_t tb = 0;
  rocprim::counting_iterator<uint64_t> it(b0);
  IHIP(rocprim::select(nullptr, tb, it, *E, d_cnt, n, LineEnd{B, b1}, s));
  void* tmp = nullptr;
  ITRY(db.get(reinterpret_cast<char**>(&tmp), tb, err));
  IHIP(rocprim::select(tmp, tb, it, *E, d_cnt, n, LineEnd{B, b1}, s));
  IHIP(hipMemcpyAsync(nE, d_cnt, 8, hipMemcpyDeviceToHost, s));
  IHIP(hipStreamSynchronize(s));
  return PR_OK;
}

// lines of a region: one per line end, plus a final unterminated line
uint64_t line_count(uint64_t b0, uint64_t b1, uint64_t nE, uint64_t last_end) {
  if (b1 == b0) return 0;
  if (nE == 0) return 1;
  return nE + (last_end + 1 < b1 ? 1 : 0);
}

// distinct tokens in first-appearance order: number[t] (dense index of t's string), the
// count, and (optionally) each distinct string's first token bytes
int dedupe(const char* B, const uint64_t* off, const uint32_t* len, const uint32_t* tag,
           uint32_t T, DevBufs& db, uint32_t** number, uint32_t* count, uint64_t** f_off,
           uint32_t** f_len, uint32_t** f_tag, hipStream_t s, std::string* err) {
  *count = 0;
  uint64_t cap = 1024;
  while (cap < 2ull * T) cap <<= 1;
  uint32_t *slots, *first, *slot_of, *flag, *rank;
  ITRY(db.get(&slots, cap, err));
  ITRY(db.get(&first, cap, err));
  ITRY(db.get(&slot_of, T, err));
  ITRY(db.get(&flag, T, err));
  ITRY(db.get(&rank, T, err));
  ITRY(db.get(number, T, err));
  if (T == 0) return PR_OK;
  IHIP(hipMemsetAsync(slots, 0, 4 * cap, s));
  IHIP(hipMemsetAsync(first, 0xFF, 4 * cap, s));
  hipLaunchKernelGGL(k_intern, dim3(blocks(T)), dim3(IB), 0, s, B, off, len, tag, T, slots, first, cap - 1, slot_of);
  hipLaunchKernelGGL(k_first_flag, dim3(blocks(T)), dim3(IB), 0, s, slot_of, first, T, flag);
  IHIP(hipGetLastError());
  size_t tb = 0;
  IHIP(rocprim::exclusive_scan(nullptr, tb, flag, rank, 0u, T, rocprim::plus<uint32_t>(), s));
  char* tmp = nullptr;
  ITRY(db.get(&tmp, tb, err));
  IHIP(rocprim::exclusive_scan(tmp, tb, flag, rank, 0u, T, rocprim::plus<uint32_t>(), s));
  hipLaunchKernelGGL(k_number, dim3(blocks(T)), dim3(IB), 0, s, slot_of, first, rank, T, *number);
  IHIP(hipGetLastError());
  uint32_t lr[2];
  IHIP(hipMemcpyAsync(&lr[0], rank + (T - 1), 4, hipMemcpyDeviceToHost, s));
  IHIP(hipMemcpyAsync(&lr[1], flag + (T - 1), 4, hipMemcpyDeviceToHost, s));
  IHIP(hipStreamSynchronize(s));
  *count = lr[0] + lr[1];
  if (f_off) {
    ITRY(db.get(f_off, *count, err));
    ITRY(db.get(f_len, *count, err));
    if (f_tag) ITRY(db.get(f_tag, *count, err));
    hipLaunchKernelGGL(k_firsts, dim3(blocks(T)), dim3(IB), 0, s, flag, rank, off, len, tag, T,
                       *f_off, *f_len, f_tag ? *f_tag : nullptr);
    IHIP(hipGetLastError());
  }
  return PR_OK;
}

template <class T>
int to_host(std::vector<T>* h, const T* d, uint64_t n, hipStream_t s, std::string* err) {
  h->resize(n);
  if (n) IHIP(hipMemcpyAsync(h->data(), d, n * sizeof(T), hipMemcpyDeviceToHost, s));
  return PR_OK;
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
  if (T64 >= (1ull << 30)) {
    if (err) *err = "input too large for the device ingest (>= 2^30 id tokens)";
    return PR_E_ARG;
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
