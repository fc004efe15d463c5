// Device text-scanning helpers shared by the PageRank ingest (ingest.hip) and the TF-IDF job
// (tfidf.hip): line ends, byte-keyed open-addressing interning with first-appearance
// numbering, scratch buffers.  Internal linkage: each translation unit gets its own copy.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include <rocprim/rocprim.hpp>

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

// fold: ASCII letters compare case-insensitively (TF-IDF words are lowercased, Spark.java:39)
__device__ inline unsigned char fold_byte(char c, bool fold) {
  const unsigned char u = static_cast<unsigned char>(c);
  return (fold && u >= 'A' && u <= 'Z') ? static_cast<unsigned char>(u | 0x20) : u;
}

__device__ inline uint64_t hash_span(const char* p, uint32_t n, uint64_t h, bool fold = false) {
  h ^= 0xCBF29CE484222325ull ^ (static_cast<uint64_t>(n) * 0x9E3779B97F4A7C15ull);
  for (uint32_t i = 0; i < n; ++i) h = (h ^ fold_byte(p[i], fold)) * 0x100000001B3ull;
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  return h;
}

__device__ inline bool same_span(const char* B, uint64_t a, uint32_t la, uint64_t b, uint32_t lb,
                                 bool fold = false) {
  if (la != lb) return false;
  for (uint32_t i = 0; i < la; ++i)
    if (fold_byte(B[a + i], fold) != fold_byte(B[b + i], fold)) return false;
  return true;
}

// token t = bytes [off[t], off[t] + len[t]) (and tag[t] when tag != nullptr: pairs are keyed
// by (id, title)); slot_of[t] = its string's slot, first[slot] = smallest token index
__global__ void k_intern(const char* B, const uint64_t* off, const uint32_t* len,
                         const uint32_t* tag, uint32_t T, uint32_t* slots, uint32_t* first,
                         uint64_t mask, uint32_t* slot_of, bool fold) {
  const uint32_t t = blockIdx.x * IB + threadIdx.x;
  if (t >= T) return;
  const uint64_t o = off[t];
  const uint32_t n = len[t];
  const uint32_t g = tag ? tag[t] : 0u;
  uint64_t h = hash_span(B + o, n, tag ? (static_cast<uint64_t>(g) + 1) * 0xD6E8FEB86659FD93ull : 0, fold) & mask;
  for (;;) {
    uint32_t s = __hip_atomic_load(&slots[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 0) {
      s = atomicCAS(&slots[h], 0u, t + 1);
      if (s == 0) break;
    }
    const uint32_t u = s - 1;
    if ((!tag || tag[u] == g) && same_span(B, off[u], len[u], o, n, fold)) break;
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
           uint32_t** f_len, uint32_t** f_tag, hipStream_t s, std::string* err,
           bool fold = false) {
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
  hipLaunchKernelGGL(k_intern, dim3(blocks(T)), dim3(IB), 0, s, B, off, len, tag, T, slots, first, cap - 1, slot_of, fold);
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
}  // namespace prmi
