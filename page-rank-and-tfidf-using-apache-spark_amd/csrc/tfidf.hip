// The reference's second job, TF-IDF over a tab-separated document dump (Spark.java:22-173;
// SURVEY.md §8f #4), on the device.  Byte model as in ingest.hip.
//
//   1. the dump goes to one device buffer; line ends and tab positions by rocprim::select;
//   2. one thread per line finds columns[1] (title) and columns[3] (text) of s.split("\t")
//      (Spark.java:36-39, :53) from the line's tab positions, or marks the line malformed;
//   3. titles are interned (byte-keyed table, text_device.h): titleCount = distinct titles
//      (:50-56);
//   4. one wave per line cleans the text (:38-42) without rewriting it: a byte is inside a
//      tag "<...>" when the last '<' at or before it follows the last '>' before it and a
//      '>' closes the field after it (exactly the leftmost-first matches of <[^>]*>); a
//      literal backslash-n outside tags becomes a space; a word is a maximal run of ASCII
//      letters that survives, plus the leading "" that split("\\s+") yields when the cleaned
//      text starts with a space (and [""] for an empty text).  Pass 1 counts words per line,
//      pass 2 writes (offset, length, title) tokens at scanned offsets;
//   5. words are interned case-folded (toLowerCase, :40), (word, title) keys are radix
//      sorted and run-length encoded: tf per key (:57-71) and, per word, df = number of
//      titles (:75-93), with the word's keys contiguous;
//   6. a lookup (:140) finds the word on the device and returns its (title, tf) keys; the
//      host evaluates tf * Math.log(titleCount / df) with integer division (:130-131) and
//      sorts (:147-162).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "engine.h"
#include "text_device.h"

namespace prmi {
namespace {

struct IsTab {
  const char* B;
  __device__ bool operator()(const uint64_t& i) const { return B[i] == '\t'; }
};

__device__ inline uint64_t lower_bound_u64(const uint64_t* a, uint64_t n, uint64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (a[m] < v) lo = m + 1; else hi = m;
  }
  return lo;
}

// columns[1] and columns[3] of line k.  Java's split drops trailing empty fields, so
// columns[i] exists iff some byte other than '\t' follows the i-th tab.
// status: 0 ok, 1 no columns[1], 3 no columns[3]; bad_title: the title has no byte other
// than ',' (its key "word,title" then splits into < 2 fields at :106)
__global__ void k_tf_fields(const char* B, const uint64_t* E, uint64_t nE, uint64_t L,
                            uint64_t b1, const uint64_t* tabs, uint64_t ntabs_all,
                            uint64_t* t_off, uint32_t* t_len, uint64_t* x_off, uint32_t* x_len,
                            uint8_t* status, uint8_t* bad_title) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * IB + threadIdx.x;
  if (k >= L) return;
  uint64_t s, e;
  line_bounds(B, E, nE, 0, b1, k, &s, &e);
  const uint64_t a = lower_bound_u64(tabs, ntabs_all, s);
  const uint64_t z = lower_bound_u64(tabs, ntabs_all, e);
  const uint64_t nt = z - a;
  auto after = [&](uint64_t i) {  // a non-tab byte follows tab i (1-based)
    return e - tabs[a + i - 1] - 1 > nt - i;
  };
  uint8_t st = 0;
  if (nt < 1 || !after(1)) st = 1;
  else if (nt < 3 || !after(3)) st = 3;
  status[k] = st;
  t_off[k] = s;
  t_len[k] = 0;
  x_off[k] = s;
  x_len[k] = 0;
  bad_title[k] = 0;
  if (st) return;
  const uint64_t t0 = tabs[a] + 1, t1 = nt >= 2 ? tabs[a + 1] : e;
  const uint64_t x0 = tabs[a + 2] + 1, x1 = nt >= 4 ? tabs[a + 3] : e;
  t_off[k] = t0;
  t_len[k] = static_cast<uint32_t>(t1 - t0);
  x_off[k] = x0;
  x_len[k] = static_cast<uint32_t>(x1 - x0);
  bool comma_only = true;
  for (uint64_t q = t0; q < t1 && comma_only; ++q) comma_only = B[q] == ',';
  bad_title[k] = comma_only ? 1 : 0;
}

__device__ inline bool is_alpha(char c) {
  const unsigned char u = static_cast<unsigned char>(c) | 0x20;
  return u >= 'a' && u <= 'z';
}

__device__ inline int64_t wave_max_incl(int64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(v, d);
    if (lane >= d) v = y > v ? y : v;
  }
  return v;
}

// One wave per line: the words of its cleaned text (Spark.java:38-43).  WRITE = 0 counts
// them into cnt[line]; WRITE = 1 writes tokens from base[line] on.  lead[line] = 1 when the
// first word is the empty string.
template <int WRITE>
__global__ __launch_bounds__(256) void k_tf_words(const char* B, const uint64_t* x_off,
                                                  const uint32_t* x_len, uint64_t L,
                                                  uint32_t* cnt, uint8_t* lead,
                                                  const uint64_t* base, uint64_t* w_off,
                                                  uint32_t* w_len) {
  const int lane = threadIdx.x & 63;
  const uint64_t wid = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 6;
  for (uint64_t l = wid; l < L; l += nw) {
    const int64_t s = static_cast<int64_t>(x_off[l]), e = s + x_len[l];
    uint64_t out = WRITE ? base[l] : 0;
    if (e == s) {  // "".split("\\s+") == [""]
      if (WRITE) {
        if (lane == 0) {
          w_off[out] = static_cast<uint64_t>(s);
          w_len[out] = 0;
        }
      } else if (lane == 0) {
        cnt[l] = 1;
        lead[l] = 1;
      }
      continue;
    }
    // the field's last '>' (a '<' only opens a tag if some '>' follows it)
    int64_t lastgt = -1;
    for (int64_t b = s; b < e; b += 64) {
      const int64_t p = b + lane;
      const uint64_t m = __ballot(p < e && B[p] == '>');
      if (m) lastgt = b + 63 - __builtin_clzll(m);
    }
    int64_t ltc = -1, gtc = -1;       // carries: last '<' / '>' of the previous chunks
    bool letc = false, escc = false;  // previous byte: letter / escape backslash
    bool first_letter = false;
    uint32_t n = 0;
    if (WRITE && lead[l]) {
      if (lane == 0) {
        w_off[out] = static_cast<uint64_t>(s);
        w_len[out] = 0;
      }
      ++out;
    }
    for (int64_t b = s; b < e; b += 64) {
      const int64_t p = b + lane;
      const bool in = p < e;
      const char c = in ? B[p] : 0;
      const char c1 = (p + 1 < e) ? B[p + 1] : 0;
      const int64_t lti = max(ltc, wave_max_incl(in && c == '<' ? p : -1, lane));
      const int64_t gti = max(gtc, wave_max_incl(in && c == '>' ? p : -1, lane));
      int64_t gte = __shfl_up(gti, 1);
      if (lane == 0) gte = gtc;
      const bool masked = in && lti > gte && p <= lastgt;
      // the next byte's tag state, for the backslash-n test
      const int64_t lt1 = max(lti, c1 == '<' ? p + 1 : -1);
      const bool masked1 = (p + 1 < e) && lt1 > gti && p + 1 <= lastgt;
      const bool esc = in && c == '\\' && !masked && c1 == 'n' && !masked1;
      bool esc_prev = __shfl_up(esc ? 1 : 0, 1) != 0;
      if (lane == 0) esc_prev = escc;
      const bool letter = in && !masked && !esc_prev && is_alpha(c);
      bool let_prev = __shfl_up(letter ? 1 : 0, 1) != 0;
      if (lane == 0) let_prev = letc;
      const bool start = letter && !let_prev;
      if (b == s) first_letter = __shfl(letter ? 1 : 0, 0) != 0;
      const uint64_t m = __ballot(start);
      if (WRITE && start) {
        const uint64_t below = lane ? __popcll(m & ((1ull << lane) - 1)) : 0;
        int64_t q = p + 1;
        while (q < e && is_alpha(B[q])) ++q;
        w_off[out + n + below] = static_cast<uint64_t>(p);
        w_len[out + n + below] = static_cast<uint32_t>(q - p);
      }
      n += static_cast<uint32_t>(__popcll(m));
      ltc = __shfl(lti, 63);
      gtc = __shfl(gti, 63);
      letc = __shfl(letter ? 1 : 0, 63) != 0;
      escc = __shfl(esc ? 1 : 0, 63) != 0;
    }
    if (!WRITE && lane == 0) {
      // a cleaned text that starts with a space splits into a leading "" (only if words
      // follow: an all-space text splits into nothing)
      const bool lz = n > 0 && !first_letter;
      cnt[l] = n + (lz ? 1u : 0u);
      lead[l] = lz ? 1 : 0;
    }
  }
}

__global__ void k_tf_keys(const uint32_t* word_no, const uint32_t* line_title,
                          const uint64_t* base, const uint32_t* cnt, uint64_t L, uint64_t* keys) {
  const uint64_t l = static_cast<uint64_t>(blockIdx.x) * IB + threadIdx.x;
  if (l >= L) return;
  const uint64_t t = line_title[l];
  for (uint64_t i = base[l], e = base[l] + cnt[l]; i < e; ++i)
    keys[i] = (static_cast<uint64_t>(word_no[i]) << 32) | t;
}

__global__ void k_tf_find(const char* B, const uint64_t* f_off, const uint32_t* f_len, uint32_t nw,
                          const char* q, uint32_t ql, uint32_t* found) {
  const uint32_t w = blockIdx.x * IB + threadIdx.x;
  if (w >= nw || f_len[w] != ql) return;
  const char* p = B + f_off[w];
  for (uint32_t i = 0; i < ql; ++i)
    if (fold_byte(p[i], true) != static_cast<unsigned char>(q[i])) return;
  atomicMin(found, w);
}

__global__ void k_u32_of_key(const uint64_t* keys, uint64_t n, uint32_t* hi) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * IB + threadIdx.x;
  if (i < n) hi[i] = static_cast<uint32_t>(keys[i] >> 32);
}

}  // namespace

void tf_free(TfidfState* t) {
  for (void* p : {static_cast<void*>(t->B), static_cast<void*>(t->w_off),
                  static_cast<void*>(t->w_len), static_cast<void*>(t->keys),
                  static_cast<void*>(t->tf), static_cast<void*>(t->w_start)})
    if (p) (void)hipFree(p);
  *t = TfidfState();
}

int tf_ingest(TfidfState* t, const char* data, size_t len, TfidfError* te, hipStream_t s,
              std::string* err) {
  tf_free(t);
  te->failed = false;
  DevBufs db;
  char* B = nullptr;
  IHIP(hipMalloc(&B, len + 1));
  t->B = B;
  t->bytes = len;
  if (len) IHIP(hipMemcpyAsync(B, data, len, hipMemcpyHostToDevice, s));
  uint64_t *E, nE;
  ITRY(line_ends(B, 0, len, db, &E, &nE, s, err));
  uint64_t last = 0;
  if (nE) IHIP(hipMemcpyAsync(&last, E + (nE - 1), 8, hipMemcpyDeviceToHost, s));
  // tab positions
  uint64_t *tabs, *d_nt, ntabs = 0;
  ITRY(db.get(&tabs, len, err));
  ITRY(db.get(&d_nt, 1, err));
  if (len) {
    size_t tb = 0;
    rocprim::counting_iterator<uint64_t> it(0);
    IHIP(rocprim::select(nullptr, tb, it, tabs, d_nt, len, IsTab{B}, s));
    char* tmp = nullptr;
    ITRY(db.get(&tmp, tb, err));
    IHIP(rocprim::select(tmp, tb, it, tabs, d_nt, len, IsTab{B}, s));
    IHIP(hipMemcpyAsync(&ntabs, d_nt, 8, hipMemcpyDeviceToHost, s));
  }
  IHIP(hipStreamSynchronize(s));
  const uint64_t L = line_count(0, len, nE, last);
  if (L >= (1ull << 30)) {
    if (err) *err = "too many lines for the device TF-IDF (>= 2^30)";
    return PR_E_ARG;
  }
  t->lines = L;
  uint64_t *t_off, *x_off;
  uint32_t *t_len, *x_len;
  uint8_t *status, *bad;
  ITRY(db.get(&t_off, L, err)); ITRY(db.get(&t_len, L, err));
  ITRY(db.get(&x_off, L, err)); ITRY(db.get(&x_len, L, err));
  ITRY(db.get(&status, L, err)); ITRY(db.get(&bad, L, err));
  if (L) hipLaunchKernelGGL(k_tf_fields, dim3(blocks(L)), dim3(IB), 0, s, B, E, nE, L, static_cast<uint64_t>(len), tabs, ntabs, t_off, t_len, x_off, x_len, status, bad);
  IHIP(hipGetLastError());
  std::vector<uint8_t> hst;
  ITRY(to_host(&hst, status, L, s, err));
  IHIP(hipStreamSynchronize(s));
  // :50-56 (the titles job) dies on a line without columns[1] before anything else runs;
  // then :35-39 on a line without columns[3]
  for (int want : {1, 3}) {
    for (uint64_t k = 0; k < L; ++k)
      if (hst[k] == want) {
        te->failed = true;
        te->index = want;
        te->line = k + 1;
        return PR_E_PARSE;
      }
  }
  // titles
  uint32_t *title_no, n_titles;
  uint64_t* ft_off;
  uint32_t* ft_len;
  ITRY(dedupe(B, t_off, t_len, nullptr, static_cast<uint32_t>(L), db, &title_no, &n_titles, &ft_off, &ft_len, nullptr, s, err));
  t->n_docs = n_titles;
  {
    std::vector<uint64_t> o;
    std::vector<uint32_t> ln;
    ITRY(to_host(&o, ft_off, n_titles, s, err));
    ITRY(to_host(&ln, ft_len, n_titles, s, err));
    IHIP(hipStreamSynchronize(s));
    t->title_off.assign(n_titles + 1, 0);
    t->titles.clear();
    for (uint32_t i = 0; i < n_titles; ++i) {
      t->titles.append(data + o[i], ln[i]);
      t->title_off[i + 1] = t->titles.size();
    }
  }
  // words: count, scan, write
  uint32_t* cnt;
  uint8_t* lead;
  uint64_t* wbase;
  ITRY(db.get(&cnt, L, err)); ITRY(db.get(&lead, L, err)); ITRY(db.get(&wbase, L + 1, err));
  const uint32_t wgrid = static_cast<uint32_t>(std::min<uint64_t>((L + 3) / 4, 65536));
  if (L) hipLaunchKernelGGL((k_tf_words<0>), dim3(wgrid), dim3(256), 0, s, B, x_off, x_len, L, cnt, lead, static_cast<const uint64_t*>(nullptr), static_cast<uint64_t*>(nullptr), static_cast<uint32_t*>(nullptr));
  IHIP(hipGetLastError());
  uint64_t T = 0;
  if (L) {
    size_t tb = 0;
    IHIP(rocprim::exclusive_scan(nullptr, tb, cnt, wbase, uint64_t(0), L + 0, rocprim::plus<uint64_t>(), s));
    char* tmp = nullptr;
    ITRY(db.get(&tmp, tb, err));
    IHIP(rocprim::exclusive_scan(tmp, tb, cnt, wbase, uint64_t(0), L, rocprim::plus<uint64_t>(), s));
    uint64_t lb = 0;
    uint32_t lc = 0;
    IHIP(hipMemcpyAsync(&lb, wbase + (L - 1), 8, hipMemcpyDeviceToHost, s));
    IHIP(hipMemcpyAsync(&lc, cnt + (L - 1), 4, hipMemcpyDeviceToHost, s));
    IHIP(hipStreamSynchronize(s));
    T = lb + lc;
  }
  if (T >= (1ull << 31)) {
    if (err) *err = "too many words for the device TF-IDF (>= 2^31)";
    return PR_E_ARG;
  }
  t->tokens = T;
  // :106 a title with nothing but commas (or empty) in a document that has words
  {
    std::vector<uint8_t> hb;
    std::vector<uint32_t> hc;
    std::vector<uint8_t> hl;
    ITRY(to_host(&hb, bad, L, s, err));
    ITRY(to_host(&hc, cnt, L, s, err));
    ITRY(to_host(&hl, lead, L, s, err));
    IHIP(hipStreamSynchronize(s));
    for (uint64_t k = 0; k < L; ++k)
      if (hb[k] && hc[k]) {
        te->failed = true;
        te->index = hl[k] ? 0 : 1;  // the document's first key: "" + "," + title splits to []
        te->line = k + 1;
        return PR_E_PARSE;
      }
  }
  uint64_t* w_off;
  uint32_t* w_len;
  IHIP(hipMalloc(&w_off, 8 * (T ? T : 1)));
  t->w_off = w_off;
  IHIP(hipMalloc(&w_len, 4 * (T ? T : 1)));
  t->w_len = w_len;
  if (L) hipLaunchKernelGGL((k_tf_words<1>), dim3(wgrid), dim3(256), 0, s, B, x_off, x_len, L, cnt, lead, static_cast<const uint64_t*>(wbase), w_off, w_len);
  IHIP(hipGetLastError());
  // words (case-folded) -> ids; first token of each word kept for lookups
  uint32_t *word_no, n_words;
  uint64_t* fw_off;
  uint32_t* fw_len;
  ITRY(dedupe(B, w_off, w_len, nullptr, static_cast<uint32_t>(T), db, &word_no, &n_words, &fw_off, &fw_len, nullptr, s, err, true));
  t->n_words = n_words;
  // keep the distinct words' first tokens (in place of the token arrays)
  {
    uint64_t* wo;
    uint32_t* wl;
    IHIP(hipMalloc(&wo, 8ull * (n_words ? n_words : 1)));
    IHIP(hipMalloc(&wl, 4ull * (n_words ? n_words : 1)));
    if (n_words) {
      IHIP(hipMemcpyAsync(wo, fw_off, 8ull * n_words, hipMemcpyDeviceToDevice, s));
      IHIP(hipMemcpyAsync(wl, fw_len, 4ull * n_words, hipMemcpyDeviceToDevice, s));
    }
    IHIP(hipStreamSynchronize(s));
    (void)hipFree(t->w_off);
    (void)hipFree(t->w_len);
    t->w_off = wo;
    t->w_len = wl;
  }
  // (word, title) keys -> sorted -> run-length: tf per key
  uint64_t *keys, *ksorted;
  ITRY(db.get(&keys, T, err));
  ITRY(db.get(&ksorted, T, err));
  if (L) hipLaunchKernelGGL(k_tf_keys, dim3(blocks(L)), dim3(IB), 0, s, word_no, title_no, wbase, cnt, L, keys);
  IHIP(hipGetLastError());
  int wb = 1;
  while ((1ull << wb) < n_words) ++wb;
  uint64_t* ukeys;
  uint32_t *tf, *d_np;
  IHIP(hipMalloc(&ukeys, 8 * (T ? T : 1)));
  t->keys = ukeys;
  IHIP(hipMalloc(&tf, 4 * (T ? T : 1)));
  t->tf = tf;
  ITRY(db.get(&d_np, 1, err));
  uint32_t np = 0;
  if (T) {
    size_t tb = 0;
    IHIP(rocprim::radix_sort_keys(nullptr, tb, keys, ksorted, T, 0, 32 + wb, s));
    char* tmp = nullptr;
    ITRY(db.get(&tmp, tb, err));
    IHIP(rocprim::radix_sort_keys(tmp, tb, keys, ksorted, T, 0, 32 + wb, s));
    size_t tb2 = 0;
    IHIP(rocprim::run_length_encode(nullptr, tb2, ksorted, T, ukeys, tf, d_np, s));
    char* tmp2 = nullptr;
    ITRY(db.get(&tmp2, tb2, err));
    IHIP(rocprim::run_length_encode(tmp2, tb2, ksorted, T, ukeys, tf, d_np, s));
    IHIP(hipMemcpyAsync(&np, d_np, 4, hipMemcpyDeviceToHost, s));
    IHIP(hipStreamSynchronize(s));
  }
  t->n_pairs = np;
  // df per word = its keys (word ids are dense and all present); w_start = exclusive scan
  uint32_t* w_start;
  IHIP(hipMalloc(&w_start, 4ull * (n_words + 1)));
  t->w_start = w_start;
  if (np) {
    uint32_t *hi, *uw, *dfc, *d_nu;
    ITRY(db.get(&hi, np, err));
    ITRY(db.get(&uw, np, err));
    ITRY(db.get(&dfc, n_words + 1, err));
    ITRY(db.get(&d_nu, 1, err));
    hipLaunchKernelGGL(k_u32_of_key, dim3(blocks(np)), dim3(IB), 0, s, ukeys, static_cast<uint64_t>(np), hi);
    size_t tb = 0;
    IHIP(rocprim::run_length_encode(nullptr, tb, hi, np, uw, dfc, d_nu, s));
    char* tmp = nullptr;
    ITRY(db.get(&tmp, tb, err));
    IHIP(rocprim::run_length_encode(tmp, tb, hi, np, uw, dfc, d_nu, s));
    IHIP(hipMemsetAsync(dfc + n_words, 0, 4, s));
    size_t tb2 = 0;
    IHIP(rocprim::exclusive_scan(nullptr, tb2, dfc, w_start, 0u, n_words + 1, rocprim::plus<uint32_t>(), s));
    char* tmp2 = nullptr;
    ITRY(db.get(&tmp2, tb2, err));
    IHIP(rocprim::exclusive_scan(tmp2, tb2, dfc, w_start, 0u, n_words + 1, rocprim::plus<uint32_t>(), s));
    uint32_t nu = 0;
    IHIP(hipMemcpyAsync(&nu, d_nu, 4, hipMemcpyDeviceToHost, s));
    IHIP(hipStreamSynchronize(s));
    if (nu != n_words) {
      if (err) *err = "TF-IDF: word ids are not dense";
      return PR_E_HIP;
    }
  } else {
    IHIP(hipMemsetAsync(w_start, 0, 4ull * (n_words + 1), s));
  }
  IHIP(hipStreamSynchronize(s));
  t->ready = true;
  return PR_OK;
}

int tf_lookup(TfidfState* t, const char* word, size_t wlen, std::vector<uint32_t>* titles,
              std::vector<uint32_t>* tfs, uint32_t* df, hipStream_t s, std::string* err) {
  titles->clear();
  tfs->clear();
  *df = 0;
  if (!t->ready || t->n_words == 0) return PR_OK;
  DevBufs db;
  char* q;
  uint32_t* found;
  ITRY(db.get(&q, wlen + 1, err));
  ITRY(db.get(&found, 1, err));
  if (wlen) IHIP(hipMemcpyAsync(q, word, wlen, hipMemcpyHostToDevice, s));
  IHIP(hipMemsetAsync(found, 0xFF, 4, s));
  hipLaunchKernelGGL(k_tf_find, dim3(blocks(t->n_words)), dim3(IB), 0, s, static_cast<const char*>(t->B), static_cast<const uint64_t*>(t->w_off), static_cast<const uint32_t*>(t->w_len), t->n_words, static_cast<const char*>(q), static_cast<uint32_t>(wlen), found);
  IHIP(hipGetLastError());
  uint32_t w = 0;
  IHIP(hipMemcpyAsync(&w, found, 4, hipMemcpyDeviceToHost, s));
  IHIP(hipStreamSynchronize(s));
  if (w == 0xFFFFFFFFu) return PR_OK;  // lookup of an absent key: an empty list
  uint32_t r[2];
  IHIP(hipMemcpyAsync(r, t->w_start + w, 8, hipMemcpyDeviceToHost, s));
  IHIP(hipStreamSynchronize(s));
  const uint32_t n = r[1] - r[0];
  *df = n;
  std::vector<uint64_t> k(n);
  tfs->resize(n);
  if (n) {
    IHIP(hipMemcpyAsync(k.data(), t->keys + r[0], 8ull * n, hipMemcpyDeviceToHost, s));
    IHIP(hipMemcpyAsync(tfs->data(), t->tf + r[0], 4ull * n, hipMemcpyDeviceToHost, s));
  }
  IHIP(hipStreamSynchronize(s));
  titles->resize(n);
  for (uint32_t i = 0; i < n; ++i) (*titles)[i] = static_cast<uint32_t>(k[i]);
  return PR_OK;
}

}  // namespace prmi
