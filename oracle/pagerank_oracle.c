/*
 * TEST INFRASTRUCTURE ONLY -- dense C restatement of PageRank.java (the oracle).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code,
 * and only as the checker or as the reported CPU baseline ("kind": "port").  It is never
 * linked into, or called by, the product library (libprmi355x.so).
 *
 * PARITY STATUS: parity unpinned against Spark itself -- the reference ships no tests,
 * goldens or recorded topPage, and has no JVM/Spark to run in this image.
 * This file is pinned by the Appendix-B known-answer tests and by bit-exact agreement with
 * the literal-RDD restatement oracle/pagerank_literal.py on thousands of random graphs.
 *
 * What it restates (citations into /root/reference/PageRank.java):
 *   ingest   :26-51   Hadoop TextInputFormat lines, String.split("\t"), ids as exact byte
 *                     strings, distinct arcs, distinct (id,title) pairs, AIOOBE on <2 fields
 *   N_tot    :60      distinct raw mapping lines
 *   dangling :56,64   w[v] = #distinct titles of v when v has no out-edge
 *   iterate  :92-164  dense masked form:
 *                       x = r/outdeg ; a = sum_v w[v] r[v] / N_tot (empty -> crash :125)
 *                       c = A^T x    ; r' = c>0 ? 0.15 + (c + a)*0.85 : 0   (:143)
 *   exact mode: every sum Spark leaves unordered (:125 reduce, :139 reduceByKey(Sum)) is
 *   taken exactly (fixed-point superaccumulator, then one correct rounding).
 *   fast mode: plain fp64 pull loop over OpenMP threads (the CPU baseline).
 *   R-MAT:   Graph500 a/b/c/d = .57/.19/.19/.05 quadrant recursion driven by
 *            Philox-4x32-10 (Salmon et al., SC'11) keyed by (seed, edge index); integer
 *            thresholds so host and device produce bit-identical edge streams.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define ORC_OK 0
#define ORC_E_PARSE (-2)
#define ORC_E_EMPTY_DANGLING (-3)
#define ORC_E_OOM (-6)

/* ------------------------------------------------------------------------------------ */
/* exact summation: 8 x 32-bit chunks (held in u64 for carry room), unit 2^-96           */
/* ------------------------------------------------------------------------------------ */
#define SA_LIMBS 8
#define SA_BASE_EXP (-96)
typedef struct { uint64_t l[SA_LIMBS]; } superacc;

static void sa_zero(superacc* a) { memset(a, 0, sizeof(*a)); }

/* add w * v (v >= 0 finite, w >= 0 integer < 2^32) exactly (bits below 2^-96 truncated) */
static void sa_add_mul(superacc* a, double v, uint32_t w) {
  if (v == 0.0 || w == 0) return;
  uint64_t bits; memcpy(&bits, &v, 8);
  int ebits = (int)((bits >> 52) & 0x7FF);
  uint64_t m = bits & ((1ull << 52) - 1);
  int e;
  if (ebits == 0) { e = -1074; } else { m |= (1ull << 52); e = ebits - 1075; }
  int s = e - SA_BASE_EXP;
  unsigned __int128 q = (unsigned __int128)m * w;
  if (s < 0) { if (-s >= 128) return; q >>= (-s); s = 0; }
  int li = s >> 5, bo = s & 31;
  q <<= bo;
  for (int k = 0; k < 4 && li + k < SA_LIMBS; ++k) {
    a->l[li + k] += (uint64_t)(q & 0xFFFFFFFFu);
    q >>= 32;
  }
}
static void sa_add(superacc* a, double v) { sa_add_mul(a, v, 1u); }
static double sa_to_double(const superacc* in) {
  uint32_t c[SA_LIMBS + 2];
  uint64_t carry = 0;
  for (int i = 0; i < SA_LIMBS; ++i) {
    uint64_t t = in->l[i] + carry;   /* chunks < 2^63 by construction */
    c[i] = (uint32_t)t;
    carry = t >> 32;
  }
  c[SA_LIMBS] = (uint32_t)carry;
  c[SA_LIMBS + 1] = (uint32_t)(carry >> 32);
  const int nl = SA_LIMBS + 2;
  int top = -1;
  for (int i = nl - 1; i >= 0; --i)
    if (c[i]) { top = i * 32 + 31 - __builtin_clz(c[i]); break; }
  if (top < 0) return 0.0;
#define SA_BIT(p) ((p) < 0 ? 0u : ((c[(p) >> 5] >> ((p) & 31)) & 1u))
  if (top < 53) {
    uint64_t m = 0;
    for (int p = top; p >= 0; --p) m = (m << 1) | SA_BIT(p);
    return ldexp((double)m, SA_BASE_EXP);
  }
  uint64_t m = 0;
  for (int p = top; p > top - 53; --p) m = (m << 1) | SA_BIT(p);
  int lowest = top - 52;                  /* weight of m's LSB */
  unsigned rb = SA_BIT(lowest - 1);
  unsigned sticky = 0;
  for (int p = lowest - 2; p >= 0 && !sticky; --p) sticky |= SA_BIT(p);
#undef SA_BIT
  if (rb && (sticky || (m & 1))) {
    m += 1;
    if (m == (1ull << 53)) { m >>= 1; lowest += 1; }
  }
  return ldexp((double)m, lowest + SA_BASE_EXP);
}

/* ------------------------------------------------------------------------------------ */
/* byte-string hash set (first-appearance indices)                                       */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  uint64_t* slots;   /* 0 = empty, else index+1 */
  uint64_t cap;      /* power of two */
  uint64_t n;
  uint64_t* off;     /* per entry: offset into arena */
  uint32_t* len;
  uint64_t ent_cap;
  char* arena;
  uint64_t arena_len, arena_cap;
} strset;

static uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xFF51AFD7ED558CCDull);
  for (size_t i = 0; i < n; ++i) { h ^= (unsigned char)p[i]; h *= 0x100000001B3ull; }
  h ^= h >> 33; h *= 0xC4CEB9FE1A85EC53ull; h ^= h >> 29;
  return h;
}
static int ss_init(strset* s) {
  memset(s, 0, sizeof(*s));
  s->cap = 1024; s->slots = calloc(s->cap, 8);
  s->ent_cap = 512; s->off = malloc(8 * s->ent_cap); s->len = malloc(4 * s->ent_cap);
  s->arena_cap = 1 << 16; s->arena = malloc(s->arena_cap);
  return (s->slots && s->off && s->len && s->arena) ? 0 : -1;
}
static void ss_free(strset* s) { free(s->slots); free(s->off); free(s->len); free(s->arena); }
static const char* ss_get(const strset* s, uint64_t i, size_t* n) { *n = s->len[i]; return s->arena + s->off[i]; }
/* returns index, *is_new set; UINT64_MAX on OOM */
static uint64_t ss_insert(strset* s, const char* p, size_t n, int* is_new) {
  if ((s->n + 1) * 2 > s->cap) {
    uint64_t nc = s->cap * 2; uint64_t* ns = calloc(nc, 8);
    if (!ns) return UINT64_MAX;
    for (uint64_t i = 0; i < s->cap; ++i) if (s->slots[i]) {
      uint64_t idx = s->slots[i] - 1; size_t ln; const char* q = ss_get(s, idx, &ln);
      uint64_t h = hash_bytes(q, ln) & (nc - 1);
      while (ns[h]) h = (h + 1) & (nc - 1);
      ns[h] = s->slots[i];
    }
    free(s->slots); s->slots = ns; s->cap = nc;
  }
  uint64_t h = hash_bytes(p, n) & (s->cap - 1);
  while (s->slots[h]) {
    uint64_t idx = s->slots[h] - 1;
    if (s->len[idx] == n && memcmp(s->arena + s->off[idx], p, n) == 0) { *is_new = 0; return idx; }
    h = (h + 1) & (s->cap - 1);
  }
  if (s->n == s->ent_cap) {
    s->ent_cap *= 2;
    s->off = realloc(s->off, 8 * s->ent_cap); s->len = realloc(s->len, 4 * s->ent_cap);
    if (!s->off || !s->len) return UINT64_MAX;
  }
  while (s->arena_len + n + 1 > s->arena_cap) {
    s->arena_cap *= 2; s->arena = realloc(s->arena, s->arena_cap);
    if (!s->arena) return UINT64_MAX;
  }
  memcpy(s->arena + s->arena_len, p, n);
  s->off[s->n] = s->arena_len; s->len[s->n] = (uint32_t)n;
  s->arena_len += n;
  s->slots[h] = s->n + 1;
  *is_new = 1;
  return s->n++;
}

/* ------------------------------------------------------------------------------------ */
/* graph                                                                                 */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  uint32_t n;            /* dense vertex slots */
  uint64_t m_raw;        /* raw arcs */
  uint64_t nnz;          /* distinct arcs */
  uint64_t n_tot;        /* :60 */
  uint64_t* row_ptr;     /* [n+1] pull CSR by destination */
  uint32_t* col;         /* [nnz] sources, ascending within a row */
  uint32_t* outdeg;      /* [n] */
  uint32_t* indeg;       /* [n] */
  uint32_t* mapw;        /* [n] #distinct titles */
  uint32_t* dang_w;      /* [n] mapw if outdeg==0 else 0 */
  int has_text;
  strset ids;            /* dense id -> bytes (text graphs) */
  uint64_t n_pairs;
  uint32_t* pair_id;     /* distinct (id,title) pairs in first-appearance order */
  uint64_t* pair_title_off;
  uint32_t* pair_title_len;
  char* titles;          /* arena holding titles */
  int err;
  int64_t err_line;      /* 1-based line of the parse error (arcs: +, mapping: -) */
} orc_graph;

static void lsd_sort_u64(uint64_t* a, uint64_t n, int bits) {
  uint64_t* tmp = malloc(8 * (n ? n : 1));
  uint64_t* cnt = malloc(8 * 65536);
  uint64_t *src = a, *dst = tmp;
  for (int sh = 0; sh < bits; sh += 16) {
    memset(cnt, 0, 8 * 65536);
    for (uint64_t i = 0; i < n; ++i) cnt[(src[i] >> sh) & 0xFFFF]++;
    uint64_t s = 0;
    for (int d = 0; d < 65536; ++d) { uint64_t c = cnt[d]; cnt[d] = s; s += c; }
    for (uint64_t i = 0; i < n; ++i) dst[cnt[(src[i] >> sh) & 0xFFFF]++] = src[i];
    uint64_t* t = src; src = dst; dst = t;
  }
  if (src != a) memcpy(a, src, 8 * n);
  free(tmp); free(cnt);
}

/* Parallel sort for large edge lists (R-MAT scale 24-28 in the config tests): one MSD pass on
 * the top 16 significant bits (per-thread histograms, stable scatter), then every bucket is
 * LSD-sorted on the remaining bits by 8-bit digits.  Same result as lsd_sort_u64. */
static void lsd_sort_small(uint64_t* a, uint64_t* tmp, uint64_t n, int bits) {
  uint64_t cnt[256];
  uint64_t *src = a, *dst = tmp;
  for (int sh = 0; sh < bits; sh += 8) {
    memset(cnt, 0, sizeof(cnt));
    for (uint64_t i = 0; i < n; ++i) cnt[(src[i] >> sh) & 0xFF]++;
    uint64_t s = 0;
    for (int d = 0; d < 256; ++d) { uint64_t c = cnt[d]; cnt[d] = s; s += c; }
    for (uint64_t i = 0; i < n; ++i) dst[cnt[(src[i] >> sh) & 0xFF]++] = src[i];
    uint64_t* t = src; src = dst; dst = t;
  }
  if (src != a) memcpy(a, src, 8 * n);
}
static void par_sort_u64(uint64_t* a, uint64_t n, int bits) {
  if (n < (1u << 22) || bits <= 16) { lsd_sort_u64(a, n, bits); return; }
  const int sh = bits - 16;
  const uint64_t NB = 1u << 16;
  int nt = omp_get_max_threads();
  uint64_t* hist = calloc((size_t)nt * NB, 8);
  uint64_t* tmp = malloc(8 * n);
#pragma omp parallel num_threads(nt)
  {
    const int t = omp_get_thread_num();
    const uint64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    uint64_t* h = hist + (size_t)t * NB;
    for (uint64_t i = lo; i < hi; ++i) h[a[i] >> sh]++;
#pragma omp barrier
#pragma omp single
    {
      uint64_t s = 0;
      for (uint64_t b = 0; b < NB; ++b)
        for (int q = 0; q < nt; ++q) { uint64_t c = hist[(size_t)q * NB + b]; hist[(size_t)q * NB + b] = s; s += c; }
    }
    for (uint64_t i = lo; i < hi; ++i) tmp[h[a[i] >> sh]++] = a[i];
  }
  /* after the scatter, thread nt-1's counter of bucket b is the end of bucket b */
  uint64_t* start = malloc(8 * (NB + 1));
  start[0] = 0;
  for (uint64_t b = 0; b < NB; ++b) start[b + 1] = hist[(size_t)(nt - 1) * NB + b];
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t b = 0; b < (int64_t)NB; ++b)
    lsd_sort_small(tmp + start[b], a + start[b], start[b + 1] - start[b], sh);
  memcpy(a, tmp, 8 * n);
  free(start); free(tmp); free(hist);
}

/* keys: (dst<<32 | src) raw edges, consumed */
static int build_csr(orc_graph* g, uint64_t* keys, uint64_t m) {
  int bits = 32;
  while (bits < 64 && ((uint64_t)g->n > (1ull << (bits - 32)))) ++bits;
  par_sort_u64(keys, m, bits);
  uint64_t u = 0;
  for (uint64_t i = 0; i < m; ++i)
    if (i == 0 || keys[i] != keys[i - 1]) keys[u++] = keys[i];
  g->nnz = u;
  g->row_ptr = calloc((size_t)g->n + 1, 8);
  g->col = malloc(4 * (u ? u : 1));
  g->outdeg = calloc(g->n ? g->n : 1, 4);
  g->indeg = calloc(g->n ? g->n : 1, 4);
  g->dang_w = calloc(g->n ? g->n : 1, 4);
  if (!g->row_ptr || !g->col || !g->outdeg || !g->indeg || !g->dang_w) return ORC_E_OOM;
  for (uint64_t i = 0; i < u; ++i) {
    uint32_t d = (uint32_t)(keys[i] >> 32), s = (uint32_t)keys[i];
    g->col[i] = s; g->indeg[d]++; g->outdeg[s]++;
  }
  for (uint32_t v = 0; v < g->n; ++v) g->row_ptr[v + 1] = g->row_ptr[v] + g->indeg[v];
  for (uint32_t v = 0; v < g->n; ++v) g->dang_w[v] = g->outdeg[v] == 0 ? g->mapw[v] : 0;
  return ORC_OK;
}

/* Hadoop line iteration + Java split("\t") semantics (PageRank.java:39-40,47-49) */
typedef struct { const char* p; size_t n; size_t i; } line_iter;
static int next_line(line_iter* it, const char** s, size_t* len) {
  if (it->i >= it->n) return 0;
  size_t st = it->i, i = st;
  while (i < it->n && it->p[i] != '\n' && it->p[i] != '\r') ++i;
  *s = it->p + st; *len = i - st;
  if (i < it->n) { if (it->p[i] == '\r' && i + 1 < it->n && it->p[i + 1] == '\n') ++i; ++i; }
  it->i = i;
  return 1;
}
/* returns 0 ok (key=[ks,kl), val=[vs,vl)), -1 if < 2 fields after trailing-empty strip */
static int split_pair(const char* s, size_t n, const char** ks, size_t* kl, const char** vs, size_t* vl) {
  const char* t = memchr(s, '\t', n);
  if (!t) return -1;
  size_t k = (size_t)(t - s);
  const char* rest = t + 1; size_t rn = n - k - 1;
  size_t j = 0; while (j < rn && rest[j] == '\t') ++j;
  if (j == rn) return -1;              /* every later field empty -> stripped */
  const char* t2 = memchr(rest, '\t', rn);
  *ks = s; *kl = k; *vs = rest; *vl = t2 ? (size_t)(t2 - rest) : rn;
  return 0;
}

void orc_free(orc_graph* g);

orc_graph* orc_from_text(const char* arcs, size_t alen, const char* map, size_t mlen) {
  orc_graph* g = calloc(1, sizeof(orc_graph));
  g->has_text = 1;
  ss_init(&g->ids);
  /* :60 distinct raw mapping lines (counted before anything is parsed) */
  strset lines; ss_init(&lines);
  line_iter it = { map, mlen, 0 }; const char* s; size_t n; int nw;
  while (next_line(&it, &s, &n)) ss_insert(&lines, s, n, &nw);
  g->n_tot = lines.n;
  ss_free(&lines);
  /* :35-42 arcs */
  uint64_t cap = 1024, m = 0;
  uint64_t* keys = malloc(8 * cap);
  it = (line_iter){ arcs, alen, 0 };
  int64_t ln = 0;
  while (next_line(&it, &s, &n)) {
    ++ln;
    const char *ks, *vs; size_t kl, vl;
    if (split_pair(s, n, &ks, &kl, &vs, &vl)) { g->err = ORC_E_PARSE; g->err_line = ln; free(keys); return g; }
    uint32_t a = (uint32_t)ss_insert(&g->ids, ks, kl, &nw);
    uint32_t b = (uint32_t)ss_insert(&g->ids, vs, vl, &nw);
    if (m == cap) { cap *= 2; keys = realloc(keys, 8 * cap); }
    keys[m++] = ((uint64_t)b << 32) | a;
  }
  g->m_raw = m;
  /* :43-51 mapping pairs, distinct */
  strset pairs; ss_init(&pairs);
  uint64_t pcap = 1024; g->pair_id = malloc(4 * pcap);
  it = (line_iter){ map, mlen, 0 }; ln = 0;
  char* buf = malloc(64); size_t bcap = 64;
  while (next_line(&it, &s, &n)) {
    ++ln;
    const char *ks, *vs; size_t kl, vl;
    if (split_pair(s, n, &ks, &kl, &vs, &vl)) { g->err = ORC_E_PARSE; g->err_line = -ln; free(keys); free(buf); ss_free(&pairs); return g; }
    uint32_t id = (uint32_t)ss_insert(&g->ids, ks, kl, &nw);
    if (vl + 4 > bcap) { bcap = vl + 4; buf = realloc(buf, bcap); }
    memcpy(buf, &id, 4); memcpy(buf + 4, vs, vl);
    uint64_t pi = ss_insert(&pairs, buf, vl + 4, &nw);
    if (nw) {
      if (pi == pcap) { pcap *= 2; g->pair_id = realloc(g->pair_id, 4 * pcap); }
      g->pair_id[pi] = id;
    }
  }
  free(buf);
  g->n_pairs = pairs.n;
  g->titles = pairs.arena; pairs.arena = NULL;
  g->pair_title_off = malloc(8 * (pairs.n ? pairs.n : 1));
  g->pair_title_len = malloc(4 * (pairs.n ? pairs.n : 1));
  for (uint64_t i = 0; i < pairs.n; ++i) { g->pair_title_off[i] = pairs.off[i] + 4; g->pair_title_len[i] = pairs.len[i] - 4; }
  ss_free(&pairs);
  g->n = (uint32_t)g->ids.n;
  g->mapw = calloc(g->n ? g->n : 1, 4);
  for (uint64_t i = 0; i < g->n_pairs; ++i) g->mapw[g->pair_id[i]]++;
  g->err = build_csr(g, keys, m);
  free(keys);
  return g;
}

/* in-memory edges (ids are 0..n-1), mapping multiplicity per id, N_tot */
orc_graph* orc_from_edges(const uint32_t* src, const uint32_t* dst, uint64_t m, uint32_t n,
                          const uint32_t* mapw, uint64_t n_tot) {
  orc_graph* g = calloc(1, sizeof(orc_graph));
  g->n = n; g->m_raw = m; g->n_tot = n_tot;
  g->mapw = malloc(4 * (n ? n : 1));
  memcpy(g->mapw, mapw, 4 * (size_t)n);
  uint64_t* keys = malloc(8 * (m ? m : 1));
  for (uint64_t i = 0; i < m; ++i) keys[i] = ((uint64_t)dst[i] << 32) | src[i];
  g->err = build_csr(g, keys, m);
  free(keys);
  return g;
}

/* ---- Philox-4x32-10 + R-MAT ---------------------------------------------------------- */
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
  }
}
/* thresholds floor(p * 2^32) for cumulative a, a+b, a+b+c = .57, .76, .95 */
#define RMAT_TA 2448131358u
#define RMAT_TAB 3264175144u
#define RMAT_TABC 4080218931u
void orc_rmat_edge(uint64_t seed, int scale, uint64_t e, uint32_t* s_out, uint32_t* d_out) {
  uint32_t s = 0, d = 0;
  uint32_t w[4];
  for (int lv = 0; lv < scale; ++lv) {
    if ((lv & 3) == 0) {
      w[0] = (uint32_t)e; w[1] = (uint32_t)(e >> 32); w[2] = (uint32_t)(lv >> 2); w[3] = 0x524D4154u; /* "RMAT" */
      philox4x32_10(w, (uint32_t)seed, (uint32_t)(seed >> 32));
    }
    uint32_t u = w[lv & 3];
    uint32_t sb = u >= RMAT_TAB, db = (u >= RMAT_TA && u < RMAT_TAB) || u >= RMAT_TABC;
    s = (s << 1) | sb; d = (d << 1) | db;
  }
  *s_out = s; *d_out = d;
}
void orc_rmat_edges(uint64_t seed, int scale, uint64_t first, uint64_t count, uint32_t* src, uint32_t* dst) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)count; ++i) orc_rmat_edge(seed, scale, first + (uint64_t)i, &src[i], &dst[i]);
}
orc_graph* orc_from_rmat(int scale, int edge_factor, uint64_t seed) {
  uint32_t n = 1u << scale;
  uint64_t m = (uint64_t)edge_factor << scale;
  uint32_t* s = malloc(4 * m); uint32_t* d = malloc(4 * m);
  orc_rmat_edges(seed, scale, 0, m, s, d);
  uint32_t* w = malloc(4 * (size_t)n);
  for (uint32_t i = 0; i < n; ++i) w[i] = 1;
  orc_graph* g = orc_from_edges(s, d, m, n, w, n);
  free(s); free(d); free(w);
  return g;
}

/* ---- accessors ----------------------------------------------------------------------- */
int orc_error(const orc_graph* g, int64_t* line) { if (line) *line = g->err_line; return g->err; }
uint32_t orc_num_vertices(const orc_graph* g) { return g->n; }
uint64_t orc_nnz(const orc_graph* g) { return g->nnz; }
uint64_t orc_raw_edges(const orc_graph* g) { return g->m_raw; }
uint64_t orc_n_tot(const orc_graph* g) { return g->n_tot; }
uint64_t orc_num_pairs(const orc_graph* g) { return g->n_pairs; }
void orc_degrees(const orc_graph* g, uint32_t* outdeg, uint32_t* indeg, uint32_t* dang_w) {
  if (outdeg) memcpy(outdeg, g->outdeg, 4 * (size_t)g->n);
  if (indeg) memcpy(indeg, g->indeg, 4 * (size_t)g->n);
  if (dang_w) memcpy(dang_w, g->dang_w, 4 * (size_t)g->n);
}
const uint64_t* orc_row_ptr(const orc_graph* g) { return g->row_ptr; }
const uint32_t* orc_col(const orc_graph* g) { return g->col; }
const char* orc_id_bytes(const orc_graph* g, uint32_t v, size_t* len) {
  if (!g->has_text) { *len = 0; return NULL; }
  return ss_get(&g->ids, v, len);
}
void orc_pair(const orc_graph* g, uint64_t i, uint32_t* id, const char** title, size_t* len) {
  *id = g->pair_id[i]; *title = g->titles + g->pair_title_off[i]; *len = g->pair_title_len[i];
}
static uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 31;
  return x;
}
/* order-free digest of the distinct edge set in dense-id space: {sum, xor} of mix64(src<<32|dst) */
void orc_edge_digest(const orc_graph* g, uint64_t out[2]) {
  uint64_t s = 0, x = 0;
  for (uint32_t d = 0; d < g->n; ++d)
    for (uint64_t e = g->row_ptr[d]; e < g->row_ptr[d + 1]; ++e) {
      uint64_t h = mix64(((uint64_t)g->col[e] << 32) | d);
      s += h; x ^= h;
    }
  out[0] = s; out[1] = x;
}

/* ------------------------------------------------------------------------------------ */
/* iteration over a pull CSR (dense masked form)                                         */
/* ------------------------------------------------------------------------------------ */
static double now_s(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }

/* ranks_out[v]: final rank, 0.0 = undefined.  iterations==0 -> r=1 on sources only.
 * exact=1: exact sums; exact=0: plain fp64 (baseline).  tol>0: stop once
 * sum|r'-r| / sum r' <= tol (r^0 = 1 everywhere).  Returns 0 or ORC_E_EMPTY_DANGLING;
 * *iters_done = iterations performed (the failing one included on error). */
/* The general form: r0 = initial rank of every page, base = damping base (1.0 and 0.15 for
 * PageRank.java:78,:143; 1/N_tot and 0.15/N_tot for the normalized option); r_init != NULL
 * starts from those ranks instead (a resumed run). */
int orc_pagerank_csr_ex(uint32_t n, const uint64_t* row_ptr, const uint32_t* col,
                        const uint32_t* outdeg, const uint32_t* dang_w, uint64_t n_tot,
                        int iterations, int exact, int threads, double tol, double r0,
                        double base, const double* r_init, double* ranks_out,
                        double* sec_per_iter, int* iters_done, double* last_resid) {
  if (threads > 0) omp_set_num_threads(threads);
  double* r = ranks_out;
  double* x = malloc(8 * (size_t)(n ? n : 1));
  double* rn = malloc(8 * (size_t)(n ? n : 1));
  for (uint32_t v = 0; v < n; ++v) r[v] = r_init ? r_init[v] : r0;
  int rc = ORC_OK, t = 0;
  double t0 = now_s(), resid = -1.0;
  for (t = 1; t <= iterations; ++t) {
    /* :94-117 contribution vector (one IEEE division per source, same operands as :113) */
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < (int64_t)n; ++v) x[v] = outdeg[v] ? r[v] / (double)outdeg[v] : 0.0;
    /* :121-138 dangling mass */
    double a;
    uint64_t cnt = 0;
    if (exact) {
      superacc acc; sa_zero(&acc);
      for (uint32_t v = 0; v < n; ++v) if (dang_w[v] && r[v] > 0.0) { sa_add_mul(&acc, r[v], dang_w[v]); cnt += dang_w[v]; }
      a = sa_to_double(&acc);
    } else {
      double s = 0.0;
#pragma omp parallel for reduction(+ : s, cnt) schedule(static)
      for (int64_t v = 0; v < (int64_t)n; ++v) if (dang_w[v] && r[v] > 0.0) { s += (double)dang_w[v] * r[v]; cnt += dang_w[v]; }
      a = s;
    }
    if (cnt == 0) { rc = ORC_E_EMPTY_DANGLING; break; }
    const double addthis = a / (double)n_tot;
    /* :139-145 per-destination sum + damping */
    if (exact) {
#pragma omp parallel for schedule(dynamic, 1024)
      for (int64_t d = 0; d < (int64_t)n; ++d) {
        superacc acc; sa_zero(&acc);
        for (uint64_t e = row_ptr[d]; e < row_ptr[d + 1]; ++e) sa_add(&acc, x[col[e]]);
        double c = sa_to_double(&acc);
        rn[d] = c > 0.0 ? base + (c + addthis) * 0.85 : 0.0;
      }
    } else {
#pragma omp parallel for schedule(dynamic, 1024)
      for (int64_t d = 0; d < (int64_t)n; ++d) {
        double c = 0.0;
        for (uint64_t e = row_ptr[d]; e < row_ptr[d + 1]; ++e) c += x[col[e]];
        rn[d] = c > 0.0 ? base + (c + addthis) * 0.85 : 0.0;
      }
    }
    if (tol > 0.0) {
      superacc dr, sr; sa_zero(&dr); sa_zero(&sr);
      for (uint32_t v = 0; v < n; ++v) { sa_add(&dr, fabs(rn[v] - r[v])); sa_add(&sr, rn[v]); }
      double den = sa_to_double(&sr);
      resid = den > 0.0 ? sa_to_double(&dr) / den : 0.0;
    }
    memcpy(r, rn, 8 * (size_t)n);
    if (tol > 0.0 && resid <= tol) { ++t; break; }
  }
  double el = now_s() - t0;
  int done = (rc == ORC_OK) ? t - 1 : t;
  if (iters_done) *iters_done = done;
  if (sec_per_iter) *sec_per_iter = done > 0 ? el / done : 0.0;
  if (last_resid) *last_resid = resid;
  if (iterations == 0 && !r_init) /* the loop never ran: ranks = sources at r0 (:76-83) */
    for (uint32_t v = 0; v < n; ++v) r[v] = outdeg[v] ? r0 : 0.0;
  free(x); free(rn);
  return rc;
}

int orc_pagerank_csr(uint32_t n, const uint64_t* row_ptr, const uint32_t* col,
                     const uint32_t* outdeg, const uint32_t* dang_w, uint64_t n_tot,
                     int iterations, int exact, int threads, double tol,
                     double* ranks_out, double* sec_per_iter, int* iters_done,
                     double* last_resid) {
  return orc_pagerank_csr_ex(n, row_ptr, col, outdeg, dang_w, n_tot, iterations, exact, threads,
                             tol, 1.0, 0.15, NULL, ranks_out, sec_per_iter, iters_done,
                             last_resid);
}

int orc_run(const orc_graph* g, int iterations, int exact, int threads, double tol,
            double* ranks_out, double* sec_per_iter, int* iters_done, double* last_resid) {
  if (g->err) return g->err;
  return orc_pagerank_csr(g->n, g->row_ptr, g->col, g->outdeg, g->dang_w, g->n_tot, iterations,
                          exact, threads, tol, ranks_out, sec_per_iter, iters_done, last_resid);
}

/* normalized: r0 = 1/N_tot, base = 0.15/N_tot; r_init: resume from those ranks */
int orc_run_ex(const orc_graph* g, int iterations, int exact, int threads, double tol,
               int normalized, const double* r_init, double* ranks_out, double* sec_per_iter,
               int* iters_done, double* last_resid) {
  if (g->err) return g->err;
  const double r0 = normalized ? 1.0 / (double)g->n_tot : 1.0;
  const double base = normalized ? 0.15 / (double)g->n_tot : 0.15;
  return orc_pagerank_csr_ex(g->n, g->row_ptr, g->col, g->outdeg, g->dang_w, g->n_tot,
                             iterations, exact, threads, tol, r0, base, r_init, ranks_out,
                             sec_per_iter, iters_done, last_resid);
}

/* exact-sum helper exported for tests: correctly rounded sum of w[i]*v[i] */
double orc_exact_dot_u32(const double* v, const uint32_t* w, uint64_t n) {
  superacc a; sa_zero(&a);
  for (uint64_t i = 0; i < n; ++i) sa_add_mul(&a, v[i], w ? w[i] : 1u);
  return sa_to_double(&a);
}

void orc_free(orc_graph* g) {
  if (!g) return;
  free(g->row_ptr); free(g->col); free(g->outdeg); free(g->indeg); free(g->mapw); free(g->dang_w);
  if (g->has_text) ss_free(&g->ids);
  free(g->pair_id); free(g->pair_title_off); free(g->pair_title_len); free(g->titles);
  free(g);
}
