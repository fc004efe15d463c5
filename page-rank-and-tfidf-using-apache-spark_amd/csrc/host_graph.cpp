// Host-side ingest of the reference's two text inputs (PageRank.java:26-60).
//
// Rules:
//   * lines as Hadoop TextInputFormat yields them to spark.textFile (:26,:29): terminators
//     \n, \r, \r\n; a final unterminated line counts; bytes are kept raw (the reference
//     decodes UTF-8, so inputs with malformed UTF-8 may differ -- DESIGN.md);
//   * s.split("\t") then parts[0], parts[1] (:39-40, :47-49): trailing empty fields are
//     dropped, so a line needs a non-tab byte after its first tab, else the job dies with
//     ArrayIndexOutOfBoundsException -> PR_E_PARSE;
//   * ids are exact byte strings ("007" != "7"); dense ids are assigned in first-appearance
//     order over the arcs (src then dst per line), then the mapping ids;
//   * N_tot = number of distinct raw mapping lines (:60), counted on whole lines;
//   * mapw[id] = number of distinct (id, title) pairs (:43-51), the dangling multiplicity
//     of :56 once the id turns out to have no out-edge.
#include "host_graph.h"

#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

namespace prmi {

static inline uint64_t hash_bytes(const char* p, size_t n) {
  // 64-bit FNV-1a over 8-byte words, finalised with a murmur mix.
  uint64_t h = 0xCBF29CE484222325ull ^ (n * 0x9E3779B97F4A7C15ull);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, p + i, 8);
    h = (h ^ w) * 0x100000001B3ull;
    h ^= h >> 29;
  }
  for (; i < n; ++i) h = (h ^ (unsigned char)p[i]) * 0x100000001B3ull;
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  return h;
}

StrTable::StrTable() : slots_(1024, 0) {}

void StrTable::rehash(size_t cap) {
  std::vector<uint64_t> ns(cap, 0);
  for (uint64_t i = 0; i < off_.size(); ++i) {
    uint64_t h = hash_bytes(arena_.data() + off_[i], len_[i]) & (cap - 1);
    while (ns[h]) h = (h + 1) & (cap - 1);
    ns[h] = i + 1;
  }
  slots_.swap(ns);
  indexed_ = true;
}

void StrTable::reserve(size_t entries, size_t bytes) {
  off_.reserve(entries);
  len_.reserve(entries);
  arena_.reserve(bytes);
  size_t cap = slots_.size();
  while (cap < entries * 2) cap *= 2;
  if (cap != slots_.size() || !indexed_) rehash(cap);
}

void StrTable::grow() { rehash(slots_.size() * 2); }

void StrTable::adopt(std::string arena, std::vector<uint64_t> off, std::vector<uint32_t> len) {
  arena_ = std::move(arena);
  off_ = std::move(off);
  len_ = std::move(len);
  slots_.assign(1024, 0);
  indexed_ = false;
}

uint32_t StrTable::intern(const char* p, size_t n, bool* is_new) {
  if (!indexed_) {
    size_t cap = 1024;
    while (cap < (off_.size() + 1) * 2) cap *= 2;
    rehash(cap);
  }
  if ((off_.size() + 1) * 2 > slots_.size()) grow();
  const uint64_t mask = slots_.size() - 1;
  uint64_t h = hash_bytes(p, n) & mask;
  while (uint64_t s = slots_[h]) {
    const uint64_t i = s - 1;
    if (len_[i] == n && std::memcmp(arena_.data() + off_[i], p, n) == 0) {
      *is_new = false;
      return static_cast<uint32_t>(i);
    }
    h = (h + 1) & mask;
  }
  const uint64_t idx = off_.size();
  off_.push_back(arena_.size());
  len_.push_back(static_cast<uint32_t>(n));
  arena_.append(p, n);
  slots_[h] = idx + 1;
  *is_new = true;
  return static_cast<uint32_t>(idx);
}

namespace {

struct Lines {
  const char* p;
  size_t n, i = 0;
  bool next(const char** s, size_t* len) {
    if (i >= n) return false;
    size_t st = i, j = i;
    while (j < n && p[j] != '\n' && p[j] != '\r') ++j;
    *s = p + st;
    *len = j - st;
    if (j < n) {
      if (p[j] == '\r' && j + 1 < n && p[j + 1] == '\n') ++j;
      ++j;
    }
    i = j;
    return true;
  }
};

// parts[0], parts[1] of s.split("\t"); false when fewer than 2 fields survive.
inline bool split_pair(const char* s, size_t n, const char** k, size_t* kl, const char** v,
                       size_t* vl) {
  const char* t = static_cast<const char*>(std::memchr(s, '\t', n));
  if (!t) return false;
  const size_t klen = static_cast<size_t>(t - s);
  const char* rest = t + 1;
  const size_t rn = n - klen - 1;
  size_t j = 0;
  while (j < rn && rest[j] == '\t') ++j;
  if (j == rn) return false;
  const char* t2 = static_cast<const char*>(std::memchr(rest, '\t', rn));
  *k = s;
  *kl = klen;
  *v = rest;
  *vl = t2 ? static_cast<size_t>(t2 - rest) : rn;
  return true;
}

}  // namespace

bool ingest_text(const char* arcs, size_t alen, const char* map, size_t mlen, HostGraph* g,
                 ParseError* err) {
  g->text = true;
  // :60 -- distinct raw mapping lines (an action on unparsed lines)
  {
    StrTable lines;
    Lines it{map, mlen};
    const char* s;
    size_t n;
    bool nw;
    while (it.next(&s, &n)) lines.intern(s, n, &nw);
    g->n_tot = lines.size();
  }
  // :35-41 -- arcs
  {
    g->ids.reserve(alen / 16 + 16, alen / 2 + 16);
    g->src.reserve(alen / 12 + 1);
    g->dst.reserve(alen / 12 + 1);
    Lines it{arcs, alen};
    const char* s;
    size_t n;
    uint64_t ln = 0;
    while (it.next(&s, &n)) {
      ++ln;
      const char *k, *v;
      size_t kl, vl;
      if (!split_pair(s, n, &k, &kl, &v, &vl)) {
        err->failed = true;
        err->in_mapping = false;
        err->line = ln;
        err->text.assign(s, n > 200 ? 200 : n);
        return false;
      }
      bool nw;
      g->src.push_back(g->ids.intern(k, kl, &nw));
      g->dst.push_back(g->ids.intern(v, vl, &nw));
    }
    g->m_raw = g->src.size();
  }
  // :43-51 -- mapping pairs, distinct
  {
    StrTable pairs;
    std::string key;
    Lines it{map, mlen};
    const char* s;
    size_t n;
    uint64_t ln = 0;
    while (it.next(&s, &n)) {
      ++ln;
      const char *k, *v;
      size_t kl, vl;
      if (!split_pair(s, n, &k, &kl, &v, &vl)) {
        err->failed = true;
        err->in_mapping = true;
        err->line = ln;
        err->text.assign(s, n > 200 ? 200 : n);
        return false;
      }
      bool nw;
      const uint32_t id = g->ids.intern(k, kl, &nw);
      key.assign(reinterpret_cast<const char*>(&id), 4);
      key.append(v, vl);
      pairs.intern(key.data(), key.size(), &nw);
      if (nw) {
        g->pair_id.push_back(id);
        g->pair_off.push_back(g->titles.size());
        g->pair_len.push_back(static_cast<uint32_t>(vl));
        g->titles.append(v, vl);
      }
    }
  }
  g->n = static_cast<uint32_t>(g->ids.size());
  g->n_pairs = g->pair_id.size();
  g->mapw.assign(g->n, 0);
  for (uint32_t id : g->pair_id) g->mapw[id]++;
  return true;
}

// ---------------------------------------------------------------------------------------
// Double.toString (PageRank.java:197: page + "\t" + rank).  Digits: the shortest decimal
// that round-trips (std::to_chars), which is what JDK >= 19 prints for normal doubles.
// Layout: plain with >= 1 fractional digit for 1e-3 <= |v| < 1e7, else d.dddE[-]n.
// ---------------------------------------------------------------------------------------
int java_double_to_string(double v, char* buf, size_t cap) {
  std::string out;
  if (v != v) {
    out = "NaN";
  } else if (v == 1.0 / 0.0) {
    out = "Infinity";
  } else if (v == -1.0 / 0.0) {
    out = "-Infinity";
  } else if (v == 0.0) {
    out = std::signbit(v) ? "-0.0" : "0.0";
  } else {
    if (v < 0) out.push_back('-');
    const double a = v < 0 ? -v : v;
    char tmp[64];
    auto res = std::to_chars(tmp, tmp + sizeof(tmp), a, std::chars_format::scientific);
    *res.ptr = 0;
    // tmp = d[.ddd]e[+-]xx
    std::string digits;
    const char* q = tmp;
    for (; *q && *q != 'e'; ++q)
      if (*q != '.') digits.push_back(*q);
    const int exp10 = std::atoi(q + 1);  // value = d.ddd * 10^exp10
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    if (a >= 1e-3 && a < 1e7) {
      const int ip = exp10 + 1;  // digits before the decimal point
      if (ip <= 0) {
        out += "0.";
        out.append(static_cast<size_t>(-ip), '0');
        out += digits;
      } else if (ip >= static_cast<int>(digits.size())) {
        out += digits;
        out.append(static_cast<size_t>(ip) - digits.size(), '0');
        out += ".0";
      } else {
        out += digits.substr(0, ip);
        out += '.';
        out += digits.substr(ip);
      }
    } else {
      out += digits[0];
      out += '.';
      out += digits.size() > 1 ? digits.substr(1) : std::string("0");
      out += 'E';
      out += std::to_string(exp10);
    }
  }
  if (cap) {
    const size_t c = out.size() < cap - 1 ? out.size() : cap - 1;
    std::memcpy(buf, out.data(), c);
    buf[c] = 0;
  }
  return static_cast<int>(out.size());
}

}  // namespace prmi
