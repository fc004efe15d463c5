// Host-side graph ingest: the text half of PageRank.java:26-60 (no device code here).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace prmi {

// Byte-string -> dense index table, indices in first-appearance order.
class StrTable {
 public:
  StrTable();
  // Returns the index of [p, p+n); *is_new tells whether it was inserted.
  uint32_t intern(const char* p, size_t n, bool* is_new);
  uint64_t size() const { return off_.size(); }
  const char* get(uint64_t i, size_t* n) const {
    *n = len_[i];
    return arena_.data() + off_[i];
  }
  void reserve(size_t entries, size_t bytes);
  // take over strings already distinct and in index order (the device ingest); the hash
  // index is rebuilt on the next intern()
  void adopt(std::string arena, std::vector<uint64_t> off, std::vector<uint32_t> len);

 private:
  void grow();
  void rehash(size_t cap);
  bool indexed_ = true;
  std::vector<uint64_t> slots_;  // 0 empty, else index + 1
  std::vector<uint64_t> off_;
  std::vector<uint32_t> len_;
  std::string arena_;
};

struct HostGraph {
  bool text = false;              // ids/titles are byte strings from files
  uint32_t n = 0;                 // dense vertex slots
  uint64_t m_raw = 0;             // arc lines / edges
  uint64_t n_tot = 0;             // PageRank.java:60
  std::vector<uint32_t> src, dst; // raw arcs as dense ids (PageRank.java:36-41)
  std::vector<uint32_t> mapw;     // distinct titles per id (PageRank.java:43-51)
  StrTable ids;                   // dense id -> id string (text graphs)
  // distinct (id, title) pairs in first-appearance order (text graphs)
  std::vector<uint32_t> pair_id;
  std::vector<uint64_t> pair_off;
  std::vector<uint32_t> pair_len;
  std::string titles;
  uint64_t n_pairs = 0;           // == pair_id.size() for text graphs; == sum(mapw) otherwise
  // pairs grouped by id (built on the first top-K of a text graph)
  std::vector<uint64_t> pair_first, pairs_by_id;
};

struct ParseError {
  bool failed = false;
  bool in_mapping = false;
  uint64_t line = 0;              // 1-based
  std::string text;
};

// Parse the two reference input files (contents already in memory).
// Returns false and fills *err on a malformed line (the reference's AIOOBE).
bool ingest_text(const char* arcs, size_t alen, const char* map, size_t mlen, HostGraph* g,
                 ParseError* err);

// Java Double.toString (JDK >= 19 shortest-digits layout). Returns length written.
int java_double_to_string(double v, char* buf, size_t cap);

}  // namespace prmi
