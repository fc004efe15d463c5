// prmi355x C ABI (include/prmi355x.h): host runtime around the device engine.
//
// One context = one process = one GPU.  The round loop of PageRank.java:92-164 runs here:
// per round one fused SpMV launch (engine.hip), then -- on more than one rank -- one RCCL
// all-gather of the new contribution vector x' (this replaces the reduceByKey shuffle at
// :139) and one all-gather of the 32-word exact partial record (replaces the driver-side
// reduce at :125), then a one-thread finalize that produces the next round's addthis.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "engine.h"
#include "host_graph.h"
#include "prmi355x.h"

using prmi::DevGraph;
using prmi::HostGraph;

struct pr_ctx {
  pr_opts opts{};
  int device = -1;
  bool has_device = false;
  hipStream_t stream = nullptr;
  std::vector<hipEvent_t> kev;   // spmv-kernel event pairs (first 64 rounds)
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  ncclComm_t comm = nullptr;
  std::string err;
  HostGraph hg;
  bool have_graph = false;
  enum { SRC_NONE, SRC_TEXT, SRC_EDGES, SRC_RMAT } source = SRC_NONE;
  DevGraph dg;
  int last_iters = -1;           // rounds behind the current ranks (-1: no run yet)
  bool host_ranks_valid = false;
  std::vector<double> h_ranks;
  double ms_ingest = 0;
  std::vector<pr_ctx*> group;    // single-process rank group (pr_comm_init_local)
  int seed_rounds = 0;           // pr_set_ranks: rounds behind the seed (0 = no seed)
  prmi::TfidfState tf;           // the TF-IDF job (Spark.java)
  // multi-rank exchange: a comm stream beside the compute stream, chunk events
  hipStream_t comm_stream = nullptr;
  std::vector<hipEvent_t> ev_chunk;
  std::vector<hipEvent_t> ev_pack;  // rank group: chunk k of this member's send buffer is packed
  hipEvent_t ev_rec = nullptr, ev_done = nullptr;
  hipEvent_t ev_x0 = nullptr;     // chunk 0 of this round's x' (the hot prefix) has landed here
  int xchunks = 4;                // PR_XCHUNKS: row-launch chunks of the x' exchange
  int sx_checked = 0;             // sparse exchange: chunk count whose lists the ranks agreed on
  bool sx_ok = false;             //   (RCCL: count matrices compared once, all ranks alike)
  bool ingest_fallback = false;  // last text ingest went to the host parser (too large)
  // caller-staged exchange (pr_comm_init_external / pr_ext_*): the caller moves each
  // round's x slot + exact record between ranks with a transport of its own
  bool external = false;
  int ext_iters = 0, ext_done = 0;
  double ext_tol = 0.0;
  bool ext_tracked = false;
  prmi::IterState ext_hs{};
  std::vector<hipEvent_t> ext_kev;  // SpMV event pairs of the externally exchanged rounds
  // progress of the running (or last) round loop, readable from another thread (pr_progress):
  // rounds whose work has been enqueued, and the event recorded behind each of them
  std::atomic<int> prog_enq{0};
  std::atomic<int> prog_done_hint{0};
  std::vector<hipEvent_t> prog_ev;  // [PROG_EVENTS] ring: round t records prog_ev[(t-1) % PROG_EVENTS]
  // pr_run_static: this device's static scratch (resolved once in pr_create)
  prmi::StaticScratch scratch{};
};

namespace {

int fail(pr_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(c, x)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return fail((c), e_ == hipErrorOutOfMemory ? PR_E_OOM : PR_E_HIP,                \
                  std::string(#x) + ": " + hipGetErrorString(e_));                     \
  } while (0)

#define NCCLCHK(c, x)                                                                  \
  do {                                                                                 \
    ncclResult_t r_ = (x);                                                             \
    if (r_ != ncclSuccess)                                                             \
      return fail((c), PR_E_RCCL, std::string(#x) + ": " + ncclGetErrorString(r_));    \
  } while (0)

int need_device(pr_ctx* c) {
  if (!c) return PR_E_ARG;
  if (!c->has_device) return fail(c, PR_E_NODEV, "context has no device (PR_DEVICE_NONE)");
  HIPCHK(c, hipSetDevice(c->device));
  return PR_OK;
}

int need_graph(pr_ctx* c) {
  if (!c->have_graph) return fail(c, PR_E_ARG, "no graph: call pr_ingest_* / pr_load_edges / pr_generate_rmat first");
  return PR_OK;
}

int need_comm(pr_ctx* c) {
  if (c->opts.n_ranks > 1 && !c->comm && c->group.empty() && !c->external)
    return fail(c, PR_E_ARG, "n_ranks > 1 requires pr_comm_init (or pr_comm_init_external) before building a graph");
  return PR_OK;
}

// Sparse x' exchange (PR_SPARSE_X: 1 = on, the default; 0 = the dense slot exchange): only
// the x' entries a peer's edges reference travel (scale 26: 86 % of a slot at p = 2, 70 % at
// p = 4, 55 % at p = 8).
bool want_sx(const pr_ctx* c) {
  int v = 1;
  if (const char* e = getenv("PR_SPARSE_X")) v = atoi(e);
  return c->opts.n_ranks > 1 && v != 0;
}

// Where the sparse exchange packs a chunk's send buffers (PR_PACKCOMM: 1 = on the comm stream,
// the default; 0 = on the compute stream behind the chunk's rows).  The packs are four short
// launches per round (48 us per rank at 8 ranks, scale 26, against 0.17 ms of row launches);
// only the sends need them, so they run ahead of each chunk's sends and the compute stream goes
// straight on to the next chunk's rows.
bool pack_on_comm() {
  int v = 1;
  if (const char* e = getenv("PR_PACKCOMM")) v = atoi(e);
  return v != 0;
}

// Overlapped exchange (PR_XOVERLAP: 1 = on, the default; 0 = the round-2 schedule): the next
// round's stream launch is cut in two.  Its first part -- every LDS phase and the L2-hot-range
// tasks, almost all of its work -- reads only the hot prefix of each x slot, which travels as
// chunk 0 of the exchange, so it starts as soon as that chunk has landed, while the other chunks,
// the record all-gather and finalize are still under way; the cold-segment tasks and the row
// launch (which needs the new addthis) follow once everything is in.  Needs the slice-major
// layout with LDS blocks (p divides 8); off when a tolerance makes the host read every round.
bool want_overlap(const pr_ctx* c, double tol) {
  int v = 1;
  if (const char* e = getenv("PR_XOVERLAP")) v = atoi(e);
  return c->opts.n_ranks > 1 && v != 0 && tol == 0.0 && prmi::dev_can_split_stream(&c->dg);
}

// RCCL ranks: build the lists, then check once that every rank's receive counts equal its
// peers' send counts (an all-gather of the count matrices); any mismatch anywhere turns the
// sparse exchange off on every rank (a count mismatch inside a grouped send/recv would hang)
int sx_setup_rccl(pr_ctx* c, const std::vector<prmi::XChunk>& plan, bool& sx) {
  DevGraph* g = &c->dg;
  const int p = c->opts.n_ranks, K = static_cast<int>(plan.size());
  if (c->sx_checked == K) {
    sx = c->sx_ok;
    return PR_OK;
  }
  // a rank whose lists fail to build still joins the two collectives below (with a veto), so
  // no rank waits alone; every rank then runs the dense exchange
  std::string e;
  const int prep = prmi::dev_sx_prepare(g, plan, &e);
  const size_t m = static_cast<size_t>(K) * p;
  std::vector<uint64_t> mine(m, 0), all(m * p, 0);
  if (!prep)
    for (size_t i = 0; i < m; ++i) mine[i] = g->sx_so[i + 1] - g->sx_so[i];
  if (prep) fprintf(stderr, "[prmi355x] rank %d: sparse exchange lists: %s\n", c->opts.rank, e.c_str());
  uint64_t *d_cnt = nullptr, *d_flag = nullptr;
  HIPCHK(c, hipMalloc(&d_cnt, 8 * (m + m * p)));
  HIPCHK(c, hipMalloc(&d_flag, 8));
  HIPCHK(c, hipMemcpy(d_cnt, mine.data(), 8 * m, hipMemcpyHostToDevice));
  ncclResult_t nr = ncclAllGather(d_cnt, d_cnt + m, m, ncclUint64, c->comm, c->stream);
  if (nr == ncclSuccess && hipStreamSynchronize(c->stream) == hipSuccess)
    (void)hipMemcpy(all.data(), d_cnt + m, 8 * m * p, hipMemcpyDeviceToHost);
  uint64_t bad = (nr == ncclSuccess && !prep) ? 0 : 1;
  for (int k = 0; k < K && !bad; ++k)
    for (int r = 0; r < p; ++r) {
      if (r == c->opts.rank) continue;
      const size_t me = static_cast<size_t>(k) * p + c->opts.rank, i = static_cast<size_t>(k) * p + r;
      if (all[static_cast<size_t>(r) * m + me] != g->sx_ro[i + 1] - g->sx_ro[i]) bad = 1;
    }
  if (nr == ncclSuccess) {
    (void)hipMemcpy(d_flag, &bad, 8, hipMemcpyHostToDevice);
    nr = ncclAllReduce(d_flag, d_flag, 1, ncclUint64, ncclSum, c->comm, c->stream);
    if (nr == ncclSuccess && hipStreamSynchronize(c->stream) == hipSuccess)
      (void)hipMemcpy(&bad, d_flag, 8, hipMemcpyDeviceToHost);
  }
  (void)hipFree(d_cnt);
  (void)hipFree(d_flag);
  if (nr != ncclSuccess) return fail(c, PR_E_RCCL, std::string("sparse exchange check: ") + ncclGetErrorString(nr));
  if (bad) fprintf(stderr, "[prmi355x] rank %d: sparse exchange lists disagree across ranks; dense exchange\n", c->opts.rank);
  c->sx_checked = K;
  c->sx_ok = bad == 0;
  sx = c->sx_ok;
  return PR_OK;
}

// Progress marks: one event per round behind the round's last enqueued work (a ring; the
// watchdog thread of a caller only looks at recent rounds).  Created before the loop starts,
// never resized while a loop runs.
constexpr int PROG_EVENTS = 256;
int ensure_progress(pr_ctx* c) {
  while (static_cast<int>(c->prog_ev.size()) < PROG_EVENTS) {
    hipEvent_t e;
    HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->prog_ev.push_back(e);
  }
  c->prog_enq.store(0, std::memory_order_release);
  c->prog_done_hint.store(0, std::memory_order_release);
  return PR_OK;
}
int mark_progress(pr_ctx* c, int t, hipStream_t s) {
  HIPCHK(c, hipEventRecord(c->prog_ev[(t - 1) % PROG_EVENTS], s));
  c->prog_enq.store(t, std::memory_order_release);
  return PR_OK;
}

// comm stream + events of the chunked exchange (created on first use)
int ensure_xchg(pr_ctx* c) {
  if (!c->comm_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
  if (!c->ev_rec) HIPCHK(c, hipEventCreateWithFlags(&c->ev_rec, hipEventDisableTiming));
  if (!c->ev_done) HIPCHK(c, hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
  if (!c->ev_x0) HIPCHK(c, hipEventCreateWithFlags(&c->ev_x0, hipEventDisableTiming));
  if (const char* e = getenv("PR_XCHUNKS")) c->xchunks = std::max(1, atoi(e));
  return PR_OK;
}

int build_device(pr_ctx* c, const prmi::BuildInput& in0) {
  std::string e;
  prmi::BuildInput in = in0;
  in.normalized = (c->opts.flags & PR_F_NORMALIZED) != 0;
  c->seed_rounds = 0;
  c->sx_checked = 0;  // a new graph: the sparse-exchange lists are rebuilt and re-checked
  int rc = prmi::dev_build(&c->dg, in, c->stream, &e);
  if (rc) return fail(c, rc, "device build: " + e);
  c->last_iters = -1;
  c->host_ranks_valid = false;
  if ((c->opts.flags & PR_F_VERBOSE) || getenv("PR_VERBOSE"))
    fprintf(stderr, "[prmi355x] rank %d build %.1f ms: n=%u nnz=%llu rows=%u local_rows=%u local_nnz=%llu segments/slice=%u pairs=%llu pieces=%llu tasks=%u streams=%zu row_blocks=%u\n",
            c->opts.rank, c->dg.ms_build, c->dg.n, (unsigned long long)c->dg.nnz, c->dg.R,
            c->dg.lrows, (unsigned long long)c->dg.lnnz, c->dg.nseg,
            (unsigned long long)c->dg.n_pairs, (unsigned long long)c->dg.n_pieces,
            c->dg.ntask, (size_t)c->dg.n_streams, c->dg.nb_rows);
  if ((c->opts.flags & PR_F_VERBOSE) || getenv("PR_VERBOSE")) {
    // algorithmic HBM bytes of one round per array (each array touched once)
    const prmi::DevGraph& g = c->dg;
    const uint64_t xlds = 8ull * prmi::NSLICE * g.nlds * g.hot_h;
    auto U = [](uint64_t v) { return static_cast<unsigned long long>(v); };
    fprintf(stderr, "[prmi355x] rank %d round bytes: col16=%llu col32=%llu bits=%llu task_piece=%llu "
            "x_lds=%llu x_rest=%llu piece_w=%llu piece_r=%llu roff=%llu row_maps=%llu meta=%llu "
            "x_out=%llu n_col16=%llu n_col32=%llu lines=%llu runs=%llu\n",
            c->opts.rank, U(2ull * g.n_col16), U(4ull * g.n_col32), U(g.stream_len / 8),
            U(4ull * (g.ntask + 1ull)), U(std::min<uint64_t>(xlds, 8ull * g.X)),
            U(8ull * g.X - std::min<uint64_t>(xlds, 8ull * g.X)), U(8ull * g.n_pieces),
            U(8ull * g.n_pieces), U(12ull * 64 * g.n_groups),
            U(12ull * g.n_lines + 4ull * g.n_runs + 12ull * g.nb_rows), U(4ull * g.lrows),
            U(8ull * g.lA), U(g.n_col16), U(g.n_col32), U(g.n_lines), U(g.n_runs));
  }
  return PR_OK;
}

bool read_file(const char* path, std::string* out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out->resize(sz > 0 ? static_cast<size_t>(sz) : 0);
  size_t got = sz > 0 ? fread(&(*out)[0], 1, out->size(), f) : 0;
  fclose(f);
  return got == out->size();
}

// Ranks of the last run, on the host, by original vertex id.  Collective (p > 1).
int gather_ranks(pr_ctx* c) {
  if (c->host_ranks_valid) return PR_OK;
  if (c->last_iters < 0) return fail(c, PR_E_ARG, "no completed pr_run");
  int rc = need_device(c);
  if (rc) return rc;
  if (!c->group.empty()) {  // sum every member's scattered rows (one nonzero per page)
    c->h_ranks.assign(c->dg.n, 0.0);
    std::vector<double> part(c->dg.n);
    for (pr_ctx* m : c->group) {
      HIPCHK(c, hipSetDevice(m->device));
      rc = prmi::dev_scatter_ranks(&m->dg, c->last_iters, m->stream);
      if (rc) return fail(c, rc, "scatter ranks");
      if (m->dg.n)
        HIPCHK(c, hipMemcpyAsync(part.data(), m->dg.r_full, 8ull * m->dg.n, hipMemcpyDeviceToHost, m->stream));
      HIPCHK(c, hipStreamSynchronize(m->stream));
      for (uint32_t v = 0; v < m->dg.n; ++v) c->h_ranks[v] += part[v];
    }
    HIPCHK(c, hipSetDevice(c->device));
    c->host_ranks_valid = true;
    return PR_OK;
  }
  rc = prmi::dev_scatter_ranks(&c->dg, c->last_iters, c->stream);
  if (rc) return fail(c, rc, "scatter ranks");
  // (external exchange: this rank's pages only; the caller sums over its ranks)
  if (c->opts.n_ranks > 1 && c->dg.n && !c->external)
    NCCLCHK(c, ncclAllReduce(c->dg.r_full, c->dg.r_full, c->dg.n, ncclFloat64, ncclSum, c->comm, c->stream));
  c->h_ranks.resize(c->dg.n);
  if (c->dg.n)
    HIPCHK(c, hipMemcpyAsync(c->h_ranks.data(), c->dg.r_full, 8ull * c->dg.n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->host_ranks_valid = true;
  return PR_OK;
}

uint64_t pair_count(const pr_ctx* c) {
  if (c->source == pr_ctx::SRC_TEXT) return c->hg.n_pairs;
  if (c->hg.mapw.empty()) return c->dg.n;
  uint64_t s = 0;
  for (uint32_t w : c->hg.mapw) s += w;
  return s;
}

// pair i -> (vertex, title).  Generated / in-memory graphs: title "v<id>" ("v<id>#j" for
// the j-th extra title of an id mapped several times).
struct PairIndex {
  std::vector<uint64_t> first;  // in-memory graphs with mapw: first pair of each vertex
};

void pair_at(const pr_ctx* c, const PairIndex& pi, uint64_t i, uint32_t* v, std::string* title) {
  if (c->source == pr_ctx::SRC_TEXT) {
    *v = c->hg.pair_id[i];
    title->assign(c->hg.titles.data() + c->hg.pair_off[i], c->hg.pair_len[i]);
    return;
  }
  if (c->hg.mapw.empty()) {
    *v = static_cast<uint32_t>(i);
    *title = "v" + std::to_string(i);
    return;
  }
  auto it = std::upper_bound(pi.first.begin(), pi.first.end(), i);
  const uint32_t vv = static_cast<uint32_t>(it - pi.first.begin() - 1);
  *v = vv;
  const uint64_t j = i - pi.first[vv];
  *title = "v" + std::to_string(vv) + (j ? "#" + std::to_string(j) : "");
}

PairIndex make_pair_index(const pr_ctx* c) {
  PairIndex pi;
  if (c->source != pr_ctx::SRC_TEXT && !c->hg.mapw.empty()) {
    pi.first.resize(c->hg.mapw.size() + 1);
    pi.first[0] = 0;
    for (size_t v = 0; v < c->hg.mapw.size(); ++v) pi.first[v + 1] = pi.first[v] + c->hg.mapw[v];
  }
  return pi;
}

// PageRank.java:167-189: ranks.join(mappings) -> (rank,(id,title)) -> sortByKey(false) ->
// take(k).  Ties (unspecified order in Spark) broken by (title bytes, id).
struct TopRow {
  double r;
  uint64_t pair;
  uint32_t v;
};

// Candidates of the whole job: every rank selects on its device (dev_topk_candidates) over
// its own pages; the union holds the global top k (ranks own disjoint pages).
int topk_candidates(pr_ctx* c, uint64_t k, std::vector<uint32_t>* ids, std::vector<double>* rs) {
  if (c->last_iters < 0) return fail(c, PR_E_ARG, "no completed pr_run");
  int rc = need_device(c);
  if (rc) return rc;
  ids->clear();
  rs->clear();
  std::vector<uint32_t> mi;
  std::vector<double> mr;
  std::string err;
  if (!c->group.empty()) {
    for (pr_ctx* m : c->group) {
      HIPCHK(c, hipSetDevice(m->device));
      rc = prmi::dev_scatter_ranks(&m->dg, c->last_iters, m->stream);
      if (!rc) rc = prmi::dev_topk_candidates(&m->dg, k, &mi, &mr, m->stream, &err);
      if (rc) {
        (void)hipSetDevice(c->device);
        return fail(c, rc, "top-K selection: " + err);
      }
      ids->insert(ids->end(), mi.begin(), mi.end());
      rs->insert(rs->end(), mr.begin(), mr.end());
    }
    HIPCHK(c, hipSetDevice(c->device));
    return PR_OK;
  }
  rc = prmi::dev_scatter_ranks(&c->dg, c->last_iters, c->stream);
  if (!rc) rc = prmi::dev_topk_candidates(&c->dg, k, ids, rs, c->stream, &err);
  if (rc) return fail(c, rc, "top-K selection: " + err);
  const int p = c->opts.n_ranks;
  if (p <= 1 || c->external) return PR_OK;  // external exchange: this rank's candidates
  // all-gather the per-rank candidate counts, then the candidates padded to the largest count
  uint64_t* d_cnt = nullptr;
  HIPCHK(c, hipMalloc(&d_cnt, 8ull * p));
  std::vector<uint64_t> cnt(p);
  cnt[c->opts.rank] = ids->size();
  HIPCHK(c, hipMemcpyAsync(d_cnt + c->opts.rank, &cnt[c->opts.rank], 8, hipMemcpyHostToDevice, c->stream));
  ncclResult_t nr = ncclAllGather(d_cnt + c->opts.rank, d_cnt, 1, ncclUint64, c->comm, c->stream);
  if (nr == ncclSuccess) {
    (void)hipMemcpyAsync(cnt.data(), d_cnt, 8ull * p, hipMemcpyDeviceToHost, c->stream);
    (void)hipStreamSynchronize(c->stream);
  }
  (void)hipFree(d_cnt);
  if (nr != ncclSuccess) return fail(c, PR_E_RCCL, std::string("ncclAllGather: ") + ncclGetErrorString(nr));
  const uint64_t M = *std::max_element(cnt.begin(), cnt.end());
  if (M == 0) return PR_OK;
  uint32_t* d_ids = nullptr;
  double* d_rs = nullptr;
  HIPCHK(c, hipMalloc(&d_ids, 4ull * M * p));
  if (hipMalloc(&d_rs, 8ull * M * p) != hipSuccess) {
    (void)hipFree(d_ids);
    return fail(c, PR_E_OOM, "top-K exchange buffers");
  }
  const uint64_t off = static_cast<uint64_t>(c->opts.rank) * M;
  std::vector<uint32_t> ai(M * p);
  std::vector<double> ar(M * p);
  bool ok = true;
  if (!ids->empty()) {
    ok = ok && hipMemcpyAsync(d_ids + off, ids->data(), 4 * ids->size(), hipMemcpyHostToDevice, c->stream) == hipSuccess;
    ok = ok && hipMemcpyAsync(d_rs + off, rs->data(), 8 * rs->size(), hipMemcpyHostToDevice, c->stream) == hipSuccess;
  }
  nr = ncclGroupStart();
  if (nr == ncclSuccess) nr = ncclAllGather(d_ids + off, d_ids, M, ncclUint32, c->comm, c->stream);
  if (nr == ncclSuccess) nr = ncclAllGather(d_rs + off, d_rs, M, ncclFloat64, c->comm, c->stream);
  const ncclResult_t ge = ncclGroupEnd();
  if (nr == ncclSuccess) nr = ge;
  if (nr == ncclSuccess) {
    ok = ok && hipMemcpyAsync(ai.data(), d_ids, 4ull * M * p, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
    ok = ok && hipMemcpyAsync(ar.data(), d_rs, 8ull * M * p, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
  }
  ok = hipStreamSynchronize(c->stream) == hipSuccess && ok;
  (void)hipFree(d_ids);
  (void)hipFree(d_rs);
  if (nr != ncclSuccess) return fail(c, PR_E_RCCL, std::string("ncclAllGather: ") + ncclGetErrorString(nr));
  if (!ok) return fail(c, PR_E_HIP, "top-K exchange copies");
  ids->clear();
  rs->clear();
  for (int q = 0; q < p; ++q)
    for (uint64_t i = 0; i < cnt[q]; ++i) {
      ids->push_back(ai[q * M + i]);
      rs->push_back(ar[q * M + i]);
    }
  return PR_OK;
}

// text graphs: the mapping pairs of every id (pairs grouped by id, in pair order)
void ensure_pairs_by_id(pr_ctx* c) {
  HostGraph& h = c->hg;
  if (h.pair_first.size() == static_cast<size_t>(h.n) + 1) return;
  h.pair_first.assign(static_cast<size_t>(h.n) + 1, 0);
  for (uint32_t id : h.pair_id) h.pair_first[id + 1]++;
  for (uint32_t v = 0; v < h.n; ++v) h.pair_first[v + 1] += h.pair_first[v];
  h.pairs_by_id.resize(h.pair_id.size());
  std::vector<uint64_t> at(h.pair_first.begin(), h.pair_first.end() - 1);
  for (uint64_t i = 0; i < h.pair_id.size(); ++i) h.pairs_by_id[at[h.pair_id[i]]++] = i;
}

int topk_rows(pr_ctx* c, uint32_t k, std::vector<TopRow>* out) {
  out->clear();
  std::vector<uint32_t> ids;
  std::vector<double> rs;
  int rc = topk_candidates(c, k, &ids, &rs);
  if (rc) return rc;
  const PairIndex pi = make_pair_index(c);
  if (c->source == pr_ctx::SRC_TEXT) ensure_pairs_by_id(c);
  std::vector<TopRow> rows;
  for (size_t i = 0; i < ids.size(); ++i) {
    const uint32_t v = ids[i];
    uint64_t b = v, e = v + 1ull;  // the pairs of page v
    if (c->source == pr_ctx::SRC_TEXT) {
      b = c->hg.pair_first[v];
      e = c->hg.pair_first[v + 1];
    } else if (!c->hg.mapw.empty()) {
      b = pi.first[v];
      e = pi.first[v + 1];
    }
    for (uint64_t q = b; q < e; ++q)
      rows.push_back({rs[i], c->source == pr_ctx::SRC_TEXT ? c->hg.pairs_by_id[q] : q, v});
  }
  // rank descending; runs of equal rank (ties) then by (title bytes, page), titles built
  // only for the tied runs that reach into the first k rows
  std::sort(rows.begin(), rows.end(), [](const TopRow& a, const TopRow& b) {
    return a.r != b.r ? a.r > b.r : a.pair < b.pair;
  });
  const size_t kk = std::min<size_t>(k, rows.size());
  std::vector<std::pair<std::string, TopRow>> run;
  for (size_t a = 0; a < kk;) {
    size_t b = a + 1;
    while (b < rows.size() && rows[b].r == rows[a].r) ++b;
    if (b - a > 1) {
      run.clear();
      for (size_t q = a; q < b; ++q) {
        uint32_t vv;
        std::string t;
        pair_at(c, pi, rows[q].pair, &vv, &t);
        run.emplace_back(std::move(t), rows[q]);
      }
      std::sort(run.begin(), run.end(), [](const auto& x, const auto& y) {
        return x.first != y.first ? x.first < y.first : x.second.v < y.second.v;
      });
      for (size_t q = a; q < b; ++q) rows[q] = run[q - a].second;
    }
    a = b;
  }
  rows.resize(kk);
  *out = std::move(rows);
  return PR_OK;
}

}  // namespace

extern "C" {

const char* pr_version(void) {
  static const char v[] = "0.1";
  return v;
}

void pr_opts_default(pr_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->device = PR_DEVICE_FROM_RANK;
  o->n_ranks = 1;
  o->rank = 0;
  o->topk = 100;
}

int pr_create(pr_ctx** out, const pr_opts* opts) {
  if (!out) return PR_E_ARG;
  *out = nullptr;
  pr_ctx* c = new (std::nothrow) pr_ctx();
  if (!c) return PR_E_OOM;
  if (opts) c->opts = *opts; else pr_opts_default(&c->opts);
  if (c->opts.n_ranks < 1 || c->opts.rank < 0 || c->opts.rank >= c->opts.n_ranks) {
    delete c;
    return PR_E_ARG;
  }
  if (c->opts.topk == 0) c->opts.topk = 100;
  c->dg.p = c->opts.n_ranks;
  c->dg.rank = c->opts.rank;
  if (c->opts.device != PR_DEVICE_NONE) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
      delete c;
      return PR_E_HIP;
    }
    c->device = c->opts.device >= 0 ? c->opts.device : c->opts.rank % ndev;
    if (c->device >= ndev || hipSetDevice(c->device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev_start) != hipSuccess || hipEventCreate(&c->ev_stop) != hipSuccess) {
      delete c;
      return PR_E_HIP;
    }
    c->has_device = true;
    // device address of the static scratch (pr_run_static), once per device, here at set-up;
    // a failure only disables that entry point
    std::string e;
    if (prmi::dev_static_scratch(c->device, &c->scratch, &e) != PR_OK) c->scratch = prmi::StaticScratch{};
  }
  *out = c;
  return PR_OK;
}

void pr_destroy(pr_ctx* c) {
  if (!c) return;
  if (c->has_device) {
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    prmi::tf_free(&c->tf);
    prmi::dev_free(&c->dg);
    for (hipEvent_t e : c->kev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_chunk) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_pack) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->prog_ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ext_kev) (void)hipEventDestroy(e);
    if (c->ev_rec) (void)hipEventDestroy(c->ev_rec);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->ev_x0) (void)hipEventDestroy(c->ev_x0);
    if (c->comm_stream) {
      (void)hipStreamSynchronize(c->comm_stream);
      (void)hipStreamDestroy(c->comm_stream);
    }
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->ev_stop) (void)hipEventDestroy(c->ev_stop);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  }
  delete c;
}

const char* pr_last_error(const pr_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pr_comm_unique_id(uint8_t id_out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  if (!id_out) return PR_E_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return PR_E_RCCL;
  std::memcpy(id_out, &id, 128);
  return PR_OK;
}

int pr_comm_init(pr_ctx* c, const uint8_t id[128]) {
  int rc = need_device(c);
  if (rc) return rc;
  if (!id) return fail(c, PR_E_ARG, "null id");
  if (c->comm) return PR_OK;
  if (c->opts.n_ranks == 1) return PR_OK;
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  NCCLCHK(c, ncclCommInitRank(&c->comm, c->opts.n_ranks, uid, c->opts.rank));
  return PR_OK;
}

int pr_comm_init_local(pr_ctx** ctxs, int32_t n) {
  if (!ctxs || n < 1) return PR_E_ARG;
  std::vector<pr_ctx*> g(ctxs, ctxs + n);
  for (int i = 0; i < n; ++i) {
    pr_ctx* c = ctxs[i];
    if (!c || !c->has_device || c->opts.n_ranks != n || c->opts.rank != i || c->comm)
      return c ? fail(c, PR_E_ARG, "local group: member i must have n_ranks = n, rank = i, a device, no RCCL comm") : PR_E_ARG;
  }
  for (int i = 0; i < n; ++i) ctxs[i]->group = g;
  return PR_OK;
}

int pr_run_group(pr_ctx** ctxs, int32_t n, int32_t iterations, double tol, pr_stats* st) {
  prmi::Span span("prmi:run_group");
  if (!ctxs || n < 1) return PR_E_ARG;
  pr_ctx* c0 = ctxs[0];
  for (int i = 0; i < n; ++i) {
    pr_ctx* c = ctxs[i];
    if (!c || static_cast<int>(c->group.size()) != n || c->group[i] != c) return fail(c0, PR_E_ARG, "not a local group");
    int rc = need_graph(c);
    if (rc) return rc;
  }
  if (iterations < 0) return fail(c0, PR_E_ARG, "iterations < 0");
  pr_stats s{};
  s.nnz = c0->dg.nnz;
  s.n_vertices = c0->dg.n;
  s.bytes_per_iter = 4ull * c0->dg.nnz + 24ull * c0->dg.n + 8;
  for (int i = 0; i < n; ++i) {
    ctxs[i]->host_ranks_valid = false;
    ctxs[i]->last_iters = -1;
  }
  auto finish = [&](int done) {
    for (int i = 0; i < n; ++i) ctxs[i]->last_iters = done;
  };
  if (iterations == 0) {
    finish(0);
    if (st) *st = s;
    return PR_OK;
  }
  // every member seeded alike (pr_set_ranks / pr_checkpoint_load on each), as pr_run
  for (int i = 1; i < n; ++i)
    if (ctxs[i]->dg.seeded != c0->dg.seeded || ctxs[i]->seed_rounds != c0->seed_rounds)
      return fail(c0, PR_E_ARG, "local group: members seeded differently (call set_ranks on every member)");
  const int r0 = c0->dg.seeded ? c0->seed_rounds : 0;  // rounds behind the starting ranks
  if (!c0->dg.seeded && c0->dg.W0 == 0) {  // round 1 reduces an empty danglingMap (:125)
    s.failed_iteration = 1;
    if (st) *st = s;
    return fail(c0, PR_E_EMPTY_DANGLING, "java.lang.UnsupportedOperationException: empty collection (iteration 1)");
  }
  const bool tracked = tol > 0.0 || (c0->opts.flags & PR_F_TRACK_RESIDUAL);
  {
    HIPCHK(c0, hipSetDevice(c0->device));
    int rcp = ensure_progress(c0);
    if (rcp) return rcp;
  }
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) {
    HIPCHK(c0, hipSetDevice(ctxs[i]->device));
    int rc = prmi::dev_reset_state(&ctxs[i]->dg, ctxs[i]->stream);
    if (rc) return fail(c0, rc, "reset state");
  }
  int done = iterations;
  prmi::IterState hs{};
  const bool ov = n > 1 && want_overlap(c0, tol);  // the schedule of pr_run, see want_overlap
  // PR_XDELAY_US (measurements only): every chunk's copies start that late on the comm
  // streams, standing in for a transfer time that device copies on one GPU do not have
  int xdelay = 0;
  if (const char* e = getenv("PR_XDELAY_US")) xdelay = std::max(0, atoi(e));
  std::vector<std::vector<prmi::XChunk>> plans(n);
  for (int i = 0; i < n; ++i) {
    pr_ctx* m = ctxs[i];
    HIPCHK(c0, hipSetDevice(m->device));
    int rc = ensure_xchg(m);
    if (rc) return fail(c0, rc, "exchange streams");
    plans[i] = prmi::dev_exchange_plan(&m->dg, m->xchunks, ov);
    while (m->ev_chunk.size() < plans[i].size()) {
      hipEvent_t e;
      HIPCHK(c0, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      m->ev_chunk.push_back(e);
    }
    while (m->ev_pack.size() < plans[i].size()) {
      hipEvent_t e;
      HIPCHK(c0, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      m->ev_pack.push_back(e);
    }
  }
  for (int i = 1; i < n; ++i)
    if (plans[i].size() != plans[0].size()) return fail(c0, PR_E_ARG, "local group: exchange plans differ");
  // sparse exchange: every member's lists, and rank r's send counts to q equal q's receive
  // counts from r for every chunk (the lists of pr_run's RCCL path, checked here on the host)
  const bool sx = n > 1 && want_sx(c0);
  const bool pkc = sx && pack_on_comm();
  if (sx) {
    for (int i = 0; i < n; ++i) {
      HIPCHK(c0, hipSetDevice(ctxs[i]->device));
      std::string e;
      int rc = prmi::dev_sx_prepare(&ctxs[i]->dg, plans[i], &e);
      if (rc) return fail(c0, rc, "sparse exchange: " + e);
    }
    for (size_t k = 0; k < plans[0].size(); ++k)
      for (int r = 0; r < n; ++r)
        for (int q = 0; q < n; ++q) {
          if (q == r) continue;
          const size_t is = k * n + q, ir = k * n + r;
          const DevGraph &gr = ctxs[r]->dg, &gq = ctxs[q]->dg;
          if (gr.sx_so[is + 1] - gr.sx_so[is] != gq.sx_ro[ir + 1] - gq.sx_ro[ir])
            return fail(c0, PR_E_ARG, "sparse exchange: send / receive lists disagree");
        }
  }
  for (int t = 1; t <= iterations; ++t) {
    const int mode = tracked ? 2 : (t == iterations ? 1 : 0);
    prmi::Span round("prmi:round");
    // the schedule of pr_run's chunked exchange, with device copies for ncclSend/Recv: each
    // member's rows run in chunks; member q's comm stream copies chunk k of every peer's
    // slot as soon as that peer's chunk event fires, then the records, then finalize
    for (int i = 0; i < n; ++i) {
      pr_ctx* m = ctxs[i];
      HIPCHK(c0, hipSetDevice(m->device));
      int rc = PR_OK;
      if (ov) {
        if (t > 1) HIPCHK(c0, hipStreamWaitEvent(m->stream, m->ev_x0, 0));
        rc = prmi::dev_round_stream(&m->dg, t, m->stream, nullptr, 1);
        // (every member's ev_done: its copies out of this member's buffers have run too)
        if (t > 1)
          for (int q = 0; q < n; ++q) HIPCHK(c0, hipStreamWaitEvent(m->stream, ctxs[q]->ev_done, 0));
        if (!rc) rc = prmi::dev_round_stream(&m->dg, t, m->stream, nullptr, 2);
      } else {
        rc = prmi::dev_round_stream(&m->dg, t, m->stream, nullptr, 0);
      }
      for (size_t k = 0; !rc && k < plans[i].size(); ++k) {
        rc = prmi::dev_round_rows(&m->dg, t, mode, plans[i][k].b0, plans[i][k].b1, m->stream);
        if (!rc && sx && !pkc) rc = prmi::dev_sx_pack(&m->dg, t, static_cast<int>(k), m->stream);
        if (!rc && hipEventRecord(m->ev_chunk[k], m->stream) != hipSuccess) rc = PR_E_HIP;
      }
      if (!rc) rc = prmi::dev_round_rows(&m->dg, t, mode, m->dg.nb_rows_a, m->dg.nb_rows, m->stream);
      if (!rc) rc = prmi::dev_round_reduce(&m->dg, m->stream, nullptr);
      if (rc) return fail(c0, rc, "round compute");
      HIPCHK(c0, hipEventRecord(m->ev_rec, m->stream));
    }
    // chunk by chunk, as on a rank's comm stream under RCCL: pack (the sender's comm stream),
    // the copies that stand for send / recv, unpack (the receiver's)
    for (size_t k = 0; k < plans[0].size(); ++k) {
      if (pkc)
        for (int r = 0; r < n; ++r) {
          pr_ctx* mr = ctxs[r];
          HIPCHK(c0, hipSetDevice(mr->device));
          HIPCHK(c0, hipStreamWaitEvent(mr->comm_stream, mr->ev_chunk[k], 0));
          int rcp = prmi::dev_sx_pack(&mr->dg, t, static_cast<int>(k), mr->comm_stream);
          if (rcp) return fail(c0, rcp, "sparse exchange pack");
          HIPCHK(c0, hipEventRecord(mr->ev_pack[k], mr->comm_stream));
        }
      for (int q = 0; q < n; ++q) {
        pr_ctx* mq = ctxs[q];
        DevGraph* dst = &mq->dg;
        HIPCHK(c0, hipSetDevice(mq->device));
        // (the event behind which member r's chunk k may be read)
        auto ready = [&](int r) { return pkc ? ctxs[r]->ev_pack[k] : ctxs[r]->ev_chunk[k]; };
        if (xdelay) {
          for (int r = 0; r < n; ++r)
            if (r != q) HIPCHK(c0, hipStreamWaitEvent(mq->comm_stream, ready(r), 0));
          int rcd = prmi::dev_delay_us(xdelay, mq->comm_stream);
          if (rcd) return fail(c0, rcd, "delay kernel");
        }
        for (int r = 0; r < n; ++r) {
          if (r == q) continue;
          DevGraph* src = &ctxs[r]->dg;
          HIPCHK(c0, hipStreamWaitEvent(mq->comm_stream, ready(r), 0));
          if (sx) {  // r's packed entries for q -> q's receive buffer, as ncclSend / ncclRecv
            const size_t is = k * n + q, ir = k * n + r;
            const uint64_t cnt = src->sx_so[is + 1] - src->sx_so[is];
            if (cnt)
              HIPCHK(c0, hipMemcpyPeerAsync(dst->sx_rbuf + dst->sx_ro[ir], mq->device,
                                            src->sx_sbuf + src->sx_so[is], ctxs[r]->device,
                                            8ull * cnt, mq->comm_stream));
            continue;
          }
          const uint64_t base = static_cast<uint64_t>(r) * src->maxA;
          for (const prmi::XPiece& pc : plans[q][k].pieces)
            HIPCHK(c0, hipMemcpyPeerAsync(prmi::dev_x_out(dst, t) + base + pc.off, mq->device,
                                          prmi::dev_x_out(src, t) + base + pc.off, ctxs[r]->device,
                                          8ull * pc.cnt, mq->comm_stream));
        }
        if (sx) {
          int rc = prmi::dev_sx_unpack(dst, t, static_cast<int>(k), mq->comm_stream);
          if (rc) return fail(c0, rc, "sparse exchange unpack");
        }
        if (k == 0) HIPCHK(c0, hipEventRecord(mq->ev_x0, mq->comm_stream));
      }
    }
    for (int q = 0; q < n; ++q) {
      pr_ctx* mq = ctxs[q];
      DevGraph* dst = &mq->dg;
      HIPCHK(c0, hipSetDevice(mq->device));
      for (int r = 0; r < n; ++r) {
        DevGraph* src = &ctxs[r]->dg;
        HIPCHK(c0, hipStreamWaitEvent(mq->comm_stream, ctxs[r]->ev_rec, 0));
        HIPCHK(c0, hipMemcpyPeerAsync(dst->rec_all + static_cast<uint64_t>(r) * prmi::REC_WORDS,
                                      mq->device, src->rec_local, ctxs[r]->device,
                                      8ull * prmi::REC_WORDS, mq->comm_stream));
      }
      int rc = prmi::dev_round_finalize(dst, t, tracked, mq->comm_stream);
      if (rc) return fail(c0, rc, "round finalize");
      HIPCHK(c0, hipEventRecord(mq->ev_done, mq->comm_stream));
    }
    // round t+1 starts once every member has its x' and a (and every copy out of this
    // member's slot has run, so the slot may be rewritten two rounds later)
    if (!ov || t == iterations)
      for (int i = 0; i < n; ++i) {
        HIPCHK(c0, hipSetDevice(ctxs[i]->device));
        for (int q = 0; q < n; ++q) HIPCHK(c0, hipStreamWaitEvent(ctxs[i]->stream, ctxs[q]->ev_done, 0));
      }
    {
      HIPCHK(c0, hipSetDevice(c0->device));
      int rcp = mark_progress(c0, t, ov ? c0->comm_stream : c0->stream);
      if (rcp) return rcp;
    }
    if (tol == 0.0) continue;
    HIPCHK(c0, hipMemcpyAsync(&hs, c0->dg.state, sizeof(hs), hipMemcpyDeviceToHost, c0->stream));
    HIPCHK(c0, hipStreamSynchronize(c0->stream));
    if (tol > 0.0 && hs.resid <= tol) {
      done = t;
      break;
    }
  }
  for (int i = 0; i < n; ++i) {
    HIPCHK(c0, hipSetDevice(ctxs[i]->device));
    HIPCHK(c0, hipStreamSynchronize(ctxs[i]->stream));
    HIPCHK(c0, hipStreamSynchronize(ctxs[i]->comm_stream));
  }
  HIPCHK(c0, hipSetDevice(c0->device));
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  HIPCHK(c0, hipMemcpyAsync(&hs, c0->dg.state, sizeof(hs), hipMemcpyDeviceToHost, c0->stream));
  HIPCHK(c0, hipStreamSynchronize(c0->stream));
  s.iterations = done;
  s.ms_total = ms;
  s.ms_per_iter = ms / done;
  s.gteps = static_cast<double>(c0->dg.nnz) / (s.ms_per_iter * 1e-3) / 1e9;
  s.residual = tracked ? hs.resid : 0.0;
  s.rank_sum = tracked ? hs.rank_sum : 0.0;
  if (hs.err_iter != 0 && hs.err_iter <= done) {
    s.failed_iteration = r0 + hs.err_iter;
    if (st) *st = s;
    return fail(c0, PR_E_EMPTY_DANGLING,
                "java.lang.UnsupportedOperationException: empty collection (iteration " +
                    std::to_string(r0 + hs.err_iter) + ")");
  }
  finish(done);
  if (st) *st = s;
  return PR_OK;
}

int pr_comm_init_external(pr_ctx* c) {
  int rc = need_device(c);
  if (rc) return rc;
  if (c->comm || !c->group.empty()) return fail(c, PR_E_ARG, "context already has a transport");
  if (c->opts.n_ranks < 2) return fail(c, PR_E_ARG, "external exchange needs n_ranks > 1");
  c->external = true;
  return PR_OK;
}

int pr_ext_begin(pr_ctx* c, int32_t iterations, double tol, uint64_t* bytes_per_rank) {
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  if (!c->external) return fail(c, PR_E_ARG, "pr_ext_* needs pr_comm_init_external");
  if (iterations < 1) return fail(c, PR_E_ARG, "iterations < 1");
  DevGraph* g = &c->dg;
  if (!g->seeded && g->W0 == 0) return fail(c, PR_E_EMPTY_DANGLING, "java.lang.UnsupportedOperationException: empty collection (iteration 1)");
  c->ext_iters = iterations;
  c->ext_done = 0;
  c->ext_tol = tol;
  c->ext_tracked = tol > 0.0 || (c->opts.flags & PR_F_TRACK_RESIDUAL);
  c->ext_hs = prmi::IterState{};
  c->host_ranks_valid = false;
  c->last_iters = -1;
  const int nk = std::min(iterations, 64);
  while (static_cast<int>(c->ext_kev.size()) < 2 * nk) {
    hipEvent_t e;
    HIPCHK(c, hipEventCreate(&e));
    c->ext_kev.push_back(e);
  }
  rc = ensure_progress(c);
  if (rc) return rc;
  rc = prmi::dev_reset_state(g, c->stream);
  if (rc) return fail(c, rc, "reset state");
  if (bytes_per_rank) *bytes_per_rank = 8ull * g->maxA + 8ull * prmi::REC_WORDS;
  return PR_OK;
}

int pr_ext_round(pr_ctx* c, int32_t t, void* send) {
  prmi::Span span("prmi:ext_round");
  int rc = need_device(c);
  if (rc) return rc;
  if (!c->external || t != c->ext_done + 1 || t > c->ext_iters || !send)
    return fail(c, PR_E_ARG, "pr_ext_round: call pr_ext_begin, then rounds 1, 2, ... in order");
  DevGraph* g = &c->dg;
  const int mode = c->ext_tracked ? 2 : (t == c->ext_iters ? 1 : 0);
  const bool timed = 2 * t <= static_cast<int>(c->ext_kev.size());
  rc = prmi::dev_round_compute(g, t, mode, c->stream, timed ? c->ext_kev[2 * (t - 1)] : nullptr,
                               timed ? c->ext_kev[2 * (t - 1) + 1] : nullptr);
  if (rc) return fail(c, rc, "round compute");
  // this rank's slot of x' and its exact record, in that order
  char* out = static_cast<char*>(send);
  const double* xs = prmi::dev_x_out(g, t) + static_cast<uint64_t>(g->rank) * g->maxA;
  if (g->maxA) HIPCHK(c, hipMemcpyAsync(out, xs, 8ull * g->maxA, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(out + 8ull * g->maxA, g->rec_local, 8ull * prmi::REC_WORDS, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PR_OK;
}

int pr_ext_complete(pr_ctx* c, int32_t t, const void* recv_all, int32_t* stop) {
  prmi::Span span("prmi:ext_complete");
  int rc = need_device(c);
  if (rc) return rc;
  if (!c->external || t != c->ext_done + 1 || !recv_all)
    return fail(c, PR_E_ARG, "pr_ext_complete: after pr_ext_round of the same round");
  DevGraph* g = &c->dg;
  const int p = c->opts.n_ranks;
  const uint64_t unit = 8ull * g->maxA + 8ull * prmi::REC_WORDS;
  const char* in = static_cast<const char*>(recv_all);
  double* xf = prmi::dev_x_out(g, t);
  for (int r = 0; r < p; ++r) {
    if (r != g->rank && g->maxA)
      HIPCHK(c, hipMemcpyAsync(xf + static_cast<uint64_t>(r) * g->maxA, in + r * unit, 8ull * g->maxA, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(g->rec_all + static_cast<uint64_t>(r) * prmi::REC_WORDS, in + r * unit + 8ull * g->maxA, 8ull * prmi::REC_WORDS, hipMemcpyHostToDevice, c->stream));
  }
  rc = prmi::dev_round_finalize(g, t, c->ext_tracked, c->stream);
  if (rc) return fail(c, rc, "round finalize");
  HIPCHK(c, hipMemcpyAsync(&c->ext_hs, g->state, sizeof(c->ext_hs), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->ext_done = t;
  c->prog_enq.store(t, std::memory_order_release);       // (the stream was synchronized above)
  c->prog_done_hint.store(t, std::memory_order_release);
  const bool conv = c->ext_tol > 0.0 && c->ext_hs.resid <= c->ext_tol;
  if (stop) *stop = conv ? 1 : 0;
  // the reduce of a round (PageRank.java:125) saw an empty danglingMap: the job dies there
  if (c->ext_hs.err_iter != 0 && c->ext_hs.err_iter <= t) {
    const int t0 = g->seeded ? c->seed_rounds : 0;
    if (stop) *stop = 1;
    return fail(c, PR_E_EMPTY_DANGLING,
                "java.lang.UnsupportedOperationException: empty collection (iteration " +
                    std::to_string(t0 + c->ext_hs.err_iter) + ")");
  }
  return PR_OK;
}

int pr_ext_end(pr_ctx* c, pr_stats* st) {
  if (!c) return PR_E_ARG;
  if (!c->external || c->ext_done < 1) return fail(c, PR_E_ARG, "pr_ext_end: no completed round");
  pr_stats s{};
  s.nnz = c->dg.nnz;
  s.n_vertices = c->dg.n;
  s.iterations = c->ext_done;
  {  // average SpMV time of the rounds that carried events (the first 64)
    double kms = 0.0;
    int nm = 0;
    for (int t = 0; t < c->ext_done && 2 * t + 1 < static_cast<int>(c->ext_kev.size()); ++t) {
      float k = 0.f;
      if (hipEventElapsedTime(&k, c->ext_kev[2 * t], c->ext_kev[2 * t + 1]) == hipSuccess) {
        kms += k;
        ++nm;
      }
    }
    s.ms_spmv_kernel = nm ? kms / nm : 0.0;
  }
  s.residual = c->ext_tracked ? c->ext_hs.resid : 0.0;
  s.rank_sum = c->ext_tracked ? c->ext_hs.rank_sum : 0.0;
  c->last_iters = c->ext_done;
  c->host_ranks_valid = false;
  if (st) *st = s;
  return PR_OK;
}

int pr_ingest_buffers(pr_ctx* c, const char* arcs, size_t alen, const char* map, size_t mlen) {
  prmi::Span span("prmi:ingest");
  if (!c || (!arcs && alen) || (!map && mlen)) return fail(c, PR_E_ARG, "bad buffers");
  int rc = need_comm(c);
  if (rc) return rc;
  auto t0 = std::chrono::steady_clock::now();
  c->hg = HostGraph();
  c->have_graph = false;
  c->ingest_fallback = false;
  prmi::ParseError pe;
  bool parsed = true;
  if (c->has_device) {  // device ingest (ingest.hip); host parser for host-only contexts
    std::string err;
    HIPCHK(c, hipSetDevice(c->device));
    rc = prmi::dev_ingest_text(arcs ? arcs : "", alen, map ? map : "", mlen, &c->hg, &pe, c->stream, &err);
    if (rc == prmi::INGEST_NOFIT || rc == PR_E_OOM) {
      // too large for the device tables / line index: the host parser has no such limit
      if ((c->opts.flags & PR_F_VERBOSE) || getenv("PR_VERBOSE"))
        fprintf(stderr, "[prmi355x] device ingest: %s; parsing on the host\n", err.c_str());
      (void)hipGetLastError();
      c->hg = HostGraph();
      parsed = prmi::ingest_text(arcs ? arcs : "", alen, map ? map : "", mlen, &c->hg, &pe);
      c->ingest_fallback = true;
    } else if (rc == PR_E_PARSE) {
      parsed = false;
    } else if (rc) {
      c->hg = HostGraph();
      return fail(c, rc, "device ingest: " + err);
    }
  } else {
    parsed = prmi::ingest_text(arcs ? arcs : "", alen, map ? map : "", mlen, &c->hg, &pe);
  }
  if (!parsed) {
    c->hg = HostGraph();
    return fail(c, PR_E_PARSE,
                std::string("java.lang.ArrayIndexOutOfBoundsException: 1 (") +
                    (pe.in_mapping ? "mapping" : "arcs") + " line " + std::to_string(pe.line) +
                    ": \"" + pe.text + "\")");
  }
  c->ms_ingest = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  c->source = pr_ctx::SRC_TEXT;
  if (c->has_device) {
    prmi::BuildInput in;
    in.n = c->hg.n;
    in.m = c->hg.m_raw;
    in.n_tot = c->hg.n_tot;
    in.h_src = c->hg.src.data();
    in.h_dst = c->hg.dst.data();
    in.h_mapw = c->hg.mapw.data();
    rc = build_device(c, in);
    if (rc) return rc;
    // raw edge lists are no longer needed on the host
    std::vector<uint32_t>().swap(c->hg.src);
    std::vector<uint32_t>().swap(c->hg.dst);
  }
  c->have_graph = true;
  return PR_OK;
}

int pr_ingest_files(pr_ctx* c, const char* arcs_path, const char* mapping_path) {
  if (!c || !arcs_path || !mapping_path) return fail(c, PR_E_ARG, "null path");
  std::string a, m;
  if (!read_file(arcs_path, &a)) return fail(c, PR_E_IO, std::string("cannot read ") + arcs_path);
  if (!read_file(mapping_path, &m)) return fail(c, PR_E_IO, std::string("cannot read ") + mapping_path);
  return pr_ingest_buffers(c, a.data(), a.size(), m.data(), m.size());
}

int pr_load_edges(pr_ctx* c, const uint32_t* src, const uint32_t* dst, uint64_t m, uint32_t n,
                  const uint32_t* mapw, uint64_t n_tot) {
  if (!c || (m && (!src || !dst))) return fail(c, PR_E_ARG, "bad edge arrays");
  int rc = need_comm(c);
  if (rc) return rc;
  for (uint64_t i = 0; i < m; ++i)
    if (src[i] >= n || dst[i] >= n) return fail(c, PR_E_ARG, "edge endpoint >= n");
  c->hg = HostGraph();
  c->have_graph = false;
  c->hg.n = n;
  c->hg.m_raw = m;
  if (mapw) {
    c->hg.mapw.assign(mapw, mapw + n);
    c->hg.n_tot = n_tot;
  } else {
    c->hg.n_tot = n_tot ? n_tot : n;
  }
  c->source = pr_ctx::SRC_EDGES;
  if (c->has_device) {
    prmi::BuildInput in;
    in.n = n;
    in.m = m;
    in.n_tot = c->hg.n_tot;
    in.h_src = src;
    in.h_dst = dst;
    in.h_mapw = mapw;
    rc = build_device(c, in);
    if (rc) return rc;
  }
  c->have_graph = true;
  return PR_OK;
}

int pr_generate_rmat(pr_ctx* c, int32_t scale, int32_t edge_factor, uint64_t seed) {
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_comm(c);
  if (rc) return rc;
  if (scale < 1 || scale > 31 || edge_factor < 1) return fail(c, PR_E_ARG, "bad R-MAT size");
  c->hg = HostGraph();
  c->have_graph = false;
  c->hg.n = 1u << scale;
  c->hg.m_raw = static_cast<uint64_t>(edge_factor) << scale;
  c->hg.n_tot = c->hg.n;
  c->source = pr_ctx::SRC_RMAT;
  prmi::BuildInput in;
  in.n = c->hg.n;
  in.m = c->hg.m_raw;
  in.n_tot = c->hg.n_tot;
  in.rmat = true;
  in.scale = scale;
  in.edge_factor = edge_factor;
  in.seed = seed;
  rc = build_device(c, in);
  if (rc) return rc;
  c->have_graph = true;
  return PR_OK;
}

int pr_graph_get_info(pr_ctx* c, pr_graph_info* o) {
  if (!c || !o) return PR_E_ARG;
  int rc = need_graph(c);
  if (rc) return rc;
  std::memset(o, 0, sizeof(*o));
  o->n_vertices = c->hg.n;
  o->raw_edges = c->hg.m_raw;
  o->n_tot = c->hg.n_tot;
  o->n_pairs = pair_count(c);
  o->ms_ingest = c->ms_ingest;
  o->ingest_flags = c->ingest_fallback ? 1u : 0u;
  if (c->has_device) {
    o->nnz = c->dg.nnz;
    o->dangling_entries = c->dg.n_dang_entries;
    o->n_sources = static_cast<uint64_t>(c->dg.nA) + c->dg.nC;
    o->n_rows = c->dg.R;
    o->local_rows = c->dg.lrows;
    o->local_nnz = c->dg.lnnz;
    o->ms_build = c->dg.ms_build;
    o->place_tried = static_cast<uint64_t>(c->dg.place_tried);
    o->place_ms_first = c->dg.place_ms_first;
    o->place_ms_best = c->dg.place_ms_best;
  }
  return PR_OK;
}

int pr_run(pr_ctx* c, int32_t iterations, double tol, pr_stats* st) {
  prmi::Span span("prmi:run");
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  if (iterations < 0) return fail(c, PR_E_ARG, "iterations < 0");
  if (!c->group.empty()) return pr_run_group(c->group.data(), static_cast<int32_t>(c->group.size()), iterations, tol, st);
  if (c->external) return fail(c, PR_E_ARG, "externally exchanged context: drive the rounds with pr_ext_*");
  DevGraph* g = &c->dg;
  pr_stats s{};
  s.nnz = g->nnz;
  s.n_vertices = g->n;
  s.bytes_per_iter = 4ull * g->nnz + 24ull * g->n + 8;
  c->host_ranks_valid = false;
  c->last_iters = -1;
  if (iterations == 0) {  // the loop never runs: ranks = 1.0 on sources (PageRank.java:76-83)
    c->last_iters = 0;
    if (st) *st = s;
    return PR_OK;
  }
  const int t0 = g->seeded ? c->seed_rounds : 0;  // rounds behind the starting ranks
  if (!g->seeded && g->W0 == 0) {  // round 1 reduces an empty danglingMap (PageRank.java:125)
    s.failed_iteration = 1;
    if (st) *st = s;
    return fail(c, PR_E_EMPTY_DANGLING, "java.lang.UnsupportedOperationException: empty collection (iteration 1)");
  }
  const bool tracked = tol > 0.0 || (c->opts.flags & PR_F_TRACK_RESIDUAL);
  const int nk = std::min(iterations, 64);
  while (static_cast<int>(c->kev.size()) < 4 * nk) {  // per round: [A0, A1, B0, B1]
    hipEvent_t e;
    HIPCHK(c, hipEventCreate(&e));
    c->kev.push_back(e);
  }
  int done = iterations;
  prmi::IterState hs{};
  const int p = c->opts.n_ranks;
  std::vector<prmi::XChunk> plan;
  bool sx = false;  // sparse x' exchange this run
  const bool ov = want_overlap(c, tol);
  const bool pkc = pack_on_comm();
  if (p > 1) {  // (before ev_start: list building and its collectives are set-up, not rounds)
    rc = ensure_xchg(c);
    if (rc) return rc;
    plan = prmi::dev_exchange_plan(g, c->xchunks, ov);
    while (c->ev_chunk.size() < plan.size()) {
      hipEvent_t e;
      HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      c->ev_chunk.push_back(e);
    }
    if (want_sx(c)) {
      rc = sx_setup_rccl(c, plan, sx);
      if (rc) return rc;
    }
  }
  rc = ensure_progress(c);
  if (rc) return rc;
  rc = prmi::dev_reset_state(g, c->stream);
  if (rc) return fail(c, rc, "reset state");
  HIPCHK(c, hipEventRecord(c->ev_start, c->stream));
  for (int t = 1; t <= iterations; ++t) {
    const int mode = tracked ? 2 : (t == iterations ? 1 : 0);
    prmi::Span round("prmi:round");
    hipEvent_t e0 = t <= nk ? c->kev[4 * (t - 1)] : nullptr;      // stream launch (part 1)
    hipEvent_t eA1 = t <= nk ? c->kev[4 * (t - 1) + 1] : nullptr;  // overlapped: end of part 1
    hipEvent_t eB0 = t <= nk ? c->kev[4 * (t - 1) + 2] : nullptr;  //   and start of part 2
    hipEvent_t e1 = t <= nk ? c->kev[4 * (t - 1) + 3] : nullptr;   // end of the row launch
    if (p == 1) {
      rc = prmi::dev_round_single(g, t, mode, tracked, c->stream, e0, e1);
      if (rc) return fail(c, rc, "round");
    } else {
      // Chunked exchange replacing the reduceByKey shuffle (PageRank.java:139): the row
      // launch runs in chunks of class-A row blocks; as chunk k's x' slot pieces are final,
      // the comm stream sends them to every peer (grouped ncclSend/ncclRecv over xGMI, one
      // direct link per peer) while the compute stream runs the next chunk.  The exact
      // records are all-gathered after the last rows and finalize runs on the comm stream.
      // The next round's stream launch waits for all of that, or (overlapped, want_overlap)
      // its first part only for chunk 0.
      double* xf = prmi::dev_x_out(g, t);
      if (ov) {
        // part 1 needs chunk 0 of the last round only; part 2 and the rows need the rest of
        // x', and the rows the new addthis (both behind ev_done on the comm stream)
        if (t > 1) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_x0, 0));
        rc = prmi::dev_round_stream(g, t, c->stream, e0, 1);
        if (rc) return fail(c, rc, "round compute");
        if (eA1) HIPCHK(c, hipEventRecord(eA1, c->stream));
        if (t > 1) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_done, 0));
        rc = prmi::dev_round_stream(g, t, c->stream, eB0, 2);
      } else {
        rc = prmi::dev_round_stream(g, t, c->stream, e0, 0);
      }
      if (rc) return fail(c, rc, "round compute");
      for (size_t k = 0; k < plan.size(); ++k) {
        rc = prmi::dev_round_rows(g, t, mode, plan[k].b0, plan[k].b1, c->stream);
        if (!rc && sx && !pkc) rc = prmi::dev_sx_pack(g, t, static_cast<int>(k), c->stream);
        if (rc) return fail(c, rc, "round rows");
        HIPCHK(c, hipEventRecord(c->ev_chunk[k], c->stream));
      }
      rc = prmi::dev_round_rows(g, t, mode, g->nb_rows_a, g->nb_rows, c->stream);  // class B
      if (!rc) rc = prmi::dev_round_reduce(g, c->stream, e1);
      if (rc) return fail(c, rc, "round rows");
      HIPCHK(c, hipEventRecord(c->ev_rec, c->stream));
      for (size_t k = 0; k < plan.size(); ++k) {
        HIPCHK(c, hipStreamWaitEvent(c->comm_stream, c->ev_chunk[k], 0));
        if (sx && pkc) {
          rc = prmi::dev_sx_pack(g, t, static_cast<int>(k), c->comm_stream);
          if (rc) return fail(c, rc, "sparse exchange pack");
        }
        NCCLCHK(c, ncclGroupStart());
        if (sx) {  // the packed entries each peer references (counts agreed in sx_setup_rccl)
          for (int q = 0; q < p; ++q) {
            if (q == g->rank) continue;
            const size_t i = k * p + q;
            const uint64_t ns = g->sx_so[i + 1] - g->sx_so[i], nrv = g->sx_ro[i + 1] - g->sx_ro[i];
            if (ns) NCCLCHK(c, ncclSend(g->sx_sbuf + g->sx_so[i], ns, ncclFloat64, q, c->comm, c->comm_stream));
            if (nrv) NCCLCHK(c, ncclRecv(g->sx_rbuf + g->sx_ro[i], nrv, ncclFloat64, q, c->comm, c->comm_stream));
          }
        } else {
          for (const prmi::XPiece& pc : plan[k].pieces)
            for (int q = 0; q < p; ++q) {
              if (q == g->rank) continue;
              NCCLCHK(c, ncclSend(xf + static_cast<uint64_t>(g->rank) * g->maxA + pc.off, pc.cnt, ncclFloat64, q, c->comm, c->comm_stream));
              NCCLCHK(c, ncclRecv(xf + static_cast<uint64_t>(q) * g->maxA + pc.off, pc.cnt, ncclFloat64, q, c->comm, c->comm_stream));
            }
        }
        NCCLCHK(c, ncclGroupEnd());
        if (sx) {
          rc = prmi::dev_sx_unpack(g, t, static_cast<int>(k), c->comm_stream);
          if (rc) return fail(c, rc, "sparse exchange unpack");
        }
        if (k == 0) HIPCHK(c, hipEventRecord(c->ev_x0, c->comm_stream));  // the hot prefix is in
      }
      HIPCHK(c, hipStreamWaitEvent(c->comm_stream, c->ev_rec, 0));
      NCCLCHK(c, ncclAllGather(g->rec_local, g->rec_all, prmi::REC_WORDS, ncclUint64, c->comm, c->comm_stream));
      rc = prmi::dev_round_finalize(g, t, tracked, c->comm_stream);
      if (rc) return fail(c, rc, "round finalize");
      HIPCHK(c, hipEventRecord(c->ev_done, c->comm_stream));
      // round t+1 needs x' and a: all of it at once, or (overlapped) in the two steps above
      if (!ov || t == iterations) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_done, 0));
    }
    rc = mark_progress(c, t, p > 1 ? c->comm_stream : c->stream);
    if (rc) return rc;
    if (tol > 0.0) {
      HIPCHK(c, hipMemcpyAsync(&hs, g->state, sizeof(hs), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      if (hs.resid <= tol) {
        done = t;
        break;
      }
    }
  }
  HIPCHK(c, hipEventRecord(c->ev_stop, c->stream));
  HIPCHK(c, hipMemcpyAsync(&hs, g->state, sizeof(hs), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  float ms = 0.f;
  HIPCHK(c, hipEventElapsedTime(&ms, c->ev_start, c->ev_stop));
  double kms = 0.0;
  const int nmeas = std::min(done, nk);
  for (int t = 0; t < nmeas; ++t) {
    float k = 0.f, k2 = 0.f;
    if (p > 1 && ov) {  // the two parts of the round's SpMV, without the wait between them
      if (hipEventElapsedTime(&k, c->kev[4 * t], c->kev[4 * t + 1]) == hipSuccess &&
          hipEventElapsedTime(&k2, c->kev[4 * t + 2], c->kev[4 * t + 3]) == hipSuccess)
        kms += k + k2;
    } else if (hipEventElapsedTime(&k, c->kev[4 * t], c->kev[4 * t + 3]) == hipSuccess) {
      kms += k;
    }
  }
  s.iterations = done;
  s.ms_total = ms;
  s.ms_per_iter = ms / done;
  s.ms_spmv_kernel = nmeas ? kms / nmeas : 0.0;
  s.gteps = s.ms_per_iter > 0 ? static_cast<double>(g->nnz) / (s.ms_per_iter * 1e-3) / 1e9 : 0.0;
  s.residual = tracked ? hs.resid : 0.0;
  s.rank_sum = tracked ? hs.rank_sum : 0.0;
  // the reduce of round err_iter saw an empty danglingMap: the reference dies there
  // (not under the timing-only row filters, whose ranks are wrong by construction)
  if (hs.err_iter != 0 && hs.err_iter <= done && !g->tune.dropdeg && !g->tune.keepdeg) {
    s.failed_iteration = t0 + hs.err_iter;
    if (st) *st = s;
    return fail(c, PR_E_EMPTY_DANGLING,
                "java.lang.UnsupportedOperationException: empty collection (iteration " +
                    std::to_string(t0 + hs.err_iter) + ")");
  }
  c->last_iters = done;
  if (st) *st = s;
  return PR_OK;
}

// pr_run for callers that cannot allocate: the round loop of a single-GPU context with every
// per-round scratch array (piece sums, record shards, record, round state) in this device's
// static scratch instead of the context's own buffers.  Same kernels, same order of sums.
int pr_run_static(pr_ctx* c, int32_t iterations, double tol, pr_stats* st) {
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  if (iterations < 0) return fail(c, PR_E_ARG, "iterations < 0");
  if (c->opts.n_ranks != 1 || !c->group.empty() || c->external)
    return fail(c, PR_E_ARG, "pr_run_static: single-GPU contexts only (n_ranks = 1)");
  if (!c->scratch.partial) return fail(c, PR_E_HIP, "pr_run_static: the static scratch of this device could not be resolved");
  DevGraph* g = &c->dg;
  if (g->n_pieces > c->scratch.max_pieces)
    return fail(c, PR_E_ARG, "pr_run_static: the graph needs " + std::to_string(g->n_pieces) +
                                 " piece sums per round, the static scratch holds " +
                                 std::to_string(c->scratch.max_pieces) + " (use pr_run)");
  pr_stats s{};
  s.nnz = g->nnz;
  s.n_vertices = g->n;
  s.bytes_per_iter = 4ull * g->nnz + 24ull * g->n + 8;
  c->host_ranks_valid = false;
  c->last_iters = -1;
  if (iterations == 0) {
    c->last_iters = 0;
    if (st) *st = s;
    return PR_OK;
  }
  const int t0 = g->seeded ? c->seed_rounds : 0;
  if (!g->seeded && g->W0 == 0) {
    s.failed_iteration = 1;
    if (st) *st = s;
    return fail(c, PR_E_EMPTY_DANGLING, "java.lang.UnsupportedOperationException: empty collection (iteration 1)");
  }
  const bool tracked = tol > 0.0 || (c->opts.flags & PR_F_TRACK_RESIDUAL);
  // the rounds run on the context's graph with its scratch arrays swapped for the static ones
  struct Swap {
    DevGraph* g;
    double* partial;
    uint64_t *shards, *rec;
    prmi::IterState* state;
    ~Swap() {
      g->partial = partial;
      g->shards = shards;
      g->rec_local = rec;
      g->state = state;
      g->no_alloc = false;
    }
  } swap{g, g->partial, g->shards, g->rec_local, g->state};
  g->partial = c->scratch.partial;
  g->shards = c->scratch.shards;
  g->rec_local = c->scratch.rec;
  g->state = c->scratch.state;
  g->no_alloc = true;
  // the scratch keeps the last call's contents: state and shards start from this launch
  rc = prmi::dev_reset_state_kernel(g, c->stream);
  if (rc) return fail(c, rc, "reset state");
  HIPCHK(c, hipEventRecord(c->ev_start, c->stream));
  int done = iterations;
  prmi::IterState hs{};
  for (int t = 1; t <= iterations; ++t) {
    const int mode = tracked ? 2 : (t == iterations ? 1 : 0);
    rc = prmi::dev_round_single(g, t, mode, tracked, c->stream, nullptr, nullptr);
    if (rc) return fail(c, rc, "round");
    if (tol > 0.0) {
      HIPCHK(c, hipMemcpyAsync(&hs, g->state, sizeof(hs), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      if (hs.resid <= tol) {
        done = t;
        break;
      }
    }
  }
  HIPCHK(c, hipEventRecord(c->ev_stop, c->stream));
  HIPCHK(c, hipMemcpyAsync(&hs, g->state, sizeof(hs), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  float ms = 0.f;
  HIPCHK(c, hipEventElapsedTime(&ms, c->ev_start, c->ev_stop));
  s.iterations = done;
  s.ms_total = ms;
  s.ms_per_iter = ms / done;
  s.gteps = s.ms_per_iter > 0 ? static_cast<double>(g->nnz) / (s.ms_per_iter * 1e-3) / 1e9 : 0.0;
  s.residual = tracked ? hs.resid : 0.0;
  s.rank_sum = tracked ? hs.rank_sum : 0.0;
  if (hs.err_iter != 0 && hs.err_iter <= done) {
    s.failed_iteration = t0 + hs.err_iter;
    if (st) *st = s;
    return fail(c, PR_E_EMPTY_DANGLING,
                "java.lang.UnsupportedOperationException: empty collection (iteration " +
                    std::to_string(t0 + hs.err_iter) + ")");
  }
  c->last_iters = done;
  if (st) *st = s;
  return PR_OK;
}

// Diagnostics of the running (or last) round loop; callable from another thread while the
// loop's entry point blocks (it reads two atomics and queries events, nothing else).
int pr_progress(pr_ctx* c, int32_t* rounds_enqueued, int32_t* rounds_done) {
  if (!c) return PR_E_ARG;
  const int enq = c->prog_enq.load(std::memory_order_acquire);
  int done = std::min(c->prog_done_hint.load(std::memory_order_acquire), enq);
  if (c->has_device && static_cast<int>(c->prog_ev.size()) == PROG_EVENTS) {
    // rounds complete in order: advance past every recent round whose event has fired
    done = std::max(done, enq - PROG_EVENTS);
    while (done < enq && hipEventQuery(c->prog_ev[done % PROG_EVENTS]) == hipSuccess) ++done;
    c->prog_done_hint.store(done, std::memory_order_release);
  }
  if (rounds_enqueued) *rounds_enqueued = enq;
  if (rounds_done) *rounds_done = done;
  return PR_OK;
}

int pr_layout_map(int32_t n_ranks, int32_t rank, uint32_t n_a, uint32_t n_b, uint32_t n_c,
                  uint64_t count, const uint32_t* internal_ids, uint32_t* owner_out,
                  uint32_t* local_row_out, uint64_t* x_pos_out, uint64_t dims_out[4]) {
  if (count && !internal_ids) return PR_E_ARG;
  return prmi::host_layout_map(n_ranks, rank, n_a, n_b, n_c, count, internal_ids, owner_out,
                               local_row_out, x_pos_out, dims_out);
}

int pr_debug_move_array(pr_ctx* c, const char* name) {
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  HIPCHK(c, hipDeviceSynchronize());
  std::string e;
  rc = prmi::dev_move_array(&c->dg, name, &e);
  if (rc) return fail(c, rc, "move array: " + e);
  return PR_OK;
}

int pr_selftest_sum_order(pr_ctx* c, uint32_t cases, uint32_t launches, uint64_t* copies,
                          uint64_t* differing, uint64_t* lane_order_cases) {
  int rc = need_device(c);
  if (rc) return rc;
  if (!copies || !differing || !lane_order_cases || cases == 0 || launches == 0)
    return fail(c, PR_E_ARG, "pr_selftest_sum_order: null output or empty test");
  std::string e;
  rc = prmi::dev_selftest_lds_order(cases, launches, c->stream, copies, differing, lane_order_cases, &e);
  if (rc) return fail(c, rc, "self-test: " + e);
  return PR_OK;
}

int pr_comm_query(pr_ctx* c, int32_t* transport, int32_t* comm_ranks, int32_t* comm_rank) {
  if (!c) return PR_E_ARG;
  int tr = 0, n = 1, r = 0;
  if (c->comm) {
    tr = 1;
    NCCLCHK(c, ncclCommCount(c->comm, &n));
    NCCLCHK(c, ncclCommUserRank(c->comm, &r));
  } else if (!c->group.empty()) {
    tr = 2;
    n = static_cast<int>(c->group.size());
    r = c->opts.rank;
  } else if (c->external) {
    tr = 3;
    n = c->opts.n_ranks;
    r = c->opts.rank;
  }
  if (transport) *transport = tr;
  if (comm_ranks) *comm_ranks = n;
  if (comm_rank) *comm_rank = r;
  return PR_OK;
}

int pr_get_ranks(pr_ctx* c, double* out, uint64_t n) {
  if (!c || !out) return PR_E_ARG;
  int rc = gather_ranks(c);
  if (rc) return rc;
  if (n < c->h_ranks.size()) return fail(c, PR_E_ARG, "output buffer too small");
  std::memcpy(out, c->h_ranks.data(), 8 * c->h_ranks.size());
  return PR_OK;
}

int pr_topk(pr_ctx* c, uint32_t k, uint64_t* pair_out, uint32_t* id_out, double* rank_out,
            uint32_t* count) {
  if (!c) return PR_E_ARG;
  std::vector<TopRow> rows;
  int rc = topk_rows(c, k, &rows);
  if (rc) return rc;
  for (size_t i = 0; i < rows.size(); ++i) {
    if (pair_out) pair_out[i] = rows[i].pair;
    if (id_out) id_out[i] = rows[i].v;
    if (rank_out) rank_out[i] = rows[i].r;
  }
  if (count) *count = static_cast<uint32_t>(rows.size());
  return PR_OK;
}

int pr_write_top_page(pr_ctx* c, const char* path) {
  if (!c) return PR_E_ARG;
  std::vector<TopRow> rows;
  int rc = topk_rows(c, c->opts.topk, &rows);
  if (rc) return rc;
  if (c->opts.rank != 0) return PR_OK;
  const PairIndex pi = make_pair_index(c);
  std::string out;
  char num[64];
  for (const TopRow& row : rows) {
    uint32_t v;
    std::string t;
    pair_at(c, pi, row.pair, &v, &t);
    prmi::java_double_to_string(row.r, num, sizeof(num));
    out += t;
    out += '\t';
    out += num;
    out += '\n';
  }
  FILE* f = fopen(path ? path : "./topPage", "wb");
  if (!f) return fail(c, PR_E_IO, std::string("java.io.IOException: cannot open ") + (path ? path : "./topPage"));
  const size_t w = fwrite(out.data(), 1, out.size(), f);
  const int cl = fclose(f);
  if (w != out.size() || cl != 0) return fail(c, PR_E_IO, "java.io.IOException: short write");
  return PR_OK;
}

int pr_write_rank_dump(pr_ctx* c, const char* path) {
  if (!c || !path) return c ? fail(c, PR_E_ARG, "null path") : PR_E_ARG;
  int rc = gather_ranks(c);  // collective
  if (rc) return rc;
  if (c->opts.rank != 0) return PR_OK;
  FILE* f = fopen(path, "wb");
  if (!f) return fail(c, PR_E_IO, std::string("java.io.IOException: cannot open ") + path);
  const PairIndex pi = make_pair_index(c);
  const bool text = c->source == pr_ctx::SRC_TEXT;
  if (text) ensure_pairs_by_id(c);
  std::string out;
  out.reserve(1 << 22);
  char num[64];
  bool ok = true;
  for (uint32_t v = 0; v < c->hg.n && ok; ++v) {
    const double r = c->h_ranks[v];
    if (!(r > 0.0)) continue;  // not in the ranks RDD
    prmi::java_double_to_string(r, num, sizeof(num));
    std::string id;
    if (text) {
      size_t n;
      const char* p = c->hg.ids.get(v, &n);
      id.assign(p, n);
    } else {
      id = std::to_string(v);
    }
    uint64_t b = v, e = v + 1ull;  // the mapping pairs of page v (:167 join)
    if (text) {
      b = c->hg.pair_first[v];
      e = c->hg.pair_first[v + 1];
    } else if (!c->hg.mapw.empty()) {
      b = pi.first[v];
      e = pi.first[v + 1];
    }
    auto row = [&](const std::string& title) {
      out += id;
      out += '\t';
      out += title;
      out += '\t';
      out += num;
      out += '\n';
    };
    if (b == e) row("");  // a ranked page without a title (the join would drop it)
    for (uint64_t q = b; q < e; ++q) {
      uint32_t vv;
      std::string t;
      pair_at(c, pi, text ? c->hg.pairs_by_id[q] : q, &vv, &t);
      row(t);
    }
    if (out.size() >= (1u << 22)) {
      ok = fwrite(out.data(), 1, out.size(), f) == out.size();
      out.clear();
    }
  }
  if (ok && !out.empty()) ok = fwrite(out.data(), 1, out.size(), f) == out.size();
  ok = (fclose(f) == 0) && ok;
  return ok ? PR_OK : fail(c, PR_E_IO, "java.io.IOException: short write");
}

int pr_id_string(pr_ctx* c, uint32_t v, char* buf, size_t cap, size_t* len) {
  if (!c) return PR_E_ARG;
  int rc = need_graph(c);
  if (rc) return rc;
  if (v >= c->hg.n) return fail(c, PR_E_ARG, "vertex out of range");
  std::string s;
  if (c->source == pr_ctx::SRC_TEXT) {
    size_t n;
    const char* p = c->hg.ids.get(v, &n);
    s.assign(p, n);
  } else {
    s = std::to_string(v);
  }
  if (len) *len = s.size();
  if (buf && cap) std::memcpy(buf, s.data(), std::min(cap, s.size()));
  return PR_OK;
}

int pr_pair(pr_ctx* c, uint64_t i, uint32_t* id, char* title, size_t cap, size_t* len) {
  if (!c) return PR_E_ARG;
  int rc = need_graph(c);
  if (rc) return rc;
  if (i >= pair_count(c)) return fail(c, PR_E_ARG, "pair out of range");
  const PairIndex pi = make_pair_index(c);
  uint32_t v;
  std::string t;
  pair_at(c, pi, i, &v, &t);
  if (id) *id = v;
  if (len) *len = t.size();
  if (title && cap) std::memcpy(title, t.data(), std::min(cap, t.size()));
  return PR_OK;
}

int pr_get_degrees(pr_ctx* c, uint32_t* outdeg, uint32_t* indeg, uint32_t* dang_w, uint64_t n) {
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  const uint64_t nv = c->dg.n;
  if (n < nv) return fail(c, PR_E_ARG, "buffer too small");
  if (nv) {
    if (outdeg) HIPCHK(c, hipMemcpyAsync(outdeg, c->dg.outdeg, 4 * nv, hipMemcpyDeviceToHost, c->stream));
    if (indeg) HIPCHK(c, hipMemcpyAsync(indeg, c->dg.indeg, 4 * nv, hipMemcpyDeviceToHost, c->stream));
    if (dang_w) HIPCHK(c, hipMemcpyAsync(dang_w, c->dg.dang_w, 4 * nv, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PR_OK;
}

int pr_edge_digest(pr_ctx* c, uint64_t digest_out[2]) {
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  if (!digest_out) return PR_E_ARG;
  digest_out[0] = c->dg.digest[0];
  digest_out[1] = c->dg.digest[1];
  return PR_OK;
}

int pr_export_csr(pr_ctx* c, uint64_t* row_ptr, uint32_t* col, uint32_t* outdeg, uint32_t* dang_w,
                  uint64_t* n_out, uint64_t* nnz_out) {
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  if (c->opts.n_ranks != 1) return fail(c, PR_E_ARG, "pr_export_csr needs a single-rank context");
  const DevGraph& g = c->dg;
  if (n_out) *n_out = g.n;
  if (nnz_out) *nnz_out = g.nnz;
  if (!row_ptr && !col && !outdeg && !dang_w) return PR_OK;
  const uint32_t n = g.n;
  std::vector<uint32_t> perm(n), od(n), dw(n);
  if (n) {
    HIPCHK(c, hipMemcpyAsync(perm.data(), g.perm, 4ull * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(od.data(), g.outdeg, 4ull * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(dw.data(), g.dang_w, 4ull * n, hipMemcpyDeviceToHost, c->stream));
  }
  if (row_ptr || col) {
    std::string e;
    rc = prmi::dev_export_csr(&c->dg, row_ptr, col, c->stream, &e);
    if (rc) return fail(c, rc, "export csr: " + e);
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (row_ptr)
    for (uint64_t k = g.lrows + 1ull; k <= n; ++k) row_ptr[k] = g.nnz;
  for (uint32_t k = 0; k < n; ++k) {
    if (outdeg) outdeg[k] = od[perm[k]];
    if (dang_w) dang_w[k] = dw[perm[k]];
  }
  return PR_OK;
}

int pr_format_double(double v, char* buf, size_t cap) {
  return prmi::java_double_to_string(v, buf, cap);
}

}  // extern "C"

// ---- resume / checkpoint ----------------------------------------------
namespace {

struct CkptHeader {
  char magic[8];        // "PRMICKP1"
  uint32_t version;     // 1
  uint32_t flags;       // PR_F_NORMALIZED of the run
  uint64_t n, nnz, n_tot, digest0, digest1;
  int64_t rounds;       // rounds behind the ranks
};
static_assert(sizeof(CkptHeader) == 64, "checkpoint header layout");

int seed_one(pr_ctx* c, const double* ranks, uint64_t n, int32_t rounds_done) {
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  std::string err;
  if (!ranks) {
    c->last_iters = -1;
    c->host_ranks_valid = false;
    c->seed_rounds = 0;
    rc = prmi::dev_seed_state(&c->dg, nullptr, c->stream, &err);
    return rc ? fail(c, rc, "seed: " + err) : PR_OK;
  }
  if (n != c->dg.n) return fail(c, PR_E_ARG, "ranks: length != vertex count");
  if (rounds_done < 1) return fail(c, PR_E_ARG, "rounds_done must be >= 1 (round 0 is r^0: start fresh instead)");
  std::vector<uint32_t> indeg(n);
  if (n) HIPCHK(c, hipMemcpyAsync(indeg.data(), c->dg.indeg, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint64_t v = 0; v < n; ++v) {
    const double r = ranks[v];
    if (!(r >= 0.0) || r == HUGE_VAL)
      return fail(c, PR_E_ARG, "ranks: page " + std::to_string(v) + " is negative or not finite");
    if (r > 0.0 && indeg[v] == 0)
      return fail(c, PR_E_ARG, "ranks: page " + std::to_string(v) + " has no in-link, so no rank after round 1");
  }
  c->last_iters = -1;  // the seed replaces the last run's state
  c->host_ranks_valid = false;
  rc = prmi::dev_seed_state(&c->dg, ranks, c->stream, &err);
  if (rc) return fail(c, rc, "seed: " + err);
  c->seed_rounds = rounds_done;
  return PR_OK;
}

}  // namespace

int pr_set_ranks(pr_ctx* c, const double* ranks, uint64_t n, int32_t rounds_done) {
  if (!c) return PR_E_ARG;
  return seed_one(c, ranks, n, rounds_done);
}

int pr_checkpoint_save(pr_ctx* c, const char* path) {
  if (!c || !path) return c ? fail(c, PR_E_ARG, "null path") : PR_E_ARG;
  int rc = gather_ranks(c);  // collective
  if (rc) return rc;
  if (c->opts.rank != 0) return PR_OK;
  CkptHeader h{};
  std::memcpy(h.magic, "PRMICKP1", 8);
  h.version = 1;
  h.flags = c->opts.flags & PR_F_NORMALIZED;
  h.n = c->dg.n;
  h.nnz = c->dg.nnz;
  h.n_tot = c->dg.n_tot;
  h.digest0 = c->dg.digest[0];
  h.digest1 = c->dg.digest[1];
  h.rounds = static_cast<int64_t>(c->dg.seeded ? c->seed_rounds : 0) + c->last_iters;
  FILE* f = fopen(path, "wb");
  if (!f) return fail(c, PR_E_IO, std::string("cannot open ") + path);
  bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
  if (h.n) ok = ok && fwrite(c->h_ranks.data(), 8, h.n, f) == h.n;
  ok = (fclose(f) == 0) && ok;
  return ok ? PR_OK : fail(c, PR_E_IO, std::string("short write: ") + path);
}

int pr_checkpoint_load(pr_ctx* c, const char* path) {
  if (!c || !path) return c ? fail(c, PR_E_ARG, "null path") : PR_E_ARG;
  int rc = need_device(c);
  if (rc) return rc;
  rc = need_graph(c);
  if (rc) return rc;
  FILE* f = fopen(path, "rb");
  if (!f) return fail(c, PR_E_IO, std::string("cannot open ") + path);
  CkptHeader h{};
  bool ok = fread(&h, sizeof(h), 1, f) == 1 && std::memcmp(h.magic, "PRMICKP1", 8) == 0 && h.version == 1;
  std::vector<double> r;
  if (ok && h.n == c->dg.n) {
    r.resize(h.n);
    ok = h.n == 0 || fread(r.data(), 8, h.n, f) == h.n;
  }
  fclose(f);
  if (!ok) return fail(c, PR_E_IO, std::string("not a prmi355x checkpoint: ") + path);
  if (h.n != c->dg.n || h.nnz != c->dg.nnz || h.n_tot != c->dg.n_tot ||
      h.digest0 != c->dg.digest[0] || h.digest1 != c->dg.digest[1])
    return fail(c, PR_E_ARG, "checkpoint belongs to another graph");
  if (h.flags != (c->opts.flags & PR_F_NORMALIZED))
    return fail(c, PR_E_ARG, "checkpoint normalization differs from this context's");
  if (h.rounds < 0 || h.rounds > INT32_MAX) return fail(c, PR_E_ARG, "checkpoint round count");
  if (h.rounds == 0) return seed_one(c, nullptr, 0, 0);  // round 0 = r^0: a fresh start
  return seed_one(c, r.data(), r.size(), static_cast<int32_t>(h.rounds));
}

// ---- TF-IDF (Spark.java:22-173) -----------------------------------------
namespace {

struct TfRow {
  double v;
  uint32_t title;
  std::string key;  // lowercased title up to its first ',' (Spark.java:106, :155-156)
  std::string full;
};

// Spark.java:120-162 for `word`: rows sorted by tfidf descending, then the lowercased
// truncated title (Collections.sort is stable; Spark's lookup order is unspecified, so the
// full title bytes decide the rest)
int tf_rows(pr_ctx* c, const char* word, size_t wlen, std::vector<TfRow>* rows) {
  int rc = need_device(c);
  if (rc) return rc;
  if (!c->tf.ready) return fail(c, PR_E_ARG, "no TF-IDF input: call pr_tfidf_ingest_* first");
  std::vector<uint32_t> titles, tfs;
  uint32_t df = 0;
  std::string err;
  rc = prmi::tf_lookup(&c->tf, word, wlen, &titles, &tfs, &df, c->stream, &err);
  if (rc) return fail(c, rc, "tfidf lookup: " + err);
  rows->clear();
  if (titles.empty()) return PR_OK;
  // :130-131  Math.log(titleCount / dword): Long / Integer is an integer division
  const double idf = std::log(static_cast<double>(static_cast<uint64_t>(c->tf.n_docs) / df));
  for (size_t i = 0; i < titles.size(); ++i) {
    TfRow r;
    r.v = static_cast<double>(static_cast<int32_t>(tfs[i])) * idf;  // :131 int * double
    r.title = titles[i];
    r.full.assign(c->tf.titles, c->tf.title_off[r.title], c->tf.title_off[r.title + 1] - c->tf.title_off[r.title]);
    const size_t comma = r.full.find(',');
    r.key = r.full.substr(0, comma);
    for (char& ch : r.key)
      if (ch >= 'A' && ch <= 'Z') ch = static_cast<char>(ch | 0x20);
    rows->push_back(std::move(r));
  }
  std::sort(rows->begin(), rows->end(), [](const TfRow& a, const TfRow& b) {
    if (a.v != b.v) return a.v > b.v;
    if (a.key != b.key) return a.key < b.key;
    return a.full < b.full;
  });
  return PR_OK;
}

}  // namespace

int pr_tfidf_ingest_buffer(pr_ctx* c, const char* data, size_t len) {
  prmi::Span span("prmi:tfidf");
  if (!c || (!data && len)) return c ? fail(c, PR_E_ARG, "bad buffer") : PR_E_ARG;
  int rc = need_device(c);
  if (rc) return rc;
  prmi::TfidfError te;
  std::string err;
  rc = prmi::tf_ingest(&c->tf, data ? data : "", len, &te, c->stream, &err);
  if (rc == PR_E_PARSE) {
    prmi::tf_free(&c->tf);
    return fail(c, PR_E_PARSE, "java.lang.ArrayIndexOutOfBoundsException: " + std::to_string(te.index) +
                                   " (line " + std::to_string(te.line) + ")");
  }
  if (rc) {
    prmi::tf_free(&c->tf);
    return fail(c, rc, "tfidf ingest: " + err);
  }
  return PR_OK;
}

int pr_tfidf_ingest_file(pr_ctx* c, const char* path) {
  if (!c || !path) return c ? fail(c, PR_E_ARG, "null path") : PR_E_ARG;
  std::string d;
  if (!read_file(path, &d)) return fail(c, PR_E_IO, std::string("cannot read ") + path);
  return pr_tfidf_ingest_buffer(c, d.data(), d.size());
}

int pr_tfidf_info(pr_ctx* c, uint64_t* docs, uint64_t* words, uint64_t* pairs, uint64_t* tokens) {
  if (!c) return PR_E_ARG;
  if (!c->tf.ready) return fail(c, PR_E_ARG, "no TF-IDF input");
  if (docs) *docs = c->tf.n_docs;
  if (words) *words = c->tf.n_words;
  if (pairs) *pairs = c->tf.n_pairs;
  if (tokens) *tokens = c->tf.tokens;
  return PR_OK;
}

int pr_tfidf_lookup(pr_ctx* c, const char* word, size_t wlen, uint32_t k, uint32_t* title_out,
                    double* tfidf_out, uint32_t* count) {
  if (!c || (!word && wlen)) return c ? fail(c, PR_E_ARG, "bad word") : PR_E_ARG;
  std::vector<TfRow> rows;
  int rc = tf_rows(c, word ? word : "", wlen, &rows);
  if (rc) return rc;
  const size_t n = std::min<size_t>(k, rows.size());
  for (size_t i = 0; i < n; ++i) {
    if (title_out) title_out[i] = rows[i].title;
    if (tfidf_out) tfidf_out[i] = rows[i].v;
  }
  if (count) *count = static_cast<uint32_t>(n);
  return PR_OK;
}

int pr_tfidf_title(pr_ctx* c, uint32_t t, char* buf, size_t cap, size_t* len) {
  if (!c) return PR_E_ARG;
  if (!c->tf.ready || t >= c->tf.n_docs) return fail(c, PR_E_ARG, "title index out of range");
  const uint64_t a = c->tf.title_off[t], b = c->tf.title_off[t + 1];
  if (len) *len = b - a;
  if (buf && cap) {
    const size_t m = std::min<size_t>(cap, b - a);
    std::memcpy(buf, c->tf.titles.data() + a, m);
  }
  return PR_OK;
}

int pr_tfidf_write_output(pr_ctx* c, const char* word, const char* path) {
  if (!c) return PR_E_ARG;
  const char* w = word ? word : "cloud";  // :140 idf.lookup("cloud")
  std::vector<TfRow> rows;
  int rc = tf_rows(c, w, std::strlen(w), &rows);
  if (rc) return rc;
  std::string out = "total docs are " + std::to_string(c->tf.n_docs) + "\n";  // :165
  char num[64];
  for (size_t i = 0; i < rows.size() && i < 100; ++i) {  // :166-169
    const std::string& t = rows[i].full;
    prmi::java_double_to_string(rows[i].v, num, sizeof(num));
    out += t.substr(0, t.find(','));  // kv[0] of "title,tfidf".split(",")
    out += '\t';
    out += num;
    out += '\n';
  }
  FILE* f = fopen(path ? path : "./output", "wb");
  if (!f) return fail(c, PR_E_IO, std::string("java.io.IOException: cannot open ") + (path ? path : "./output"));
  const size_t wr = fwrite(out.data(), 1, out.size(), f);
  const int cl = fclose(f);
  if (wr != out.size() || cl != 0) return fail(c, PR_E_IO, "java.io.IOException: short write");
  return PR_OK;
}
