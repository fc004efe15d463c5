// Device engine interface (implemented in engine.hip; driven by api.cpp).
//
// Layout in HBM (DESIGN.md "Data layout"):
//   internal vertex order  k = 0..n-1, sorted by (class, in-degree desc, original id):
//     class A [0,nA)        in>=1, out>=1   rows and columns
//     class B [nA,R)        in>=1, out==0   rows only (dangling pages that get links)
//     class C [R,R+nC)      in==0, out>=1   columns only (rank undefined after round 1)
//     class D [R+nC,n)      in==0, out==0   neither
//   rows k < R are dealt to ranks in chunks of 16: chunk c = k>>4 goes to rank c % p
//   XCD slicing: the columns of x are cut into 8 slices by 128-byte chunk (slice = chunk
//   index mod 8).  Slice j's edges are processed only by workgroups with blockIdx % 8 == j
//   (one XCD), so each XCD's L2 caches 1/8 of x.  Inside a slice the columns are in hotness
//   order (position q), cut into segments: nlds LDS blocks of H entries, an L2-hot range,
//   then cold ranges.  Stream groups per slice: one per LDS block (16-bit columns) + one for
//   the rest (32-bit x positions), each sorted by (segment, local row, q) and padded to
//   whole 1024-edge tasks.
//   A "pair" = the edges of one (row, slice, segment); a "piece" = a pair cut at task
//   boundaries.  The stream kernel writes one partial sum per piece (stream order); the row
//   kernel reads, per 1024-row block, one contiguous run per stream (runs table) and adds
//   the pieces in a fixed order.
#pragma once

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdint>
#include <string>
#include <vector>

#include "host_graph.h"

namespace prmi {

// roctx ranges (rocprofv3 --marker-trace): host-side spans of the build phases, ingest, runs
// and rounds.  Scope = one push/pop; next() closes the previous phase and opens another.
class Span {
 public:
  explicit Span(const char* name) { roctxRangePushA(name); depth_ = 1; }
  ~Span() { while (depth_-- > 0) roctxRangePop(); }
  void next(const char* phase) {
    if (depth_ > 1) { roctxRangePop(); --depth_; }
    roctxRangePushA(phase);
    ++depth_;
  }
  Span(const Span&) = delete;
  Span& operator=(const Span&) = delete;

 private:
  int depth_ = 0;
};

constexpr int SA_LIMBS = 10;       // exact accumulator: 10 x 32-bit chunks, unit 2^-96
constexpr int SA_BASE_EXP = -96;
constexpr int NSHARD = 256;        // atomic shards for the per-iteration partials
constexpr int REC_WORDS = 32;      // record: [0,10) dangling mass, [10] dangling count,
                                   //         [11,21) sum|dr|, [21,31) sum r
constexpr int REC_DSUM = 0, REC_DCNT = 10, REC_RESID = 11, REC_RSUM = 21;
constexpr int BLOCK = 256;
constexpr int NSLICE = 8;          // one slice per XCD
constexpr int CHUNK = 16;          // rows dealt per rank chunk = entries per 128-B x line

constexpr int EPL = 16;            // stream edges per lane per task
constexpr int TASK = 64 * EPL;     // stream edges per wave task (1024)

struct IterState {
  double a;          // addthis for the next round (PageRank.java:135-138)
  double resid;      // relative L1 residual of the last round (tracked mode)
  double resid_abs;
  double rank_sum;
  uint64_t dcnt;     // defined dangling entries after the last round
  int32_t err_iter;  // first round whose reduce (:125) would see an empty RDD, 0 = none
  int32_t iter;
};

struct Tuning {
  uint32_t qh = 131072; // PR_QH: L2-hot segment length per slice after the LDS blocks (1 MiB;
                        // 3.5 MiB before the dedicated L2 waves: 128 Ki entries measured best
                        // with them, profiles/r02/)
  uint32_t rb = 1024;   // PR_RB: rows per row-launch block (64..1024)
  uint32_t rb_heavy = 256;  // PR_RBH: rows per heavy row-launch block
  uint32_t rxg = 16;     // PR_RXG: consecutive row-launch blocks per XCD (1 = round-robin)
  uint32_t heavy_deg = 128; // PR_HDEG: rows with in-degree >= this get heavy blocks (0 = none)
  int nlds = 20;        // PR_NLDS: LDS blocks per slice (each swept with its own LDS fill).  Unset,
                        // the build sizes it to the graph: 0.41 B^0.77 for a slice of B blocks'
                        // worth of class-A columns (21 blocks at R-MAT scale 26 on one rank)
  uint32_t seg = 262144;  // PR_SEG: cold segment length per slice (x entries, 2 MiB)
  // PR_NT: 2 = non-temporal piece stores (they stop evicting x from the L2s: +3 %), 0 =
  // regular stores.  Non-temporal stream loads and LDS fills were measured slower.
  int nt = 2;
  uint32_t hot_lds = 20480;  // PR_HOTLDS: LDS block length (x entries, capped by the staging room)
  uint32_t colmask = 0xFFFFFFFFu;  // PR_COLMASK: timing-only gather working-set restriction
  int dbg = 0;          // PR_DBG: timing-only experiments in the stream kernel (see StreamArgs)
  int stream_wg = 1;    // PR_STREAM_WG: stream workgroups per CU (1 with the LDS copy)
  int l2mode = 0;       // PR_L2MODE: 0 = L2 tasks interleaved with the LDS phases, 1 = last
  int l2w = 4;          // PR_L2W: waves per stream workgroup dedicated to the L2 group
                        // (of 16; 0 = L2 tasks shared out over the LDS phases as in round 1;
                        // 2/3/4/5/6/8 measured at scale 26, 3-4 best)
  uint32_t dpull = 0;   // PR_DPULL: direct-pull experiment for rows below this in-degree
                        // (timing only, single rank; engine.hip spmv_dpull)
  uint32_t dropdeg = 0; // PR_DROPDEG: rows below this in-degree leave the streams (timing only)
  uint32_t keepdeg = 0; // PR_KEEPDEG: rows at or above this in-degree leave the streams (timing only)
  int dyntail = 100;    // PR_DYNTAIL: percent of the LDS phases whose tasks go to the slice's
                        // workgroups in fixed shares; the later phases are claimed slice-wide
  int early = 0;        // PR_EARLY: LDS waves claim and fetch a phase's first task before its barrier
  int dyng = 4;         // PR_DYNG: tasks per slice-wide claim
  int dynl2 = 0;        // PR_DYNL2: the L2-role waves claim their tasks slice-wide too
  int stream_cus = 32;  // PR_STREAM_CUS: stream workgroups (= compute units) per XCD; 31 at p > 1
  int l2late = 0;       // PR_L2LATE: L2-role waves prefetch the next task's columns after
                        // their gathers instead of before (see StreamArgs::l2late)
  int place = 1;        // PR_PLACE: the build may move the partial array to faster memory
                        // (dev_tune_placement); PR_PLACE_MIN_MB [1024]: arrays below stay put
  int lean = 1;         // PR_LEAN: 1 = the lean per-task instruction stream of the stream launch
                        // (fma-form piece sums, DPP-masked scans, SDWA LDS addresses: -11 %
                        // VALU instructions, time unchanged), 0 = the earlier form; both
                        // produce bit-identical sums
};

struct DevGraph {
  bool built = false;
  int p = 1, rank = 0;
  uint32_t n = 0;
  uint64_t m_raw = 0, nnz = 0, n_tot = 0;
  uint32_t nA = 0, nB = 0, nC = 0, nD = 0, R = 0;
  uint32_t maxA = 0;              // x slot length per rank
  bool sm = false;                // slice-major x layout (p divides 8)
  bool snake = false;             // snake chunk -> slice order (single rank, engine.hip chunk_slice)
  uint32_t SL = 0, SLC = 0;       // slice region lengths (class A / class C)
  uint64_t X = 0;                 // x length
  uint32_t lrows = 0, lA = 0;
  uint64_t lnnz = 0;
  uint64_t W0 = 0;                // sum of dangling weights (round-1 dangling mass)
  uint64_t n_dang_entries = 0;
  uint64_t digest[2] = {0, 0};
  double ms_build = 0;
  // slice streams: group gr = slice * (nlds + 1) + (LDS block, or nlds = the L2 part) owns
  // tasks [gtask[gr], gtask[gr+1]) = stream positions gtask*TASK.. and sorted-key edges
  // [gstart[gr], gstart[gr+1]) (a group's tail task is padded with PAD_COL edges)
  std::vector<uint32_t> gtask;
  std::vector<uint64_t> gstart;
  std::vector<uint64_t> gbase;    // first edge of each group in col16 (LDS groups) / col (L2)
  uint32_t* d_gtask = nullptr;
  uint64_t* d_gstart = nullptr;
  uint64_t* d_gbase = nullptr;
  uint64_t n_col16 = 0, n_col32 = 0;
  uint32_t ntask = 0;
  uint32_t nlds = 0, hot_h = 0;   // LDS blocks per slice and their length (x entries)
  uint32_t nseg = 0;              // segments per slice (LDS blocks + L2-hot + cold)
  uint64_t n_pieces = 0, n_pairs = 0;
  uint64_t n_lines = 0, n_runs = 0;  // row-launch 64-piece lines, non-empty (block, stream) runs
  uint64_t n_groups = 0;             // row-launch 8-line groups
  uint64_t stream_len = 0;        // padded length of col (multiple of TASK)
  // device arrays
  uint32_t* col = nullptr;        // [n_col32] L2-group edges: x position of the source
  uint16_t* col16 = nullptr;      // [n_col16] LDS-group edges: source offset inside the block
  uint16_t* bits = nullptr;       // [stream_len/16] pair-start flags
  uint32_t* task_piece = nullptr; // [tasks+1] first piece of each task
  double* partial = nullptr;      // [n_pieces] per-piece partial sums
  uint16_t* roff = nullptr;       // [n_pieces] row of each piece, relative to its row block
  uint32_t* runs = nullptr;       // [(nb_rows+1) * n_streams] first piece of (row block, stream)
  // row-launch maps (engine.hip RowArgs): non-empty runs per block, 64-piece line maps
  uint32_t* nebase = nullptr;     // per block: start - pre of each non-empty run
  uint32_t* ne_off = nullptr;     // [nb_rows + 1]
  uint32_t* l_off = nullptr;      // [nb_rows + 1] first line of each block
  uint32_t* btot = nullptr;       // [nb_rows] pieces per block
  uint32_t* lfirst = nullptr;     // [lines] block-relative run of the line's first piece
  uint64_t* lmask = nullptr;      // [lines] run starts inside the line
  uint32_t* goff = nullptr;       // [nb_rows + 1] first 8-line group of each block
  uint32_t* roffL = nullptr;      // [groups * 64 * 3] row offsets in row-launch order (10-bit, 3 per dword)
  bool roff16 = false;            // PR_ROFF16: the earlier 8 x u16 layout (A/B only)
  uint32_t* meta = nullptr;
  uint32_t* perm = nullptr;       // internal -> original
  uint32_t* outdeg = nullptr;     // by original id
  uint32_t* indeg = nullptr;
  uint32_t* dang_w = nullptr;
  uint32_t* mapw = nullptr;       // [n] mapping pairs per page (nullptr: every page once)
  // initial rank and damping base: 1.0 and 0.15 (PageRank.java:78, :143), or 1/N_tot and
  // 0.15/N_tot with PR_F_NORMALIZED
  double r0 = 1.0, base = 0.15;
  // pr_set_ranks / checkpoint resume: runs start from these instead of r^0
  bool seeded = false;
  double* x_seed = nullptr;       // [X] x of the seed ranks (every rank's slots)
  double* r_seed = nullptr;       // [lrows] the seed ranks of this rank's rows
  IterState seed_state{};
  double* x_init = nullptr;
  double* xbuf[2] = {nullptr, nullptr};
  double* r_loc[2] = {nullptr, nullptr};
  double* r_full = nullptr;       // [n] by original id (output staging)
  uint64_t* shards = nullptr;     // [NSHARD][REC_WORDS]
  uint32_t* stream_cnt = nullptr; // [NSLICE * 72] slice-wide task counters of the stream launch
                                  // (zeroed by the round's record reduction)
  uint64_t* rec_local = nullptr;  // [REC_WORDS]
  uint64_t* rec_all = nullptr;    // [p][REC_WORDS]
  // sparse x' exchange (p > 1): which class-A x entries each rank's edges reference, computed
  // at build from the replicated edge set (no exchange needed to agree on it).  sx_send bit
  // q * maxA + o: peer q references entry o of this rank's slot; sx_recv bit x: this rank
  // references x position x of a peer's slot.  Host copies; the per-chunk lists are built at
  // the first exchanged run (dev_sx_prepare).
  std::vector<uint32_t> sx_send, sx_recv;
  uint32_t* sx_spos = nullptr;    // [sends] slot-relative entries to pack, by (chunk, peer)
  uint32_t* sx_rpos = nullptr;    // [recvs] absolute x positions to unpack, by (chunk, peer)
  double* sx_sbuf = nullptr;      // [sends]
  double* sx_rbuf = nullptr;      // [recvs]
  std::vector<uint64_t> sx_so, sx_ro;  // [chunks * p + 1] offsets of each (chunk, peer) list
  int sx_chunks = 0;              // chunk count the lists were built for (0 = none)
  uint64_t sx_plan_sig = 0;       // and a hash of that plan's pieces
  uint32_t l2split[NSLICE] = {0}; // first L2-group task of each slice that needs x behind the
                                  // hot prefix (the two-part stream launch of p > 1)
  IterState* state = nullptr;
  // row launch: blocks of 1024 rows (class A, then class B), streams = slices x segments
  uint32_t nb_rows = 0, nb_rows_a = 0, n_streams = 0;
  uint32_t row_rb = 1024;          // rows per row-launch block
  uint32_t row_nbH = 0, row_rbH = 256, row_lH = 0;  // heavy row blocks (first lH rows)
  // direct-pull experiment (PR_DPULL): column-major 64-row groups of the low in-degree rows
  uint32_t* dp_ell = nullptr;      // [dp_gbase[dp_groups]] x positions, PAD_COL padding
  uint32_t* dp_gbase = nullptr;    // [dp_groups + 1] first slot of each group
  double* dp_out = nullptr;        // [64 * dp_groups] the sums (a side array: not the ranks)
  uint32_t dp_groups = 0;
  bool no_alloc = false;           // inside pr_run_static: nothing may allocate (no PR_STAMPS)
  // dev_tune_placement: placements timed beyond the first, stream launch with the first and
  // with the chosen one
  int place_tried = 0;
  double place_ms_first = 0, place_ms_best = 0;
  Tuning tune;
};

// Static scratch of the allocation-free run (one file-scope device array per GPU, engine.hip):
// room for the per-piece partial sums of graphs up to STATIC_SCRATCH_PIECES pieces, the record
// shards, the round record and the round state.  32 MiB + 66 KiB per GPU, held until the
// process ends.
constexpr uint64_t STATIC_SCRATCH_PIECES = 4ull << 20;
struct StaticScratch {
  double* partial = nullptr;
  uint64_t* shards = nullptr;
  uint64_t* rec = nullptr;
  IterState* state = nullptr;
  uint64_t max_pieces = 0;
};
// The scratch of `device` (which must be the current device): resolves the array's device
// address on first use per device, no allocation.
int dev_static_scratch(int device, StaticScratch* out, std::string* err);
// dev_reset_state through one kernel launch (no host-memory copy, no memset).
int dev_reset_state_kernel(DevGraph* g, hipStream_t s);

struct BuildInput {
  uint32_t n = 0;
  uint64_t m = 0;
  uint64_t n_tot = 0;
  const uint32_t* h_src = nullptr;  // host raw edges (dense ids) unless rmat
  const uint32_t* h_dst = nullptr;
  const uint32_t* h_mapw = nullptr; // host; nullptr = every id mapped once
  bool rmat = false;
  int scale = 0;
  int edge_factor = 0;
  uint64_t seed = 0;
  bool normalized = false;          // PR_F_NORMALIZED: r^0 = 1/N_tot, base 0.15/N_tot
};

// Builds the per-rank CSR and all iteration buffers.  Returns 0 or a PR_E_* code.
int dev_build(DevGraph* g, const BuildInput& in, hipStream_t s, std::string* err);
void dev_free(DevGraph* g);

// One round t (1-based) of the loop PageRank.java:92-164 for this rank's rows, up to the
// point where x' and the partial record are ready for the exchange.
// mode: 0 = x' only, 1 = also write r', 2 = tracked (r', exact residual + rank sum).
int dev_round_compute(DevGraph* g, int t, int mode, hipStream_t s, hipEvent_t ev0,
                      hipEvent_t ev1);
// The same in three steps (the row launch may be cut into block ranges [b0, b1), e.g. for the
// chunked exchange): the stream launch; rows of blocks [b0, b1); the record reduction.
// part 0: the whole stream launch.  Parts 1 and 2 cut it for the overlapped exchange (p > 1,
// dev_can_split_stream): part 1 = the first LDS phases + the L2-hot-range tasks, which read
// only the hot prefix of each x slot sub-region (chunk 0 of a hot-first exchange plan) and the
// constant class-C entries; part 2 = the other LDS phases + the cold-segment tasks, which read
// the rest as well.
int dev_round_stream(DevGraph* g, int t, hipStream_t s, hipEvent_t ev0, int part = 0);
bool dev_can_split_stream(const DevGraph* g);
int dev_round_rows(DevGraph* g, int t, int mode, uint32_t b0, uint32_t b1, hipStream_t s);
int dev_round_reduce(DevGraph* g, hipStream_t s, hipEvent_t ev1);
// p = 1: the whole round (stream, rows, then record reduction + finalize in one launch).
int dev_round_single(DevGraph* g, int t, int mode, bool tracked, hipStream_t s, hipEvent_t ev0,
                     hipEvent_t ev1);
// Chunked x' exchange: chunk k = class-A row blocks [b0, b1) of this rank + the slot-relative
// pieces (offset, count) its rows complete; pieces are identical on every rank.
struct XPiece {
  uint64_t off, cnt;
};
struct XChunk {
  uint32_t b0 = 0, b1 = 0;
  std::vector<XPiece> pieces;
};
// hot_first: chunk 0 = the hot prefix (LDS blocks + L2-hot range) of every slot sub-region
std::vector<XChunk> dev_exchange_plan(const DevGraph* g, int K, bool hot_first = false);
// Sparse exchange: build the per-(chunk, peer) pack / unpack lists for `plan` (once per chunk
// count); pack chunk k of this rank's slot of x'(t) into sx_sbuf; unpack chunk k's received
// entries from sx_rbuf into x'(t).  Lists are in (chunk, peer, piece, entry) order on every
// rank, so rank r's send list for q is q's receive list for r.
int dev_sx_prepare(DevGraph* g, const std::vector<XChunk>& plan, std::string* err);
int dev_sx_pack(DevGraph* g, int t, int k, hipStream_t s);
int dev_sx_unpack(DevGraph* g, int t, int k, hipStream_t s);
// After the exchange: combine p records -> next round's addthis / error / residual.
int dev_round_finalize(DevGraph* g, int t, bool tracked, hipStream_t s);
// Round-1 state (r^0 == 1): a = W0 / n_tot.
int dev_reset_state(DevGraph* g, hipStream_t s);
// x' buffer of round t (this rank's slot starts at rank*maxA).
double* dev_x_out(DevGraph* g, int t);
// Scatter this rank's final ranks into r_full (by original id; zeros elsewhere).
// iterations == 0 reproduces ranks = 1.0 on sources (PageRank.java:76-83).
int dev_scatter_ranks(DevGraph* g, int iterations, hipStream_t s);
// Seed the next runs with ranks by original id (host, n entries; 0 = undefined): x, this
// rank's row ranks and the exact dangling mass of the seed.  ranks == nullptr clears it.
int dev_seed_state(DevGraph* g, const double* ranks, hipStream_t s, std::string* err);
// Host copy of this rank's pull CSR (single-rank graphs: internal ids, sources ascending).
// Top-K candidates of this rank (PageRank.java:167-189): every mapped page whose rank is >=
// the k-th largest rank counted with mapping-pair multiplicity among this rank's pages
// (ties at the boundary included), from r_full (call dev_scatter_ranks first).
int dev_topk_candidates(DevGraph* g, uint64_t k, std::vector<uint32_t>* ids,
                        std::vector<double>* rs, hipStream_t s, std::string* err);
// ---- TF-IDF job (tfidf.hip; Spark.java:22-173) ------------------------
struct TfidfError {
  bool failed = false;
  int index = 0;       // the ArrayIndexOutOfBoundsException index (1, 3, or 0/1 at :83/:106)
  uint64_t line = 0;   // 1-based line of the document that dies
};
struct TfidfState {
  bool ready = false;
  char* B = nullptr;               // the dump on the device (word bytes are read from it)
  uint64_t bytes = 0, lines = 0, tokens = 0;
  uint32_t n_docs = 0, n_words = 0, n_pairs = 0;  // titleCount (:56), distinct words, keys
  uint64_t* w_off = nullptr;       // [n_words] first occurrence of each word in B
  uint32_t* w_len = nullptr;
  uint64_t* keys = nullptr;        // [n_pairs] (word << 32 | title), sorted: a word's keys
  uint32_t* tf = nullptr;          //           are contiguous; tf = count (:66-71)
  uint32_t* w_start = nullptr;     // [n_words + 1] first key of each word; df = the run
  std::string titles;              // distinct titles, host (output strings)
  std::vector<uint64_t> title_off;
};
void tf_free(TfidfState* t);
int tf_ingest(TfidfState* t, const char* data, size_t len, TfidfError* te, hipStream_t s,
              std::string* err);
// the (title, tf) keys of `word` (exact bytes; words are lowercase) and its df
int tf_lookup(TfidfState* t, const char* word, size_t wlen, std::vector<uint32_t>* titles,
              std::vector<uint32_t>* tfs, uint32_t* df, hipStream_t s, std::string* err);

// Text ingest on the device (ingest.hip): same result as ingest_text (host_graph.cpp).
// PR_E_PARSE with *pe filled on a malformed line; INGEST_NOFIT (or PR_E_OOM) when the input
// does not fit the device path -- the caller then parses on the host.
constexpr int INGEST_NOFIT = 100;
int dev_ingest_text(const char* arcs, size_t alen, const char* map, size_t mlen, HostGraph* g,
                    ParseError* pe, hipStream_t s, std::string* err);
int dev_export_csr(DevGraph* g, uint64_t* row_ptr, uint32_t* col, hipStream_t s, std::string* err);
// Self-test of the order in which one ds_add_f64 instruction applies its lanes' same-address
// adds (the row launch's sums rest on it): `cases` lane/address/value patterns, each launched
// `launches` times on a grid covering every CU.  copies = accumulator sets compared, differing =
// those that differ from the first copy of their case, lane_order_cases = cases whose bits
// equal the ascending-lane serial sum.
// The kernels' layout functions on the host: for cnt internal vertex ids k (rows: k < nA + nB;
// columns: class A k < nA, class C nA + nB <= k < nA + nB + nC) the owner rank and local row of
// each row (0xFFFFFFFF for non-rows) and the x position of each column (~0 for non-columns), as
// rank `rank` of p sees them; dims = {slot length maxA, x length, local rows, local class-A rows}.
int host_layout_map(int p, int rank, uint32_t nA, uint32_t nB, uint32_t nC, uint64_t cnt,
                    const uint32_t* k, uint32_t* owner, uint32_t* local, uint64_t* xp,
                    uint64_t dims[4]);
// The stream launch's rate depends on which physical memory holds the partial array: the same
// kernels on the same graph run the launch in 1.55 or in 1.67 ms (R-MAT scale 26), for as long
// as the allocation lives.  The build therefore times the launch with a few more placements of
// the array -- each allocated while other device memory is held, which is released again before
// the timing -- keeps the fastest and frees the others; then the same for the LDS groups' column
// stream, the largest array the launch reads (2 % more).  Best effort: an allocation that fails
// ends the search, never the build.
int dev_tune_placement(DevGraph* g, hipStream_t s);
// Placement experiment: move one of the round's arrays ("partial", "col16", "col", "bits",
// "roffL", "x", "maps", "meta") to a fresh allocation (new buffer, device copy, old one freed).
// PR_CONTIG=1: the new buffer is physically contiguous; PR_VMM_MB=m: it is a virtual range
// backed by separately created m-MB chunks.
int dev_move_array(DevGraph* g, const char* name, std::string* err);
// A one-wave kernel that sleeps ~us microseconds on stream s (exchange measurements only).
int dev_delay_us(int us, hipStream_t s);
int dev_selftest_lds_order(uint32_t cases, uint32_t launches, hipStream_t s, uint64_t* copies,
                           uint64_t* differing, uint64_t* lane_order_cases, std::string* err);
// Internal id of this rank's local row l (host copy of the device mapping).
inline uint32_t row_internal(const DevGraph* g, uint32_t l) {
  return (((l / CHUNK) * static_cast<uint32_t>(g->p) + static_cast<uint32_t>(g->rank)) * CHUNK) +
         (l % CHUNK);
}

}  // namespace prmi
