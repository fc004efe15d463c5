/*
 * prmi355x -- MI355X-native PageRank engine: the drop-in C ABI.
 *
 * This library replaces the per-iteration hot path of the reference Spark job
 * (ajak6/Page-Rank-and-TFIDF-using-Apache-Spark, PageRank.java) -- the contribution
 * flatMapToPair (PageRank.java:94-117), the dangling-mass reduce (:121-138) and the
 * reduceByKey(Sum) + damping rank update (:139-160) -- together with the graph ingest that
 * feeds it (:26-83) and the top-K output it drains into (:167-204).  Every entry point
 * below names the reference code it stands in for.
 *
 * Plain C: pointers + sizes only.  All host buffers are caller-allocated; the library owns
 * device memory until pr_destroy().  A context is NOT thread-safe (one caller thread per
 * context); calls block until their device work is complete.  Every function returns
 * PR_OK (0) or a negative PR_E_* code; pr_last_error() holds the message.
 *
 * Multi-GPU: one process per GPU.  Each process creates a context with opts.n_ranks /
 * opts.rank, exchanges the 128-byte id from pr_comm_unique_id() (rank 0) out of band, and
 * calls pr_comm_init() before ingesting.  Ingest/generation is replicated; every rank keeps
 * the rows (destination pages) dealt to it.  pr_run / pr_get_ranks / pr_topk /
 * pr_write_top_page are collective (all ranks call them).
 */
#ifndef PRMI355X_H
#define PRMI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRMI355X_VERSION_MAJOR 0
#define PRMI355X_VERSION_MINOR 1

/* ---- error codes (reference failure -> code) ---------------------------------------- */
#define PR_OK 0
#define PR_E_ARG (-1)            /* bad argument / call order                              */
#define PR_E_PARSE (-2)          /* line with < 2 tab fields: ArrayIndexOutOfBoundsException
                                    at PageRank.java:40 (arcs) / :49 (mapping)            */
#define PR_E_EMPTY_DANGLING (-3) /* danglingMap.values().reduce on an empty RDD:
                                    UnsupportedOperationException("empty collection"),
                                    PageRank.java:125                                       */
#define PR_E_HIP (-4)            /* HIP runtime failure                                     */
#define PR_E_RCCL (-5)           /* RCCL failure                                            */
#define PR_E_OOM (-6)            /* host or device allocation failed                        */
#define PR_E_IO (-7)             /* file open/read/write failed (PageRank.java:201-204)     */
#define PR_E_NODEV (-8)          /* context created without a device (host-only)           */

/* pr_opts.device special values */
#define PR_DEVICE_FROM_RANK (-1) /* use opts.rank % visible device count                    */
#define PR_DEVICE_NONE (-2)      /* host-only context: ingest parses, nothing runs on a GPU */

typedef struct pr_ctx pr_ctx;

/* Replaces the hard-coded job constants of PageRank.java: iteration count (:92),
 * damping 0.15/0.85 (:143), top-K 100 (:189,:193), output ./topPage (:192). */
typedef struct {
  int32_t device;   /* HIP device ordinal, or PR_DEVICE_FROM_RANK / PR_DEVICE_NONE        */
  int32_t n_ranks;  /* processes (GPUs) sharing the graph; 1 = single GPU                 */
  int32_t rank;     /* this process's rank, 0 <= rank < n_ranks                           */
  uint32_t topk;    /* rows written by pr_write_top_page; 100 = reference (:189)          */
  uint32_t flags;   /* PR_F_* below                                                       */
  uint32_t reserved[7];
} pr_opts;

#define PR_F_TRACK_RESIDUAL 0x1u /* compute the exact L1 residual every iteration          */
#define PR_F_VERBOSE 0x2u        /* phase timings on stderr                                */
#define PR_F_NORMALIZED 0x4u     /* normalized PageRank (not in the reference):
                                    r^0 = 1/N_tot and r' = 0.15/N_tot + (c + a)*0.85, so the
                                    ranks sum to ~1 instead of ~N_tot (PageRank.java:78,:143
                                    use 1.0 and 0.15)                                       */

typedef struct {
  int32_t iterations;     /* iterations executed                                          */
  int32_t failed_iteration; /* 1-based iteration that hit PR_E_EMPTY_DANGLING, else 0    */
  double ms_total;        /* device time of the whole iteration loop (HIP events)          */
  double ms_per_iter;
  double ms_spmv_kernel;  /* average duration of the fused SpMV kernel per iteration       */
  double gteps;           /* nnz / ms_per_iter                                            */
  double residual;        /* last relative L1 residual sum|r'-r| / sum r' (if tracked)    */
  double rank_sum;        /* sum of ranks after the run (exact; if tracked)               */
  uint64_t nnz;           /* distinct edges of the whole graph                            */
  uint64_t n_vertices;
  uint64_t defined;       /* vertices with a defined rank after the run (whole graph)      */
  uint64_t bytes_per_iter;/* algorithmic bytes per iteration                  */
  uint64_t reserved[6];
} pr_stats;

typedef struct {
  uint64_t n_vertices;    /* dense vertex slots (ids seen in arcs or mapping)             */
  uint64_t raw_edges;     /* arc lines / generated edges                                  */
  uint64_t nnz;           /* distinct (src,dst) pairs: distinct() at PageRank.java:42     */
  uint64_t n_tot;         /* mappingFile.distinct().count(), PageRank.java:60             */
  uint64_t n_pairs;       /* distinct (id,title) pairs, PageRank.java:51                  */
  uint64_t dangling_entries; /* |subtractByKey(...).keys()|, PageRank.java:56              */
  uint64_t n_sources;     /* keys of adjacencyList (outdeg >= 1), PageRank.java:42,76     */
  uint64_t n_rows;        /* vertices with in-degree >= 1 (whole graph)                   */
  uint64_t local_rows;    /* rows owned by this rank                                      */
  uint64_t local_nnz;     /* edges owned by this rank                                     */
  double ms_ingest;       /* host parse + hashing                                         */
  double ms_build;        /* device CSR build                                             */
  uint64_t ingest_flags;  /* bit 0: the text was parsed on the host because it does not fit
                             the device ingest (>= 2^30 id tokens or device memory)         */
  uint64_t place_tried;   /* placements of the per-piece sums the build timed beyond the first */
  double place_ms_first;  /* stream launch with the array as first allocated, 0 = not timed   */
  double place_ms_best;   /* ... and with the placement the build kept                        */
  uint64_t reserved[2];
} pr_graph_info;

/* Library version "major.minor". */
const char* pr_version(void);
/* Identity of the sources the library was compiled from (hash of csrc/, include/ and the
 * Makefile, page-rank-and-tfidf-using-apache-spark_amd/source_hash.py).  The tests compare it
 * with the checked-out tree, so a stale binary is never tested as HEAD. */
const char* pr_build_id(void);
void pr_opts_default(pr_opts* opts);

/* SparkConf + JavaSparkContext (PageRank.java:22-23): binds the device / rank. */
int pr_create(pr_ctx** out, const pr_opts* opts);
/* spark.stop()-equivalent: frees device memory and the id table. */
void pr_destroy(pr_ctx* ctx);
/* Message of the last failing call on this context ("" if none). */
const char* pr_last_error(const pr_ctx* ctx);

/* Multi-GPU rendezvous.  Replaces the Spark shuffle transport that moves contributions
 * between executors (reduceByKey at PageRank.java:139) with RCCL over xGMI. */
int pr_comm_unique_id(uint8_t id_out[128]);
int pr_comm_init(pr_ctx* ctx, const uint8_t id[128]);

/* Single-process rank group: n contexts created with n_ranks = n and rank = 0..n-1 (on one
 * device or several) exchange x and the partial records by device copies instead of RCCL.
 * Then call the ingest/generate function on every member, pr_run_group() for the rounds,
 * and pr_get_ranks / pr_topk / pr_write_top_page on any member. */
int pr_comm_init_local(pr_ctx** ctxs, int32_t n);
int pr_run_group(pr_ctx** ctxs, int32_t n, int32_t iterations, double tol, pr_stats* stats);

/* Caller-staged exchange: the per-round exchange of the reduceByKey shuffle (:139) and of
 * the dangling reduce (:125) over a transport the caller owns (MPI, a host collective, ...)
 * instead of RCCL.  One process per rank, contexts with n_ranks > 1 and
 * pr_comm_init_external() before the graph is built.  Then per run:
 *   pr_ext_begin(ctx, T, tol, &unit)            unit = bytes each rank contributes per round
 *   for t = 1..T:
 *     pr_ext_round(ctx, t, send)                round t's SpMV; send <- this rank's unit
 *     <caller all-gathers the p units, rank order, into recv (p * unit bytes)>
 *     pr_ext_complete(ctx, t, recv, &stop)      peers' units in, next round's addthis;
 *                                               stop = 1 once the residual is <= tol
 *   pr_ext_end(ctx, &stats)
 * pr_ext_complete returns PR_E_EMPTY_DANGLING where the reference dies (:125).  Buffers are
 * caller-owned host memory.  Outputs of an externally exchanged context are this rank's only:
 * pr_get_ranks returns its pages' ranks (0.0 elsewhere; the caller sums over ranks) and
 * pr_topk its pages' top rows. */
int pr_comm_init_external(pr_ctx* ctx);
int pr_ext_begin(pr_ctx* ctx, int32_t iterations, double tol, uint64_t* bytes_per_rank);
int pr_ext_round(pr_ctx* ctx, int32_t t, void* send);
int pr_ext_complete(pr_ctx* ctx, int32_t t, const void* recv_all, int32_t* stop);
int pr_ext_end(pr_ctx* ctx, pr_stats* stats);

/* Diagnostics (no counterpart in the reference; Spark's web UI and log4j lines play this role
 * there).  pr_progress reports the round loop that is running or ran last on this context:
 * rounds whose work has been handed to the device and rounds the device has finished.  It may
 * be called from another thread while pr_run / pr_run_group block, e.g. by a watchdog that
 * wants to name the round in which a multi-GPU exchange stopped making progress.
 * pr_comm_query reports the transport behind a context (0 none, 1 RCCL, 2 in-process rank
 * group, 3 caller-staged) and, for RCCL, ncclCommCount / ncclCommUserRank of its communicator. */
int pr_progress(pr_ctx* ctx, int32_t* rounds_enqueued, int32_t* rounds_done);
/* Self-test behind the "same graph, same bits" property of reduceByKey(Sum)'s replacement
 * (PageRank.java:139, :208-213 leave the order of the adds open; the engine fixes it): the row
 * launch adds a row's pieces with one LDS double-add instruction per 64 pieces, and lanes of
 * one instruction that hit the same row are applied in an order the hardware chooses.  This
 * call issues that instruction form with `cases` different lane / row / value patterns,
 * `launches` times each, from 8192 waves spread over every compute unit, and compares all
 * accumulators bit for bit: *copies = accumulator sets compared, *differing = sets that differ
 * from the first of their pattern (0 = the order is a function of the pattern alone),
 * *lane_order_cases = patterns whose bits equal the serial sum in ascending lane order. */
int pr_selftest_sum_order(pr_ctx* ctx, uint32_t cases, uint32_t launches, uint64_t* copies,
                          uint64_t* differing, uint64_t* lane_order_cases);

/* Measurement aid without a counterpart in the reference: moves one of the arrays a round
 * touches ("partial" = the per-piece sums between the two launches of PageRank.java:139's
 * replacement, "col16", "col", "bits", "roffL", "x", "maps", "meta") to a fresh device
 * allocation -- new buffer, device copy, old one freed.  Results do not change; the round's time
 * can: the stream launch's rate depends on which physical memory the partial array occupies
 * (scripts/probes/placement_probe.cpp).  PR_CONTIG=1 asks for a physically contiguous buffer,
 * PR_VMM_MB=m / PR_VMM_KB=k for a virtual range backed by separately created chunks (PR_VMM_GAP_GB=g:
 * g GB of device memory skipped between consecutive chunks). */
int pr_debug_move_array(pr_ctx* ctx, const char* name);
int pr_comm_query(pr_ctx* ctx, int32_t* transport, int32_t* comm_ranks, int32_t* comm_rank);

/* The engine's partitioner, on the host.  Spark's HashPartitioner decides which executor owns
 * a key of the reduceByKey shuffle (PageRank.java:139) and the join at :95; here rows are dealt
 * to ranks in chunks of 16 internal vertex ids and every source's contribution has a fixed
 * place in the x vector (slice-major when n_ranks divides 8).  pr_layout_map evaluates the very
 * functions the kernels use, compiled for the host (no device needed): for `count` internal
 * vertex ids (the engine's order: class A = pages with in- and out-links [0, n_a), class B =
 * in-links only [n_a, n_a + n_b), class C = out-links only, the next n_c) it writes the owner
 * rank and local row of each row (0xFFFFFFFF where the id is not a row) and the x position of
 * each column (~0 where it is not a column) as rank `rank` of `n_ranks` holds them; dims_out =
 * {x slot length per rank, x length, local rows, local class-A rows}.  Any output may be NULL. */
int pr_layout_map(int32_t n_ranks, int32_t rank, uint32_t n_a, uint32_t n_b, uint32_t n_c,
                  uint64_t count, const uint32_t* internal_ids, uint32_t* owner_out,
                  uint32_t* local_row_out, uint64_t* x_pos_out, uint64_t dims_out[4]);

/* textFile(arcs)/textFile(mapping) + mapToPair(split) + distinct + groupByKey + cache +
 * subtractByKey + distinct().count() (PageRank.java:26-60), then the device CSR build. */
int pr_ingest_files(pr_ctx* ctx, const char* arcs_path, const char* mapping_path);
int pr_ingest_buffers(pr_ctx* ctx, const char* arcs, size_t arcs_len,
                      const char* mapping, size_t mapping_len);

/* In-memory graph (ids already dense, 0..n-1): the same job on a pre-parsed link list.
 * mapw[v] = number of distinct titles of v (0 = v absent from the mapping); n_tot as
 * PageRank.java:60.  mapw may be NULL (every id mapped once, n_tot = n). */
int pr_load_edges(pr_ctx* ctx, const uint32_t* src, const uint32_t* dst, uint64_t m,
                  uint32_t n, const uint32_t* mapw, uint64_t n_tot);

/* Synthetic Graph500 R-MAT (a,b,c,d = .57,.19,.19,.05), edge_factor << scale edges,
 * generated on the device (Philox-4x32-10 keyed by seed and edge index); mapping = every
 * id 0..2^scale-1 once with title "v<id>", n_tot = 2^scale. */
int pr_generate_rmat(pr_ctx* ctx, int32_t scale, int32_t edge_factor, uint64_t seed);

int pr_graph_get_info(pr_ctx* ctx, pr_graph_info* out);

/* The loop at PageRank.java:92-164: `iterations` rounds of contribution SpMV + dangling
 * redistribution + damping.  tol > 0 stops early once the relative L1 residual is <= tol
 * (implies PR_F_TRACK_RESIDUAL).  Returns PR_E_EMPTY_DANGLING where the reference job
 * would die at :125 (stats->failed_iteration says which round).  Collective. */
int pr_run(pr_ctx* ctx, int32_t iterations, double tol, pr_stats* stats);

/* pr_run without allocation.  No counterpart in the reference: it exists for callers that
 * cannot allocate device memory while they run rounds (code under HIP graph capture, tight
 * serving loops, harnesses that forbid hipMalloc).  Same rounds, same kernels and bit-identical
 * ranks as pr_run on a single-GPU context (n_ranks = 1), but everything a round writes besides
 * the context's own x / rank vectors -- the per-piece partial sums, the record shards, the round
 * record and the round state -- lives in a fixed file-scope device array (32 MiB + 66 KiB per
 * GPU, held until the process ends) instead of the context's buffers, and the call makes no
 * hipMalloc / hipFree (its state reset and clears are kernel launches, per-round kernel timing
 * is off: stats->ms_spmv_kernel = 0).  Limit: graphs of at most 4 Mi piece sums per round
 * (about 10 M distinct edges); larger ones get PR_E_ARG with the sizes in pr_last_error.
 * Every context on one GPU shares that GPU's array: calls that overlap in time on one GPU race
 * (calls in sequence are fine: each call resets what must start at zero). */
int pr_run_static(pr_ctx* ctx, int32_t iterations, double tol, pr_stats* stats);

/* Resume (the reference has no checkpoint).  pr_set_ranks seeds the
 * following pr_run calls with ranks by vertex id (as pr_get_ranks returns them, 0.0 =
 * undefined) reached after `rounds_done` >= 1 rounds: pr_run(T) then computes rounds
 * rounds_done+1 .. rounds_done+T of one uninterrupted run, bit-identical to it (the seed's
 * x = r/outdeg and exact dangling mass equal the engine's own).  Only pages with in-links
 * may carry a rank.  ranks == NULL clears the seed.  Every rank passes the whole vector.
 * pr_checkpoint_save writes the last run's ranks with the total round count and the graph's
 * identity (vertex count, nnz, N_tot, edge digest, PR_F_NORMALIZED); rank 0 writes, the
 * call is collective.  pr_checkpoint_load checks the identity against the current graph
 * and seeds from the file. */
int pr_set_ranks(pr_ctx* ctx, const double* ranks, uint64_t n, int32_t rounds_done);
int pr_checkpoint_save(pr_ctx* ctx, const char* path);
int pr_checkpoint_load(pr_ctx* ctx, const char* path);

/* Final `ranks` RDD as a dense array indexed by vertex id (0.0 = no rank: the page is
 * absent from the reference's ranks RDD).  n must be >= n_vertices.  Collective. */
int pr_get_ranks(pr_ctx* ctx, double* out, uint64_t n);

/* ranks.join(mappings) -> sortByKey(false) -> take(k) (PageRank.java:167-189).  Writes up
 * to k rows: pair index (into the distinct (id,title) pairs, see pr_pair), vertex id and
 * rank, descending by rank; equal ranks ordered by (title bytes, id).  *count = rows
 * written.  Collective. */
int pr_topk(pr_ctx* ctx, uint32_t k, uint64_t* pair_out, uint32_t* id_out, double* rank_out,
            uint32_t* count);

/* FileWriter("./topPage") loop (PageRank.java:190-204): `title \t Double.toString(rank)`
 * for the top opts.topk rows.  Only rank 0 writes.  Collective. */
int pr_write_top_page(pr_ctx* ctx, const char* path);

/* Full rank dump (extends the output contract of PageRank.java:167-204):
 * every page of the final ranks RDD, in vertex-id order (first appearance in the input), one
 * line per mapping pair of the page -- `id \t title \t Double.toString(rank)` -- i.e. the
 * rows of ranks.join(mappings) (:168) without sortByKey/take; a ranked page with no title
 * gets one line with an empty title.  Only rank 0 writes.  Collective. */
int pr_write_rank_dump(pr_ctx* ctx, const char* path);

/* Id / title strings (the reference's String keys).  *len = full length; at most cap
 * bytes copied.  For generated / in-memory graphs the id string is the decimal id. */
int pr_id_string(pr_ctx* ctx, uint32_t v, char* buf, size_t cap, size_t* len);
int pr_pair(pr_ctx* ctx, uint64_t i, uint32_t* id, char* title, size_t cap, size_t* len);

/* Structure checks (bit-exact CSR/degree construction): per-vertex out-degree (distinct
 * out-neighbours, PageRank.java:103-108), in-degree and dangling weight (:56), and an
 * order-free digest {sum, xor} of mix64(src<<32|dst) over the distinct edge set. */
int pr_get_degrees(pr_ctx* ctx, uint32_t* outdeg, uint32_t* indeg, uint32_t* dang_w,
                   uint64_t n);
int pr_edge_digest(pr_ctx* ctx, uint64_t digest_out[2]);

/* Host copy of the pull CSR in the engine's internal numbering (single-rank contexts):
 * a square graph over internal ids 0..n-1 -- row_ptr[n+1] by destination, col = source
 * ids (ascending within a row), out-degree and dangling weight per internal id.  The same
 * graph relabelled, for external baselines.  Pass NULL buffers to query sizes. */
int pr_export_csr(pr_ctx* ctx, uint64_t* row_ptr, uint32_t* col, uint32_t* outdeg,
                  uint32_t* dang_w, uint64_t* n, uint64_t* nnz);

/* ---- the repository's second job: TF-IDF (Spark.java:22-173) ----------
 * Input: the tab-separated dump Spark.java:26 reads (one document per line, title in column
 * 1, text in column 3).  pr_tfidf_ingest_* cleans every text (:38-42), counts (word, title)
 * pairs (:57-71), document frequencies (:75-93) and titleCount = distinct titles (:50-56)
 * on the device; PR_E_PARSE where the reference dies with ArrayIndexOutOfBoundsException
 * (a line without columns[1] or columns[3]; a title made only of commas, :106).
 * pr_tfidf_lookup is idf.lookup(word) + the sort of :140-162: up to k rows (title index,
 * tf * Math.log(titleCount / df) with integer division), tfidf descending, ties by the
 * lowercased title up to its first comma.  pr_tfidf_write_output writes the ./output file
 * of :164-171 ("total docs are N" + the first 100 `title\ttfidf` rows).  Per context;
 * independent of the PageRank graph.  Needs a device. */
int pr_tfidf_ingest_buffer(pr_ctx* ctx, const char* data, size_t len);
int pr_tfidf_ingest_file(pr_ctx* ctx, const char* path);
int pr_tfidf_info(pr_ctx* ctx, uint64_t* docs, uint64_t* words, uint64_t* pairs,
                  uint64_t* tokens);
int pr_tfidf_lookup(pr_ctx* ctx, const char* word, size_t wlen, uint32_t k,
                    uint32_t* title_out, double* tfidf_out, uint32_t* count);
int pr_tfidf_title(pr_ctx* ctx, uint32_t title, char* buf, size_t cap, size_t* len);
int pr_tfidf_write_output(pr_ctx* ctx, const char* word, const char* path);

/* Java Double.toString layout (PageRank.java:197 string concatenation). Returns length. */
int pr_format_double(double v, char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* PRMI355X_H */
