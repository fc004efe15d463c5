// prmi355x device engine (gfx950 / CDNA4).
//
// Replaces, per round, PageRank.java:94-160 -- the contribution flatMapToPair (:94-117), the
// dangling-mass reduce (:121-138), reduceByKey(Sum) (:139, Sum :208-213) and the damping /
// dangling-update maps (:140-160) -- with a pull SpMV over the transposed graph in two
// launches: the stream launch (one XCD per column slice; LDS-blocked gathers; one partial sum
// per piece of a (row, slice, segment) pair) and the row launch (each row's pieces added in a
// fixed order + the fused epilogue), plus two single-workgroup reductions.  The graph build
// (K1) replaces distinct().groupByKey() (:42), the urlCount loop (:103-108) and
// subtractByKey (:56).
//
// Numerics (DESIGN.md "Parity"):
//   * x = r / outdeg is one IEEE division per source (same operands as :113, bit-exact);
//   * each row's sum is an fp64 sum whose order is fixed by the stream layout (deterministic
//     for a given graph and rank count);
//   * r' = 0.15 + (c + a) * 0.85 is evaluated unfused in Java's order (:143);
//   * the dangling mass, residual and rank sum are EXACT (integer superaccumulator, then one
//     correct rounding), so addthis (:135) equals the correctly rounded exact value.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string.h>

#include <rocprim/rocprim.hpp>

#include "engine.h"
#include "prmi355x.h"
#include "sa_round.h"

namespace prmi {

#define HIPTRY(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      if (err) *err = std::string(#x) + ": " + hipGetErrorString(e_);              \
      return e_ == hipErrorOutOfMemory ? PR_E_OOM : PR_E_HIP;                      \
    }                                                                              \
  } while (0)

// =======================================================================================
// device helpers
// =======================================================================================
__device__ __host__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = min(v, __shfl_xor(v, m));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m));
  return v;
}

// Exact fixed-point image of w*v (v >= 0 finite, w < 2^32): returns the first limb index
// li and four 32-bit chunks for limbs li..li+3; -1 when the value is zero / below 2^-96.
__device__ __forceinline__ int sa_chunks(double v, uint32_t w, uint32_t& c0, uint32_t& c1,
                                         uint32_t& c2, uint32_t& c3) {
  c0 = c1 = c2 = c3 = 0;
  if (!(v > 0.0) || w == 0) return -1;
  const uint64_t bits = static_cast<uint64_t>(__double_as_longlong(v));
  const int eb = static_cast<int>((bits >> 52) & 0x7FF);
  uint64_t m = bits & ((1ull << 52) - 1);
  int e;
  if (eb == 0) {
    e = -1074;
  } else {
    m |= 1ull << 52;
    e = eb - 1075;
  }
  int s = e - SA_BASE_EXP;
  unsigned __int128 q = static_cast<unsigned __int128>(m) * w;
  if (s < 0) {
    if (-s >= 128) return -1;
    q >>= -s;
    s = 0;
  }
  q <<= (s & 31);
  c0 = static_cast<uint32_t>(q);
  c1 = static_cast<uint32_t>(q >> 32);
  c2 = static_cast<uint32_t>(q >> 64);
  c3 = static_cast<uint32_t>(q >> 96);
  return s >> 5;
}

// Adds one wave's superaccumulator contributions into lds_wave[base + L].  Only the limb
// window the wave actually touches is reduced (usually 4-5 limbs).
__device__ __forceinline__ void wave_accum_sa(uint64_t* lds_wave, int base, int li, uint32_t c0,
                                              uint32_t c1, uint32_t c2, uint32_t c3) {
  const bool valid = li >= 0;
  const int lo = __builtin_amdgcn_readfirstlane(wave_min_i(valid ? li : 1000));
  int hi = __builtin_amdgcn_readfirstlane(wave_max_i(valid ? li + 3 : -1));
  if (hi > SA_LIMBS - 1) hi = SA_LIMBS - 1;
  for (int L = lo; L <= hi; ++L) {
    const int k = L - li;
    const uint32_t c =
        !valid ? 0u : (k == 0 ? c0 : (k == 1 ? c1 : (k == 2 ? c2 : (k == 3 ? c3 : 0u))));
    const uint64_t s = wave_sum_u64(c);
    if ((threadIdx.x & 63) == 0) lds_wave[base + L] += s;
  }
}

// Correct rounding of a superaccumulator (limbs hold 32-bit chunks plus carries): the
// register-only form of sa_round.h (checked bit for bit against the bit-loop form on the CPU)
static_assert(SA_LIMBS == SA_NLIMBS && SA_BASE_EXP == SA_EXP0, "sa_round.h limb layout");
__device__ __forceinline__ double sa_to_double_dev(const uint64_t* limb) { return sa_round_fast(limb); }

// =======================================================================================
// the round: slice streams (per-piece partial sums) + fused row launch (combine + epilogue)
// =======================================================================================
// Row launch: rows are cut into blocks of RB rows (class-A blocks, then class-B blocks).  For
// every block and every stream k = (slice, segment), the block's pieces of stream k are one
// contiguous run of the partial array (pieces are in stream order, rows ascending inside a
// stream).  The block's non-empty runs, concatenated in stream order, form its piece
// sequence i = 0 .. tot-1; run q covers i in [pre_q, pre_q + len_q) and piece i of run q is
// partial[nebase_q + i] (nebase_q = run start - pre_q).  The sequence is cut into 64-piece
// LINES; for every line the build stores the run of its first piece (lfirst) and a 64-bit
// mask of the positions where a new run starts (lmask), so lane l of a line finds its piece
// as nebase[lfirst + popcount(lmask & bits 1..l)] + i: no search.  Each wave adds a fixed
// quarter of the block's lines into its own LDS accumulator; c[row] = (acc0 + acc1) + (acc2 +
// acc3).  Then PageRank.java's damping / contribution epilogue.
constexpr int RB = 1024;           // rows per row-launch block
constexpr int MAX_NS = 1024;       // streams (slices x segments) the row launch supports
constexpr int EPR = 8;             // lines per wave per step (one piece per lane per line)
struct RowArgs {
  const uint32_t* nebase;  // [ne_off[NB]] per block: start - pre of each non-empty run
  const uint32_t* ne_off;  // [NB + 1] first run of each block in nebase
  const uint32_t* l_off;   // [NB + 1] first line of each block in lfirst / lmask
  const uint32_t* tot;     // [NB] pieces of each block
  const uint32_t* lfirst;  // [lines + pad] run (block-relative) of each line's first piece
  const uint64_t* lmask;   // [lines + pad] bit j: piece j of the line starts a run (j >= 1)
  const double* partial;   // per-piece partial sums of this round
  const uint32_t* roffL;   // row offsets in row-launch order: per 8-line group, lane-major,
                           // lane l's 8 ten-bit values packed 3 per dword (12 bytes: value u
                           // in dword u / 3 at bit 10 (u % 3); RB = 1024 rows need 10 bits)
  uint32_t roffL_bytes;    // bytes of roffL (the buffer-load range)
  uint32_t roff16;         // PR_ROFF16=1: the earlier layout (8 x u16 per lane per group, A/B)
  const uint32_t* goff;    // [NB + 1] first 8-line group of each block
  uint32_t NS, nbA, lA, lrows;
  uint32_t rb;             // rows per block (<= RB)
  uint32_t nbH, rbH, lH;   // heavy blocks: the first lH class-A rows in nbH blocks of rbH rows
  const uint32_t* meta;
  double* x_out;           // this rank's slot of the next x
  const double* r_old;     // tracked mode: previous ranks (nullptr = r^0 == 1)
  double* r_out;
  const IterState* st;
  uint64_t* shards;
  uint32_t p, rank, sm, SL;  // x layout: where local row l's x' goes inside this rank's slot
  uint32_t snake;            // snake chunk -> slice order (chunk_slice)
  uint32_t dbg;              // PR_DBG timing experiments: 16 no LDS adds, 32 no epilogue, 64 no
                             // pieces; 128 non-temporal piece loads (not timing-only)
  double base, r0;           // damping base (0.15) and initial rank (1.0), or their /N_tot forms
  uint32_t b0;               // first row block of this launch (the row launch may be chunked)
  uint32_t xg, xfull;        // XCD groups: xg consecutive blocks per XCD in the first xfull
};

// chunk c (16 columns) -> slice.  Snake order (single rank): c mod 8, reversed in every odd
// group of 8, so the hottest chunk of a group alternates between slice 0 and slice 7 and no
// slice systematically receives the hotter half (chunks are in-degree ordered).  With p > 1
// plain c mod 8, which keeps each rank's chunks in its own slices.
__device__ __host__ __forceinline__ uint32_t chunk_slice(uint32_t c, uint32_t snake) {
  const uint32_t sl = c % NSLICE;
  return (snake && ((c / NSLICE) & 1u)) ? NSLICE - 1 - sl : sl;
}
// the chunk of slice sl in group g (inverse of chunk_slice)
__device__ __host__ __forceinline__ uint32_t slice_chunk(uint32_t g, uint32_t sl, uint32_t snake) {
  return g * NSLICE + ((snake && (g & 1u)) ? NSLICE - 1 - sl : sl);
}
// offset of local row l's x entry inside this rank's slot (see Layout / xpos)
__device__ __forceinline__ uint32_t xslot_of(const RowArgs& A, uint32_t l) {
  if (!A.sm) return l;
  const uint32_t c = (l / CHUNK) * A.p + A.rank, sl = chunk_slice(c, A.snake);
  return (sl / A.p) * A.SL + (c / NSLICE) * CHUNK + (l % CHUNK);
}


// Epilogue of one row (leader = the row exists): r', x' or the row's dangling weight, and in
// tracked mode r'; the exact partials (dangling mass + count for class-B rows; residual +
// rank sum in tracked mode) go into this wave's LDS record (flushed once per block).
template <int MODE>
__device__ __forceinline__ void row_finish(const RowArgs& A, double a, uint32_t cls,
                                           uint32_t row, double c, bool leader, uint32_t mt,
                                           double ro, uint64_t* lw) {
  double r = 0.0;
  uint32_t w = 0;
  if (leader) {
    // PageRank.java:143  0.15 + (sum + addthis) * 0.85, unfused (base = 0.15 / N_tot when
    // normalized)
    r = c > 0.0 ? __dadd_rn(A.base, __dmul_rn(__dadd_rn(c, a), 0.85)) : 0.0;
    if (cls == 0)
      A.x_out[xslot_of(A, row)] = r / static_cast<double>(mt);  // :113  rank / urlCount
    else
      w = mt;
    if (MODE >= 1) A.r_out[row] = r;
  }
  uint32_t c0, c1, c2, c3;
  if (cls == 1) {  // uniform over the workgroup
    // PageRank.java:125-134  sum of danglingMap values (w entries per page)
    const int li = sa_chunks(leader ? r : 0.0, w, c0, c1, c2, c3);
    wave_accum_sa(lw, REC_DSUM, li, c0, c1, c2, c3);
    const uint64_t cnt = wave_sum_u64((leader && r > 0.0) ? w : 0u);
    if ((threadIdx.x & 63) == 0) lw[REC_DCNT] += cnt;
  }
  if (MODE == 2) {
    const double d = fabs(r - ro);
    int li = sa_chunks(leader ? d : 0.0, 1u, c0, c1, c2, c3);
    wave_accum_sa(lw, REC_RESID, li, c0, c1, c2, c3);
    li = sa_chunks(leader ? r : 0.0, 1u, c0, c1, c2, c3);
    wave_accum_sa(lw, REC_RSUM, li, c0, c1, c2, c3);
  }
}

// the block's 4 wave records -> one atomic shard (after a barrier)
__device__ __forceinline__ void flush_records(const RowArgs& A, uint64_t (*lds)[REC_WORDS]) {
  if (threadIdx.x < REC_WORDS) {
    const int t = threadIdx.x;
    const uint64_t s = (lds[0][t] + lds[1][t]) + (lds[2][t] + lds[3][t]);
    if (s) atomicAdd(reinterpret_cast<unsigned long long*>(
                         &A.shards[(blockIdx.x % NSHARD) * REC_WORDS + t]),
                     static_cast<unsigned long long>(s));
  }
}

// The row launch (PageRank.java:139-145 reduceByKey(Sum) + mapValues, and the inputs of
// :113 and :125-134 for the next round).
template <int MODE>
__global__ __launch_bounds__(BLOCK) void spmv_rows(RowArgs A) {
  __shared__ double acc[4][RB];
  __shared__ uint32_t nb[MAX_NS];   // the block's non-empty runs: start - pre
  __shared__ uint64_t lds[4][REC_WORDS];
  // workgroups go round-robin over the 8 XCDs: give each XCD runs of xg consecutive blocks,
  // so the piece lines that two neighbouring blocks' runs share are fetched into one L2
  uint32_t bl = blockIdx.x;
  if (bl < A.xfull) {
    const uint32_t span = NSLICE * A.xg, r = bl % span;
    bl = (bl - r) + (r % NSLICE) * A.xg + r / NSLICE;
  }
  const uint32_t b = bl + A.b0;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < 4 * RB; i += BLOCK) (&acc[0][0])[i] = 0.0;
  for (int i = tid; i < 4 * REC_WORDS; i += BLOCK) (&lds[0][0])[i] = 0;
  // the block's rows; their epilogue inputs are loaded now, used after the piece loop
  const bool clsB = b >= A.nbA;
  // the highest in-degree rows (one piece per stream each) come first in smaller blocks, so
  // no single block's piece loop outlasts the launch when a rank holds few blocks
  const bool heavy = b < A.nbH;
  const uint32_t rb0 = clsB ? A.lA + (b - A.nbA) * A.rb
                            : (heavy ? b * A.rbH : A.lH + (b - A.nbH) * A.rb);
  const uint32_t rb1 = min(rb0 + (heavy ? A.rbH : A.rb), clsB ? A.lrows : A.lA);
  constexpr int RPT = RB / BLOCK;  // rows per thread
  uint32_t mt[RPT];
  double ro[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const uint32_t row = rb0 + tid + q * BLOCK;
    mt[q] = row < rb1 ? A.meta[row] : 0u;
    ro[q] = 0.0;
    if (MODE == 2 && row < rb1) ro[q] = A.r_old ? A.r_old[row] : A.r0;
  }
  const uint32_t ne0 = A.ne_off[b], nne = A.ne_off[b + 1] - ne0;
  const uint32_t tot = A.tot[b];
  const uint32_t L0 = A.l_off[b], nl = A.l_off[b + 1] - L0;
  const uint32_t G0 = A.goff[b];
  // this wave's quarter of the block's 8-line groups; a step = one group (EPR lines), lane l
  // takes piece l of each line and the group's 8 row offsets of lane l in one 16-byte load
  const uint32_t ng = (nl + EPR - 1) / EPR;
  const uint32_t lo = (ng * wv / 4) * EPR;
  const uint32_t hi = min((ng * (wv + 1) / 4) * EPR, nl);
  double* aw = acc[wv];
  const uint64_t lbits = (2ull << lane) - 2ull;  // bits 1 .. lane
  double va[EPR], vb[EPR], sink = 0.0;
  uint32_t ra[EPR], rbuf[EPR];
  uint32_t fa[EPR];
  uint64_t ma[EPR];
  // line maps of a step, fetched one step ahead of their use: wave-uniform, so scalar loads
  // (constant address space + a readfirstlane index) that leave the vector memory pipe to
  // the piece reads; the arrays are padded by 2 * EPR lines, so a step may read past the
  // block's lines (those lanes are masked)
  typedef const __attribute__((address_space(4))) uint32_t* cu32p;
  typedef const __attribute__((address_space(4))) uint64_t* cu64p;
  const cu32p lf = (cu32p)(A.lfirst);
  const cu64p lm = (cu64p)(A.lmask);
  auto maps = [&](uint32_t L) {
    const uint32_t Lb = __builtin_amdgcn_readfirstlane(L0 + L);
#pragma unroll
    for (int u = 0; u < EPR; ++u) {
      fa[u] = lf[Lb + u];
      ma[u] = lm[Lb + u];
    }
  };
  typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
  const __amdgpu_buffer_rsrc_t rofr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(A.roffL), static_cast<short>(0), static_cast<int>(A.roffL_bytes), 0x00020000);
  auto issue = [&](uint32_t L, double (&vv)[EPR], uint32_t (&rr)[EPR]) {
#pragma unroll
    for (int u = 0; u < EPR; ++u) {
      const uint32_t i = (L + u) * 64u + static_cast<uint32_t>(lane);
      const uint32_t q = fa[u] + static_cast<uint32_t>(__popcll(ma[u] & lbits));
      const uint32_t pc = (L + u < hi && i < tot) ? nb[q] + i : 0u;  // never past the pieces
      if (A.dbg & 128u) vv[u] = __builtin_nontemporal_load(A.partial + pc);  // experiment
      else vv[u] = A.partial[pc];
    }
    // one 12-byte load per step: lane l's 8 row offsets, 10 bits each (buffer offsets are
    // 32-bit: roffL stays below 4 GiB, 768 bytes per 8-line group)
    if (A.roff16) {
      typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
      const u16x8 r8 = *reinterpret_cast<const u16x8*>(
          reinterpret_cast<const uint16_t*>(A.roffL) +
          ((static_cast<uint64_t>(G0 + L / EPR) * 64u) + static_cast<uint32_t>(lane)) * EPR);
#pragma unroll
      for (int u = 0; u < EPR; ++u) rr[u] = r8[u];
    } else {
      const u32x3 r3 = __builtin_amdgcn_raw_buffer_load_b96(
          rofr, ((G0 + L / EPR) * 64u + static_cast<uint32_t>(lane)) * 12u, 0, 0);
#pragma unroll
      for (int u = 0; u < EPR; ++u) rr[u] = (r3[u / 3] >> (10 * (u % 3))) & 0x3FFu;
    }
    maps(L + EPR);
  };
  auto add = [&](uint32_t L, const double (&vv)[EPR], const uint32_t (&rr)[EPR]) {
    // LDS adds in lane order inside each instruction: a fixed order for a fixed layout
#pragma unroll
    for (int u = 0; u < EPR; ++u)
      if (L + u < hi && (L + u) * 64u + static_cast<uint32_t>(lane) < tot) {
        if (A.dbg & 16u) sink += vv[u] + rr[u];
        else atomicAdd(&aw[rr[u]], vv[u]);
      }
  };
  const uint32_t hi_loop = (A.dbg & 64u) ? lo : hi;  // timing: no piece loads at all
  if (lo < hi_loop) maps(lo);  // (scalar loads: in flight beside the run bases)
  for (uint32_t q = tid; q < nne; q += BLOCK) nb[q] = A.nebase[ne0 + q];
  __syncthreads();
  if (lo < hi_loop) issue(lo, va, ra);
  for (uint32_t L = lo; L < hi_loop; L += 2 * EPR) {
    const bool n1 = L + EPR < hi, n2 = L + 2 * EPR < hi;
    if (n1) issue(L + EPR, vb, rbuf);
    add(L, va, ra);
    if (n2) issue(L + 2 * EPR, va, ra);
    if (n1) add(L + EPR, vb, rbuf);
  }
  if (A.dbg & 16u) aw[lane] = sink;
  __syncthreads();
  if (A.dbg & 32u) return;
  // epilogue over the block's rows
  const double a = A.st->a;
  uint64_t* lw = lds[wv];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int l = tid + q * BLOCK;
    const uint32_t row = rb0 + l;
    double c = (acc[0][l] + acc[1][l]) + (acc[2][l] + acc[3][l]);
    if (A.dbg & 64u) c = 1.0;
    row_finish<MODE>(A, a, clsB ? 1u : 0u, row, c, row < rb1, mt[q], ro[q], lw);
  }
  if (clsB || MODE == 2) {  // uniform over the workgroup
    __syncthreads();
    flush_records(A, lds);
  }
}

// ---- the stream launch: persistent, slice j = blockIdx % 8 (one XCD per slice) ----------
// Slice j's stream is cut into tasks of TASK = 1024 edges; wave w of the XCD takes tasks
// w, w + W, w + 2W, ... (W = waves per XCD), so the XCD sweeps the stream front to back and
// its L2 holds the segment being swept.  Lane i of a task owns edges [16i, 16i+16): four
// 16-byte column loads, a 16-bit pair-start mask, sixteen independent gathers (the first H
// entries of the slice's region from an LDS copy).  Pieces are summed in edge order inside
// a lane; pieces that cross lanes are joined by a segmented scan over the wave.  Every
// summation order is fixed by the stream layout (deterministic).
struct StreamArgs {
  const uint32_t* col;       // L2-group edges: x position (u32)
  const uint16_t* col16;     // LDS-group edges: offset inside the LDS block (u16; H = zero slot)
  const uint64_t* gbase;     // [groups] first edge of each group in col / col16
  const uint16_t* bits;
  const uint32_t* task_piece;
  const uint32_t* gtask;     // [8 * (nlds + 1) + 1] first task of each stream group
  const double* x_in;
  double* partial;
  uint32_t hot_base[NSLICE]; // x position of each slice region's start
  uint32_t nlds, H;          // LDS blocks per slice, entries per block
  uint32_t colmask;          // PR_COLMASK (timing experiments only)
  uint32_t dbg;              // PR_DBG timing experiments: 1 no stores, 2 no L2 gathers, 4 no
                             // starts, 8 no LDS gathers, 2048 / 4096 LDS-group / L2-group
                             // columns from L2 (wrong sums)
  uint32_t x_bytes;          // bytes of x (< 2^31: the buffer-load range check drops LDS lanes
                             // and PAD_COL padding)
  uint32_t l2mode;           // PR_L2MODE: 0 = L2 tasks interleaved 1/nlds per LDS phase,
                             //            1 = all L2 tasks in one final phase
  uint64_t* stamps;          // PR_STAMPS diagnostics: per (workgroup, phase) the phase start
                             // and every wave's end (s_memrealtime, 100 MHz); nullptr = off
  uint32_t l2w;              // PR_L2W: waves per workgroup dedicated to the L2 group (0 = the
                             // L2 tasks are shared out over the LDS phases, see l2mode)
  uint32_t wgdyn;            // PR_WGDYN: LDS waves claim their workgroup's tasks from an LDS
                             // counter (1) or take them round-robin (0)
  uint32_t* gcnt;            // [NSLICE * GCNT] task counters of the slice-wide claims (zero at launch)
  uint32_t early;            // PR_EARLY: first task of a phase claimed and fetched before its barrier
  uint32_t dyng;             // tasks per slice-wide claim (PR_DYNG)
  uint32_t l2dyn;            // PR_DYNL2: the L2-role waves claim their tasks slice-wide as well
  uint32_t dyn0;             // LDS phases >= dyn0 deal their tasks to the slice's workgroups from
                             // gcnt instead of in fixed shares (PR_DYNTAIL)
  uint32_t l2lo[NSLICE];     // L2-group tasks [l2lo, l2hi) of each slice this launch sweeps
  uint32_t l2hi[NSLICE];
  uint32_t ph_lo, ph_hi;     // LDS phases [ph_lo, ph_hi) this launch runs (all of them unless
                             // the launch is one part of a cut launch)
  uint32_t part;             // 2 with ph_lo == ph_hi: no LDS phase at all, every wave sweeps
                             // the L2 tasks above; otherwise informational
  uint32_t l2late;           // PR_L2LATE: the L2-role waves issue the next task's column loads
                             // after their sixteen gathers have landed instead of before them
                             // (vmcnt counts in order: gathers issued behind the prefetch wait
                             // for it), A/B switch
};
constexpr int STREAM_BLOCK = 1024;
constexpr uint32_t GCNT = 72;      // slice-wide task counters per slice: one per LDS phase (<= 64),
                                   // slots 64 / 65 for the L2 role (whole or first part / second part)
constexpr int STG = 256;           // per-wave LDS staging window for piece stores (doubles)
// LDS left for the x block: H entries + a zero slot (index H, the 16-bit padding column)
constexpr uint32_t HOT_MAX = 20480 - (STREAM_BLOCK / 64) * STG - 8;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ---- DPP cross-lane steps (gfx9 wave64: row shifts, row broadcasts, wave shifts) ----------
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114,
              DPP_ROW_SHR8 = 0x118, DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143,
              DPP_WAVE_SHL1 = 0x130, DPP_WAVE_SHR1 = 0x138;
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);  // invalid source -> 0
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = static_cast<uint64_t>(__double_as_longlong(v));
  const uint32_t lo = static_cast<uint32_t>(dpp_i<CTRL>(static_cast<int>(u)));
  const uint32_t hi = static_cast<uint32_t>(dpp_i<CTRL>(static_cast<int>(u >> 32)));
  return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
}
// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
  const int rl = lane & 15;
  int t;
  t = dpp_i<DPP_ROW_SHR1>(v); if (rl >= 1) v += t;
  t = dpp_i<DPP_ROW_SHR2>(v); if (rl >= 2) v += t;
  t = dpp_i<DPP_ROW_SHR4>(v); if (rl >= 4) v += t;
  t = dpp_i<DPP_ROW_SHR8>(v); if (rl >= 8) v += t;
  t = dpp_i<DPP_ROW_BCAST15>(v); if (lane & 16) v += t;   // rows 1, 3 add lanes 15, 47
  t = dpp_i<DPP_ROW_BCAST31>(v); if (lane >= 32) v += t;  // rows 2, 3 add lane 31
  return v;
}
// segmented inclusive scan: (F, S) o (F', S') = (F | F', F' ? S' : S + S'), F = lane starts a
// segment; the same fixed combination tree for a given flag pattern
__device__ __forceinline__ double wave_seg_scan(double S, int F, int lane) {
  const int rl = lane & 15;
  double Su;
  int Fu;
#define PRMI_SEG_STEP(CTRL, COND)          \
  Su = dpp_d<CTRL>(S);                     \
  Fu = dpp_i<CTRL>(F);                     \
  if (COND) {                              \
    if (!F) S = Su + S;                    \
    F |= Fu;                               \
  }
  PRMI_SEG_STEP(DPP_ROW_SHR1, rl >= 1)
  PRMI_SEG_STEP(DPP_ROW_SHR2, rl >= 2)
  PRMI_SEG_STEP(DPP_ROW_SHR4, rl >= 4)
  PRMI_SEG_STEP(DPP_ROW_SHR8, rl >= 8)
  PRMI_SEG_STEP(DPP_ROW_BCAST15, (lane & 16) != 0)
  PRMI_SEG_STEP(DPP_ROW_BCAST31, lane >= 32)
#undef PRMI_SEG_STEP
  return S;
}

// ---- lean forms (the LEAN stream variant): the same sums in the same order, fewer VALU ops.
// The scan steps need no per-lane conditions: row shifts zero-fill the lanes whose source lies
// outside the row (bound_ctrl), and the row broadcasts only write the rows that take them
// (row mask 0xA / 0xC; the other rows keep the zero `old`).  A lane that reads zero adds
// nothing: S + 0 = S, F | 0 = F.
template <int CTRL>
__device__ __forceinline__ int dppz_i(int v) {
  if constexpr (CTRL == DPP_ROW_BCAST15) return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xA, 0xF, false);
  else if constexpr (CTRL == DPP_ROW_BCAST31) return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xC, 0xF, false);
  else return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dppz_d(double v) {
  const uint64_t u = static_cast<uint64_t>(__double_as_longlong(v));
  const uint32_t lo = static_cast<uint32_t>(dppz_i<CTRL>(static_cast<int>(u)));
  const uint32_t hi = static_cast<uint32_t>(dppz_i<CTRL>(static_cast<int>(u >> 32)));
  return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
}
__device__ __forceinline__ int wave_incl_scan_lean(int v) {
  v += dppz_i<DPP_ROW_SHR1>(v);
  v += dppz_i<DPP_ROW_SHR2>(v);
  v += dppz_i<DPP_ROW_SHR4>(v);
  v += dppz_i<DPP_ROW_SHR8>(v);
  v += dppz_i<DPP_ROW_BCAST15>(v);
  v += dppz_i<DPP_ROW_BCAST31>(v);
  return v;
}
// the segmented scan of wave_seg_scan with the combine S = F ? S : Su + S written as
// fma(Su, !F, S): for !F = 1 that is the correctly rounded Su + S, for !F = 0 exactly S
__device__ __forceinline__ double wave_seg_scan_lean(double S, int F) {
#define PRMI_SEG_STEP_L(CTRL)                                                   \
  {                                                                             \
    const double Su = dppz_d<CTRL>(S);                                          \
    const int Fu = dppz_i<CTRL>(F);                                             \
    S = __builtin_fma(Su, static_cast<double>(static_cast<uint32_t>(F ^ 1)), S); \
    F |= Fu;                                                                    \
  }
  PRMI_SEG_STEP_L(DPP_ROW_SHR1)
  PRMI_SEG_STEP_L(DPP_ROW_SHR2)
  PRMI_SEG_STEP_L(DPP_ROW_SHR4)
  PRMI_SEG_STEP_L(DPP_ROW_SHR8)
  PRMI_SEG_STEP_L(DPP_ROW_BCAST15)
  PRMI_SEG_STEP_L(DPP_ROW_BCAST31)
#undef PRMI_SEG_STEP_L
  return S;
}
// byte offset (x 8) of the low / high 16-bit half of a word in one SDWA shift
__device__ __forceinline__ uint32_t lds_off_lo(uint32_t w) {
  uint32_t r;
  asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
      : "=v"(r) : "v"(w));
  return r;
}
__device__ __forceinline__ uint32_t lds_off_hi(uint32_t w) {
  uint32_t r;
  asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
      : "=v"(r) : "v"(w));
  return r;
}

// Sixteen exec-masked buffer gathers x[off/8] into v[k] (lanes outside gm[k] keep v[k]),
// then one s_waitcnt: the asm block ends with its loads landed, so the compiler never sees
// an in-flight destination.
__device__ __forceinline__ void gather16(double (&v)[EPL], const uint32_t (&qo)[EPL],
                                         const uint64_t (&gm)[EPL], __amdgpu_buffer_rsrc_t xr) {
  uint64_t sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n"
      "s_and_b64 exec, %[sv], %[m0]\n  buffer_load_dwordx2 %[d0], %[o0], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m1]\n  buffer_load_dwordx2 %[d1], %[o1], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m2]\n  buffer_load_dwordx2 %[d2], %[o2], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m3]\n  buffer_load_dwordx2 %[d3], %[o3], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m4]\n  buffer_load_dwordx2 %[d4], %[o4], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m5]\n  buffer_load_dwordx2 %[d5], %[o5], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m6]\n  buffer_load_dwordx2 %[d6], %[o6], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m7]\n  buffer_load_dwordx2 %[d7], %[o7], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m8]\n  buffer_load_dwordx2 %[d8], %[o8], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m9]\n  buffer_load_dwordx2 %[d9], %[o9], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m10]\n buffer_load_dwordx2 %[d10], %[o10], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m11]\n buffer_load_dwordx2 %[d11], %[o11], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m12]\n buffer_load_dwordx2 %[d12], %[o12], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m13]\n buffer_load_dwordx2 %[d13], %[o13], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m14]\n buffer_load_dwordx2 %[d14], %[o14], %[rs], 0 offen\n"
      "s_and_b64 exec, %[sv], %[m15]\n buffer_load_dwordx2 %[d15], %[o15], %[rs], 0 offen\n"
      "s_mov_b64 exec, %[sv]\n"
      "s_waitcnt vmcnt(0)\n"
      : [d0] "+v"(v[0]), [d1] "+v"(v[1]), [d2] "+v"(v[2]), [d3] "+v"(v[3]),
        [d4] "+v"(v[4]), [d5] "+v"(v[5]), [d6] "+v"(v[6]), [d7] "+v"(v[7]),
        [d8] "+v"(v[8]), [d9] "+v"(v[9]), [d10] "+v"(v[10]), [d11] "+v"(v[11]),
        [d12] "+v"(v[12]), [d13] "+v"(v[13]), [d14] "+v"(v[14]), [d15] "+v"(v[15]),
        [sv] "=&s"(sv)
      : [o0] "v"(qo[0]), [o1] "v"(qo[1]), [o2] "v"(qo[2]), [o3] "v"(qo[3]),
        [o4] "v"(qo[4]), [o5] "v"(qo[5]), [o6] "v"(qo[6]), [o7] "v"(qo[7]),
        [o8] "v"(qo[8]), [o9] "v"(qo[9]), [o10] "v"(qo[10]), [o11] "v"(qo[11]),
        [o12] "v"(qo[12]), [o13] "v"(qo[13]), [o14] "v"(qo[14]), [o15] "v"(qo[15]),
        [m0] "s"(gm[0]), [m1] "s"(gm[1]), [m2] "s"(gm[2]), [m3] "s"(gm[3]),
        [m4] "s"(gm[4]), [m5] "s"(gm[5]), [m6] "s"(gm[6]), [m7] "s"(gm[7]),
        [m8] "s"(gm[8]), [m9] "s"(gm[9]), [m10] "s"(gm[10]), [m11] "s"(gm[11]),
        [m12] "s"(gm[12]), [m13] "s"(gm[13]), [m14] "s"(gm[14]), [m15] "s"(gm[15]),
        [rs] "s"(xr)
      : "memory");
}

// NT: 2 = non-temporal piece stores.  SPLIT: dedicated L2 waves (A.l2w).  STAMPS: PR_STAMPS
// diagnostics.  The variants are separate instantiations so that the default one carries no
// register cost for the others.
// EXP: a bit mask of what the instantiation carries beyond the plain launch.  The A/B switches
// each live in an instantiation of their own (1 = PR_L2LATE=1, 2 = PR_L2LATE=2, 4 = PR_DBG=8192):
// together inside the default one they cost 12 VGPRs and pushed its hot loop into scratch spills
// (1.65 -> 1.99 ms per launch).  So do the features a single rank's plain launch never uses
// (8 = slice-wide task claims, 16 = early first-task fetch, 32 = the cut launch of the overlapped
// exchange): compiled into the default instantiation their wave-uniform state doubled its SGPR
// spills (25 -> 47 registers kept in VGPR lanes, read back inside the task loop) and cost the
// stream launch 6 % (1.67 -> 1.78 ms).  The default of the template parameter is "everything"
// for the older variants; the shipped lean kernel is instantiated with 0, 32 and 56.
constexpr int EXP_ALL = 8 | 16 | 32;
template <int NT, bool SPLIT, bool STAMPS, int NTC = 0, bool LEAN = false, int EXP = EXP_ALL>
__global__ __launch_bounds__(STREAM_BLOCK) void spmv_stream(StreamArgs A) {
  extern __shared__ __attribute__((aligned(16))) double hot[];
  const uint32_t j = blockIdx.x % NSLICE;
  const uint32_t wpb = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  // Roles (PR_L2W): with l2w > 0 the last l2w waves of every workgroup sweep the L2 group
  // (gathers through the XCD's L2) for the whole launch while the other LW waves run the LDS
  // phases: latency-bound gathers beside bandwidth-bound LDS tasks.  The LW waves then sync
  // with an LDS-counter barrier of their own (the L2 waves never wait).
  constexpr bool X_DYN = (EXP & 8) != 0, X_EARLY = (EXP & 16) != 0, X_PARTS = (EXP & 32) != 0;
  const bool onlyl2 = X_PARTS && A.part == 2u && A.ph_lo >= A.ph_hi;
  const bool split = SPLIT && A.l2w != 0u && A.nlds != 0u && !onlyl2;
  const uint32_t LW = split ? wpb - A.l2w : wpb;
  const bool l2role = split && wv >= LW;
  const uint32_t rw = l2role ? A.l2w : LW;  // waves per workgroup in this wave's role
  const uint32_t w = (blockIdx.x / NSLICE) * rw + (l2role ? wv - LW : wv);
  const uint32_t nw = (gridDim.x / NSLICE) * rw;
  // the barrier counter lives in the spare words after the LDS block's zero slot (the dynamic
  // LDS request is already the whole 160 KiB: no static __shared__ may be added)
  uint32_t& bar_cnt = *reinterpret_cast<uint32_t*>(hot + A.H + 1);
  // with split roles, a phase's LDS tasks are dealt to the slice's workgroups round-robin
  // (task u to workgroup u mod 32) and the workgroup's LDS waves claim its tasks from this
  // counter, so no wave idles at the phase barrier while a sibling still has a backlog
  // (two counters, one per phase parity: a wave that is done with phase gi may claim its first
  // tasks of phase gi + 1 -- and start fetching their columns -- before the phase barrier)
  uint32_t* tcnt = reinterpret_cast<uint32_t*>(hot + A.H + 2);
  // slice-wide claims: "this phase has no task left" flags, one per phase parity
  uint32_t* skipf = reinterpret_cast<uint32_t*>(hot + A.H + 3);
  const bool wgdyn = split && !l2role && A.wgdyn != 0u;
  const uint32_t qwg = blockIdx.x / NSLICE, nqwg = gridDim.x / NSLICE;
  uint32_t bar_gen = 0;
  if (split) {
    if (threadIdx.x == 0) {
      bar_cnt = 0;
      tcnt[0] = tcnt[1] = 0;
    }
    __syncthreads();
  }
  auto block_barrier = [&]() {
    if (!split) {
      __syncthreads();
      return;
    }
    // the LW LDS-role waves only: arrive on an LDS counter, spin until all LW arrived
    ++bar_gen;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(&bar_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&bar_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < bar_gen * LW)
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  const double* __restrict__ x = A.x_in;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(x), static_cast<short>(0),
                                        static_cast<int>(A.x_bytes), 0x00020000);
  const uint32_t* __restrict__ col = A.col;
  const uint16_t* __restrict__ col16 = A.col16;
  const uint16_t* __restrict__ bits = A.bits;
  const uint32_t* __restrict__ tpa = A.task_piece;
  double* __restrict__ part = A.partial;
  const uint32_t cm = A.colmask;
  const uint32_t ngs = A.nlds + 1;
  double* stg = hot + (A.nlds ? A.H + 8u : 0u) + (threadIdx.x >> 6) * STG;
  // software pipeline: the next task's stream words are in flight while this task gathers.
  // An LDS-group task is 16 x u16 per lane (two 16-byte loads), an L2 task 16 x u32 (four).
  u32x4 cn[4];
  uint32_t bnx = 0, tpn = 0;
  const uint32_t l2g = j * ngs + A.nlds;
  const uint32_t l2g0 = A.gtask[l2g];              // first task of the slice's L2 group
  // the part of it this launch sweeps (all of it unless the launch is one part of a cut launch)
  const uint32_t l2b = X_PARTS ? A.l2lo[j] : l2g0, l2e = X_PARTS ? A.l2hi[j] : A.gtask[l2g + 1];
  const uint64_t l2base = A.gbase[l2g];
  auto fetch = [&](uint32_t tt, bool lds_task, uint32_t gtb, uint64_t gbs) {
    // PR_DBG=2048 / 4096 (timing only, wrong sums): every LDS-group / L2-group task reads the
    // columns of one of its group's first 64 tasks (L2-resident), its own flags and piece base
    // -- the cost of the column stream's HBM latency (4096 also concentrates the L2 gathers)
    const bool fake = lds_task ? (A.dbg & 2048u) != 0u : (A.dbg & 4096u) != 0u;
    const uint32_t tc = fake ? (tt - gtb) % 64u : tt - gtb;
    const uint64_t o = gbs + static_cast<uint64_t>(tc) * TASK + lane * EPL;
    // groups are padded to whole tasks: these loads never leave the stream buffers
    if (lds_task) {
      const u32x4* cp = reinterpret_cast<const u32x4*>(col16 + o);
      if constexpr ((NTC & 1) != 0) {  // PR_NTC bits: non-temporal loads of 1 col16, 2 col, 4 flags
        cn[0] = __builtin_nontemporal_load(cp);
        cn[1] = __builtin_nontemporal_load(cp + 1);
      } else {
        cn[0] = cp[0];
        cn[1] = cp[1];
      }
    } else {
      const u32x4* cp = reinterpret_cast<const u32x4*>(col + o);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr ((NTC & 2) != 0) cn[q] = __builtin_nontemporal_load(cp + q);
        else cn[q] = cp[q];
      }
    }
    const uint64_t so = static_cast<uint64_t>(tt) * TASK + lane * EPL;
    if constexpr ((NTC & 4) != 0) bnx = __builtin_nontemporal_load(bits + so / EPL);
    else bnx = bits[so / EPL];
    tpn = tpa[tt];
  };
  // Phases: phase gi < nlds holds LDS block gi and sweeps that block's tasks interleaved
  // with 1/nlds of the L2 part's tasks (LDS-bound and L2-bound work side by side); with no
  // LDS blocks the single phase is the whole stream.
  const bool l2last = A.l2mode == 1u && A.nlds && !split;  // one final phase for every L2 task
  const uint32_t nph = (A.nlds && !onlyl2) ? A.nlds + ((l2last || split) ? 1u : 0u) : 1u;  // (stamp slots)
  const uint32_t g0 = l2role ? A.nlds : ((split && X_PARTS) ? A.ph_lo : 0u),
                 g1 = split ? (l2role ? A.nlds + 1u : (X_PARTS ? A.ph_hi : A.nlds)) : nph;
  for (uint32_t gi = g0; gi < g1; ++gi) {
    uint32_t tb = l2b, te = l2b, rb = l2b, re = l2e;  // LDS-block tasks, L2 share
    uint64_t lbase = 0;
    bool gdyn = false, lds_phase = false;
    uint32_t gslot = gi;  // counter of this phase's slice-wide claims
    if (onlyl2 || (gi == A.nlds && (l2last || l2role))) {
      // the L2 phase / role: no LDS block, the whole L2 group (segments swept in order); with
      // l2dyn its tasks go to the slice's L2 waves in claim order, front to back
      gdyn = X_DYN && l2role && A.l2dyn != 0u && A.gcnt != nullptr;
      gslot = A.part == 2u ? 65u : 64u;
    } else if (A.nlds) {
      lds_phase = true;
      tb = A.gtask[j * ngs + gi];
      te = A.gtask[j * ngs + gi + 1];
      lbase = A.gbase[j * ngs + gi];
      rb = l2b + static_cast<uint32_t>((static_cast<uint64_t>(l2e - l2b) * gi) / A.nlds);
      re = l2b + static_cast<uint32_t>((static_cast<uint64_t>(l2e - l2b) * (gi + 1)) / A.nlds);
      if (l2last || split) rb = re = l2b;
      // Late phases may deal their tasks slice-wide (PR_DYNTAIL): every LDS wave of the slice's
      // workgroups claims from one counter, so a workgroup that has fallen behind (1-3 of a
      // slice's 32 end 40-160 us after the others, different ones every launch) is left fewer
      // tasks, and none of a phase the others have already emptied -- then it skips the fill.
      gdyn = X_DYN && wgdyn && A.gcnt != nullptr && gi >= A.dyn0;
    }
    // entering an LDS phase: barrier (every wave is done with the previous block), fill, reset
    // of the other parity's task counter, barrier
    auto enter_phase = [&]() {
      const uint32_t hb = A.hot_base[j] + gi * A.H;
      if (gdyn && threadIdx.x == 0)
        skipf[gi & 1u] = __hip_atomic_load(&A.gcnt[j * GCNT + gi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= te - tb ? 1u : 0u;
      block_barrier();  // every wave is done with the previous block (and sees the flag)
      const bool skip = gdyn && skipf[gi & 1u] != 0u;
      if (skip) te = tb;
      if (te > tb) {
        // LDS-DMA fill: one global_load_lds_dwordx4 moves 1 KiB (128 entries) per wave
        // instruction straight into LDS (no registers); H is even and hb 16-byte aligned
        const uint32_t nfill = (A.H + 127u) / 128u;
        for (uint32_t q = wv; q < nfill; q += LW) {
          const uint32_t e0 = q * 128u + 2u * static_cast<uint32_t>(lane);
          if (e0 < A.H) __builtin_amdgcn_global_load_lds(x + hb + e0, hot + q * 128u, 16, 0, 0);
        }
        // (vmcnt counts in order: the wait also covers column words fetched ahead of the fill)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) hot[A.H] = 0.0;  // the padding column
      }
      if (threadIdx.x == 0) tcnt[(gi + 1u) & 1u] = 0;  // (wave 0 is an LDS wave)
      if (!skip) block_barrier();
    };
    // PR_EARLY: with workgroup-local claims a wave claims its first tasks of the phase and
    // fetches the first one's column words before it enters the phase, so that fetch's HBM
    // latency passes during the barrier and the fill instead of after them
    const bool early = X_EARLY && lds_phase && wgdyn && !gdyn && A.early != 0u;
    if (lds_phase && !early) enter_phase();
    uint64_t* stp = STAMPS ? A.stamps + (static_cast<uint64_t>(blockIdx.x) * nph + gi) * 17u : nullptr;
    const uint32_t nL = te - tb, nR = re - rb, nm = min(nL, nR);
    // virtual index u -> task: alternate LDS / L2 tasks while both last, then the rest
    auto is_lds = [&](uint32_t u) -> bool {
      if (u < 2 * nm) return (u & 1u) == 0u;
      return nL > nR;
    };
    auto task_of = [&](uint32_t u) -> uint32_t {
      if (u < 2 * nm) return (u & 1u) ? rb + (u >> 1) : tb + (u >> 1);
      return nL > nR ? tb + (u - nm) : rb + (u - nm);
    };
    auto fetch_u = [&](uint32_t u) {
      const bool lt = is_lds(u);
      fetch(task_of(u), lt, lt ? tb : l2g0, lt ? lbase : l2base);
    };
    const uint32_t nu = nL + nR;
    // slice-wide claims take A.dyng consecutive tasks per atomic (one address serves the whole
    // slice: single-task claims saturate it)
    uint32_t gcur = 0, gend = 0;
    auto claim = [&]() -> uint32_t {
      if (gdyn && gcur < gend) return gcur++;
      uint32_t m = 0;
      if (lane == 0) m = gdyn ? atomicAdd(&A.gcnt[j * GCNT + gslot], A.dyng) : atomicAdd(&tcnt[gi & 1u], 1u);
      m = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(m)));
      if (!gdyn) return qwg + nqwg * m;
      gcur = m + 1u;
      gend = m + A.dyng;
      return m;
    };
    const bool dyn = (wgdyn && gi < A.nlds) || gdyn;
    uint32_t u = dyn ? claim() : w;
    uint32_t un = dyn ? (u < nu ? claim() : nu) : w + nw;
    if (u < nu) fetch_u(u);
    if (early) enter_phase();
    if (stp && threadIdx.x == 0) stp[0] = __builtin_amdgcn_s_memrealtime();
    while (u < nu) {
      const bool lds_task = is_lds(u);
      u32x4 cv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) cv[q] = cn[q];
      uint32_t b = bnx;
      const uint32_t tp0 = tpn;
      if (A.dbg & 4u) b = 0;
      if (lane == 0) b |= 1u;  // a task always starts a piece
      // next task's stream words first: they stay in flight while this task gathers
      const bool late = (EXP & 1) != 0 && l2role && A.l2late == 1u;
      if (un < nu && !late) fetch_u(un);
      const uint32_t unn = dyn ? (un < nu ? claim() : nu) : un + nw;
      double v[EPL];
      if (lds_task) {
        // every source of an LDS-group task is inside the block (padding reads the zero slot)
        if (A.dbg & 8u) {  // timing: no LDS gathers
#pragma unroll
          for (int k = 0; k < EPL; ++k)
            v[k] = __longlong_as_double(static_cast<long long>(cv[k >> 3][(k >> 1) & 3] & 0x3FFFu));
        } else if constexpr (LEAN) {
          // one SDWA shift per address (the block starts at LDS byte 0: no static LDS here)
          const char* hb = reinterpret_cast<const char*>(hot);
#pragma unroll
          for (int k = 0; k < EPL; ++k) {
            const uint32_t wd = cv[k >> 3][(k >> 1) & 3];
            v[k] = *reinterpret_cast<const double*>(hb + ((k & 1) ? lds_off_hi(wd) : lds_off_lo(wd)));
          }
        } else {
#pragma unroll
          for (int k = 0; k < EPL; ++k) {
            const uint32_t wd = cv[k >> 3][(k >> 1) & 3];
            v[k] = hot[(k & 1) ? (wd >> 16) : (wd & 0xFFFFu)];
          }
        }
      } else {
        // sixteen buffer gathers issued back to back; PAD_COL lanes fall outside the buffer
        // range and read 0
        uint32_t qo[EPL];
        uint64_t gm[EPL];
#pragma unroll
        for (int k = 0; k < EPL; ++k) {
          v[k] = 0.0;
          qo[k] = (cv[k >> 2][k & 3] & cm) * 8u;
          gm[k] = ~0ull;
        }
        if (A.dbg & 2u) {
#pragma unroll
          for (int k = 0; k < EPL; ++k) v[k] = static_cast<double>(qo[k] & 0xFFFF);
        } else {
          gather16(v, qo, gm, xr);
        }
        if (late && un < nu) fetch_u(un);
      }
    // exclusive prefix (over lanes) of the piece starts -> first piece index of this lane
    const int cnt = __popc(b);
    const int C = LEAN ? wave_incl_scan_lean(cnt) : wave_incl_scan(cnt, lane);
    const uint32_t first = static_cast<uint32_t>(C - cnt);  // task-relative index of the lane's first start
    const uint32_t total = static_cast<uint32_t>(__builtin_amdgcn_readlane(C, 63));  // pieces of the task
    // PR_DBG=8192 (timing only, wrong sums): a task made almost only of single-edge pieces
    // stores its sixteen gathered values per lane as if lane l's edge k were piece 64 k + l --
    // the store pattern of a column-major all-singles task: no sums, no scan, no staging
    const bool fastd = (EXP & 4) != 0 && (A.dbg & 8192u) != 0u && total >= 768u;
    if (fastd) {
#pragma unroll
      for (int k = 0; k < EPL; ++k)
        if (64u * k + static_cast<uint32_t>(lane) < total)
          __builtin_nontemporal_store(v[k], part + tp0 + 64u * k + lane);
    } else {
    // one pass over the lane's edges: pv[k] = the running sum just before edge k (for a start
    // bit k that is the piece closing before k; for the lane's first start it is the head,
    // the edges before it), run = the open piece at the lane's end.  Same adds, same order as
    // a plain left-to-right sum per piece.
    double run = 0.0;
    double pv[EPL];
    double S;
    if constexpr (LEAN) {
      // run = start ? v : run + v as fma(run, !start, v): exactly v, or the correctly rounded
      // run + v (three ops per edge: bit extract, convert, fma)
      const uint32_t nb = ~b;
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        pv[k] = run;
        run = __builtin_fma(run, static_cast<double>((nb >> k) & 1u), v[k]);
      }
      // the segmented scan only matters when some lane holds no start (a piece crossing a
      // whole lane); otherwise every lane's inclusive value is its own open piece
      if (__builtin_amdgcn_ballot_w64(b == 0u) == 0ull) S = run;
      else S = wave_seg_scan_lean(run, b != 0u ? 1 : 0);
    } else {
#pragma unroll
      for (int k = 0; k < EPL; ++k) {
        pv[k] = run;
        const double t = run + v[k];
        run = ((b >> k) & 1u) ? v[k] : t;
      }
      // segmented inclusive scan of the open piece over lanes (flag: lane holds a start)
      S = wave_seg_scan(run, b != 0u ? 1 : 0, lane);
    }
    const double carry = dpp_d<DPP_WAVE_SHR1>(S);
    const uint32_t bn = static_cast<uint32_t>(dpp_i<DPP_WAVE_SHL1>(static_cast<int>(b)));
    const bool closes = lane == 63 || (bn & 1u) != 0u;  // next edge starts a piece
    // Pieces go to the wave's LDS staging window (STG pieces at a time) and leave it as
    // contiguous 512-byte stores: one L2 request per line instead of one per piece.  Start
    // bit k >= 1 closes the piece with index first - 1 + (starts before k, bit 0 included).
    for (uint32_t w0 = 0; w0 < total; w0 += STG) {
      const uint32_t wn = min(total - w0, static_cast<uint32_t>(STG));
      if (first + cnt > w0 && first < w0 + wn + 1u) {
        // window slot of the next closing piece: piece first - 1 closes at the lane's first
        // start k >= 1 (when edge 0 starts a piece, that earlier piece closed in lane - 1)
        uint32_t idx = first - 1u + (b & 1u) - w0;
#pragma unroll
        for (int k = 1; k < EPL; ++k) {
          const uint32_t bit = (b >> k) & 1u;
          if (bit && idx < wn) stg[idx] = pv[k];
          idx += bit;
        }
        // the head piece (closing at the lane's first start k0 > 0) also holds the pieces
        // open in earlier lanes: carry + head, one add, fixed up in place (same lane wrote it)
        const uint32_t hs = first - 1u - w0;
        if (b != 0u && !(b & 1u) && hs < wn) stg[hs] = carry + stg[hs];
        if (b == 0u) {
          if (closes && first - 1u - w0 < wn) stg[first - 1u - w0] = S;  // inside a longer piece
        } else if (closes && static_cast<uint32_t>(C) - 1u - w0 < wn) {
          stg[static_cast<uint32_t>(C) - 1u - w0] = run;  // the lane's last piece
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (LEAN && !(A.dbg & 1u)) {
        // two pieces per lane per store instruction (16 B at 8-B alignment: the device runs
        // in unaligned mode), half the store instructions (+0.8 %, profiles/r02/vmem); a
        // trailing odd piece goes alone
        typedef double d2v __attribute__((ext_vector_type(2)));
#pragma unroll 1
        for (uint32_t i = 2u * static_cast<uint32_t>(lane); i < wn; i += 128u) {
          if (i + 1u < wn) {
            const d2v pr = *reinterpret_cast<const d2v*>(stg + i);
            if constexpr (NT >= 2) __builtin_nontemporal_store(pr, reinterpret_cast<d2v*>(part + tp0 + w0 + i));
            else *reinterpret_cast<d2v*>(part + tp0 + w0 + i) = pr;
          } else {
            if constexpr (NT >= 2) __builtin_nontemporal_store(stg[i], part + tp0 + w0 + i);
            else part[tp0 + w0 + i] = stg[i];
          }
        }
      } else if (!(A.dbg & 1u))
        for (uint32_t i = lane; i < wn; i += 64) {
          if constexpr (NT >= 2) __builtin_nontemporal_store(stg[i], part + tp0 + w0 + i);
          else part[tp0 + w0 + i] = stg[i];
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    }  // !fastd
      // PR_L2LATE=2 (A/B): the L2-role waves wait for their piece stores right here; the cost
      // bounds what the gathers' in-order wait can lose to stores still in flight
      if ((EXP & 2) != 0 && l2role && A.l2late == 2u) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u = un;
      un = unn;
    }
    if (stp && lane == 0) stp[1 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---- self-test of the row launch's summation order ---------------------------------------
// The row launch adds pieces into LDS accumulators with one ds_add_f64 per lane per line; lanes
// of one instruction that hit the same row collide, and the sums are only reproducible if the
// hardware applies such same-address adds in an order that depends on nothing but the lanes
// and addresses.  k_lds_order issues exactly that instruction form -- 64 lanes, one atomicAdd,
// addresses drawn from M rows, values whose exponents differ so that every order rounds
// differently -- from every wave of a large grid and stores the accumulators' bits; the host
// compares all copies (dev_selftest_lds_order).
__device__ __host__ __forceinline__ uint64_t st_mix(uint64_t c, uint64_t l) {
  uint64_t x = (c + 1) * 0x9E3779B97F4A7C15ull + l * 0xD1B54A32D192ED03ull;
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}
constexpr int ST_ROWS = 8;  // accumulator rows of a case (M = 1 + case % 8 of them are hit)
__device__ __host__ __forceinline__ void st_case(uint32_t c, uint32_t lane, uint32_t* row, double* val) {
  const uint64_t h = st_mix(c, lane);
  const uint32_t M = 1u + c % ST_ROWS;
  *row = static_cast<uint32_t>(h % M);
  // 1.m x 2^-e, e in [0, 40): sums of such values round differently in different orders
  const uint64_t mant = (h >> 12) & ((1ull << 52) - 1);
  const uint64_t e = 1023ull - (h >> 3) % 40ull;
  const uint64_t bits = (e << 52) | mant;
#ifdef __HIP_DEVICE_COMPILE__
  *val = __longlong_as_double(static_cast<long long>(bits));
#else
  memcpy(val, &bits, 8);
#endif
}
__global__ __launch_bounds__(BLOCK) void k_lds_order(uint32_t c, uint64_t* out) {
  __shared__ double acc[BLOCK / 64][ST_ROWS];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < ST_ROWS) acc[wv][lane] = 0.0;
  __syncthreads();
  uint32_t row;
  double val;
  st_case(c, lane, &row, &val);
  atomicAdd(&acc[wv][row], val);  // one ds_add_f64 over the 64 lanes, as spmv_rows issues them
  __syncthreads();
  if (lane < ST_ROWS)
    out[(static_cast<uint64_t>(blockIdx.x) * (BLOCK / 64) + wv) * ST_ROWS + lane] =
        static_cast<uint64_t>(__double_as_longlong(acc[wv][lane]));
}

// Sum the NSHARD shards into one record and clear them for the next round (one 256-thread
// workgroup; `out`, when given, is an LDS copy of the record for a fused finalize).
__device__ __forceinline__ void reduce_shards_body(uint64_t* shards, uint64_t* rec, uint64_t (*part)[REC_WORDS],
                                                   uint64_t* out, uint32_t* gcnt) {
  // (the stream launch's slice-wide task counters start the next round at zero)
  if (gcnt)
    for (int i = threadIdx.x; i < NSLICE * static_cast<int>(GCNT); i += BLOCK) gcnt[i] = 0;
  const int w = threadIdx.x & 31, g = threadIdx.x >> 5;
  uint64_t s = 0;
  for (int i = g * (NSHARD / 8); i < (g + 1) * (NSHARD / 8); ++i) {
    uint64_t* p = &shards[i * REC_WORDS + w];
    s += *p;
    *p = 0;
  }
  part[g][w] = s;
  __syncthreads();
  if (threadIdx.x < REC_WORDS) {
    uint64_t t = 0;
    for (int k = 0; k < 8; ++k) t += part[k][threadIdx.x];
    rec[threadIdx.x] = t;
    if (out) out[threadIdx.x] = t;
  }
}

__global__ __launch_bounds__(BLOCK) void reduce_shards(uint64_t* shards, uint64_t* rec, uint32_t* gcnt) {
  __shared__ uint64_t part[8][REC_WORDS];
  reduce_shards_body(shards, rec, part, nullptr, gcnt);
}

// Combine the p rank records (integer sums: order-free, exact) -> next round's addthis.
// Run by one full wave: lanes 0 / 1 / 2 sum and round the dangling mass / residual / rank sum
// side by side (the three roundings were serial on one thread before).
__device__ __forceinline__ void finalize_wave(const uint64_t* rec_all, int p, int t, uint64_t n_tot,
                                              uint32_t extra_pages, double r0, int tracked, IterState* st) {
  const int lane = threadIdx.x & 63;
  double v = 0.0;
  if (lane < (tracked ? 3 : 1)) {
    const int off = lane == 0 ? REC_DSUM : (lane == 1 ? REC_RESID : REC_RSUM);
    uint64_t acc[SA_LIMBS];
#pragma unroll
    for (int i = 0; i < SA_LIMBS; ++i) acc[i] = 0;
    for (int r = 0; r < p; ++r) {
      const uint64_t* q = rec_all + r * REC_WORDS + off;
#pragma unroll
      for (int i = 0; i < SA_LIMBS; ++i) acc[i] += q[i];
    }
    if (lane == 1) {
      // round 1: the pages that are not rows drop from r0 to undefined, |dr| = r0 each
      uint32_t c0, c1, c2, c3;
      const int li = sa_chunks(r0, extra_pages, c0, c1, c2, c3);
      if (li >= 0) {
        const uint32_t cs[4] = {c0, c1, c2, c3};
#pragma unroll
        for (int i = 0; i < SA_LIMBS; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (i == li + q) acc[i] += cs[q];
      }
    }
    v = sa_to_double_dev(acc);
  }
  const double a = __shfl(v, 0), ra = __shfl(v, 1), rs = __shfl(v, 2);
  if (lane != 0) return;
  uint64_t dcnt = 0;
  for (int r = 0; r < p; ++r) dcnt += rec_all[r * REC_WORDS + REC_DCNT];
  // :135  accum.setValue(sum / totalVertices)
  st->a = a / static_cast<double>(n_tot);
  st->dcnt = dcnt;
  if (dcnt == 0 && st->err_iter == 0) st->err_iter = t + 1;
  if (tracked) {
    st->resid_abs = ra;
    st->rank_sum = rs;
    st->resid = rs > 0.0 ? ra / rs : 0.0;
  }
  st->iter = t;
}

__global__ __launch_bounds__(64) void finalize_round(const uint64_t* rec_all, int p, int t, uint64_t n_tot,
                                                     uint32_t extra_pages, double r0, int tracked, IterState* st) {
  finalize_wave(rec_all, p, t, n_tot, extra_pages, r0, tracked, st);
}

// p = 1: the record reduction and the finalize in one launch (one launch gap less per round).
__global__ __launch_bounds__(BLOCK) void reduce_finalize(uint64_t* shards, uint64_t* rec, int t, uint64_t n_tot,
                                                         uint32_t extra_pages, double r0, int tracked,
                                                         IterState* st, uint32_t* gcnt) {
  __shared__ uint64_t part[8][REC_WORDS];
  __shared__ uint64_t tot[REC_WORDS];
  reduce_shards_body(shards, rec, part, tot, gcnt);
  __syncthreads();
  if (threadIdx.x < 64) finalize_wave(tot, 1, t, n_tot, extra_pages, r0, tracked, st);
}

// Large launches (edge counts reach 2^32 at R-MAT scale 28) loop over blocks: every thread of
// a block runs the same iterations, so block- and wave-level operations in the body stay
// uniform, and the grid stays far below the 2^32 work-item limit.
#define PRMI_BLOCK_LOOP(n) \
  for (uint64_t blk_ = blockIdx.x; blk_ * blockDim.x < (n); blk_ += gridDim.x)

// =======================================================================================
// graph build (K1): keys -> sort -> unique -> degrees -> vertex order -> local CSR
// =======================================================================================
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
  }
}

// Graph500 R-MAT quadrant thresholds floor(p * 2^32) of the cumulative a, a+b, a+b+c.
constexpr uint32_t kRmatA = 2448131358u, kRmatAB = 3264175144u, kRmatABC = 4080218931u;

__global__ void k_rmat_keys(uint64_t seed, int scale, uint64_t m, uint64_t* keys) {
  PRMI_BLOCK_LOOP(m) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e >= m) continue;
    uint32_t s = 0, d = 0, w[4] = {0, 0, 0, 0};
    for (int lv = 0; lv < scale; ++lv) {
      if ((lv & 3) == 0) {
        w[0] = static_cast<uint32_t>(e);
        w[1] = static_cast<uint32_t>(e >> 32);
        w[2] = static_cast<uint32_t>(lv >> 2);
        w[3] = 0x524D4154u;  // "RMAT"
        philox4x32_10(w, static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
      }
      const uint32_t u = w[lv & 3];
      const uint32_t sb = u >= kRmatAB;
      const uint32_t db = (u >= kRmatA && u < kRmatAB) || u >= kRmatABC;
      s = (s << 1) | sb;
      d = (d << 1) | db;
    }
    keys[e] = (static_cast<uint64_t>(d) << scale) | s;
  }
}

__global__ void k_make_keys(const uint32_t* src, const uint32_t* dst, uint64_t m, int nb,
                            uint64_t* keys) {
  PRMI_BLOCK_LOOP(m) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e < m) keys[e] = (static_cast<uint64_t>(dst[e]) << nb) | src[e];
  }
}

// Degrees and the edge-set digest of the distinct edges (sorted by dst, then src).
// out-degree (PageRank.java:103-108 urlCount): one integer atomic per edge on its source.
// in-degree: run lengths of dst in the sorted keys (no atomics): the first edge of a run
// records its position, the last one its end; k_indeg_from_runs subtracts.
// digest {sum, xor} of mix64(src<<32|dst): per-block partials into DIGEST_SHARDS shards
// (single-address atomics from every block serialised this kernel at scale 26).
constexpr int DIGEST_SHARDS = 4096;
__global__ void k_degrees(const uint64_t* uk, uint64_t nnz, int nb, uint32_t* outdeg,
                          uint64_t* run_lo, uint64_t* run_hi, unsigned long long* digest) {
  __shared__ unsigned long long ssum[BLOCK / 64], sxor[BLOCK / 64];
  PRMI_BLOCK_LOOP(nnz) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    uint64_t h = 0;
    if (e < nnz) {
      const uint64_t k = uk[e];
      const uint32_t d = static_cast<uint32_t>(k >> nb);
      const uint32_t s = static_cast<uint32_t>(k & ((1ull << nb) - 1));
      atomicAdd(&outdeg[s], 1u);
      if (e == 0 || static_cast<uint32_t>(uk[e - 1] >> nb) != d) run_lo[d] = e;
      if (e + 1 == nnz || static_cast<uint32_t>(uk[e + 1] >> nb) != d) run_hi[d] = e + 1;
      h = mix64((static_cast<uint64_t>(s) << 32) | d);
    }
    uint64_t hs = h, hx = h;
  #pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      hs += __shfl_xor(hs, m);
      hx ^= __shfl_xor(hx, m);
    }
    if ((threadIdx.x & 63) == 0) {
      ssum[threadIdx.x >> 6] = hs;
      sxor[threadIdx.x >> 6] = hx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long a = 0, x = 0;
      for (int i = 0; i < BLOCK / 64; ++i) {
        a += ssum[i];
        x ^= sxor[i];
      }
      const uint64_t sh = 2 * (blk_ % DIGEST_SHARDS);
      atomicAdd(&digest[sh], a);
      atomicXor(&digest[sh + 1], x);
    }
    __syncthreads();  // the next iteration reuses the shared partials
  }
}

__global__ void k_indeg_from_runs(const uint64_t* run_lo, const uint64_t* run_hi, uint32_t n,
                                  uint32_t* indeg) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) indeg[v] = static_cast<uint32_t>(run_hi[v] - run_lo[v]);
}

// dangling weight (PageRank.java:56) + class key for the vertex order
constexpr int W_SHARDS = 64;
__global__ void k_vertex_keys(const uint32_t* outdeg, const uint32_t* indeg, const uint32_t* mapw,
                              uint32_t n, uint32_t* dang_w, uint64_t* vkey, uint32_t* vid,
                              unsigned long long* sums /* [W_SHARDS] shards of W0 */) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t w = 0;
  if (v < n) {
    const uint32_t o = outdeg[v], i = indeg[v];
    w = o == 0 ? (mapw ? mapw[v] : 1u) : 0u;
    dang_w[v] = w;
    const uint64_t cls = i ? (o ? 0 : 1) : (o ? 2 : 3);
    vkey[v] = (cls << 32) | (0xFFFFFFFFu - i);
    vid[v] = v;
  }
  uint64_t s = w;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  // one shard per (block mod W_SHARDS): no single-address atomic from every wave
  if ((threadIdx.x & 63) == 0 && s)
    atomicAdd(&sums[blockIdx.x % W_SHARDS], static_cast<unsigned long long>(s));
}

__global__ void k_class_count(const uint64_t* vkey_sorted, uint32_t n, unsigned* cnt) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const uint32_t c = static_cast<uint32_t>(vkey_sorted[v] >> 32);
  const uint32_t cp = v ? static_cast<uint32_t>(vkey_sorted[v - 1] >> 32) : 0xFFFFFFFFu;
  // class boundaries: cnt[c] = first internal index of class c (set once per class)
  if (c != cp) cnt[c] = v;
}

__global__ void k_inverse(const uint32_t* perm, uint32_t n, uint32_t* inv) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) inv[perm[k]] = k;
}

// rows dealt to ranks in chunks of CHUNK internal ids; slices by 128-byte x line
struct Layout {
  uint32_t p, rank, nA, R, nC, maxA;
  uint32_t sm;        // slice-major x (p divides 8): every slice is one contiguous region
  uint32_t SL, SLC;   // entries per slice region: class-A part / class-C part
  uint32_t snake;     // snake chunk -> slice order (chunk_slice; single rank only)
};
__device__ __host__ __forceinline__ uint32_t owner_of(const Layout& L, uint32_t k) {
  return (k / CHUNK) % L.p;
}
__device__ __host__ __forceinline__ uint32_t local_of(const Layout& L, uint32_t k) {
  return ((k / CHUNK) / L.p) * CHUNK + (k % CHUNK);
}
__device__ __host__ __forceinline__ uint32_t row_of(const Layout& L, uint32_t l) {
  return ((l / CHUNK) * L.p + L.rank) * CHUNK + (l % CHUNK);
}
// x position of column k.  Slice-major: A entries sit in the region of their owner rank,
// inside it in the sub-region of their slice (chunk c = k>>4 has slice c&7 and, as p
// divides 8, owner c%p = (c&7)%p), chunks of a slice in order -- each XCD's slice is one
// contiguous, hotness-ordered address range (all L2 sets and channels in use).
__device__ __host__ __forceinline__ uint32_t xpos(const Layout& L, uint32_t k) {
  if (k < L.nA) {
    if (!L.sm) return owner_of(L, k) * L.maxA + local_of(L, k);
    const uint32_t c = k / CHUNK, sl = chunk_slice(c, L.snake);
    return (sl % L.p) * L.maxA + (sl / L.p) * L.SL + (c / NSLICE) * CHUNK + (k % CHUNK);
  }
  const uint32_t kc = k - L.R;
  if (!L.sm) return L.p * L.maxA + kc;
  const uint32_t c = kc / CHUNK;
  return L.p * L.maxA + chunk_slice(c, L.snake) * L.SLC + (c / NSLICE) * CHUNK + (kc % CHUNK);
}
// slice of a column = its 128-byte chunk index mod 8 (independent of the rank count)
__device__ __forceinline__ uint32_t slice_of(const Layout& L, uint32_t k) {
  return chunk_slice((k < L.nA ? k : k - L.R) / CHUNK, L.snake);
}

// x of every column from r^0 (r0 on all sources) or, for a seed, from ranks by original id
__global__ void k_x_init(const uint32_t* perm, const uint32_t* outdeg, uint32_t n, Layout L,
                         double r0, const double* ranks, double* x_init) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const bool col = k < L.nA || (k >= L.R && k < L.R + L.nC);
  const uint32_t v = perm[k];
  if (col) x_init[xpos(L, k)] = (ranks ? ranks[v] : r0) / static_cast<double>(outdeg[v]);
}

// seed ranks of this rank's rows
__global__ void k_r_seed(const uint32_t* perm, const double* ranks, uint32_t lrows, Layout L,
                         double* r_seed) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l < lrows) r_seed[l] = ranks[perm[row_of(L, l)]];
}

// exact dangling mass + defined-entry count of a seed (PageRank.java:125-134) -> rec
__global__ __launch_bounds__(BLOCK) void k_seed_dangling(const double* ranks, const uint32_t* dang_w,
                                                         uint32_t n, uint64_t* rec) {
  __shared__ uint64_t lds[BLOCK / 64][REC_WORDS];
  for (int i = threadIdx.x; i < (BLOCK / 64) * REC_WORDS; i += BLOCK) (&lds[0][0])[i] = 0;
  __syncthreads();
  const uint32_t v = blockIdx.x * BLOCK + threadIdx.x;
  const double r = v < n ? ranks[v] : 0.0;
  const uint32_t w = v < n ? dang_w[v] : 0u;
  uint64_t* lw = lds[threadIdx.x >> 6];
  uint32_t c0, c1, c2, c3;
  const int li = sa_chunks(r, w, c0, c1, c2, c3);
  wave_accum_sa(lw, REC_DSUM, li, c0, c1, c2, c3);
  const uint64_t cnt = wave_sum_u64((r > 0.0) ? w : 0u);
  if ((threadIdx.x & 63) == 0) lw[REC_DCNT] += cnt;
  __syncthreads();
  if (threadIdx.x < REC_WORDS) {
    uint64_t t = 0;
    for (int q = 0; q < BLOCK / 64; ++q) t += lds[q][threadIdx.x];
    if (t) atomicAdd(reinterpret_cast<unsigned long long*>(&rec[threadIdx.x]),
                     static_cast<unsigned long long>(t));
  }
}

// ---- slice streams -----------------------------------------------------------------------
// q-space of a slice: class-A columns [0, SLq) in hotness order, then class-C columns.
// Segments of q: nlds LDS blocks of H entries, the L2-hot range of QL entries, then cold
// ranges of S entries.  Stream groups per slice: one per LDS block + one for everything
// after it; every group starts on a task boundary (padding: col = PAD, gathers read 0).
constexpr uint32_t PAD_COL = 0xFFFFFFFFu;
static_assert(PAD_COL == 0xFFFFFFFFu, "the build pads col with memset(0xFF)");
struct StreamGeo {
  uint32_t SLq;       // q-space length of the class-A part of one slice
  uint32_t nlds, H;   // LDS blocks per slice and their length
  uint32_t QL, S;     // L2-hot range length, cold segment length (x entries)
  int qb, rb, sgb;    // key fields: q within segment | local row | segment | slice
};
__device__ __forceinline__ void col_slice_q(const Layout& L, const StreamGeo& G, uint32_t k,
                                            uint32_t& sl, uint32_t& q) {
  if (k < L.nA) {
    const uint32_t c = k / CHUNK;
    sl = chunk_slice(c, L.snake);
    q = (c / NSLICE) * CHUNK + k % CHUNK;
  } else {
    const uint32_t kc = k - L.R, c = kc / CHUNK;
    sl = chunk_slice(c, L.snake);
    q = G.SLq + (c / NSLICE) * CHUNK + kc % CHUNK;
  }
}
__device__ __forceinline__ uint32_t col_of_slice_q(const Layout& L, const StreamGeo& G,
                                                   uint32_t sl, uint32_t q) {
  if (q < G.SLq) return slice_chunk(q / CHUNK, sl, L.snake) * CHUNK + q % CHUNK;
  const uint32_t qc = q - G.SLq;
  return L.R + slice_chunk(qc / CHUNK, sl, L.snake) * CHUNK + qc % CHUNK;
}
__device__ __forceinline__ void seg_of_q(const StreamGeo& G, uint32_t q, uint32_t& seg,
                                         uint32_t& qin) {
  const uint32_t ql = G.nlds * G.H;
  if (q < ql) {
    seg = q / G.H;
    qin = q % G.H;
  } else if (q - ql < G.QL) {
    seg = G.nlds;
    qin = q - ql;
  } else {
    seg = G.nlds + 1 + (q - ql - G.QL) / G.S;
    qin = (q - ql - G.QL) % G.S;
  }
}
__device__ __forceinline__ uint32_t q_of_seg(const StreamGeo& G, uint32_t seg, uint32_t qin) {
  if (seg < G.nlds) return seg * G.H + qin;
  if (seg == G.nlds) return G.nlds * G.H + qin;
  return G.nlds * G.H + G.QL + (seg - G.nlds - 1) * G.S + qin;
}
__device__ __forceinline__ uint32_t group_of_key(const StreamGeo& G, uint64_t k) {
  const uint32_t sl = static_cast<uint32_t>(k >> (G.sgb + G.rb + G.qb));
  const uint32_t seg = static_cast<uint32_t>(k >> (G.rb + G.qb)) & ((1u << G.sgb) - 1u);
  return sl * (G.nlds + 1) + min(seg, G.nlds);
}
// internal column id of an x position (inverse of xpos)
__device__ __forceinline__ uint32_t col_of_xpos(const Layout& L, uint32_t x) {
  const uint32_t PA = L.p * L.maxA;
  if (x < PA) {
    const uint32_t r = x / L.maxA, y = x % L.maxA;
    if (!L.sm) return ((y / CHUNK) * L.p + r) * CHUNK + y % CHUNK;
    const uint32_t sl = (y / L.SL) * L.p + r, rem = y % L.SL;
    return slice_chunk(rem / CHUNK, sl, L.snake) * CHUNK + rem % CHUNK;
  }
  const uint32_t qc = x - PA;
  if (!L.sm) return L.R + qc;
  const uint32_t sl = qc / L.SLC, rem = qc % L.SLC;
  return L.R + slice_chunk(rem / CHUNK, sl, L.snake) * CHUNK + rem % CHUNK;
}

// relabel unique edges to stream keys (slice, segment, local row, q within segment); with p > 1
// the edges of other ranks' rows get DROP_KEY and a rocprim::select keeps this rank's
constexpr uint64_t DROP_KEY = ~0ull;
struct NotDropped {
  __device__ __host__ bool operator()(uint64_t k) const { return k != DROP_KEY; }
};
__global__ void k_stream_keys(const uint64_t* uk, uint64_t nnz, int nb, const uint32_t* inv,
                              Layout L, StreamGeo G, uint64_t* out, const uint32_t* indeg,
                              uint32_t dropdeg, uint32_t keepdeg) {
  PRMI_BLOCK_LOOP(nnz) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e >= nnz) continue;
    const uint64_t k = uk[e];
    // PR_DROPDEG (timing only, wrong ranks): rows below this in-degree leave the streams
    // (PR_KEEPDEG: rows at or above that in-degree leave instead)
    if (dropdeg || keepdeg) {
      const uint32_t di = indeg[static_cast<uint32_t>(k >> nb)];
      if (di < dropdeg || (keepdeg && di >= keepdeg)) {
        out[e] = DROP_KEY;
        continue;
      }
    }
    const uint32_t kd = inv[static_cast<uint32_t>(k >> nb)];
    const uint32_t ks = inv[static_cast<uint32_t>(k & ((1ull << nb) - 1))];
    uint32_t sl, q, seg, qin;
    col_slice_q(L, G, ks, sl, q);
    seg_of_q(G, q, seg, qin);
    const uint64_t key = (static_cast<uint64_t>(sl) << (G.sgb + G.rb + G.qb)) |
                         (static_cast<uint64_t>(seg) << (G.rb + G.qb)) |
                         (static_cast<uint64_t>(local_of(L, kd)) << G.qb) | qin;
    out[e] = owner_of(L, kd) == L.rank ? key : DROP_KEY;
  }
}

// sparse x' exchange: mark the class-A x entries that cross ranks.  Edge (dst kd, src ks):
// the row's owner q reads source ks, whose x' lives in owner r's slot.  A plain load first, so
// hub sources (one word, many edges) cost one atomic per word, not one per edge.
__global__ void k_sx_bits(const uint64_t* uk, uint64_t nnz, int nb, const uint32_t* inv, Layout L,
                          uint32_t* sbits, uint32_t* rbits) {
  PRMI_BLOCK_LOOP(nnz) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e >= nnz) continue;
    const uint64_t k = uk[e];
    const uint32_t kd = inv[static_cast<uint32_t>(k >> nb)];
    const uint32_t ks = inv[static_cast<uint32_t>(k & ((1ull << nb) - 1))];
    if (ks >= L.nA) continue;  // class-C sources are constant after round 1: never exchanged
    const uint32_t q = owner_of(L, kd), r = owner_of(L, ks);
    if (q == r || (q != L.rank && r != L.rank)) continue;
    const uint32_t xp = xpos(L, ks);  // inside slot r
    const uint64_t bit = r == L.rank ? static_cast<uint64_t>(q) * L.maxA + (xp - r * L.maxA) : xp;
    uint32_t* w = (r == L.rank ? sbits : rbits) + (bit >> 5);
    const uint32_t m = 1u << (bit & 31);
    if (!(__builtin_nontemporal_load(w) & m)) atomicOr(w, m);
  }
}
__global__ void k_sx_pack(const double* slot, const uint32_t* pos, uint64_t n, double* buf) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) buf[i] = slot[pos[i]];
}
__global__ void k_sx_unpack(double* x, const uint32_t* pos, uint64_t n, const double* buf) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) x[pos[i]] = buf[i];
}

// first sorted edge of each stream group (atomicMin; empty groups keep the sentinel)
__global__ void k_group_starts(const uint64_t* key, uint64_t n, StreamGeo G,
                               unsigned long long* starts) {
  PRMI_BLOCK_LOOP(n) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e >= n) continue;
    const uint32_t gr = group_of_key(G, key[e]);
    if (e == 0 || group_of_key(G, key[e - 1]) != gr)
      atomicMin(&starts[gr], static_cast<unsigned long long>(e));
  }
}

// first sorted edge of slice j whose segment lies behind the L2-hot range (one thread per slice,
// lower bound over the sorted stream keys)
__global__ void k_cold_start(const uint64_t* key, uint64_t n, StreamGeo G, uint64_t* idx) {
  const uint32_t j = threadIdx.x;
  if (j >= NSLICE) return;
  const uint64_t want = (static_cast<uint64_t>(j) << (G.sgb + G.rb + G.qb)) |
                        (static_cast<uint64_t>(G.nlds + 1u) << (G.rb + G.qb));
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (key[mid] < want) lo = mid + 1; else hi = mid;
  }
  idx[j] = lo;
}

// column of every stream edge (LDS groups: u16 offset inside the block; L2 group: x position)
__global__ void k_stream_fill(const uint64_t* key, uint64_t n, Layout L, StreamGeo G,
                              const uint64_t* gstart, const uint64_t* gbase, uint32_t* col,
                              uint16_t* col16) {
  PRMI_BLOCK_LOOP(n) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e >= n) continue;
    const uint64_t k = key[e];
    const uint32_t gr = group_of_key(G, k);
    const uint64_t rel = e - gstart[gr];
    const uint32_t sl = static_cast<uint32_t>(k >> (G.sgb + G.rb + G.qb));
    const uint32_t seg = static_cast<uint32_t>(k >> (G.rb + G.qb)) & ((1u << G.sgb) - 1u);
    const uint32_t qin = static_cast<uint32_t>(k & ((1ull << G.qb) - 1));
    if (seg < G.nlds) col16[gbase[gr] + rel] = static_cast<uint16_t>(qin);
    else col[gbase[gr] + rel] = xpos(L, col_of_slice_q(L, G, sl, q_of_seg(G, seg, qin)));
  }
}

// pair-start flags, one 32-bit word per thread (indexed by stream position = task * TASK +
// offset; groups start on task boundaries, so a word never spans two groups): bit b is set
// when edge pos0 + b starts a (row, slice, segment) pair.  No atomics on the words; the pair
// count goes to NPAIR_SHARDS shards.
constexpr int NPAIR_SHARDS = 1024;
__global__ void k_stream_bits(const uint64_t* key, const uint64_t* gstart, const uint32_t* gtask,
                              uint32_t ngroups, uint64_t nwords, int qb, uint32_t* bits32,
                              unsigned long long* npair) {
  PRMI_BLOCK_LOOP(nwords) {
    const uint64_t w = blk_ * blockDim.x + threadIdx.x;
    uint32_t word = 0;
    if (w < nwords) {
      const uint64_t pos0 = w * 32;
      const uint64_t t = pos0 / TASK;
      uint32_t lo = 0, hi = ngroups - 1;  // last group whose first task <= t
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (gtask[mid] <= t) lo = mid; else hi = mid - 1;
      }
      const uint64_t rel0 = pos0 - static_cast<uint64_t>(gtask[lo]) * TASK;
      const uint64_t g0 = gstart[lo], glen = gstart[lo + 1] - g0;
      uint64_t prev = rel0 ? key[g0 + rel0 - 1] >> qb : ~0ull;
      for (int b = 0; b < 32 && rel0 + b < glen; ++b) {
        const uint64_t cur = key[g0 + rel0 + b] >> qb;
        if (cur != prev) word |= 1u << b;
        prev = cur;
      }
      bits32[w] = word;
    }
    const uint64_t c = wave_sum_u64(__popc(word));
    if ((threadIdx.x & 63) == 0 && c)
      atomicAdd(&npair[blk_ % NPAIR_SHARDS], static_cast<unsigned long long>(c));
  }
}

__global__ void k_fill_u16(uint16_t* a, uint64_t n, uint16_t v) {
  PRMI_BLOCK_LOOP(n) {
    const uint64_t i = blk_ * blockDim.x + threadIdx.x;
    if (i < n) a[i] = v;
  }
}

// pieces of each task (piece starts: the task's first edge and every pair start)
__global__ void k_task_count(const uint32_t* bits32, uint32_t ntask, uint32_t* cnt) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntask) return;
  if (t == ntask) {
    cnt[t] = 0;
    return;
  }
  const uint64_t w0 = static_cast<uint64_t>(t) * (TASK / 32);
  uint32_t c = 0;
  for (int i = 0; i < TASK / 32; ++i) c += __popc(bits32[w0 + i] | (i == 0 ? 1u : 0u));
  cnt[t] = c;
}

// piece index of stream position pos; also whether pos starts a piece
__device__ __forceinline__ uint32_t piece_of(const uint32_t* bits32, const uint32_t* task_piece,
                                             uint64_t pos, bool* starts) {
  const uint64_t t = pos / TASK;
  const uint64_t w0 = t * (TASK / 32), wp = pos / 32;
  const uint32_t bit = static_cast<uint32_t>(pos % 32);
  uint32_t c = 0;
  for (uint64_t w = w0; w < wp; ++w) c += __popc(bits32[w] & (w == w0 ? ~1u : ~0u));
  const uint32_t last = bits32[wp] & (wp == w0 ? ~1u : ~0u);
  c += __popc(last & (bit == 31 ? ~0u : ((2u << bit) - 1u)));
  if (starts) *starts = (pos % TASK) == 0 || ((bits32[wp] >> bit) & 1u);
  return task_piece[t] + c;
}

// row and stream (slice * nseg + segment) of every piece (from the stream keys)
__global__ void k_piece_rows(const uint64_t* key, uint64_t n, StreamGeo G, uint32_t nseg,
                             const uint64_t* gstart, const uint32_t* gtask, const uint32_t* bits32,
                             const uint32_t* task_piece, uint32_t* piece_row,
                             uint32_t* piece_stream) {
  PRMI_BLOCK_LOOP(n) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e >= n) continue;
    const uint64_t k = key[e];
    const uint32_t gr = group_of_key(G, k);
    const uint64_t pos = static_cast<uint64_t>(gtask[gr]) * TASK + (e - gstart[gr]);
    bool st = false;
    const uint32_t pc = piece_of(bits32, task_piece, pos, &st);
    if (st) {
      piece_row[pc] = static_cast<uint32_t>(k >> G.qb) & ((1u << G.rb) - 1u);
      const uint32_t sl = static_cast<uint32_t>(k >> (G.sgb + G.rb + G.qb));
      const uint32_t seg = static_cast<uint32_t>(k >> (G.rb + G.qb)) & ((1u << G.sgb) - 1u);
      piece_stream[pc] = sl * nseg + seg;
    }
  }
}

// row offsets in row-launch order (RowArgs::roffL): one workgroup per block; each wave walks
// the block's lines exactly as spmv_rows does and stores lane l's offsets of an 8-line group
// contiguously
__global__ __launch_bounds__(BLOCK) void k_roff_lines(const uint16_t* roff, const uint32_t* nebase,
                                                      const uint32_t* ne_off, const uint32_t* l_off,
                                                      const uint32_t* btot, const uint32_t* lfirst,
                                                      const uint64_t* lmask, const uint32_t* goff,
                                                      uint32_t* roffL, uint32_t roff16) {
  const uint32_t b = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t L0 = l_off[b], nl = l_off[b + 1] - L0, tot = btot[b], ne0 = ne_off[b];
  const uint32_t G0 = goff[b], ng = (nl + EPR - 1) / EPR;
  const uint64_t lbits = (2ull << lane) - 2ull;
  for (uint32_t gi = wv; gi < ng; gi += BLOCK / 64) {
    uint32_t w[3] = {0u, 0u, 0u};
    for (int u = 0; u < EPR; ++u) {
      const uint32_t L = gi * EPR + u, i = L * 64u + static_cast<uint32_t>(lane);
      uint32_t r = 0;
      if (L < nl && i < tot) {
        const uint32_t q = lfirst[L0 + L] + static_cast<uint32_t>(__popcll(lmask[L0 + L] & lbits));
        r = roff[nebase[ne0 + q] + i];  // < RB = 1024: 10 bits
      }
      w[u / 3] |= r << (10 * (u % 3));
    }
    const uint64_t gl = (static_cast<uint64_t>(G0 + gi) * 64u) + static_cast<uint32_t>(lane);
    if (roff16) {  // the earlier layout: lane l's 8 offsets as 8 x u16 in 16 bytes
      uint16_t* d16 = reinterpret_cast<uint16_t*>(roffL) + gl * EPR;
      for (int u = 0; u < EPR; ++u) d16[u] = static_cast<uint16_t>((w[u / 3] >> (10 * (u % 3))) & 0x3FFu);
    } else {
      uint32_t* dst = roffL + gl * 3u;
      dst[0] = w[0];
      dst[1] = w[1];
      dst[2] = w[2];
    }
  }
}

// PR_PIECE_STATS (build-time report): pieces and edges by row in-degree bin (bin b holds
// in-degrees [2^b, 2^(b+1))) and by segment kind (0 LDS block, 1 L2-hot, 2 cold)
constexpr int PS_BINS = 24;
__device__ __forceinline__ int ps_bin(uint32_t d) { return d ? min(31 - __clz(d), PS_BINS - 1) : 0; }
__device__ __forceinline__ uint32_t ps_kind(uint32_t seg, uint32_t nlds) {
  return seg < nlds ? 0u : (seg == nlds ? 1u : 2u);
}
__global__ void k_ps_edges(const uint64_t* key, uint64_t n, StreamGeo G, uint32_t* rowcnt) {
  PRMI_BLOCK_LOOP(n) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e < n) atomicAdd(&rowcnt[static_cast<uint32_t>(key[e] >> G.qb) & ((1u << G.rb) - 1u)], 1u);
  }
}
// hist[bin][kind][0 pieces | 1 edges], rows[bin]
__global__ void k_ps_pieces(const uint32_t* prow, const uint32_t* pstream, uint64_t np,
                            uint32_t nseg, uint32_t nlds, const uint32_t* rowcnt,
                            unsigned long long* hist) {
  __shared__ unsigned long long h[PS_BINS * 3];
  for (int i = threadIdx.x; i < PS_BINS * 3; i += blockDim.x) h[i] = 0;
  __syncthreads();
  PRMI_BLOCK_LOOP(np) {
    const uint64_t i = blk_ * blockDim.x + threadIdx.x;
    if (i < np)
      atomicAdd(&h[ps_bin(rowcnt[prow[i]]) * 3 + ps_kind(pstream[i] % nseg, nlds)], 1ull);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < PS_BINS * 3; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[(i / 3) * 6 + (i % 3) * 2], h[i]);
}
__global__ void k_ps_edge_kinds(const uint64_t* key, uint64_t n, StreamGeo G, uint32_t nlds,
                                const uint32_t* rowcnt, unsigned long long* hist,
                                unsigned long long* rows) {
  __shared__ unsigned long long h[PS_BINS * 3];
  for (int i = threadIdx.x; i < PS_BINS * 3; i += blockDim.x) h[i] = 0;
  __syncthreads();
  PRMI_BLOCK_LOOP(n) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e < n) {
      const uint64_t k = key[e];
      const uint32_t l = static_cast<uint32_t>(k >> G.qb) & ((1u << G.rb) - 1u);
      const uint32_t seg = static_cast<uint32_t>(k >> (G.rb + G.qb)) & ((1u << G.sgb) - 1u);
      atomicAdd(&h[ps_bin(rowcnt[l]) * 3 + ps_kind(seg, nlds)], 1ull);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < PS_BINS * 3; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[(i / 3) * 6 + (i % 3) * 2 + 1], h[i]);
  (void)rows;
}
__global__ void k_ps_rows(const uint32_t* rowcnt, uint32_t nrows, unsigned long long* rows) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l < nrows && rowcnt[l]) atomicAdd(&rows[ps_bin(rowcnt[l])], 1ull);
}

// row blocks of the row launch: class-A rows in blocks of RB, then class-B rows
struct RowBlocks {
  uint32_t lA, nbA, NB, NS, rb;
  uint32_t nbH, rbH, lH;  // heavy blocks first: rows [0, lH) in blocks of rbH
};
__device__ __forceinline__ uint32_t block_of_row(const RowBlocks& B, uint32_t l) {
  if (l < B.lH) return l / B.rbH;
  return l < B.lA ? B.nbH + (l - B.lH) / B.rb : B.nbA + (l - B.lA) / B.rb;
}
__device__ __forceinline__ uint32_t block_row0(const RowBlocks& B, uint32_t b) {
  if (b < B.nbH) return b * B.rbH;
  return b < B.nbA ? B.lH + (b - B.nbH) * B.rb : B.lA + (b - B.nbA) * B.rb;
}

// local class-A rows with in-degree >= thr (a prefix: rows are in-degree sorted)
__global__ void k_count_heavy(const uint32_t* perm, const uint32_t* indeg, uint32_t lA, Layout L,
                              uint32_t thr, unsigned* cnt) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  const bool h = l < lA && indeg[perm[row_of(L, l)]] >= thr;
  const uint64_t m = __ballot(h);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(cnt, static_cast<unsigned>(__popcll(m)));
}

// ---- direct-pull experiment (PR_DPULL = D, timing only; single rank) ------------------------
// Rows with in-degree < D (a suffix of the class-A rows and a suffix of the class-B rows: rows
// are in-degree sorted) leave nothing in the streams when PR_DROPDEG = D is set as well, and a
// thread per row sums x over the row's sources straight through the L1 / L2 instead.  Their
// columns are stored per group of 64 consecutive rows, column-major (entry k of lane l at
// base + 64 k + l, padded to the group's longest row with PAD_COL, whose gather reads 0), so
// a wave reads them fully coalesced.  The sums go to a side array: this measures what such a
// path costs, it does not feed the ranks.
struct DpGeo {
  uint32_t lAdp, lA, lBdp, lrows;  // direct-pull rows: [lAdp, lA) and [lBdp, lrows)
};
__device__ __forceinline__ uint32_t dp_of_row(const DpGeo& D, uint32_t l) {
  if (l >= D.lAdp && l < D.lA) return l - D.lAdp;
  if (l >= D.lBdp && l < D.lrows) return (D.lA - D.lAdp) + (l - D.lBdp);
  return 0xFFFFFFFFu;
}
__device__ __forceinline__ uint32_t row_of_dp(const DpGeo& D, uint32_t i) {
  const uint32_t na = D.lA - D.lAdp;
  return i < na ? D.lAdp + i : D.lBdp + (i - na);
}
__global__ void k_count_ge(const uint32_t* perm, const uint32_t* indeg, uint32_t l0, uint32_t l1,
                           Layout L, uint32_t thr, unsigned* cnt) {
  const uint32_t l = l0 + blockIdx.x * blockDim.x + threadIdx.x;
  const bool h = l < l1 && indeg[perm[row_of(L, l)]] >= thr;
  const uint64_t m = __ballot(h);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(cnt, static_cast<unsigned>(__popcll(m)));
}
// in-degree of every direct-pull row and 64 x the longest row of each 64-row group
__global__ void k_dp_deg(const uint32_t* perm, const uint32_t* indeg, DpGeo D, Layout L,
                         uint32_t ndp, uint32_t* deg, uint32_t* gw) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t d = i < ndp ? indeg[perm[row_of(L, row_of_dp(D, i))]] : 0u;
  if (i < ndp) deg[i] = d;
  const int mx = wave_max_i(static_cast<int>(d));
  if ((threadIdx.x & 63) == 0 && i < ndp) gw[i >> 6] = 64u * static_cast<uint32_t>(mx);
}
// (direct-pull row << 32 | x position) of every edge into such a row, appended in any order
__global__ void k_dp_keys(const uint64_t* uk, uint64_t nnz, int nb, const uint32_t* inv,
                          const uint32_t* indeg, Layout L, DpGeo D, uint32_t thr, uint64_t* out,
                          unsigned long long* cnt) {
  PRMI_BLOCK_LOOP(nnz) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    uint64_t key = DROP_KEY;
    if (e < nnz) {
      const uint64_t k = uk[e];
      const uint32_t dv = static_cast<uint32_t>(k >> nb);
      if (indeg[dv] < thr) {
        const uint32_t i = dp_of_row(D, local_of(L, inv[dv]));
        const uint32_t ks = inv[static_cast<uint32_t>(k & ((1ull << nb) - 1))];
        if (i != 0xFFFFFFFFu) key = (static_cast<uint64_t>(i) << 32) | xpos(L, ks);
      }
    }
    const bool take = key != DROP_KEY;
    const uint64_t m = __ballot(take);
    if (!m) continue;
    unsigned long long base = 0;
    const int lane = threadIdx.x & 63;
    if (lane == 0) base = atomicAdd(cnt, static_cast<unsigned long long>(__popcll(m)));
    base = __shfl(base, 0);
    if (take) out[base + __popcll(m & ((1ull << lane) - 1ull))] = key;
  }
}
__global__ void k_dp_fill(const uint64_t* key, uint64_t ne, const uint32_t* rowstart,
                          const uint32_t* gbase, uint32_t* ell) {
  PRMI_BLOCK_LOOP(ne) {
    const uint64_t e = blk_ * blockDim.x + threadIdx.x;
    if (e >= ne) continue;
    const uint32_t i = static_cast<uint32_t>(key[e] >> 32);
    const uint32_t k = static_cast<uint32_t>(e) - rowstart[i];
    ell[gbase[i >> 6] + 64u * k + (i & 63u)] = static_cast<uint32_t>(key[e]);
  }
}
// one wave per 64-row group, lane = row; eight gathers in flight per lane
__global__ __launch_bounds__(BLOCK) void spmv_dpull(const uint32_t* __restrict__ ell,
                                                    const uint32_t* __restrict__ gbase,
                                                    const double* x, uint32_t x_bytes,
                                                    uint32_t ngroups, double* __restrict__ out) {
  const uint32_t g = blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
  if (g >= ngroups) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t b0 = gbase[g], W = (gbase[g + 1] - b0) >> 6;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(x), static_cast<short>(0), static_cast<int>(x_bytes), 0x00020000);
  const uint32_t* e = ell + b0 + lane;
  double c = 0.0;
  uint32_t k = 0;
  auto gat = [&](uint32_t col) -> double {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(xr, col * 8u, 0, 0);  // PAD_COL: out of range, 0
    return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(v[1]) << 32) | v[0]));
  };
  for (; k + 8 <= W; k += 8) {
    uint32_t cc[8];
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) cc[u] = e[64u * (k + u)];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = gat(cc[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u) c += v[u];
  }
  for (; k < W; ++k) c += gat(e[64u * k]);
  out[g * 64u + lane] = c;
}

// per-piece row offset in its block + run starts T[block][stream] (sentinel where empty)
__global__ void k_runs(const uint32_t* prow, const uint32_t* pstream, uint64_t np, RowBlocks B,
                       uint16_t* roff, uint32_t* T, uint32_t* sstart) {
  PRMI_BLOCK_LOOP(np) {
    const uint64_t i = blk_ * blockDim.x + threadIdx.x;
    if (i >= np) continue;
    const uint32_t l = prow[i], k = pstream[i], b = block_of_row(B, l);
    roff[i] = static_cast<uint16_t>(l - block_row0(B, b));
    const bool first = i == 0 || pstream[i - 1] != k || block_of_row(B, prow[i - 1]) != b;
    if (first) T[static_cast<uint64_t>(b) * B.NS + k] = static_cast<uint32_t>(i);
    if (i == 0 || pstream[i - 1] != k) sstart[k] = static_cast<uint32_t>(i);
  }
}

__global__ void k_fill_f64(double* a, uint64_t n, double v) {
  PRMI_BLOCK_LOOP(n) {
    const uint64_t i = blk_ * blockDim.x + threadIdx.x;
    if (i < n) a[i] = v;
  }
}

__global__ void k_iota(uint32_t* a, uint64_t n) {
  PRMI_BLOCK_LOOP(n) {
    const uint64_t i = blk_ * blockDim.x + threadIdx.x;
    if (i < n) a[i] = static_cast<uint32_t>(i);
  }
}

__global__ void k_local_meta(const uint32_t* perm, const uint32_t* outdeg, const uint32_t* dang_w,
                             uint32_t lrows, uint32_t lA, Layout L, uint32_t* meta) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= lrows) return;
  const uint32_t v = perm[row_of(L, l)];
  meta[l] = l < lA ? outdeg[v] : dang_w[v];
}

// export: (internal row << 32 | internal source) of every stream edge
__global__ void k_piece_row_runs(const uint32_t* T, const uint16_t* roff, RowBlocks B,
                                 uint32_t* piece_row) {
  PRMI_BLOCK_LOOP(static_cast<uint64_t>(B.NB) * B.NS) {
    const uint64_t t = blk_ * blockDim.x + threadIdx.x;
    if (t >= static_cast<uint64_t>(B.NB) * B.NS) continue;
    const uint32_t b = static_cast<uint32_t>(t / B.NS);
    const uint32_t r0 = block_row0(B, b);
    for (uint32_t i = T[t]; i < T[t + B.NS]; ++i) piece_row[i] = r0 + roff[i];
  }
}
__global__ void k_export_keys(const uint32_t* col, const uint16_t* col16, const uint32_t* bits32,
                              const uint32_t* task_piece, const uint32_t* piece_row, Layout L,
                              const uint64_t* gstart, const uint32_t* gtask, const uint64_t* gbase,
                              uint32_t ngroups, uint32_t nlds, uint32_t H, uint64_t stream_len,
                              uint64_t* out) {
  PRMI_BLOCK_LOOP(stream_len) {
    const uint64_t pos = blk_ * blockDim.x + threadIdx.x;
    if (pos >= stream_len) continue;
    const uint32_t t = static_cast<uint32_t>(pos / TASK);
    uint32_t lo = 0, hi = ngroups - 1;  // last group whose first task <= t
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) / 2;
      if (gtask[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const uint64_t rel = pos - static_cast<uint64_t>(gtask[lo]) * TASK;
    if (rel >= gstart[lo + 1] - gstart[lo]) continue;  // padding
    const uint32_t pc = piece_of(bits32, task_piece, pos, nullptr);
    const uint32_t row = row_of(L, piece_row[pc]);
    const uint32_t j = lo / (nlds + 1), gi = lo % (nlds + 1);
    uint32_t xp;
    if (gi < nlds) xp = (j % L.p) * L.maxA + (j / L.p) * L.SL + gi * H + col16[gbase[lo] + rel];
    else xp = col[gbase[lo] + rel];
    out[gstart[lo] + rel] = (static_cast<uint64_t>(row) << 32) | col_of_xpos(L, xp);
  }
}
__global__ void k_export_split(const uint64_t* key, uint64_t n, uint32_t* col, uint64_t* row_ptr) {
  PRMI_BLOCK_LOOP(n) {
    const uint64_t i = blk_ * blockDim.x + threadIdx.x;
    if (i >= n) continue;
    const uint64_t k = key[i];
    col[i] = static_cast<uint32_t>(k);
    if (i == 0 || (key[i - 1] >> 32) != (k >> 32)) row_ptr[k >> 32] = i;
  }
}

__global__ void k_scatter_ranks(const uint32_t* perm, const double* r_loc, uint32_t lrows,
                                Layout L, double* r_full) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l < lrows) r_full[perm[row_of(L, l)]] = r_loc[l];
}

__global__ void k_sources_one(const uint32_t* outdeg, uint32_t n, double r0, double* r_full) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) r_full[v] = outdeg[v] ? r0 : 0.0;
}

// ---- top-K selection (PageRank.java:167-189 join(mappings) + sortByKey(false) + take(k)) --
// A weighted radix select over the bit patterns of r_full: defined ranks are positive
// doubles, which order like their bits.  A page weighs its number of mapping pairs (the
// join at :167 emits one record per (id, title); ids outside the mapping weigh 0 and never
// reach the output).  Digits of SEL_BITS from the top; pass d histograms, per digit, the
// weight and the page count of the pages whose key matches the prefix chosen so far.
constexpr int SEL_BITS = 11, SEL_BINS = 1 << SEL_BITS;
__global__ __launch_bounds__(BLOCK) void k_select_hist(const double* r, const uint32_t* mapw,
                                                       uint32_t n, uint64_t prefix, uint64_t pmask,
                                                       int shift, uint32_t dmask,
                                                       unsigned long long* hist) {
  __shared__ unsigned long long hw[SEL_BINS], hc[SEL_BINS];
  for (int i = threadIdx.x; i < SEL_BINS; i += BLOCK) hw[i] = hc[i] = 0;
  __syncthreads();
  for (uint32_t v = blockIdx.x * BLOCK + threadIdx.x; v < n; v += gridDim.x * BLOCK) {
    const uint64_t key = static_cast<uint64_t>(__double_as_longlong(r[v]));
    const uint32_t w = mapw ? mapw[v] : 1u;
    if (key == 0 || w == 0 || (key & pmask) != prefix) continue;
    const uint32_t d = static_cast<uint32_t>(key >> shift) & dmask;
    atomicAdd(&hw[d], static_cast<unsigned long long>(w));
    atomicAdd(&hc[d], 1ull);
  }
  __syncthreads();
  for (int i = threadIdx.x; i <= static_cast<int>(dmask); i += BLOCK)
    if (hc[i]) {
      atomicAdd(&hist[i], hw[i]);
      atomicAdd(&hist[SEL_BINS + i], hc[i]);
    }
}

// every mapped page whose key is >= lb (order of the output is arbitrary; the host sorts)
__global__ void k_select_emit(const double* r, const uint32_t* mapw, uint32_t n, uint64_t lb,
                              uint32_t* ids, double* rs, unsigned* cnt, uint32_t cap) {
  const uint32_t v = blockIdx.x * BLOCK + threadIdx.x;
  if (v >= n) return;
  const double x = r[v];
  const uint64_t key = static_cast<uint64_t>(__double_as_longlong(x));
  if (key < lb || (mapw && mapw[v] == 0)) return;
  const unsigned i = atomicAdd(cnt, 1u);
  if (i < cap) {
    ids[i] = v;
    rs[i] = x;
  }
}

// =======================================================================================
// host side of the build
// =======================================================================================
namespace {

// blocks for n items, capped: kernels over edge-sized ranges loop (PRMI_BLOCK_LOOP) past it;
// the others are launched on vertex counts (< 2^32 / BLOCK blocks)
inline uint32_t grid_for(uint64_t n) { return static_cast<uint32_t>((n + BLOCK - 1) / BLOCK); }
inline uint32_t grid_loop(uint64_t n) {
  return static_cast<uint32_t>(std::min<uint64_t>((n + BLOCK - 1) / BLOCK, 1u << 22));
}

int bits_for(uint64_t n) {
  if (n <= 2) return 1;
  return 64 - __builtin_clzll(n - 1);
}

template <class T>
int dmalloc(T** p, size_t count, std::string* err) {
  *p = nullptr;
  if (count == 0) count = 1;
  HIPTRY(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  return PR_OK;
}

struct Temp {
  void* p = nullptr;
  size_t bytes = 0;
  ~Temp() { if (p) (void)hipFree(p); }
  int ensure(size_t b, std::string* err) {
    if (b <= bytes) return PR_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    HIPTRY(hipMalloc(&p, b ? b : 1));
    bytes = b;
    return PR_OK;
  }
};

#define TRY(x)                  \
  do {                          \
    int rc_ = (x);              \
    if (rc_ != PR_OK) return rc_; \
  } while (0)

int env_int(const char* name, int def) {
  const char* s = getenv(name);
  return s && *s ? atoi(s) : def;
}

}  // namespace

void dev_free(DevGraph* g) {
  auto F = [](void* p) { if (p) (void)hipFree(p); };
  F(g->col); F(g->bits); F(g->task_piece); F(g->partial); F(g->roff); F(g->runs);
  F(g->nebase); F(g->ne_off); F(g->l_off); F(g->btot); F(g->lfirst); F(g->lmask);
  F(g->goff); F(g->roffL);
  F(g->sx_spos); F(g->sx_rpos); F(g->sx_sbuf); F(g->sx_rbuf);
  F(g->d_gtask); F(g->d_gstart); F(g->d_gbase); F(g->col16);
  F(g->meta); F(g->perm); F(g->outdeg); F(g->indeg); F(g->dang_w);
  F(g->x_init); F(g->xbuf[0]); F(g->xbuf[1]); F(g->r_loc[0]); F(g->r_loc[1]); F(g->r_full);
  F(g->shards); F(g->rec_local); F(g->rec_all); F(g->state); F(g->mapw);
  F(g->x_seed); F(g->r_seed);
  F(g->dp_ell); F(g->dp_gbase); F(g->dp_out); F(g->stream_cnt);
  const int p = g->p, rank = g->rank;
  *g = DevGraph();
  g->p = p;
  g->rank = rank;
}

namespace {

Layout layout_of(const DevGraph* g) {
  return Layout{static_cast<uint32_t>(g->p), static_cast<uint32_t>(g->rank), g->nA, g->R, g->nC,
                g->maxA, g->sm ? 1u : 0u, g->SL, g->SLC, g->snake ? 1u : 0u};
}

// rows owned by rank j among internal ids [0, cnt) when chunks of CHUNK are dealt round-robin
uint32_t owned_rows(uint32_t cnt, uint32_t p, uint32_t j) {
  const uint32_t full = cnt / CHUNK, rem = cnt % CHUNK;
  uint32_t r = CHUNK * (full / p + (j < full % p ? 1u : 0u));
  if (rem && full % p == j) r += rem;
  return r;
}

// The row deal and x layout of rank `rank` of `p` for a graph with nA / nB / nC vertices in
// classes A / B / C: everything dev_build and the exchange derive from the class counts.
struct LayoutDims {
  Layout L;
  uint64_t X;            // x length
  uint32_t lrows, lA;    // local rows, local class-A rows
};
LayoutDims make_layout(int p, int rank, uint32_t nA, uint32_t nB, uint32_t nC) {
  LayoutDims d{};
  const uint32_t P = static_cast<uint32_t>(p), RK = static_cast<uint32_t>(rank);
  const bool sm = (NSLICE % P) == 0 && env_int("PR_SLICE_MAJOR", 1) != 0;
  const bool snake = sm && P == 1 && env_int("PR_SNAKE", 1) != 0;
  uint32_t SL = 0, SLC = 0, maxA = 0;
  if (sm) {
    const uint32_t chA = (nA + CHUNK - 1) / CHUNK, chC = (nC + CHUNK - 1) / CHUNK;
    SL = CHUNK * ((chA + NSLICE - 1) / NSLICE);
    SLC = CHUNK * ((chC + NSLICE - 1) / NSLICE);
    maxA = (NSLICE / P) * SL;
    d.X = static_cast<uint64_t>(P) * maxA + static_cast<uint64_t>(NSLICE) * SLC;
  } else {
    for (uint32_t j = 0; j < P; ++j) maxA = std::max(maxA, owned_rows(nA, P, j));
    maxA = (maxA + CHUNK - 1) / CHUNK * CHUNK;
    d.X = static_cast<uint64_t>(P) * maxA + nC;
  }
  d.L = Layout{P, RK, nA, nA + nB, nC, maxA, sm ? 1u : 0u, SL, SLC, snake ? 1u : 0u};
  d.lrows = owned_rows(nA + nB, P, RK);
  d.lA = owned_rows(nA, P, RK);
  return d;
}


}  // namespace

int dev_build(DevGraph* g, const BuildInput& in, hipStream_t s, std::string* err) {
  Span span("prmi:build");
  auto t0 = std::chrono::steady_clock::now();
  const int p = g->p, rank = g->rank;
  dev_free(g);
  Tuning& T = g->tune;
  // p >= 2: a 1.5 MiB L2-hot range (per-rank SpMV -3 % at p = 2 and 4, -2 % at p = 8)
  const int qh_def = p >= 2 ? 196608 : static_cast<int>(T.qh);  // (p = 1: Tuning::qh)
  T.qh = static_cast<uint32_t>(std::max(CHUNK, env_int("PR_QH", qh_def)));
  T.seg = static_cast<uint32_t>(std::max(CHUNK, env_int("PR_SEG", static_cast<int>(T.seg))));
  T.nt = env_int("PR_NT", T.nt);
  T.hot_lds = static_cast<uint32_t>(std::max(0, std::min(20480, env_int("PR_HOTLDS", static_cast<int>(T.hot_lds)))));
  T.dbg = env_int("PR_DBG", 0);
  T.lean = env_int("PR_LEAN", T.lean);
  T.rb_heavy = static_cast<uint32_t>(std::max(64, std::min(RB, env_int("PR_RBH", static_cast<int>(T.rb_heavy)))));
  T.heavy_deg = static_cast<uint32_t>(std::max(0, env_int("PR_HDEG", static_cast<int>(T.heavy_deg))));
  T.rb = static_cast<uint32_t>(std::max(64, std::min(RB, env_int("PR_RB", static_cast<int>(T.rb)))));
  T.rxg = static_cast<uint32_t>(std::max(1, std::min(4096, env_int("PR_RXG", static_cast<int>(T.rxg)))));
  // LDS blocks per slice: PR_NLDS overrides; otherwise the count follows the graph and the
  // rank count (below, once the slice length is known)
  const int nlds_env = env_int("PR_NLDS", -1);
  T.stream_wg = std::max(1, std::min(2, env_int("PR_STREAM_WG", T.stream_wg)));
  if (const char* cm = getenv("PR_COLMASK")) T.colmask = static_cast<uint32_t>(strtoul(cm, nullptr, 0));
  T.l2mode = env_int("PR_L2MODE", T.l2mode);
  T.l2w = std::max(0, std::min(12, env_int("PR_L2W", T.l2w)));
  T.l2late = env_int("PR_L2LATE", T.l2late);
  // p > 1: the stream launch leaves one compute unit of every XCD free.  Its workgroups hold a
  // compute unit's whole LDS for the length of the launch, so nothing else can start beside
  // them -- and with the overlapped exchange RCCL's send/recv kernels must run beside part 1 of
  // the launch, or the chunks behind the hot prefix only travel once it has ended.
  T.stream_cus = env_int("PR_STREAM_CUS", p > 1 ? 31 : T.stream_cus);
  T.dpull = static_cast<uint32_t>(std::max(0, env_int("PR_DPULL", 0)));
  T.dropdeg = static_cast<uint32_t>(std::max(0, env_int("PR_DROPDEG", 0)));
  T.keepdeg = static_cast<uint32_t>(std::max(0, env_int("PR_KEEPDEG", 0)));
  const uint32_t n = in.n;
  const uint64_t m = in.m;
  g->n = n;
  g->m_raw = m;
  g->n_tot = in.n_tot;
  if (in.normalized) {
    if (in.n_tot == 0) {
      if (err) *err = "normalized ranks need N_tot > 0 (an empty mapping divides by zero)";
      return PR_E_ARG;
    }
    g->r0 = 1.0 / static_cast<double>(in.n_tot);
    g->base = 0.15 / static_cast<double>(in.n_tot);
  }
  const int nb = in.rmat ? std::max(1, in.scale) : bits_for(n);
  // raw edge keys (dst, src) take 2*nb bits
  if (2 * nb > 64) {
    if (err) *err = "more than 2^32 vertices is not supported (64-bit edge keys)";
    return PR_E_ARG;
  }
  Temp tmp;

  span.next("prmi:build:raw keys");
  // ---- raw keys (dst << nb | src) ------------------------------------------------------
  uint64_t *kA = nullptr, *kB = nullptr;
  TRY(dmalloc(&kA, m, err));
  TRY(dmalloc(&kB, m, err));
  struct Guard {
    uint64_t** a;
    uint64_t** b;
    ~Guard() {
      if (*a) (void)hipFree(*a);
      if (*b) (void)hipFree(*b);
    }
  } guard{&kA, &kB};
  if (in.rmat) {
    if (m) hipLaunchKernelGGL(k_rmat_keys, dim3(grid_loop(m)), dim3(BLOCK), 0, s, in.seed, in.scale, m, kA);
  } else if (m) {
    uint32_t *ds = nullptr, *dd = nullptr;
    TRY(dmalloc(&ds, m, err));
    TRY(dmalloc(&dd, m, err));
    HIPTRY(hipMemcpyAsync(ds, in.h_src, m * 4, hipMemcpyHostToDevice, s));
    HIPTRY(hipMemcpyAsync(dd, in.h_dst, m * 4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_make_keys, dim3(grid_loop(m)), dim3(BLOCK), 0, s, ds, dd, m, nb, kA);
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(ds);
    (void)hipFree(dd);
  }
  HIPTRY(hipGetLastError());

  span.next("prmi:build:distinct");
  // ---- distinct() (PageRank.java:42): sort + unique -------------------------------------
  uint64_t nnz = 0;
  uint64_t* uniq = nullptr;  // points into kA or kB
  {
    rocprim::double_buffer<uint64_t> db(kA, kB);
    size_t tb = 0;
    HIPTRY(rocprim::radix_sort_keys(nullptr, tb, db, m, 0, 2 * nb, s));
    TRY(tmp.ensure(tb, err));
    if (m) HIPTRY(rocprim::radix_sort_keys(tmp.p, tb, db, m, 0, 2 * nb, s));
    uint64_t* sorted = db.current();
    uint64_t* other = sorted == kA ? kB : kA;
    uint64_t* d_cnt = nullptr;
    TRY(dmalloc(&d_cnt, 1, err));
    HIPTRY(rocprim::unique(nullptr, tb, sorted, other, d_cnt, m, rocprim::equal_to<uint64_t>(), s));
    TRY(tmp.ensure(tb, err));
    HIPTRY(hipMemsetAsync(d_cnt, 0, 8, s));
    if (m) HIPTRY(rocprim::unique(tmp.p, tb, sorted, other, d_cnt, m, rocprim::equal_to<uint64_t>(), s));
    HIPTRY(hipMemcpyAsync(&nnz, d_cnt, 8, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(d_cnt);
    uniq = other;
  }
  g->nnz = nnz;

  span.next("prmi:build:degrees + vertex order");
  // ---- degrees + digest + dangling weights + vertex order -------------------------------
  TRY(dmalloc(&g->outdeg, n, err));
  TRY(dmalloc(&g->indeg, n, err));
  TRY(dmalloc(&g->dang_w, n, err));
  TRY(dmalloc(&g->perm, n, err));
  unsigned long long* d_sums = nullptr;  // shards of W0
  unsigned long long* d_dig = nullptr;   // digest shards
  TRY(dmalloc(&d_sums, W_SHARDS, err));
  TRY(dmalloc(&d_dig, 2 * DIGEST_SHARDS, err));
  HIPTRY(hipMemsetAsync(d_sums, 0, 8ull * W_SHARDS, s));
  HIPTRY(hipMemsetAsync(d_dig, 0, 16ull * DIGEST_SHARDS, s));
  HIPTRY(hipMemsetAsync(g->outdeg, 0, 4ull * (n ? n : 1), s));
  {
    uint64_t *run_lo = nullptr, *run_hi = nullptr;  // per dst: [first, one past last) edge
    TRY(dmalloc(&run_lo, n, err));
    if (dmalloc(&run_hi, n, err) != PR_OK) {
      (void)hipFree(run_lo);
      return PR_E_OOM;
    }
    HIPTRY(hipMemsetAsync(run_lo, 0, 8ull * (n ? n : 1), s));
    HIPTRY(hipMemsetAsync(run_hi, 0, 8ull * (n ? n : 1), s));
    if (nnz) hipLaunchKernelGGL(k_degrees, dim3(grid_loop(nnz)), dim3(BLOCK), 0, s, uniq, nnz, nb, g->outdeg, run_lo, run_hi, d_dig);
    if (n) hipLaunchKernelGGL(k_indeg_from_runs, dim3(grid_for(n)), dim3(BLOCK), 0, s, run_lo, run_hi, n, g->indeg);
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(run_lo);
    (void)hipFree(run_hi);
  }
  {
    std::vector<unsigned long long> dig(2 * DIGEST_SHARDS);
    HIPTRY(hipMemcpyAsync(dig.data(), d_dig, 16ull * DIGEST_SHARDS, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(d_dig);
    unsigned long long a = 0, x = 0;
    for (int i = 0; i < DIGEST_SHARDS; ++i) {
      a += dig[2 * i];
      x ^= dig[2 * i + 1];
    }
    g->digest[0] = a;
    g->digest[1] = x;
  }
  uint32_t* d_mapw = nullptr;
  if (in.h_mapw) {
    TRY(dmalloc(&d_mapw, n, err));
    HIPTRY(hipMemcpyAsync(d_mapw, in.h_mapw, 4ull * n, hipMemcpyHostToDevice, s));
  }
  uint64_t *vk = nullptr, *vk2 = nullptr;
  uint32_t* vid = nullptr;
  TRY(dmalloc(&vk, n, err));
  TRY(dmalloc(&vk2, n, err));
  TRY(dmalloc(&vid, n, err));
  if (n) hipLaunchKernelGGL(k_vertex_keys, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->outdeg, g->indeg, d_mapw, n, g->dang_w, vk, vid, d_sums);
  HIPTRY(hipGetLastError());
  {
    size_t tb = 0;
    HIPTRY(rocprim::radix_sort_pairs(nullptr, tb, vk, vk2, vid, g->perm, n, 0, 34, s));
    TRY(tmp.ensure(tb, err));
    if (n) HIPTRY(rocprim::radix_sort_pairs(tmp.p, tb, vk, vk2, vid, g->perm, n, 0, 34, s));
  }
  unsigned* d_cls = nullptr;
  TRY(dmalloc(&d_cls, 4, err));
  unsigned cls_first[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  HIPTRY(hipMemcpyAsync(d_cls, cls_first, 16, hipMemcpyHostToDevice, s));
  if (n) hipLaunchKernelGGL(k_class_count, dim3(grid_for(n)), dim3(BLOCK), 0, s, vk2, n, d_cls);
  unsigned long long sums[W_SHARDS];
  HIPTRY(hipMemcpyAsync(cls_first, d_cls, 16, hipMemcpyDeviceToHost, s));
  HIPTRY(hipMemcpyAsync(sums, d_sums, 8ull * W_SHARDS, hipMemcpyDeviceToHost, s));
  HIPTRY(hipStreamSynchronize(s));
  (void)hipFree(d_cls);
  (void)hipFree(d_sums);
  (void)hipFree(vk);
  (void)hipFree(vk2);
  g->mapw = d_mapw;  // kept: the top-K selection weighs pages by their mapping pairs
  uint64_t w0 = 0;
  for (int i = 0; i < W_SHARDS; ++i) w0 += sums[i];
  g->W0 = w0;
  g->n_dang_entries = w0;
  uint32_t start[5];
  start[4] = n;
  for (int c = 3; c >= 0; --c) start[c] = cls_first[c] == 0xFFFFFFFFu ? start[c + 1] : cls_first[c];
  g->nA = start[1] - start[0];
  g->nB = start[2] - start[1];
  g->nC = start[3] - start[2];
  g->nD = start[4] - start[3];
  g->R = g->nA + g->nB;
  {
    const LayoutDims d = make_layout(p, rank, g->nA, g->nB, g->nC);
    g->sm = d.L.sm != 0;
    g->snake = d.L.snake != 0;
    g->SL = d.L.SL;
    g->SLC = d.L.SLC;
    g->maxA = d.L.maxA;
    g->X = d.X;
    g->lrows = d.lrows;
    g->lA = d.lA;
  }
  const Layout L = layout_of(g);

  span.next("prmi:build:x vectors + row data");
  // ---- x vectors ------------------------------------------------------------------------
  TRY(dmalloc(&g->x_init, g->X, err));
  TRY(dmalloc(&g->xbuf[0], g->X, err));
  TRY(dmalloc(&g->xbuf[1], g->X, err));
  HIPTRY(hipMemsetAsync(g->x_init, 0, 8 * (g->X ? g->X : 1), s));
  HIPTRY(hipMemsetAsync(g->xbuf[0], 0, 8 * (g->X ? g->X : 1), s));
  HIPTRY(hipMemsetAsync(g->xbuf[1], 0, 8 * (g->X ? g->X : 1), s));
  if (n) hipLaunchKernelGGL(k_x_init, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->perm, g->outdeg, n, L, g->r0, static_cast<const double*>(nullptr), g->x_init);
  uint32_t* inv = vid;  // reuse: n entries
  if (n) hipLaunchKernelGGL(k_inverse, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->perm, n, inv);

  // ---- per-row data ------------------------------------------------------------------------
  const uint32_t lrows = g->lrows;
  TRY(dmalloc(&g->meta, lrows, err));
  if (lrows) hipLaunchKernelGGL(k_local_meta, dim3(grid_for(lrows)), dim3(BLOCK), 0, s, g->perm, g->outdeg, g->dang_w, lrows, g->lA, L, g->meta);

  if (g->X >= (1ull << 28)) {  // gathers address x through a buffer descriptor (2^31 bytes)
    if (err) *err = "x vector longer than 2^28 entries is not supported";
    return PR_E_ARG;
  }
  // ---- stream geometry -----------------------------------------------------------------------
  StreamGeo G{};
  {
    const uint32_t chA = (g->nA + CHUNK - 1) / CHUNK, chC = (g->nC + CHUNK - 1) / CHUNK;
    G.SLq = CHUNK * ((chA + NSLICE - 1) / NSLICE);
    const uint64_t qtot = static_cast<uint64_t>(G.SLq) + CHUNK * ((chC + NSLICE - 1) / NSLICE);
    // LDS blocks: slice-major x (each slice one contiguous range), byte offsets of x below
    // 2^31 (buffer loads), blocks inside the class-A part of every slice
    G.H = HOT_MAX;
    G.nlds = 0;
    if (g->sm && g->X < (1ull << 28) && T.hot_lds > 0) {
      G.H = std::min<uint32_t>(HOT_MAX, T.hot_lds) & ~1u;  // even: 16-byte LDS-DMA fills
      // LDS blocks per slice follow the graph: with B = (class-A columns of a slice) / H, the
      // measured optimum on one rank is 1 / 3 / 8 / 20 / 52-64 blocks at R-MAT scale 20 / 22 /
      // 24 / 26 / 28 (B = 3.5 / 13 / 46 / 168 / 610), i.e. 0.41 B^0.77: the hot share worth an
      // LDS fill shrinks slowly as the graph grows (23 % of a slice's columns at scale 22, 9 %
      // at scale 28).  A fixed 20 cost 25 % at scale 22 and 13 % at scale 28.  A rank of p >= 4
      // takes 0.6 x that: its share of every phase shrinks with p while the per-phase cost
      // stays (scale 26 at 8 ranks: flat from 10 to 15 blocks, 6 and 8 lose 3-7 %; at 4 ranks
      // flat from 12 to 20; scale 28 at 8 ranks: 34 against 12); two ranks keep the single-rank
      // count (scale 26: 19-24 blocks 2.81-2.90 ms for both shares, 15 blocks 3.02, 11 2.95).
      // Cold segments widen until the row launch's stream table holds every (slice, segment).
      int want = nlds_env;
      if (want < 0) {
        const double f = p >= 4 ? 0.6 : 1.0;
        want = static_cast<int>(0.41 * f * std::pow(static_cast<double>(g->SL) / G.H, 0.77) + 0.5);
        want = std::max(1, want);
      }
      T.nlds = std::max(0, std::min(64, want));
      G.nlds = std::min<uint32_t>(static_cast<uint32_t>(T.nlds), g->SL / G.H);
    }
    g->nlds = G.nlds;
    g->hot_h = G.H;
    G.S = T.seg;
    G.QL = T.qh;
    const uint64_t ql = static_cast<uint64_t>(G.nlds) * G.H;
    const uint64_t rest = qtot > ql + G.QL ? qtot - ql - G.QL : 0;
    if (!getenv("PR_SEG"))  // (an explicit PR_SEG is taken as given and checked below)
      while (NSLICE * (G.nlds + 1u + (rest + G.S - 1) / G.S) > static_cast<uint64_t>(MAX_NS) && G.S < (1u << 30))
        G.S *= 2;
    T.seg = G.S;
    g->nseg = G.nlds + 1u + static_cast<uint32_t>((rest + G.S - 1) / G.S);
    G.qb = bits_for(std::max({G.H, G.QL, G.S}));
    G.rb = bits_for(std::max<uint64_t>(lrows, 2));
    G.sgb = bits_for(std::max<uint64_t>(g->nseg, 2));
  }
  const int key_bits = 3 + G.sgb + G.rb + G.qb;
  if (key_bits > 64) {
    if (err) *err = "stream keys need more than 64 bits (raise PR_SEG)";
    return PR_E_ARG;
  }
  const uint32_t NG = NSLICE * (G.nlds + 1);

  span.next("prmi:build:stream keys + sort");
  // ---- local edges: stream keys, stable radix sort -------------------------------------------
  uint64_t* lk_in = uniq == kA ? kB : kA;  // free buffer
  unsigned long long* d_cnt = nullptr;     // [0] local edges [1] unused [2..] group starts
  TRY(dmalloc(&d_cnt, 2 + NG, err));
  HIPTRY(hipMemsetAsync(d_cnt, 0, 16, s));
  HIPTRY(hipMemsetAsync(d_cnt + 2, 0xFF, 8ull * NG, s));
  if (nnz) hipLaunchKernelGGL(k_stream_keys, dim3(grid_loop(nnz)), dim3(BLOCK), 0, s, uniq, nnz, nb, inv, L, G, lk_in, g->indeg, T.dropdeg, T.keepdeg);
  if (T.dpull && p == 1 && nnz && lrows) {
    // direct-pull experiment: the column-major row groups of the rows below T.dpull
    span.next("prmi:build:direct-pull rows");
    unsigned* hc = nullptr;
    TRY(dmalloc(&hc, 2, err));
    HIPTRY(hipMemsetAsync(hc, 0, 8, s));
    if (g->lA) hipLaunchKernelGGL(k_count_ge, dim3(grid_for(g->lA)), dim3(BLOCK), 0, s, g->perm, g->indeg, 0u, g->lA, L, T.dpull, hc);
    if (lrows > g->lA) hipLaunchKernelGGL(k_count_ge, dim3(grid_for(lrows - g->lA)), dim3(BLOCK), 0, s, g->perm, g->indeg, g->lA, lrows, L, T.dpull, hc + 1);
    unsigned nge[2] = {0, 0};
    HIPTRY(hipMemcpyAsync(nge, hc, 8, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(hc);
    const DpGeo D{nge[0], g->lA, g->lA + nge[1], lrows};
    const uint32_t ndp = (D.lA - D.lAdp) + (D.lrows - D.lBdp), ngr = (ndp + 63) / 64;
    if (ndp) {
      uint32_t *deg = nullptr, *rowstart = nullptr, *gw = nullptr;
      TRY(dmalloc(&deg, ndp + 1ull, err));
      TRY(dmalloc(&rowstart, ndp + 1ull, err));
      TRY(dmalloc(&gw, ngr + 1ull, err));
      TRY(dmalloc(&g->dp_gbase, ngr + 1ull, err));
      HIPTRY(hipMemsetAsync(deg, 0, 4ull * (ndp + 1), s));
      HIPTRY(hipMemsetAsync(gw, 0, 4ull * (ngr + 1), s));
      hipLaunchKernelGGL(k_dp_deg, dim3(grid_for(ndp)), dim3(BLOCK), 0, s, g->perm, g->indeg, D, L, ndp, deg, gw);
      size_t tb = 0;
      HIPTRY(rocprim::exclusive_scan(nullptr, tb, deg, rowstart, 0u, ndp + 1ull, rocprim::plus<uint32_t>(), s));
      TRY(tmp.ensure(tb, err));
      HIPTRY(rocprim::exclusive_scan(tmp.p, tb, deg, rowstart, 0u, ndp + 1ull, rocprim::plus<uint32_t>(), s));
      HIPTRY(rocprim::exclusive_scan(nullptr, tb, gw, g->dp_gbase, 0u, ngr + 1ull, rocprim::plus<uint32_t>(), s));
      TRY(tmp.ensure(tb, err));
      HIPTRY(rocprim::exclusive_scan(tmp.p, tb, gw, g->dp_gbase, 0u, ngr + 1ull, rocprim::plus<uint32_t>(), s));
      uint32_t ne = 0, nell = 0;
      HIPTRY(hipMemcpyAsync(&ne, rowstart + ndp, 4, hipMemcpyDeviceToHost, s));
      HIPTRY(hipMemcpyAsync(&nell, g->dp_gbase + ngr, 4, hipMemcpyDeviceToHost, s));
      HIPTRY(hipStreamSynchronize(s));
      uint64_t *dk = nullptr, *dk2 = nullptr;
      unsigned long long* dc = nullptr;
      TRY(dmalloc(&dk, ne, err));
      TRY(dmalloc(&dk2, ne, err));
      TRY(dmalloc(&dc, 1, err));
      HIPTRY(hipMemsetAsync(dc, 0, 8, s));
      hipLaunchKernelGGL(k_dp_keys, dim3(grid_loop(nnz)), dim3(BLOCK), 0, s, uniq, nnz, nb, inv, g->indeg, L, D, T.dpull, dk, dc);
      unsigned long long got = 0;
      HIPTRY(hipMemcpyAsync(&got, dc, 8, hipMemcpyDeviceToHost, s));
      HIPTRY(hipStreamSynchronize(s));
      (void)hipFree(dc);
      if (got != ne) {
        if (err) *err = "direct-pull rows: edge count mismatch";
        return PR_E_HIP;
      }
      rocprim::double_buffer<uint64_t> db(dk, dk2);
      HIPTRY(rocprim::radix_sort_keys(nullptr, tb, db, ne, 0, 64, s));
      TRY(tmp.ensure(tb, err));
      if (ne) HIPTRY(rocprim::radix_sort_keys(tmp.p, tb, db, ne, 0, 64, s));
      TRY(dmalloc(&g->dp_ell, nell, err));
      TRY(dmalloc(&g->dp_out, 64ull * ngr, err));
      HIPTRY(hipMemsetAsync(g->dp_ell, 0xFF, 4ull * std::max<uint32_t>(nell, 1), s));
      if (ne) hipLaunchKernelGGL(k_dp_fill, dim3(grid_loop(ne)), dim3(BLOCK), 0, s, db.current(), ne, rowstart, g->dp_gbase, g->dp_ell);
      HIPTRY(hipStreamSynchronize(s));
      HIPTRY(hipGetLastError());
      (void)hipFree(dk);
      (void)hipFree(dk2);
      (void)hipFree(deg);
      (void)hipFree(rowstart);
      (void)hipFree(gw);
      g->dp_groups = ngr;
      fprintf(stderr, "[prmi355x] direct-pull experiment: in-degree < %u: %u rows (%u class A, %u class B), %u edges, %u column slots (%.1f %% padding)\n",
              T.dpull, ndp, D.lA - D.lAdp, D.lrows - D.lBdp, ne, nell, nell ? 100.0 * (nell - ne) / nell : 0.0);
    }
  }
  if (p > 1 && g->maxA) {  // sparse x' exchange: the cross-rank entries (host bitmaps)
    const uint64_t words = (static_cast<uint64_t>(p) * g->maxA + 31) / 32;
    uint32_t *sb = nullptr, *rb = nullptr;
    TRY(dmalloc(&sb, words, err));
    TRY(dmalloc(&rb, words, err));
    HIPTRY(hipMemsetAsync(sb, 0, 4 * words, s));
    HIPTRY(hipMemsetAsync(rb, 0, 4 * words, s));
    if (nnz) hipLaunchKernelGGL(k_sx_bits, dim3(grid_loop(nnz)), dim3(BLOCK), 0, s, uniq, nnz, nb, inv, L, sb, rb);
    g->sx_send.resize(words);
    g->sx_recv.resize(words);
    HIPTRY(hipMemcpyAsync(g->sx_send.data(), sb, 4 * words, hipMemcpyDeviceToHost, s));
    HIPTRY(hipMemcpyAsync(g->sx_recv.data(), rb, 4 * words, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(sb);
    (void)hipFree(rb);
  }
  uint64_t lnnz = nnz;
  uint64_t* lk_alt = uniq;  // the unique keys are dead from here: sort scratch
  if ((p > 1 || T.dropdeg || T.keepdeg) && nnz) {  // keep this rank's rows' edges (order-preserving select)
    size_t tb = 0;
    HIPTRY(rocprim::select(nullptr, tb, lk_in, uniq, d_cnt, nnz, NotDropped(), s));
    TRY(tmp.ensure(tb, err));
    HIPTRY(rocprim::select(tmp.p, tb, lk_in, uniq, d_cnt, nnz, NotDropped(), s));
    HIPTRY(hipMemcpyAsync(&lnnz, d_cnt, 8, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    lk_alt = lk_in;
    lk_in = uniq;
  }
  g->lnnz = lnnz;
  uint64_t* lk = nullptr;
  {
    rocprim::double_buffer<uint64_t> db(lk_in, lk_alt);
    size_t tb = 0;
    HIPTRY(rocprim::radix_sort_keys(nullptr, tb, db, lnnz, 0, key_bits, s));
    TRY(tmp.ensure(tb, err));
    if (lnnz) HIPTRY(rocprim::radix_sort_keys(tmp.p, tb, db, lnnz, 0, key_bits, s));
    lk = db.current();
  }
  if (lnnz) hipLaunchKernelGGL(k_group_starts, dim3(grid_loop(lnnz)), dim3(BLOCK), 0, s, lk, lnnz, G, d_cnt + 2);
  std::vector<unsigned long long> hst(NG);
  HIPTRY(hipMemcpyAsync(hst.data(), d_cnt + 2, 8ull * NG, hipMemcpyDeviceToHost, s));
  HIPTRY(hipStreamSynchronize(s));
  g->gstart.assign(NG + 1, lnnz);
  for (int i = static_cast<int>(NG) - 1; i >= 0; --i) g->gstart[i] = std::min<uint64_t>(hst[i], g->gstart[i + 1]);
  g->gtask.assign(NG + 1, 0);
  uint64_t tasks = 0;
  for (uint32_t i = 0; i < NG; ++i) {
    g->gtask[i] = static_cast<uint32_t>(tasks);
    tasks += (g->gstart[i + 1] - g->gstart[i] + TASK - 1) / TASK;
    if (tasks > 0xFFFFFFF0ull) {
      if (err) *err = "too many stream tasks";
      return PR_E_ARG;
    }
  }
  g->gtask[NG] = static_cast<uint32_t>(tasks);
  g->ntask = static_cast<uint32_t>(tasks);
  {
    // Split point of each slice's L2 group for the two-part stream launch (p > 1): tasks
    // before l2split[j] hold only L2-hot-range edges (x positions inside the hot prefix); the
    // task that holds the first cold-segment edge and everything behind it need the whole x.
    uint64_t* d_idx = nullptr;
    TRY(dmalloc(&d_idx, NSLICE, err));
    uint64_t hidx[NSLICE];
    hipLaunchKernelGGL(k_cold_start, dim3(1), dim3(64), 0, s, lk, lnnz, G, d_idx);
    HIPTRY(hipMemcpyAsync(hidx, d_idx, 8ull * NSLICE, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(d_idx);
    for (uint32_t j = 0; j < NSLICE; ++j) {
      const uint32_t l2g = j * (G.nlds + 1) + G.nlds;
      const uint64_t a = g->gstart[l2g], b = g->gstart[l2g + 1];
      const uint64_t i = std::min(std::max(hidx[j], a), b);
      g->l2split[j] = i >= b ? g->gtask[l2g + 1] : g->gtask[l2g] + static_cast<uint32_t>((i - a) / TASK);
    }
  }
  g->stream_len = tasks * TASK;
  TRY(dmalloc(&g->d_gtask, NG + 1ull, err));
  TRY(dmalloc(&g->d_gstart, NG + 1ull, err));
  HIPTRY(hipMemcpyAsync(g->d_gtask, g->gtask.data(), 4ull * (NG + 1), hipMemcpyHostToDevice, s));
  HIPTRY(hipMemcpyAsync(g->d_gstart, g->gstart.data(), 8ull * (NG + 1), hipMemcpyHostToDevice, s));

  span.next("prmi:build:stream arrays");
  // ---- stream arrays: columns (u16 for LDS groups, u32 for the L2 group), flags, pieces --------
  {
    g->gbase.assign(NG + 1, 0);
    uint64_t n16 = 0, n32 = 0;
    for (uint32_t i = 0; i < NG; ++i) {
      const uint64_t len = static_cast<uint64_t>(g->gtask[i + 1] - g->gtask[i]) * TASK;
      const bool lds_group = (i % (G.nlds + 1)) < G.nlds;
      g->gbase[i] = lds_group ? n16 : n32;
      (lds_group ? n16 : n32) += len;
    }
    g->n_col16 = n16;
    g->n_col32 = n32;
  }
  TRY(dmalloc(&g->d_gbase, NG + 1ull, err));
  HIPTRY(hipMemcpyAsync(g->d_gbase, g->gbase.data(), 8ull * (NG + 1), hipMemcpyHostToDevice, s));
  TRY(dmalloc(&g->col, g->n_col32, err));
  TRY(dmalloc(&g->col16, g->n_col16, err));
  TRY(dmalloc(&g->bits, g->stream_len / EPL + 2, err));
  HIPTRY(hipMemsetAsync(g->col, 0xFF, 4 * std::max<uint64_t>(g->n_col32, 1), s));  // PAD_COL
  if (g->n_col16) hipLaunchKernelGGL(k_fill_u16, dim3(grid_loop(g->n_col16)), dim3(BLOCK), 0, s, g->col16, g->n_col16, static_cast<uint16_t>(G.H));  // zero slot
  HIPTRY(hipMemsetAsync(g->bits, 0, 2 * (g->stream_len / EPL + 2), s));
  uint32_t* bits32 = reinterpret_cast<uint32_t*>(g->bits);
  if (lnnz) hipLaunchKernelGGL(k_stream_fill, dim3(grid_loop(lnnz)), dim3(BLOCK), 0, s, lk, lnnz, L, G, g->d_gstart, g->d_gbase, g->col, g->col16);
  unsigned long long* d_npair = nullptr;
  TRY(dmalloc(&d_npair, NPAIR_SHARDS, err));
  HIPTRY(hipMemsetAsync(d_npair, 0, 8ull * NPAIR_SHARDS, s));
  if (g->stream_len) hipLaunchKernelGGL(k_stream_bits, dim3(grid_loop(g->stream_len / 32)), dim3(BLOCK), 0, s, lk, g->d_gstart, g->d_gtask, NG, g->stream_len / 32, G.qb, bits32, d_npair);
  TRY(dmalloc(&g->task_piece, tasks + 1ull, err));
  {
    uint32_t* tcnt = nullptr;
    TRY(dmalloc(&tcnt, tasks + 1ull, err));
    hipLaunchKernelGGL(k_task_count, dim3(grid_for(tasks + 1ull)), dim3(BLOCK), 0, s, bits32, g->ntask, tcnt);
    size_t tb = 0;
    HIPTRY(rocprim::exclusive_scan(nullptr, tb, tcnt, g->task_piece, 0u, tasks + 1ull, rocprim::plus<uint32_t>(), s));
    TRY(tmp.ensure(tb, err));
    HIPTRY(rocprim::exclusive_scan(tmp.p, tb, tcnt, g->task_piece, 0u, tasks + 1ull, rocprim::plus<uint32_t>(), s));
    uint32_t np = 0;
    std::vector<unsigned long long> hp(NPAIR_SHARDS);
    HIPTRY(hipMemcpyAsync(&np, g->task_piece + tasks, 4, hipMemcpyDeviceToHost, s));
    HIPTRY(hipMemcpyAsync(hp.data(), d_npair, 8ull * NPAIR_SHARDS, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(tcnt);
    (void)hipFree(d_npair);
    g->n_pieces = np;
    g->n_pairs = 0;
    for (unsigned long long v : hp) g->n_pairs += v;
    // pieces <= pairs + tasks (a task boundary cuts at most one pair); piece indices are u32
    if (g->n_pairs + tasks > 0xFFFFFFFFull) {
      if (err) *err = "too many pieces for one rank (use more ranks)";
      return PR_E_ARG;
    }
  }
  const uint64_t NP = g->n_pieces;
  span.next("prmi:build:row maps");
  // ---- row launch: row blocks, per-piece row offsets, run table ------------------------------
  RowBlocks RBk{};
  const uint32_t rbs = T.rb;
  RBk.lA = g->lA;
  RBk.rb = rbs;
  RBk.rbH = std::min(T.rb_heavy, rbs);
  RBk.nbH = RBk.lH = 0;
  if (T.heavy_deg && g->lA) {
    unsigned* hc = nullptr;
    TRY(dmalloc(&hc, 1, err));
    HIPTRY(hipMemsetAsync(hc, 0, 4, s));
    hipLaunchKernelGGL(k_count_heavy, dim3(grid_for(g->lA)), dim3(BLOCK), 0, s, g->perm, g->indeg, g->lA, L, T.heavy_deg, hc);
    unsigned nh = 0;
    HIPTRY(hipMemcpyAsync(&nh, hc, 4, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(hc);
    RBk.nbH = (nh + RBk.rbH - 1) / RBk.rbH;
    RBk.lH = std::min(RBk.nbH * RBk.rbH, g->lA);
  }
  RBk.nbA = RBk.nbH + (g->lA - RBk.lH + rbs - 1) / rbs;
  RBk.NB = RBk.nbA + (lrows - g->lA + rbs - 1) / rbs;
  g->row_rb = rbs;
  g->row_nbH = RBk.nbH;
  g->row_rbH = RBk.rbH;
  g->row_lH = RBk.lH;
  RBk.NS = NSLICE * g->nseg;
  if (RBk.NS > static_cast<uint32_t>(MAX_NS)) {
    if (err) *err = "too many stream segments for the row launch (raise PR_SEG)";
    return PR_E_ARG;
  }
  g->nb_rows = RBk.NB;
  g->nb_rows_a = RBk.nbA;
  g->n_streams = RBk.NS;
  {
    uint32_t *prow = nullptr, *pstream = nullptr, *sst = nullptr;
    TRY(dmalloc(&prow, NP, err));
    TRY(dmalloc(&pstream, NP, err));
    TRY(dmalloc(&sst, RBk.NS, err));
    TRY(dmalloc(&g->roff, NP, err));
    const uint64_t tn = (RBk.NB + 1ull) * RBk.NS;
    TRY(dmalloc(&g->runs, tn, err));
    HIPTRY(hipMemsetAsync(g->runs, 0xFF, 4 * tn, s));
    HIPTRY(hipMemsetAsync(sst, 0xFF, 4ull * RBk.NS, s));
    if (lnnz) hipLaunchKernelGGL(k_piece_rows, dim3(grid_loop(lnnz)), dim3(BLOCK), 0, s, lk, lnnz, G, g->nseg, g->d_gstart, g->d_gtask, bits32, g->task_piece, prow, pstream);
    if (NP) hipLaunchKernelGGL(k_runs, dim3(grid_loop(NP)), dim3(BLOCK), 0, s, prow, pstream, NP, RBk, g->roff, g->runs, sst);
    if (env_int("PR_PIECE_STATS", 0) && lrows) {
      uint32_t* rowcnt = nullptr;
      unsigned long long *hist = nullptr, *rows = nullptr;
      TRY(dmalloc(&rowcnt, lrows, err));
      TRY(dmalloc(&hist, PS_BINS * 6, err));
      TRY(dmalloc(&rows, PS_BINS, err));
      HIPTRY(hipMemsetAsync(rowcnt, 0, 4ull * lrows, s));
      HIPTRY(hipMemsetAsync(hist, 0, 8ull * PS_BINS * 6, s));
      HIPTRY(hipMemsetAsync(rows, 0, 8ull * PS_BINS, s));
      if (lnnz) hipLaunchKernelGGL(k_ps_edges, dim3(grid_loop(lnnz)), dim3(BLOCK), 0, s, lk, lnnz, G, rowcnt);
      if (NP) hipLaunchKernelGGL(k_ps_pieces, dim3(grid_loop(NP)), dim3(BLOCK), 0, s, prow, pstream, NP, g->nseg, g->nlds, rowcnt, hist);
      if (lnnz) hipLaunchKernelGGL(k_ps_edge_kinds, dim3(grid_loop(lnnz)), dim3(BLOCK), 0, s, lk, lnnz, G, g->nlds, rowcnt, hist, rows);
      hipLaunchKernelGGL(k_ps_rows, dim3(grid_for(lrows)), dim3(BLOCK), 0, s, rowcnt, lrows, rows);
      std::vector<unsigned long long> hh(PS_BINS * 6), hr(PS_BINS);
      HIPTRY(hipMemcpyAsync(hh.data(), hist, 8ull * PS_BINS * 6, hipMemcpyDeviceToHost, s));
      HIPTRY(hipMemcpyAsync(hr.data(), rows, 8ull * PS_BINS, hipMemcpyDeviceToHost, s));
      HIPTRY(hipStreamSynchronize(s));
      (void)hipFree(rowcnt);
      (void)hipFree(hist);
      (void)hipFree(rows);
      fprintf(stderr, "[piece stats] rank %d: local in-degree bin, rows, edges, pieces, pieces/edge; "
              "by segment kind LDS / L2-hot / cold: edges, pieces\n", rank);
      for (int b = 0; b < PS_BINS; ++b) {
        if (!hr[b]) continue;
        unsigned long long e = 0, pc = 0;
        for (int k = 0; k < 3; ++k) { pc += hh[b * 6 + k * 2]; e += hh[b * 6 + k * 2 + 1]; }
        fprintf(stderr, "[piece stats] deg [%u, %u) rows %llu edges %llu pieces %llu p/e %.3f | "
                "LDS %llu %llu | hot %llu %llu | cold %llu %llu\n",
                1u << b, b >= 31 ? 0xFFFFFFFFu : (2u << b), hr[b], e, pc, e ? double(pc) / e : 0.0,
                hh[b * 6 + 1], hh[b * 6 + 0], hh[b * 6 + 3], hh[b * 6 + 2], hh[b * 6 + 5], hh[b * 6 + 4]);
      }
      // pieces per task, LDS-block tasks vs L2-group tasks: the stream launch stages a task's
      // pieces through a 256-piece window, one pass per started window
      std::vector<uint32_t> tp(g->ntask + 1);
      HIPTRY(hipMemcpyAsync(tp.data(), g->task_piece, 4ull * tp.size(), hipMemcpyDeviceToHost, s));
      HIPTRY(hipStreamSynchronize(s));
      const uint32_t ngs = g->nlds + 1;
      for (int kind = 0; kind < 2; ++kind) {
        unsigned long long hist8[9] = {0}, nt = 0, np = 0, passes = 0;
        for (int j = 0; j < NSLICE; ++j)
          for (uint32_t gi = kind ? g->nlds : 0; gi < (kind ? ngs : g->nlds); ++gi)
            for (uint32_t t = g->gtask[j * ngs + gi]; t < g->gtask[j * ngs + gi + 1]; ++t) {
              const uint32_t c = tp[t + 1] - tp[t];
              ++hist8[std::min(c / 128u, 8u)];
              ++nt;
              np += c;
              passes += (c + 255u) / 256u;
            }
        fprintf(stderr, "[piece stats] %s tasks %llu pieces/task %.1f staging passes/task %.2f | "
                "by 128-piece bucket:", kind ? "L2" : "LDS", nt, nt ? double(np) / nt : 0.0,
                nt ? double(passes) / nt : 0.0);
        for (int q = 0; q < 9; ++q) fprintf(stderr, " %llu", hist8[q]);
        fprintf(stderr, "\n");
      }
    }
    // fill the empty runs: T[NB][k] = end of stream k, T[b][k] = T[b+1][k] where empty
    std::vector<uint32_t> hT(tn), hs(RBk.NS);
    HIPTRY(hipMemcpyAsync(hT.data(), g->runs, 4 * tn, hipMemcpyDeviceToHost, s));
    HIPTRY(hipMemcpyAsync(hs.data(), sst, 4ull * RBk.NS, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    const uint32_t NSs = RBk.NS;
    std::vector<uint32_t> send(NSs);
    uint32_t nxt = static_cast<uint32_t>(NP);
    for (int k = static_cast<int>(NSs) - 1; k >= 0; --k) {
      send[k] = nxt;
      if (hs[k] != 0xFFFFFFFFu) nxt = hs[k];
    }
    for (uint32_t k = 0; k < NSs; ++k) {
      hT[static_cast<uint64_t>(RBk.NB) * NSs + k] = send[k];
      for (int bb = static_cast<int>(RBk.NB) - 1; bb >= 0; --bb) {
        uint32_t& v = hT[static_cast<uint64_t>(bb) * NSs + k];
        if (v == 0xFFFFFFFFu) v = hT[static_cast<uint64_t>(bb + 1) * NSs + k];
      }
    }
    HIPTRY(hipMemcpyAsync(g->runs, hT.data(), 4 * tn, hipMemcpyHostToDevice, s));
    // row-launch maps (see RowArgs): per block the non-empty runs (start - pre), the piece
    // count, and per 64-piece line the run of its first piece + the run-start mask
    {
      const uint32_t NB = RBk.NB;
      std::vector<uint32_t> hne, hneoff(NB + 1), hloff(NB + 1), htot(NB);
      std::vector<uint32_t> hlf;
      std::vector<uint64_t> hlm;
      std::vector<uint32_t> pre_q;  // per block: pre of each non-empty run
      uint64_t lines = 0;
      for (uint32_t bb = 0; bb < NB; ++bb) {
        hneoff[bb] = static_cast<uint32_t>(hne.size());
        hloff[bb] = static_cast<uint32_t>(lines);
        pre_q.clear();
        uint32_t pre = 0;
        for (uint32_t k = 0; k < NSs; ++k) {
          const uint32_t st0 = hT[static_cast<uint64_t>(bb) * NSs + k];
          const uint32_t len = hT[static_cast<uint64_t>(bb + 1) * NSs + k] - st0;
          if (!len) continue;
          hne.push_back(st0 - pre);
          pre_q.push_back(pre);
          pre += len;
        }
        htot[bb] = pre;
        const uint32_t nl = (pre + 63) / 64;
        uint32_t q = 0;
        for (uint32_t L = 0; L < nl; ++L) {
          const uint32_t i0 = L * 64;
          while (q + 1 < pre_q.size() && pre_q[q + 1] <= i0) ++q;
          uint64_t m = 0;
          for (uint32_t r = q + 1; r < pre_q.size() && pre_q[r] < i0 + 64; ++r) m |= 1ull << (pre_q[r] - i0);
          hlf.push_back(static_cast<uint32_t>(q));
          hlm.push_back(m);
        }
        lines += nl;
        if (lines > 0xFFFFFFF0ull) {
          if (err) *err = "too many row-launch lines";
          return PR_E_ARG;
        }
      }
      hneoff[NB] = static_cast<uint32_t>(hne.size());
      hloff[NB] = static_cast<uint32_t>(lines);
      g->n_lines = lines;
      g->n_runs = hne.size();
      TRY(dmalloc(&g->nebase, hne.size(), err));
      TRY(dmalloc(&g->ne_off, NB + 1ull, err));
      TRY(dmalloc(&g->l_off, NB + 1ull, err));
      TRY(dmalloc(&g->btot, NB, err));
      TRY(dmalloc(&g->lfirst, lines + 2 * EPR, err));  // + the row launch's read-ahead
      TRY(dmalloc(&g->lmask, lines + 2 * EPR, err));
      HIPTRY(hipMemsetAsync(g->lfirst, 0, 4ull * (lines + 2 * EPR), s));
      HIPTRY(hipMemsetAsync(g->lmask, 0, 8ull * (lines + 2 * EPR), s));
      if (!hne.empty()) HIPTRY(hipMemcpyAsync(g->nebase, hne.data(), 4 * hne.size(), hipMemcpyHostToDevice, s));
      HIPTRY(hipMemcpyAsync(g->ne_off, hneoff.data(), 4ull * (NB + 1), hipMemcpyHostToDevice, s));
      HIPTRY(hipMemcpyAsync(g->l_off, hloff.data(), 4ull * (NB + 1), hipMemcpyHostToDevice, s));
      if (NB) HIPTRY(hipMemcpyAsync(g->btot, htot.data(), 4ull * NB, hipMemcpyHostToDevice, s));
      if (lines) {
        HIPTRY(hipMemcpyAsync(g->lfirst, hlf.data(), 4 * lines, hipMemcpyHostToDevice, s));
        HIPTRY(hipMemcpyAsync(g->lmask, hlm.data(), 8 * lines, hipMemcpyHostToDevice, s));
      }
      // 8-line groups per block and the row offsets in row-launch order
      std::vector<uint32_t> hgoff(NB + 1);
      uint64_t groups = 0;
      for (uint32_t bb = 0; bb < NB; ++bb) {
        hgoff[bb] = static_cast<uint32_t>(groups);
        groups += (hloff[bb + 1] - hloff[bb] + EPR - 1) / EPR;
      }
      hgoff[NB] = static_cast<uint32_t>(groups);
      g->n_groups = groups;
      TRY(dmalloc(&g->goff, NB + 1ull, err));
      // 12 bytes per (group, lane); the row launch reads it through a buffer resource with
      // 32-bit offsets
      if (std::max<uint64_t>(groups, 1) * 64 * 12 >= (1ull << 32)) {
        if (err) *err = "row-launch groups exceed the 4 GiB row-offset buffer";
        return PR_E_ARG;
      }
      g->roff16 = env_int("PR_ROFF16", 0) != 0;
      TRY(dmalloc(&g->roffL, std::max<uint64_t>(groups, 1) * 64 * (g->roff16 ? 4 : 3), err));
      HIPTRY(hipMemcpyAsync(g->goff, hgoff.data(), 4ull * (NB + 1), hipMemcpyHostToDevice, s));
      if (NB) hipLaunchKernelGGL(k_roff_lines, dim3(NB), dim3(BLOCK), 0, s, g->roff, g->nebase, g->ne_off, g->l_off, g->btot, g->lfirst, g->lmask, g->goff, g->roffL, g->roff16 ? 1u : 0u);
      HIPTRY(hipGetLastError());
      HIPTRY(hipStreamSynchronize(s));
    }
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(prow);
    (void)hipFree(pstream);
    (void)hipFree(sst);
  }
  HIPTRY(hipGetLastError());
  (void)hipFree(d_cnt);
  (void)hipFree(kA);
  (void)hipFree(kB);
  kA = kB = nullptr;
  (void)hipFree(vid);
  TRY(dmalloc(&g->partial, NP, err));
  // PR_DBG experiments may skip the partial stores: keep every rank defined
  if (T.dbg && NP) hipLaunchKernelGGL(k_fill_f64, dim3(grid_loop(NP)), dim3(BLOCK), 0, s, g->partial, NP, 1.0);

  span.next("prmi:build:iteration buffers");
  // ---- iteration buffers ----------------------------------------------------------------
  TRY(dmalloc(&g->r_loc[0], lrows, err));
  TRY(dmalloc(&g->r_loc[1], lrows, err));
  TRY(dmalloc(&g->r_full, n, err));
  TRY(dmalloc(&g->shards, static_cast<size_t>(NSHARD) * REC_WORDS, err));
  TRY(dmalloc(&g->rec_local, REC_WORDS, err));
  TRY(dmalloc(&g->rec_all, static_cast<size_t>(p) * REC_WORDS, err));
  TRY(dmalloc(&g->state, 1, err));
  TRY(dmalloc(&g->stream_cnt, NSLICE * GCNT, err));
  HIPTRY(hipMemsetAsync(g->stream_cnt, 0, 4ull * NSLICE * GCNT, s));
  HIPTRY(hipMemsetAsync(g->shards, 0, 8ull * NSHARD * REC_WORDS, s));
  HIPTRY(hipMemsetAsync(g->r_loc[0], 0, 8ull * (lrows ? lrows : 1), s));
  HIPTRY(hipMemsetAsync(g->r_loc[1], 0, 8ull * (lrows ? lrows : 1), s));
  HIPTRY(hipStreamSynchronize(s));
  HIPTRY(hipGetLastError());
  g->built = true;
  span.next("prmi:build:placement");
  (void)dev_tune_placement(g, s);
  g->ms_build = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return PR_OK;
}

int dev_reset_state(DevGraph* g, hipStream_t s) {
  std::string* err = nullptr;
  IterState st{};
  if (g->seeded) {
    st = g->seed_state;
  } else {
    // :125-135 round 1: W0 dangling entries at r0 each (one exact product), / N_tot
    st.a = g->n_tot ? (static_cast<double>(g->W0) * g->r0) / static_cast<double>(g->n_tot) : 0.0;
    st.dcnt = g->W0;
  }
  HIPTRY(hipMemcpyAsync(g->state, &st, sizeof(st), hipMemcpyHostToDevice, s));
  HIPTRY(hipMemsetAsync(g->shards, 0, 8ull * NSHARD * REC_WORDS, s));
  if (g->stream_cnt) HIPTRY(hipMemsetAsync(g->stream_cnt, 0, 4ull * NSLICE * GCNT, s));
  return PR_OK;
}

double* dev_x_out(DevGraph* g, int t) { return g->xbuf[(t - 1) & 1]; }

// ---- static scratch of the allocation-free run (pr_run_static) ---------------------------
// One file-scope device array per GPU holds everything a round writes besides the graph's own
// x / rank buffers: the per-piece partial sums, the atomic record shards, the round record and
// the round state.  Host code never uses the array's name as an address: dev_static_scratch()
// asks the runtime once per device (hipGetSymbolAddress, that device current) and hands out
// that pointer.
constexpr uint64_t SS_PARTIAL = 0;                                                     // doubles
constexpr uint64_t SS_SHARDS = SS_PARTIAL + 8ull * STATIC_SCRATCH_PIECES;              // u64 shards
constexpr uint64_t SS_REC = SS_SHARDS + 8ull * NSHARD * REC_WORDS;                     // u64 record
constexpr uint64_t SS_STATE = SS_REC + 8ull * REC_WORDS;                               // IterState
constexpr uint64_t SS_BYTES = SS_STATE + 256;
static_assert(sizeof(IterState) <= 256, "IterState outgrew its scratch slot");
static __device__ __align__(256) unsigned char scratch[SS_BYTES];

namespace {
constexpr int SS_MAX_DEV = 64;
void* g_scratch_ptr[SS_MAX_DEV] = {nullptr};

__global__ void k_state_set(IterState* st, IterState v, uint64_t* shards, uint32_t nwords, uint32_t* gcnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *st = v;
  if (i < nwords) shards[i] = 0;
  if (gcnt && i < NSLICE * GCNT) gcnt[i] = 0;
}
}  // namespace

int dev_static_scratch(int device, StaticScratch* out, std::string* err) {
  if (device < 0 || device >= SS_MAX_DEV) {
    if (err) *err = "static scratch: device ordinal out of range";
    return PR_E_ARG;
  }
  if (!g_scratch_ptr[device]) {
    void* ptr = nullptr;
    HIPTRY(hipGetSymbolAddress(&ptr, HIP_SYMBOL(scratch)));  // (the caller made `device` current)
    g_scratch_ptr[device] = ptr;
  }
  unsigned char* b = static_cast<unsigned char*>(g_scratch_ptr[device]);
  out->partial = reinterpret_cast<double*>(b + SS_PARTIAL);
  out->shards = reinterpret_cast<uint64_t*>(b + SS_SHARDS);
  out->rec = reinterpret_cast<uint64_t*>(b + SS_REC);
  out->state = reinterpret_cast<IterState*>(b + SS_STATE);
  out->max_pieces = STATIC_SCRATCH_PIECES;
  return PR_OK;
}

// dev_reset_state with kernels only (no copy from pageable host memory, no memset node): the
// state travels as a kernel argument and the same launch clears the shards.
int dev_reset_state_kernel(DevGraph* g, hipStream_t s) {
  std::string* err = nullptr;
  IterState st{};
  if (g->seeded) {
    st = g->seed_state;
  } else {
    st.a = g->n_tot ? (static_cast<double>(g->W0) * g->r0) / static_cast<double>(g->n_tot) : 0.0;
    st.dcnt = g->W0;
  }
  const uint32_t nw = NSHARD * REC_WORDS;
  hipLaunchKernelGGL(k_state_set, dim3((nw + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, g->state, st, g->shards, nw, g->stream_cnt);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

namespace {

void launch_stream(const DevGraph* g, const StreamArgs& A, hipStream_t s) {
  const size_t lds = 8ull * ((A.nlds ? A.H + 8u : 0u) + (STREAM_BLOCK / 64) * STG);
  // persistent grid: 32 CUs per XCD, one 1024-thread block per CU (the LDS holds one x
  // block + the staging windows); PR_STREAM_WG blocks per CU without LDS blocks
  const int per_cu = A.nlds ? 1 : std::max(1, g->tune.stream_wg);
  // (PR_STREAM_CUS < 32 leaves compute units of every XCD to other kernels, e.g. RCCL's)
  const int cus = A.nlds ? std::max(1, std::min(32, g->tune.stream_cus)) : 32;
  const dim3 gr(NSLICE * cus * per_cu), bl(STREAM_BLOCK);
  static bool attr_set = false;  // allow the >64 KB dynamic LDS request
  if (!attr_set) {
    for (const void* f : {reinterpret_cast<const void*>(&spmv_stream<0, false, false>),
                          reinterpret_cast<const void*>(&spmv_stream<2, false, false>),
                          reinterpret_cast<const void*>(&spmv_stream<2, true, false>),
                          reinterpret_cast<const void*>(&spmv_stream<2, false, true>),
                          reinterpret_cast<const void*>(&spmv_stream<2, true, true>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const bool split = A.l2w && A.nlds, st = A.stamps != nullptr;
  static const int ntc = env_int("PR_NTC", 0);
  static bool nattr = false;
  if (!nattr) {
    for (const void* f : {reinterpret_cast<const void*>(&spmv_stream<2, true, false, 1>),
                          reinterpret_cast<const void*>(&spmv_stream<2, true, false, 3>),
                          reinterpret_cast<const void*>(&spmv_stream<2, true, false, 5>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    nattr = true;
  }
  if (ntc && split && !st && g->tune.nt == 2) {
    if (ntc == 1) hipLaunchKernelGGL((spmv_stream<2, true, false, 1>), gr, bl, lds, s, A);
    else if (ntc == 3) hipLaunchKernelGGL((spmv_stream<2, true, false, 3>), gr, bl, lds, s, A);
    else hipLaunchKernelGGL((spmv_stream<2, true, false, 5>), gr, bl, lds, s, A);
    return;
  }
  // PR_LEAN=0: the earlier instruction stream (A/B switch; both give identical sums)
  const bool lean = g->tune.lean != 0;
  static bool lattr = false;
  if (!lattr) {
    for (const void* f : {reinterpret_cast<const void*>(&spmv_stream<2, true, false, 0, true, 0>),
                          reinterpret_cast<const void*>(&spmv_stream<2, true, false, 0, true, 32>),
                          reinterpret_cast<const void*>(&spmv_stream<2, true, false, 0, true, 8>),
                          reinterpret_cast<const void*>(&spmv_stream<2, true, false, 0, true, EXP_ALL>),
                          reinterpret_cast<const void*>(&spmv_stream<2, true, true, 0, true>),
                          reinterpret_cast<const void*>(&spmv_stream<0, true, false, 0, true>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    lattr = true;
  }
  // what the launch needs of the kernel beyond the plain single-rank form (see EXP)
  const bool want_dyn = A.gcnt != nullptr && (A.dyn0 < A.nlds || A.l2dyn != 0u);
  // (slice-wide claims alone, on an uncut launch, have an instantiation of their own)
  const int feat = (want_dyn && A.early == 0u && A.part == 0u) ? 8
                   : ((want_dyn || A.early != 0u) ? EXP_ALL : (A.part != 0u ? 32 : 0));
  const int exper = g->tune.l2late == 1 ? 1 : (g->tune.l2late == 2 ? 2 : ((g->tune.dbg & (8192 | 16384)) ? 4 : 0));
  // (PR_DBG=16384 runs the PR_DBG=8192 instantiation with its fast path off: that variant
  // carries 22 spilled registers, so its A/B partner must carry them too)
  if (exper && !feat && g->tune.nt == 2 && split && lean && !st) {
    static bool eattr = false;
    if (!eattr) {
      for (const void* f : {reinterpret_cast<const void*>(&spmv_stream<2, true, false, 0, true, 1>),
                            reinterpret_cast<const void*>(&spmv_stream<2, true, false, 0, true, 2>),
                            reinterpret_cast<const void*>(&spmv_stream<2, true, false, 0, true, 4>)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      eattr = true;
    }
    if (exper == 1) hipLaunchKernelGGL((spmv_stream<2, true, false, 0, true, 1>), gr, bl, lds, s, A);
    else if (exper == 2) hipLaunchKernelGGL((spmv_stream<2, true, false, 0, true, 2>), gr, bl, lds, s, A);
    else hipLaunchKernelGGL((spmv_stream<2, true, false, 0, true, 4>), gr, bl, lds, s, A);
    return;
  }
  if (g->tune.nt == 0 && split && lean && !st) hipLaunchKernelGGL((spmv_stream<0, true, false, 0, true>), gr, bl, lds, s, A);
  else if (g->tune.nt != 2) hipLaunchKernelGGL((spmv_stream<0, false, false>), gr, bl, lds, s, A);
  else if (split && st && lean) hipLaunchKernelGGL((spmv_stream<2, true, true, 0, true>), gr, bl, lds, s, A);
  else if (split && lean && feat == EXP_ALL) hipLaunchKernelGGL((spmv_stream<2, true, false, 0, true, EXP_ALL>), gr, bl, lds, s, A);
  else if (split && lean && feat == 32) hipLaunchKernelGGL((spmv_stream<2, true, false, 0, true, 32>), gr, bl, lds, s, A);
  else if (split && lean && feat == 8) hipLaunchKernelGGL((spmv_stream<2, true, false, 0, true, 8>), gr, bl, lds, s, A);
  else if (split && lean) hipLaunchKernelGGL((spmv_stream<2, true, false, 0, true, 0>), gr, bl, lds, s, A);
  else if (split && st) hipLaunchKernelGGL((spmv_stream<2, true, true>), gr, bl, lds, s, A);
  else if (split) hipLaunchKernelGGL((spmv_stream<2, true, false>), gr, bl, lds, s, A);
  else if (st) hipLaunchKernelGGL((spmv_stream<2, false, true>), gr, bl, lds, s, A);
  else hipLaunchKernelGGL((spmv_stream<2, false, false>), gr, bl, lds, s, A);
}

}  // namespace

int dev_round_stream(DevGraph* g, int t, hipStream_t s, hipEvent_t ev0, int part) {
  std::string* err = nullptr;
  const double* x_in = t == 1 ? (g->seeded ? g->x_seed : g->x_init) : g->xbuf[t & 1];
  StreamArgs S{};
  S.col = g->col;
  S.col16 = g->col16;
  S.gbase = g->d_gbase;
  S.bits = g->bits;
  S.task_piece = g->task_piece;
  S.gtask = g->d_gtask;
  S.x_in = x_in;
  S.partial = g->partial;
  for (int j = 0; j < NSLICE; ++j)
    S.hot_base[j] = g->sm ? (j % g->p) * g->maxA + (j / g->p) * g->SL : 0u;
  S.nlds = g->nlds;
  S.H = g->hot_h;
  S.colmask = g->tune.colmask;
  S.l2mode = static_cast<uint32_t>(g->tune.l2mode);
  const bool stamps = t == 1 && part == 0 && !g->no_alloc && getenv("PR_STAMPS") && g->nlds && g->ntask;
  const uint32_t nph = g->nlds + ((g->tune.l2mode == 1 || g->tune.l2w) ? 1u : 0u);
  std::vector<uint64_t> hst;
  uint64_t* dst = nullptr;
  if (stamps) {
    hst.assign(static_cast<size_t>(NSLICE) * 32 * nph * 17, 0);
    HIPTRY(hipMalloc(&dst, 8 * hst.size()));
    HIPTRY(hipMemsetAsync(dst, 0, 8 * hst.size(), s));
  }
  S.stamps = dst;
  S.l2w = static_cast<uint32_t>(g->tune.l2w);
  S.wgdyn = static_cast<uint32_t>(env_int("PR_WGDYN", 1) != 0);
  S.l2late = static_cast<uint32_t>(g->tune.l2late);
  S.gcnt = g->stream_cnt;
  S.l2dyn = static_cast<uint32_t>(env_int("PR_DYNL2", g->tune.dynl2) != 0);
  S.early = static_cast<uint32_t>(env_int("PR_EARLY", g->tune.early) != 0);
  S.dyng = static_cast<uint32_t>(std::max(1, std::min(64, env_int("PR_DYNG", g->tune.dyng))));
  {  // PR_DYNTAIL: percent of the LDS phases that keep fixed shares (100 = every phase)
    const int pct = std::max(0, std::min(100, env_int("PR_DYNTAIL", g->tune.dyntail)));
    S.dyn0 = pct >= 100 ? 0xFFFFFFFFu : (g->nlds * static_cast<uint32_t>(pct) + 99u) / 100u;
  }
  S.part = static_cast<uint32_t>(part);
  // A cut launch: part 1 = the first LDS phases + the L2-hot-range tasks, part 2 = the other
  // phases + the cold-segment tasks, so both parts keep LDS-bound and L2-bound work side by
  // side.  The L2 waves' work splits about 10 : 7 between the hot range and the cold segments
  // (R-MAT scale 26), so part 1 takes 60 % of the phases (PR_XCUT percent).
  uint32_t cut = g->nlds;
  if (part != 0 && g->tune.l2w > 0) {
    const int pct = std::max(1, std::min(100, env_int("PR_XCUT", 60)));
    cut = std::min<uint32_t>(g->nlds, (g->nlds * static_cast<uint32_t>(pct) + 99u) / 100u);
  }
  S.ph_lo = part == 2 ? cut : 0u;
  S.ph_hi = part == 1 ? cut : g->nlds;
  uint64_t l2tasks = 0;
  for (uint32_t j = 0; j < NSLICE; ++j) {
    const uint32_t l2g = j * (g->nlds + 1) + g->nlds;
    S.l2lo[j] = part == 2 ? g->l2split[j] : g->gtask[l2g];
    S.l2hi[j] = part == 1 ? g->l2split[j] : g->gtask[l2g + 1];
    l2tasks += S.l2hi[j] - S.l2lo[j];
  }
  S.dbg = static_cast<uint32_t>(g->tune.dbg);
  S.x_bytes = static_cast<uint32_t>(std::min<uint64_t>(8ull * g->X, 0x7FFFFFFFull));
  if (ev0) HIPTRY(hipEventRecord(ev0, s));
  if (part == 2 ? (l2tasks != 0 || S.ph_lo < S.ph_hi) : g->ntask != 0) launch_stream(g, S, s);
  if (stamps) {  // PR_STAMPS: per-phase time of the stream launch (diagnostics only)
    HIPTRY(hipMemcpyAsync(hst.data(), dst, 8 * hst.size(), hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(dst);
    const uint32_t nwg = NSLICE * static_cast<uint32_t>(std::max(1, std::min(32, g->tune.stream_cus)));
    double prev_end = 0;
    uint64_t t0 = ~0ull;
    for (uint32_t b = 0; b < nwg; ++b) t0 = std::min<uint64_t>(t0, hst[(static_cast<size_t>(b) * nph) * 17]);
    for (uint32_t gi = 0; gi < nph; ++gi) {
      double st_avg = 0, end_avg = 0, end_max = 0, span_avg = 0, wait_avg = 0;
      for (uint32_t b = 0; b < nwg; ++b) {
        const uint64_t* q = &hst[(static_cast<size_t>(b) * nph + gi) * 17];
        uint64_t e = 0;
        for (int w = 1; w <= 16; ++w) e = std::max(e, q[w]);
        // barrier wait: how long the LDS waves that finished early wait for the last one
        double ws = 0;
        int wn = 0;
        for (int w = 1; w <= 16; ++w)
          if (q[w]) { ws += static_cast<double>(e - q[w]); ++wn; }
        wait_avg += wn ? ws / wn * 0.01 : 0.0;
        st_avg += (q[0] - t0) * 0.01;
        end_avg += (e - t0) * 0.01;
        end_max = std::max(end_max, (e - t0) * 0.01);
        span_avg += (e - q[0]) * 0.01;
      }
      st_avg /= nwg; end_avg /= nwg; span_avg /= nwg; wait_avg /= nwg;
      uint64_t lt = 0, l2t = 0;  // tasks of the phase over the 8 slices
      const uint32_t ngs = g->nlds + 1;
      for (int j = 0; j < NSLICE; ++j) {
        const uint32_t l2n = g->gtask[j * ngs + g->nlds + 1] - g->gtask[j * ngs + g->nlds];
        if (gi < g->nlds) {
          lt += g->gtask[j * ngs + gi + 1] - g->gtask[j * ngs + gi];
          if (g->tune.l2mode != 1 && !g->tune.l2w) l2t += (static_cast<uint64_t>(l2n) * (gi + 1)) / g->nlds - (static_cast<uint64_t>(l2n) * gi) / g->nlds;
        } else {
          l2t += l2n;
        }
      }
      fprintf(stderr, "[stamps] phase %2u start %8.1f us  end avg %8.1f max %8.1f  span avg %7.1f  fill+wait %6.1f  wave wait %6.1f  lds tasks %7llu  l2 tasks %7llu\n",
              gi, st_avg, end_avg, end_max, span_avg, st_avg - prev_end, wait_avg, (unsigned long long)lt, (unsigned long long)l2t);
      prev_end = end_avg;
    }
    // per slice (= XCD): tasks and when its workgroups finish (the launch's tail)
    const uint32_t ngs = g->nlds + 1;
    for (int j = 0; j < NSLICE; ++j) {
      double e_avg = 0, e_max = 0, e_min = 1e30;
      int cnt = 0;
      for (uint32_t b = static_cast<uint32_t>(j); b < nwg; b += NSLICE) {
        uint64_t e = 0;
        for (uint32_t gi = 0; gi < nph; ++gi)
          for (int w = 1; w <= 16; ++w) e = std::max(e, hst[(static_cast<size_t>(b) * nph + gi) * 17 + w]);
        const double et = (e - t0) * 0.01;
        e_avg += et; e_max = std::max(e_max, et); e_min = std::min(e_min, et); ++cnt;
      }
      const uint64_t lds_t = g->gtask[j * ngs + g->nlds] - g->gtask[j * ngs];
      const uint64_t l2_t = g->gtask[j * ngs + g->nlds + 1] - g->gtask[j * ngs + g->nlds];
      fprintf(stderr, "[stamps] slice %d: lds tasks %7llu l2 tasks %7llu  workgroup end min %8.1f avg %8.1f max %8.1f us\n",
              j, (unsigned long long)lds_t, (unsigned long long)l2_t, e_min, e_avg / std::max(cnt, 1), e_max);
      if (getenv("PR_STAMPS_WG")) {  // every workgroup of the slice: end of its LDS role / L2 role
        fprintf(stderr, "[stamps] slice %d workgroup ends (lds role | l2 role):", j);
        for (uint32_t b = static_cast<uint32_t>(j); b < nwg; b += NSLICE) {
          uint64_t el = 0, e2 = 0;
          for (uint32_t gi = 0; gi < nph; ++gi)
            for (int w = 1; w <= 16; ++w) {
              const uint64_t v = hst[(static_cast<size_t>(b) * nph + gi) * 17 + w];
              if (gi == g->nlds) e2 = std::max(e2, v); else el = std::max(el, v);
            }
          fprintf(stderr, " %.0f|%.0f", el ? (el - t0) * 0.01 : 0.0, e2 ? (e2 - t0) * 0.01 : 0.0);
        }
        fprintf(stderr, "\n");
      }
    }
  }
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_round_rows(DevGraph* g, int t, int mode, uint32_t b0, uint32_t b1, hipStream_t s) {
  std::string* err = nullptr;
  RowArgs A{};
  A.nebase = g->nebase;
  A.ne_off = g->ne_off;
  A.l_off = g->l_off;
  A.tot = g->btot;
  A.lfirst = g->lfirst;
  A.lmask = g->lmask;
  A.partial = g->partial;
  A.roffL = g->roffL;
  A.roffL_bytes = static_cast<uint32_t>(std::max<uint64_t>(g->n_groups, 1) * 64 * 12);
  A.roff16 = g->roff16 ? 1u : 0u;
  A.goff = g->goff;
  A.dbg = static_cast<uint32_t>(g->tune.dbg);
  A.NS = g->n_streams;
  A.rb = g->row_rb;
  A.nbH = g->row_nbH;
  A.rbH = g->row_rbH;
  A.lH = g->row_lH;
  A.nbA = g->nb_rows_a;
  A.lA = g->lA;
  A.lrows = g->lrows;
  A.meta = g->meta;
  A.x_out = dev_x_out(g, t) + static_cast<uint64_t>(g->rank) * g->maxA;
  A.r_old = t == 1 ? (g->seeded ? g->r_seed : nullptr) : g->r_loc[(t - 1) & 1];
  A.base = g->base;
  A.r0 = g->r0;
  A.r_out = g->r_loc[t & 1];
  A.st = g->state;
  A.shards = g->shards;
  A.p = static_cast<uint32_t>(g->p);
  A.rank = static_cast<uint32_t>(g->rank);
  A.sm = g->sm ? 1u : 0u;
  A.snake = g->snake ? 1u : 0u;
  A.SL = g->SL;
  A.b0 = b0;
  A.xg = std::max(1u, g->tune.rxg);
  A.xfull = (b1 - b0) / (NSLICE * A.xg) * (NSLICE * A.xg);
  if (b1 > b0) {
    const dim3 gr(b1 - b0), bl(BLOCK);
    if (mode == 0) hipLaunchKernelGGL((spmv_rows<0>), gr, bl, 0, s, A);
    else if (mode == 1) hipLaunchKernelGGL((spmv_rows<1>), gr, bl, 0, s, A);
    else hipLaunchKernelGGL((spmv_rows<2>), gr, bl, 0, s, A);
  }
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_round_reduce(DevGraph* g, hipStream_t s, hipEvent_t ev1) {
  std::string* err = nullptr;
  if (ev1) HIPTRY(hipEventRecord(ev1, s));
  hipLaunchKernelGGL(reduce_shards, dim3(1), dim3(BLOCK), 0, s, g->shards, g->rec_local, g->stream_cnt);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_round_compute(DevGraph* g, int t, int mode, hipStream_t s, hipEvent_t ev0,
                      hipEvent_t ev1) {
  int rc = dev_round_stream(g, t, s, ev0, 0);
  if (!rc) rc = dev_round_rows(g, t, mode, 0, g->nb_rows, s);
  if (!rc) rc = dev_round_reduce(g, s, ev1);
  return rc;
}

int dev_round_single(DevGraph* g, int t, int mode, bool tracked, hipStream_t s, hipEvent_t ev0,
                     hipEvent_t ev1) {
  std::string* err = nullptr;
  if (g->p != 1) return PR_E_ARG;
  int rc = dev_round_stream(g, t, s, ev0, 0);
  if (!rc) rc = dev_round_rows(g, t, mode, 0, g->nb_rows, s);
  if (rc) return rc;
  if (g->dp_groups) {  // direct-pull experiment (timing only): inside the SpMV event bracket
    const double* x_in = t == 1 ? (g->seeded ? g->x_seed : g->x_init) : g->xbuf[t & 1];
    hipLaunchKernelGGL(spmv_dpull, dim3((g->dp_groups + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0, s,
                       g->dp_ell, g->dp_gbase, x_in,
                       static_cast<uint32_t>(std::min<uint64_t>(8ull * g->X, 0x7FFFFFFFull)), g->dp_groups, g->dp_out);
    if (t == 1 && getenv("PR_DPULL_CHECK")) {  // the side sums against a host walk of the same slots
      std::vector<uint32_t> gb(g->dp_groups + 1ull);
      HIPTRY(hipMemcpyAsync(gb.data(), g->dp_gbase, 4ull * gb.size(), hipMemcpyDeviceToHost, s));
      HIPTRY(hipStreamSynchronize(s));
      std::vector<uint32_t> ell(std::max<uint32_t>(gb.back(), 1));
      std::vector<double> xs(g->X), out(64ull * g->dp_groups);
      HIPTRY(hipMemcpy(ell.data(), g->dp_ell, 4ull * gb.back(), hipMemcpyDeviceToHost));
      HIPTRY(hipMemcpy(xs.data(), x_in, 8ull * g->X, hipMemcpyDeviceToHost));
      HIPTRY(hipMemcpy(out.data(), g->dp_out, 8ull * out.size(), hipMemcpyDeviceToHost));
      uint64_t bad = 0, nz = 0;
      for (uint32_t gr = 0; gr < g->dp_groups; ++gr)
        for (uint32_t l = 0; l < 64; ++l) {
          double c = 0.0;
          for (uint32_t k = 0; k < (gb[gr + 1] - gb[gr]) / 64; ++k) {
            const uint32_t col = ell[gb[gr] + 64 * k + l];
            c += col == PAD_COL ? 0.0 : xs[col];
          }
          bad += c != out[64ull * gr + l];
          nz += c != 0.0;
        }
      fprintf(stderr, "[dpull check] %u groups, %llu nonzero row sums, %llu mismatches\n", g->dp_groups,
              static_cast<unsigned long long>(nz), static_cast<unsigned long long>(bad));
    }
  }
  if (ev1) HIPTRY(hipEventRecord(ev1, s));
  const uint32_t extra = (t == 1 && !g->seeded) ? g->n - g->R : 0u;  // as dev_round_finalize
  hipLaunchKernelGGL(reduce_finalize, dim3(1), dim3(BLOCK), 0, s, g->shards, g->rec_local, t, g->n_tot, extra,
                     g->r0, tracked ? 1 : 0, g->state, g->stream_cnt);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

// Exchange plan of the chunked x' exchange (p > 1): chunk k covers the slot positions
// [P_{k-1}, P_k) of every slice sub-region of a rank's slot (the same on every rank), and the
// class-A row blocks [b0, b1) that write them on this rank.
int dev_tune_placement(DevGraph* g, hipStream_t s) {
  g->place_tried = 0;
  g->place_ms_first = g->place_ms_best = 0;
  const size_t bytes = 8ull * g->n_pieces;
  const size_t min_bytes = static_cast<size_t>(std::max(1, env_int("PR_PLACE_MIN_MB", 1024))) << 20;
  // (small graphs run from the caches; the PR_DBG timing switches may leave pieces unwritten)
  if (env_int("PR_PLACE", g->tune.place) <= 0 || !g->partial || !g->ntask || !g->nlds || bytes < min_bytes || g->tune.dbg)
    return PR_OK;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return PR_OK;
  const size_t keep = 16ull << 30;  // left alone for the caller
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return PR_OK;
  const bool na = g->no_alloc;
  g->no_alloc = true;  // (no PR_STAMPS dump from these launches)
  // the search may take this long (holding memory means clearing it first: up to 30 ms per GB)
  const auto t_begin = std::chrono::steady_clock::now();
  const double budget_ms = std::max(0, env_int("PR_PLACE_BUDGET_MS", 1600));
  auto spent = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count(); };
  // the stream launch's time with the current array: pairs of launches until three pairs in a
  // row agree to 1 % (memory released just before is still being cleared in the background)
  auto measure = [&](float* out) -> bool {
    float h[3] = {-1.f, -1.f, -1.f};
    for (int it = 0; it < 60; ++it) {
      float ms = 0.f;
      bool ok = hipEventRecord(e0, s) == hipSuccess;
      for (int r = 0; r < 2 && ok; ++r) ok = dev_round_stream(g, 1, s, nullptr, 0) == PR_OK;
      ok = ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
           hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
      if (!ok) return false;
      h[0] = h[1];
      h[1] = h[2];
      h[2] = 0.5f * ms;
      if (h[0] > 0.f) {
        const float lo = std::min(h[0], std::min(h[1], h[2])), hi = std::max(h[0], std::max(h[1], h[2]));
        if (hi <= 1.01f * lo) break;
      }
    }
    *out = std::min(h[2], h[1] > 0.f ? h[1] : h[2]);
    return true;
  };
  // a candidate: `bytes` allocated while other device memory is held, which is released again
  // before the launch is timed.  kind 0: G GB in 1-GB blocks; kind 1: one block of G GB that has
  // been allocated and released once before
  auto candidate = [&](int kind, size_t G, size_t nbytes) -> void* {
    if (fr < keep + nbytes + (G << 30)) return nullptr;
    std::vector<void*> held;
    bool whole = true;
    if (kind == 0) {
      for (size_t i = 0; i < G; ++i) {
        void* b = nullptr;
        if (spent() > budget_ms || hipMalloc(&b, 1ull << 30) != hipSuccess) {
          whole = false;
          break;
        }
        held.push_back(b);
      }
    } else {
      void* b = nullptr;
      if (hipMalloc(&b, G << 30) == hipSuccess) {
        (void)hipFree(b);
        b = nullptr;
        if (hipMalloc(&b, G << 30) == hipSuccess) held.push_back(b);
      }
    }
    void* c = nullptr;
    if (!whole || hipMalloc(&c, nbytes) != hipSuccess) c = nullptr;
    for (void* b : held) (void)hipFree(b);
    (void)hipGetLastError();
    return c;
  };
  struct Plan { int kind; size_t G; };
  // the search for one array: `slot` points at the engine's pointer to it; `copy`: it holds data
  // (the partial array is rewritten by every launch, the column stream is not); a candidate
  // replaces the current placement when it is faster, the search ends when one is faster than
  // `stop` x the first timing
  auto search = [&](void** slot, size_t nbytes, bool copy, float first_ms, float stop, std::initializer_list<Plan> plan) -> float {
    float best_ms = first_ms;
    for (const Plan& pl : plan) {
      if (spent() > budget_ms) break;
      void* c = candidate(pl.kind, pl.G, nbytes);
      if (!c) continue;
      void* prev = *slot;
      if (copy && hipMemcpyAsync(c, prev, nbytes, hipMemcpyDeviceToDevice, s) != hipSuccess) {
        (void)hipFree(c);
        break;
      }
      *slot = c;
      float ms = 0.f;
      const bool ok = measure(&ms);
      ++g->place_tried;
      (void)hipStreamSynchronize(s);
      if (ok && ms < best_ms) {
        (void)hipFree(prev);
        best_ms = ms;
      } else {
        *slot = prev;
        (void)hipFree(c);
      }
      if (env_int("PR_VERBOSE", 0) > 1)
        fprintf(stderr, "[prmi355x] placement kind %d behind %zu GB (%.1f GB array): stream launch %.3f ms\n", pl.kind, pl.G,
                nbytes / 1073741824.0, ms);
      if (!ok || best_ms < stop * first_ms) break;
    }
    return best_ms;
  };
  float first = 0.f, best = 0.f;
  if (measure(&first)) {
    // the partial array: two rates, 7 % apart -- stop at the first candidate that has the fast
    // one (on a box that has run nothing yet that is, most often, the first)
    best = search(reinterpret_cast<void**>(&g->partial), bytes, false, first, 0.955f, {{0, 96}, {0, 64}, {1, 48}});
    // the LDS groups' column stream, the largest array the launch reads: worth 2 % more
    const size_t cbytes = 2ull * g->n_col16;
    if (g->col16 && cbytes >= min_bytes) best = search(reinterpret_cast<void**>(&g->col16), cbytes, true, best, 0.985f, {{0, 96}, {0, 64}});
  }
  (void)hipGetLastError();
  (void)hipStreamSynchronize(s);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  g->no_alloc = na;
  g->place_ms_first = first;
  g->place_ms_best = best;
  if (env_int("PR_VERBOSE", 0))
    fprintf(stderr, "[prmi355x] placement of the partial array and the column stream: stream launch %.3f ms as built, %.3f ms chosen after %d more placements (%.1f of %.1f GB free, %.0f ms)\n",
            first, best, g->place_tried, fr / 1073741824.0, tot / 1073741824.0, spent());
  return PR_OK;
}

bool dev_can_split_stream(const DevGraph* g) {
  // the hot prefix of a slice's q-space is a prefix of every slot sub-region only in the
  // slice-major x layout, and a split needs LDS blocks (the two-role stream kernel)
  return g->p > 1 && g->sm && g->nlds > 0;
}

std::vector<XChunk> dev_exchange_plan(const DevGraph* g, int K, bool hot_first) {
  std::vector<XChunk> out;
  const uint32_t p = static_cast<uint32_t>(g->p);
  const uint32_t nsub = g->sm ? NSLICE / p : 1u;          // sub-regions of a slot
  const uint64_t SLr = g->sm ? g->SL : g->maxA;            // entries per sub-region
  const uint32_t rows_per_pos = g->sm ? nsub : 1u;         // local rows per sub-region position
  K = std::max(1, std::min<int>(K, static_cast<int>(std::max<uint64_t>(SLr / CHUNK, 1))));
  // hot_first: chunk 0 is exactly the hot prefix of every sub-region -- the positions the LDS
  // blocks and the L2-hot range cover, all that the first part of the next round's stream
  // launch reads -- and the other K - 1 chunks share the rest
  uint64_t hot = 0;
  if (hot_first && dev_can_split_stream(g)) {
    hot = static_cast<uint64_t>(g->nlds) * g->hot_h + g->tune.qh;
    hot = std::min<uint64_t>((hot + CHUNK - 1) / CHUNK * CHUNK, SLr);
    if (K < 2 && hot < SLr) K = 2;
  }
  auto block_row0 = [&](uint32_t b) -> uint64_t {
    if (b < g->row_nbH) return static_cast<uint64_t>(b) * g->row_rbH;
    return g->row_lH + static_cast<uint64_t>(b - g->row_nbH) * g->row_rb;
  };
  uint64_t prev = 0;
  uint32_t bprev = 0;
  for (int k = 0; k < K; ++k) {
    uint64_t P = (k == K - 1) ? SLr : ((SLr * (k + 1)) / K) / CHUNK * CHUNK;
    if (hot) P = k == 0 ? hot : (k == K - 1 ? SLr : hot + ((SLr - hot) * k / (K - 1)) / CHUNK * CHUNK);
    if (P < prev) P = prev;
    // local rows below P map below P in every sub-region: l < P * rows_per_pos
    const uint64_t Lrow = P * rows_per_pos;
    uint32_t b1 = bprev;
    if (k == K - 1) b1 = g->nb_rows_a;
    else while (b1 < g->nb_rows_a && block_row0(b1) < Lrow) ++b1;
    XChunk c;
    c.b0 = bprev;
    c.b1 = b1;
    for (uint32_t sub = 0; sub < nsub; ++sub)
      if (P > prev) c.pieces.push_back({sub * SLr + prev, P - prev});
    out.push_back(c);
    prev = P;
    bprev = b1;
  }
  return out;
}

int dev_sx_prepare(DevGraph* g, const std::vector<XChunk>& plan, std::string* err) {
  const uint32_t p = static_cast<uint32_t>(g->p), me = static_cast<uint32_t>(g->rank);
  const int K = static_cast<int>(plan.size());
  uint64_t sig = 0x9E3779B97F4A7C15ull * static_cast<uint64_t>(K);
  for (const XChunk& c : plan)
    for (const XPiece& pc : c.pieces) sig = mix64(sig ^ (pc.off * 0x100000001B3ull + pc.cnt));
  if (g->sx_chunks == K && g->sx_plan_sig == sig) return PR_OK;
  g->sx_chunks = 0;
  if (p < 2 || g->sx_send.empty()) {
    if (err) *err = "sparse exchange: no cross-rank bitmaps (single rank?)";
    return PR_E_ARG;
  }
  for (void* q : {static_cast<void*>(g->sx_spos), static_cast<void*>(g->sx_rpos),
                  static_cast<void*>(g->sx_sbuf), static_cast<void*>(g->sx_rbuf)})
    if (q) (void)hipFree(q);
  g->sx_spos = g->sx_rpos = nullptr;
  g->sx_sbuf = g->sx_rbuf = nullptr;
  auto bit = [](const std::vector<uint32_t>& b, uint64_t i) { return (b[i >> 5] >> (i & 31)) & 1u; };
  std::vector<uint32_t> sp, rp;
  g->sx_so.assign(static_cast<size_t>(K) * p + 1, 0);
  g->sx_ro.assign(static_cast<size_t>(K) * p + 1, 0);
  for (int k = 0; k < K; ++k)
    for (uint32_t q = 0; q < p; ++q) {
      g->sx_so[static_cast<size_t>(k) * p + q] = sp.size();
      g->sx_ro[static_cast<size_t>(k) * p + q] = rp.size();
      if (q == me) continue;
      for (const XPiece& pc : plan[k].pieces)
        for (uint64_t o = pc.off; o < pc.off + pc.cnt && o < g->maxA; ++o) {
          if (bit(g->sx_send, static_cast<uint64_t>(q) * g->maxA + o)) sp.push_back(static_cast<uint32_t>(o));
          const uint64_t xq = static_cast<uint64_t>(q) * g->maxA + o;
          if (bit(g->sx_recv, xq)) rp.push_back(static_cast<uint32_t>(xq));
        }
    }
  g->sx_so.back() = sp.size();
  g->sx_ro.back() = rp.size();
  if (getenv("PR_VERBOSE"))
    fprintf(stderr, "[prmi355x] rank %u sparse x' exchange: sends %zu entries, receives %zu (dense: %llu each way, %.1f %% / %.1f %%)\n",
            me, sp.size(), rp.size(), static_cast<unsigned long long>(p - 1) * g->maxA,
            100.0 * sp.size() / std::max<double>(1.0, static_cast<double>(p - 1) * g->maxA),
            100.0 * rp.size() / std::max<double>(1.0, static_cast<double>(p - 1) * g->maxA));
  if (!sp.empty()) {
    TRY(dmalloc(&g->sx_spos, sp.size(), err));
    TRY(dmalloc(&g->sx_sbuf, sp.size(), err));
    HIPTRY(hipMemcpy(g->sx_spos, sp.data(), 4 * sp.size(), hipMemcpyHostToDevice));
  }
  if (!rp.empty()) {
    TRY(dmalloc(&g->sx_rpos, rp.size(), err));
    TRY(dmalloc(&g->sx_rbuf, rp.size(), err));
    HIPTRY(hipMemcpy(g->sx_rpos, rp.data(), 4 * rp.size(), hipMemcpyHostToDevice));
  }
  g->sx_chunks = K;
  g->sx_plan_sig = sig;
  return PR_OK;
}

int dev_sx_pack(DevGraph* g, int t, int k, hipStream_t s) {
  std::string* err = nullptr;
  const uint64_t a = g->sx_so[static_cast<size_t>(k) * g->p], b = g->sx_so[static_cast<size_t>(k + 1) * g->p];
  if (b > a)
    hipLaunchKernelGGL(k_sx_pack, dim3(static_cast<uint32_t>((b - a + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                       dev_x_out(g, t) + static_cast<uint64_t>(g->rank) * g->maxA, g->sx_spos + a, b - a,
                       g->sx_sbuf + a);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_sx_unpack(DevGraph* g, int t, int k, hipStream_t s) {
  std::string* err = nullptr;
  const uint64_t a = g->sx_ro[static_cast<size_t>(k) * g->p], b = g->sx_ro[static_cast<size_t>(k + 1) * g->p];
  if (b > a)
    hipLaunchKernelGGL(k_sx_unpack, dim3(static_cast<uint32_t>((b - a + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                       dev_x_out(g, t), g->sx_rpos + a, b - a, g->sx_rbuf + a);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_round_finalize(DevGraph* g, int t, bool tracked, hipStream_t s) {
  std::string* err = nullptr;
  const uint64_t* rec = g->p > 1 ? g->rec_all : g->rec_local;
  // round 1 starts from r^0 == 1 on every page: pages that are not rows drop to 0 (|dr|=1)
  // (a seed has no defined page outside the rows: nothing drops).  Every rank finalizes the
  // same p records, so every rank adds the term: all ranks see one global residual and take
  // the same stop decision.
  const uint32_t extra = (t == 1 && !g->seeded) ? g->n - g->R : 0u;
  hipLaunchKernelGGL(finalize_round, dim3(1), dim3(64), 0, s, rec, g->p, t, g->n_tot, extra, g->r0, tracked ? 1 : 0, g->state);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_scatter_ranks(DevGraph* g, int iterations, hipStream_t s) {
  std::string* err = nullptr;
  const uint32_t n = g->n;
  HIPTRY(hipMemsetAsync(g->r_full, 0, 8ull * (n ? n : 1), s));
  if (iterations == 0 && g->seeded) {  // a seeded context that ran no round: the seed
    if (g->lrows) hipLaunchKernelGGL(k_scatter_ranks, dim3(grid_for(g->lrows)), dim3(BLOCK), 0, s, g->perm, static_cast<const double*>(g->r_seed), g->lrows, layout_of(g), g->r_full);
  } else if (iterations == 0) {
    if (g->rank == 0 && n) hipLaunchKernelGGL(k_sources_one, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->outdeg, n, g->r0, g->r_full);
  } else if (g->lrows) {
    hipLaunchKernelGGL(k_scatter_ranks, dim3(grid_for(g->lrows)), dim3(BLOCK), 0, s, g->perm, g->r_loc[iterations & 1], g->lrows, layout_of(g), g->r_full);
  }
  HIPTRY(hipGetLastError());
  return PR_OK;
}

// Host evaluation of the layout functions the kernels use (the same inline code, compiled for
// the host): owner rank, local row and x position of internal vertices.
int host_layout_map(int p, int rank, uint32_t nA, uint32_t nB, uint32_t nC, uint64_t cnt,
                    const uint32_t* k, uint32_t* owner, uint32_t* local, uint64_t* xp,
                    uint64_t dims[4]) {
  if (p < 1 || rank < 0 || rank >= p) return PR_E_ARG;
  if (static_cast<uint64_t>(nA) + nB + nC > 0xFFFFFFFFull) return PR_E_ARG;
  const LayoutDims d = make_layout(p, rank, nA, nB, nC);
  const uint32_t R = nA + nB;
  for (uint64_t i = 0; i < cnt; ++i) {
    const uint32_t v = k[i];
    const bool row = v < R, col = v < nA || (v >= R && v - R < nC);
    if (!row && !col) return PR_E_ARG;  // class-D vertices have neither a row nor an x entry
    if (owner) owner[i] = row ? owner_of(d.L, v) : 0xFFFFFFFFu;
    if (local) local[i] = row ? local_of(d.L, v) : 0xFFFFFFFFu;
    if (xp) xp[i] = col ? xpos(d.L, v) : ~0ull;
  }
  if (dims) {
    dims[0] = d.L.maxA;
    dims[1] = d.X;
    dims[2] = d.lrows;
    dims[3] = d.lA;
  }
  return PR_OK;
}

int dev_seed_state(DevGraph* g, const double* ranks, hipStream_t s, std::string* err) {
  g->seeded = false;
  if (!ranks) return PR_OK;
  const uint32_t n = g->n;
  const Layout L = layout_of(g);
  if (!g->x_seed) TRY(dmalloc(&g->x_seed, g->X, err));
  if (!g->r_seed) TRY(dmalloc(&g->r_seed, g->lrows, err));
  HIPTRY(hipMemsetAsync(g->x_seed, 0, 8ull * (g->X ? g->X : 1), s));
  if (n) HIPTRY(hipMemcpyAsync(g->r_full, ranks, 8ull * n, hipMemcpyHostToDevice, s));
  uint64_t* rec = nullptr;
  IterState* st = nullptr;
  TRY(dmalloc(&rec, REC_WORDS, err));
  if (dmalloc(&st, 1, err) != PR_OK) {
    (void)hipFree(rec);
    return PR_E_OOM;
  }
  struct Free {
    void *a, *b;
    ~Free() { (void)hipFree(a); (void)hipFree(b); }
  } fr{rec, st};
  HIPTRY(hipMemsetAsync(rec, 0, 8ull * REC_WORDS, s));
  HIPTRY(hipMemsetAsync(st, 0, sizeof(IterState), s));
  if (n) {
    hipLaunchKernelGGL(k_x_init, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->perm, g->outdeg, n, L, g->r0, static_cast<const double*>(g->r_full), g->x_seed);
    hipLaunchKernelGGL(k_seed_dangling, dim3(grid_for(n)), dim3(BLOCK), 0, s, static_cast<const double*>(g->r_full), static_cast<const uint32_t*>(g->dang_w), n, rec);
  }
  if (g->lrows) hipLaunchKernelGGL(k_r_seed, dim3(grid_for(g->lrows)), dim3(BLOCK), 0, s, g->perm, static_cast<const double*>(g->r_full), g->lrows, L, g->r_seed);
  // every rank sees the whole seed: the dangling record is complete on each (p = 1 here)
  hipLaunchKernelGGL(finalize_round, dim3(1), dim3(64), 0, s, static_cast<const uint64_t*>(rec), 1, 0, g->n_tot, 0u, g->r0, 0, st);
  HIPTRY(hipGetLastError());
  HIPTRY(hipMemcpyAsync(&g->seed_state, st, sizeof(IterState), hipMemcpyDeviceToHost, s));
  HIPTRY(hipStreamSynchronize(s));
  g->seed_state.iter = 0;
  g->seeded = true;
  return PR_OK;
}

int dev_topk_candidates(DevGraph* g, uint64_t k, std::vector<uint32_t>* ids,
                        std::vector<double>* rs, hipStream_t s, std::string* err) {
  ids->clear();
  rs->clear();
  const uint32_t n = g->n;
  if (k == 0 || n == 0) return PR_OK;
  constexpr uint64_t CAP = 1u << 16;  // stop refining once the boundary digit holds <= CAP
  unsigned long long* hist = nullptr;
  TRY(dmalloc(&hist, 2 * SEL_BINS, err));
  struct Free {
    std::vector<void*> v;
    ~Free() { for (void* p : v) if (p) (void)hipFree(p); }
  } fr;
  fr.v.push_back(hist);
  std::vector<unsigned long long> h(2 * SEL_BINS);
  uint64_t prefix = 0, pmask = 0, need = k, count = 0;  // count: pages with key >= lb
  int top = 64;
  const uint32_t grid = std::min<uint32_t>(grid_for(n), 4096);
  while (top > 0) {
    const int shift = std::max(top - SEL_BITS, 0), width = top - shift;
    const uint32_t dmask = (1u << width) - 1;
    HIPTRY(hipMemsetAsync(hist, 0, 16ull * SEL_BINS, s));
    hipLaunchKernelGGL(k_select_hist, dim3(grid), dim3(BLOCK), 0, s, g->r_full, g->mapw, n,
                       prefix, pmask, shift, dmask, hist);
    HIPTRY(hipGetLastError());
    HIPTRY(hipMemcpyAsync(h.data(), hist, 16ull * SEL_BINS, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
    uint64_t above = 0;
    int d = static_cast<int>(dmask);
    for (; d >= 0; --d) {
      if (above + h[d] >= need) break;
      above += h[d];
      count += h[SEL_BINS + d];
    }
    if (d < 0) break;  // (first pass only) fewer than k weighted pages: take them all
    need -= above;
    prefix |= static_cast<uint64_t>(d) << shift;
    pmask |= static_cast<uint64_t>(dmask) << shift;
    top = shift;
    if (h[d] <= CAP || top == 0) {
      count += h[SEL_BINS + d];
      break;
    }
  }
  const uint64_t lb = std::max<uint64_t>(prefix, 1);
  if (count == 0) return PR_OK;
  if (count > 0xFFFFFFFFull) {
    if (err) *err = "top-K candidate set too large";
    return PR_E_ARG;
  }
  uint32_t* d_ids = nullptr;
  double* d_rs = nullptr;
  unsigned* d_cnt = nullptr;
  TRY(dmalloc(&d_ids, count, err)); fr.v.push_back(d_ids);
  TRY(dmalloc(&d_rs, count, err)); fr.v.push_back(d_rs);
  TRY(dmalloc(&d_cnt, 1, err)); fr.v.push_back(d_cnt);
  HIPTRY(hipMemsetAsync(d_cnt, 0, 4, s));
  hipLaunchKernelGGL(k_select_emit, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->r_full, g->mapw, n,
                     lb, d_ids, d_rs, d_cnt, static_cast<uint32_t>(count));
  HIPTRY(hipGetLastError());
  unsigned got = 0;
  HIPTRY(hipMemcpyAsync(&got, d_cnt, 4, hipMemcpyDeviceToHost, s));
  HIPTRY(hipStreamSynchronize(s));
  if (got != count) {
    if (err) *err = "top-K selection: candidate count mismatch";
    return PR_E_HIP;
  }
  ids->resize(count);
  rs->resize(count);
  HIPTRY(hipMemcpyAsync(ids->data(), d_ids, 4ull * count, hipMemcpyDeviceToHost, s));
  HIPTRY(hipMemcpyAsync(rs->data(), d_rs, 8ull * count, hipMemcpyDeviceToHost, s));
  HIPTRY(hipStreamSynchronize(s));
  return PR_OK;
}


// One wave that sleeps for about `us` microseconds (s_memrealtime ticks at 100 MHz); bounded by
// an iteration cap, so it ends whatever the clock does.  Measurements only.
// a virtual range of `size` bytes backed by separately created chunks of `chunk` bytes
static int vmm_alloc(void** out, size_t size, size_t chunk, std::string* err) {
  int dev = 0;
  HIPTRY(hipGetDevice(&dev));
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  HIPTRY(hipMemGetAllocationGranularity(&gran, &prop, chunk < (2u << 20) ? hipMemAllocationGranularityMinimum
                                                                            : hipMemAllocationGranularityRecommended));
  if (env_int("PR_VERBOSE", 0)) fprintf(stderr, "[vmm] granularity %zu, chunk %zu\n", gran, chunk);
  chunk = (chunk + gran - 1) / gran * gran;
  const size_t total = (size + chunk - 1) / chunk * chunk;
  void* va = nullptr;
  HIPTRY(hipMemAddressReserve(&va, total, gran, nullptr, 0));
  // PR_VMM_GAP_GB=g: g GB of device memory are skipped between consecutive chunks (held by
  // allocations that are released once every chunk exists), so the chunks spread over the device
  const size_t gap = static_cast<size_t>(std::max(0, env_int("PR_VMM_GAP_GB", 0))) << 30;
  std::vector<void*> spacers;
  for (size_t off = 0; off < total; off += chunk) {
    hipMemGenericAllocationHandle_t h;
    HIPTRY(hipMemCreate(&h, chunk, &prop, 0));
    HIPTRY(hipMemMap(static_cast<char*>(va) + off, chunk, 0, h, 0));
    if (gap && off + chunk < total) {
      void* sp = nullptr;
      if (hipMalloc(&sp, gap) == hipSuccess) spacers.push_back(sp);
      else (void)hipGetLastError();
    }
  }
  for (void* sp : spacers) (void)hipFree(sp);
  hipMemAccessDesc d{};
  d.location = prop.location;
  d.flags = hipMemAccessFlagsProtReadWrite;
  HIPTRY(hipMemSetAccess(va, total, &d, 1));
  *out = va;
  return PR_OK;
}

int dev_move_array(DevGraph* g, const char* name, std::string* err) {
  const std::string nm = name ? name : "";
  auto move = [&](auto** pp) -> int {
    if (!*pp) return PR_OK;
    void* base = nullptr;
    size_t size = 0;
    HIPTRY(hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t*>(&base), &size, reinterpret_cast<hipDeviceptr_t>(*pp)));
    if (base != static_cast<void*>(*pp)) {
      if (err) *err = "array is not the start of its allocation";
      return PR_E_ARG;
    }
    void* fresh = nullptr;
    const int vmm_mb = env_int("PR_VMM_MB", 0), vmm_kb = env_int("PR_VMM_KB", 0);
    if (vmm_mb > 0 || vmm_kb > 0) {
      int rc = vmm_alloc(&fresh, size, vmm_kb > 0 ? static_cast<size_t>(vmm_kb) << 10 : static_cast<size_t>(vmm_mb) << 20, err);
      if (rc) return rc;
    } else if (env_int("PR_CONTIG", 0)) {
      HIPTRY(hipExtMallocWithFlags(&fresh, size, hipDeviceMallocContiguous));
    } else {
      HIPTRY(hipMalloc(&fresh, size));
    }
    HIPTRY(hipMemcpy(fresh, *pp, size, hipMemcpyDeviceToDevice));
    if (env_int("PR_VERBOSE", 0))
      fprintf(stderr, "[move] %s: %p -> %p (%.1f MB) | col16 %p col %p bits %p x %p %p\n", nm.c_str(), static_cast<void*>(*pp), fresh,
              size / 1048576.0, static_cast<void*>(g->col16), static_cast<void*>(g->col), static_cast<void*>(g->bits),
              static_cast<void*>(g->xbuf[0]), static_cast<void*>(g->xbuf[1]));
    HIPTRY(hipFree(*pp));
    *pp = static_cast<std::remove_reference_t<decltype(**pp)>*>(fresh);
    return PR_OK;
  };
  int rc = PR_OK;
  if (nm == "partial") rc = move(&g->partial);
  else if (nm == "col16") rc = move(&g->col16);
  else if (nm == "col") rc = move(&g->col);
  else if (nm == "bits") rc = move(&g->bits);
  else if (nm == "roffL") rc = move(&g->roffL);
  else if (nm == "meta") rc = move(&g->meta);
  else if (nm == "x") {
    rc = move(&g->xbuf[0]);
    if (!rc) rc = move(&g->xbuf[1]);
    if (!rc) rc = move(&g->x_init);
  } else if (nm == "maps") {
    rc = move(&g->nebase);
    if (!rc) rc = move(&g->lfirst);
    if (!rc) rc = move(&g->lmask);
  } else {
    if (err) *err = "unknown array";
    return PR_E_ARG;
  }
  return rc;
}

__global__ void k_delay(uint32_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < (1u << 22); ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(64);
  }
}
int dev_delay_us(int us, hipStream_t s) {
  std::string* err = nullptr;
  if (us > 0) hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, static_cast<uint32_t>(std::min(us, 1000000)) * 100u);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_selftest_lds_order(uint32_t cases, uint32_t launches, hipStream_t s, uint64_t* copies,
                           uint64_t* differing, uint64_t* lane_order_cases, std::string* err) {
  constexpr uint32_t GRID = 2048;  // 8 workgroups per CU: every CU and XCD takes part
  const uint64_t nw = static_cast<uint64_t>(GRID) * (BLOCK / 64);
  uint64_t* d = nullptr;
  TRY(dmalloc(&d, nw * ST_ROWS, err));
  struct Free {
    void* p;
    ~Free() { (void)hipFree(p); }
  } fr{d};
  std::vector<uint64_t> h(nw * ST_ROWS);
  *copies = *differing = *lane_order_cases = 0;
  for (uint32_t c = 0; c < cases; ++c) {
    // the sum in ascending lane order, one rounding per add (what a serial loop gives)
    double seq[ST_ROWS] = {0};
    for (uint32_t l = 0; l < 64; ++l) {
      uint32_t row;
      double v;
      st_case(c, l, &row, &v);
      seq[row] += v;
    }
    uint64_t first[ST_ROWS];
    bool have = false;
    for (uint32_t it = 0; it < launches; ++it) {
      hipLaunchKernelGGL(k_lds_order, dim3(GRID), dim3(BLOCK), 0, s, c, d);
      HIPTRY(hipGetLastError());
      HIPTRY(hipMemcpyAsync(h.data(), d, 8 * h.size(), hipMemcpyDeviceToHost, s));
      HIPTRY(hipStreamSynchronize(s));
      if (!have) {
        memcpy(first, h.data(), sizeof(first));
        have = true;
      }
      for (uint64_t w = 0; w < nw; ++w) {
        ++*copies;
        if (memcmp(&h[w * ST_ROWS], first, sizeof(first)) != 0) ++*differing;
      }
    }
    bool same = true;
    for (int r = 0; r < ST_ROWS; ++r) {
      uint64_t b;
      memcpy(&b, &seq[r], 8);
      same = same && b == first[r];
    }
    if (same) ++*lane_order_cases;
  }
  return PR_OK;
}

int dev_export_csr(DevGraph* g, uint64_t* row_ptr, uint32_t* col, hipStream_t s, std::string* err) {
  const Layout L = layout_of(g);
  const uint64_t m = g->lnnz;
  Temp tmp;
  uint32_t* prow = nullptr;
  uint64_t *k0 = nullptr, *k1 = nullptr, *rp = nullptr;
  uint32_t* c = nullptr;
  struct Free {
    std::vector<void*> v;
    ~Free() { for (void* p : v) if (p) (void)hipFree(p); }
  } fr;
  TRY(dmalloc(&prow, g->n_pieces, err)); fr.v.push_back(prow);
  TRY(dmalloc(&k0, m, err)); fr.v.push_back(k0);
  TRY(dmalloc(&k1, m, err)); fr.v.push_back(k1);
  TRY(dmalloc(&rp, g->lrows + 1ull, err)); fr.v.push_back(rp);
  TRY(dmalloc(&c, m, err)); fr.v.push_back(c);
  const RowBlocks RBk{g->lA, g->nb_rows_a, g->nb_rows, g->n_streams, g->row_rb,
                      g->row_nbH, g->row_rbH, g->row_lH};
  if (g->nb_rows) hipLaunchKernelGGL(k_piece_row_runs, dim3(grid_loop(static_cast<uint64_t>(g->nb_rows) * g->n_streams)), dim3(BLOCK), 0, s, g->runs, g->roff, RBk, prow);
  if (g->stream_len) hipLaunchKernelGGL(k_export_keys, dim3(grid_loop(g->stream_len)), dim3(BLOCK), 0, s, g->col, g->col16, reinterpret_cast<const uint32_t*>(g->bits), g->task_piece, prow, L, g->d_gstart, g->d_gtask, g->d_gbase, static_cast<uint32_t>(g->gtask.size() - 1), g->nlds, g->hot_h, g->stream_len, k0);
  rocprim::double_buffer<uint64_t> db(k0, k1);
  size_t tb = 0;
  HIPTRY(rocprim::radix_sort_keys(nullptr, tb, db, m, 0, 64, s));
  TRY(tmp.ensure(tb, err));
  if (m) HIPTRY(rocprim::radix_sort_keys(tmp.p, tb, db, m, 0, 64, s));
  HIPTRY(hipMemsetAsync(rp, 0, 8ull * (g->lrows + 1), s));
  if (m) hipLaunchKernelGGL(k_export_split, dim3(grid_loop(m)), dim3(BLOCK), 0, s, db.current(), m, c, rp);
  HIPTRY(hipGetLastError());
  if (row_ptr) HIPTRY(hipMemcpyAsync(row_ptr, rp, 8ull * g->lrows, hipMemcpyDeviceToHost, s));
  if (col && m) HIPTRY(hipMemcpyAsync(col, c, 4ull * m, hipMemcpyDeviceToHost, s));
  HIPTRY(hipStreamSynchronize(s));
  if (row_ptr) row_ptr[g->lrows] = m;
  return PR_OK;
}

}  // namespace prmi

