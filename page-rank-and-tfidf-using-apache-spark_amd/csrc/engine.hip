// prmi355x device engine (gfx950 / CDNA4).
//
// Replaces, per round, PageRank.java:94-160 -- the contribution flatMapToPair (:94-117), the
// dangling-mass reduce (:121-138), reduceByKey(Sum) (:139, Sum :208-213) and the damping /
// dangling-update maps (:140-160) -- with a pull SpMV over the transposed graph in two
// launches (XCD-sliced partial sums for heavy rows; a fused row launch that combines them,
// handles the light rows and applies the epilogue) plus two single-workgroup reductions.  The graph build (K1) replaces
// distinct().groupByKey() (:42), the urlCount loop (:103-108) and subtractByKey (:56).
//
// Numerics (DESIGN.md "Parity"):
//   * x = r / outdeg is one IEEE division per source (same operands as :113, bit-exact);
//   * each row's sum is a fixed-shape tree that depends only on the row's in-degree
//     (deterministic, identical for any number of ranks);
//   * r' = 0.15 + (c + a) * 0.85 is evaluated unfused in Java's order (:143);
//   * the dangling mass, residual and rank sum are EXACT (integer superaccumulator, then one
//     correct rounding), so addthis (:135) equals the correctly rounded exact value.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string.h>

#include <rocprim/rocprim.hpp>

#include "engine.h"
#include "prmi355x.h"

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
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
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

// Correct rounding of a superaccumulator (limbs hold 32-bit chunks plus carries).
__device__ double sa_to_double_dev(const uint64_t* limb) {
  uint32_t c[SA_LIMBS + 2];
  uint64_t carry = 0;
  for (int i = 0; i < SA_LIMBS; ++i) {
    const uint64_t t = limb[i] + carry;
    c[i] = static_cast<uint32_t>(t);
    carry = t >> 32;
  }
  c[SA_LIMBS] = static_cast<uint32_t>(carry);
  c[SA_LIMBS + 1] = static_cast<uint32_t>(carry >> 32);
  int top = -1;
  for (int i = SA_LIMBS + 1; i >= 0; --i)
    if (c[i]) {
      top = i * 32 + 31 - __clz(c[i]);
      break;
    }
  if (top < 0) return 0.0;
  auto bit = [&](int p) -> uint32_t { return p < 0 ? 0u : ((c[p >> 5] >> (p & 31)) & 1u); };
  if (top < 53) {
    uint64_t m = 0;
    for (int p = top; p >= 0; --p) m = (m << 1) | bit(p);
    return ldexp(static_cast<double>(m), SA_BASE_EXP);
  }
  uint64_t m = 0;
  for (int p = top; p > top - 53; --p) m = (m << 1) | bit(p);
  int lowest = top - 52;
  const uint32_t rb = bit(lowest - 1);
  uint32_t sticky = 0;
  for (int p = lowest - 2; p >= 0 && !sticky; --p) sticky |= bit(p);
  if (rb && (sticky || (m & 1))) {
    m += 1;
    if (m == (1ull << 53)) {
      m >>= 1;
      lowest += 1;
    }
  }
  return ldexp(static_cast<double>(m), lowest + SA_BASE_EXP);
}

// =======================================================================================
// the round: XCD-sliced partial sums + fused row launch (combine / light rows / epilogue)
// =======================================================================================
struct StepArgs {
  const Bin* bins;
  int nbins;
  const uint64_t* row_ptr;
  const uint32_t* col;
  const uint32_t* meta;
  const double* x_in;
  double* x_out;          // this rank's slot of the next x
  const double* r_old;    // tracked mode: previous ranks (nullptr = r^0 == 1)
  double* r_out;
  const HubSeg* segs;     // hub segments of this launch
  double* hub_part;
  const HubRow* hubs;
  const IterState* st;
  uint64_t* shards;
  const uint32_t* sb;     // [9][nS] slice offsets of sliced rows
  double* part;           // [8][nS] slice partials
  uint32_t nS;
  uint32_t hub_tiles;     // per-slice stride of the sliced hub segment table
  uint32_t colmask;       // timing experiments only (PR_COLMASK); all-ones in production
  uint32_t block_base;    // first grid block of this launch (PR_SPLIT timing mode)
  uint32_t p, rank, sm, SL;  // x layout: where local row l's x' goes inside this rank's slot
  uint32_t tile_end;         // slice launch: one past the last wave-tile of this launch
  uint32_t hot_n;            // slice launch: x entries per slice cached in LDS
  uint32_t hot_base[NSLICE]; // slice launch: x position of each slice region's start
};

// offset of local row l's x entry inside this rank's slot (see Layout / xpos)
__device__ __forceinline__ uint32_t xslot_of(const StepArgs& A, uint32_t l) {
  if (!A.sm) return l;
  const uint32_t c = (l / CHUNK) * A.p + A.rank, sl = c % NSLICE;
  return (sl / A.p) * A.SL + (c / NSLICE) * CHUNK + (l % CHUNK);
}

__device__ __forceinline__ int find_bin(const Bin* bins, int nbins, uint32_t t) {
  int lo = 0, hi = nbins - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (bins[mid].block_begin <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Streamed (read-once) operands: non-temporal loads keep them from evicting the hot part
// of x from the XCD's L2 (NT = 1).
template <int NT, class T>
__device__ __forceinline__ T ld_stream(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// Gathers of x: plain loads, or -- in the persistent slice kernel -- the first H entries of
// the slice's region (its hottest sources) served from an LDS copy.
struct GatherX {
  const double* __restrict__ x;
  uint32_t cm;  // PR_COLMASK (timing experiments only)
  __device__ __forceinline__ double operator()(uint32_t q) const { return x[q & cm]; }
};
struct GatherLds {
  const double* __restrict__ x;
  const double* lds;
  uint32_t base, H, cm;
  __device__ __forceinline__ double operator()(uint32_t q) const {
    q &= cm;
    const uint32_t o = q - base;
    return o < H ? lds[o] : x[q];
  }
};

// Partial sum of x[col[e]] over e = beg + lane, beg + lane + S, ... < end, with four
// independent gathers in flight per lane.  Fixed order: depends on (end-beg, S) only.
template <int S, int NT, class Gx>
__device__ __forceinline__ double strided_sum(const uint32_t* __restrict__ col, const Gx& gx,
                                              uint64_t beg, uint64_t end, int lane) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  for (uint64_t e = beg + lane; e < end; e += 4ull * S) {
    const uint64_t e1 = e + S, e2 = e + 2ull * S, e3 = e + 3ull * S;
    const uint32_t c0 = ld_stream<NT>(col + e);
    const uint32_t c1 = e1 < end ? ld_stream<NT>(col + e1) : 0u;
    const uint32_t c2 = e2 < end ? ld_stream<NT>(col + e2) : 0u;
    const uint32_t c3 = e3 < end ? ld_stream<NT>(col + e3) : 0u;
    const double v0 = gx(c0);
    const double v1 = e1 < end ? gx(c1) : 0.0;
    const double v2 = e2 < end ? gx(c2) : 0.0;
    const double v3 = e3 < end ? gx(c3) : 0.0;
    s0 += v0;
    s1 += v1;
    s2 += v2;
    s3 += v3;
  }
  return (s0 + s1) + (s2 + s3);
}

// Workgroup-wide sum (fixed tree), valid in thread 0.
__device__ __forceinline__ double block_sum(double s, double* red) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// Epilogue for one row per group leader, then the block's exact partials (dangling mass +
// count for class-B rows; residual + rank sum in tracked mode) into the atomic shards.
template <int MODE>
__device__ __forceinline__ void row_epilogue(const StepArgs& A, double a, uint32_t cls,
                                             uint32_t row, double c, bool leader,
                                             uint64_t (*lds)[REC_WORDS]) {
  double r = 0.0;
  uint32_t w = 0;
  if (leader) {
    // PageRank.java:143  0.15 + (sum + addthis) * 0.85, unfused
    r = c > 0.0 ? __dadd_rn(0.15, __dmul_rn(__dadd_rn(c, a), 0.85)) : 0.0;
    const uint32_t mt = A.meta[row];
    if (cls == 0)
      A.x_out[xslot_of(A, row)] = r / static_cast<double>(mt);  // :113  rank / urlCount
    else
      w = mt;
    if (MODE >= 1) A.r_out[row] = r;
  }
  const bool acc = (cls == 1) || (MODE == 2);  // uniform over the workgroup
  if (!acc) return;
  for (int i = threadIdx.x; i < 4 * REC_WORDS; i += BLOCK) (&lds[0][0])[i] = 0;
  __syncthreads();
  uint64_t* lw = lds[threadIdx.x >> 6];
  uint32_t c0, c1, c2, c3;
  if (cls == 1) {
    // PageRank.java:125-134  sum of danglingMap values (w entries per page)
    const int li = sa_chunks(leader ? r : 0.0, w, c0, c1, c2, c3);
    wave_accum_sa(lw, REC_DSUM, li, c0, c1, c2, c3);
    const uint64_t cnt = wave_sum_u64((leader && r > 0.0) ? w : 0u);
    if ((threadIdx.x & 63) == 0) lw[REC_DCNT] += cnt;
  }
  if (MODE == 2) {
    double ro = 0.0;
    if (leader) ro = A.r_old ? A.r_old[row] : 1.0;
    const double d = fabs(r - ro);
    int li = sa_chunks(leader ? d : 0.0, 1u, c0, c1, c2, c3);
    wave_accum_sa(lw, REC_RESID, li, c0, c1, c2, c3);
    li = sa_chunks(leader ? r : 0.0, 1u, c0, c1, c2, c3);
    wave_accum_sa(lw, REC_RSUM, li, c0, c1, c2, c3);
  }
  __syncthreads();
  if (threadIdx.x < REC_WORDS) {
    const int t = threadIdx.x;
    const uint64_t s = (lds[0][t] + lds[1][t]) + (lds[2][t] + lds[3][t]);
    if (s) atomicAdd(reinterpret_cast<unsigned long long*>(
                         &A.shards[(blockIdx.x % NSHARD) * REC_WORDS + t]),
                     static_cast<unsigned long long>(s));
  }
}

// G lanes per row (G <= 64): a workgroup takes 256/G consecutive rows of one bin.
template <int G, int MODE, int NT>
__device__ __forceinline__ void group_tile(const StepArgs& A, double a, const Bin& b,
                                           uint32_t blk, uint64_t (*lds)[REC_WORDS]) {
  constexpr uint32_t RPB = BLOCK / G;
  const uint32_t row = b.row_begin + blk * RPB + threadIdx.x / G;
  const int gl = threadIdx.x % G;
  const bool active = row < b.row_end;
  double s = 0.0;
  if (active)
    s = strided_sum<G, NT>(A.col, GatherX{A.x_in, A.colmask}, ld_stream<NT>(A.row_ptr + row),
                           ld_stream<NT>(A.row_ptr + row + 1), gl);
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  row_epilogue<MODE>(A, a, b.cls, row, s, active && gl == 0, lds);
}

// Sliced rows: the row sum is a fixed tree over the 8 slice partials.
template <int MODE>
__device__ __forceinline__ void combine_tile(const StepArgs& A, double a, const Bin& b,
                                             uint32_t blk, uint64_t (*lds)[REC_WORDS]) {
  const uint32_t i = blk * BLOCK + threadIdx.x;
  const uint32_t row = b.row_begin + i;
  const bool active = row < b.row_end;
  double c = 0.0;
  if (active) {
    const uint32_t sr = b.srow_begin + i;
    const double* p = A.part + sr;
    const uint64_t S = A.nS;
    c = ((p[0] + p[S]) + (p[2 * S] + p[3 * S])) + ((p[4 * S] + p[5 * S]) + (p[6 * S] + p[7 * S]));
  }
  row_epilogue<MODE>(A, a, b.cls, row, c, active, lds);
}

template <int MODE, int NT>
__global__ __launch_bounds__(BLOCK) void spmv_round(StepArgs A) {
  __shared__ uint64_t lds[4][REC_WORDS];
  __shared__ double red[4];
  const uint32_t b = blockIdx.x + A.block_base;
  const Bin bin = A.bins[find_bin(A.bins, A.nbins, b)];
  const uint32_t blk = b - bin.block_begin;
  const double a = A.st->a;
  switch (bin.kind) {
    case 0: group_tile<1, MODE, NT>(A, a, bin, blk, lds); break;
    case 1: group_tile<2, MODE, NT>(A, a, bin, blk, lds); break;
    case 2: group_tile<4, MODE, NT>(A, a, bin, blk, lds); break;
    case 3: group_tile<8, MODE, NT>(A, a, bin, blk, lds); break;
    case 4: group_tile<16, MODE, NT>(A, a, bin, blk, lds); break;
    case 5: group_tile<32, MODE, NT>(A, a, bin, blk, lds); break;
    case 6: group_tile<64, MODE, NT>(A, a, bin, blk, lds); break;
    case KIND_COMBINE: combine_tile<MODE>(A, a, bin, blk, lds); break;
    case KIND_BLOCK: {
      const uint32_t row = bin.row_begin + blk;
      double s = strided_sum<BLOCK, NT>(A.col, GatherX{A.x_in, A.colmask}, A.row_ptr[row],
                                        A.row_ptr[row + 1], threadIdx.x);
      s = block_sum(s, red);
      row_epilogue<MODE>(A, a, bin.cls, row, s, threadIdx.x == 0, lds);
      break;
    }
    default: {  // KIND_HUB: one segment of an unsliced split row (combined in hub_round)
      const HubSeg seg = A.segs[bin.seg_begin + blk];
      double s = strided_sum<BLOCK, NT>(A.col, GatherX{A.x_in, A.colmask}, seg.e_begin,
                                        seg.e_end, threadIdx.x);
      s = block_sum(s, red);
      if (threadIdx.x == 0) A.hub_part[seg.part] = s;
      break;
    }
  }
}

// ---- the slice launch: persistent, slice j = blockIdx % 8 (one XCD per slice) ----------
// Every wave walks the wave-tiles of its slice with a static stride; a tile is 64/G rows of
// a grouped bin, one (row, slice) sub-list of a long row, or one hub segment.  The first H
// entries of the slice's x region (its hottest sources) are copied to LDS once per round.
constexpr int SLICE_BLOCK = 1024;

__device__ __forceinline__ double wave_sum(double s) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  return s;
}

template <int G, int NT, class Gx>
__device__ __forceinline__ void slice_group(const StepArgs& A, const Gx& gx, const Bin& b,
                                            uint32_t tile, uint32_t j, int lane) {
  constexpr uint32_t RPW = 64 / G;
  const uint32_t i = tile * RPW + lane / G;
  const uint32_t row = b.row_begin + i;
  const int gl = lane % G;
  const bool active = row < b.row_end;
  double s = 0.0;
  const uint32_t sr = b.srow_begin + i;
  if (active) {
    const uint64_t base = ld_stream<NT>(A.row_ptr + row);
    const uint64_t beg = base + ld_stream<NT>(A.sb + static_cast<uint64_t>(j) * A.nS + sr);
    const uint64_t end = base + ld_stream<NT>(A.sb + static_cast<uint64_t>(j + 1) * A.nS + sr);
    s = strided_sum<G, NT>(A.col, gx, beg, end, gl);
  }
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (active && gl == 0) A.part[static_cast<uint64_t>(j) * A.nS + sr] = s;
}

template <int NT, class Gx>
__device__ __forceinline__ void slice_tile(const StepArgs& A, const Gx& gx, uint32_t t,
                                           uint32_t j, int lane) {
  const Bin bin = A.bins[find_bin(A.bins, A.nbins, t)];
  const uint32_t tt = t - bin.block_begin;
  switch (bin.kind) {
    case 0: slice_group<1, NT>(A, gx, bin, tt, j, lane); break;
    case 1: slice_group<2, NT>(A, gx, bin, tt, j, lane); break;
    case 2: slice_group<4, NT>(A, gx, bin, tt, j, lane); break;
    case 3: slice_group<8, NT>(A, gx, bin, tt, j, lane); break;
    case 4: slice_group<16, NT>(A, gx, bin, tt, j, lane); break;
    case 5: slice_group<32, NT>(A, gx, bin, tt, j, lane); break;
    case 6: slice_group<64, NT>(A, gx, bin, tt, j, lane); break;
    case KIND_BLOCK: {  // one long (row, slice) sub-list per wave
      const uint32_t row = bin.row_begin + tt;
      const uint32_t sr = bin.srow_begin + tt;
      const uint64_t base = A.row_ptr[row];
      const uint64_t beg = base + A.sb[static_cast<uint64_t>(j) * A.nS + sr];
      const uint64_t end = base + A.sb[static_cast<uint64_t>(j + 1) * A.nS + sr];
      const double s = wave_sum(strided_sum<64, NT>(A.col, gx, beg, end, lane));
      if (lane == 0) A.part[static_cast<uint64_t>(j) * A.nS + sr] = s;
      break;
    }
    default: {  // KIND_HUB: slice j's segment list (padded with empty segments)
      const HubSeg seg = A.segs[static_cast<uint64_t>(j) * A.hub_tiles + bin.seg_begin + tt];
      const double s = wave_sum(strided_sum<64, NT>(A.col, gx, seg.e_begin, seg.e_end, lane));
      if (lane == 0 && seg.part != 0xFFFFFFFFu) A.hub_part[seg.part] = s;
      break;
    }
  }
}

template <int NT, bool HOT>
__global__ __launch_bounds__(SLICE_BLOCK) void spmv_slices(StepArgs A) {
  extern __shared__ __attribute__((aligned(16))) double hot[];
  const uint32_t j = blockIdx.x % NSLICE, bi = blockIdx.x / NSLICE;
  const uint32_t nb = gridDim.x / NSLICE, nw = blockDim.x / 64;
  const int lane = threadIdx.x & 63;
  const uint32_t w0 = bi * nw + threadIdx.x / 64, stride = nb * nw;
  if constexpr (HOT) {
    const uint32_t base = A.hot_base[j], H = A.hot_n;
    for (uint32_t i = threadIdx.x; i < H; i += blockDim.x) hot[i] = A.x_in[base + i];
    __syncthreads();
    const GatherLds gx{A.x_in, hot, base, H, A.colmask};
    for (uint32_t t = A.block_base + w0; t < A.tile_end; t += stride) slice_tile<NT>(A, gx, t, j, lane);
  } else {
    const GatherX gx{A.x_in, A.colmask};
    for (uint32_t t = A.block_base + w0; t < A.tile_end; t += stride) slice_tile<NT>(A, gx, t, j, lane);
  }
}

// Split rows: sum the segment partials in segment order, then the same epilogue.
template <int MODE>
__global__ __launch_bounds__(BLOCK) void hub_round(StepArgs A) {
  __shared__ uint64_t lds[4][REC_WORDS];
  __shared__ double red[4];
  const HubRow h = A.hubs[blockIdx.x];
  double s = 0.0;
  for (uint32_t i = h.part_begin + threadIdx.x; i < h.part_end; i += BLOCK) s += A.hub_part[i];
  s = block_sum(s, red);
  row_epilogue<MODE>(A, A.st->a, h.cls, h.row, s, threadIdx.x == 0, lds);
}

// Sum the NSHARD shards into one record and clear them for the next round.
__global__ __launch_bounds__(BLOCK) void reduce_shards(uint64_t* shards, uint64_t* rec) {
  __shared__ uint64_t part[8][REC_WORDS];
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
  }
}

// Combine the p rank records (integer sums: order-free, exact) -> next round's addthis.
__global__ void finalize_round(const uint64_t* rec_all, int p, int t, uint64_t n_tot,
                               uint64_t extra_resid, int tracked, IterState* st) {
  if (threadIdx.x != 0) return;
  uint64_t dsum[SA_LIMBS] = {0}, res[SA_LIMBS] = {0}, rsum[SA_LIMBS] = {0};
  uint64_t dcnt = 0;
  for (int r = 0; r < p; ++r) {
    const uint64_t* q = rec_all + r * REC_WORDS;
    for (int i = 0; i < SA_LIMBS; ++i) {
      dsum[i] += q[REC_DSUM + i];
      res[i] += q[REC_RESID + i];
      rsum[i] += q[REC_RSUM + i];
    }
    dcnt += q[REC_DCNT];
  }
  // :135  accum.setValue(sum / totalVertices)
  st->a = sa_to_double_dev(dsum) / static_cast<double>(n_tot);
  st->dcnt = dcnt;
  if (dcnt == 0 && st->err_iter == 0) st->err_iter = t + 1;
  if (tracked) {
    // whole units: 1.0 = 2^96 units = bit 0 of limb 3
    res[3] += extra_resid & 0xFFFFFFFFull;
    res[4] += extra_resid >> 32;
    const double ra = sa_to_double_dev(res);
    const double rs = sa_to_double_dev(rsum);
    st->resid_abs = ra;
    st->rank_sum = rs;
    st->resid = rs > 0.0 ? ra / rs : 0.0;
  }
  st->iter = t;
}

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
  const uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
  if (e >= m) return;
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

__global__ void k_make_keys(const uint32_t* src, const uint32_t* dst, uint64_t m, int nb,
                            uint64_t* keys) {
  const uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
  if (e < m) keys[e] = (static_cast<uint64_t>(dst[e]) << nb) | src[e];
}

__global__ void k_degrees(const uint64_t* uk, uint64_t nnz, int nb, uint32_t* outdeg,
                          uint32_t* indeg, unsigned long long* digest) {
  __shared__ unsigned long long ssum[BLOCK / 64], sxor[BLOCK / 64];
  const uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
  uint64_t h = 0;
  if (e < nnz) {
    const uint64_t k = uk[e];
    const uint32_t d = static_cast<uint32_t>(k >> nb);
    const uint32_t s = static_cast<uint32_t>(k & ((1ull << nb) - 1));
    atomicAdd(&outdeg[s], 1u);
    atomicAdd(&indeg[d], 1u);
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
    atomicAdd(&digest[0], a);
    atomicXor(&digest[1], x);
  }
}

// dangling weight (PageRank.java:56) + class key for the vertex order
__global__ void k_vertex_keys(const uint32_t* outdeg, const uint32_t* indeg, const uint32_t* mapw,
                              uint32_t n, uint32_t* dang_w, uint64_t* vkey, uint32_t* vid,
                              unsigned long long* sums /* [0]=W0 [1]=dangling entries */) {
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
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(&sums[0], static_cast<unsigned long long>(s));
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
__device__ __forceinline__ uint32_t xpos(const Layout& L, uint32_t k) {
  if (k < L.nA) {
    if (!L.sm) return owner_of(L, k) * L.maxA + local_of(L, k);
    const uint32_t c = k / CHUNK, sl = c % NSLICE;
    return (sl % L.p) * L.maxA + (sl / L.p) * L.SL + (c / NSLICE) * CHUNK + (k % CHUNK);
  }
  const uint32_t kc = k - L.R;
  if (!L.sm) return L.p * L.maxA + kc;
  const uint32_t c = kc / CHUNK;
  return L.p * L.maxA + (c % NSLICE) * L.SLC + (c / NSLICE) * CHUNK + (kc % CHUNK);
}
// slice of a column = its 128-byte chunk index mod 8 (independent of the rank count)
__device__ __forceinline__ uint32_t slice_of(const Layout& L, uint32_t k) {
  return ((k < L.nA ? k : k - L.R) / CHUNK) % NSLICE;
}

__global__ void k_x_init(const uint32_t* perm, const uint32_t* outdeg, uint32_t n, Layout L,
                         double* x_init) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const bool col = k < L.nA || (k >= L.R && k < L.R + L.nC);
  if (col) x_init[xpos(L, k)] = 1.0 / static_cast<double>(outdeg[perm[k]]);
}

// relabel unique edges to (local row, slice, internal source) and keep this rank's rows;
// rows with in-degree >= ks get their edges grouped by the slice of the source's x line
__global__ void k_relabel(const uint64_t* uk, uint64_t nnz, int nb, const uint32_t* inv,
                          const uint32_t* indeg, uint32_t ks, Layout L,
                          unsigned long long* counter, uint64_t* out) {
  const uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
  bool keep = false;
  uint64_t key = 0;
  if (e < nnz) {
    const uint64_t k = uk[e];
    const uint32_t d = static_cast<uint32_t>(k >> nb);
    const uint32_t kd = inv[d];
    const uint32_t ksrc = inv[static_cast<uint32_t>(k & ((1ull << nb) - 1))];
    keep = owner_of(L, kd) == L.rank;
    const uint64_t sl = indeg[d] >= ks ? slice_of(L, ksrc) : 0u;
    key = (static_cast<uint64_t>(local_of(L, kd)) << (nb + 3)) | (sl << nb) | ksrc;
  }
  if (L.p == 1) {
    if (e < nnz) out[e] = key;
    return;
  }
  // wave-aggregated append
  const uint64_t mask = __ballot(keep);
  if (!mask) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll(static_cast<long long>(mask)) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(counter, static_cast<unsigned long long>(__popcll(mask)));
  base = __shfl(base, leader);
  if (keep) out[base + __popcll(mask & ((1ull << lane) - 1))] = key;
}

struct SliceRows {
  uint32_t lA, sA, sB, nS;
};
__device__ __forceinline__ int srow_of(const SliceRows& S, uint32_t l) {
  if (l < S.sA) return static_cast<int>(l);
  if (l >= S.lA && l - S.lA < S.sB) return static_cast<int>(S.sA + (l - S.lA));
  return -1;
}

// col = x position of the source; per (sliced row, slice) edge counts
__global__ void k_col(const uint64_t* lk, uint64_t lnnz, int nb, Layout L, SliceRows S,
                      uint32_t* col, uint32_t* cnt) {
  const uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
  if (e >= lnnz) return;
  const uint64_t key = lk[e];
  col[e] = xpos(L, static_cast<uint32_t>(key & ((1ull << nb) - 1)));
  const int sr = srow_of(S, static_cast<uint32_t>(key >> (nb + 3)));
  if (sr >= 0) {
    const uint32_t sl = static_cast<uint32_t>((key >> nb) & 7);
    atomicAdd(&cnt[static_cast<uint64_t>(sl) * S.nS + sr], 1u);
  }
}

// sb[j][srow] = edges of the row in slices < j (relative to the row start)
__global__ void k_slice_prefix(const uint32_t* cnt, uint32_t nS, uint32_t* sb) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nS) return;
  uint32_t acc = 0;
  for (int j = 0; j < NSLICE; ++j) {
    sb[static_cast<uint64_t>(j) * nS + r] = acc;
    acc += cnt[static_cast<uint64_t>(j) * nS + r];
  }
  sb[static_cast<uint64_t>(NSLICE) * nS + r] = acc;
}

__global__ void k_local_rows(const uint32_t* perm, const uint32_t* indeg, const uint32_t* outdeg,
                             const uint32_t* dang_w, uint32_t lrows, uint32_t lA, Layout L,
                             uint64_t* deg64, uint32_t* ldeg, uint32_t* meta) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l > lrows) return;
  if (l == lrows) {
    deg64[l] = 0;
    return;
  }
  const uint32_t v = perm[row_of(L, l)];
  const uint32_t d = indeg[v];
  deg64[l] = d;
  ldeg[l] = d;
  meta[l] = l < lA ? outdeg[v] : dang_w[v];
}

__global__ void k_scatter_ranks(const uint32_t* perm, const double* r_loc, uint32_t lrows,
                                Layout L, double* r_full) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l < lrows) r_full[perm[row_of(L, l)]] = r_loc[l];
}

__global__ void k_sources_one(const uint32_t* outdeg, uint32_t n, double* r_full) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) r_full[v] = outdeg[v] ? 1.0 : 0.0;
}

// =======================================================================================
// host side of the build
// =======================================================================================
namespace {

inline uint32_t grid_for(uint64_t n) { return static_cast<uint32_t>((n + BLOCK - 1) / BLOCK); }

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
  F(g->row_ptr); F(g->col); F(g->meta); F(g->perm); F(g->outdeg); F(g->indeg); F(g->dang_w);
  F(g->sb); F(g->part);
  F(g->x_init); F(g->xbuf[0]); F(g->xbuf[1]); F(g->r_loc[0]); F(g->r_loc[1]); F(g->r_full);
  F(g->shards); F(g->rec_local); F(g->rec_all); F(g->state); F(g->d_bins); F(g->d_sbins);
  F(g->d_hubs); F(g->d_segs); F(g->d_ssegs); F(g->hub_part);
  for (auto e : g->split_ev) (void)hipEventDestroy(e);
  const int p = g->p, rank = g->rank;
  *g = DevGraph();
  g->p = p;
  g->rank = rank;
}

namespace {

Layout layout_of(const DevGraph* g) {
  return Layout{static_cast<uint32_t>(g->p), static_cast<uint32_t>(g->rank), g->nA, g->R, g->nC,
                g->maxA, g->sm ? 1u : 0u, g->SL, g->SLC};
}

// rows owned by rank j among internal ids [0, cnt) when chunks of CHUNK are dealt round-robin
uint32_t owned_rows(uint32_t cnt, uint32_t p, uint32_t j) {
  const uint32_t full = cnt / CHUNK, rem = cnt % CHUNK;
  uint32_t r = CHUNK * (full / p + (j < full % p ? 1u : 0u));
  if (rem && full % p == j) r += rem;
  return r;
}

uint16_t kind_for(uint64_t len, const Tuning& T) {
  if (len > T.kb) return KIND_BLOCK;
  const uint64_t want = (len + T.epl - 1) / T.epl;
  uint16_t kd = 0;
  while ((1ull << kd) < want && kd < 6) ++kd;
  return kd;
}

}  // namespace

int dev_build(DevGraph* g, const BuildInput& in, hipStream_t s, std::string* err) {
  auto t0 = std::chrono::steady_clock::now();
  const int p = g->p, rank = g->rank;
  dev_free(g);
  Tuning& T = g->tune;
  T.epl = std::max(1, env_int("PR_EPL", T.epl));
  T.kb = static_cast<uint32_t>(std::max(64, env_int("PR_KB", static_cast<int>(T.kb))));
  T.kh = static_cast<uint32_t>(std::max(static_cast<int>(T.kb), env_int("PR_KH", static_cast<int>(T.kh))));
  T.seg = static_cast<uint32_t>(std::max(256, env_int("PR_SEG", static_cast<int>(T.seg))));
  T.ks = static_cast<uint32_t>(std::max(1, env_int("PR_KS", static_cast<int>(T.ks))));
  T.nt = env_int("PR_NT", T.nt);
  T.hot_lds = static_cast<uint32_t>(std::max(0, std::min(20480, env_int("PR_HOTLDS", static_cast<int>(T.hot_lds)))));
  T.split = env_int("PR_SPLIT", 0);
  if (const char* cm = getenv("PR_COLMASK")) T.colmask = static_cast<uint32_t>(strtoul(cm, nullptr, 0));
  const uint32_t n = in.n;
  const uint64_t m = in.m;
  g->n = n;
  g->m_raw = m;
  g->n_tot = in.n_tot;
  const int nb = in.rmat ? std::max(1, in.scale) : bits_for(n);
  // edge keys (local row, slice, source) take 2*nb + 3 bits
  if (2 * nb + 3 > 64) {
    if (err) *err = "more than 2^30 vertices is not supported (64-bit edge keys)";
    return PR_E_ARG;
  }
  const uint32_t ks = T.ks;
  const int key_bits = 2 * nb + 3;
  Temp tmp;

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
    if (m) hipLaunchKernelGGL(k_rmat_keys, dim3(grid_for(m)), dim3(BLOCK), 0, s, in.seed, in.scale, m, kA);
  } else if (m) {
    uint32_t *ds = nullptr, *dd = nullptr;
    TRY(dmalloc(&ds, m, err));
    TRY(dmalloc(&dd, m, err));
    HIPTRY(hipMemcpyAsync(ds, in.h_src, m * 4, hipMemcpyHostToDevice, s));
    HIPTRY(hipMemcpyAsync(dd, in.h_dst, m * 4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_make_keys, dim3(grid_for(m)), dim3(BLOCK), 0, s, ds, dd, m, nb, kA);
    HIPTRY(hipStreamSynchronize(s));
    (void)hipFree(ds);
    (void)hipFree(dd);
  }
  HIPTRY(hipGetLastError());

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

  // ---- degrees + digest + dangling weights + vertex order -------------------------------
  TRY(dmalloc(&g->outdeg, n, err));
  TRY(dmalloc(&g->indeg, n, err));
  TRY(dmalloc(&g->dang_w, n, err));
  TRY(dmalloc(&g->perm, n, err));
  unsigned long long* d_sums = nullptr;  // [0,2) digest, [2] W0
  TRY(dmalloc(&d_sums, 4, err));
  HIPTRY(hipMemsetAsync(d_sums, 0, 32, s));
  HIPTRY(hipMemsetAsync(g->outdeg, 0, 4ull * (n ? n : 1), s));
  HIPTRY(hipMemsetAsync(g->indeg, 0, 4ull * (n ? n : 1), s));
  if (nnz) hipLaunchKernelGGL(k_degrees, dim3(grid_for(nnz)), dim3(BLOCK), 0, s, uniq, nnz, nb, g->outdeg, g->indeg, d_sums);
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
  if (n) hipLaunchKernelGGL(k_vertex_keys, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->outdeg, g->indeg, d_mapw, n, g->dang_w, vk, vid, d_sums + 2);
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
  unsigned long long sums[4];
  HIPTRY(hipMemcpyAsync(cls_first, d_cls, 16, hipMemcpyDeviceToHost, s));
  HIPTRY(hipMemcpyAsync(sums, d_sums, 32, hipMemcpyDeviceToHost, s));
  HIPTRY(hipStreamSynchronize(s));
  (void)hipFree(d_cls);
  (void)hipFree(d_sums);
  (void)hipFree(vk);
  (void)hipFree(vk2);
  if (d_mapw) (void)hipFree(d_mapw);
  g->digest[0] = sums[0];
  g->digest[1] = sums[1];
  g->W0 = sums[2];
  g->n_dang_entries = sums[2];
  uint32_t start[5];
  start[4] = n;
  for (int c = 3; c >= 0; --c) start[c] = cls_first[c] == 0xFFFFFFFFu ? start[c + 1] : cls_first[c];
  g->nA = start[1] - start[0];
  g->nB = start[2] - start[1];
  g->nC = start[3] - start[2];
  g->nD = start[4] - start[3];
  g->R = g->nA + g->nB;
  const uint32_t P = static_cast<uint32_t>(p), RK = static_cast<uint32_t>(rank);
  g->sm = (NSLICE % P) == 0 && env_int("PR_SLICE_MAJOR", 1) != 0;
  if (g->sm) {
    const uint32_t chA = (g->nA + CHUNK - 1) / CHUNK, chC = (g->nC + CHUNK - 1) / CHUNK;
    g->SL = CHUNK * ((chA + NSLICE - 1) / NSLICE);
    g->SLC = CHUNK * ((chC + NSLICE - 1) / NSLICE);
    g->maxA = (NSLICE / P) * g->SL;
    g->X = static_cast<uint64_t>(P) * g->maxA + static_cast<uint64_t>(NSLICE) * g->SLC;
  } else {
    uint32_t maxA = 0;
    for (uint32_t j = 0; j < P; ++j) maxA = std::max(maxA, owned_rows(g->nA, P, j));
    g->maxA = (maxA + CHUNK - 1) / CHUNK * CHUNK;
    g->X = static_cast<uint64_t>(P) * g->maxA + g->nC;
  }
  g->lrows = owned_rows(g->R, P, RK);
  g->lA = owned_rows(g->nA, P, RK);
  const Layout L = layout_of(g);

  // ---- x vectors ------------------------------------------------------------------------
  if (env_int("PR_XUNCACHED", 0)) {  // experiment: x in uncached device memory (32-B reads)
    for (double** px : {&g->x_init, &g->xbuf[0], &g->xbuf[1]})
      HIPTRY(hipExtMallocWithFlags(reinterpret_cast<void**>(px), 8 * (g->X ? g->X : 1), hipDeviceMallocUncached));
  } else {
    TRY(dmalloc(&g->x_init, g->X, err));
    TRY(dmalloc(&g->xbuf[0], g->X, err));
    TRY(dmalloc(&g->xbuf[1], g->X, err));
  }
  HIPTRY(hipMemsetAsync(g->x_init, 0, 8 * (g->X ? g->X : 1), s));
  HIPTRY(hipMemsetAsync(g->xbuf[0], 0, 8 * (g->X ? g->X : 1), s));
  HIPTRY(hipMemsetAsync(g->xbuf[1], 0, 8 * (g->X ? g->X : 1), s));
  if (n) hipLaunchKernelGGL(k_x_init, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->perm, g->outdeg, n, L, g->x_init);
  uint32_t* inv = vid;  // reuse: n entries
  if (n) hipLaunchKernelGGL(k_inverse, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->perm, n, inv);

  // ---- per-row data: in-degrees (host copy for the schedule), meta, row pointers --------
  const uint32_t lrows = g->lrows;
  uint64_t* deg64 = nullptr;
  uint32_t* ldeg = nullptr;
  TRY(dmalloc(&deg64, lrows + 1ull, err));
  TRY(dmalloc(&ldeg, lrows, err));
  TRY(dmalloc(&g->meta, lrows, err));
  TRY(dmalloc(&g->row_ptr, lrows + 1ull, err));
  hipLaunchKernelGGL(k_local_rows, dim3(grid_for(lrows + 1ull)), dim3(BLOCK), 0, s, g->perm, g->indeg, g->outdeg, g->dang_w, lrows, g->lA, L, deg64, ldeg, g->meta);
  {
    size_t tb = 0;
    HIPTRY(rocprim::exclusive_scan(nullptr, tb, deg64, g->row_ptr, uint64_t(0), lrows + 1ull, rocprim::plus<uint64_t>(), s));
    TRY(tmp.ensure(tb, err));
    HIPTRY(rocprim::exclusive_scan(tmp.p, tb, deg64, g->row_ptr, uint64_t(0), lrows + 1ull, rocprim::plus<uint64_t>(), s));
  }
  std::vector<uint32_t> hdeg(lrows);
  if (lrows) HIPTRY(hipMemcpyAsync(hdeg.data(), ldeg, 4ull * lrows, hipMemcpyDeviceToHost, s));
  HIPTRY(hipStreamSynchronize(s));
  (void)hipFree(deg64);
  (void)hipFree(ldeg);
  std::vector<uint64_t> hrow(lrows + 1ull, 0);
  for (uint32_t l = 0; l < lrows; ++l) hrow[l + 1] = hrow[l] + hdeg[l];
  // rows are sorted by in-degree (descending) inside each class: sliced rows and hubs lead
  auto lead = [&](uint32_t b, uint32_t e, uint64_t thr) {
    uint32_t i = b;
    while (i < e && hdeg[i] >= thr) ++i;
    return i - b;
  };
  g->sA = lead(0, g->lA, ks);
  g->sB = lead(g->lA, lrows, ks);
  g->hA = std::min(g->sA, lead(0, g->lA, T.kh + 1ull));
  g->hB = std::min(g->sB, lead(g->lA, lrows, T.kh + 1ull));
  g->nS = g->sA + g->sB;
  const SliceRows SR{g->lA, g->sA, g->sB, g->nS};

  // ---- local edges: relabel, keep own rows, sort by (local row, slice, source) ----------
  uint64_t* lk_in = uniq == kA ? kB : kA;  // free buffer
  unsigned long long* d_lc = nullptr;
  TRY(dmalloc(&d_lc, 1, err));
  HIPTRY(hipMemsetAsync(d_lc, 0, 8, s));
  if (nnz) hipLaunchKernelGGL(k_relabel, dim3(grid_for(nnz)), dim3(BLOCK), 0, s, uniq, nnz, nb, inv, g->indeg, ks, L, d_lc, lk_in);
  uint64_t lnnz = nnz;
  if (p > 1) {
    HIPTRY(hipMemcpyAsync(&lnnz, d_lc, 8, hipMemcpyDeviceToHost, s));
    HIPTRY(hipStreamSynchronize(s));
  }
  (void)hipFree(d_lc);
  g->lnnz = lnnz;
  uint64_t* lk_sorted = nullptr;
  {
    rocprim::double_buffer<uint64_t> db(lk_in, uniq);
    size_t tb = 0;
    HIPTRY(rocprim::radix_sort_keys(nullptr, tb, db, lnnz, 0, key_bits, s));
    TRY(tmp.ensure(tb, err));
    if (lnnz) HIPTRY(rocprim::radix_sort_keys(tmp.p, tb, db, lnnz, 0, key_bits, s));
    lk_sorted = db.current();
  }
  TRY(dmalloc(&g->col, lnnz, err));
  uint32_t* cnt = nullptr;
  TRY(dmalloc(&cnt, static_cast<size_t>(NSLICE) * g->nS, err));
  if (g->nS) HIPTRY(hipMemsetAsync(cnt, 0, 4ull * NSLICE * g->nS, s));
  if (lnnz) hipLaunchKernelGGL(k_col, dim3(grid_for(lnnz)), dim3(BLOCK), 0, s, lk_sorted, lnnz, nb, L, SR, g->col, cnt);
  TRY(dmalloc(&g->sb, (NSLICE + 1ull) * g->nS, err));
  if (g->nS) hipLaunchKernelGGL(k_slice_prefix, dim3(grid_for(g->nS)), dim3(BLOCK), 0, s, cnt, g->nS, g->sb);
  HIPTRY(hipStreamSynchronize(s));
  HIPTRY(hipGetLastError());
  (void)hipFree(cnt);
  (void)hipFree(kA);
  (void)hipFree(kB);
  kA = kB = nullptr;
  (void)hipFree(vid);
  TRY(dmalloc(&g->part, static_cast<size_t>(NSLICE) * g->nS, err));

  // ---- schedule ---------------------------------------------------------------------------
  // hub rows' slice offsets on the host (sliced hubs are split per slice into segments)
  std::vector<uint32_t> hsb;  // [9][hA+hB]
  const uint32_t nh_s = g->hA + g->hB;
  if (nh_s) {
    hsb.resize((NSLICE + 1ull) * nh_s);
    for (int j = 0; j <= NSLICE; ++j) {
      if (g->hA) HIPTRY(hipMemcpyAsync(&hsb[j * nh_s], g->sb + static_cast<uint64_t>(j) * g->nS, 4ull * g->hA, hipMemcpyDeviceToHost, s));
      if (g->hB) HIPTRY(hipMemcpyAsync(&hsb[j * nh_s + g->hA], g->sb + static_cast<uint64_t>(j) * g->nS + g->sA, 4ull * g->hB, hipMemcpyDeviceToHost, s));
    }
    HIPTRY(hipStreamSynchronize(s));
  }
  uint32_t next_part = 0;
  // (a) slice launch over sliced rows: kinds by the expected per-slice length k/8
  {
    std::vector<std::vector<HubSeg>> lists(NSLICE);
    uint32_t tiles = 0, hub_tiles = 0;
    for (int cls = 0; cls < 2; ++cls) {
      const uint32_t r0 = cls ? g->lA : 0;
      const uint32_t nsl = cls ? g->sB : g->sA, nhub = cls ? g->hB : g->hA;
      const uint32_t srow0 = cls ? g->sA : 0, hub_i0 = cls ? g->hA : 0;
      if (nhub) {  // hub rows: per-slice segment lists, padded to equal length
        Bin b{};
        b.block_begin = tiles;
        b.row_begin = r0;
        b.row_end = r0 + nhub;
        b.kind = KIND_HUB;
        b.cls = static_cast<uint16_t>(cls);
        b.seg_begin = hub_tiles;
        b.srow_begin = srow0;
        size_t before[NSLICE];
        for (int j = 0; j < NSLICE; ++j) before[j] = lists[j].size();
        for (uint32_t i = 0; i < nhub; ++i) {
          const uint32_t l = r0 + i;
          HubRow h{l, next_part, 0, static_cast<uint32_t>(cls)};
          for (int j = 0; j < NSLICE; ++j) {
            const uint64_t e0 = hrow[l] + hsb[j * nh_s + hub_i0 + i];
            const uint64_t e1 = hrow[l] + hsb[(j + 1) * nh_s + hub_i0 + i];
            for (uint64_t e = e0; e < e1; e += T.seg)
              lists[j].push_back({e, std::min<uint64_t>(e + T.seg, e1), next_part++, 0});
          }
          h.part_end = next_part;
          g->hubs.push_back(h);
        }
        size_t T_ = 0;
        for (int j = 0; j < NSLICE; ++j) T_ = std::max(T_, lists[j].size() - before[j]);
        for (int j = 0; j < NSLICE; ++j)
          while (lists[j].size() - before[j] < T_) lists[j].push_back({0, 0, 0xFFFFFFFFu, 0});
        tiles += static_cast<uint32_t>(T_);
        hub_tiles += static_cast<uint32_t>(T_);
        g->sbins.push_back(b);
        g->sbin_edges.push_back(hrow[r0 + nhub] - hrow[r0]);
      }
      uint32_t i = nhub;
      while (i < nsl) {  // non-hub sliced rows: runs of equal kind
        const uint16_t kd = kind_for((hdeg[r0 + i] + NSLICE - 1) / NSLICE, T);
        uint32_t e = i + 1;
        while (e < nsl && kind_for((hdeg[r0 + e] + NSLICE - 1) / NSLICE, T) == kd) ++e;
        Bin b{};
        b.block_begin = tiles;
        b.row_begin = r0 + i;
        b.row_end = r0 + e;
        b.kind = kd;
        b.cls = static_cast<uint16_t>(cls);
        b.srow_begin = srow0 + i;
        const uint32_t rows = e - i;
        tiles += kd == KIND_BLOCK ? rows : (rows + (64u >> kd) - 1) / (64u >> kd);
        g->sbins.push_back(b);
        g->sbin_edges.push_back(hrow[r0 + e] - hrow[r0 + i]);
        i = e;
      }
    }
    g->slice_tiles = tiles;
    g->hub_tiles = hub_tiles;
    std::vector<HubSeg> flat(static_cast<size_t>(NSLICE) * hub_tiles);
    for (int j = 0; j < NSLICE; ++j)
      for (uint32_t t = 0; t < hub_tiles; ++t) flat[static_cast<size_t>(j) * hub_tiles + t] = lists[j][t];
    TRY(dmalloc(&g->d_ssegs, flat.size(), err));
    if (!flat.empty()) HIPTRY(hipMemcpyAsync(g->d_ssegs, flat.data(), flat.size() * sizeof(HubSeg), hipMemcpyHostToDevice, s));
    TRY(dmalloc(&g->d_sbins, g->sbins.size(), err));
    if (!g->sbins.empty()) HIPTRY(hipMemcpyAsync(g->d_sbins, g->sbins.data(), g->sbins.size() * sizeof(Bin), hipMemcpyHostToDevice, s));
  }
  // (b) row launch: combine bins for sliced non-hub rows, then unsliced rows by kind
  {
    struct Run { uint16_t kind, cls; uint32_t b, e, srow; };
    std::vector<Run> runs;
    for (int cls = 0; cls < 2; ++cls) {
      const uint32_t r0 = cls ? g->lA : 0;
      const uint32_t nsl = cls ? g->sB : g->sA, nhub = cls ? g->hB : g->hA;
      const uint32_t srow0 = cls ? g->sA : 0;
      if (nsl > nhub) runs.push_back({KIND_COMBINE, static_cast<uint16_t>(cls), r0 + nhub, r0 + nsl, srow0 + nhub});
      const uint32_t e0 = cls ? lrows : g->lA;
      uint32_t i = r0 + nsl;
      while (i < e0) {
        const uint16_t kd = hdeg[i] > T.kh ? static_cast<uint16_t>(KIND_HUB) : kind_for(hdeg[i], T);
        uint32_t e = i + 1;
        while (e < e0 && (hdeg[e] > T.kh ? static_cast<uint16_t>(KIND_HUB) : kind_for(hdeg[e], T)) == kd) ++e;
        runs.push_back({kd, static_cast<uint16_t>(cls), i, e, 0});
        i = e;
      }
    }
    std::stable_sort(runs.begin(), runs.end(), [](const Run& a, const Run& b) {
      auto w = [](uint16_t k) { return k == KIND_COMBINE ? 100 : static_cast<int>(k); };
      return w(a.kind) > w(b.kind);
    });
    std::vector<HubSeg> segs;
    uint32_t blocks = 0;
    for (const Run& r : runs) {
      Bin b{};
      b.block_begin = blocks;
      b.row_begin = r.b;
      b.row_end = r.e;
      b.kind = r.kind;
      b.cls = r.cls;
      b.srow_begin = r.srow;
      b.seg_begin = static_cast<uint32_t>(segs.size());
      if (r.kind == KIND_HUB) {
        for (uint32_t l = r.b; l < r.e; ++l) {
          HubRow h{l, next_part, 0, r.cls};
          for (uint64_t e = hrow[l]; e < hrow[l + 1]; e += T.seg)
            segs.push_back({e, std::min<uint64_t>(e + T.seg, hrow[l + 1]), next_part++, 0});
          h.part_end = next_part;
          g->hubs.push_back(h);
        }
        blocks += static_cast<uint32_t>(segs.size()) - b.seg_begin;
      } else if (r.kind == KIND_BLOCK) {
        blocks += r.e - r.b;
      } else if (r.kind == KIND_COMBINE) {
        blocks += (r.e - r.b + BLOCK - 1) / BLOCK;
      } else {
        const uint32_t rpb = BLOCK >> r.kind;
        blocks += (r.e - r.b + rpb - 1) / rpb;
      }
      g->bins.push_back(b);
      g->bin_edges.push_back(hrow[r.e] - hrow[r.b]);
    }
    g->total_blocks = blocks;
    TRY(dmalloc(&g->d_bins, g->bins.size(), err));
    if (!g->bins.empty()) HIPTRY(hipMemcpyAsync(g->d_bins, g->bins.data(), g->bins.size() * sizeof(Bin), hipMemcpyHostToDevice, s));
    TRY(dmalloc(&g->d_segs, segs.size(), err));
    if (!segs.empty()) HIPTRY(hipMemcpyAsync(g->d_segs, segs.data(), segs.size() * sizeof(HubSeg), hipMemcpyHostToDevice, s));
  }
  g->n_parts = next_part;
  TRY(dmalloc(&g->d_hubs, g->hubs.size(), err));
  if (!g->hubs.empty()) HIPTRY(hipMemcpyAsync(g->d_hubs, g->hubs.data(), g->hubs.size() * sizeof(HubRow), hipMemcpyHostToDevice, s));
  TRY(dmalloc(&g->hub_part, next_part, err));

  // ---- iteration buffers ----------------------------------------------------------------
  TRY(dmalloc(&g->r_loc[0], lrows, err));
  TRY(dmalloc(&g->r_loc[1], lrows, err));
  TRY(dmalloc(&g->r_full, n, err));
  TRY(dmalloc(&g->shards, static_cast<size_t>(NSHARD) * REC_WORDS, err));
  TRY(dmalloc(&g->rec_local, REC_WORDS, err));
  TRY(dmalloc(&g->rec_all, static_cast<size_t>(p) * REC_WORDS, err));
  TRY(dmalloc(&g->state, 1, err));
  HIPTRY(hipMemsetAsync(g->shards, 0, 8ull * NSHARD * REC_WORDS, s));
  HIPTRY(hipMemsetAsync(g->r_loc[0], 0, 8ull * (lrows ? lrows : 1), s));
  HIPTRY(hipMemsetAsync(g->r_loc[1], 0, 8ull * (lrows ? lrows : 1), s));
  HIPTRY(hipStreamSynchronize(s));
  HIPTRY(hipGetLastError());
  g->built = true;
  g->ms_build = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return PR_OK;
}

int dev_reset_state(DevGraph* g, hipStream_t s) {
  std::string* err = nullptr;
  IterState st{};
  st.a = g->n_tot ? static_cast<double>(g->W0) / static_cast<double>(g->n_tot) : 0.0;
  st.dcnt = g->W0;
  HIPTRY(hipMemcpyAsync(g->state, &st, sizeof(st), hipMemcpyHostToDevice, s));
  HIPTRY(hipMemsetAsync(g->shards, 0, 8ull * NSHARD * REC_WORDS, s));
  return PR_OK;
}

double* dev_x_out(DevGraph* g, int t) { return g->xbuf[(t - 1) & 1]; }

namespace {

// launch helpers for both grids (template dispatch on MODE / NT)
void launch_rows(const DevGraph* g, StepArgs A, int mode, uint32_t base, uint32_t nblk,
                 hipStream_t s) {
  A.block_base = base;
  const dim3 gr(nblk), bl(BLOCK);
  if (g->tune.nt) {
    if (mode == 0) hipLaunchKernelGGL((spmv_round<0, 1>), gr, bl, 0, s, A);
    else if (mode == 1) hipLaunchKernelGGL((spmv_round<1, 1>), gr, bl, 0, s, A);
    else hipLaunchKernelGGL((spmv_round<2, 1>), gr, bl, 0, s, A);
  } else {
    if (mode == 0) hipLaunchKernelGGL((spmv_round<0, 0>), gr, bl, 0, s, A);
    else if (mode == 1) hipLaunchKernelGGL((spmv_round<1, 0>), gr, bl, 0, s, A);
    else hipLaunchKernelGGL((spmv_round<2, 0>), gr, bl, 0, s, A);
  }
}
void launch_slices(const DevGraph* g, StepArgs A, uint32_t t0, uint32_t t1, hipStream_t s) {
  A.block_base = t0;
  A.tile_end = t1;
  const bool hot = A.hot_n > 0;
  const size_t lds = hot ? 8ull * A.hot_n : 0;
  // persistent grid: 32 CUs per XCD; one 1024-thread block per CU with the LDS copy of the
  // hot x prefix, two without it
  const dim3 gr(NSLICE * 32 * (hot ? 1 : 2)), bl(SLICE_BLOCK);
  static bool attr_set = false;  // allow the >64 KB dynamic LDS request
  if (hot && !attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&spmv_slices<0, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&spmv_slices<1, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  if (g->tune.nt) {
    if (hot) hipLaunchKernelGGL((spmv_slices<1, true>), gr, bl, lds, s, A);
    else hipLaunchKernelGGL((spmv_slices<1, false>), gr, bl, 0, s, A);
  } else {
    if (hot) hipLaunchKernelGGL((spmv_slices<0, true>), gr, bl, lds, s, A);
    else hipLaunchKernelGGL((spmv_slices<0, false>), gr, bl, 0, s, A);
  }
}

}  // namespace

int dev_round_compute(DevGraph* g, int t, int mode, hipStream_t s, hipEvent_t ev0,
                      hipEvent_t ev1) {
  std::string* err = nullptr;
  StepArgs A{};
  A.row_ptr = g->row_ptr;
  A.col = g->col;
  A.meta = g->meta;
  A.x_in = t == 1 ? g->x_init : g->xbuf[t & 1];
  A.x_out = dev_x_out(g, t) + static_cast<uint64_t>(g->rank) * g->maxA;
  A.r_old = t == 1 ? nullptr : g->r_loc[(t - 1) & 1];
  A.r_out = g->r_loc[t & 1];
  A.hub_part = g->hub_part;
  A.hubs = g->d_hubs;
  A.st = g->state;
  A.shards = g->shards;
  A.sb = g->sb;
  A.part = g->part;
  A.nS = g->nS;
  A.hub_tiles = g->hub_tiles;
  A.colmask = g->tune.colmask;
  A.p = static_cast<uint32_t>(g->p);
  A.rank = static_cast<uint32_t>(g->rank);
  A.sm = g->sm ? 1u : 0u;
  A.SL = g->SL;
  A.hot_n = g->sm ? std::min(g->tune.hot_lds, g->SL) : 0u;
  for (int j = 0; j < NSLICE; ++j)
    A.hot_base[j] = g->sm ? (j % g->p) * g->maxA + (j / g->p) * g->SL : 0u;
  StepArgs AS = A;  // slice launch
  AS.bins = g->d_sbins;
  AS.nbins = static_cast<int>(g->sbins.size());
  AS.segs = g->d_ssegs;
  A.bins = g->d_bins;
  A.nbins = static_cast<int>(g->bins.size());
  A.segs = g->d_segs;
  if (ev0) HIPTRY(hipEventRecord(ev0, s));
  if (g->tune.split) {
    // timing mode: one launch per bin, each bracketed by events (DevGraph::split_ms)
    const size_t nsb = g->sbins.size(), nrb = g->bins.size();
    if (g->split_ev.empty()) {
      g->split_ev.resize(2 * (nsb + nrb));
      for (auto& e : g->split_ev) HIPTRY(hipEventCreate(&e));
      g->split_ms.assign(nsb + nrb, 0.0);
    }
    for (size_t i = 0; i < nsb + nrb; ++i) {
      const bool sl = i < nsb;
      const std::vector<Bin>& bv = sl ? g->sbins : g->bins;
      const size_t k = sl ? i : i - nsb;
      const uint32_t tot = sl ? g->slice_tiles : g->total_blocks;
      const uint32_t b0 = bv[k].block_begin;
      const uint32_t b1 = k + 1 < bv.size() ? bv[k + 1].block_begin : tot;
      HIPTRY(hipEventRecord(g->split_ev[2 * i], s));
      if (b1 > b0) {
        if (sl) launch_slices(g, AS, b0, b1, s);
        else launch_rows(g, A, mode, b0, b1 - b0, s);
      }
      HIPTRY(hipEventRecord(g->split_ev[2 * i + 1], s));
    }
    HIPTRY(hipStreamSynchronize(s));
    for (size_t i = 0; i < nsb + nrb; ++i) {
      float ms = 0.f;
      HIPTRY(hipEventElapsedTime(&ms, g->split_ev[2 * i], g->split_ev[2 * i + 1]));
      g->split_ms[i] += ms;
    }
  } else {
    if (g->slice_tiles) launch_slices(g, AS, 0, g->slice_tiles, s);
    if (g->total_blocks) launch_rows(g, A, mode, 0, g->total_blocks, s);
  }
  if (ev1) HIPTRY(hipEventRecord(ev1, s));
  if (!g->hubs.empty()) {
    const uint32_t nh = static_cast<uint32_t>(g->hubs.size());
    if (mode == 0) hipLaunchKernelGGL(hub_round<0>, dim3(nh), dim3(BLOCK), 0, s, A);
    else if (mode == 1) hipLaunchKernelGGL(hub_round<1>, dim3(nh), dim3(BLOCK), 0, s, A);
    else hipLaunchKernelGGL(hub_round<2>, dim3(nh), dim3(BLOCK), 0, s, A);
  }
  hipLaunchKernelGGL(reduce_shards, dim3(1), dim3(BLOCK), 0, s, g->shards, g->rec_local);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_round_finalize(DevGraph* g, int t, bool tracked, hipStream_t s) {
  std::string* err = nullptr;
  const uint64_t* rec = g->p > 1 ? g->rec_all : g->rec_local;
  // round 1 starts from r^0 == 1 on every page: pages that are not rows drop to 0 (|dr|=1)
  const uint64_t extra = (t == 1 && g->rank == 0) ? static_cast<uint64_t>(g->n - g->R) : 0;
  hipLaunchKernelGGL(finalize_round, dim3(1), dim3(64), 0, s, rec, g->p, t, g->n_tot, extra, tracked ? 1 : 0, g->state);
  HIPTRY(hipGetLastError());
  return PR_OK;
}

int dev_scatter_ranks(DevGraph* g, int iterations, hipStream_t s) {
  std::string* err = nullptr;
  const uint32_t n = g->n;
  HIPTRY(hipMemsetAsync(g->r_full, 0, 8ull * (n ? n : 1), s));
  if (iterations == 0) {
    if (g->rank == 0 && n) hipLaunchKernelGGL(k_sources_one, dim3(grid_for(n)), dim3(BLOCK), 0, s, g->outdeg, n, g->r_full);
  } else if (g->lrows) {
    hipLaunchKernelGGL(k_scatter_ranks, dim3(grid_for(g->lrows)), dim3(BLOCK), 0, s, g->perm, g->r_loc[iterations & 1], g->lrows, layout_of(g), g->r_full);
  }
  HIPTRY(hipGetLastError());
  return PR_OK;
}

}  // namespace prmi
