// Correct rounding of the exact superaccumulator (engine.hip: dangling mass, residual, rank
// sum).  SA_NLIMBS limbs of 64 bits each hold a 32-bit chunk plus carries; limb i weighs
// 2^(32 i + SA_EXP0).  Both forms return the value rounded to nearest-even.
//   sa_round_bits: bit by bit (the round-1 form; kept as the reference the fast form is checked
//                  against, tests/test_sa_round.py)
//   sa_round_fast: word by word in fully unrolled loops, so the limb copy stays in registers
//                  (the bit loop indexes a private array at run time, which goes to scratch
//                  memory: ~7 us for a one-thread finalize)
// Compiles as HIP device/host code and as plain C++ (the CPU check).
#pragma once
#include <cmath>
#include <cstdint>

#ifdef __HIPCC__
#define PRMI_HD __host__ __device__
#else
#define PRMI_HD
#endif

namespace prmi {

constexpr int SA_NLIMBS = 10;   // = engine.h SA_LIMBS
constexpr int SA_EXP0 = -96;    // = engine.h SA_BASE_EXP

PRMI_HD inline int sa_clz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __clz(static_cast<int>(x));
#else
  return __builtin_clz(x);
#endif
}

PRMI_HD inline void sa_words(const uint64_t* limb, uint32_t (&c)[SA_NLIMBS + 2]) {
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < SA_NLIMBS; ++i) {
    const uint64_t t = limb[i] + carry;
    c[i] = static_cast<uint32_t>(t);
    carry = t >> 32;
  }
  c[SA_NLIMBS] = static_cast<uint32_t>(carry);
  c[SA_NLIMBS + 1] = static_cast<uint32_t>(carry >> 32);
}

PRMI_HD inline double sa_round_bits(const uint64_t* limb) {
  uint32_t c[SA_NLIMBS + 2];
  sa_words(limb, c);
  int top = -1;
  for (int i = SA_NLIMBS + 1; i >= 0; --i)
    if (c[i]) {
      top = i * 32 + 31 - sa_clz32(c[i]);
      break;
    }
  if (top < 0) return 0.0;
  auto bit = [&](int p) -> uint32_t { return p < 0 ? 0u : ((c[p >> 5] >> (p & 31)) & 1u); };
  if (top < 53) {
    uint64_t m = 0;
    for (int p = top; p >= 0; --p) m = (m << 1) | bit(p);
    return ldexp(static_cast<double>(m), SA_EXP0);
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
  return ldexp(static_cast<double>(m), lowest + SA_EXP0);
}

PRMI_HD inline double sa_round_fast(const uint64_t* limb) {
  constexpr int NW = SA_NLIMBS + 2;
  uint32_t c[NW];
  sa_words(limb, c);
  int top = -1;  // highest set bit: the last nonzero word in ascending order
#pragma unroll
  for (int i = 0; i < NW; ++i)
    if (c[i]) top = i * 32 + 31 - sa_clz32(c[i]);
  if (top < 0) return 0.0;
  if (top < 53)  // only words 0 and 1 can be nonzero
    return ldexp(static_cast<double>((static_cast<uint64_t>(c[1]) << 32) | c[0]), SA_EXP0);
  int lowest = top - 52;  // m = bits [lowest, top], round bit = lowest - 1 (>= 0)
  const int rp = lowest - 1;
  uint64_t m = 0;
  uint32_t rb = 0, sticky = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int b0 = i * 32;
    const uint64_t w = c[i];
    const int d = b0 - lowest;  // where the word's bit 0 lands relative to bit `lowest`
    if (d >= 0) m |= d < 64 ? (w << d) : 0ull;  // (bits past 63 lie above top: zero)
    else if (d > -32) m |= w >> (-d);
    if (rp >= b0 && rp < b0 + 32) rb = (c[i] >> (rp - b0)) & 1u;
    if (b0 + 32 <= rp) sticky |= c[i];
    else if (b0 < rp) sticky |= c[i] & ((1u << (rp - b0)) - 1u);
  }
  if (rb && (sticky || (m & 1))) {
    m += 1;
    if (m == (1ull << 53)) {
      m >>= 1;
      lowest += 1;
    }
  }
  return ldexp(static_cast<double>(m), lowest + SA_EXP0);
}

}  // namespace prmi
