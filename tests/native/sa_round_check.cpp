// CPU check: sa_round_fast (the device form) against sa_round_bits (the bit-loop form) on
// random superaccumulator states, including carries in every limb and round-to-even ties.
// Prints the number of cases and exits 1 on the first mismatch.  Built by tests/test_sa_round.py.
#include <cstdio>
#include <cstring>
#include <random>
#include "sa_round.h"

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 rng(12345);
  uint64_t limb[prmi::SA_NLIMBS];
  for (long k = 0; k < n; ++k) {
    const int mode = static_cast<int>(k % 6);
    for (int i = 0; i < prmi::SA_NLIMBS; ++i) {
      uint64_t v = rng();
      switch (mode) {
        case 0: v &= 0xFFFFFFFFull; break;                       // canonical chunks
        case 1: break;                                           // full 64-bit carries
        case 2: v = (rng() % 4 == 0) ? (v & 0xFFFFFFFFull) : 0; break;  // sparse
        case 3: v = (i < 2) ? v : 0; break;                      // small values (top < 53 too)
        case 4: v = (rng() & 1) ? 0xFFFFFFFFull : 0; break;      // long carry chains
        default: v = (i == (int)(rng() % prmi::SA_NLIMBS)) ? (v & 0xFFFFFFFFull) : 0; break;
      }
      limb[i] = v;
    }
    if (mode == 5 && (k & 1)) {  // exact tie: 54 significant bits ending in ...1 followed by zeros
      std::memset(limb, 0, sizeof(limb));
      const int w = 2 + static_cast<int>(rng() % 6);
      const uint64_t m = (rng() | (1ull << 53)) & ((1ull << 54) - 1);
      limb[w] = m & 0xFFFFFFFFull;
      limb[w + 1] = m >> 32;
    }
    const double a = prmi::sa_round_bits(limb), b = prmi::sa_round_fast(limb);
    if (std::memcmp(&a, &b, sizeof(double)) != 0) {
      std::printf("MISMATCH case %ld: bits %.17g fast %.17g\n", k, a, b);
      return 1;
    }
  }
  std::printf("ok %ld\n", n);
  return 0;
}
