// Host-side bootstrap draws (bootstrap_disp, apis/imaging_classes.py:8-48 / the notebooks' convergence_test):
// `times` successive calls of CPython's random.sample(range(lo, lo + n), k) from a given Mersenne Twister
// state, bit for bit.  The reference draws with Python's `random`; the product keeps its draws (so a seeded run
// resamples the same passes) but forms them here instead of through ~10^5 interpreted calls per convergence
// test.  The state is CPython's random.getstate()[1]: 624 words + the index, updated in place, so the caller
// hands it back with random.setstate() and the interpreter's generator continues exactly where Python's own
// calls would have left it.
//   genrand_uint32            CPython Modules/_randommodule.c (MT19937, Matsumoto & Nishimura)
//   getrandbits(k <= 32)      genrand_uint32() >> (32 - k)
//   _randbelow(m)             k = m.bit_length(); r = getrandbits(k) until r < m  (0 for m == 0)
//   sample(population, k)     Lib/random.py (3.10): setsize = 21 (+ 4 ** ceil(log(3 k, 4)) for k > 5);
//                             n <= setsize: pool swap-remove, else rejection against a set of taken indices
#include <math.h>
#include <stdint.h>

#include <vector>

#include "dvh_common.h"
#include "dvh.h"

namespace {

struct MT {
  uint32_t* mt;  // [624] words, then [624] = index
  uint32_t next() {
    constexpr int N = 624, M = 397;
    constexpr uint32_t A = 0x9908b0dfU, UP = 0x80000000U, LO = 0x7fffffffU;
    uint32_t idx = mt[N];
    if (idx >= (uint32_t)N) {
      int kk;
      uint32_t y;
      for (kk = 0; kk < N - M; kk++) {
        y = (mt[kk] & UP) | (mt[kk + 1] & LO);
        mt[kk] = mt[kk + M] ^ (y >> 1) ^ ((y & 1U) ? A : 0U);
      }
      for (; kk < N - 1; kk++) {
        y = (mt[kk] & UP) | (mt[kk + 1] & LO);
        mt[kk] = mt[kk + (M - N)] ^ (y >> 1) ^ ((y & 1U) ? A : 0U);
      }
      y = (mt[N - 1] & UP) | (mt[0] & LO);
      mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ ((y & 1U) ? A : 0U);
      idx = 0;
    }
    uint32_t y = mt[idx++];
    mt[N] = idx;
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
  }
  int64_t below(int64_t m) {  // random._randbelow_with_getrandbits (m < 2^32)
    if (m <= 0) return 0;
    int k = 0;
    while ((m >> k) != 0) ++k;  // m.bit_length()
    int64_t r;
    do r = (int64_t)(next() >> (32 - k));
    while (r >= m);
    return r;
  }
};

}  // namespace

DVH_API int dvh_random_sample(uint32_t* state, int64_t lo, int64_t n, int32_t k, int32_t times, int64_t* out) {
  if (!state || (!out && times > 0 && k > 0)) return dvh::set_error(-2, "null pointer argument");
  if (n < 0 || n >= (int64_t)1 << 32) return dvh::set_error(-4, "population size outside [0, 2^32)");
  if (k < 0 || k > n) return dvh::set_error(-2, "Sample larger than population or is negative");
  if (state[624] > 624) return dvh::set_error(-2, "invalid Mersenne Twister index");
  MT g{state};
  int64_t setsize = 21;
  if (k > 5) setsize += (int64_t)pow(4.0, ceil(log((double)k * 3) / log(4.0)));
  std::vector<int64_t> pool;
  std::vector<uint8_t> taken;
  for (int32_t t = 0; t < times; ++t) {
    int64_t* res = out + (int64_t)t * k;
    if (n <= setsize) {
      pool.resize((size_t)n);
      for (int64_t i = 0; i < n; ++i) pool[(size_t)i] = lo + i;
      for (int32_t i = 0; i < k; ++i) {
        const int64_t j = g.below(n - i);
        res[i] = pool[(size_t)j];
        pool[(size_t)j] = pool[(size_t)(n - i - 1)];
      }
    } else {
      taken.assign((size_t)n, 0);
      for (int32_t i = 0; i < k; ++i) {
        int64_t j = g.below(n);
        while (taken[(size_t)j]) j = g.below(n);
        taken[(size_t)j] = 1;
        res[i] = lo + j;
      }
    }
  }
  return 0;
}
