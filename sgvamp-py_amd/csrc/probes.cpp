// Hutchinson probes of the LMMSE step (src/sgvamp.py:326):
//   u = np.random.binomial(p=1/2, n=1, size=M) * 2 - 1
// drawn from the cohort's legacy numpy RandomState stream (MT19937), in C.
//
// numpy's legacy binomial (numpy/random/src/legacy/legacy-distributions.c ->
// random_binomial_inversion for n*p <= 30) with n = 1, p = 1/2 consumes exactly
// one legacy double U per sample and returns 1 iff U > qn, qn = exp(n log q) =
// 0.5 exactly; the legacy double is U = ((a >> 5) * 2^26 + (b >> 6)) / 2^53
// from two consecutive 32-bit outputs a, b.  So u = +1 iff (a >> 5) > 2^26, or
// (a >> 5) == 2^26 and (b >> 6) > 0 -- the stream and the values of
// RandomState.binomial bit for bit (tests/test_abi.py checks against numpy).
//
// A rank draws the whole stream (stream order is the reference's: every rank
// of an M-marker run advances by M samples) but tempers and stores only its own
// slice [lo, hi): outside it the state only advances (twists).  numpy's path
// takes ~35 ns per sample (binomial) -- at M = 1e6 and K = 8 cohorts that is
// 280 ms of host work per VAMP iteration against a ~20 ms GPU step.
#include <algorithm>
#include <cstdint>
#include <cstring>

#include "sgvamp_hip.h"

namespace {

constexpr int MT_N = 624, MT_M = 397;
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;

// numpy mt19937_gen, in vectors of W words: i < N - M reads only old words
// (k[i + 1], k[i + M]); i >= N - M reads k[i + M - N], updated W or more
// positions earlier (N - M = 227 >= W), so increasing order is exact
template <int W>
struct Twist {
  typedef uint32_t V __attribute__((vector_size(4 * W)));
  __attribute__((always_inline)) static inline V ld(const uint32_t* p) {
    V v;
    std::memcpy(&v, p, sizeof v);
    return v;
  }
  __attribute__((always_inline)) static inline V step(V x, V y, V m) {
    const V z = (x & UPPER) | (y & LOWER);
    return m ^ (z >> 1) ^ ((-(z & 1u)) & MATRIX_A);
  }
  __attribute__((always_inline)) static inline void run(uint32_t* k) {
    int i = 0;
    for (; i + W <= MT_N - MT_M; i += W) {
      const V v = step(ld(k + i), ld(k + i + 1), ld(k + i + MT_M));
      std::memcpy(k + i, &v, sizeof v);
    }
    for (; i < MT_N - MT_M; ++i) {
      const uint32_t z = (k[i] & UPPER) | (k[i + 1] & LOWER);
      k[i] = k[i + MT_M] ^ (z >> 1) ^ (-(z & 1u) & MATRIX_A);
    }
    for (; i + W <= MT_N - 1; i += W) {
      const V v = step(ld(k + i), ld(k + i + 1), ld(k + i + (MT_M - MT_N)));
      std::memcpy(k + i, &v, sizeof v);
    }
    for (; i < MT_N - 1; ++i) {
      const uint32_t z = (k[i] & UPPER) | (k[i + 1] & LOWER);
      k[i] = k[i + (MT_M - MT_N)] ^ (z >> 1) ^ (-(z & 1u) & MATRIX_A);
    }
    const uint32_t z = (k[MT_N - 1] & UPPER) | (k[0] & LOWER);
    k[MT_N - 1] = k[MT_M - 1] ^ (z >> 1) ^ (-(z & 1u) & MATRIX_A);
  }
};

__attribute__((target("avx2"))) void twist_avx2(uint32_t* k) { Twist<8>::run(k); }
void twist_sse2(uint32_t* k) { Twist<4>::run(k); }
const bool g_avx2 = __builtin_cpu_supports("avx2");
inline void mt_twist(uint32_t* k) {
  if (g_avx2)
    twist_avx2(k);
  else
    twist_sse2(k);
}

inline uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// advance by `words` 32-bit outputs without using them
inline void mt_skip(uint32_t* k, int32_t& pos, int64_t words) {
  while (words > 0) {
    if (pos >= MT_N) {
      mt_twist(k);
      pos = 0;
    }
    const int64_t adv = words < (int64_t)(MT_N - pos) ? words : (int64_t)(MT_N - pos);
    pos += (int32_t)adv;
    words -= adv;
  }
}

inline uint32_t mt_raw(uint32_t* k, int32_t& pos) {
  if (pos >= MT_N) {
    mt_twist(k);
    pos = 0;
  }
  return k[pos++];
}

// u = +1 iff the legacy double of (a, b) exceeds 0.5 (see the file comment)
inline int8_t probe_of(uint32_t ta, uint32_t braw) {
  const uint32_t a = ta >> 5;
  return (a > (1u << 26) || (a == (1u << 26) && (temper(braw) >> 6) > 0)) ? 1 : -1;
}

}  // namespace

extern "C" int sgv_probe_draw(uint32_t* key, int32_t* pos, int64_t n, int64_t lo, int64_t hi,
                              int8_t* out) {
  if (!key || !pos || n < 0 || lo < 0 || hi < lo || hi > n || (hi > lo && !out) || *pos < 0 ||
      *pos > MT_N)
    return SGV_ERR_ARG;
  int32_t p = *pos;
  mt_skip(key, p, 2 * lo);
  int64_t i = lo;
  if (p % 2 == 0) {   // samples never straddle a block: whole runs of pairs per block
    while (i < hi) {
      if (p >= MT_N) {
        mt_twist(key);
        p = 0;
      }
      const int64_t m = std::min<int64_t>((MT_N - p) / 2, hi - i);
      const uint32_t* w = key + p;
      int8_t* o = out + (i - lo);
      for (int64_t j = 0; j < m; ++j) o[j] = probe_of(temper(w[2 * j]), w[2 * j + 1]);
      p += (int32_t)(2 * m);
      i += m;
    }
  }
  for (; i < hi; ++i) {   // odd stream position (32-bit draws made elsewhere): one by one
    const uint32_t ta = temper(mt_raw(key, p));
    out[i - lo] = probe_of(ta, mt_raw(key, p));
  }
  mt_skip(key, p, 2 * (n - hi));
  *pos = p;
  return SGV_OK;
}
