// Host-side sanitizer run of the library's host-only code (tests/test_asan_host.py):
// csrc/hybrd.cpp (the fsolve restatement) and csrc/probes.cpp (the MT19937
// binomial probe stream) built with -fsanitize=address,undefined and driven on
// a few systems and on split / whole probe draws.  GPU code is out of reach of
// the sanitizers on this pool; this covers the host code the GPU tests call.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "sgvamp_hip.h"

extern "C" int sgv_probe_draw(uint32_t* key, int32_t* pos, int64_t n, int64_t lo, int64_t hi,
                              int8_t* out);

static int rosen(void*, int n, const double* x, double* f) {
  (void)n;
  f[0] = 10.0 * (x[1] - x[0] * x[0]);
  f[1] = 1.0 - x[0];
  return 0;
}
static int trig(void*, int n, const double* x, double* f) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += std::cos(x[i]);
  for (int i = 0; i < n; ++i) f[i] = n - s + (i + 1) * (1.0 - std::cos(x[i])) - std::sin(x[i]);
  return 0;
}
static int rootless(void*, int n, const double* x, double* f) {
  for (int i = 0; i < n; ++i) f[i] = x[i] * x[i] + 1.0;
  return 0;
}
static int stop_early(void* u, int n, const double* x, double* f) {
  int* calls = (int*)u;
  if (++*calls > 3) return -1;
  return trig(nullptr, n, x, f);
}

static void seed_mt(uint32_t* key, uint32_t s) {   // the standard MT19937 init_genrand
  key[0] = s;
  for (int i = 1; i < 624; ++i) key[i] = 1812433253u * (key[i - 1] ^ (key[i - 1] >> 30)) + i;
}

int main() {
  int bad = 0;
  {
    double x[2] = {-1.2, 1.0}, f[2];
    int nfev = 0;
    const int ier = sgv_fsolve(2, rosen, nullptr, x, f, &nfev);
    std::printf("rosenbrock ier=%d nfev=%d x=(%.6f, %.6f)\n", ier, nfev, x[0], x[1]);
    bad += ier != 1 || std::fabs(x[0] - 1.0) > 1e-8;
  }
  for (int n : {1, 3, 10, 40}) {
    std::vector<double> x(n, 1.0 / n), f(n);
    int nfev = 0;
    const int ier = sgv_fsolve(n, trig, nullptr, x.data(), f.data(), &nfev);
    std::printf("trig n=%d ier=%d nfev=%d\n", n, ier, nfev);
    bad += ier < 1 || ier > 5;
  }
  {
    double x[3] = {1.0, 2.0, 3.0}, f[3];
    int nfev = 0;
    const int ier = sgv_fsolve(3, rootless, nullptr, x, f, &nfev);
    std::printf("rootless ier=%d nfev=%d\n", ier, nfev);
    bad += ier == 1;
  }
  {
    double x[4] = {0.1, 0.2, 0.3, 0.4}, f[4];
    int nfev = 0, calls = 0;
    const int ier = sgv_fsolve(4, stop_early, &calls, x, f, &nfev);
    std::printf("stopped ier=%d nfev=%d\n", ier, nfev);
  }
  // probe stream: one call draws samples [lo, hi) of a stream of n (2 words
  // each) and leaves the key 2n words on; the pieces [0, a), [a, b), [b, n)
  // drawn from copies of one state equal the whole draw, every state after
  // equals the whole draw's, at even and odd stream positions
  const int64_t n = 5000;
  for (int32_t p0 : {624, 0, 1, 17}) {
    for (int64_t a : {0, 1, 311, 624, 1247}) {
      for (int64_t b : {a, a + 1, a + 700, n}) {
        if (b > n) continue;
        uint32_t k0[624];
        seed_mt(k0, 12345u);
        std::vector<int8_t> whole(n), parts(n);
        uint32_t kw[624];
        std::memcpy(kw, k0, sizeof k0);
        int32_t pw = p0;
        bad += sgv_probe_draw(kw, &pw, n, 0, n, whole.data()) != 0;
        const int64_t cut[4] = {0, a, b, n};
        for (int s = 0; s < 3; ++s) {
          uint32_t k[624];
          std::memcpy(k, k0, sizeof k0);
          int32_t p = p0;
          bad += sgv_probe_draw(k, &p, n, cut[s], cut[s + 1], parts.data() + cut[s]) != 0;
          bad += p != pw || std::memcmp(k, kw, sizeof k) != 0;
        }
        bad += std::memcmp(whole.data(), parts.data(), n) != 0;
      }
    }
  }
  {   // argument checks
    uint32_t k[624];
    seed_mt(k, 1u);
    int32_t p = 624;
    int8_t o[4];
    bad += sgv_probe_draw(k, &p, 4, 3, 2, o) == 0;
    bad += sgv_probe_draw(k, &p, 4, 0, 5, o) == 0;
    bad += sgv_probe_draw(nullptr, &p, 4, 0, 4, o) == 0;
  }
  std::printf(bad ? "FAILED %d\n" : "ok\n", bad);
  return bad ? 1 : 0;
}
