// Synthetic inputs on the device, following the reference's simulation recipe
// (simulation/sim_gen_phen_mult.py:36-55) with a counter-based RNG so that the
// CPU restatement (oracle/synth_oracle.py) reproduces the genotypes bit for bit:
//   x[i][n] ~ Binomial(2, 0.4): two 32-bit halves of splitmix64(key) compared
//            with floor(0.4 * 2^32); key = seed*C1 + gmarker*C2 + n (mod 2^64)
//   X_std[i][n] = (x - mean_i) / std_i    (population std, exact from counts)
//   G = X_std / sqrt(N);  R_b = G_b G_b^T;  g[n] = sum_i X_std[i][n] beta_i;
//   r_b = G_b y
// Compiled with -ffp-contract=off; the GEMM uses explicit fma.
#include "common.h"

namespace sgv {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int geno(uint64_t seed, int64_t gi, int n) {
  const uint64_t key = seed * 0xD1B54A32D192ED03ull + (uint64_t)gi * 0x9E3779B97F4A7C15ull +
                       (uint64_t)n;
  const uint64_t h = splitmix64(key);
  constexpr uint64_t T = 1717986918ull;  // floor(0.4 * 2^32)
  return (int)((h >> 32) < T) + (int)((h & 0xffffffffull) < T);
}

// one workgroup per marker: exact integer moments -> mean, std
__global__ __launch_bounds__(256) void k_geno_stats(uint64_t seed, int64_t gm0, int nsamp,
                                                    double* __restrict__ mean,
                                                    double* __restrict__ sd) {
  const int i = blockIdx.x;
  long long s1 = 0, s2 = 0;
  for (int n = threadIdx.x; n < nsamp; n += 256) {
    const int x = geno(seed, gm0 + i, n);
    s1 += x;
    s2 += x * x;
  }
  __shared__ long long sm1[256], sm2[256];
  sm1[threadIdx.x] = s1;
  sm2[threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sm1[threadIdx.x] += sm1[threadIdx.x + o];
      sm2[threadIdx.x] += sm2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const long long S1 = sm1[0], S2 = sm2[0], N = nsamp;
    const long long num = N * S2 - S1 * S1;  // N^2 var, exact
    mean[i] = (double)S1 / (double)N;
    sd[i] = sqrt((double)num / ((double)N * (double)N));
  }
}

hipError_t launch_geno_stats(uint64_t seed, int64_t gm0, int n, int nsamp, double* d_mean,
                             double* d_std, hipStream_t st) {
  hipLaunchKernelGGL(k_geno_stats, dim3(n), dim3(256), 0, st, seed, gm0, nsamp, d_mean, d_std);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_geno_G(uint64_t seed, int64_t gm0, int nsamp, int ldg,
                                                const double* __restrict__ mean,
                                                const double* __restrict__ sd,
                                                double* __restrict__ G) {
  const int i = blockIdx.y;
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= ldg) return;
  double v = 0.0;
  if (n < nsamp) {
    const double xs = ((double)geno(seed, gm0 + i, n) - mean[i]) / sd[i];
    v = xs / sqrt((double)nsamp);
  }
  G[(int64_t)i * ldg + n] = v;
}

hipError_t launch_geno_G(uint64_t seed, int64_t gm0, int n, int nsamp, int ldg,
                         const double* d_mean, const double* d_std, double* d_G,
                         hipStream_t st) {
  hipLaunchKernelGGL(k_geno_G, dim3((ldg + 255) / 256, n), dim3(256), 0, st, seed, gm0, nsamp,
                     ldg, d_mean, d_std, d_G);
  return hipGetLastError();
}

// R = G G^T (n x n, symmetric; upper tiles computed, mirrored).  64x64 tiles,
// 256 threads x (4 x 4) outputs, K-steps of 16 staged through LDS.
__global__ __launch_bounds__(256) void k_syrk_nt(const double* __restrict__ G, int n, int kpad,
                                                 int ldg, double* __restrict__ R, int64_t lda,
                                                 int packed, const int64_t* __restrict__ poff,
                                                 const int64_t* __restrict__ pw) {
  const int tj = blockIdx.x, ti = blockIdx.y;
  if (ti > tj) return;
  const int i0 = ti * 64, j0 = tj * 64;
  __shared__ double As[16][64 + 2];
  __shared__ double Bs[16][64 + 2];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  double acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
  for (int k0 = 0; k0 < kpad; k0 += 16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = threadIdx.x + 256 * e;
      const int r = idx >> 4, kk = idx & 15;
      As[kk][r] = (i0 + r < n) ? G[(int64_t)(i0 + r) * ldg + k0 + kk] : 0.0;
      Bs[kk][r] = (j0 + r < n) ? G[(int64_t)(j0 + r) * ldg + k0 + kk] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      double av[4], bv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) av[a] = As[kk][ty + 16 * a];
#pragma unroll
      for (int b = 0; b < 4; ++b) bv[b] = Bs[kk][tx + 16 * b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_fma(av[a], bv[b], acc[a][b]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int i = i0 + ty + 16 * a, j = j0 + tx + 16 * b;
      if (i < n && j < n) {
        if (packed) {
          double* p = sym_addr(R, poff, pw, i, j);
          if (p) *p = acc[a][b];
          p = sym_addr(R, poff, pw, j, i);
          if (p) *p = acc[a][b];
        } else {
          R[(int64_t)i * lda + j] = acc[a][b];
          R[(int64_t)j * lda + i] = acc[a][b];
        }
      }
    }
}

hipError_t launch_syrk_nt(const double* d_G, int n, int nsamp, int ldg, double* d_R, int64_t lda,
                          int packed, const int64_t* d_poff, const int64_t* d_pw, hipStream_t st) {
  const int nt = (n + 63) / 64;
  const int kpad = (nsamp + 15) / 16 * 16;  // <= ldg, zero padded
  hipLaunchKernelGGL(k_syrk_nt, dim3(nt, nt), dim3(256), 0, st, d_G, n, kpad, ldg, d_R, lda,
                     packed, d_poff, d_pw);
  return hipGetLastError();
}

// g[n] = sum_i X_std[i][n] * beta[i]  (simulation/sim_gen_phen_mult.py:44, g = X @ beta)
__global__ __launch_bounds__(256) void k_g_accum(uint64_t seed, int64_t gm0, int nb, int nsamp,
                                                 const double* __restrict__ mean,
                                                 const double* __restrict__ sd,
                                                 const double* __restrict__ beta,
                                                 double* __restrict__ g) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= nsamp) return;
  double s = 0.0;
  for (int i = 0; i < nb; ++i) {
    const double b = beta[i];
    if (b == 0.0) continue;  // exact: adding +0*x changes nothing unless x is inf/nan
    const double xs = ((double)geno(seed, gm0 + i, n) - mean[i]) / sd[i];
    s = s + xs * b;
  }
  g[n] = s;
}

hipError_t launch_g_accum(uint64_t seed, int64_t gm0, int n, int nsamp, const double* d_mean,
                          const double* d_std, const double* d_beta, double* d_g,
                          hipStream_t st) {
  hipLaunchKernelGGL(k_g_accum, dim3((nsamp + 255) / 256), dim3(256), 0, st, seed, gm0, n, nsamp,
                     d_mean, d_std, d_beta, d_g);
  return hipGetLastError();
}

// out[i] = sum_n G[i][n] y[n]  (r = X^T y, sim_gen_phen_mult.py:54); one wave per row
__global__ __launch_bounds__(256) void k_row_dot(const double* __restrict__ G, int n, int nsamp,
                                                 int ldg, const double* __restrict__ y,
                                                 double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  double s = 0.0;
  for (int k = lane; k < nsamp; k += 64) s = __builtin_fma(G[(int64_t)i * ldg + k], y[k], s);
  s = wave_sum(s);
  if (lane == 0) out[i] = s;
}

hipError_t launch_row_dot(const double* d_G, int n, int nsamp, int ldg, const double* d_y,
                          double* d_out, hipStream_t st) {
  hipLaunchKernelGGL(k_row_dot, dim3((n + 3) / 4), dim3(256), 0, st, d_G, n, nsamp, ldg, d_y,
                     d_out);
  return hipGetLastError();
}

}  // namespace sgv
