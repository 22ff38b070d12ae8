// Probe: f64 MFMA / VALU FMA rates and lane layouts on gfx950.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// layout check: A[m][k] = 100*m + k, B[k][n] = (k==n? 1 : 0) etc. computed on host
__global__ void k_layout16(const double* A, const double* B, double* D) {
  const int l = threadIdx.x;
  const double a = A[(l & 15) * 4 + (l >> 4)];   // A[m=l&15][k=l>>4]
  const double b = B[(l >> 4) * 16 + (l & 15)];  // B[k=l>>4][n=l&15]
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}

__global__ void k_layout4(const double* A, const double* B, double* D) {
  const int l = threadIdx.x;
  double c = 0;
  c = __builtin_amdgcn_mfma_f64_4x4x4f64(A[l], B[l], c, 0, 0, 0);
  D[l] = c;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma_rate(double* out, int iters, long long* cyc) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  d4 c[NACC];
  for (int i = 0; i < NACC; ++i) c[i] = d4{0, 0, 0, 0};
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
  }
  long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma4_rate(double* out, int iters, long long* cyc) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double c[NACC];
  for (int i = 0; i < NACC; ++i) c[i] = 0;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[i], 0, 0, 0);
  }
  long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_fma_rate(double* out, int iters, long long* cyc) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double c[NACC];
  for (int i = 0; i < NACC; ++i) c[i] = i;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) c[i] = __builtin_fma(a, c[i], b);
  }
  long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double *dA, *dB, *dD, *dout;
  long long* dcyc;
  CK(hipMalloc(&dA, 64 * 8 * 4));
  CK(hipMalloc(&dB, 64 * 8 * 4));
  CK(hipMalloc(&dD, 256 * 8));
  CK(hipMalloc(&dout, 1 << 24));
  CK(hipMalloc(&dcyc, 8));
  // ---- 16x16x4 layout: A 16x4, B 4x16
  std::vector<double> A(64), B(64), D(256);
  for (int m = 0; m < 16; ++m)
    for (int k = 0; k < 4; ++k) A[m * 4 + k] = (m + 1) * 1000.0 + (k + 1);
  for (int k = 0; k < 4; ++k)
    for (int n = 0; n < 16; ++n) B[k * 16 + n] = (k == 0 ? 1.0 : 0.0) * (n + 1) + (k == 1 ? 1e-3 * (n + 1) : 0.0);
  CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
  k_layout16<<<1, 64>>>(dA, dB, dD);
  CK(hipMemcpy(D.data(), dD, 256 * 8, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int m = (l >> 4) + 4 * r, n = l & 15;
      double ref = 0;
      for (int k = 0; k < 4; ++k) ref += A[m * 4 + k] * B[k * 16 + n];
      if (D[l * 4 + r] != ref) ++bad;
    }
  printf("layout16x16x4 (row=(l>>4)+4r, col=l&15): %s (%d bad)\n", bad ? "MISMATCH" : "ok", bad);
  // ---- 4x4x4 (4 blocks?) probe: print raw result for A = onehot patterns
  for (int l = 0; l < 64; ++l) A[l] = l + 1;
  for (int trial = 0; trial < 0; trial += 1) {
    std::vector<double> Bv(64, 0.0);
    Bv[trial] = 1.0;
    CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, Bv.data(), 512, hipMemcpyHostToDevice));
    k_layout4<<<1, 64>>>(dA, dB, dD);
    std::vector<double> R(64);
    CK(hipMemcpy(R.data(), dD, 512, hipMemcpyDeviceToHost));
    printf("4x4x4 B-onehot lane %2d ->", trial);
    for (int l = 0; l < 64; ++l)
      if (R[l] != 0) printf(" D[%d]=A%d", l, (int)R[l] - 1);
    printf("\n");
  }
  // ---- rates
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20000;
  for (int wps = 1; wps <= 2; ++wps) {
    const int nblk = 256 * wps;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      k_mfma_rate<8><<<nblk, 256>>>(dout, iters, dcyc);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
    }
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long cyc;
    CK(hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost));
    const double flops = 2.0 * 16 * 16 * 4 * 8.0 * iters * nblk * 4;
    printf("mfma_f64_16x16x4 waves/SIMD=%d: %.3f ms  %.1f TF  cycles/mfma(clock64)=%.1f\n", wps, ms,
           flops / ms / 1e9, (double)cyc / (iters * 8.0));
  }
  for (int wps = 1; wps <= 2; ++wps) {
    const int nblk = 256 * wps;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      k_mfma4_rate<8><<<nblk, 256>>>(dout, iters, dcyc);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
    }
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long cyc;
    CK(hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost));
    const double flops = 2.0 * 4 * 4 * 4 * 4 * 8.0 * iters * nblk * 4;
    printf("mfma_f64_4x4x4 (4 blocks) waves/SIMD=%d: %.3f ms  %.1f TF  cycles/mfma(clock64)=%.1f\n", wps,
           ms, flops / ms / 1e9, (double)cyc / (iters * 8.0));
  }
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int nblk = 256 * wps;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      k_fma_rate<16><<<nblk, 256>>>(dout, iters, dcyc);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
    }
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long cyc;
    CK(hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost));
    const double flops = 2.0 * 16 * iters * (double)nblk * 256;
    printf("v_fma_f64 waves/SIMD=%d: %.3f ms  %.1f TF  cycles/fma(clock64)=%.2f\n", wps, ms,
           flops / ms / 1e9, (double)cyc / (iters * 16.0));
  }
  // dependent-accumulator latency: one wave per SIMD, NACC independent chains
  // (cycles per MFMA at NACC = 1 is the dependent issue-to-issue latency)
  auto chains = [&](auto kern, const char* name, int nacc) {
    const int nblk = 256;
    kern<<<nblk, 256>>>(dout, iters, dcyc);
    CK(hipDeviceSynchronize());
    long long cyc;
    CK(hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost));
    printf("%s chains=%d: cycles/mfma(clock64)=%.1f\n", name, nacc, (double)cyc / (iters * (double)nacc));
  };
  chains(k_mfma4_rate<1>, "mfma_f64_4x4x4", 1);
  chains(k_mfma4_rate<2>, "mfma_f64_4x4x4", 2);
  chains(k_mfma4_rate<4>, "mfma_f64_4x4x4", 4);
  chains(k_mfma4_rate<8>, "mfma_f64_4x4x4", 8);
  chains(k_mfma_rate<1>, "mfma_f64_16x16x4", 1);
  chains(k_mfma_rate<2>, "mfma_f64_16x16x4", 2);
  chains(k_mfma_rate<4>, "mfma_f64_16x16x4", 4);
  chains(k_mfma_rate<8>, "mfma_f64_16x16x4", 8);
  printf("done\n");
  return 0;
}
