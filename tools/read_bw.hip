// Achievable HBM read bandwidth on this MI355X: stream B bytes once with 16-B
// loads per lane (plain and nontemporal), grid-stride, several occupancies.
//   hipcc -O3 --offload-arch=gfx950 tools/read_bw.hip -o tools/read_bw && tools/read_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void k_read(const d2* __restrict__ p, size_t n, double* out) {
  const size_t tid = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * 256;
  d2 acc = {0.0, 0.0};
  size_t i = tid;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    d2 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      v[u] = NT ? __builtin_nontemporal_load(
                      (const __attribute__((address_space(1))) d2*)(p + i + u * stride))
                : *(const __attribute__((address_space(1))) d2*)(p + i + u * stride);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc += v[u];
  }
  for (; i < n; i += stride) acc += p[i];
  if (acc.x == 12345.678) out[0] = acc.y;   // keep the loads alive
}

// row-chunked pattern like the LD passes: each wave streams 1 KiB-wide rows of a block
template <bool NT>
__global__ __launch_bounds__(256) void k_read_rows(const d2* __restrict__ p, size_t n, int per,
                                                   double* out) {
  const size_t base = (size_t)blockIdx.x * per * 256;
  d2 acc = {0.0, 0.0};
  for (int j = 0; j < per; j += 8) {
    d2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t idx = base + (size_t)(j + u) * 256 + threadIdx.x;
      v[u] = NT ? __builtin_nontemporal_load((const __attribute__((address_space(1))) d2*)(p + idx))
                : *(const __attribute__((address_space(1))) d2*)(p + idx);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  if (acc.x == 12345.678) out[0] = acc.y;
}

// occupancy sweep: U 1-KiB row loads in flight per wave, WGs per CU pinned by
// dynamic LDS (160 KiB / lds_kib)
template <int U>
__global__ __launch_bounds__(256) void k_read_occ(const d2* __restrict__ p, size_t n, int per,
                                                  double* out) {
  extern __shared__ double dyn[];
  const size_t base = (size_t)blockIdx.x * per * 256;
  d2 acc = {0.0, 0.0};
  for (int j = 0; j < per; j += U) {
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = __builtin_nontemporal_load(
          (const __attribute__((address_space(1))) d2*)(p + base + (size_t)(j + u) * 256 + threadIdx.x));
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x == 12345.678) { dyn[threadIdx.x] = acc.y; out[0] = dyn[(threadIdx.x + 1) & 255]; }
}

// LD-pass tile patterns over a row-major matrix with row stride W doubles:
// one WG per 256-row x 1024-column tile; each wave owns 8 consecutive rows per
// sub-sweep.  ROWMAJ = 0: the 8 rows are read together, 1 KiB per row per step
// (k_sym_pass order); ROWMAJ = 1: one row's 8 KiB at a time.
template <int ROWMAJ>
__global__ __launch_bounds__(256) void k_read_tile(const double* __restrict__ p, int W, int ntc,
                                                   double* out) {
  extern __shared__ double dyn[];
  const int tr = blockIdx.x / ntc, tc = blockIdx.x % ntc;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const double* base = p + (size_t)tr * 256 * W + tc * 1024 + 2 * lane;
  d2 acc = {0.0, 0.0};
  for (int sub = 0; sub < 8; ++sub) {
    const int r0 = sub * 32 + wid * 8;
    if (ROWMAJ == 0) {
#pragma unroll 2
      for (int s = 0; s < 8; ++s) {
        d2 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r)
          v[r] = __builtin_nontemporal_load((const __attribute__((address_space(1))) d2*)(
              base + (size_t)(r0 + r) * W + s * 128));
#pragma unroll
        for (int r = 0; r < 8; ++r) acc += v[r];
      }
    } else {
#pragma unroll 2
      for (int r = 0; r < 8; ++r) {
        d2 v[8];
#pragma unroll
        for (int s = 0; s < 8; ++s)
          v[s] = __builtin_nontemporal_load((const __attribute__((address_space(1))) d2*)(
              base + (size_t)(r0 + r) * W + s * 128));
#pragma unroll
        for (int s = 0; s < 8; ++s) acc += v[s];
      }
    }
  }
  if (acc.x == 12345.678) { dyn[threadIdx.x] = acc.y; out[0] = dyn[(threadIdx.x + 1) & 255]; }
}

template <class F>
static void timeit(const char* name, F launch, double bytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("%-40s %8.3f ms  %7.0f GB/s\n", name, best, bytes / best / 1e6);
}

int main() {
  const size_t bytes = (size_t)20 << 30;   // 20 GiB
  const size_t n = bytes / 16;
  d2* p;
  double* out;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(p, 0, bytes));
  int cus = 256;
  for (int wpc : {8, 16, 32, 64}) {
    const int grid = cus * wpc;
    char nm[64];
    snprintf(nm, sizeof nm, "grid-stride u4 plain  blocks/CU=%d", wpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_read<4, false>), dim3(grid), dim3(256), 0, 0, p, n, out); }, (double)bytes);
    snprintf(nm, sizeof nm, "grid-stride u4 nt     blocks/CU=%d", wpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_read<4, true>), dim3(grid), dim3(256), 0, 0, p, n, out); }, (double)bytes);
    snprintf(nm, sizeof nm, "grid-stride u8 nt     blocks/CU=%d", wpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_read<8, true>), dim3(grid), dim3(256), 0, 0, p, n, out); }, (double)bytes);
  }
  for (int per : {64, 256, 1024}) {
    const size_t grid = n / ((size_t)per * 256);
    char nm[64];
    snprintf(nm, sizeof nm, "chunked per-block %4d KiB nt", per * 4);
    timeit(nm, [&] { hipLaunchKernelGGL(k_read_rows<true>, dim3(grid), dim3(256), 0, 0, p, n, per, out); }, (double)grid * per * 256 * 16);
    snprintf(nm, sizeof nm, "chunked per-block %4d KiB plain", per * 4);
    timeit(nm, [&] { hipLaunchKernelGGL(k_read_rows<false>, dim3(grid), dim3(256), 0, 0, p, n, per, out); }, (double)grid * per * 256 * 16);
  }
  CK(hipFuncSetAttribute((const void*)k_read_occ<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_read_occ<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_read_tile<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_read_tile<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  for (int W : {25088, 25104, 24576, 24592, 24704, 16384, 16400, 12288, 12304, 20480, 20496}) {   // row strides (doubles)
    const int ntc = W / 1024;
    const int ntr = (int)(n * 2 / ((size_t)256 * W));
    const size_t grid = (size_t)ntr * ntc;
    const double by = (double)grid * 256 * 1024 * 8;
    for (int lds_kib : {64}) {
      char nm[80];
      snprintf(nm, sizeof nm, "tile W=%d %d WG/CU 8rows x 1KiB", W, 160 / lds_kib);
      timeit(nm, [&] { hipLaunchKernelGGL(k_read_tile<0>, dim3(grid), dim3(256), lds_kib * 1024, 0, (const double*)p, W, ntc, out); }, by);
      snprintf(nm, sizeof nm, "tile W=%d %d WG/CU 1row x 8KiB", W, 160 / lds_kib);
      timeit(nm, [&] { hipLaunchKernelGGL(k_read_tile<1>, dim3(grid), dim3(256), lds_kib * 1024, 0, (const double*)p, W, ntc, out); }, by);
    }
  }
  for (int lds_kib : {80, 54, 40, 32, 20, 10}) {
    const int per = 256;
    const size_t grid = n / ((size_t)per * 256);
    char nm[80];
    snprintf(nm, sizeof nm, "occ %d WG/CU u8  (%3d KiB/CU in flight)", 160 / lds_kib, 160 / lds_kib * 4 * 8);
    timeit(nm, [&] { hipLaunchKernelGGL(k_read_occ<8>, dim3(grid), dim3(256), lds_kib * 1024, 0, p, n, per, out); }, (double)grid * per * 256 * 16);
    snprintf(nm, sizeof nm, "occ %d WG/CU u16 (%3d KiB/CU in flight)", 160 / lds_kib, 160 / lds_kib * 4 * 16);
    timeit(nm, [&] { hipLaunchKernelGGL(k_read_occ<16>, dim3(grid), dim3(256), lds_kib * 1024, 0, p, n, per, out); }, (double)grid * per * 256 * 16);
  }
  return 0;
}
