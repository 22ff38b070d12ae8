// Streaming-read ceiling of the MFMA LD pass's access pattern (sym_mfma.hip)
// against the same tiles read as 1 KiB row segments.  A workgroup of 4 waves
// reads one 256-row x 512-column tile of a row-major matrix (row stride W
// doubles); wave w owns columns 128w..128w+127.  Per 16-row group:
//   frag:  16 loads per wave, each 4 rows x 256 B (lane: row 4a + (l >> 4),
//          columns 32t + 2(l & 15)) -- the MFMA column-fragment load;
//   rows:  16 loads per wave, each one row x 1 KiB (lane: columns 2l).
// U loads in flight per wave (the kernel keeps 8: two 32-column steps).
//   hipcc -O3 --offload-arch=gfx950 tools/read_pattern.hip -o tools/read_pattern
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ d2 ldnt(const double* p) {
  return __builtin_nontemporal_load((const __attribute__((address_space(1))) d2*)p);
}

template <int MODE, int U>
__global__ __launch_bounds__(256, 2) void k_tile(const double* __restrict__ p, int64_t W, int ntc,
                                                 double* out) {
  const int tr = blockIdx.x / ntc, tc = blockIdx.x % ntc;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lo = lane & 15, hi = lane >> 4;
  const double* base = p + (int64_t)tr * 256 * W + tc * 512 + wid * 128;
  d2 acc = {0.0, 0.0};
  for (int g = 0; g < 16; ++g) {
    for (int q0 = 0; q0 < 16; q0 += U) {
      d2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u;
        if (MODE == 0) {   // frag: q = 4t + a
          const int t = q >> 2, a = q & 3;
          v[u] = ldnt(base + (int64_t)(16 * g + 4 * a + hi) * W + 32 * t + 2 * lo);
        } else {           // rows: q = row of the group
          v[u] = ldnt(base + (int64_t)(16 * g + q) * W + 2 * lane);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u];
    }
  }
  if (acc.x == 12345.678) out[threadIdx.x] = acc.y;
}

template <class F>
static double timeit(F launch, double bytes) {
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
  return bytes / best / 1e6;
}

int main() {
  double* out;
  CK(hipMalloc(&out, 256 * sizeof(double)));
  for (int64_t W : {15616, 15872, 16384}) {       // panel-like row strides (doubles)
    const int64_t rows = 256 * 64;                   // 64 panels
    const int ntc = (int)(W / 512);
    const size_t bytes = (size_t)rows * W * 8;
    double* p;
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 0, bytes));
    const int grid = (int)(rows / 256) * ntc;
    const double used = (double)grid * 256 * 512 * 8;
    printf("W=%lld (%.1f GB): frag U8 %6.0f  frag U16 %6.0f  rows U8 %6.0f  rows U16 %6.0f GB/s\n",
           (long long)W, bytes / 1e9,
           timeit([&] { hipLaunchKernelGGL((k_tile<0, 8>), dim3(grid), dim3(256), 0, 0, p, W, ntc, out); }, used),
           timeit([&] { hipLaunchKernelGGL((k_tile<0, 16>), dim3(grid), dim3(256), 0, 0, p, W, ntc, out); }, used),
           timeit([&] { hipLaunchKernelGGL((k_tile<1, 8>), dim3(grid), dim3(256), 0, 0, p, W, ntc, out); }, used),
           timeit([&] { hipLaunchKernelGGL((k_tile<1, 16>), dim3(grid), dim3(256), 0, 0, p, W, ntc, out); }, used));
    CK(hipFree(p));
  }
  return 0;
}
