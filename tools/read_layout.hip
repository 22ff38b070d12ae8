// Streaming-read ceiling of the MFMA LD pass's traversal for two storage
// layouts of the same bytes, at the north star's footprint:
//   panel:  a panel is 256 rows x W doubles, row-major (the packed layout);
//           a workgroup owns one 512-column chunk over 8 panels (a strip) and
//           each wave reads, per 16-row group, 4 steps of 16 rows x 256 B
//           (4 loads of 4 rows x 256 B: lane row 4a + (l >> 4), pair l & 15);
//   frag:   the same per-wave steps stored in traversal order, so every
//           wave-step is one contiguous 4 KiB (4 loads of 1 KiB).
// Two steps of loads in flight per wave, two workgroups per CU (LDS-bound like
// the pass), a sum keeps the loads alive.
//   hipcc -O3 --offload-arch=gfx950 tools/read_layout.hip -o tools/read_layout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ d2 ldnt(const double* p) {
  return __builtin_nontemporal_load((const __attribute__((address_space(1))) d2*)p);
}

constexpr int NPS = 8;   // panels per strip

// grid: strips = (panel group) x (chunk); each strip reads NPS panels x 256 rows x 512 cols
template <int MODE>
__global__ __launch_bounds__(256, 2) void k_strip(const double* __restrict__ p, int64_t W, int nch,
                                                  double* out) {
  __shared__ double pad[8192];   // 64 KiB: two workgroups per CU, as the pass
  const int sg = blockIdx.x / nch, ch = blockIdx.x % nch;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int lo = lane & 15, hi = lane >> 4;
  d2 acc = {0.0, 0.0};
  // step index s = (panel, g, t): 8 x 16 x 4
  auto addr = [&](int s, int a) -> const double* {
    const int pn = s >> 6, g = (s >> 2) & 15, t = s & 3;
    const int64_t panel = (int64_t)sg * NPS + pn;
    if (MODE == 0) {
      const double* base = p + panel * 256 * W + (int64_t)ch * 512 + wid * 128;
      return base + (int64_t)(16 * g + 4 * a + hi) * W + 32 * t + 2 * lo;
    } else {
      // this tile (panel, chunk) = 256 x 512 doubles = 1 MiB, traversal order
      const double* base = p + (panel * nch + ch) * (256 * 512);
      return base + ((((int64_t)g * 4 + wid) * 4 + t) * 4 + a) * 128 + 2 * lane;
    }
  };
  d2 q0[4], q1[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) q0[a] = ldnt(addr(0, a));
#pragma unroll
  for (int a = 0; a < 4; ++a) q1[a] = ldnt(addr(1, a));
  constexpr int NS = NPS * 16 * 4;
  for (int s = 0; s < NS; s += 2) {
    d2 c[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) c[a] = q0[a];
    const int n0 = s + 2 < NS ? s + 2 : s;
#pragma unroll
    for (int a = 0; a < 4; ++a) q0[a] = ldnt(addr(n0, a));
#pragma unroll
    for (int a = 0; a < 4; ++a) acc += c[a];
#pragma unroll
    for (int a = 0; a < 4; ++a) c[a] = q1[a];
    const int n1 = s + 3 < NS ? s + 3 : s + 1;
#pragma unroll
    for (int a = 0; a < 4; ++a) q1[a] = ldnt(addr(n1, a));
#pragma unroll
    for (int a = 0; a < 4; ++a) acc += c[a];
  }
  pad[threadIdx.x] = acc.x;
  __syncthreads();
  if (pad[255 - threadIdx.x] == 12345.678) out[threadIdx.x] = acc.y;
}

static int g_reps = 5;
template <class F>
static double timeit(F launch, double bytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < g_reps; ++r) {
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

int main(int argc, char** argv) {
  if (argc > 1) g_reps = std::atoi(argv[1]);   // repetitions per timing (power sampling: many)
  double* out;
  CK(hipMalloc(&out, 256 * sizeof(double)));
  const int64_t W = 15872;           // 31 chunks of 512
  const int nch = (int)(W / 512);
  for (int npanels : {64, 1920}) {   // 2 GB and 61 GB
    const size_t bytes = (size_t)npanels * 256 * W * 8;
    double* p;
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 0, bytes));
    const int grid = (npanels / NPS) * nch;
    const double used = (double)grid * NPS * 256 * 512 * 8;
    const double a = timeit([&] { hipLaunchKernelGGL(k_strip<0>, dim3(grid), dim3(256), 0, 0, p, W, nch, out); }, used);
    const double b = timeit([&] { hipLaunchKernelGGL(k_strip<1>, dim3(grid), dim3(256), 0, 0, p, W, nch, out); }, used);
    const double c = timeit([&] { hipLaunchKernelGGL(k_strip<0>, dim3(grid), dim3(256), 0, 0, p, W, nch, out); }, used);
    const double d = timeit([&] { hipLaunchKernelGGL(k_strip<1>, dim3(grid), dim3(256), 0, 0, p, W, nch, out); }, used);
    printf("%.1f GB: panel %6.0f %6.0f  frag %6.0f %6.0f GB/s\n", bytes / 1e9, a, c, b, d);
    CK(hipFree(p));
  }
  return 0;
}
