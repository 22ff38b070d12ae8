// Checks the register-only transposes of sgvamp-py_amd/csrc/xpose.h against the
// row fragment the LDS tile yields (one wave, element ids as doubles): prints
// the mismatching lanes/registers of each form.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sgvamp-py_amd/csrc \
//       tools/xpose_probe.hip -o tools/xpose_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#include "xpose.h"

using namespace sgv;

__global__ void k(double* out) {
  const int lane = threadIdx.x;
  const int lo = lane & 15, hi = lane >> 4, bq = (lane >> 2) & 3, n4 = lane & 3;
  d2 cf[4], rf1[4], rf2[4];
  for (int a = 0; a < 4; ++a)
    for (int e = 0; e < 2; ++e) cf[a][e] = 1000.0 * (4 * a + hi) + 2 * lo + e;   // (row, column)
  xpose_perm(cf, rf1, (lane & 2) != 0, (lane & 1) != 0);
  xpose_bperm(cf, rf2, 4 * (16 * n4 + 4 * bq + hi));
  for (int r = 0; r < 4; ++r)
    for (int e = 0; e < 2; ++e) {
      const double want = 1000.0 * (4 * r + n4) + 2 * (hi + 4 * bq) + e;
      out[(0 * 8 + 2 * r + e) * 64 + lane] = rf1[r][e] - want;
      out[(1 * 8 + 2 * r + e) * 64 + lane] = rf2[r][e] - want;
    }
}

int main() {
  double* d;
  static double h[2 * 8 * 64];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int f = 0; f < 2; ++f) {
    int bad = 0;
    for (int i = 0; i < 8 * 64; ++i)
      if (h[f * 512 + i] != 0.0) {
        if (bad < 8) std::printf("form %d: reg %d elem %d lane %d off by %g\n", f + 1, i / 128,
                                 (i / 64) & 1, i & 63, h[f * 512 + i]);
        ++bad;
      }
    std::printf("form %d (%s): %d of 512 wrong\n", f + 1, f ? "ds_bpermute" : "permlane+dpp", bad);
  }
  return 0;
}
