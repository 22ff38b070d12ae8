// The box's own streaming-read ceiling, for the bench line's context: every
// workgroup streams its own contiguous 256 KiB with 16-B nontemporal loads, 8
// in flight per thread (the best of tools/read_bw.hip's patterns: 6.9-7.2 TB/s
// on the boxes of round 1).  The LD passes' roofline peak stays the guide's
// 8 TB/s; this number says how much of the gap the box itself leaves.
#include "common.h"

namespace sgv {

constexpr int RB_PER = 64;   // 16-B loads per thread: 64 x 256 threads x 16 B = 256 KiB per workgroup

__global__ __launch_bounds__(256) void k_read_probe(const d2* __restrict__ p, double* out) {
  const size_t base = (size_t)blockIdx.x * RB_PER * 256;
  d2 acc = {0.0, 0.0};
  for (int j = 0; j < RB_PER; j += 8) {
    d2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ldg_nt(p + base + (size_t)(j + u) * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  if (acc.x == 12345.678) out[threadIdx.x] = acc.y;   // never true: keeps the loads
}

hipError_t launch_read_probe(const double* buf, size_t bytes, double* out, hipStream_t st) {
  const size_t per_wg = (size_t)RB_PER * 256 * sizeof(d2);
  const size_t grid = bytes / per_wg;
  if (grid < 1 || grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_read_probe, dim3((unsigned)grid), dim3(256), 0, st, (const d2*)buf, out);
  return hipGetLastError();
}

}  // namespace sgv
