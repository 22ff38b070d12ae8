// Gap between back-to-back kernels on one stream with (a) no events,
// (b) hipEventRecord after every kernel, (c) the event bound to the kernel
// through hipExtLaunchKernelGGL's stop event.  Read the gaps from a
// rocprofv3 kernel trace (tools/evgap_read.py).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

template <int TAG>
__global__ void k_tick(double* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5 + TAG;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const int n = 1 << 20, reps = 200;
  double* p;
  CK(hipMalloc(&p, n * sizeof(double)));
  CK(hipMemset(p, 0, n * sizeof(double)));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t evt, evn;
  CK(hipEventCreate(&evt));
  CK(hipEventCreateWithFlags(&evn, hipEventDisableTiming));
  const dim3 g(n / 256), b(256);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_tick<0>, g, b, 0, st, p, n);
  CK(hipStreamSynchronize(st));
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k_tick<1>, g, b, 0, st, p, n);
    CK(hipEventRecord((r & 1) ? evt : evn, st));
  }
  CK(hipStreamSynchronize(st));
  for (int r = 0; r < reps; ++r)
    hipExtLaunchKernelGGL(k_tick<2>, g, b, 0, st, nullptr, (r & 1) ? evt : evn, 0, p, n);
  CK(hipStreamSynchronize(st));
  for (int r = 0; r < reps; ++r)
    hipExtLaunchKernelGGL(k_tick<3>, g, b, 0, st, (r & 1) ? evt : evn, nullptr, 0, p, n);
  CK(hipStreamSynchronize(st));
  float ms = 0;
  hipEvent_t a, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&z));
  hipExtLaunchKernelGGL(k_tick<4>, g, b, 0, st, a, nullptr, 0, p, n);
  for (int r = 0; r < 8; ++r) hipLaunchKernelGGL(k_tick<4>, g, b, 0, st, p, n);
  hipExtLaunchKernelGGL(k_tick<4>, g, b, 0, st, nullptr, z, 0, p, n);
  CK(hipStreamSynchronize(st));
  CK(hipEventElapsedTime(&ms, a, z));
  std::printf("ext start/stop events over 10 kernels: %.3f ms\n", ms);
  std::printf("done\n");
  return 0;
}
