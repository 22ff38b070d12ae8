// What v_permlane16_swap / v_permlane32_swap and the quad DPP moves do to lane
// data on this device (one wave): prints, per lane, the source lane each output
// holds.  hipcc --offload-arch=gfx950 -O2 tools/permlane_probe.hip -o /tmp/pp
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  unsigned x = l, y = 100 + l;
  auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
  auto s = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  out[128 + l] = s[0];
  out[192 + l] = s[1];
  out[256 + l] = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);
  out[320 + l] = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
}

int main() {
  unsigned* d;
  unsigned h[384];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char* names[6] = {"p16 vdst", "p16 src", "p32 vdst", "p32 src", "dpp 4E", "dpp B1"};
  for (int i = 0; i < 6; ++i) {
    std::printf("%s:", names[i]);
    for (int l = 0; l < 64; ++l) std::printf(" %u", h[64 * i + l]);
    std::printf("\n");
  }
  return 0;
}
