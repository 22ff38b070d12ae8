// Register-only transposes of the MFMA pass's 16 x 32 sub-tile (sym_mfma.hip,
// tools/xpose_probe.hip): the column fragment's lane layout to the row
// fragment's.
#pragma once
#include "common.h"

namespace sgv {

// The row fragment is the column fragment with lane bits (5,4) and (1,0)
// exchanged, register for register: rf[r] at lane 16 h + 4 b + n = cf[r] at lane
// 16 n + 4 b + h.  Besides the LDS tile (XP = 0) two register-only forms
// (A/B, SGV_MF_XPOSE):
// XP = 1: permlane32/16_swap exchange lane bits 5 / 4 with the register bits of
//   r (1 / 0), quad DPP moves + selects exchange lane bits 1 / 0 with them, and
//   a second permlane pass puts r back: (L54 r)(L10 r)(L54 r) = (L54 L10);
//   16 + 32 + 16 swaps / selects (+ 32 DPP moves) per 4-KiB step, no LDS.
// XP = 2: ds_bpermute_b32 (the LDS crossbar, no LDS storage), 16 per step.
__device__ __forceinline__ void xp_p32(unsigned& x, unsigned& y) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}
__device__ __forceinline__ void xp_p16(unsigned& x, unsigned& y) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}
// lane bit `B` (0 or 1) <-> the register bit distinguishing x (0) from y (1)
template <int B>
__device__ __forceinline__ void xp_quad(unsigned& x, unsigned& y, bool sel) {
  constexpr int CTRL = B == 0 ? 0xB1 : 0x4E;   // quad_perm [1,0,3,2] / [2,3,0,1]
  const unsigned dx = (unsigned)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true);
  const unsigned dy = (unsigned)__builtin_amdgcn_mov_dpp((int)y, CTRL, 0xF, 0xF, true);
  const unsigned nx = sel ? dy : x;
  y = sel ? y : dx;
  x = nx;
}
__device__ __forceinline__ void xp_rows(unsigned (&v)[4]) {   // (L5 r1)(L4 r0)
  xp_p32(v[0], v[2]);
  xp_p32(v[1], v[3]);
  xp_p16(v[0], v[1]);
  xp_p16(v[2], v[3]);
}
__device__ __forceinline__ void xpose_perm(const d2* cf, d2* rf, bool l1, bool l0) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {   // the 4 dwords of a d2, each over the 4 registers
    unsigned v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // through a scalar: __builtin_bit_cast of a vector-element lvalue reads
      // element 0 whatever the index (clang, ROCm 7.2)
      const double d = cf[r][e >> 1];
      const unsigned long long u = __builtin_bit_cast(unsigned long long, d);
      v[r] = (unsigned)(e & 1 ? u >> 32 : u);
    }
    xp_rows(v);
    xp_quad<1>(v[0], v[2], l1);
    xp_quad<1>(v[1], v[3], l1);
    xp_quad<0>(v[0], v[1], l0);
    xp_quad<0>(v[2], v[3], l0);
    xp_rows(v);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double d = rf[r][e >> 1];
      unsigned long long u = __builtin_bit_cast(unsigned long long, d);
      u = e & 1 ? ((u & 0xFFFFFFFFull) | ((unsigned long long)v[r] << 32))
                : ((u & 0xFFFFFFFF00000000ull) | v[r]);
      rf[r][e >> 1] = __builtin_bit_cast(double, u);
    }
  }
}
__device__ __forceinline__ void xpose_bperm(const d2* cf, d2* rf, int src4) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const double d = cf[r][e];   // a scalar first (see xpose_perm)
      const unsigned long long u = __builtin_bit_cast(unsigned long long, d);
      const unsigned lo32 = (unsigned)__builtin_amdgcn_ds_bpermute(src4, (int)(unsigned)u);
      const unsigned hi32 = (unsigned)__builtin_amdgcn_ds_bpermute(src4, (int)(unsigned)(u >> 32));
      rf[r][e] = __builtin_bit_cast(double, (unsigned long long)lo32 | ((unsigned long long)hi32 << 32));
    }
}

}  // namespace sgv
