// Multi-RHS symmetric LD pass on the f64 matrix cores (v_mfma_f64_16x16x4f64).
//
// For 3..16 right-hand sides a VALU pass runs out of operands before HBM
// runs out of bytes: each stored R_ij feeds 2*NC FMAs whose P operands must
// be in registers, so the VALU kernels (sym_pass.hip) re-read P or spill
// column partials through LDS at a multiple of the HBM traffic.  A 16x16x4
// MFMA takes ONE f64 of R and ONE f64 of P per lane and does 16 FMAs per lane:
// the matrix core does the register blocking.  On gfx950 the f64 MFMA rate
// is about the f64 VALU rate (tools/mfma_probe.hip: ~47 TF at 2 waves/SIMD),
// so with the RHS padded to 16 columns the pass costs ~16 MFMAs per 4 KiB of
// stored R for any NC <= 16 -- close to the HBM time of the same bytes.
//
// Same items (panel x 512-column chunk), partial layout and finalize as the
// VALU pass (class 1): rowpart[item][256][NC], colpart[item][NC][512].
//
// One 256-thread workgroup per item; wave w owns chunk columns
// [128 w, 128 w + 128) and sweeps the panel's rows in 16-row groups.  Each
// 16 x 32 sub-tile (4 KiB) is loaded from HBM once, 16 B per lane:
//   col fragment  lane l: R[row 4a + (l>>4)][col 2(l&15) + e]  (a = 0..3)
//       -> A operand (m = column, k = row) of  Dcol[col][c] += R[j][col] P[j][c]
// and written to a per-wave LDS tile (rows padded to 34 doubles), from which
// the transposed fragment is read back without bank conflicts:
//   row fragment  lane l: R[row (l&15)][col 8s + 2(l>>4) + e]  (s = 0..3)
//       -> A operand (m = row, k = column) of  Drow[row][c] += R[row][i] P[i][c]
// The row-part B operands (P at the wave's 128 columns) stay in registers for
// the whole item.
// Dcol accumulates over all 256 rows in registers and is complete per item;
// Drow is summed over the 4 waves through LDS once per 16-row group, in wave
// order.  The B operands come from Pk, the RHS interleaved as Pk[i][16].
// f64 C/D layout (cdna_hip_programming.md): D[(l>>4) + 4r][l & 15], r = 0..3.
#include "common.h"

namespace sgv {

typedef double d4 __attribute__((ext_vector_type(4)));

#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

// wave-local LDS ordering point: lanes of one wave exchange data through the
// tile.  The LDS executes a wave's DS instructions in order, so the write ->
// read (and read -> next write) order only has to survive compilation: a
// wavefront-scope fence, which emits no wait (an inline-asm lgkmcnt(0) would
// make the compiler drain vmcnt as well, stalling on the prefetched loads).
__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

constexpr int MF_CW = 512;            // chunk width (class 1 items)
constexpr int MF_WC = MF_CW / 4;      // columns per wave
constexpr int MF_NT = MF_WC / 32;     // 32-column steps per wave

__global__ __launch_bounds__(256, 2) void k_sym_mfma(const SymItem* __restrict__ items,
                                                     const double* __restrict__ pk, int ncol,
                                                     double* __restrict__ rowpart,
                                                     double* __restrict__ colpart) {
  constexpr int LDP = 34;                     // staging row pitch (doubles): conflict-free
  __shared__ double red[2][4][256];
  __shared__ __attribute__((aligned(16))) double stg[4][16 * LDP];
  const SymItem it = items[blockIdx.x];
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int lo = lane & 15, hi = lane >> 4;
  const double* base = it.P + (it.c0 - it.r0);        // panel row 0, chunk column 0
  const int64_t w = it.w;
  const double* pkb = pk + (int64_t)it.voff * 16;     // Pk of this block (block-relative index)
  const int cw0 = wid * MF_WC;                         // first chunk column of this wave

  double* sb = stg[wid];
  // row-part B operands (P at this wave's columns), reused by every row group
  double brow[MF_NT][4][2];
#pragma unroll
  for (int t = 0; t < MF_NT; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int col = cw0 + 32 * t + 8 * s + 2 * hi + e;
        const double v = ldg(pkb + (int64_t)(it.c0 + (col < it.nc ? col : 0)) * 16 + lo);
        brow[t][s][e] = col < it.nc ? v : 0.0;
      }
  d4 dcol[MF_NT][2];
#pragma unroll
  for (int t = 0; t < MF_NT; ++t) dcol[t][0] = dcol[t][1] = d4{0.0, 0.0, 0.0, 0.0};

  // fragment loads of step (g, t), 16 B per lane; rows past H clamp (their P is 0)
  auto load_cf = [&](int g, int t, d2* cf) {
    const int xc = cw0 + 32 * t + 2 * lo;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int rB = 16 * g + 4 * a + hi;
      const double* row = base + (int64_t)(rB < it.H ? rB : it.H - 1) * w;
      // branch-free: a column past the chunk loads column 0 (finite), meets a
      // zero B in the row part and is never stored by the column part
      cf[a] = ldg_nt((const d2*)(row + (xc < it.nc ? xc : 0)));
    }
  };
  auto load_bcol = [&](int g, double* bc) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int rB = 16 * g + 4 * a + hi;
      const double v = ldg(pkb + (int64_t)(it.r0 + (rB < it.H ? rB : 0)) * 16 + lo);
      bc[a] = rB < it.H ? v : 0.0;
    }
  };
  const int ng = (it.H + 15) / 16;
  d2 cfn[4];
  double bcn[4];
  load_cf(0, 0, cfn);
  load_bcol(0, bcn);

#pragma unroll 1
  for (int g = 0; g < ng; ++g) {                      // ng is uniform over the workgroup
    double bcol[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) bcol[a] = bcn[a];
    d4 drow0 = d4{0.0, 0.0, 0.0, 0.0}, drow1 = drow0;
#pragma unroll
    for (int t = 0; t < MF_NT; ++t) {
      d2 cf[4], rf[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) cf[a] = cfn[a];
      // next step's loads are issued here, ahead of this step's LDS and MFMA work
      if (t + 1 < MF_NT) {
        load_cf(g, t + 1, cfn);
      } else if (g + 1 < ng) {
        load_cf(g + 1, 0, cfn);
        load_bcol(g + 1, bcn);
      }
      lds_order();                                     // previous step's tile reads done
#pragma unroll
      for (int a = 0; a < 4; ++a) *(d2*)(sb + (4 * a + hi) * LDP + 2 * lo) = cf[a];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        dcol[t][0] = MFMA64(cf[a].x, bcol[a], dcol[t][0]);
        dcol[t][1] = MFMA64(cf[a].y, bcol[a], dcol[t][1]);
      }
      lds_order();                                     // tile written
#pragma unroll
      for (int s = 0; s < 4; ++s) rf[s] = *(const d2*)(sb + lo * LDP + 8 * s + 2 * hi);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        drow0 = MFMA64(rf[s].x, brow[t][s][0], drow0);
        drow1 = MFMA64(rf[s].y, brow[t][s][1], drow1);
      }
    }
    // row sums of this 16-row group: waves 0..3 in order
    double* rb = red[g & 1][wid];
#pragma unroll
    for (int r = 0; r < 4; ++r) rb[((hi + 4 * r) << 4) + lo] = drow0[r] + drow1[r];
    __syncthreads();
    {
      const int t = threadIdx.x, row = t >> 4, cc = t & 15;
      const double s = ((red[g & 1][0][t] + red[g & 1][1][t]) + red[g & 1][2][t]) + red[g & 1][3][t];
      if (16 * g + row < it.H && cc < ncol)
        rowpart[((int64_t)it.item * SYM_H + 16 * g + row) * ncol + cc] = s;
    }
  }

  // column sums (complete over the panel's rows), right of the diagonal block only
  if (lo < ncol) {
    double* out = colpart + ((int64_t)it.item * ncol + lo) * MF_CW;
#pragma unroll
    for (int t = 0; t < MF_NT; ++t)
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int jl = cw0 + 32 * t + 2 * (hi + 4 * r) + e;
          if (jl < it.nc && it.c0 + jl >= it.diag_end) out[jl] = dcol[t][e][r];
        }
  }
}

// Pk[i][c] = in[c][i] for c < ncol, 0 for ncol <= c < 16 (i over the padded vector)
__global__ __launch_bounds__(256) void k_pack16(PassArgs pa, int ncol, int64_t mpad,
                                                double* __restrict__ pk) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= mpad * 16) return;
  const int64_t i = t >> 4;
  const int c = (int)(t & 15);
  pk[t] = c < ncol ? pa.in[c][i] : 0.0;
}

hipError_t launch_sym_mfma(int nc, const SymItem* d_items, int nitems, const PassArgs& pa,
                           int64_t mpad, double* d_pk, double* rowpart, double* colpart,
                           hipStream_t st) {
  if (nc < 1 || nc > 16) return hipErrorInvalidValue;
  const int64_t n16 = mpad * 16;
  hipLaunchKernelGGL(k_pack16, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st, pa, nc,
                     mpad, d_pk);
  hipLaunchKernelGGL(k_sym_mfma, dim3(nitems), dim3(256), 0, st, d_items, d_pk, nc, rowpart,
                     colpart);
  return hipGetLastError();
}

}  // namespace sgv
