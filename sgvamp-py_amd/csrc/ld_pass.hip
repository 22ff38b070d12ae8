// LD pass: Y = R_b P for every LD block b, all RHS columns of one LD matrix
// in one sweep over the LD bytes.  This is the mat-vec inside scipy's cg
// (iterative.py:411, reached from src/sgvamp.py:316,332) and the R products of
// gamw learning (src/sgvamp.py:352,359), batched over right-hand sides.
//
// HBM-bound: every byte of R_b is read once per pass (16-B nontemporal loads,
// 1 KiB per wave instruction, rows 1 KiB aligned); the RHS panel (<= 16 x n_b
// f64) is re-read from L2/L1 and reused in registers across RWI rows.
//
// Fused epilogue per row i and column c:
//   out[c][i] = c1[c] * (R in[c])[i] + c2[c] * in[c][i]
//     CG:    q = A p with A = gamw R_s + gam2 I, R_s = (1-s)R + sI:
//            c1 = gamw(1-s), c2 = gamw s + gam2
//     gamw:  R_s v:  c1 = 1-s, c2 = s
//   partial[g][c] = sum over the group's rows of dot[c][i] * out[c][i]
// Workgroup = 4 waves; wave w owns rows row0 + 8w .. 8w+7 of one block and
// sweeps the full row length (in 8/RWI sub-sweeps of RWI rows); lanes cover
// 128 consecutive columns per step.
#include "common.h"

namespace sgv {

constexpr int LD_RW = 8;  // rows per wave (a row group = 4 waves = 32 rows)

template <int NC, int RWI>
__global__ __launch_bounds__(256) void k_ld_pass(const BlkDesc* __restrict__ blks,
                                                 const RowGroup* __restrict__ rgs, PassArgs pa,
                                                 double* __restrict__ partials) {
  static_assert(RWI * NC <= 64, "one epilogue round per sub-sweep");
  static_assert(LD_RW % RWI == 0, "sub-sweeps");
  __shared__ double red[4][LD_RW * NC];

  const RowGroup rg = rgs[blockIdx.x];
  if (pa.run && !ldg(pa.run)) return;   // no-op pass (pipelined CG past its stop test)
  const BlkDesc bd = blks[rg.blk];
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);   // provably wave-uniform
  const int64_t n = bd.n;
  const int64_t nfull = n & ~(int64_t)127;

  const double* pp[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) pp[c] = pa.in[c] + bd.voff;

  // per-lane epilogue role (static selects, no dynamic indexing of kernargs)
  const int myr = lane / NC, myc = lane % NC;
  const double* ip = pa.in[0];
  double* op = pa.out[0];
  const double* dp = pa.dot[0];
  double* yp = pa.yout[0];
  double c1 = pa.c1[0], c2 = pa.c2[0];
#pragma unroll
  for (int c = 1; c < NC; ++c)
    if (myc == c) {
      ip = pa.in[c];
      op = pa.out[c];
      dp = pa.dot[c];
      yp = pa.yout[c];
      c1 = pa.c1[c];
      c2 = pa.c2[c];
    }

#pragma unroll 1
  for (int h = 0; h < LD_RW / RWI; ++h) {
    const int64_t rbase = (int64_t)rg.row0 + (int64_t)wid * LD_RW + h * RWI;
    const double* rp[RWI];
#pragma unroll
    for (int r = 0; r < RWI; ++r) {
      int64_t row = rbase + r;
      row = row < n ? row : n - 1;  // clamp: duplicate row hits cache, output masked
      rp[r] = bd.R + row * bd.lda;
    }
    double acc[RWI][NC];
#pragma unroll
    for (int r = 0; r < RWI; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[r][c] = 0.0;

#pragma unroll 2
    for (int64_t j = 2 * lane; j < nfull; j += 128) {
      d2 rv[RWI];
#pragma unroll
      for (int r = 0; r < RWI; ++r) rv[r] = ldg_nt((const d2*)(rp[r] + j));
      d2 pv[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) pv[c] = ldg((const d2*)(pp[c] + j));
#pragma unroll
      for (int r = 0; r < RWI; ++r)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          acc[r][c] = __builtin_fma(rv[r].x, pv[c].x, acc[r][c]);
          acc[r][c] = __builtin_fma(rv[r].y, pv[c].y, acc[r][c]);
        }
    }
    {
      // tail: j < n; element j+1 may be the zero padding of R and of the vector
      const int64_t j = nfull + 2 * lane;
      if (j < n) {
        d2 rv[RWI];
#pragma unroll
        for (int r = 0; r < RWI; ++r) rv[r] = ldg_nt((const d2*)(rp[r] + j));
        d2 pv[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) pv[c] = ldg((const d2*)(pp[c] + j));
#pragma unroll
        for (int r = 0; r < RWI; ++r)
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            acc[r][c] = __builtin_fma(rv[r].x, pv[c].x, acc[r][c]);
            acc[r][c] = __builtin_fma(rv[r].y, pv[c].y, acc[r][c]);
          }
      }
    }
    // wave reduction (butterfly: every lane holds every row/column total)
#pragma unroll
    for (int r = 0; r < RWI; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[r][c] = wave_sum(acc[r][c]);

    double y = 0.0;
#pragma unroll
    for (int r = 0; r < RWI; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (lane == r * NC + c) y = acc[r][c];
    const int64_t row = rbase + myr;
    double contrib = 0.0;
    if (lane < RWI * NC && row < n) {
      const int64_t idx = bd.voff + row;
      const double in = ip[idx];
      const double o = c1 * y + c2 * in;
      op[idx] = o;
      if (yp) yp[idx] = pa.ys1 * y + pa.ys0 * in;
      if (dp) contrib = dp[idx] * o;
    }
    if (lane < RWI * NC) red[wid][h * RWI * NC + lane] = contrib;
  }
  __syncthreads();
  if ((int)threadIdx.x < NC) {
    const int c = threadIdx.x;
    double s = 0.0;
    // fixed order: waves 0..3, rows 0..7
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int r = 0; r < LD_RW; ++r) s += red[w][r * NC + c];
    partials[(int64_t)rg.part * NC + c] = s;
  }
}

int ld_pass_rows_per_group() { return 4 * LD_RW; }

template <int NC>
static hipError_t launch_nc(const BlkDesc* d_blks, const RowGroup* d_rg, int nrg,
                            const PassArgs& pa, double* d_part, hipStream_t st) {
  constexpr int RWI = (NC <= 3) ? 8 : (NC <= 6) ? 4 : (NC <= 12) ? 2 : 1;
  hipLaunchKernelGGL((k_ld_pass<NC, RWI>), dim3(nrg), dim3(256), 0, st, d_blks, d_rg, pa,
                     d_part);
  return hipGetLastError();
}

hipError_t launch_ld_pass(int nc, const BlkDesc* d_blks, const RowGroup* d_rg, int nrg,
                          const PassArgs& pa, double* d_part, hipStream_t st) {
  switch (nc) {
    case 1: return launch_nc<1>(d_blks, d_rg, nrg, pa, d_part, st);
    case 2: return launch_nc<2>(d_blks, d_rg, nrg, pa, d_part, st);
    case 3: return launch_nc<3>(d_blks, d_rg, nrg, pa, d_part, st);
    case 4: return launch_nc<4>(d_blks, d_rg, nrg, pa, d_part, st);
    case 5: return launch_nc<5>(d_blks, d_rg, nrg, pa, d_part, st);
    case 6: return launch_nc<6>(d_blks, d_rg, nrg, pa, d_part, st);
    case 7: return launch_nc<7>(d_blks, d_rg, nrg, pa, d_part, st);
    case 8: return launch_nc<8>(d_blks, d_rg, nrg, pa, d_part, st);
    case 9: return launch_nc<9>(d_blks, d_rg, nrg, pa, d_part, st);
    case 10: return launch_nc<10>(d_blks, d_rg, nrg, pa, d_part, st);
    case 11: return launch_nc<11>(d_blks, d_rg, nrg, pa, d_part, st);
    case 12: return launch_nc<12>(d_blks, d_rg, nrg, pa, d_part, st);
    case 13: return launch_nc<13>(d_blks, d_rg, nrg, pa, d_part, st);
    case 14: return launch_nc<14>(d_blks, d_rg, nrg, pa, d_part, st);
    case 15: return launch_nc<15>(d_blks, d_rg, nrg, pa, d_part, st);
    case 16: return launch_nc<16>(d_blks, d_rg, nrg, pa, d_part, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace sgv
