// Symmetric (packed upper-triangle) LD pass: Y = R_b P reading each stored
// element of a symmetric LD block once -- about half the bytes of the dense
// pass (ld_pass.hip).  Same fused epilogue and partial dots.
//
// Packed layout of an n x n block: panels of SYM_H = 256 rows; panel g
// (rows r0 = 256 g .. r0 + H - 1) stores columns r0 .. n-1 (its 256 x 256
// diagonal block in full, everything right of it), row-major with row stride
// w_g = round_up(n - r0, 128) doubles (rows 1 KiB aligned).
//
// k_sym_pass: one workgroup per (panel, chunk of NSEG*128 columns).  Every
// element R_ij read feeds the row sum y_i += R_ij p_j and, right of the
// diagonal block (j >= r0 + H), the transpose contribution y_j += R_ij p_i.
// Row sums are written per (item, row); column sums per (item, column), each
// combined over the 4 waves in a fixed order through LDS.
// k_sym_finalize: one workgroup per panel; row i sums its panel's row parts
// (chunk order) and the column parts of every earlier panel of the block
// (panel order), then applies out = c1*y + c2*in and the partial dot.
// All orders are fixed: bitwise reproducible, no atomics.
#include "common.h"

#include <cstdlib>

namespace sgv {

template <int NC, int RWI, int NSEG, bool SKIP, int OCC = 1>
__global__ __launch_bounds__(256, OCC) void k_sym_pass(const SymItem* __restrict__ items, PassArgs pa,
                                                  double* __restrict__ rowpart,
                                                  double* __restrict__ colpart) {
  constexpr int CW = NSEG * 128;
  static_assert(RWI * NC <= 16, "row results per sub-sweep");
  // per-wave column partials: lane l owns columns 2l, 2l+1 of every segment,
  // so read-modify-writes are private; waves are summed in order at the end
  __shared__ d2 cbw[4][NC][CW / 2];
  // the item's row sums, stored as one contiguous 16-B-store burst at the end
  __shared__ __attribute__((aligned(16))) double rbuf[SYM_H * NC];

  const SymItem it = items[blockIdx.x];
  if (pa.run && !ldg(pa.run)) return;   // no-op pass (pipelined CG past its stop test)
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);   // provably wave-uniform
  const double* pp[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) pp[c] = pa.in[c] + it.voff;
  const bool has_cols = it.c0 + it.nc > it.diag_end;   // uniform
  // SKIP: the ragged last chunk of a panel sweeps only its stored 128-column
  // segments (at CW = 1024 and n = 15,625, 6 % of all segments lie past the
  // stored columns); the skipped ones would add R * 0 to the row sums and
  // column sums nobody reads -- bitwise the same results
  const int nseg = SKIP ? min(NSEG, (it.nc + 127) / 128) : NSEG;   // uniform
  if (has_cols) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      for (int s = 0; s < NSEG; ++s) cbw[wid][c][s * 64 + lane] = d2{0.0, 0.0};
  }

  constexpr int NSUB = SYM_H / (4 * RWI);
#pragma unroll 1
  for (int sub = 0; sub < NSUB; ++sub) {
    const int rbase = sub * 4 * RWI + wid * RWI;   // panel-relative first row of this wave
    if (rbase >= it.H) break;                      // wave-uniform
    const double* rp[RWI];
    double prow[RWI][NC];
#pragma unroll
    for (int r = 0; r < RWI; ++r) {
      const int rr = rbase + r;
      const bool ok = rr < it.H;
      rp[r] = it.P + (int64_t)(ok ? rr : it.H - 1) * it.w + (it.c0 - it.r0);
#pragma unroll
      for (int c = 0; c < NC; ++c) prow[r][c] = ok ? pp[c][it.r0 + rr] : 0.0;
    }
    double racc[RWI][NC];
#pragma unroll
    for (int r = 0; r < RWI; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) racc[r][c] = 0.0;

#pragma unroll 2
    for (int s = 0; s < nseg; ++s) {
      const int jl = s * 128 + 2 * lane;            // chunk-relative column
      const bool valid = jl < it.nc;
      d2 rv[RWI];
      d2 pv[NC];
#pragma unroll
      for (int r = 0; r < RWI; ++r)
        rv[r] = ldg_nt((const d2*)(rp[r] + (valid ? jl : 0)));
      // branch-free: an invalid column loads column 0 of its row (finite) and
      // meets a zero P; its column sums are never stored
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const d2 v = ldg((const d2*)(pp[c] + it.c0 + (valid ? jl : 0)));
        pv[c] = valid ? v : d2{0.0, 0.0};
      }
#pragma unroll
      for (int r = 0; r < RWI; ++r)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          racc[r][c] = __builtin_fma(rv[r].x, pv[c].x, racc[r][c]);
          racc[r][c] = __builtin_fma(rv[r].y, pv[c].y, racc[r][c]);
        }
      if (it.c0 + s * 128 >= it.diag_end) {         // wave-uniform: right of the diagonal block
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          d2 cv = cbw[wid][c][s * 64 + lane];
#pragma unroll
          for (int r = 0; r < RWI; ++r) {
            cv.x = __builtin_fma(rv[r].x, prow[r][c], cv.x);
            cv.y = __builtin_fma(rv[r].y, prow[r][c], cv.y);
          }
          cbw[wid][c][s * 64 + lane] = cv;
        }
      }
    }
    // all RWI x NC row sums at once (halving reduction)
    constexpr int P = Pow2Ceil<RWI * NC>::value;
    constexpr int SH = (P >= 64) ? 0 : (P >= 32) ? 1 : (P >= 16) ? 2 : (P >= 8) ? 3
                     : (P >= 4) ? 4 : (P >= 2) ? 5 : 6;
    double v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = (k < RWI * NC) ? racc[k / NC][k % NC] : 0.0;
    const double y = wave_reduce_many<P>(v);
    const int idx = (lane >> SH) & (P - 1);
    const int rr = idx / NC, cc = idx % NC;
    if ((lane & ((1 << SH) - 1)) == 0 && idx < RWI * NC && rbase + rr < it.H)
      rbuf[(rbase + rr) * NC + cc] = y;
  }
  __syncthreads();
  {
    const int n = it.H * NC;
    double* dst = rowpart + (int64_t)it.item * SYM_H * NC;
    for (int i = threadIdx.x; 2 * i < n; i += 256) {
      if (2 * i + 1 < n)
        *(d2*)(dst + 2 * i) = *(const d2*)(rbuf + 2 * i);
      else
        dst[2 * i] = rbuf[2 * i];
    }
  }

  // column parts: waves 0..3 in order.  The item's whole NC x CW slot is
  // written with 16-B stores, a wave covering 1 KiB contiguously: columns the
  // finalize never reads (inside the diagonal block, past the block edge) get
  // don't-care values.  Per-column predicated 8-B stores here cost ~8 % of the
  // pass (measured) for < 1 % of its bytes.
  if (has_cols) {
    __syncthreads();
    d2* out = (d2*)(colpart + (int64_t)it.item * NC * CW);
    for (int t = threadIdx.x; t < NC * CW / 2; t += 256) {
      const int c = t / (CW / 2), q = t % (CW / 2);
      const d2 a = cbw[0][c][q], b = cbw[1][c][q], e = cbw[2][c][q], f = cbw[3][c][q];
      out[t] = d2{((a.x + b.x) + e.x) + f.x, ((a.y + b.y) + e.y) + f.y};
    }
  }
}

// one workgroup per panel, FIN_Q threads per panel row (row t = r0 + (thread
// & 255), part q = thread >> 8): part q sums the row's chunk row-parts
// item_begin + q, + 2q, ... and the column parts of the block's earlier panels
// q, q + FIN_Q, ...; the parts are then added in order q = 0..3.  The item
// offsets of the earlier panels are staged in LDS first, so the column-partial
// loads are independent of each other (no descriptor load in the chain) and,
// with NC a compile-time constant, unconditional: the compiler keeps them in
// flight together.  Splitting the chains 4 ways shortens the latency-bound
// loop (at one LD block per GPU the finalize was ~4 % of the pass).
template <int NC>
__global__ __launch_bounds__(256 * FIN_Q) void k_sym_finalize(const SymPanel* __restrict__ panels,
                                                              int cw, PassArgs pa,
                                                              const double* __restrict__ rowpart,
                                                              const double* __restrict__ colpart,
                                                              double* __restrict__ partials) {
  constexpr int PCH = 1024;   // panels staged per round
  __shared__ int s_ib[PCH];
  const SymPanel pn = panels[blockIdx.x];
  if (pa.run && !ldg(pa.run)) return;
  FinPre<NC> pre;
  fin_prefetch<NC>(pn, pa, pre);
  const int t = threadIdx.x & 255, q = threadIdx.x >> 8;
  double y[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) y[c] = 0.0;
  const int i = pn.r0 + (t < pn.H ? t : 0);   // block-relative row
  // this panel's row parts, chunk order within the part
#pragma unroll 4
  for (int itm = pn.item_begin + q; itm < pn.item_end; itm += FIN_Q) {
    const double* rp = rowpart + ((int64_t)itm * SYM_H + t) * NC;
#pragma unroll
    for (int c = 0; c < NC; ++c) y[c] += ldg(rp + c);
  }
  // column parts of the earlier panels of this block, panel order within the part
  // (band blocks: only the panels gmin .. g-1 store columns of these rows)
  for (int g0 = pn.gmin; g0 < pn.g; g0 += PCH) {
    const int gn = min(PCH, pn.g - g0);
    __syncthreads();
    for (int k = threadIdx.x; k < gn; k += 256 * FIN_Q)
      s_ib[k] = panels[pn.blk_panel0 + g0 + k].item_begin;
    __syncthreads();
#pragma unroll 4
    for (int k = q; k < gn; k += FIN_Q) {
      const int rel = i - (g0 + k) * SYM_H;      // column relative to that panel's first row
      const int ch = rel / cw;
      const double* cp = colpart + ((int64_t)(s_ib[k] + ch) * NC) * cw + (rel - ch * cw);
#pragma unroll
      for (int c = 0; c < NC; ++c) y[c] += ldg(cp + (int64_t)c * cw);
    }
  }
  fin_epilogue<NC>(pn, pa, y, partials, pre);
}

// the stored segments of a chunk only (bitwise the same; north-star blocks NC = 2
// -2.5 %, profiles/r03/sym_skip_ab.jsonl)
template <int NC, int NSEG>
static hipError_t launch_sym_nc(const SymItem* d_items, int nitems, const PassArgs& pa,
                                double* rowpart, double* colpart, hipStream_t st) {
  constexpr int RWI = (NC <= 2) ? 8 : (NC <= 4) ? 4 : (NC <= 8) ? 2 : 1;   // RWI*NC <= 16
  hipLaunchKernelGGL((k_sym_pass<NC, RWI, NSEG, true>), dim3(nitems), dim3(256), 0, st, d_items,
                     pa, rowpart, colpart);
  return hipGetLastError();
}

// (nc, class) -> instantiation; NSEG = 8 >> cls.  Supported classes per nc:
// nc <= 2: 0, 1;  nc <= 4: 1, 2;  nc <= 8: 2, 3;  nc <= 16: 3.
hipError_t launch_sym_pass(int nc, int cls, const SymItem* d_items, int nitems,
                           const PassArgs& pa, double* rowpart, double* colpart, hipStream_t st) {
#define SYM_CASE(N, C)                                                                       \
  if (nc == N && cls == C)                                                                   \
    return launch_sym_nc<N, (8 >> C)>(d_items, nitems, pa, rowpart, colpart, st);
  SYM_CASE(1, 0) SYM_CASE(1, 1) SYM_CASE(2, 0) SYM_CASE(2, 1)
  SYM_CASE(3, 1) SYM_CASE(3, 2) SYM_CASE(4, 1) SYM_CASE(4, 2)
  SYM_CASE(5, 2) SYM_CASE(5, 3) SYM_CASE(6, 2) SYM_CASE(6, 3) SYM_CASE(7, 2) SYM_CASE(7, 3)
  SYM_CASE(8, 2) SYM_CASE(8, 3)
  SYM_CASE(9, 3) SYM_CASE(10, 3) SYM_CASE(11, 3) SYM_CASE(12, 3) SYM_CASE(13, 3) SYM_CASE(14, 3)
  SYM_CASE(15, 3) SYM_CASE(16, 3)
#undef SYM_CASE
  return hipErrorInvalidValue;
}

// ---- coupled band pieces --------------------------------------------------
// One workgroup per (CouplingTask, 64-row quarter), CPL_NP waves: thread (q, r)
// sums the inner index range [q L, (q + 1) L) (L = ceil(inner / CPL_NP), in
// increasing k) for output row 64 y + r, and the CPL_NP parts are added in
// order 0, 1, ... -- a fixed order on every rank, so the coupling sums are the
// same whichever rank holds the source rows.  Per chunk of CPL_CH steps the
// workgroup stages each part's next CPL_CH source values (all NC columns) in
// LDS once, and every row thread reads them from there (one broadcast per
// column) instead of issuing NC global loads per inner index; the C loads of
// CPL_U consecutive steps go out before their FMAs.  Remote sources sit in
// the gathered halo [rank][2][nc][hstride]: task.src = 2 rank + slot.  Rows of
// a slot no task writes stay as cleared.
constexpr int CPL_CH = 32;
constexpr int CPL_U = 8;
// 8 parts: the band bench's pass -0.8 % against 4 (profiles/r05/cpl_parts_bench.jsonl)
template <int NC, int CPL_NP>   // CPL_NP: parts (waves) per workgroup
__global__ __launch_bounds__(64 * CPL_NP) void k_coupling_lds(
    const CouplingTask* __restrict__ tasks, PassArgs pa, const double* __restrict__ halo,
    int64_t hstride, double* __restrict__ cpbuf) {
  __shared__ double part[CPL_NP - 1][64][NC];
  __shared__ double s_src[CPL_NP][CPL_CH][NC];
  const CouplingTask tk = tasks[blockIdx.x];
  if (pa.run && !ldg(pa.run)) return;
  const int r = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int row = 64 * blockIdx.y + r;                 // within the task
  const bool live = row < tk.nrows;
  const int L = (tk.inner + CPL_NP - 1) / CPL_NP;
  const int k0 = q * L, k1 = min(tk.inner, k0 + L);
  const double* m = tk.m + tk.row0 + (live ? row : 0);
  double y[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) y[c] = 0.0;
  for (int i0 = 0; i0 < L; i0 += CPL_CH) {
    // stage: value (part qq, step ii, column c) = src_c[qq L + i0 + ii] inside the part's range
    for (int e = threadIdx.x; e < CPL_NP * CPL_CH * NC; e += 64 * CPL_NP) {
      const int c = e % NC, ii = (e / NC) % CPL_CH, qq = e / (NC * CPL_CH);
      const int k = qq * L + i0 + ii;
      const int kend = min(tk.inner, (qq + 1) * L);
      double v = 0.0;
      if (k < kend)
        v = tk.local ? pa.in[c][tk.src + k] : halo[(tk.src * NC + c) * hstride + k];
      s_src[qq][ii][c] = v;
    }
    __syncthreads();
    const int n = min(CPL_CH, k1 - (k0 + i0));   // this part's steps in the chunk (may be <= 0)
    if (live) {
      int ii = 0;
      for (; ii + CPL_U <= n; ii += CPL_U) {
        double a[CPL_U];
#pragma unroll
        for (int u = 0; u < CPL_U; ++u) a[u] = m[(int64_t)(k0 + i0 + ii + u) * tk.ldm];
#pragma unroll
        for (int u = 0; u < CPL_U; ++u)
#pragma unroll
          for (int c = 0; c < NC; ++c) y[c] += a[u] * s_src[q][ii + u][c];
      }
      for (; ii < n; ++ii) {
        const double a = m[(int64_t)(k0 + i0 + ii) * tk.ldm];
#pragma unroll
        for (int c = 0; c < NC; ++c) y[c] += a * s_src[q][ii][c];
      }
    }
    __syncthreads();
  }
  if (q > 0) {
#pragma unroll
    for (int c = 0; c < NC; ++c) part[q - 1][r][c] = y[c];
  }
  __syncthreads();
  if (q == 0 && live) {
    double* out = cpbuf + ((int64_t)tk.cp * 256 + tk.prow0 + row) * NC;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      double v = y[c];
#pragma unroll
      for (int p = 0; p < CPL_NP - 1; ++p) v += part[p][r][c];
      out[c] = v;
    }
  }
}

hipError_t launch_coupling(int nc, const CouplingTask* d_tasks, int ntasks, const PassArgs& pa,
                           const double* halo, int64_t hstride, double* cpbuf, int ncp_slots,
                           hipStream_t st) {
  if (ntasks <= 0) return hipSuccess;
  const hipError_t e = hipMemsetAsync(cpbuf, 0, sizeof(double) * (size_t)ncp_slots * 256 * nc, st);
  if (e != hipSuccess) return e;
#define CPL_CASE(N)                                                                          \
  case N:                                                                                    \
    hipLaunchKernelGGL((k_coupling_lds<N, 8>), dim3(ntasks, 4), dim3(512), 0, st, d_tasks,   \
                       pa, halo, hstride, cpbuf);                                            \
    break;
  switch (nc) {
    CPL_CASE(1) CPL_CASE(2) CPL_CASE(3) CPL_CASE(4) CPL_CASE(5) CPL_CASE(6) CPL_CASE(7) CPL_CASE(8)
    CPL_CASE(9) CPL_CASE(10) CPL_CASE(11) CPL_CASE(12) CPL_CASE(13) CPL_CASE(14) CPL_CASE(15)
    CPL_CASE(16)
    default: return hipErrorInvalidValue;
  }
#undef CPL_CASE
  return hipGetLastError();
}

// the halo a rank sends: per slot s (0: head of its first block, 1: tail of its
// last), nc columns of hstride doubles (len[s] used, the rest zero)
__global__ __launch_bounds__(256) void k_halo_pack(PassArgs pa, int nc, int64_t src0, int len0,
                                                   int64_t src1, int len1, int64_t hstride,
                                                   double* __restrict__ send) {
  if (pa.run && !ldg(pa.run)) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= hstride) return;
  const int s = blockIdx.y, c = blockIdx.z;
  const int len = s ? len1 : len0;
  const int64_t src = s ? src1 : src0;
  send[((int64_t)s * nc + c) * hstride + j] = j < len ? pa.in[c][src + j] : 0.0;
}

hipError_t launch_halo_pack(const PassArgs& pa, int nc, int64_t src0, int len0, int64_t src1,
                            int len1, int64_t hstride, double* send, hipStream_t st) {
  hipLaunchKernelGGL(k_halo_pack, dim3((unsigned)((hstride + 255) / 256), 2, nc), dim3(256), 0, st,
                     pa, nc, src0, len0, src1, len1, hstride, send);
  return hipGetLastError();
}

hipError_t launch_sym_finalize(int nc, int cls, const SymPanel* d_panels, int npanels,
                               const PassArgs& pa, const double* rowpart, const double* colpart,
                               double* partials, hipStream_t st) {
  const int cw = 1024 >> cls;
#define FIN_CASE(N)                                                                              \
  case N:                                                                                        \
    hipLaunchKernelGGL(k_sym_finalize<N>, dim3(npanels), dim3(256 * FIN_Q), 0, st, d_panels, cw, pa,     \
                       rowpart, colpart, partials);                                              \
    break;
  switch (nc) {
    FIN_CASE(1) FIN_CASE(2) FIN_CASE(3) FIN_CASE(4) FIN_CASE(5) FIN_CASE(6) FIN_CASE(7) FIN_CASE(8)
    FIN_CASE(9) FIN_CASE(10) FIN_CASE(11) FIN_CASE(12) FIN_CASE(13) FIN_CASE(14) FIN_CASE(15)
    FIN_CASE(16)
    default: return hipErrorInvalidValue;
  }
#undef FIN_CASE
  return hipGetLastError();
}

}  // namespace sgv
