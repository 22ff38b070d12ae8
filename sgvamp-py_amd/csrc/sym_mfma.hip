// Multi-RHS symmetric LD pass on the f64 matrix cores.
//
// For 3..16 right-hand sides a VALU pass runs out of operands before HBM runs
// out of bytes: each stored R_ij feeds 2*NC FMAs whose P operands must sit in
// registers, so the VALU kernels (sym_pass.hip) re-read P or spill column
// partials through LDS at a multiple of the HBM traffic.  An MFMA takes ONE
// f64 of R and ONE f64 of P per lane and lets the matrix core do the register
// blocking.  Of the two f64 shapes, v_mfma_f64_4x4x4f64 (4 blocks of 4x4x4)
// costs 17 cycles for 256 MACs (~71 TF) and v_mfma_f64_16x16x4f64 140 cycles
// for 1024 (~47 TF) (tools/mfma_probe.hip; one accumulator chain: 44 / 184
// cycles per MFMA, 4 chains 18 / 144); the 4x4x4 form also needs only
// ceil(NC/4) column groups instead of padding to 16.  Per 16x32 sub-tile
// (4 KiB of R) the pass issues 16 * ceil(NC/4) of them (~270 cycles per group),
// under the ~1300-1500 cycles the same bytes take to arrive from HBM.
//
// 4x4x4 f64 lane maps (probed): block b = (l>>2)&3;
//   A_b[m][k] at lane 16k + 4b + m,  B_b[k][n] at lane 16k + 4b + n,
//   D_b[m][n] at lane 16m + 4b + n.
//
// Work items are strips (see k_sym_mfma): one 512-column chunk over several
// panels.  Row sums go to rowpart[item][256][NC] per (panel, chunk) item as in
// the VALU pass (class 1), column sums to colpart[strip][NC][512];
// k_sym_finalize_strip combines them.
//
// One workgroup per strip, NW waves; wave w owns chunk columns
// [w*512/NW, (w+1)*512/NW) and sweeps each panel's rows in 16-row groups.
// Each 16 x 32 sub-tile is loaded from HBM once, 16 B per lane:
//   col fragment  lane l: R[row 4a + (l>>4)][col pair (l&15), + e]   (a = 0..3)
//       A_b[m][k] = R[row k][pair 4b+m]: Dcol[pair][c] += R[j][i] P[j][c]
// and written to a per-wave LDS tile (16 x 32, XOR-swizzled 16-B pieces) from which
//   row fragment  lane l: R[row 4q + (l&3)][col pair (l>>4) + 4b, + e] (q = 0..3)
//       A_b[m][k] = R[row m][pair k+4b]: Drow[row][c] += R[j][i] P[i][c]
// is read back without bank conflicts.  Each 4x4x4 block contracts its own 4
// column pairs, so the 4 blocks' row partials are summed by two DPP row
// rotations per row group (fixed order), then over the waves through LDS (wave
// order).
// Dcol accumulates over all rows of the strip in registers; every order is fixed.
#include "common.h"

namespace sgv {

#define MFMA4(a, b, c) __builtin_amdgcn_mfma_f64_4x4x4f64((a), (b), (c), 0, 0, 0)

// Diagnostic build only (make EXTRA=-DSGV_MF_TRACE, tools/strip_trace.py): each
// workgroup (strip) of the last NC <= 8 MFMA pass records its start / end wall
// clock (100 MHz) and CU, to see how the launch fills the device.  Not in the
// product library.
#ifdef SGV_MF_TRACE
constexpr int MF_TRACE_MAX = 1 << 16;
__device__ unsigned long long g_mf_trace[3 * MF_TRACE_MAX];
#define MF_TRACE_BEGIN const unsigned long long tr_t0 = wall_clock64();
#define MF_TRACE_END                                                          \
  __syncthreads();                                                            \
  if (threadIdx.x == 0 && blockIdx.x < MF_TRACE_MAX) {                        \
    g_mf_trace[3 * blockIdx.x] = tr_t0;                                       \
    g_mf_trace[3 * blockIdx.x + 1] = wall_clock64();                          \
    g_mf_trace[3 * blockIdx.x + 2] = (unsigned long long)__smid();            \
  }
#else
#define MF_TRACE_BEGIN
#define MF_TRACE_END
#endif

// wave-local LDS ordering point: lanes of one wave exchange data through the
// tile.  The LDS executes a wave's DS instructions in order, so the write ->
// read (and read -> next write) order only has to survive compilation: a
// wavefront-scope fence, which emits no wait (an inline-asm lgkmcnt(0) would
// make the compiler drain vmcnt as well, stalling on the prefetched loads).
__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

constexpr int MF_CW = 512;   // chunk width (class 1 items)
constexpr int MF_LDP = 34;   // k_sym_mfma16's staging row pitch (doubles): conflict-free both ways

// Strips: a workgroup owns one 512-column chunk over up to S panels of one
// parity (g0, g0 + 2, ...: the panels whose items share that chunk's column
// alignment), so the column sums stay in registers across the panels and reach
// HBM once per strip instead of once per (panel, chunk) item.  The chunk's
// diagonal panel (r0 == c0) is the strip's last; its diagonal block (chunk
// columns 0..255, waves 0 and 1) must not feed the column sums, so those waves
// take zero B operands there (exact: R * 0 adds 0).  Row sums are still written
// per (panel, chunk) item.  Panel descriptors are wave-uniform (SGPRs); the
// prefetch of the next row group crosses panel boundaries through selects.
// Each wave keeps its row sums of the whole panel in its own LDS rows
// (wrow[wave][row][4 NG]); the four waves' values are added, in wave order, once
// per panel when the item's row partials are written (one barrier pair per
// panel).  Steps at or past the chunk's last column take no LDS or MFMA work.
// DEF: a step's row MFMAs are deferred into the next step and interleaved with
// its column MFMAs, so consecutive MFMAs of one accumulator chain sit 8 issues
// apart instead of 4 (2 at NG = 1); every chain accumulates in the same order
// (bitwise the same sums), the row fragments are double-buffered in registers.
// RAG: some item of the strip stops short of the strip's widest (band plans).
// PP (NG = 2): Pk in k_pack's PAIRED layout, so a lane's two column groups
// (columns n4 and 4 + n4) of one Pk row are one 16-B load: half the P-operand
// load instructions through the texture-address unit per row group
// SWZ (NG = 2): column-part B operands without the 4x replication over the
// MFMA blocks: blocks 0-1 take a row group's 4-row sets in the order 0 1 2 3,
// blocks 2-3 in the order 2 3 0 1 (fragment a of a lane is row set a ^ (bq &
// 2)), so one Pk load per row group (lane: row set bq) holds every set a block
// needs and ds_swizzle hands each lane its set for fragment a (swz_quad); the
// R fragment loads stay whole 128-B lines.  One box, alternating: the north
// star -0.4...-0.8 % per pass, the 8-block share -1.4 %; at NG = 1 (8-B
// operands) even to +0.4 %, so not there (profiles/r06/mf_sw_*.jsonl)
template <int NG, int PD, bool RAG = false, bool DEF = false, bool PP = false>
__global__ __launch_bounds__(256, 2) void k_sym_mfma(const SymStrip* __restrict__ strips,
                                                     const SymItem* __restrict__ sitems,
                                                     const double* __restrict__ pk, int ncol,
                                                     double* __restrict__ rowpart,
                                                     double* __restrict__ colpart,
                                                     const int* __restrict__ run, int pks) {
  constexpr int NW = 4;            // waves 0 and 1 own the diagonal half of a chunk
  constexpr int WC = MF_CW / NW;   // columns per wave
  constexpr int NT = WC / 32;      // 32-column steps per wave
  static_assert(PD >= 1 && PD <= NT && NT % PD == 0, "prefetch depth divides the steps");
  constexpr int RW = 4 * NG;       // row-sum stride of wrow
  constexpr bool SWZ = NG == 2;
  __shared__ __attribute__((aligned(16))) double rowbuf[NW * SYM_H * RW];   // wrow
  // the per-wave transpose tile: 16 rows x 32 columns, 16-B piece (row r, pair
  // p) at slot 16 r + (p ^ (r & 3)) -- unpadded (4 KiB, so the 64 KiB of row
  // sums and the tiles fit two workgroups per CU) and conflict-free both ways:
  // a write's 16-lane quarter covers one row, a row-fragment read's quarter
  // (rows 4q + (l & 3), pairs 4((l >> 2) & 3) + (l >> 4)) 16 distinct slots mod 16
  __shared__ __attribute__((aligned(16))) double stg[NW][16 * 32];
  const SymStrip sp = strips[blockIdx.x];
  if (run && !ldg(run)) return;   // no-op pass (pipelined CG past its stop test)
  MF_TRACE_BEGIN
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int lo = lane & 15, hi = lane >> 4, bq = (lane >> 2) & 3, n4 = lane & 3;
  const int pc = hi + 4 * bq;                          // this lane's column pair in a fragment
  SymItem cur = sitems[sp.it0];
  const int c0 = cur.c0, ncc = sp.ncmax;               // the strip's chunk, widest item
  const int PKS = pks;             // Pk row stride (k_pack): 4 NG
  const double* pkb = pk + (int64_t)cur.voff * PKS;   // Pk of this block (block-relative index)
  const int cw0 = wid * WC;                            // first chunk column of this wave
  const bool dhalf = cw0 < SYM_H;                      // wave inside a diagonal panel's diag block
  // A wave's 32-column steps at or past the chunk's last column (the
  // ragged last chunk of a panel: 4 % of the north star's steps) take no LDS or
  // MFMA work -- their row-part B operands are 0 and their column sums are never
  // read, so every kept sum is bitwise the same; nor do the column MFMAs of the
  // diagonal-block waves of a diagonal panel (B = 0 there).  The loads stay, so
  // the load count is the same on every path.
  const int nta = min(NT, max(0, (ncc - cw0 + 31) / 32));
  double* sb = stg[wid];

  // row-part B operands: P at this wave's columns, reused by every row group
  static_assert(!PP || NG == 2, "paired Pk rows: two column groups");
  // one Pk row's values of this lane: column 4 q + n4 for each group q
  auto ld_prow = [&](int64_t row, double* v) {
    if constexpr (PP) {
      const d2 x = ldg((const d2*)(pkb + row * PKS + 2 * n4));
      v[0] = x.x;
      v[1] = x.y;
    } else {
#pragma unroll
      for (int q = 0; q < NG; ++q) v[q] = ldg(pkb + row * PKS + 4 * q + n4);
    }
  };
  double brow[NT][2][NG];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int col = cw0 + 32 * t + 2 * pc + e;
      double v[NG];
      ld_prow(c0 + (col < ncc ? col : 0), v);
#pragma unroll
      for (int q = 0; q < NG; ++q) brow[t][e][q] = col < ncc ? v[q] : 0.0;
    }
  double dcol[NT][2][NG];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int q = 0; q < NG; ++q) dcol[t][e][q] = 0.0;

  // fragment loads of step (g, t) of a panel (b0 = its element (r0, c0)), 16 B
  // per lane, branch-free: a row past H clamps (its P is 0), a column past the
  // chunk loads column 0 (finite; it meets a zero B in the row part and is never
  // read from the column part).  The base is an opaque integer: a pointer select
  // is turned back into a branch with one load per side.  Past the strip's last
  // row group the caller passes the cache-resident Pk with stride 0 (a dummy
  // fetch: the load count is the same on every path, so the compiler never
  // drains vmcnt(0) at a branch join or the row-group loop head).
  auto load_cf = [&](uint64_t b0, int64_t ws, int H, int nci, int g, int t, d2* cf) {
    asm volatile("" : "+s"(b0));
    const int xc = cw0 + 32 * t + 2 * lo;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int rB = 16 * g + 4 * (SWZ ? a ^ (bq & 2) : a) + hi;
      const double* row = (const double*)b0 + (int64_t)(rB < H ? rB : H - 1) * ws;
      cf[a] = ldg_nt((const d2*)(row + (xc < (RAG ? nci : ncc) ? xc : 0)));
    }
  };
  // column-part B operands of row group g of a panel (first row r0): P at its
  // rows; zero past H and, for the diagonal panel, in the diagonal-block waves
  // (SWZ: bc[0] = this lane's row set bq, handed to the fragments by swz_quad)
  auto load_bcol = [&](int r0, int H, bool zero, int g, double (*bc)[NG]) {
#pragma unroll
    for (int a = 0; a < (SWZ ? 1 : 4); ++a) {
      const int rB = 16 * g + 4 * (SWZ ? bq : a) + hi;
      double v[NG];
      ld_prow(r0 + (rB < H ? rB : 0), v);
#pragma unroll
      for (int q = 0; q < NG; ++q) bc[a][q] = (rB < H && !zero) ? v[q] : 0.0;
    }
  };
  auto pbase = [&](const SymItem& x) { return (uint64_t)(x.P + (x.c0 - x.r0)); };
  // a band panel's item narrower than the strip: its columns past nci (never
  // loaded: the loads above took column 0) read as zero
  auto band_zero = [&](int nci, int t, d2* cf) {
    const int xc = cw0 + 32 * t + 2 * lo;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      cf[a].x = xc < nci ? cf[a].x : 0.0;
      cf[a].y = xc + 1 < nci ? cf[a].y : 0.0;
    }
  };

  uint64_t curb = pbase(cur);
  // ring of PD steps in flight per wave
  d2 cfq[PD][4];
  double bcn[SWZ ? 1 : 4][NG];
#pragma unroll
  for (int p = 0; p < PD; ++p) load_cf(curb, cur.w, cur.H, cur.nc, 0, p, cfq[p]);
  load_bcol(cur.r0, cur.H, dhalf && cur.r0 == c0, 0, bcn);

#pragma unroll 1
  for (int s = 0; s < sp.npan; ++s) {                  // uniform over the workgroup
    const bool more = s + 1 < sp.npan;
    const SymItem nx = sitems[sp.it0 + (more ? s + 1 : s)];
    const uint64_t nxb = more ? pbase(nx) : (uint64_t)pkb;
    const int ng = (cur.H + 15) / 16;
#pragma unroll 1
    for (int g = 0; g < ng; ++g) {
      // the next row group: this panel's g + 1, or the next panel's first
      const bool same = g + 1 < ng;
      const uint64_t gb = same ? curb : nxb;
      const int64_t gw = same ? cur.w : (more ? nx.w : 0);
      const int gH = same ? cur.H : (more ? nx.H : 1);
      const int gnc = same ? cur.nc : nx.nc;
      const int gn = same ? g + 1 : 0;
      const int gr0 = same ? cur.r0 : nx.r0;
      const bool gz = dhalf && gr0 == c0;
      double bcol[4][NG];
      // fragment a's set a ^ (bq & 2) from the lane of quad a ^ (bq & 2) of
      // this 16-lane row
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int q = 0; q < NG; ++q) bcol[a][q] = SWZ ? swz_quad(bcn[0][q], a) : bcn[SWZ ? 0 : a][q];
      double drow[4][NG];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < NG; ++q) drow[r][q] = 0.0;
      const bool colz = dhalf && cur.r0 == c0;   // this panel's column B operands are 0
      // a band item narrower than its strip (its panel's last 256 columns): a
      // step wholly past its stored end adds only zeros -- skipped like the
      // steps past the chunk; per panel, so the deferred row MFMAs (DEF) know
      // the item's last active step
      const int ntp = RAG ? min(nta, max(0, (cur.nc - cw0 + 31) / 32)) : nta;
      d2 rfb[DEF ? 2 : 1][4];                            // row fragments (DEF: this and the previous step)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        d2 cf[4];
        d2* rf = rfb[DEF ? (t & 1) : 0];
        const int slot = t % PD;                       // compile-time after unrolling
#pragma unroll
        for (int a = 0; a < 4; ++a) cf[a] = cfq[slot][a];
        // step + PD goes out here, ahead of this step's LDS and MFMA work
        if (t + PD < NT) {
          load_cf(curb, cur.w, cur.H, cur.nc, g, t + PD, cfq[slot]);
        } else {
          load_cf(gb, gw, gH, gnc, gn, t + PD - NT, cfq[slot]);
          if (t + PD == NT) load_bcol(gr0, gH, gz, gn, bcn);
        }
        if (t >= ntp) continue;                        // wave-uniform: past the chunk / item
        if (RAG && cur.nc < ncc) band_zero(cur.nc, t, cf);   // uniform: a band item's stored end
        lds_order();                                   // previous step's tile reads issued
#pragma unroll
        for (int a = 0; a < 4; ++a)
          *(d2*)(sb + 32 * (4 * (SWZ ? a ^ (bq & 2) : a) + hi) + 2 * (lo ^ hi)) = cf[a];
        lds_order();                                   // tile written
        // the row fragment reads go out right behind the writes (a wave's DS
        // operations execute in order); the column MFMAs cover their latency
#pragma unroll
        for (int r = 0; r < 4; ++r) rf[r] = *(const d2*)(sb + 32 * (4 * r + n4) + 2 * (pc ^ n4));
        // the MFMA burst at raised wave priority: the SIMD's other wave, whose
        // loads are in flight, takes the issue slots back when this one drains
        // (NC = 4/8 0.7-1.5 % faster per pass on two boxes; NC = 16 1 % slower,
        // not used there -- profiles/r02s10_prio_ab.txt)
        __builtin_amdgcn_s_setprio(1);
        // x halves of all 4*NG row chains, then the y halves: a chain's two MFMAs
        // are 4*NG issues apart instead of back to back (same per-chain order)
        auto row_mfma = [&](const d2* f, int tt) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < NG; ++q) drow[r][q] = MFMA4(f[r].x, brow[tt][0][q], drow[r][q]);
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < NG; ++q) drow[r][q] = MFMA4(f[r].y, brow[tt][1][q], drow[r][q]);
        };
        if constexpr (DEF) {
          // column level a of this step, then a quarter of the previous step's
          // row MFMAs (x halves of rows 2(a&1), +1 for a < 2, then the y halves)
          const d2* rp = rfb[(t + 1) & 1];
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            if (!colz) {
#pragma unroll
              for (int q = 0; q < NG; ++q) {
                dcol[t][0][q] = MFMA4(cf[a].x, bcol[a][q], dcol[t][0][q]);
                dcol[t][1][q] = MFMA4(cf[a].y, bcol[a][q], dcol[t][1][q]);
              }
            }
            if (t > 0) {
              const int tp = t > 0 ? t - 1 : 0;
#pragma unroll
              for (int r = 2 * (a & 1); r < 2 * (a & 1) + 2; ++r)
#pragma unroll
                for (int q = 0; q < NG; ++q)
                  drow[r][q] = MFMA4(a < 2 ? rp[r].x : rp[r].y, brow[tp][a < 2 ? 0 : 1][q], drow[r][q]);
            }
          }
          // the row group's last active step: its own row MFMAs now
          if (t == NT - 1 || t + 1 == ntp) row_mfma(rf, t);
        } else {
          if (!colz) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
              for (int q = 0; q < NG; ++q) {
                dcol[t][0][q] = MFMA4(cf[a].x, bcol[a][q], dcol[t][0][q]);
                dcol[t][1][q] = MFMA4(cf[a].y, bcol[a][q], dcol[t][1][q]);
              }
          }
          row_mfma(rf, t);
        }
        __builtin_amdgcn_s_setprio(0);
      }
      // row sums: the 4 blocks (lanes differing in bits 2,3; DPP row rotations),
      // kept per wave for the panel
      double* wb = rowbuf + (wid * SYM_H + 16 * g) * RW;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < NG; ++q) {
          double v = drow[r][q];
          v = v + row_ror<12>(v);
          v = v + row_ror<8>(v);
          if (bq == 0) wb[(4 * r + hi) * RW + 4 * q + n4] = v;   // D row 4r + m (m = hi)
        }
    }
    {   // the item's H x ncol row sums: waves in order, contiguous in rowpart
      __syncthreads();
      const int n = cur.H * ncol;
      double* dst = rowpart + (int64_t)cur.item * SYM_H * ncol;
      for (int i = threadIdx.x; 2 * i < n; i += NW * 64) {
        double v[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int k = 2 * i + e < n ? 2 * i + e : 2 * i;
          const int row = k / ncol, cc = k - row * ncol;
          const double* src = rowbuf + row * RW + cc;
          double x = src[0];
#pragma unroll
          for (int w = 1; w < NW; ++w) x += src[w * SYM_H * RW];
          v[e] = x;
        }
        if (2 * i + 1 < n)
          *(d2*)(dst + 2 * i) = d2{v[0], v[1]};
        else
          dst[2 * i] = v[0];
      }
      __syncthreads();    // the waves' rows are read before the next panel writes them
    }
    cur = nx;
    curb = nxb;
  }

  // column sums over the strip's panels: D_b[m][n] at lane 16m + 4b + n holds
  // column pair 4b + m = pc, column c = 4q + n.  Whole slot, 16-B stores
  // (columns the finalize never reads: don't care).
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int cc = 4 * q + n4;
    if (cc < ncol) {
      double* out = colpart + ((int64_t)sp.slot * ncol + cc) * MF_CW;
#pragma unroll
      for (int t = 0; t < NT; ++t)
        *(d2*)(out + cw0 + 32 * t + 2 * pc) = d2{dcol[t][0][q], dcol[t][1][q]};
    }
  }
  MF_TRACE_END
}

// Wave-pair form of k_sym_mfma (no band items): one 8-wave workgroup
// per strip, TWO waves per 128-column segment, each owning 64 columns (two
// 32-column steps).  Every sum is the 4-wave kernel's, bit for bit:
//  * a column's sum is one MFMA chain over the strip's rows in one wave, as
//    there (its wave only changed);
//  * a row's sum over a segment is the chain x0 y0 x1 y1 x2 y2 x3 y3 over the
//    segment's four steps: the first wave of the pair runs steps 0-1 from zero
//    and hands its accumulators (4 NG doubles per lane) through LDS to the
//    second, which continues with steps 2-3 -- the same MFMAs in the same order
//    -- then reduces the 4 blocks (DPP) and keeps the segment's panel row sums
//    (wrow), added over the 4 segments in order per panel as there.
// So a strip takes half the time on a workgroup holding a whole CU (8 waves, 1
// per CU: the same 2 waves per SIMD): a launch whose strips are few per slot
// (an 8-block share: ~2 strips of up to 8 panels per slot of the 4-wave form)
// drains with half the tail, with products identical to the 4-wave kernel's --
// the form can be chosen per partition.  One barrier per 16-row group: the
// hand-off (first wave: accumulators out before it; second wave: in after it,
// double-buffered by row-group parity).
// Waves s and s + 4 hold segment s (waves are dealt to SIMDs round-robin: the
// pair shares one SIMD, each SIMD runs one first and one second half); each
// pair syncs on its own LDS counters (the first wave up to HS - 1 row groups
// ahead, a ring of HS hand-off slots), barriers only at panel ends.  The other
// forms measured -- pair on two SIMDs, a barrier per row group -- were slower
// 
template <int NG, int PD, bool PP = false>
__global__ __launch_bounds__(512, 1) void k_sym_mfma_pair(const SymStrip* __restrict__ strips,
                                                          const SymItem* __restrict__ sitems,
                                                          const double* __restrict__ pk, int ncol,
                                                          double* __restrict__ rowpart,
                                                          double* __restrict__ colpart,
                                                          const int* __restrict__ run, int pks) {
  constexpr int NW = 8;
  constexpr int WC = 64;           // columns per wave
  constexpr int NT = WC / 32;      // 32-column steps per wave
  static_assert(PD >= 1 && PD <= NT && NT % PD == 0, "prefetch depth divides the steps");
  constexpr int RW = 4 * NG;
  constexpr bool SWZ = NG == 2;   // k_sym_mfma's row sets
  __shared__ __attribute__((aligned(16))) double wrow[4 * SYM_H * RW];   // [segment][row][4 NG]
  constexpr int HS = 3;                                                    // hand-off slots
  __shared__ __attribute__((aligned(16))) double hand[HS][4][4 * NG][WAVE];   // [gg % HS][segment][r, q][lane]
  __shared__ int hready[4], hdone[4];   // row groups handed / taken per segment
  __shared__ __attribute__((aligned(16))) double stg[NW][16 * 32];
  const SymStrip sp = strips[blockIdx.x];
  if (run && !ldg(run)) return;
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int seg = wid & 3;                               // 128-column segment
  const int h = wid >> 2;                                // half
  const int lo = lane & 15, hi = lane >> 4, bq = (lane >> 2) & 3, n4 = lane & 3;
  const int pc = hi + 4 * bq;
  SymItem cur = sitems[sp.it0];
  const int c0 = cur.c0, ncc = sp.ncmax;
  const int PKS = pks;
  const double* pkb = pk + (int64_t)cur.voff * PKS;
  const int cw0 = seg * 128 + h * WC;                    // first chunk column of this wave
  const bool dhalf = seg * 128 < SYM_H;                  // the 4-wave kernel's wave `seg`
  // the segment's active 32-column steps (the 4-wave kernel's nta), this wave's share
  const int nta_seg = min(4, max(0, (ncc - seg * 128 + 31) / 32));
  const int nta = min(NT, max(0, nta_seg - NT * h));
  double* sb = stg[wid];

  static_assert(!PP || NG == 2, "paired Pk rows: two column groups");
  auto ld_prow = [&](int64_t row, double* v) {   // as k_sym_mfma's
    if constexpr (PP) {
      const d2 x = ldg((const d2*)(pkb + row * PKS + 2 * n4));
      v[0] = x.x;
      v[1] = x.y;
    } else {
#pragma unroll
      for (int q = 0; q < NG; ++q) v[q] = ldg(pkb + row * PKS + 4 * q + n4);
    }
  };
  double brow[NT][2][NG];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int col = cw0 + 32 * t + 2 * pc + e;
      double v[NG];
      ld_prow(c0 + (col < ncc ? col : 0), v);
#pragma unroll
      for (int q = 0; q < NG; ++q) brow[t][e][q] = col < ncc ? v[q] : 0.0;
    }
  double dcol[NT][2][NG];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int q = 0; q < NG; ++q) dcol[t][e][q] = 0.0;

  auto load_cf = [&](uint64_t b0, int64_t ws, int H, int g, int t, d2* cf) {
    asm volatile("" : "+s"(b0));
    const int xc = cw0 + 32 * t + 2 * lo;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int rB = 16 * g + 4 * (SWZ ? a ^ (bq & 2) : a) + hi;
      const double* row = (const double*)b0 + (int64_t)(rB < H ? rB : H - 1) * ws;
      cf[a] = ldg_nt((const d2*)(row + (xc < ncc ? xc : 0)));
    }
  };
  auto load_bcol = [&](int r0, int H, bool zero, int g, double (*bc)[NG]) {
#pragma unroll
    for (int a = 0; a < (SWZ ? 1 : 4); ++a) {
      const int rB = 16 * g + 4 * (SWZ ? bq : a) + hi;
      double v[NG];
      ld_prow(r0 + (rB < H ? rB : 0), v);
#pragma unroll
      for (int q = 0; q < NG; ++q) bc[a][q] = (rB < H && !zero) ? v[q] : 0.0;
    }
  };
  auto pbase = [&](const SymItem& x) { return (uint64_t)(x.P + (x.c0 - x.r0)); };

  uint64_t curb = pbase(cur);
  d2 cfq[PD][4];
  double bcn[SWZ ? 1 : 4][NG];
#pragma unroll
  for (int p = 0; p < PD; ++p) load_cf(curb, cur.w, cur.H, 0, p, cfq[p]);
  load_bcol(cur.r0, cur.H, dhalf && cur.r0 == c0, 0, bcn);
  if (threadIdx.x < 4) hready[threadIdx.x] = hdone[threadIdx.x] = 0;
  __syncthreads();
  auto lds_wait_ge = [&](int* ctr, int v) {
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v)
      __builtin_amdgcn_s_sleep(1);
  };

  int gg = 0;
#pragma unroll 1
  for (int s = 0; s < sp.npan; ++s) {
    const bool more = s + 1 < sp.npan;
    const SymItem nx = sitems[sp.it0 + (more ? s + 1 : s)];
    const uint64_t nxb = more ? pbase(nx) : (uint64_t)pkb;
    const int ng = (cur.H + 15) / 16;
#pragma unroll 1
    for (int g = 0; g < ng; ++g, ++gg) {
      const bool same = g + 1 < ng;
      const uint64_t gb = same ? curb : nxb;
      const int64_t gw = same ? cur.w : (more ? nx.w : 0);
      const int gH = same ? cur.H : (more ? nx.H : 1);
      const int gn = same ? g + 1 : 0;
      const int gr0 = same ? cur.r0 : nx.r0;
      const bool gz = dhalf && gr0 == c0;
      double bcol[4][NG];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int q = 0; q < NG; ++q) bcol[a][q] = SWZ ? swz_quad(bcn[0][q], a) : bcn[SWZ ? 0 : a][q];
      double drow[4][NG];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < NG; ++q) drow[r][q] = 0.0;
      const bool colz = dhalf && cur.r0 == c0;
      d2 rfs[NT][4];                                     // h = 1: row fragments, used after the hand-off
      auto row_mfma = [&](const d2* f, int tt) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < NG; ++q) drow[r][q] = MFMA4(f[r].x, brow[tt][0][q], drow[r][q]);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < NG; ++q) drow[r][q] = MFMA4(f[r].y, brow[tt][1][q], drow[r][q]);
      };
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        d2 cf[4];
        const int slot = t % PD;
#pragma unroll
        for (int a = 0; a < 4; ++a) cf[a] = cfq[slot][a];
        if (t + PD < NT) {
          load_cf(curb, cur.w, cur.H, g, t + PD, cfq[slot]);
        } else {
          load_cf(gb, gw, gH, gn, t + PD - NT, cfq[slot]);
          if (t + PD == NT) load_bcol(gr0, gH, gz, gn, bcn);
        }
        if (t >= nta) continue;
        d2* rf = rfs[t];
        lds_order();
#pragma unroll
        for (int a = 0; a < 4; ++a)
          *(d2*)(sb + 32 * (4 * (SWZ ? a ^ (bq & 2) : a) + hi) + 2 * (lo ^ hi)) = cf[a];
        lds_order();
#pragma unroll
        for (int r = 0; r < 4; ++r) rf[r] = *(const d2*)(sb + 32 * (4 * r + n4) + 2 * (pc ^ n4));
        __builtin_amdgcn_s_setprio(1);
        if (!colz) {
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int q = 0; q < NG; ++q) {
              dcol[t][0][q] = MFMA4(cf[a].x, bcol[a][q], dcol[t][0][q]);
              dcol[t][1][q] = MFMA4(cf[a].y, bcol[a][q], dcol[t][1][q]);
            }
        }
        if (h == 0) row_mfma(rf, t);                     // the chain's first half
        __builtin_amdgcn_s_setprio(0);
      }
      double* hs = &hand[gg % HS][seg][0][0];
      if (h == 0) {
        lds_wait_ge(&hdone[seg], gg - HS + 1);   // slot gg % HS taken back
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < NG; ++q) hs[(r * NG + q) * WAVE + lane] = drow[r][q];
        __hip_atomic_store(&hready[seg], gg + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (h == 1) {
        lds_wait_ge(&hready[seg], gg + 1);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < NG; ++q) drow[r][q] = hs[(r * NG + q) * WAVE + lane];
        __hip_atomic_store(&hdone[seg], gg + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (t < nta) row_mfma(rfs[t], t);             // the chain's second half
        __builtin_amdgcn_s_setprio(0);
        double* wb = wrow + (seg * SYM_H + 16 * g) * RW;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < NG; ++q) {
            double v = drow[r][q];
            v = v + row_ror<12>(v);
            v = v + row_ror<8>(v);
            if (bq == 0) wb[(4 * r + hi) * RW + 4 * q + n4] = v;
          }
      }
    }
    {   // the item's H x ncol row sums: segments in order, contiguous in rowpart
      __syncthreads();
      const int n = cur.H * ncol;
      double* dst = rowpart + (int64_t)cur.item * SYM_H * ncol;
      for (int i = threadIdx.x; 2 * i < n; i += NW * 64) {
        double v[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int k = 2 * i + e < n ? 2 * i + e : 2 * i;
          const int row = k / ncol, cc = k - row * ncol;
          const double* src = wrow + row * RW + cc;
          double x = src[0];
#pragma unroll
          for (int w = 1; w < 4; ++w) x += src[w * SYM_H * RW];
          v[e] = x;
        }
        if (2 * i + 1 < n)
          *(d2*)(dst + 2 * i) = d2{v[0], v[1]};
        else
          dst[2 * i] = v[0];
      }
      __syncthreads();
    }
    cur = nx;
    curb = nxb;
  }
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int cc = 4 * q + n4;
    if (cc < ncol) {
      double* out = colpart + ((int64_t)sp.slot * ncol + cc) * MF_CW;
#pragma unroll
      for (int t = 0; t < NT; ++t)
        *(d2*)(out + cw0 + 32 * t + 2 * pc) = d2{dcol[t][0][q], dcol[t][1][q]};
    }
  }
}

// 13..16 right-hand sides: v_mfma_f64_16x16x4f64 (one 16-column group, 140
// cycles per 16x16x4) keeps fewer accumulators and B operands in registers
// than four 4x4x4 groups, which spill at 4 waves.  Same strips as above:
//   col fragment -> A (m = column, k = row); LDS tile -> row fragment
//   lane l: R[row (l&15)][col 8s + 2(l>>4) + e] -> A (m = row, k = column);
//   16x16x4 f64 C/D layout (cdna_hip_programming.md): D[(l>>4) + 4r][l & 15].
typedef double d4 __attribute__((ext_vector_type(4)));
#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)
// TB: the row-part B operands of the last TB steps kept in LDS (8 TB doubles per
// lane, 4 TB KiB per wave, read back per step as 4 x 16 B) instead of registers
template <int PD, bool RAG = false, int TB = 0>
__global__ __launch_bounds__(256, 2) void k_sym_mfma16(const SymStrip* __restrict__ strips,
                                                     const SymItem* __restrict__ sitems,
                                                     const double* __restrict__ pk, int ncol,
                                                     double* __restrict__ rowpart,
                                                     double* __restrict__ colpart,
                                                     const int* __restrict__ run) {
  constexpr int LDP = MF_LDP;
  constexpr int MF_WC = MF_CW / 4; // columns per wave
  constexpr int MF_NT = MF_WC / 32;
  __shared__ double red[2][4][256];
  __shared__ __attribute__((aligned(16))) double stg[4][16 * LDP];
  constexpr bool BL = TB > 0;
  __shared__ __attribute__((aligned(16))) double bls[BL ? 4 : 1][BL ? TB * 4 : 1][WAVE][2];
  const SymStrip sp = strips[blockIdx.x];
  if (run && !ldg(run)) return;   // no-op pass (pipelined CG past its stop test)
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int lo = lane & 15, hi = lane >> 4;
  SymItem cur = sitems[sp.it0];
  const int c0 = cur.c0, ncc = sp.ncmax;
  const double* pkb = pk + (int64_t)cur.voff * 16;    // Pk of this block (block-relative index)
  const int cw0 = wid * MF_WC;                         // first chunk column of this wave
  const bool dhalf = cw0 < SYM_H;
  const int nta = min(MF_NT, max(0, (ncc - cw0 + 31) / 32));   // as k_sym_mfma

  double* sb = stg[wid];
  // row-part B operands (P at this wave's columns), reused by every row group
  double brow[MF_NT - TB][4][2];
#pragma unroll
  for (int t = 0; t < MF_NT; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int col = cw0 + 32 * t + 8 * s + 2 * hi + e;
        const double v = ldg(pkb + (int64_t)(c0 + (col < ncc ? col : 0)) * 16 + lo);
        if (t < MF_NT - TB) brow[t < MF_NT - TB ? t : 0][s][e] = col < ncc ? v : 0.0;
        else if constexpr (BL) bls[wid][(t - (MF_NT - TB)) * 4 + s][lane][e] = col < ncc ? v : 0.0;
      }
  d4 dcol[MF_NT][2];
#pragma unroll
  for (int t = 0; t < MF_NT; ++t) dcol[t][0] = dcol[t][1] = d4{0.0, 0.0, 0.0, 0.0};

  auto load_cf = [&](uint64_t b0, int64_t ws, int H, int nci, int g, int t, d2* cf) {
    asm volatile("" : "+s"(b0));
    const int xc = cw0 + 32 * t + 2 * lo;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int rB = 16 * g + 4 * a + hi;
      const double* row = (const double*)b0 + (int64_t)(rB < H ? rB : H - 1) * ws;
      cf[a] = ldg_nt((const d2*)(row + (xc < (RAG ? nci : ncc) ? xc : 0)));
    }
  };
  auto band_zero = [&](int nci, int t, d2* cf) {   // as k_sym_mfma
    const int xc = cw0 + 32 * t + 2 * lo;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      cf[a].x = xc < nci ? cf[a].x : 0.0;
      cf[a].y = xc + 1 < nci ? cf[a].y : 0.0;
    }
  };
  auto load_bcol = [&](int r0, int H, bool zero, int g, double* bc) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int rB = 16 * g + 4 * a + hi;
      const double v = ldg(pkb + (int64_t)(r0 + (rB < H ? rB : 0)) * 16 + lo);
      bc[a] = (rB < H && !zero) ? v : 0.0;
    }
  };
  auto pbase = [&](const SymItem& x) { return (uint64_t)(x.P + (x.c0 - x.r0)); };

  static_assert(PD >= 1 && PD <= MF_NT && MF_NT % PD == 0, "prefetch depth divides the steps");
  uint64_t curb = pbase(cur);
  d2 cfq[PD][4];                                       // ring of PD steps in flight per wave
  double bcn[4];
#pragma unroll
  for (int p = 0; p < PD; ++p) load_cf(curb, cur.w, cur.H, cur.nc, 0, p, cfq[p]);
  load_bcol(cur.r0, cur.H, dhalf && cur.r0 == c0, 0, bcn);

  int gg = 0;
#pragma unroll 1
  for (int s = 0; s < sp.npan; ++s) {
    const bool more = s + 1 < sp.npan;
    const SymItem nx = sitems[sp.it0 + (more ? s + 1 : s)];
    const uint64_t nxb = more ? pbase(nx) : (uint64_t)pkb;
    const int ng = (cur.H + 15) / 16;
#pragma unroll 1
    for (int g = 0; g < ng; ++g, ++gg) {
      const bool same = g + 1 < ng;
      const uint64_t gb = same ? curb : nxb;
      const int64_t gw = same ? cur.w : (more ? nx.w : 0);
      const int gH = same ? cur.H : (more ? nx.H : 1);
      const int gn = same ? g + 1 : 0;
      const int gnc = same ? cur.nc : nx.nc;
      const int gr0 = same ? cur.r0 : nx.r0;
      const bool gz = dhalf && gr0 == c0;
      double bcol[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) bcol[a] = bcn[a];
      d4 drow0 = d4{0.0, 0.0, 0.0, 0.0}, drow1 = drow0;
      const bool colz = dhalf && cur.r0 == c0;
#pragma unroll
      for (int t = 0; t < MF_NT; ++t) {
        d2 cf[4], rf[4];
        const int slot = t % PD;                       // compile-time after unrolling
#pragma unroll
        for (int a = 0; a < 4; ++a) cf[a] = cfq[slot][a];
        // step + PD goes out here, ahead of this step's LDS and MFMA work
        if (t + PD < MF_NT) {
          load_cf(curb, cur.w, cur.H, cur.nc, g, t + PD, cfq[slot]);
        } else {
          load_cf(gb, gw, gH, gnc, gn, t + PD - MF_NT, cfq[slot]);
          if (t + PD == MF_NT) load_bcol(gr0, gH, gz, gn, bcn);
        }
        if (t >= nta) continue;
        if (RAG && cw0 + 32 * t >= cur.nc) continue;   // as k_sym_mfma
        if (RAG && cur.nc < ncc) band_zero(cur.nc, t, cf);
        lds_order();                                   // previous step's tile reads done
#pragma unroll
        for (int a = 0; a < 4; ++a) *(d2*)(sb + (4 * a + hi) * LDP + 2 * lo) = cf[a];
        lds_order();                                   // tile written
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) rf[s2] = *(const d2*)(sb + lo * LDP + 8 * s2 + 2 * hi);
        d2 bt[4];   // this step's row-part B operands
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          if (t < MF_NT - TB) bt[s2] = d2{brow[t < MF_NT - TB ? t : 0][s2][0], brow[t < MF_NT - TB ? t : 0][s2][1]};
          else if constexpr (BL) bt[s2] = *(const d2*)&bls[wid][(t - (MF_NT - TB)) * 4 + s2][lane][0];
        }
        if (!colz) {
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            dcol[t][0] = MFMA16(cf[a].x, bcol[a], dcol[t][0]);
            dcol[t][1] = MFMA16(cf[a].y, bcol[a], dcol[t][1]);
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          drow0 = MFMA16(rf[s2].x, bt[s2].x, drow0);
          drow1 = MFMA16(rf[s2].y, bt[s2].y, drow1);
        }
      }
      // row sums of this 16-row group: waves 0..3 in order
      double* rb = red[gg & 1][wid];
#pragma unroll
      for (int r = 0; r < 4; ++r) rb[((hi + 4 * r) << 4) + lo] = drow0[r] + drow1[r];
      __syncthreads();
      {
        const int t = threadIdx.x, row = t >> 4, cc = t & 15;
        const double v = ((red[gg & 1][0][t] + red[gg & 1][1][t]) + red[gg & 1][2][t]) +
                         red[gg & 1][3][t];
        if (16 * g + row < cur.H && cc < ncol)
          rowpart[((int64_t)cur.item * SYM_H + 16 * g + row) * ncol + cc] = v;
      }
    }
    cur = nx;
    curb = nxb;
  }

  // column sums over the strip's panels (whole slot, 16-B stores)
  if (lo < ncol) {
    double* out = colpart + ((int64_t)sp.slot * ncol + lo) * MF_CW;
#pragma unroll
    for (int t = 0; t < MF_NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *(d2*)(out + cw0 + 32 * t + 2 * (hi + 4 * r)) = d2{dcol[t][0][r], dcol[t][1][r]};
  }
}

// one workgroup per panel, FIN_Q threads per row (row t = r0 + (thread & 255),
// part q = thread >> 8): part q sums the panel's row parts item_begin + q, + 2q,
// ..., then the strips own_sb + q, ... of the own-parity chunk (column offset
// t) and oth_sb + q, ... of the other-parity chunk (offset 256 + t); parts are
// added in order (fin_epilogue) -- fixed order throughout
template <int NC>
__global__ __launch_bounds__(256 * FIN_Q) void k_sym_finalize_strip(
    const SymPanel* __restrict__ panels, PassArgs pa, const double* __restrict__ rowpart,
    const double* __restrict__ colpart, double* __restrict__ partials) {
  const SymPanel pn = panels[blockIdx.x];
  if (pa.run && !ldg(pa.run)) return;
  FinPre<NC> pre;
  fin_prefetch<NC>(pn, pa, pre);
  const int t = threadIdx.x & 255, q = threadIdx.x >> 8;
  const int tr = t < pn.H ? t : 0;
  double y[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) y[c] = 0.0;
#pragma unroll 4
  for (int itm = pn.item_begin + q; itm < pn.item_end; itm += FIN_Q) {
    const double* rp = rowpart + ((int64_t)itm * SYM_H + t) * NC;
#pragma unroll
    for (int c = 0; c < NC; ++c) y[c] += ldg(rp + c);
  }
#pragma unroll 4
  for (int sl = pn.own_sb + q; sl < pn.own_se; sl += FIN_Q) {
    const double* cp = colpart + (int64_t)sl * NC * MF_CW + tr;
#pragma unroll
    for (int c = 0; c < NC; ++c) y[c] += ldg(cp + c * MF_CW);
  }
#pragma unroll 4
  for (int sl = pn.oth_sb + q; sl < pn.oth_se; sl += FIN_Q) {
    const double* cp = colpart + (int64_t)sl * NC * MF_CW + SYM_H + tr;
#pragma unroll
    for (int c = 0; c < NC; ++c) y[c] += ldg(cp + c * MF_CW);
  }
  fin_epilogue<NC>(pn, pa, y, partials, pre);
}

// The same sums with one thread per panel row holding all FIN_Q parts in
// registers (part q: items item_begin + q, + FIN_Q, ..., then the own and other
// strips q, q + FIN_Q, ...; parts added in order 0..3, then the coupling sum,
// the epilogue and the panel's partial dots: wave butterfly over the same 64
// rows, waves in order) -- every addition of k_sym_finalize_strip in the same
// order, so bitwise the same outputs, in a 256-thread workgroup without the
// cross-part LDS exchange (a band panel has ~3 items and 2 strips: the
// 1024-thread form spends its time starting waves)
template <int NC>
__global__ __launch_bounds__(256) void k_sym_finalize_strip1(
    const SymPanel* __restrict__ panels, PassArgs pa, const double* __restrict__ rowpart,
    const double* __restrict__ colpart, double* __restrict__ partials) {
  const SymPanel pn = panels[blockIdx.x];
  if (pa.run && !ldg(pa.run)) return;
  const int t = threadIdx.x;
  const bool row = t < pn.H;
  const int tr = row ? t : 0;
  const int64_t idx = pn.voff + pn.r0 + tr;
  double in[NC], dt[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    in[c] = pa.in[c][idx];
    dt[c] = pa.dot[c] ? pa.dot[c][idx] : 0.0;
  }
  double y[FIN_Q][NC];
#pragma unroll
  for (int q = 0; q < FIN_Q; ++q)
#pragma unroll
    for (int c = 0; c < NC; ++c) y[q][c] = 0.0;
#pragma unroll
  for (int q = 0; q < FIN_Q; ++q) {
#pragma unroll 2
    for (int itm = pn.item_begin + q; itm < pn.item_end; itm += FIN_Q) {
      const double* rp = rowpart + ((int64_t)itm * SYM_H + t) * NC;
#pragma unroll
      for (int c = 0; c < NC; ++c) y[q][c] += ldg(rp + c);
    }
#pragma unroll 2
    for (int sl = pn.own_sb + q; sl < pn.own_se; sl += FIN_Q) {
      const double* cp = colpart + (int64_t)sl * NC * MF_CW + tr;
#pragma unroll
      for (int c = 0; c < NC; ++c) y[q][c] += ldg(cp + c * MF_CW);
    }
#pragma unroll 2
    for (int sl = pn.oth_sb + q; sl < pn.oth_se; sl += FIN_Q) {
      const double* cp = colpart + (int64_t)sl * NC * MF_CW + SYM_H + tr;
#pragma unroll
      for (int c = 0; c < NC; ++c) y[q][c] += ldg(cp + c * MF_CW);
    }
  }
  __shared__ double s_w[4][NC];
  const int lane = t & (WAVE - 1), wid = t / WAVE;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    double v = y[0][c];
#pragma unroll
    for (int p = 1; p < FIN_Q; ++p) v += y[p][c];
    if (pn.cp >= 0) v += pa.cpbuf[((int64_t)pn.cp * 256 + t) * NC + c];   // coupled pieces
    double acc = 0.0;
    if (row) {
      const double o = pa.c1[c] * v + pa.c2[c] * in[c];
      pa.out[c][idx] = o;
      if (pa.yout[c]) pa.yout[c][idx] = pa.ys1 * v + pa.ys0 * in[c];
      if (pa.dot[c]) acc = dt[c] * o;
    }
    const double sm = wave_sum(acc);
    if (lane == 0) s_w[wid][c] = sm;
  }
  __syncthreads();
  if (t < NC) partials[(int64_t)pn.part * NC + t] = ((s_w[0][t] + s_w[1][t]) + s_w[2][t]) + s_w[3][t];
}

// Pk[i][c] = in[c][i] for c < ncol, 0 for ncol <= c < PKS (i over the padded
// vector).  PKS = the columns the pass kernel's groups read: 4 (NC <= 4), 8
// (NC <= 8), 16 -- a row is one cache line's worth of what is read, so the
// pass's Pk reads (L2 misses on M = 1e6) carry no unused columns
// PAIRED (PKS = 8, the 5-8-column band walks): slot p holds column
// 4 (p & 1) + (p >> 1), so the walk's lane n4 reads its columns n4 and 4 + n4
// as one 16-B load
// One thread per row: the column reads are coalesced over the threads, the
// row is written as 16-B stores.
template <int PKS, bool PAIRED = false>
__global__ __launch_bounds__(256) void k_pack(PassArgs pa, int ncol, int64_t mpad,
                                              double* __restrict__ pk) {
  if (pa.run && !ldg(pa.run)) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= mpad) return;
  double v[PKS];
#pragma unroll
  for (int p = 0; p < PKS; ++p) {
    const int c = PAIRED ? 4 * (p & 1) + (p >> 1) : p;
    v[p] = c < ncol ? pa.in[c][i] : 0.0;
  }
  d2* row = (d2*)(pk + i * PKS);
#pragma unroll
  for (int p = 0; p < PKS; p += 2) row[p / 2] = d2{v[p], v[p + 1]};
}

// ragged: some strip item stops short of its strip's widest (band blocks):
// the RAG kernels, without the deferred row MFMAs (even there,
// profiles/r04/band2_ab.jsonl).  pair: the plan's choice of the wave-pair
// kernel (ldplan.hip mfma_pair_choice; bitwise the same products) -- 1: by the
// launch-tail model (a short launch: the 8-block share of the north star), 2
// (forced, SGV_MF_PAIR=1): every launch.  Since the column operands are loaded
// once per row group the model's choice holds at 5-8 columns too: the 8-block
// share -2...-8 %, 4 x 25,000 -2.6 % per 8-column pass; launches it does not
// pick run +1.4...+9 % with the pair form (profiles/r06/pair58_*.jsonl)
template <int NG, bool PP = false>
static void launch_mf(const SymStrip* d_strips, int nstrips, const SymItem* d_sitems,
                      const double* d_pk, int nc, double* rowpart, double* colpart,
                      const int* run, int pks, bool ragged, int pair, hipStream_t st) {
  // prefetch depth 2 measured best (PD 1/2/4: 11.64/11.16/12.27 ms at NC=4, M=1e6)
  if (ragged)
    hipLaunchKernelGGL((k_sym_mfma<NG, 2, true, false, PP>), dim3(nstrips), dim3(256), 0, st,
                       d_strips, d_sitems, d_pk, nc, rowpart, colpart, run, pks);
  else if (pair >= 1)
    hipLaunchKernelGGL((k_sym_mfma_pair<NG, 2, PP>), dim3(nstrips), dim3(512), 0, st, d_strips,
                       d_sitems, d_pk, nc, rowpart, colpart, run, pks);
  else
    hipLaunchKernelGGL((k_sym_mfma<NG, 2, false, true, PP>), dim3(nstrips), dim3(256), 0, st,
                       d_strips, d_sitems, d_pk, nc, rowpart, colpart, run, pks);
}

// 5-8-column strip passes read Pk PAIRED (k_pack), in either strip kernel.
// Bitwise the same products; one box,
// alternating: the 8-block share -0.6...-1.8 % per pass, 64 blocks even to
// -0.4 % (profiles/r06/pkpair_ab.jsonl, pkpair_bench.jsonl)
bool strip_pk_paired(int nc) { return nc > 4 && nc <= 8; }

hipError_t launch_pk(const PassArgs& pa, int nc, int64_t mpad, double* d_pk, hipStream_t st,
                     bool paired) {
  if (nc < 1 || nc > 16) return hipErrorInvalidValue;
  const int pks = nc > 8 ? 16 : nc <= 4 ? 4 : 8;
  const dim3 pg((unsigned)((mpad + 255) / 256));
  if (pks == 4)
    hipLaunchKernelGGL(k_pack<4>, pg, dim3(256), 0, st, pa, nc, mpad, d_pk);
  else if (pks == 8 && paired)
    hipLaunchKernelGGL((k_pack<8, true>), pg, dim3(256), 0, st, pa, nc, mpad, d_pk);
  else if (pks == 8)
    hipLaunchKernelGGL(k_pack<8>, pg, dim3(256), 0, st, pa, nc, mpad, d_pk);
  else
    hipLaunchKernelGGL(k_pack<16>, pg, dim3(256), 0, st, pa, nc, mpad, d_pk);
  return hipGetLastError();
}

hipError_t launch_sym_mfma(int nc, const SymStrip* d_strips, int nstrips, const SymItem* d_sitems,
                           const PassArgs& pa, const double* d_pk, double* rowpart,
                           double* colpart, bool ragged, int pair, hipStream_t st) {
  if (nc < 1 || nc > 16) return hipErrorInvalidValue;
  if (nstrips <= 0) return hipSuccess;
  const int pks = nc > 8 ? 16 : nc <= 4 ? 4 : 8;
  // 9..16 columns: one 16x16x4 group beats three/four 4x4x4 groups (register
  // pressure) and two 8-column wave sets of the 4x4x4 kernel in one 8-wave
  // workgroup re-reading the same R with the default cache policy (+33 %,
  // profiles/r03/s4/mf_sets_ab.jsonl) and three / four 4x4x4 groups at one wave
  // per SIMD with the deferred row MFMAs (+13 % / +28 %, ng4_ab.jsonl):
  // measured in DESIGN.md.  Prefetch depth 2 (with every row operand in
  // registers it spilled 3 / 7 VGPRs on dense / band plans and was still faster
  // than depth 1: profiles/r03/s4/mf16_pd_ab.jsonl, profiles/r04/band2_ab.jsonl).
  // Round 6 measured the spill-free forms on one
  // box (profiles/r06/mf16_forms_ab.jsonl, _bench_c5conv.jsonl): depth 1 (236
  // VGPRs) +1.5-2 % per pass, 8 waves of 64 columns per workgroup (188 VGPRs)
  // +8 %, and the row part on 4x4x4 MFMA in that form (210 VGPRs) +18 % -- the
  // 8-wave row-sum combine and the 4x4x4 form's DPP reductions and 4x the MFMA
  // issues cost more than they save; the spill-free form kept is the row
  // operands of the last step(s) in LDS (below).
  switch ((nc + 3) / 4) {
    case 1: launch_mf<1>(d_strips, nstrips, d_sitems, d_pk, nc, rowpart, colpart, pa.run, pks, ragged, pair, st); break;
    case 2:   // Pk paired (strip_pk_paired)
      launch_mf<2, true>(d_strips, nstrips, d_sitems, d_pk, nc, rowpart, colpart, pa.run, pks,
                         ragged, pair, st);
      break;
    default:
      // the row operands of the last steps in LDS, so nothing spills (256 VGPRs
      // with 3 / 7 spilled before): band plans the last 2 steps (-0.6 % per
      // 16-column band pass), dense plans the last one (even; 2 steps there +2 %)
      // -- profiles/r06/mf16_bl_*.jsonl, mf16_tb_*.jsonl; products bitwise equal
      if (ragged)
        hipLaunchKernelGGL((k_sym_mfma16<2, true, 2>), dim3(nstrips), dim3(256), 0, st, d_strips,
                           d_sitems, d_pk, nc, rowpart, colpart, pa.run);
      else
        hipLaunchKernelGGL((k_sym_mfma16<2, false, 1>), dim3(nstrips), dim3(256), 0, st, d_strips,
                           d_sitems, d_pk, nc, rowpart, colpart, pa.run);
      break;
  }
  return hipGetLastError();
}

#ifdef SGV_MF_TRACE
extern "C" int sgv_diag_mf_trace(unsigned long long* out, int n) {
  if (n > MF_TRACE_MAX) n = MF_TRACE_MAX;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mf_trace), sizeof(unsigned long long) * 3 * n) ==
                 hipSuccess ? n : -1;
}
#endif

// SGV_FIN_FORM (A/B, with SGV_AB=1): the strip finalize's form -- 4 = FIN_Q
// threads per panel row (k_sym_finalize_strip), 1 = one thread per row with the
// parts in registers (k_sym_finalize_strip1; bitwise the same outputs);
// default: 1 for band plans at up to 8 columns (M = 1e6, bw = 1,000: 2.126-2.134
// vs 2.156 ms per pass), 4 otherwise (dense 64 x 15,625 at 8 columns: 12.13 vs
// 11.97-12.01 ms; 16 columns even; profiles/r04/fin_*.jsonl)
static int fin_form(bool ragged, int nc) {
  const char* e = ab_env("SGV_FIN_FORM");   // per launch (a getenv): tests switch it
  const int v = (e && (e[0] == '1' || e[0] == '4')) ? e[0] - '0' : 0;
  return v ? v : (ragged && nc <= 8) ? 1 : 4;
}

hipError_t launch_sym_finalize_strip(int nc, const SymPanel* d_panels, int npanels,
                                     const PassArgs& pa, const double* rowpart,
                                     const double* colpart, double* partials, bool ragged,
                                     hipStream_t st) {
  // the partials with the default cache policy: nontemporal loads measured
  // 0.5-3 % slower (profiles/r03/s4/fin_nt_ab.jsonl; they were just written)
  if (npanels <= 0) return hipSuccess;   // a block group without packed panels
  const bool one = fin_form(ragged, nc) == 1;
#define FIN_CASE(N)                                                                        \
  case N:                                                                                  \
    if (one)                                                                               \
      hipLaunchKernelGGL(k_sym_finalize_strip1<N>, dim3(npanels), dim3(256), 0, st, d_panels, \
                         pa, rowpart, colpart, partials);                                  \
    else                                                                                   \
      hipLaunchKernelGGL(k_sym_finalize_strip<N>, dim3(npanels), dim3(256 * FIN_Q), 0, st, \
                         d_panels, pa, rowpart, colpart, partials);                        \
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
