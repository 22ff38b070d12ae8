// Packed band LD pass on the f64 matrix cores: workgroups WALK DOWN the band.
//
// A band block (windowed LD: src/main.py:199-200 .npz CSR, :251-257 PLINK .ld)
// is stored as panels of 256 rows, panel g holding columns [256 g, 256 g + E)
// (E = the band's stored extent, R = E / 256 column ranges).  The strip kernel
// (sym_mfma.hip) cuts it into 512-column chunks over the panels of one parity,
// which in a band meet only ~3 panels: per stored byte it writes and re-reads
// 2.7x the row and column partials of a dense plan, and a finalize launch adds
// them up (PMC: 1.097x the stored bytes at M = 1e6, bw = 1,000).
//
// Here one workgroup owns a WALK: W consecutive panels of one block, the whole
// stored width of each.  Panel g's rows are complete after its own items (row
// part) and the column parts of panels g - R + 1 .. g - 1 (the transposes of
// their stored elements right of their diagonal blocks) -- all inside the walk
// but for its first R - 1 panels.  So the walk keeps an LDS ring of R panel
// accumulators acc[256][NC]: panel g's items add their row sums into slot g mod
// R and their column sums into the slots of panels g + 1 .. g + R - 1; when
// panel g is done, its slot is complete and the fused epilogue writes out =
// c1 y + c2 in, R_s in, and the panel's partial dots -- no partial buffers, no
// finalize.  Only the walk's first R - 1 panels ("head" panels, unless the walk
// starts the block) lack the previous walk's column parts: they leave their
// partial sums in headbuf, the previous walk leaves its open slots in carrybuf,
// and k_walk_fin adds the two (then the coupling sums) and runs the epilogue.
// The walk partition is a function of the block alone (ldplan.hip plan_walks),
// so the summation order -- and every product -- is the same on 1 and N ranks.
//
// 8 waves per workgroup (one per CU: the ring takes R x 16 KiB of LDS), each
// wave 64 columns of a 512-column item, sweeping its 16-row groups as the strip
// kernel does (16 x 32 sub-tiles loaded once, 16 B per lane, nontemporal; the
// row fragment through a per-wave XOR-swizzled LDS tile; v_mfma_f64_4x4x4f64).
// Per row group the eight waves' row sums are added in wave order into the
// panel's slot by one of them (wave gg mod 8), synchronised through LDS
// counters instead of a barrier: a ring of WK_RD hand-off buffers lets a wave
// run up to WK_RD - 1 row groups ahead of the slowest (bounded waits: every
// wait is on a write or a combine another wave reaches without waiting on
// this one).  One barrier per panel (its epilogue).
//
// The loop's addressing is what set its speed (profiles/r05/walk_ab/): the
// first forms spent ~190 VALU per 4-KiB sub-tile (1.9x the strips), most of
// it 64-bit address arithmetic and clamps for the P operands, and re-read the
// row operands every row group.  Now the P operands of a walk come from one
// base with 32-bit offsets (16-B paired loads at 5-8 columns, k_pack's PAIRED
// layout), and the row operands are read only in an item's last row group
// (the others read one cached row): 1.68 / 1.71 / 1.99 ms at 3 / 4 / 8
// columns against 1.82 / 1.85 / 2.23 before (M = 1e6, bw = 1,000).  Buffer
// loads (of the R fragments or of the P operands) were 4-13 % slower.
//
// Summation order of row i of panel g (fixed): the column parts of panels
// g - R + 1, ..., g - 1 in panel order (in a head panel: those inside the walk,
// then the carry of the earlier ones as one term), then the row parts of the
// panel's items in item order (per item: the eight waves in order), then the
// coupling sum of a cut between band pieces.
#include "common.h"

namespace sgv {

#define MFMA4W(a, b, c) __builtin_amdgcn_mfma_f64_4x4x4f64((a), (b), (c), 0, 0, 0)

constexpr int WK_NW = 8;          // waves per workgroup
constexpr int WK_WC = 64;         // columns per wave of a 512-column item
constexpr int WK_NT = WK_WC / 32; // 32-column steps per wave
constexpr int WK_RD = 4;          // row-sum hand-off buffers (row groups in flight)

__device__ __forceinline__ void wk_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// A workgroup barrier over LDS only: the wave's DS operations complete
// (lgkmcnt(0)), then s_barrier -- without the vmcnt(0) of __syncthreads, which
// would drain the prefetched HBM fragments at every barrier.  The wavefront-
// scope fences only keep the compiler from moving LDS accesses across it.
__device__ __forceinline__ void wk_lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);   // gfx9 encoding: lgkmcnt(0), vmcnt / expcnt at max
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the fused epilogue of one panel (the walk's, or k_walk_fin's for a head
// panel): y = acc (+ the coupling sum), out = c1 y + c2 in, R_s in, and the
// panel's partial dots -- the 64-row wave butterflies added in row-quarter
// order.  `nthr` threads: thread t takes row t & 255 and, with 512 threads,
// half (t >> 8) of the columns; every load of a thread is issued before its
// first store.
template <int RW, int NH>
__device__ __forceinline__ void walk_epilogue(const SymPanel& pn, const PassArgs& pa, int ncol,
                                              const double* __restrict__ yrow, double* s_w) {
  constexpr int CPT = RW / NH;   // columns per thread
  const int t = threadIdx.x & 255, h = threadIdx.x >> 8;
  const int lane = threadIdx.x & (WAVE - 1), q4 = t / WAVE;
  const bool live = t < pn.H;
  const int64_t idx = pn.voff + pn.r0 + (live ? t : 0);
  double y[CPT], in[CPT], dt[CPT], cp[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = h * CPT + j;
    y[j] = yrow[j];
    in[j] = dt[j] = cp[j] = 0.0;
    if (c < ncol) {
      in[j] = pa.in[c][idx];
      if (pa.dot[c]) dt[j] = pa.dot[c][idx];
      if (pn.cp >= 0) cp[j] = pa.cpbuf[((int64_t)pn.cp * 256 + t) * ncol + c];   // coupled pieces
    }
  }
  double a[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = h * CPT + j;
    a[j] = 0.0;
    if (c < ncol) {
      double v = y[j];
      if (pn.cp >= 0) v += cp[j];
      if (live) {
        const double o = pa.c1[c] * v + pa.c2[c] * in[j];
        pa.out[c][idx] = o;
        if (pa.yout[c]) pa.yout[c][idx] = pa.ys1 * v + pa.ys0 * in[j];
        if (pa.dot[c]) a[j] = dt[j] * o;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = h * CPT + j;
    const double sm = wave_sum(a[j]);
    if (lane == 0 && c < ncol) s_w[q4 * RW + c] = sm;
  }
}

template <int NG>
__global__ __launch_bounds__(WK_NW * 64, 1) void k_band_walk(
    const SymWalk* __restrict__ walks, const SymPanel* __restrict__ panels,
    const SymItem* __restrict__ items, const double* __restrict__ pk, int pks, int64_t pk_rows,
    PassArgs pa, int ncol, double* __restrict__ headbuf, double* __restrict__ carrybuf,
    double* __restrict__ partials) {
  constexpr int RW = 4 * NG;                                   // accumulator row stride
  constexpr int CPT = RW / 2;                                  // epilogue columns per thread
  // column-part P operands de-replicated over the MFMA blocks (as the strips):
  // at 5-8 columns -2.8 % per pass; at 3-4 columns (8-B operands) +1.5 %, so
  // not there (M = 1e6, bw = 1,000, one box: profiles/r06/walk_sw_ab.txt)
  constexpr bool SWZ = NG == 2;
  __shared__ __attribute__((aligned(16))) double ring[WALK_RMAX][SYM_H * RW];
  __shared__ __attribute__((aligned(16))) double red[WK_RD][WK_NW][16 * RW];
  __shared__ int hready[WK_RD], hdone[WK_RD];   // writes into / combines of each buffer
  __shared__ __attribute__((aligned(16))) double stg[WK_NW][16 * 32];
  __shared__ double s_w[4 * RW];
  const SymWalk wk = walks[blockIdx.x];
  if (pa.run && !ldg(pa.run)) return;   // no-op pass (pipelined CG past its stop test)
  const int R = wk.R;
  const int lane = threadIdx.x & (WAVE - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int lo = lane & 15, hi = lane >> 4, bq = (lane >> 2) & 3, n4 = lane & 3;
  const int pc = hi + 4 * bq;                                  // column pair in a fragment
  double* sb = stg[wid];
  for (int e = threadIdx.x; e < R * SYM_H * RW; e += WK_NW * 64) (&ring[0][0])[e] = 0.0;
  if (threadIdx.x < WK_RD) hready[threadIdx.x] = hdone[threadIdx.x] = 0;
  __syncthreads();
  auto lds_wait_ge = [](int* ctr, int v) {
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v)
      __builtin_amdgcn_s_sleep(1);
  };

  // an item of the walk as this wave sees it
  struct Cur {
    const double* b0;   // element (r0, c0)
    int w;              // row stride
    int nc, c0, r0, H;
    bool colz;          // this wave's columns lie in the diagonal block
  };
  auto make = [&](const SymItem& it, const SymPanel& p) {
    Cur u;
    const int crel = it.c0 - it.r0;
    u.b0 = it.P + crel;
    u.w = (int)it.w;
    u.nc = it.nc;
    u.c0 = it.c0;
    u.r0 = p.r0;
    u.H = p.H;
    u.colz = crel + WK_WC * wid < SYM_H;
    return u;
  };
  // fragments of row group g2, step t (16 B per lane, nontemporal; rows past
  // H clamp -- their P is 0 -- and columns past the item load column 0)
  auto load_cf = [&](const Cur& u, int g2, int t, d2* cf) {
    const int xc = WK_WC * wid + 32 * t + 2 * lo;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int rB = 16 * g2 + 4 * (SWZ ? a ^ (bq & 2) : a) + hi;   // SWZ: the strips' row sets
      cf[a] = ldg_nt((const d2*)(u.b0 + (rB < u.H ? rB : u.H - 1) * u.w + (xc < u.nc ? xc : 0)));
    }
  };
  // P operands: one base per walk (its block's Pk rows; the panels of a walk
  // are one block's) and 32-bit byte offsets clamped to the Pk vector -- rows
  // or columns past the item read whatever lies there and are masked where
  // they are used (a select right behind its load would make the compiler
  // wait for each load in turn).  Pk row layout (k_pack): NG = 1 columns
  // 0..3; NG = 2 PAIRED, column 4 q + n4 at 2 n4 + q, so a lane's two groups
  // are one 16-B load
  const int64_t pvoff = panels[wk.p0].voff;
  const char* pbase = (const char*)(pk + pvoff * pks);
  const int p_rng = (int)min<int64_t>((pk_rows - pvoff) * pks * 8, 0x7FFF0000);
  const int pbyte = 8 * pks;                                   // one Pk row
  auto ld_p = [&](int off, double* v) {
    const char* pb = pbase + min(off, p_rng - pbyte);   // the last row is read whole
    if constexpr (NG == 2) {
      const d2 x = ldg((const d2*)(pb + 16 * n4));
      v[0] = x.x;
      v[1] = x.y;
    } else {
#pragma unroll
      for (int q = 0; q < NG; ++q) v[q] = ldg((const double*)(pb + 8 * (4 * q + n4)));
    }
  };
  // the masks: bit a (bcol: row valid, not the diagonal block; SWZ: bit 0 for
  // this lane's row set bq, handed to the fragments by swz_quad -- one load per
  // row group), bit 2 t + e (brow: column inside the item)
  auto load_bcol = [&](const Cur& u, int g2, double (*bc)[NG]) {
    int m = 0;
#pragma unroll
    for (int a = 0; a < (SWZ ? 1 : 4); ++a) {
      const int rB = 16 * g2 + 4 * (SWZ ? bq : a) + hi;
      m |= (rB < u.H && !u.colz) ? 1 << a : 0;
      ld_p((u.r0 + rB) * pbyte, bc[a]);
    }
    return m;
  };
  // live = false (not the item's last row group: the next item's row operands
  // are not due yet) reads the range's last row instead -- the
  // same loads on every path, L2 hits.  The offset is chosen by a scalar select
  // (a vector select's temporary landed in a register a load was still
  // filling: a wait for it)
  auto load_brow = [&](const Cur& u, bool live, double (*br)[2][NG]) {
    int m = 0;
    int so;
    asm volatile("s_cmp_lg_u32 %1, 0\n\ts_cselect_b32 %0, %2, %3"
                 : "=s"(so)
                 : "s"(__builtin_amdgcn_readfirstlane((int)live)),
                   "s"(__builtin_amdgcn_readfirstlane(u.c0 * pbyte)),
                   "s"(__builtin_amdgcn_readfirstlane(p_rng))
                 : "scc");
#pragma unroll
    for (int t = 0; t < WK_NT; ++t)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int col = WK_WC * wid + 32 * t + 2 * pc + e;     // item-relative
        m |= col < u.nc ? 1 << (2 * t + e) : 0;
        ld_p(so + col * pbyte, br[t][e]);
      }
    return m;
  };

  // the walk's first item: its first row group and P operands in flight
  SymPanel pn = panels[wk.p0];
  Cur cu = make(items[pn.item_begin], pn);
  d2 cfn[WK_NT][4];
  double bcn[SWZ ? 1 : 4][NG], brn[WK_NT][2][NG];
#pragma unroll
  for (int t = 0; t < WK_NT; ++t) load_cf(cu, 0, t, cfn[t]);
  int bcm = load_bcol(cu, 0, bcn);
  int brm = load_brow(cu, true, brn);

  int gg = 0;                                                  // row groups done
#pragma unroll 1
  for (int s = 0; s < wk.np; ++s) {
    const int g = pn.g;
    double* acc = ring[g % R];
    const int ng = (pn.H + 15) / 16;
    const bool more_panels = s + 1 < wk.np;
    const SymPanel pnx = panels[wk.p0 + (more_panels ? s + 1 : s)];
#pragma unroll 1
    for (int itx = pn.item_begin; itx < pn.item_end; ++itx) {
      // the next item of the walk (this panel's, or the next panel's first)
      const bool nx_here = itx + 1 < pn.item_end;
      const bool has_nx = nx_here || more_panels;
      const Cur cn = has_nx ? make(items[nx_here ? itx + 1 : pnx.item_begin], nx_here ? pn : pnx) : cu;
      const int crel = cu.c0 - pn.r0;                          // item's first column (panel-relative)
      const int cw0 = crel + WK_WC * wid;                      // this wave's first column
      // 32-column steps holding stored columns; the diagonal block feeds the row sums only
      const int nta = min(WK_NT, max(0, (cu.nc - WK_WC * wid + 31) / 32));
      const bool colz = cu.colz;
      double brow[WK_NT][2][NG];
#pragma unroll
      for (int t = 0; t < WK_NT; ++t)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int q = 0; q < NG; ++q) brow[t][e][q] = (brm >> (2 * t + e) & 1) ? brn[t][e][q] : 0.0;
      double dcol[WK_NT][2][NG];
#pragma unroll
      for (int t = 0; t < WK_NT; ++t)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int q = 0; q < NG; ++q) dcol[t][e][q] = 0.0;
#pragma unroll 1
      for (int g2 = 0; g2 < ng; ++g2, ++gg) {
        double bcol[4][NG];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int q = 0; q < NG; ++q)
            bcol[a][q] = SWZ ? swz_quad(bcm ? bcn[0][q] : 0.0, a) : (bcm >> a & 1) ? bcn[SWZ ? 0 : a][q] : 0.0;
        // where the next row group's loads come from: this item's next, or the
        // next item's first (then also its row operands).  Branch-free, the same
        // loads on every path (a branch join with different load counts makes
        // the compiler drain every load in flight): the row operands are re-read
        // for the current item until its last row group (cache hits)
        const bool last = g2 + 1 >= ng;
        Cur src;
        src.b0 = last ? cn.b0 : cu.b0;
        src.w = last ? cn.w : cu.w;
        src.nc = last ? cn.nc : cu.nc;
        src.c0 = last ? cn.c0 : cu.c0;
        src.r0 = last ? cn.r0 : cu.r0;
        src.H = last ? cn.H : cu.H;
        src.colz = last ? cn.colz : cu.colz;
        const int gn = last ? 0 : g2 + 1;
        double drow[4][NG];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < NG; ++q) drow[r][q] = 0.0;
#pragma unroll
        for (int t = 0; t < WK_NT; ++t) {
          // a ring of one row group per wave: step t's fragments came in with
          // the previous row group's step t and are used in place; the same step
          // of the next row group goes into their registers right after, so two
          // steps of loads stay in flight (no copy: a loop-carried copy of
          // loaded registers makes the compiler wait for the loads at the back edge)
          d2* cf = cfn[t];
          if (t < nta) {                                       // wave-uniform: inside the item
            // a step partly past the item's stored end: those columns read as 0
            const int xc = WK_WC * wid + 32 * t + 2 * lo;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
              cf[a].x = xc < cu.nc ? cf[a].x : 0.0;
              cf[a].y = xc + 1 < cu.nc ? cf[a].y : 0.0;
            }
            d2 rf[4];
            wk_lds_order();
#pragma unroll
            for (int a = 0; a < 4; ++a)
              *(d2*)(sb + 32 * (4 * (SWZ ? a ^ (bq & 2) : a) + hi) + 2 * (lo ^ hi)) = cf[a];
            wk_lds_order();
#pragma unroll
            for (int r = 0; r < 4; ++r) rf[r] = *(const d2*)(sb + 32 * (4 * r + n4) + 2 * (pc ^ n4));
            __builtin_amdgcn_s_setprio(1);
            if (!colz) {
#pragma unroll
              for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int q = 0; q < NG; ++q) {
                  dcol[t][0][q] = MFMA4W(cf[a].x, bcol[a][q], dcol[t][0][q]);
                  dcol[t][1][q] = MFMA4W(cf[a].y, bcol[a][q], dcol[t][1][q]);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int q = 0; q < NG; ++q) drow[r][q] = MFMA4W(rf[r].x, brow[t][0][q], drow[r][q]);
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int q = 0; q < NG; ++q) drow[r][q] = MFMA4W(rf[r].y, brow[t][1][q], drow[r][q]);
            __builtin_amdgcn_s_setprio(0);
          }
          load_cf(src, gn, t, cfn[t]);
          if (t == 0) {
            bcm = load_bcol(src, gn, bcn);
            brm = load_brow(src, last, brn);
          }
        }
        // the row group's row sums: 4 blocks (DPP), handed to the combining wave
        const int hs = gg % WK_RD, gen = gg / WK_RD;
        lds_wait_ge(&hdone[hs], gen);                          // buffer hs free (gg - WK_RD combined)
        double* rb = red[hs][wid];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < NG; ++q) {
            double v = drow[r][q];
            v = v + row_ror<12>(v);
            v = v + row_ror<8>(v);
            if (bq == 0) rb[(4 * r + hi) * RW + 4 * q + n4] = v;   // D row 4r + m (m = hi)
          }
        // LDS executes a wave's DS operations in order, so the counter's add
        // lands after the row sums; the wavefront-scope fences keep the
        // compiler's order and wait for nothing (the fragments stay in flight)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (lane == 0)
          __hip_atomic_fetch_add(&hready[hs], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (wid == gg % WK_NW) {   // this wave combines row group gg: the 8 waves in order
          lds_wait_ge(&hready[hs], WK_NW * (gen + 1));
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
          for (int k = 0; k < (16 * RW + WAVE - 1) / WAVE; ++k) {
            const int e = lane + WAVE * k;
            if (e < 16 * RW) {
              const int row = e / RW, cc = e - row * RW;
              const double* rr = &red[hs][0][0] + e;
              double v = rr[0];
#pragma unroll
              for (int w = 1; w < WK_NW; ++w) v += rr[w * 16 * RW];
              acc[(16 * g2 + row) * RW + cc] += v;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          if (lane == 0)
            __hip_atomic_store(&hdone[hs], gen + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      // the item's column sums: this wave's columns of ranges g + 1 .. g + R - 1
      if (!colz) {
#pragma unroll
        for (int t = 0; t < WK_NT; ++t) {
          if (t >= nta) continue;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int col = cw0 + 32 * t + 2 * pc + e;         // panel-relative
            if (col - crel >= cu.nc) continue;
            double* dst = ring[(g + col / SYM_H) % R] + (col % SYM_H) * RW;
#pragma unroll
            for (int q = 0; q < NG; ++q) dst[4 * q + n4] += dcol[t][e][q];
          }
        }
      }
      cu = cn;
    }
    wk_lds_barrier();   // panel g's slot is complete (but for a head panel's carry)
    {
      const int t = threadIdx.x & 255, h = threadIdx.x >> 8;
      double* row = acc + t * RW + h * CPT;
      if (s < wk.nhead) {   // partial: k_walk_fin adds the previous walk's carry
        double* hb = headbuf + ((int64_t)(wk.hslot + s) * SYM_H + t) * ncol + h * CPT;
#pragma unroll
        for (int j = 0; j < CPT; ++j)
          if (h * CPT + j < ncol) hb[j] = row[j];
      } else {
        walk_epilogue<RW, 2>(pn, pa, ncol, row, s_w);
      }
#pragma unroll
      for (int j = 0; j < CPT; ++j) row[j] = 0.0;             // the slot's next panel: g + R
    }
    wk_lds_barrier();
    if (s >= wk.nhead && threadIdx.x < ncol) {
      const int c = threadIdx.x;
      partials[(int64_t)pn.part * ncol + c] =
          ((s_w[0 * RW + c] + s_w[1 * RW + c]) + s_w[2 * RW + c]) + s_w[3 * RW + c];
    }
    pn = pnx;
  }
  // the open slots: column parts of the next walk's head panels
  {
    const int t = threadIdx.x & 255, h = threadIdx.x >> 8;
    const int gend = panels[wk.p0 + wk.np - 1].g + 1;
    for (int j = 0; j < wk.ncarry; ++j) {
      const double* row = ring[(gend + j) % R] + t * RW + h * CPT;
      double* cb = carrybuf + ((int64_t)(wk.cslot + j) * SYM_H + t) * ncol + h * CPT;
#pragma unroll
      for (int i = 0; i < CPT; ++i)
        if (h * CPT + i < ncol) cb[i] = row[i];
    }
  }
}

// Head panels of the walks: y = the walk's partial + the previous walk's carry
// (+ the coupling sum), then the epilogue and the panel's partial dots -- as
// k_band_walk's own epilogue
template <int RW>
__global__ __launch_bounds__(256) void k_walk_fin(const WalkFin* __restrict__ fins,
                                                  const SymPanel* __restrict__ panels, PassArgs pa,
                                                  int ncol, const double* __restrict__ headbuf,
                                                  const double* __restrict__ carrybuf,
                                                  double* __restrict__ partials) {
  __shared__ double s_w[4 * RW];
  const WalkFin f = fins[blockIdx.x];
  if (pa.run && !ldg(pa.run)) return;
  const SymPanel pn = panels[f.panel];
  const int t = threadIdx.x;
  const double* hb = headbuf + ((int64_t)f.hslot * SYM_H + t) * ncol;
  const double* cb = carrybuf + ((int64_t)f.cslot * SYM_H + t) * ncol;
  double y[RW];
#pragma unroll
  for (int c = 0; c < RW; ++c) y[c] = c < ncol ? hb[c] + cb[c] : 0.0;
  walk_epilogue<RW, 1>(pn, pa, ncol, y, s_w);
  __syncthreads();
  if (t < ncol)
    partials[(int64_t)pn.part * ncol + t] =
        ((s_w[0 * RW + t] + s_w[1 * RW + t]) + s_w[2 * RW + t]) + s_w[3 * RW + t];
}

hipError_t launch_band_walk(int nc, const SymWalk* d_walks, int nwalks, const SymPanel* d_panels,
                            const SymItem* d_items, const double* d_pk, int64_t pk_rows,
                            const PassArgs& pa,
                            double* headbuf, double* carrybuf, const WalkFin* d_fins, int nfins,
                            double* partials, hipStream_t st) {
  if (nc < 1 || nc > 8) return hipErrorInvalidValue;
  const int pks = nc <= 4 ? 4 : 8;
  if (nwalks > 0) {
    if (nc <= 4)
      hipLaunchKernelGGL(k_band_walk<1>, dim3(nwalks), dim3(WK_NW * 64), 0, st, d_walks, d_panels,
                         d_items, d_pk, pks, pk_rows, pa, nc, headbuf, carrybuf, partials);
    else
      hipLaunchKernelGGL(k_band_walk<2>, dim3(nwalks), dim3(WK_NW * 64), 0, st, d_walks, d_panels,
                         d_items, d_pk, pks, pk_rows, pa, nc, headbuf, carrybuf, partials);
  }
  if (nfins > 0) {
    if (nc <= 4)
      hipLaunchKernelGGL(k_walk_fin<4>, dim3(nfins), dim3(256), 0, st, d_fins, d_panels, pa, nc,
                         headbuf, carrybuf, partials);
    else
      hipLaunchKernelGGL(k_walk_fin<8>, dim3(nfins), dim3(256), 0, st, d_fins, d_panels, pa, nc,
                         headbuf, carrybuf, partials);
  }
  return hipGetLastError();
}

}  // namespace sgv
