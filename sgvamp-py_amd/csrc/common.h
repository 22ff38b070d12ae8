// Internal declarations shared by the HIP translation units of libsgvamp_hip.so.
// Target: gfx950 (MI355X, CDNA4), wave64.  No other target is built.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sgv {

constexpr int WAVE = 64;
constexpr int VTHREADS = 256;   // threads per workgroup of the vector kernels
constexpr int CHUNK = 1024;     // markers per chunk (vector-kernel workgroup)
constexpr int PADV = 128;       // per-block padding of device vectors and LD rows (doubles = 1 KiB)
constexpr int MAXC = 16;        // right-hand-side columns per LD pass (2 x MAXKG cohorts)
constexpr int MAXK = 32;        // cohorts per launch of the marker kernels (more: cohort groups)
constexpr int MAXCOH = 1024;    // cohorts per context (SGV_MAX_COHORTS)
constexpr int MAXKG = 8;        // cohorts per LMMSE group (one batched CG loop, <= MAXC columns)
constexpr int MAXL = 8;         // slab components (L - 1)

typedef double d2 __attribute__((ext_vector_type(2)));

// Loads through the global address space.  Pointers read out of descriptor
// structs are generic to the compiler, which then emits FLAT loads: those
// count against lgkmcnt as well as vmcnt, so every wait for an LDS access
// also drains the in-flight HBM stream.  global_load keeps the counters apart.
#define SGV_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T ldg(const T* p) {
  return *(const SGV_GLOBAL T*)p;
}
template <class T>
__device__ __forceinline__ T ldg_nt(const T* p) {   // streaming (read-once) data
  return __builtin_nontemporal_load((const SGV_GLOBAL T*)p);
}

// The value lane (l + 16 - N) mod 16 of the caller's 16-lane row holds (DPP
// row_ror:N): a VALU move, no LDS round trip as __shfl_xor's ds_bpermute.
template <int N>
__device__ __forceinline__ double row_ror(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  // every row and bank enabled and row_ror reads inside the row: each lane is
  // written, so no "old" value (mov_dpp: no v_mov of a zero per half first)
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x120 + N, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x120 + N, 0xF, 0xF, true);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)hi << 32) |
                                                (unsigned)lo));
}

// the double of the lane of quad a ^ (bq & 2) in this lane's 16-lane row, bq =
// lane bits 2-3: lane id ((l & ~4) | 4 (a & 1)) ^ 8 (a >> 1) (ds_swizzle bit
// mask mode within 32 lanes: ((l & and) | or) ^ xor); a is a compile-time
// constant after unrolling (the strip kernels and the band walk
// take their column-part P operands this way: one load per row group)
template <int A>
__device__ __forceinline__ int swz_dw(int v) {
  return __builtin_amdgcn_ds_swizzle(v, 0x1B | ((A & 1) << 7) | ((A >> 1) << 13));
}
__device__ __forceinline__ double swz_quad(double v, int a) {
  const int2 w = __builtin_bit_cast(int2, v);
  int2 r;
  switch (a) {
    case 0: r.x = swz_dw<0>(w.x); r.y = swz_dw<0>(w.y); break;
    case 1: r.x = swz_dw<1>(w.x); r.y = swz_dw<1>(w.y); break;
    case 2: r.x = swz_dw<2>(w.x); r.y = swz_dw<2>(w.y); break;
    default: r.x = swz_dw<3>(w.x); r.y = swz_dw<3>(w.y); break;
  }
  return __builtin_bit_cast(double, r);
}


// One LD block of one LD matrix: n x n dense f64, row-major, row stride lda
// (multiple of PADV, zero padded); voff = offset of the block's first marker
// in the padded device vector layout.
struct BlkDesc {
  const double* R;
  int64_t lda;
  int64_t n;
  int64_t voff;
};

// Marker chunk (never crosses an LD block; chunking restarts at every block
// start, so per-block partial sums do not depend on how blocks are spread
// over ranks).
struct ChunkDesc {
  int64_t voff;
  int32_t len;
  int32_t blk;
};

// Row group of the dense LD pass: 4 waves x 8 rows of block `blk` from row0;
// its partial sums go to partial slot `part`.
struct RowGroup {
  int32_t blk;
  int32_t row0;
  int32_t part;
  int32_t pad_;
};

// ---- packed symmetric LD blocks (sym_pass.hip) ----------------------------
constexpr int SYM_H = 256;   // rows per panel
// packed band blocks: a panel's stored column extent is a multiple of BAND_Q (a
// whole number of panels), so the earlier panels covering a panel's rows are a
// contiguous range; an MFMA strip's items may stop 256 columns short of the
// strip's widest (SymStrip::ncmax: the kernels read zeros there)
constexpr int BAND_Q = 256;
// one (panel, column chunk) work item of k_sym_pass
struct SymItem {
  const double* P;   // panel base: element (r0, r0)
  int64_t w;         // panel row stride (doubles)
  int64_t voff;      // block's offset in the padded vector layout
  int32_t r0, H;     // panel first row (block-relative), rows
  int32_t c0, nc;    // chunk first column (block-relative), columns
  int32_t item;      // rowpart/colpart slot
  int32_t diag_end;  // r0 + H: columns >= diag_end also feed the transpose sums
};
// one panel of k_sym_finalize
struct SymPanel {
  int64_t voff;
  int32_t r0, H;
  int32_t item_begin, item_end;  // this panel's chunk items (in chunk order)
  int32_t g;                     // panel index inside its block
  int32_t blk_panel0;            // index (in the panel table) of the block's first panel
  int32_t part;                  // partial slot
  int32_t gmin;                  // first earlier panel of the block storing columns of this
                                 // panel's rows (0 unless the block is a packed band)
  // MFMA strips (k_sym_finalize_strip): the column sums of this panel's rows
  // sit in the strips of two 512-column chunks -- the chunk starting at r0 (the
  // panels of this panel's parity, row offset 0) and the one starting at
  // r0 - 256 (the other parity, row offset 256); colpart slots [sb, se)
  int32_t own_sb, own_se, oth_sb, oth_se;
  // coupled band pieces (sgv_set_ld_coupling): slot of this panel's rows in the
  // coupling sums PassArgs::cpbuf [slot][256][NC], added last; -1 = none
  int32_t cp;
};
// MFMA pass work item: one 512-column chunk (block-relative c0, shared by all
// its panels) over npan panels of one parity, g0, g0 + 2, ... (increasing);
// their (panel, chunk) items are sitems[it0 .. it0 + npan), column sums go to
// colpart slot `slot`; ncmax = the widest item's columns (a band's first item
// can be narrower than the others)
struct SymStrip {
  int32_t it0, npan, slot, ncmax;
};

// band walks (band_walk.hip): a workgroup walks panels p0 .. p0 + np - 1 (one
// block, consecutive; entries of the walk panel table) with a ring of R = the
// block's stored extent / 256 panel accumulators.  The first nhead panels are
// head panels (their partial sums -> headbuf slots hslot ..), the ring's ncarry
// open slots at the end -> carrybuf slots cslot ..
constexpr int WALK_RMAX = 5;   // ring slots of LDS (extent <= 1,280 columns)
struct SymWalk {
  int32_t p0, np, nhead, ncarry;
  int32_t hslot, cslot, R, pad_;
};
// one head panel: walk panel table entry, its partial's slot, the carry slot
struct WalkFin {
  int32_t panel, hslot, cslot, pad_;
};

// element (i, j) of a packed block is stored iff j >= 256 * floor(i / 256)
__device__ __forceinline__ double* sym_addr(double* base, const int64_t* poff, const int64_t* pw,
                                            int i, int j) {
  const int g = i / SYM_H;
  const int r0 = g * SYM_H;
  if (j < r0) return nullptr;
  return base + poff[g] + (int64_t)(i - r0) * pw[g] + (j - r0);
}

// Columns of one LD pass: out[c] = c1[c] * (R in[c]) + c2[c] * in[c];
// partial[c] = sum_rows dot[c] * out[c] (dot[c] may be null).
// out = c1 * (R in) + c2 * in; optionally also yout = ys1 * (R in) + ys0 * in
// (R_s in: the CG carries R_s x along its iterates, see sgv_lmmse)
struct PassArgs {
  const double* in[MAXC];
  double* out[MAXC];
  const double* dot[MAXC];
  double* yout[MAXC];
  double c1[MAXC];
  double c2[MAXC];
  double ys1, ys0;
  // non-null: the pass runs only if *run != 0 (device-side CG control: a pass
  // enqueued ahead of the stop test becomes a no-op); every workgroup reads it
  // next to its first descriptor load
  const int* run;
  // coupling sums of the panels next to a cut between coupled band pieces
  // ([slot][256][ncol], SymPanel::cp), written by k_coupling_lds before the finalize
  const double* cpbuf;
};

// One task of k_coupling_lds: up to 256 rows of one side of the coupling between
// band pieces gb and gb + 1 (C = R[tail nr rows of gb][head nc columns of gb + 1]):
//   side 0 (rows = gb's tail):   y[i] = sum_j C[i][j] p_{gb+1}[j]   (m = C^T, nc x nr)
//   side 1 (rows = gb+1's head): y[j] = sum_i C[i][j] p_{gb}[n - nr + i] (m = C, nr x nc)
// m is read as m[k * ldm + row] (coalesced over rows), k = 0 .. inner - 1 in
// order.  The source p is pa.in[c] + src (local) or halo + src + c * hstride.
struct CouplingTask {
  const double* m;
  int64_t src;       // source offset (see above)
  int32_t ldm, inner;
  int32_t row0, nrows;   // first output row (of the task's panel slot rows), count
  int32_t cp;        // panel slot
  int32_t prow0;     // the task's first output row within that panel
  int32_t local;     // 1: the source is local (pa.in), 0: the gathered halo
};

// most values one ordered reduction carries
constexpr int MAXNV = 4 * MAXKG + MAXC;
static_assert(MAXK <= MAXNV, "per-cohort sums (denoiser, MLE) fit one ordered reduction");

struct Map16 {
  int d[MAXNV];
};

// ---- deterministic reductions --------------------------------------------
// xor-butterfly: every lane ends with the same value (each step adds two
// values in commutative order), fixed order -> bitwise reproducible.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

// Wave-reduce P values at once (P a power of two <= 64) by halving: each step
// a lane keeps one half of its values and adds its partner's copy of that half
// (log2 P steps, P-1 shuffles in all, instead of 6 P for P butterflies), then
// butterflies over the remaining lane bits.  Lane l ends with the total of
// value index (l >> (6 - log2 P)) & (P - 1); fixed order, deterministic.
template <int P>
__device__ __forceinline__ double wave_reduce_many(double (&v)[P]) {
  constexpr int LOGP = (P >= 64) ? 6 : (P >= 32) ? 5 : (P >= 16) ? 4 : (P >= 8) ? 3
                     : (P >= 4) ? 2 : (P >= 2) ? 1 : 0;
  static_assert((1 << LOGP) == P, "P must be a power of two <= 64");
  const int lane = threadIdx.x & (WAVE - 1);
#pragma unroll
  for (int step = 0; step < LOGP; ++step) {
    const int o = 32 >> step;
    const int h = P >> (step + 1);
    const bool up = (lane & o) != 0;
#pragma unroll
    for (int k = 0; k < h; ++k) {
      const double send = up ? v[k] : v[k + h];
      const double keep = up ? v[k + h] : v[k];
      v[k] = keep + __shfl_xor(send, o, WAVE);
    }
  }
#pragma unroll
  for (int o = 32 >> LOGP; o > 0; o >>= 1) v[0] += __shfl_xor(v[0], o, WAVE);
  return v[0];
}

template <int N>
struct Pow2Ceil {
  static constexpr int value = N <= 1 ? 1 : N <= 2 ? 2 : N <= 4 ? 4 : N <= 8 ? 8 : N <= 16 ? 16
                             : N <= 32 ? 32 : 64;
};

// Sum NV per-thread values over a 256-thread workgroup and store NV results
// at out[0..NV) (fixed order: wave butterfly, then waves 0..3 in order).
template <int NV>
__device__ __forceinline__ void block_reduce_store(double (&v)[NV], double* __restrict__ out,
                                                   int nv_used) {
  __shared__ double sm[VTHREADS / WAVE][NV];
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = wave_sum(v[k]);
    if (lane == 0) sm[wid][k] = s;
  }
  __syncthreads();
  if ((int)threadIdx.x < nv_used) {
    const int t = threadIdx.x;
    out[t] = ((sm[0][t] + sm[1][t]) + sm[2][t]) + sm[3][t];
  }
}

// ---- packed-pass finalize (sym_pass.hip, sym_mfma.hip) --------------------
constexpr int FIN_Q = 4;   // threads per panel row in the finalize kernels

// Combine the FIN_Q parts of a row's sum in order (part 0 first), then, on
// part 0: out = c1*y + c2*in (and yout, R_s in), and the panel's partial dots
// (wave butterfly, waves 0..3 in order) -> partials[pn.part * NC + c].
// Called by every thread of a 256*FIN_Q workgroup.
// The inputs of the epilogue (in[c] and dot[c] at this thread's row, for the
// columns c = 4b + q its part writes) do not depend on the sums: fin_prefetch
// loads them at kernel start, so their latency hides behind the partial loads.
template <int NC>
struct FinPre {
  static constexpr int NB = (NC + FIN_Q - 1) / FIN_Q;
  double in[NB], dot[NB];
};
template <int NC>
__device__ __forceinline__ void fin_prefetch(const SymPanel& pn, const PassArgs& pa,
                                             FinPre<NC>& pre) {
  const int t = threadIdx.x & 255;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
  const int64_t idx = pn.voff + pn.r0 + (t < pn.H ? t : 0);
#pragma unroll
  for (int b = 0; b < FinPre<NC>::NB; ++b) {
    const int c = b * FIN_Q + q;
    pre.in[b] = 0.0;
    pre.dot[b] = 0.0;
    if (c < NC) {
      pre.in[b] = pa.in[c][idx];
      if (pa.dot[c]) pre.dot[b] = pa.dot[c][idx];
    }
  }
}

template <int NC>
__device__ __forceinline__ void fin_epilogue(const SymPanel& pn, const PassArgs& pa, double (&y)[NC],
                                             double* __restrict__ partials,
                                             const FinPre<NC>& pre) {
  // columns in batches of FIN_Q: every part stages its sums of the batch, then
  // part q combines column 4b + q (parts in order 0..3: the same additions as
  // one part adding the others' values) and writes its outputs and partial dot
  // -- two barriers per batch instead of two per column, all 16 waves busy
  constexpr int NB = FinPre<NC>::NB;
  __shared__ double s_y[FIN_Q][FIN_Q][256];
  __shared__ double s_w[4][NC];
  const int t = threadIdx.x & 255;
  const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
  const int lane = t & (WAVE - 1), wid = t / WAVE;
  const bool row = t < pn.H;
  const int64_t idx = pn.voff + pn.r0 + (row ? t : 0);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
#pragma unroll
    for (int j = 0; j < FIN_Q; ++j)
      if (b * FIN_Q + j < NC) s_y[q][j][t] = y[b * FIN_Q + j];
    __syncthreads();
    const int c = b * FIN_Q + q;
    if (c < NC) {
      double v = s_y[0][q][t];
#pragma unroll
      for (int p = 1; p < FIN_Q; ++p) v += s_y[p][q][t];
      if (pn.cp >= 0) v += pa.cpbuf[((int64_t)pn.cp * 256 + t) * NC + c];   // coupled pieces
      double acc = 0.0;
      if (row) {
        const double in = pre.in[b];
        const double o = pa.c1[c] * v + pa.c2[c] * in;
        pa.out[c][idx] = o;
        if (pa.yout[c]) pa.yout[c][idx] = pa.ys1 * v + pa.ys0 * in;
        if (pa.dot[c]) acc = pre.dot[b] * o;
      }
      const double sm = wave_sum(acc);
      if (lane == 0) s_w[wid][c] = sm;
    }
    __syncthreads();
  }
  if (threadIdx.x < NC)
    partials[(int64_t)pn.part * NC + t] = ((s_w[0][t] + s_w[1][t]) + s_w[2][t]) + s_w[3][t];
}

// A/B tuning switch from the environment, honoured only with SGV_AB=1 (capi.hip)
const char* ab_env(const char* name);

// streaming-read probe over `bytes` of buf (diag.hip); out: >= 256 doubles
hipError_t launch_read_probe(const double* buf, size_t bytes, double* out, hipStream_t st);

// ---- launchers (defined in the .hip files) ------------------------------
// coupling sums between band pieces (sym_pass.hip): cpbuf[slot][256][nc]
hipError_t launch_coupling(int nc, const CouplingTask* d_tasks, int ntasks, const PassArgs& pa,
                           const double* halo, int64_t hstride, double* cpbuf, int ncp_slots,
                           hipStream_t st);
hipError_t launch_halo_pack(const PassArgs& pa, int nc, int64_t src0, int len0, int64_t src1,
                            int len1, int64_t hstride, double* send, hipStream_t st);
// LD pass: one workgroup per row group; partials[rg.part * nc + c].
hipError_t launch_ld_pass(int nc, const BlkDesc* d_blks, const RowGroup* d_rg, int nrg,
                          const PassArgs& pa, double* d_partials, hipStream_t st);
int ld_pass_rows_per_group();
// symmetric pass over packed blocks, then per-panel finalize (partials[panel.part * nc + c])
// chunk-width class cls: CW = 1024 >> cls columns per work item
hipError_t launch_sym_pass(int nc, int cls, const SymItem* d_items, int nitems,
                           const PassArgs& pa, double* rowpart, double* colpart, hipStream_t st);
// MFMA pass (sym_mfma.hip): launch_pk interleaves the columns into Pk, then
// launch_sym_mfma runs strips d_strips[0 .. nstrips) (one block group or all)
// paired: the 5-8-column passes' Pk layout (band walks and strips:
// strip_pk_paired)
hipError_t launch_pk(const PassArgs& pa, int nc, int64_t mpad, double* d_pk, hipStream_t st,
                     bool paired = false);
bool strip_pk_paired(int nc);
hipError_t launch_sym_mfma(int nc, const SymStrip* d_strips, int nstrips, const SymItem* d_sitems,
                           const PassArgs& pa, const double* d_pk, double* rowpart,
                           double* colpart, bool ragged, int pair, hipStream_t st);
// band walks (NC <= 8, band_walk.hip): the walks, then the head panels' finalize
hipError_t launch_band_walk(int nc, const SymWalk* d_walks, int nwalks, const SymPanel* d_panels,
                            const SymItem* d_items, const double* d_pk, int64_t pk_rows,
                            const PassArgs& pa, double* headbuf, double* carrybuf,
                            const WalkFin* d_fins, int nfins,
                            double* partials, hipStream_t st);
hipError_t launch_sym_finalize_strip(int nc, const SymPanel* d_panels, int npanels,
                                     const PassArgs& pa, const double* rowpart,
                                     const double* colpart, double* partials, bool ragged,
                                     hipStream_t st);
hipError_t launch_sym_finalize(int nc, int cls, const SymPanel* d_panels, int npanels,
                               const PassArgs& pa, const double* rowpart, const double* colpart,
                               double* partials, hipStream_t st);

// Reductions: partials[part * nv + v] with parts of local block b in
// [begin[b], begin[b+1]) -> bsum[b * nv + v] (fixed order), then
// total[v] = sum over all ranks' blocks in global block order, written to
// dst[map.d[v]].
// op 0: ordered sum; op 1: min (exact in any order)
// (ostride > 0: block b's values at bsum[b * ostride + ooff ..], two sources
// sharing one exchange)
hipError_t launch_reduce_blocks(const double* d_part, int nv, const int* d_begin, int nblk,
                                double* d_bsum, hipStream_t st, int op = 0, int ostride = 0,
                                int ooff = 0);
hipError_t launch_reduce_local(const double* d_part, int nv, const int* d_begin, int nblk,
                               const Map16& map, double* d_dst, hipStream_t st, int op = 0);
hipError_t launch_reduce_total(const double* d_bsum_all, int nranks, int nbmax, int nv,
                               const int* d_counts, const Map16& map, double* d_dst,
                               hipStream_t st, int op = 0);

// Vector kernels (vec.hip) ------------------------------------------------
struct DenoiseArgs {
  const double* r1[MAXK];
  double* xhat1;
  double ag[MAXK];          // a_k * gam1_k
  double a[MAXK], gam1[MAXK];
  double sum_ag;            // builtin sum over k, src/sgvamp.py:95
  double lam;
  int K, nslab;
  double omegas[MAXL], sigmas[MAXL];
  double s2[MAXL];          // sigma2_meta (shared by all markers)
  double sq[MAXL];          // sqrt(sigma2_meta / sigmas)
  double rho;
  int damp;
  // cohort groups (K > MAXK): np.inner over every cohort precomputed by
  // launch_den_inner; only the first group writes xhat1 (with the damping)
  const double* inner;
  int write_x;
  // non-null (with write_x, no cohort groups): the metrics sums of the written
  // xhat1 against x0 (k_metrics' four, in its order) ride in the same partials,
  // after the K derivative sums -- one ordered reduction for both
  const double* x0;
};
hipError_t launch_denoise(const ChunkDesc* d_ch, int nch, const DenoiseArgs& a, double* d_part,
                          hipStream_t st);
// inner[i] = (first ? 0 : inner[i]) + sum over the a.K cohorts of r1_k[i] * ag_k,
// in cohort order (continuing one sequential sum over the groups)
hipError_t launch_den_inner(const ChunkDesc* d_ch, int nch, const DenoiseArgs& a, double* inner,
                            int first, hipStream_t st);

struct MleArgs {
  const double* r1[MAXK];
  double a[MAXK];
  double ginv[MAXK];           // 1/gam1_k (:146); v_kl = sigma2_l + ginv_k, sv = sqrt(v)
  double sigma2[MAXL + 1];     // prior_vars0 (spike first)
  double omega[MAXL + 1];
  double exp_max;
  int K, L;                    // L = components incl. the spike (reference self.L)
};
hipError_t launch_mle_minsq(const ChunkDesc* d_ch, int nch, const MleArgs& a, double* d_part,
                            hipStream_t st);
hipError_t launch_mle_terms(const ChunkDesc* d_ch, int nch, const MleArgs& a, double* d_part,
                            hipStream_t st);

// Device-side EM control (k_em_ctl, the device EM loop of sgv_em): the prior
// scalars between steps, the last step's error and the stop flag
struct EmState {
  double lam;
  double om[MAXL];
  double err;               // max(omegas_rel_err, lam_rel_err) of the last step
  int steps;
  int done;                 // converged or em_prior_maxit reached: k_em is a no-op
};
// per-cohort constants of an EM loop (k_em_prep, from gam1 and sigmas): [0] ginv
// = 1/gam1, [1] sqrt(ginv), [2 + l] sigmas[l] + ginv, [2 + MAXL + l]
// sqrt(ginv + sigmas[l]) -- the reference's per-element expressions (:125-131),
// formed once instead of once per marker (same operations, same bits)
constexpr int EM_TAB = 2 + 2 * MAXL;
struct EmArgs {
  const EmState* st;        // non-null: lam and omegas from the device state
  const double* tab;        // [K][EM_TAB] (k_em_prep)
  const double* r1[MAXK];
  double a[MAXK];
  double gam1[MAXK];
  double scl;               // sum_k a_k (np.average weights)
  double lam;
  int K, nslab;
  double omegas[MAXL], sigmas[MAXL];
  int accum;                // cohort groups after the first add to the partials
};
constexpr int EM_NV = MAXL + 2;   // [0] sum_j avg_k(pi); [1..L-1] omega numerators; [nslab+1] denominator
hipError_t launch_em(const ChunkDesc* d_ch, int nch, const EmArgs& a, double* d_part,
                     hipStream_t st);
// fills tab[K][EM_TAB] from a.gam1 / a.sigmas (once per EM loop)
hipError_t launch_em_prep(const EmArgs& a, double* tab, hipStream_t st);
// one EM update from the reduced sums tot[EM_NV] (src/sgvamp.py:134-136) and the
// loop's stop test (:252-257); it + 1 == maxit also stops.  The state is
// copied to `mirror` (host memory).
hipError_t launch_em_ctl(EmState* d_st, EmState* mirror, const double* d_tot, int nslab,
                         double Mtot, int it, int maxit, hipStream_t st);
// k_em_reduce_ctl (one rank): the ordered reduction of k_em's partials and the
// k_em_ctl update in one single-workgroup launch (same bits)
constexpr int EM_CTL_MAXBLK = 128;   // LD blocks per rank
struct EmCtl {
  const int* begin;         // parts of LD block b: [begin[b], begin[b + 1])
  int nblk, nslab;
  EmState* mirror;
  double Mtot;
  int it, maxit;
};
hipError_t launch_em_reduce_ctl(const double* d_part, EmState* d_st, const EmCtl& f,
                                hipStream_t st);

struct CohortPtrs {   // one LMMSE cohort group
  const double* r[MAXKG];
  const double* r1[MAXKG];
  double* r2[MAXKG];
  const double* u[MAXKG];
};
struct ColPtrs {
  double* X[MAXC];
  double* X0[MAXC];
  double* Rr[MAXC];
  double* P[MAXC];
  double* Q[MAXC];
  double* RX0[MAXC];        // R_s X (the carried products)
  double* RXp[MAXC];        // copy of RX0 at the start (damping of xhat2)
};
struct InitArgs {
  CohortPtrs cp;
  ColPtrs col;
  const double* xhat1;
  int K;                    // cohorts in the group
  double alpha1[MAXKG], gamw[MAXKG], gam2[MAXKG];
  int warm[MAXC];           // residual r = b - A x0 (x0.any()); else r = b
  int save_x0;              // copy X[2k] to X0[2k] (and RX0 to RXp) for LMMSE damping
};
hipError_t launch_lmmse_init(const ChunkDesc* d_ch, int nch, const InitArgs& a, double* d_part,
                             hipStream_t st);

// Device-side CG control (k_cg_ctl, the pipelined CG of capi.hip): per column
// the scipy loop scalars; `any` = some column still iterating.
struct CgState {
  double rho[MAXC];        // r.r of the current iterate (rho_cur)
  double rho_prev[MAXC];
  double beta[MAXC];
  double atol[MAXC];
  int active[MAXC];
  int iters[MAXC];
  int info[MAXC];
  int any;
  int it;
  int zero[MAXC];          // bnrm2 == 0 at the start: x = b = 0 (iterative.py:380-381)
};
// iteration `it` of the CG (iterative.py:397-407): it > 0 first takes rho_new
// (the r.r reduction of iteration it-1) for the active columns; then the stop
// test sqrt(rho) < atol (strict), and beta = rho / rho_prev.  final_it >= 0
// instead marks the still-active columns as exhausted (iters = info =
// final_it, :420-422).  The state is also copied to `mirror` (host memory).
hipError_t launch_cg_ctl(CgState* d_st, CgState* mirror, const double* d_rho_new, int it,
                         int ncol, int final_it, hipStream_t st);
// one rank: k_reduce_local of k_cg_xr's r.r partials (iteration it - 1) + the
// control of iteration it (it >= 1) in one launch, same bits
hipError_t launch_cg_reduce_ctl(const double* d_part, const int* d_begin, int nblk,
                                CgState* d_st, CgState* mirror, int it, int ncol,
                                hipStream_t st);
// the CG prologue's scalars from the device-reduced |b|^2 (tot[c]) and |r0|^2
// (tot[MAXC + c]) (iterative.py:376-392): rho, atol = max(0, rtol |b|), active
// unless |b| == 0; then X and R_s X of the |b| == 0 columns are zeroed
hipError_t launch_cg_init(CgState* d_st, const double* d_tot, double rtol, int ncol,
                          const ChunkDesc* d_ch, int nch, double* const* X, double* const* RX,
                          hipStream_t st);
hipError_t launch_copy_f64(double* dst, const double* src, int n, hipStream_t st);

struct XrArgs {
  double* X[MAXC];
  double* Rr[MAXC];
  const double* P[MAXC];
  const double* Q[MAXC];
  double* RX[MAXC];         // RX += alpha Y (R_s x carried), if non-null
  const double* Y[MAXC];    // R_s p from the pass
  double rho[MAXC];
  const double* pq;         // device, indexed by column
  unsigned mask;
  int ncol;
  const CgState* st;        // non-null: rho and the active columns from the device state
};
hipError_t launch_cg_xr(const ChunkDesc* d_ch, int nch, const XrArgs& a, double* d_part,
                        hipStream_t st);

struct PArgs {
  double* P[MAXC];
  const double* Rr[MAXC];
  double beta[MAXC];
  unsigned mask;
  int ncol;
  const CgState* st;        // non-null: beta and the active columns from the device state
};
hipError_t launch_cg_p(const ChunkDesc* d_ch, int nch, const PArgs& a, hipStream_t st);

struct PostArgs {
  double* X[MAXC];
  const double* X0[MAXC];
  double* RX[MAXC];         // carried R_s X (rs != 0): damped with X, dotted for gamw
  const double* RXp[MAXC];
  const double* u[MAXKG];
  const double* r[MAXKG];
  int K;                    // cohorts in the group
  int damp;
  int rs;
  double rho;
};
hipError_t launch_lmmse_post(const ChunkDesc* d_ch, int nch, const PostArgs& a, double* d_part,
                             hipStream_t st);

struct R1Args {               // one LMMSE cohort group
  const double* X[MAXKG];    // xhat2_k
  const double* r2[MAXKG];
  double* r1[MAXKG];
  double alpha2[MAXKG];
  int K;
  // non-null: alpha2 from the device-reduced Tr(Sigma2) trs[k] (:340, 345-346):
  // alpha2 = gam2 trs / Mtot, damped with alpha2_prev
  const double* trs;
  double gam2[MAXKG], alpha2_prev[MAXKG];
  double Mtot, rho;
  int damp;
};
hipError_t launch_r1_update(const ChunkDesc* d_ch, int nch, const R1Args& a, hipStream_t st);

hipError_t launch_metrics(const ChunkDesc* d_ch, int nch, const double* xhat1, const double* x0,
                          double* d_part, hipStream_t st);

// generic column dots over chunks: part[c] = sum x[c]*y[c]
struct DotsArgs {
  const double* x[MAXC];
  const double* y[MAXC];
  int ncol;
};
hipError_t launch_dots(const ChunkDesc* d_ch, int nch, const DotsArgs& a, double* d_part,
                       hipStream_t st);

// scatter dense local vector -> padded layout and back
hipError_t launch_unpack(const ChunkDesc* d_ch, int nch, const int64_t* d_dense_off,
                         const double* src_dense, double* dst_pad, hipStream_t st);
hipError_t launch_unpack_i8(const ChunkDesc* d_ch, int nch, const int64_t* d_dense_off,
                            const int8_t* src_dense, double* dst_pad, hipStream_t st);
hipError_t launch_pack(const ChunkDesc* d_ch, int nch, const int64_t* d_dense_off,
                       const double* src_pad, double* dst_dense, hipStream_t st);
// y[c] = a[c] * y[c] + b[c] * x[c]
struct AxpbyArgs {
  double* y[MAXC];
  const double* x[MAXC];
  double a[MAXC], b[MAXC];
  int ncol;
};
hipError_t launch_axpby(const ChunkDesc* d_ch, int nch, const AxpbyArgs& a, hipStream_t st);

// Synthetic generator (synth.hip) ----------------------------------------
hipError_t launch_geno_stats(uint64_t seed, int64_t gmarker0, int n, int nsamp, double* d_mean,
                             double* d_std, hipStream_t st);
hipError_t launch_geno_G(uint64_t seed, int64_t gmarker0, int n, int nsamp, int ldg,
                         const double* d_mean, const double* d_std, double* d_G,
                         hipStream_t st);
// R = G G^T; packed != 0: write the packed symmetric layout (poff/pw per panel)
hipError_t launch_syrk_nt(const double* d_G, int n, int nsamp, int ldg, double* d_R, int64_t lda,
                          int packed, const int64_t* d_poff, const int64_t* d_pw, hipStream_t st);
hipError_t launch_g_accum(uint64_t seed, int64_t gmarker0, int n, int nsamp, const double* d_mean,
                          const double* d_std, const double* d_beta, double* d_g, hipStream_t st);
hipError_t launch_row_dot(const double* d_G, int n, int nsamp, int ldg, const double* d_y,
                          double* d_out, hipStream_t st);

}  // namespace sgv
