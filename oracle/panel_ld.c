/*
 * ORACLE (test infrastructure, never a product path) -- the host LD product of
 * oracle/vamp_oracle.py's PanelLD in plain C, so that the north star's own
 * 50-iteration parity gate (M = 1e6, K = 4: 63.5 GB of packed LD per pass)
 * fits the driver's GPU suite.
 *
 * What it restates: Y = R V for one symmetric LD block held as its upper
 * triangle in panels of H rows (panel g: rows r0 = g*H .. r0+h-1 over columns
 * r0 .. n-1, row stride n - r0) -- the operator the reference applies through
 * scipy's cg on A = gamw*R_s + gam2*I (/root/reference/src/sgvamp.py:312,316,
 * 332) with R the block-diagonal LD of src/main.py:199-202.  Each stored
 * element R_ij (j >= i) adds R_ij V_j to row i and, right of the panel's
 * diagonal block, R_ij V_i to row j.  Arithmetic is IEEE f64, every
 * multiply-add an explicit fused one (so a column's bits do not depend on how
 * the compiler vectorises over the columns, nor on how many columns a call
 * carries), one thread per panel range: the order of the additions is fixed,
 * whatever the caller's thread count.
 *
 * Built by oracle/Makefile (__graft_entry__.build()); loaded only by
 * oracle/vamp_oracle.py, which falls back to NumPy when it is absent.
 */
#include <stdint.h>
#include <string.h>

/* RB panel rows at a time, each stored row streamed once from its start: the
 * row sums of the RB rows stay in registers, and each transpose target Y_j is
 * read and written once per RB rows (not once per stored row).  Pointers are
 * restrict-qualified and the rows' own V entries copied to locals so the
 * compiler keeps them in registers (the first form, without, ran at ~0.4 GB/s). */
enum { RB = 4 };

static inline __attribute__((always_inline)) void rows_nc(
    int64_t w, int64_t h, int64_t nr, const double* __restrict P, const double* __restrict Vp,
    double* __restrict Yp, int64_t i0, const int NC) {
  double acc[RB][16], vi[RB][16];
  const double* row[RB];
  for (int r = 0; r < RB; ++r) {
    const int64_t i = i0 + (r < nr ? r : 0);
    row[r] = P + i * w;
    for (int c = 0; c < NC; ++c) {
      acc[r][c] = 0.0;
      vi[r][c] = r < nr ? Vp[i * NC + c] : 0.0;
    }
  }
  for (int64_t j = 0; j < h; ++j) {                 /* the panel's diagonal block: rows only */
    const double* vj = Vp + j * NC;
    for (int r = 0; r < RB; ++r) {
      const double a = row[r][j];
      for (int c = 0; c < NC; ++c) acc[r][c] = __builtin_fma(a, vj[c], acc[r][c]);
    }
  }
  for (int64_t j = h; j < w; ++j) {                 /* right of it: rows and transposes */
    const double* vj = Vp + j * NC;
    double yj[16];
    for (int c = 0; c < NC; ++c) yj[c] = Yp[j * NC + c];
    for (int r = 0; r < RB; ++r) {
      const double a = r < nr ? row[r][j] : 0.0;
      for (int c = 0; c < NC; ++c) {
        acc[r][c] = __builtin_fma(a, vj[c], acc[r][c]);
        yj[c] = __builtin_fma(a, vi[r][c], yj[c]);
      }
    }
    for (int c = 0; c < NC; ++c) Yp[j * NC + c] = yj[c];
  }
  for (int r = 0; r < nr; ++r)
    for (int c = 0; c < NC; ++c) Yp[(i0 + r) * NC + c] += acc[r][c];
}

static inline __attribute__((always_inline)) void block_nc(int64_t n, int H, const double* const* panels,
                                                           int64_t g0, int64_t g1,
                                                           const double* __restrict V,
                                                           double* __restrict Y, const int NC) {
  for (int64_t g = g0, r0 = g0 * H; g < g1 && r0 < n; r0 += H, ++g) {
    const int64_t h = (n - r0) < H ? (n - r0) : H;
    const int64_t w = n - r0;
    for (int64_t i0 = 0; i0 < h; i0 += RB)
      rows_nc(w, h, (h - i0) < RB ? (h - i0) : RB, panels[g], V + r0 * NC, Y + r0 * NC, i0, NC);
  }
}

/* Y (n x ncol, row-major, zeroed here) = the part of R V for one block that
 * panels g0 .. g1 - 1 store (their rows and, right of their diagonal blocks,
 * their transposes); the whole block is g0 = 0, g1 = its panel count.  Each
 * column's arithmetic is independent of the others (a column gives the same
 * bits alone or with others).  0 on success. */
int oracle_panel_range_matmat(int64_t n, int H, const double* const* panels, int64_t g0,
                              int64_t g1, int ncol, const double* V, double* Y) {
  if (n < 0 || H < 1 || H > 256 || ncol < 1 || ncol > 16 || g0 < 0 || g1 < g0) return -1;
  memset(Y, 0, sizeof(double) * (size_t)n * (size_t)ncol);
  switch (ncol) {   /* constant column counts: the inner loops vectorise */
#define NC_CASE(k) \
  case k:          \
    block_nc(n, H, panels, g0, g1, V, Y, k); \
    break;
    NC_CASE(1) NC_CASE(2) NC_CASE(3) NC_CASE(4) NC_CASE(5) NC_CASE(6) NC_CASE(7) NC_CASE(8)
    NC_CASE(9) NC_CASE(10) NC_CASE(11) NC_CASE(12) NC_CASE(13) NC_CASE(14) NC_CASE(15)
    NC_CASE(16)
#undef NC_CASE
  }
  return 0;
}

int oracle_panel_block_matmat(int64_t n, int H, const double* const* panels, int ncol,
                              const double* V, double* Y) {
  return oracle_panel_range_matmat(n, H, panels, 0, (n + H - 1) / H, ncol, V, Y);
}
