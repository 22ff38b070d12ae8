// The solver half of libsgvamp_hip.so's host side: the batched scipy-1.15.3 CG
// (iterative.py:375-422; pipelined, device-side control), the LMMSE step
// (src/sgvamp.py:301-364), the meta denoiser (:93-114, 270-291), the EM prior
// loop (:116-136, 250-257), the MLE prior update (:139-194, fsolve restated in
// hybrd.cpp), the operator seam (con_grad, :7,316,332) and the one-call outer
// iteration with its worker thread (:222-387).
#include "ctx.h"

// ---------------------------------------------------------------------------
// batched CG (scipy 1.15.3, iterative.py:375-422) on columns 0..ncol-1.
// On entry: X = x0, Rr = P = r0 (= b - A x0 or b), rho[c] = r0.r0,
// atol[c] = rtol*|b|.  Columns with active[c] = 0 are skipped (bnrm2 == 0).
// Column c uses LD matrix col_ld[c] and A = c1[c] R + c2[c] I.
// ---------------------------------------------------------------------------
struct CgCols {
  int ncol = 0;
  int col_ld[MAXC];
  double c1[MAXC], c2[MAXC];
  double* X[MAXC];
  double* Rr[MAXC];
  double* P[MAXC];
  double* Q[MAXC];
  double* RX[MAXC] = {};   // non-null: carry R_s x (RX += alpha R_s p), Y = R_s p scratch
  double* Y[MAXC] = {};
  double s = 0.0;          // ridge of R_s
};

static int cg_loop(sgv_ctx* c, const CgCols& cc, double* rho, const double* atol, int maxiter,
                   const int* active_in, int* iters, int* info, int* passes) {
  const int ncol = cc.ncol;
  int active[MAXC];
  double rho_prev[MAXC];
  for (int j = 0; j < ncol; ++j) {
    active[j] = active_in[j];
    rho_prev[j] = 0.0;
    if (!active[j]) {
      iters[j] = 0;
      info[j] = 0;
    }
  }
  for (int it = 0; it < maxiter; ++it) {
    unsigned mask = 0;
    for (int j = 0; j < ncol; ++j) {
      if (!active[j]) continue;
      if (std::sqrt(rho[j]) < atol[j]) {  // iterative.py:398 (strict <)
        active[j] = 0;
        iters[j] = it;
        info[j] = 0;
        continue;
      }
      mask |= 1u << j;
    }
    if (!mask) return SGV_OK;
    if (it > 0) {  // iterative.py:403-407
      PArgs pa{};
      pa.ncol = ncol;
      pa.mask = mask;
      for (int j = 0; j < ncol; ++j) {
        pa.P[j] = cc.P[j];
        pa.Rr[j] = cc.Rr[j];
        pa.beta[j] = (mask >> j & 1u) ? rho[j] / rho_prev[j] : 0.0;
      }
      HIPCHK(launch_cg_p(c->d_ch, c->nch, pa, c->st));
    }
    // q = A p (iterative.py:411): one pass per LD matrix over its active columns
    for (int ld = 0; ld < c->nld; ++ld) {
      PassArgs pa{};
      Map16 map = identity_map();
      int nc = 0;
      for (int j = 0; j < ncol; ++j) {
        if (!(mask >> j & 1u) || cc.col_ld[j] != ld) continue;
        pa.in[nc] = cc.P[j];
        pa.out[nc] = cc.Q[j];
        pa.dot[nc] = cc.P[j];
        pa.yout[nc] = cc.RX[j] ? cc.Y[j] : nullptr;
        pa.c1[nc] = cc.c1[j];
        pa.c2[nc] = cc.c2[j];
        map.d[nc] = j;
        ++nc;
      }
      if (!nc) continue;
      pa.ys1 = 1.0 - cc.s;   // Y = R_s p = (1-s) R p + s p
      pa.ys0 = cc.s;
      CHK(ld_pass(c, ld, nc, pa));
      CHK(reduce_dev(c, nc, ld_parts(c, ld), map, c->d_pq));
      if (passes) ++*passes;
    }
    // alpha = rho / p.q; x += alpha p; r -= alpha q; rho_new = r.r (:412-415)
    XrArgs xa{};
    xa.ncol = ncol;
    xa.mask = mask;
    xa.pq = c->d_pq;
    for (int j = 0; j < ncol; ++j) {
      xa.X[j] = cc.X[j];
      xa.Rr[j] = cc.Rr[j];
      xa.P[j] = cc.P[j];
      xa.Q[j] = cc.Q[j];
      xa.RX[j] = cc.RX[j];
      xa.Y[j] = cc.Y[j];
      xa.rho[j] = rho[j];
    }
    HIPCHK(launch_cg_xr(c->d_ch, c->nch, xa, c->d_part, c->st));
    double rn[MAXC];
    CHK(reduce_host(c, MAXC, c->d_ch_begin, rn));
    for (int j = 0; j < ncol; ++j)
      if (mask >> j & 1u) {
        rho_prev[j] = rho[j];
        rho[j] = rn[j];
      }
  }
  for (int j = 0; j < ncol; ++j)
    if (active[j]) {  // for-loop exhausted (iterative.py:420-422)
      iters[j] = maxiter;
      info[j] = maxiter;
    }
  return SGV_OK;
}

// spin on an event already recorded on the ctx stream
static int event_spin(sgv_ctx* c, hipEvent_t ev) {
  hipError_t e;
  while ((e = hipEventQuery(ev)) == hipErrorNotReady) __builtin_ia32_pause();
  if (e != hipSuccess) return fail(c, SGV_ERR_HIP, "event wait: %s", hipGetErrorString(e));
  return SGV_OK;
}

// Pipelined CG: the iteration of cg_loop with the stop test, beta and alpha on
// the device, so no host round trip sits between two iterations.  Iteration it
// is enqueued as [k_cg_ctl (stop test of `it`, beta), p update, LD pass(es) +
// p.q, x/r update + r.r]; the p/x/r kernels and the passes read the device
// state and become no-ops once no column is active.  The host then waits only
// for k_cg_ctl of `it` (the first kernel of the iteration: the wait overlaps
// the pass) and enqueues it + 1 behind it with the columns still active after
// that test -- so the column set of every pass is a function of the trajectory
// alone (deterministic; a column stopping at it + 1's test rides along in that
// pass unused).  When the test of `it` stops every column, that iteration's
// kernels were no-ops: their pass timers and byte counts are dropped.
// Exact column sets (default, from it = 1): the p update of `it` (a no-op for
// the columns the device state has stopped) is enqueued first, then the host
// waits for the test of `it` -- it completes while that p update runs -- and
// enqueues the passes with the columns still active after it.  A CG #1 column
// that stops one iteration before its CG #2 partner then leaves the pass
// (north star: NC 8 -> 4, one pass in three once the iteration counts split;
// the same iterates bit for bit there).  Where the smaller set crosses a kernel
// boundary (NC <= 2 runs the VALU pass, 3..16 the MFMA pass) the surviving
// columns' sums are formed in another order: equal to rounding.
// With a communicator the CG prologue's sums (|b|^2, |r0|^2: the LMMSE init
// kernel's partials, `m0`) ride in the exchange of iteration 0's p.q instead of
// one of their own: the first pass runs on p0 = r0 for every column before the
// stop test of iteration 0 is known (as the look-ahead pass does), then
// k_cg_init and the test follow the shared reduction.  Same values, one
// exchange fewer per LMMSE; only where one LD matrix serves every column.
struct CgMerge0 {
  const double* part = nullptr;   // [chunk][2 MAXC] (k_lmmse_init)
  double rtol = 0.0;
  double* const* X = nullptr;     // k_cg_init zeroes X, R_s X of |b| == 0 columns
  double* const* RX = nullptr;
};

static int cg_loop_dev(sgv_ctx* c, const CgCols& cc, const double* rho0, const double* atol,
                       int maxiter, const int* active_in, int* iters, int* info, int* passes,
                       const CgMerge0* m0 = nullptr) {
  const int ncol = cc.ncol;
  unsigned mask = 0;
  if (rho0) {
    CgState* hi = c->h_cgi;   // the previous solve's copy has completed (its mirror was read)
    std::memset(hi, 0, sizeof(CgState));
    for (int j = 0; j < ncol; ++j) {
      hi->rho[j] = rho0[j];
      hi->atol[j] = atol[j];
      hi->active[j] = active_in[j] ? 1 : 0;
      if (active_in[j]) mask |= 1u << j;
    }
    hi->any = mask ? 1 : 0;
    HIPCHK(hipMemcpyAsync(c->d_cgs, hi, sizeof(CgState), hipMemcpyHostToDevice, c->st));
  } else {
    // state set by k_cg_init on the stream; a |b| == 0 column is inactive there
    // and rides along unused in the first pass (its result is never read)
    mask = ncol >= 32 ? ~0u : (1u << ncol) - 1u;
  }
  const volatile CgState* last = nullptr;
  int executed = 0;
  // one rank: iteration it's r.r reduction and the control of it + 1 are one
  // launch (k_cg_reduce_ctl), enqueued at the end of it, when that one
  // workgroup's reduction is short (fused_ctl_pays); SGV_EM_FUSE=0 A/B
  const bool fuse = !c->comm && !c->host_ag && fused_ctl_pays(MAXC, c->nblk);
  // exact sets pay only where fewer columns make a pass cheaper: the MFMA pass
  // (>= 3 columns of one LD matrix, cost by groups of 4); the VALU pass costs
  // the same at 1 and 2 columns (C2: 3.19 vs 3.21 ms), so K = 1 and distinct-LD
  // pairs keep the look-ahead and its host read stays off the critical path
  int widest = 0;
  double wide_bytes = 0.0;   // largest pass of >= 3 columns (this rank's blocks)
  for (int j = 0; j < ncol; ++j) {
    int n = 0;
    for (int i = 0; i < ncol; ++i) n += cc.col_ld[i] == cc.col_ld[j];
    widest = std::max(widest, n);
    if (n >= 3 && c->cg_exact < 0 && !c->comm && !c->host_ag) {
      CHK(ensure_plan(c, cc.col_ld[j]));
      wide_bytes = std::max(wide_bytes, c->plan[cc.col_ld[j]].stored_bytes);
    }
  }
  const bool exact = widest >= 3 && (c->cg_exact > 0 || (c->cg_exact < 0 && !c->comm &&
                                                         !c->host_ag &&
                                                         wide_bytes >= CG_EXACT_MIN_BYTES));
  for (int it = 0; it < maxiter; ++it) {
    const size_t np0 = c->pending.size();
    const double cnt0[8] = {c->ld_launches, c->ld_bytes, c->dense_bytes, c->rhs_bytes,
                            c->aux_bytes, c->ld_flops, c->ld_flops_wide, c->ld_launches_wide};
    int npass = 0;
    CgState* slot = c->h_cgm + (it % CG_RING);
    const bool merge = m0 && it == 0;   // the prologue's sums ride with this p.q
    if ((it == 0 || !fuse) && !merge) {
      HIPCHK(launch_cg_ctl(c->d_cgs, slot, c->d_rhonew, it, ncol, -1, c->st));
      HIPCHK(hipEventRecord(c->ev_cg[it % CG_RING], c->st));
    }
    if (it > 0) {  // iterative.py:403-407
      PArgs pa{};
      pa.ncol = ncol;
      pa.mask = mask;
      pa.st = c->d_cgs;
      for (int j = 0; j < ncol; ++j) {
        pa.P[j] = cc.P[j];
        pa.Rr[j] = cc.Rr[j];
      }
      HIPCHK(launch_cg_p(c->d_ch, c->nch, pa, c->st));
    }
    const bool pre = exact && it > 0;   // the test of `it` read before its passes
    if (pre) {
      // the device's idle gap this read costs: p update done -> passes enqueued
      hipEvent_t g0, g1;
      CHK(event_pair(c, &g0, &g1));
      HIPCHK(hipEventRecord(g0, c->st));
      CHK(event_spin(c, c->ev_cg[it % CG_RING]));
      HIPCHK(hipEventRecord(g1, c->st));
      c->gpending.emplace_back(g0, g1);
      last = slot;
      if (!last->any) break;            // only the (no-op) p update was enqueued
      mask = 0;
      for (int j = 0; j < ncol; ++j)
        if (last->active[j]) mask |= 1u << j;
    }
    // q = A p (iterative.py:411): one pass per LD matrix over its columns
    for (int ld = 0; ld < c->nld; ++ld) {
      PassArgs pa{};
      Map16 map = identity_map();
      int nc = 0;
      for (int j = 0; j < ncol; ++j) {
        if (!(mask >> j & 1u) || cc.col_ld[j] != ld) continue;
        pa.in[nc] = cc.P[j];
        pa.out[nc] = cc.Q[j];
        pa.dot[nc] = cc.P[j];
        pa.yout[nc] = cc.RX[j] ? cc.Y[j] : nullptr;
        pa.c1[nc] = cc.c1[j];
        pa.c2[nc] = cc.c2[j];
        map.d[nc] = j;
        ++nc;
      }
      if (!nc) continue;
      pa.ys1 = 1.0 - cc.s;   // Y = R_s p = (1-s) R p + s p
      pa.ys0 = cc.s;
      pa.run = merge ? nullptr : &c->d_cgs->any;   // merge: the state is set after it
      CHK(ld_pass(c, ld, nc, pa));
      if (merge) {   // [|b|^2, |r0|^2] -> d_tot[0 .. 2 MAXC), p.q -> d_tot[2 MAXC + j]
        CHK(reduce_dev2(c, m0->part, 2 * MAXC, c->d_ch_begin, nc, ld_parts(c, ld), map, 2 * MAXC,
                        c->d_tot));
        HIPCHK(launch_cg_init(c->d_cgs, c->d_tot, m0->rtol, ncol, c->d_ch, c->nch, m0->X, m0->RX,
                              c->st));
        HIPCHK(launch_cg_ctl(c->d_cgs, slot, c->d_rhonew, it, ncol, -1, c->st));
        HIPCHK(hipEventRecord(c->ev_cg[it % CG_RING], c->st));
      } else {
        CHK(reduce_dev(c, nc, ld_parts(c, ld), map, c->d_pq));
      }
      ++npass;
    }
    // alpha = rho / p.q; x += alpha p; r -= alpha q; r.r (:412-415)
    XrArgs xa{};
    xa.ncol = ncol;
    xa.mask = mask;
    xa.pq = merge ? c->d_tot + 2 * MAXC : c->d_pq;
    xa.st = c->d_cgs;
    for (int j = 0; j < ncol; ++j) {
      xa.X[j] = cc.X[j];
      xa.Rr[j] = cc.Rr[j];
      xa.P[j] = cc.P[j];
      xa.Q[j] = cc.Q[j];
      xa.RX[j] = cc.RX[j];
      xa.Y[j] = cc.Y[j];
    }
    HIPCHK(launch_cg_xr(c->d_ch, c->nch, xa, c->d_part, c->st));
    if (fuse && it + 1 < maxiter) {
      HIPCHK(launch_cg_reduce_ctl(c->d_part, c->d_ch_begin, c->nblk, c->d_cgs,
                                  c->h_cgm + ((it + 1) % CG_RING), it + 1, ncol, c->st));
      HIPCHK(hipEventRecord(c->ev_cg[(it + 1) % CG_RING], c->st));
    } else {
      CHK(reduce_dev(c, MAXC, c->d_ch_begin, identity_map(), c->d_rhonew));
    }
    if (pre) {
      ++executed;
      if (passes) *passes += npass;
      continue;
    }
    // the stop test of `it` (its first kernel) decides whether it did any work
    CHK(event_spin(c, c->ev_cg[it % CG_RING]));
    last = slot;
    if (!last->any) {
      while (c->pending.size() > np0) {   // no-op passes: not timed, not counted
        c->evpool.push_back(c->pending.back().first);
        c->evpool.push_back(c->pending.back().second);
        c->pending.pop_back();
        c->pending_wide.pop_back();
      }
      c->ld_launches = cnt0[0];
      c->ld_bytes = cnt0[1];
      c->dense_bytes = cnt0[2];
      c->rhs_bytes = cnt0[3];
      c->aux_bytes = cnt0[4];
      c->ld_flops = cnt0[5];
      c->ld_flops_wide = cnt0[6];
      c->ld_launches_wide = cnt0[7];
      break;
    }
    ++executed;
    if (passes) *passes += npass;
    mask = 0;
    for (int j = 0; j < ncol; ++j)
      if (last->active[j]) mask |= 1u << j;
  }
  if (executed == maxiter) {  // for-loop exhausted (iterative.py:420-422)
    CgState* slot = c->h_cgm + (maxiter % CG_RING);
    HIPCHK(launch_cg_ctl(c->d_cgs, slot, c->d_rhonew, maxiter, ncol, maxiter, c->st));
    HIPCHK(hipEventRecord(c->ev_cg[maxiter % CG_RING], c->st));
    CHK(event_spin(c, c->ev_cg[maxiter % CG_RING]));
    last = slot;
  }
  for (int j = 0; j < ncol; ++j) {
    iters[j] = last->iters[j];
    info[j] = last->info[j];
  }
  return SGV_OK;
}

static int cg_run(sgv_ctx* c, const CgCols& cc, double* rho, const double* atol, int maxiter,
                  const int* active, int* iters, int* info, int* passes) {
  if (c->cg_pipe) return cg_loop_dev(c, cc, rho, atol, maxiter, active, iters, info, passes);
  return cg_loop(c, cc, rho, atol, maxiter, active, iters, info, passes);
}

// ---------------------------------------------------------------------------
// denoiser (src/sgvamp.py:93-114, 270-291)
// ---------------------------------------------------------------------------
// denoiser kernel + the ordered reduction of its derivative sums into h_tot[0..K);
// metrics: the four metrics sums of the new xhat1 (sgv_metrics) in the same
// reduction, h_tot[K .. K + 3] (one exchange instead of two with a communicator;
// not with more than MAXK cohorts) -- returns whether they were fused
static int denoise_enqueue(sgv_ctx* c, const double* gam1s, const double* a, double lam,
                           int nslab, const double* omegas, const double* sigmas, double rho,
                           int damp, bool metrics = false, bool* fused = nullptr) {
  DenoiseArgs da{};
  da.xhat1 = c->xhat1;
  da.nslab = nslab;
  da.lam = lam;
  da.rho = rho;
  da.damp = damp;
  da.write_x = 1;
  for (int k = 0; k < c->K; ++k) {
    const double ag = a[k] * gam1s[k];                 // self.a * gam1s
    da.sum_ag = (k == 0) ? ag : da.sum_ag + ag;        // builtin sum (:95)
  }
  for (int l = 0; l < nslab; ++l) {
    da.omegas[l] = omegas[l];
    da.sigmas[l] = sigmas[l];
    da.s2[l] = 1.0 / (da.sum_ag + 1.0 / sigmas[l]);     // :95
    da.sq[l] = std::sqrt(da.s2[l] / sigmas[l]);         // np.sqrt(sigma2_meta / sigmas)
  }
  // more than MAXK cohorts: groups of MAXK.  np.inner over all of them first
  // (one sequential sum continued group to group), then one launch per group
  // for its cohorts' derivative sums; the first also writes xhat1
  const int ng = (c->K + MAXK - 1) / MAXK;
  auto group = [&](int g) {
    da.K = std::min(MAXK, c->K - g * MAXK);
    for (int k = 0; k < da.K; ++k) {
      const int kk = g * MAXK + k;
      da.r1[k] = c->r1[kk];
      da.a[k] = a[kk];
      da.gam1[k] = gam1s[kk];
      da.ag[k] = a[kk] * gam1s[kk];
    }
  };
  if (ng > 1) {
    CHK(grow(c, &c->d_inner, &c->inner_cap, (size_t)std::max<int64_t>(c->Mpad, 1)));
    for (int g = 0; g < ng; ++g) {
      group(g);
      HIPCHK(launch_den_inner(c->d_ch, c->nch, da, c->d_inner, g == 0 ? 1 : 0, c->st));
    }
    da.inner = c->d_inner;
  }
  const bool met = metrics && ng == 1;
  if (fused) *fused = met;
  for (int g = 0; g < ng; ++g) {
    group(g);
    da.write_x = g == 0 ? 1 : 0;
    da.x0 = met ? c->x0 : nullptr;
    HIPCHK(launch_denoise(c->d_ch, c->nch, da, c->d_part, c->st));
    CHK(reduce_dev(c, da.K + (met ? 4 : 0), c->d_ch_begin, identity_map(), c->h_tot + g * MAXK));
  }
  return SGV_OK;
}

extern "C" int sgv_denoise(sgv_ctx* c, const double* gam1s, const double* a, double lam,
                           int nslab, const double* omegas, const double* sigmas, double rho,
                           int damp, double* der_sum) {
  ENTER(c);
  if (nslab < 1 || nslab > MAXL || !gam1s || !a || !omegas || !sigmas || !der_sum)
    return fail(c, SGV_ERR_ARG, "sgv_denoise: bad arguments (nslab=%d)", nslab);
  CHK(denoise_enqueue(c, gam1s, a, lam, nslab, omegas, sigmas, rho, damp));
  CHK(stream_wait(c));
  resolve_timers(c);
  for (int k = 0; k < c->K; ++k) der_sum[k] = c->h_tot[k];
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// EM prior loop (src/sgvamp.py:116-136, 250-257)
// ---------------------------------------------------------------------------
extern "C" int sgv_em(sgv_ctx* c, const double* gam1s, const double* a, int nslab,
                      const double* sigmas, int maxit, double* lam_io, double* omegas_io,
                      int* steps_out, double* final_err_out) {
  ENTER(c);
  if (nslab < 1 || nslab > MAXL || !gam1s || !a || !sigmas || !lam_io || !omegas_io)
    return fail(c, SGV_ERR_ARG, "sgv_em: bad arguments");
  // more than MAXK cohorts: one k_em launch per group of MAXK, the later ones
  // adding to the first's partials (each marker's cohort sum then runs group
  // by group); np.average's weight sum covers all cohorts
  const int ngr = (c->K + MAXK - 1) / MAXK;
  std::vector<EmArgs> eg(ngr);
  EmArgs& ea = eg[0];
  double scl = 0.0;
  for (int k = 0; k < c->K; ++k) scl = (k == 0) ? a[0] : scl + a[k];
  for (int g = 0; g < ngr; ++g) {
    EmArgs& e = eg[g];
    e = EmArgs{};
    e.K = std::min(MAXK, c->K - g * MAXK);
    e.nslab = nslab;
    for (int k = 0; k < e.K; ++k) {
      e.r1[k] = c->r1[g * MAXK + k];
      e.a[k] = a[g * MAXK + k];
      e.gam1[k] = gam1s[g * MAXK + k];
    }
    e.scl = scl;
    e.accum = g > 0 ? 1 : 0;
    for (int l = 0; l < nslab; ++l) e.sigmas[l] = sigmas[l];
    e.tab = c->d_emtab + (size_t)g * MAXK * EM_TAB;
    HIPCHK(launch_em_prep(e, c->d_emtab + (size_t)g * MAXK * EM_TAB, c->st));
  }
  auto em_groups = [&](const ChunkDesc* ch, int nch, double* part) -> int {
    for (int g = 0; g < ngr; ++g) HIPCHK(launch_em(ch, nch, eg[g], part, c->st));
    return SGV_OK;
  };
  double lam = *lam_io;
  double om[MAXL];
  for (int l = 0; l < nslab; ++l) om[l] = omegas_io[l];
  if (c->cg_pipe && maxit > 0) {
    // Device loop: k_em reads lam/omegas from the device state, k_em_ctl updates
    // it and tests convergence; step it + 1 is enqueued before the host waits
    // for step it's test, so the GPU does not idle for a host round trip per
    // step (one no-op step runs past the last).  Every rank enqueues the same
    // steps (the stop decision is made from the same global sums).
    EmState* hi = c->h_emi;   // the previous loop's init copy has completed
    std::memset(hi, 0, sizeof(EmState));
    hi->lam = lam;
    for (int l = 0; l < nslab; ++l) hi->om[l] = om[l];
    HIPCHK(hipMemcpyAsync(c->d_ems, hi, sizeof(EmState), hipMemcpyHostToDevice, c->st));
    for (EmArgs& e : eg) e.st = c->d_ems;
    // one rank: reduction + control in one launch (k_em_reduce_ctl, same bits).
    // With a communicator: the replicated EM (em_rep_setup) runs the same
    // one-rank loop over every rank's gathered r1.
    const bool rep = em_mode_pick(c, maxit);
    const bool fuse = rep || (!c->comm && !c->host_ag && fused_ctl_pays(EM_NV, c->nblk));
    hipEvent_t em0, em1;   // the loop on the device: its r1 gather to its last step
    CHK(event_pair(c, &em0, &em1));
    HIPCHK(hipEventRecord(em0, c->st));
    const ChunkDesc* ech = rep ? c->d_chg : c->d_ch;
    const int* ebeg = rep ? c->d_chg_begin : c->d_ch_begin;
    const int enb = rep ? c->nblkg : c->nblk, ench = rep ? c->nchg : c->nch;
    double* epart = rep ? c->d_partg : c->d_part;
    if (rep) {
      CHK(gather_r1(c));
      for (int k = 0; k < c->K; ++k) ea.r1[k] = c->d_r1g + (size_t)k * c->mpad_max;
    }
    auto enqueue = [&](int j) -> int {
      if (fuse) {
        CHK(em_groups(ech, ench, epart));
        const EmCtl f{ebeg, enb, nslab, c->h_emm + j % CG_RING, (double)c->Mtot, j, maxit};
        HIPCHK(launch_em_reduce_ctl(epart, c->d_ems, f, c->st));
        HIPCHK(hipEventRecord(c->ev_em[j % CG_RING], c->st));
        return SGV_OK;
      }
      CHK(em_groups(c->d_ch, c->nch, c->d_part));
      CHK(reduce_dev(c, EM_NV, c->d_ch_begin, identity_map(), c->d_emtot));
      HIPCHK(launch_em_ctl(c->d_ems, c->h_emm + j % CG_RING, c->d_emtot, nslab, (double)c->Mtot,
                           j, maxit, c->st));
      HIPCHK(hipEventRecord(c->ev_em[j % CG_RING], c->st));
      return SGV_OK;
    };
    CHK(enqueue(0));
    const volatile EmState* last = nullptr;
    for (int it = 0; it < maxit; ++it) {
      if (it + 1 < maxit) CHK(enqueue(it + 1));
      CHK(event_spin(c, c->ev_em[it % CG_RING]));
      last = c->h_emm + it % CG_RING;
      if (last->done) {
        HIPCHK(hipEventRecord(em1, c->st));   // behind the one step queued past the last
        c->empending.push_back({em0, em1});
        em0 = em1 = nullptr;
        break;
      }
    }
    if (em0) {   // maxit reached without convergence: the loop ends with its last step
      HIPCHK(hipEventRecord(em1, c->st));
      c->empending.push_back({em0, em1});
    }
    *lam_io = last->lam;
    for (int l = 0; l < nslab; ++l) omegas_io[l] = last->om[l];
    if (steps_out) *steps_out = last->steps;
    if (final_err_out) *final_err_out = last->err;
    c->em_prev_steps = last->steps;   // the same on every rank
    return SGV_OK;
  }
  double om_err = 0.0, lam_err = 0.0;
  int steps = 0;
  for (int it = 0; it < maxit; ++it) {
    for (EmArgs& e : eg) {
      e.lam = lam;
      for (int l = 0; l < nslab; ++l) e.omegas[l] = om[l];
    }
    CHK(em_groups(c->d_ch, c->nch, c->d_part));
    double tot[EM_NV];
    CHK(reduce_host(c, EM_NV, c->d_ch_begin, tot));
    const double lam_new = tot[0] / (double)c->Mtot;   // np.mean (:134)
    double om_new[MAXL];
    double dn = 0.0, on = 0.0;
    for (int l = 0; l < nslab; ++l) {
      om_new[l] = tot[1 + l] / tot[1 + nslab];         // :136
      const double d = om_new[l] - om[l];
      dn += d * d;
      on += om[l] * om[l];
    }
    om_err = std::sqrt(dn) / std::sqrt(on);            // :254
    lam_err = std::fabs(lam_new - lam) / lam_new;      // :255
    lam = lam_new;
    for (int l = 0; l < nslab; ++l) om[l] = om_new[l];
    steps = it + 1;
    if (om_err < 1e-6 && lam_err < 1e-6) break;        // :256
  }
  *lam_io = lam;
  for (int l = 0; l < nslab; ++l) omegas_io[l] = om[l];
  if (steps_out) *steps_out = steps;
  if (final_err_out) *final_err_out = std::max(om_err, lam_err);
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// LMMSE (src/sgvamp.py:301-364)
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// MLE prior update (src/sgvamp.py:139-194): the K x M x L sums of
// Lagrangian_der on the device; fsolve (MINPACK hybrd) stays on the host
// ---------------------------------------------------------------------------
// cohort group g (MAXK cohorts from g * MAXK)
static int mle_args(sgv_ctx* c, const double* gam1s, int L, const double* sigma2, int g,
                    MleArgs* m) {
  if (!gam1s || !sigma2 || L < 1 || L > MAXL + 1) return fail(c, SGV_ERR_ARG, "bad MLE arguments");
  *m = MleArgs{};
  m->K = std::min(MAXK, c->K - g * MAXK);
  m->L = L;
  for (int k = 0; k < m->K; ++k) {
    m->r1[k] = c->r1[g * MAXK + k];
    m->ginv[k] = 1.0 / gam1s[g * MAXK + k];                 // :146
  }
  for (int l = 0; l < L; ++l) m->sigma2[l] = sigma2[l];
  return SGV_OK;
}

extern "C" int sgv_mle_exp_max(sgv_ctx* c, const double* gam1s, int L, const double* sigma2,
                               double* exp_max) {
  ENTER(c);
  if (!exp_max) return fail(c, SGV_ERR_ARG, "exp_max is null");
  // :152: max over (k, m, l) of (-r1^2 / 2) / v_kl, attained at min_m r1_km^2
  double best = -std::numeric_limits<double>::infinity();
  for (int g = 0; g * MAXK < c->K; ++g) {
    MleArgs m;
    CHK(mle_args(c, gam1s, L, sigma2, g, &m));
    HIPCHK(launch_mle_minsq(c->d_ch, c->nch, m, c->d_part, c->st));
    double mn[MAXK];
    CHK(reduce_host(c, MAXK, c->d_ch_begin, mn, /*op=min*/ 1));
    for (int k = 0; k < m.K; ++k)
      for (int l = 0; l < L; ++l) best = std::max(best, -mn[k] / 2.0 / (m.sigma2[l] + m.ginv[k]));
  }
  *exp_max = best;
  return SGV_OK;
}

extern "C" int sgv_mle_terms(sgv_ctx* c, const double* a, const double* gam1s, int L,
                             const double* sigma2, const double* omega, double exp_max,
                             double* sums) {
  ENTER(c);
  if (!a || !omega || !sums) return fail(c, SGV_ERR_ARG, "bad MLE arguments");
  // one launch per cohort group; the groups' totals are added in group order
  for (int g = 0; g * MAXK < c->K; ++g) {
    MleArgs m;
    CHK(mle_args(c, gam1s, L, sigma2, g, &m));
    for (int k = 0; k < m.K; ++k) m.a[k] = a[g * MAXK + k];
    for (int l = 0; l < L; ++l) m.omega[l] = omega[l];
    m.exp_max = exp_max;
    HIPCHK(launch_mle_terms(c->d_ch, c->nch, m, c->d_part, c->st));
    double tot[MAXL + 1];
    CHK(reduce_host(c, MAXL + 1, c->d_ch_begin, tot));
    for (int l = 0; l < L; ++l) sums[l] = g == 0 ? tot[l] : sums[l] + tot[l];
  }
  return SGV_OK;
}

// The MLE prior update, src/sgvamp.py:162-194, with scipy's fsolve restated in
// hybrd.cpp; each function evaluation is one device pass over the r1 vectors
// (sgv_mle_terms), the rest the reference's host arithmetic in its order.
struct MleFn {
  sgv_ctx* c;
  const double* gam1s;
  const double* a;
  int L;
  const double* sigma2;
  const double* omega0;
  double exp_max;
  int rc;
  // the sums of the last evaluation and the omega they were taken at: the
  // Jacobian's gam column (x[L] perturbed) has the same omega, so its sums are
  // these, bitwise (the device sums are deterministic)
  double S[MAXL + 1], Sx[MAXL + 1];
  bool have_s;
};

// Lagrangian_der (:159-160) from the sums S at omega = x[:L]
static void mle_residual(const MleFn& f, const double* x, const double* S, double* y) {
  const int L = f.L;
  const double gam = x[L];
  for (int l = 0; l < L; ++l) y[l] = (S[l] + (f.omega0[l] - 1.0) / x[l]) + gam;   // :159
  double sw = 0.0;                                                                   // :160
  for (int l = 0; l < L; ++l) sw += x[l];
  y[L] = sw - 1.0;
}

static int mle_lagrangian(void* user, int n, const double* x, double* y) {
  MleFn& f = *(MleFn*)user;
  const int L = f.L;
  f.rc = sgv_mle_terms(f.c, f.a, f.gam1s, L, f.sigma2, x, f.exp_max, f.S);   // omega = x[:L]
  if (f.rc != SGV_OK) return -1;
  std::memcpy(f.Sx, x, sizeof(double) * L);
  f.have_s = true;
  mle_residual(f, x, f.S, y);
  (void)n;
  return 0;
}

// the forward-difference Jacobian's n = L + 1 points (hybrd's fdjac1): the L
// omega columns' device sums enqueued back to back with one host wait instead
// of one per point, the gam column from the base point's sums.  One cohort
// group, one rank (the host exchange waits per reduction anyway); otherwise
// point by point.  Each point's sums are the same launches as mle_lagrangian's,
// so the Jacobian is bitwise the per-point one.
static int mle_jacobian(void* user, int n, const double* x, const double* h, double* F) {
  MleFn& f = *(MleFn*)user;
  sgv_ctx* c = f.c;
  const int L = f.L;
  double xj[MAXL + 2];
  const bool base = f.have_s && std::memcmp(f.Sx, x, sizeof(double) * L) == 0;
  if (c->K > MAXK || c->comm || c->host_ag) {
    for (int j = 0; j < n; ++j) {
      std::memcpy(xj, x, sizeof(double) * n);
      xj[j] = x[j] + h[j];
      if (mle_lagrangian(user, n, xj, F + (size_t)j * n) < 0) return -1;
    }
    return 0;
  }
  f.rc = [&]() -> int {
    ENTER(c);
    MleArgs m;
    CHK(mle_args(c, f.gam1s, L, f.sigma2, 0, &m));
    for (int k = 0; k < m.K; ++k) m.a[k] = f.a[k];
    m.exp_max = f.exp_max;
    for (int j = 0; j < L; ++j) {
      for (int l = 0; l < L; ++l) m.omega[l] = l == j ? x[l] + h[l] : x[l];
      HIPCHK(launch_mle_terms(c->d_ch, c->nch, m, c->d_part, c->st));
      CHK(reduce_dev(c, MAXL + 1, c->d_ch_begin, identity_map(), c->h_tot + j * (MAXL + 1)));
    }
    CHK(stream_wait(c));
    resolve_timers(c);
    return SGV_OK;
  }();
  if (f.rc != SGV_OK) return -1;
  double base_s[MAXL + 1];
  if (base) std::memcpy(base_s, f.S, sizeof(double) * L);
  for (int j = 0; j < L; ++j) {
    std::memcpy(xj, x, sizeof(double) * n);
    xj[j] = x[j] + h[j];
    std::memcpy(f.S, c->h_tot + j * (MAXL + 1), sizeof(double) * L);
    std::memcpy(f.Sx, xj, sizeof(double) * L);
    mle_residual(f, xj, f.S, F + (size_t)j * n);
  }
  // the gam column: omega = x[:L], the base point's sums
  std::memcpy(xj, x, sizeof(double) * n);
  xj[L] = x[L] + h[L];
  if (base) {
    std::memcpy(f.S, base_s, sizeof(double) * L);
    std::memcpy(f.Sx, x, sizeof(double) * L);
    mle_residual(f, xj, f.S, F + (size_t)L * n);
    return 0;
  }
  return mle_lagrangian(user, n, xj, F + (size_t)L * n);
}

extern "C" int sgv_mle_update(sgv_ctx* c, const double* gam1s, const double* a, int nslab,
                              const double* sigmas, double* lam_io, double* omegas_io,
                              double* gam_io, int* status_out) {
  ENTER(c);
  if (!gam1s || !a || !sigmas || !lam_io || !omegas_io || !gam_io || !status_out ||
      nslab < 1 || nslab > MAXL)
    return fail(c, SGV_ERR_ARG, "sgv_mle_update: bad arguments");
  const int L = nslab + 1;
  double omega0[MAXL + 1], sigma2[MAXL + 1], x[MAXL + 2];
  omega0[0] = 1 - *lam_io;                                        // :166-168
  for (int l = 0; l < nslab; ++l) omega0[1 + l] = *lam_io * omegas_io[l];
  sigma2[0] = 1e-16;                                              // :169-171
  for (int l = 0; l < nslab; ++l) sigma2[1 + l] = sigmas[l];
  for (int l = 0; l < L; ++l) x[l] = omega0[l];                   // :173-178
  x[L] = std::isnan(*gam_io) ? 1.0 : *gam_io;
  MleFn f{c, gam1s, a, L, sigma2, omega0, 0.0, SGV_OK, {}, {}, false};
  CHK(sgv_mle_exp_max(c, gam1s, L, sigma2, &f.exp_max));           // :152, once per update
  // :179 (the forward-difference Jacobian's points batched, mle_jacobian)
  const int ier = sgv_fsolve_jac(L + 1, mle_lagrangian, mle_jacobian, &f, x, nullptr, nullptr);
  if (f.rc != SGV_OK) return f.rc;
  if (ier != 1) {                                                 // :181-184
    *status_out = SGV_MLE_NOT_CONVERGED;
    return SGV_OK;
  }
  for (int l = 0; l < L; ++l)
    if (x[l] <= 0) {                                              // :185-188
      *status_out = SGV_MLE_NEGATIVE;
      return SGV_OK;
    }
  double sw = 0.0;                                                // :190 x[:-1] /= sum(x[:-1])
  for (int l = 0; l < L; ++l) sw += x[l];
  for (int l = 0; l < L; ++l) x[l] = x[l] / sw;
  *lam_io = 1 - x[0];                                             // :191
  double ss = 0.0;                                                // :192 w / sum(x[1:-1])
  for (int l = 1; l < L; ++l) ss += x[l];
  for (int l = 0; l < nslab; ++l) omegas_io[l] = x[1 + l] / ss;
  *gam_io = x[L];                                                 // :193
  *status_out = 0;
  return SGV_OK;
}

// LMMSE of the cohorts g0 .. g0 + Kg - 1 (Kg <= MAXKG: 2 Kg <= MAXC CG columns,
// one batched CG loop); per-cohort inputs/outputs are the group's slices
static int lmmse_group(sgv_ctx* c, int g0, int Kg, const double* gamw, const double* gam2,
                       const double* alpha1, const double* alpha2_prev, int cg_maxit, double rtol,
                       int lmmse_damp, double rho, int learn_gamw, double* out, int* cg_out,
                       int* passes_out) {
  const int K = Kg, ncol = 2 * K;
  const double s = c->s;
  int passes = 0;

  // warm start needs R_s x0: carried from the previous iteration (rs_rec), or the
  // previous gamw pass; a pass only when X was set from outside
  for (int ld = 0; ld < c->nld; ++ld) {
    PassArgs pa{};
    int nc = 0;
    for (int j = 0; j < ncol; ++j) {
      if (!c->xnz[2 * g0 + j] || c->rx0_valid[2 * g0 + j] || c->ld_of[g0 + (j / 2)] != ld) continue;
      pa.in[nc] = c->X[2 * g0 + j];
      pa.out[nc] = c->RX0[2 * g0 + j];
      pa.dot[nc] = nullptr;
      pa.c1[nc] = 1.0 - s;
      pa.c2[nc] = s;
      ++nc;
      c->rx0_valid[2 * g0 + j] = 1;
    }
    if (nc) {
      CHK(ld_pass(c, ld, nc, pa));
      ++passes;
    }
  }

  // r2, mu2, r0 = b - A x0, p0 = r0 (:305-313, iterative.py:376-392)
  InitArgs ia{};
  ia.xhat1 = c->xhat1;
  ia.K = K;
  ia.save_x0 = lmmse_damp;
  for (int k = 0; k < K; ++k) {
    ia.cp.r[k] = c->r[g0 + k];
    ia.cp.r1[k] = c->r1[g0 + k];
    ia.cp.r2[k] = c->r2[g0 + k];
    ia.cp.u[k] = c->U[g0 + k];
    ia.alpha1[k] = alpha1[k];
    ia.gamw[k] = gamw[k];
    ia.gam2[k] = gam2[k];
  }
  for (int j = 0; j < ncol; ++j) {
    ia.col.X[j] = c->X[2 * g0 + j];
    ia.col.X0[j] = c->X0[2 * g0 + j];
    ia.col.Rr[j] = c->Rr[2 * g0 + j];
    ia.col.P[j] = c->P[2 * g0 + j];
    ia.col.Q[j] = c->Q[2 * g0 + j];
    ia.col.RX0[j] = c->RX0[2 * g0 + j];
    ia.col.RXp[j] = c->rs_rec ? c->RXp[2 * g0 + j] : nullptr;
    ia.warm[j] = c->xnz[2 * g0 + j];
  }
  double tot[2 * MAXC];
  const bool dev_init = c->cg_pipe;   // CG prologue on the device: no host round trip
  // with a communicator and one LD matrix for the group's columns: the prologue's
  // sums share iteration 0's exchange (cg_loop_dev, CgMerge0)
  bool one_ld = true;
  for (int k = 1; k < K; ++k) one_ld &= c->ld_of[g0 + k] == c->ld_of[g0];
  const bool merge0 = dev_init && (c->comm || c->host_ag) && one_ld;
  if (merge0) CHK(grow(c, &c->d_part2, &c->part2_cap, (size_t)c->nch * 2 * MAXC));
  HIPCHK(launch_lmmse_init(c->d_ch, c->nch, ia, merge0 ? c->d_part2 : c->d_part, c->st));
  CgMerge0 mg;
  if (merge0) {
    mg.part = c->d_part2;
    mg.rtol = rtol;
    mg.X = c->X.data() + 2 * g0;
    mg.RX = c->RX0.data() + 2 * g0;
  } else if (dev_init) {
    CHK(reduce_dev(c, 2 * MAXC, c->d_ch_begin, identity_map(), c->d_tot));
    HIPCHK(launch_cg_init(c->d_cgs, c->d_tot, rtol, ncol, c->d_ch, c->nch, c->X.data() + 2 * g0,
                          c->RX0.data() + 2 * g0, c->st));
  } else {
    CHK(reduce_host(c, 2 * MAXC, c->d_ch_begin, tot));
  }
  // carried: RX0 follows X through the CG; otherwise the gamw pass refreshes it
  for (int j = 0; j < ncol; ++j) c->rx0_valid[2 * g0 + j] = c->rs_rec ? 1 : 0;

  CgCols cc;
  cc.ncol = ncol;
  double rhov[MAXC], atol[MAXC];
  int active[MAXC], iters[MAXC], info[MAXC];
  for (int j = 0; j < ncol; ++j) {
    const int k = j / 2;
    cc.col_ld[j] = c->ld_of[g0 + k];
    cc.c1[j] = gamw[k] * (1.0 - s);           // A = gamw R_s + gam2 I (:312)
    cc.c2[j] = gamw[k] * s + gam2[k];
    cc.X[j] = c->X[2 * g0 + j];
    cc.Rr[j] = c->Rr[2 * g0 + j];
    cc.P[j] = c->P[2 * g0 + j];
    cc.Q[j] = c->Q[2 * g0 + j];
    if (c->rs_rec) {
      cc.RX[j] = c->RX0[2 * g0 + j];
      cc.Y[j] = c->Y[2 * g0 + j];
    }
    active[j] = 1;
    if (dev_init) continue;                   // k_cg_init
    const double bn = std::sqrt(tot[j]);      // bnrm2 (iterative.py:376)
    atol[j] = std::max(0.0, rtol * bn);
    rhov[j] = tot[MAXC + j];
    if (bn == 0.0) {                          // iterative.py:380-381: return b
      HIPCHK(hipMemsetAsync(c->X[2 * g0 + j], 0, sizeof(double) * c->Mpad, c->st));
      HIPCHK(hipMemsetAsync(c->RX0[2 * g0 + j], 0, sizeof(double) * c->Mpad, c->st));   // R_s 0
      active[j] = 0;
    }
  }
  cc.s = s;
  CHK(dev_init ? cg_loop_dev(c, cc, nullptr, nullptr, cg_maxit, active, iters, info, &passes,
                             merge0 ? &mg : nullptr)
               : cg_run(c, cc, rhov, atol, cg_maxit, active, iters, info, &passes));

  // damping, u.Sigma2_u, xhat2.r, x.any() (:322-323, 338, 352)
  PostArgs po{};
  po.K = K;
  po.damp = lmmse_damp;
  po.rs = c->rs_rec;
  po.rho = rho;
  for (int j = 0; j < ncol; ++j) {
    po.X[j] = c->X[2 * g0 + j];
    po.X0[j] = c->X0[2 * g0 + j];
    po.RX[j] = c->RX0[2 * g0 + j];
    po.RXp[j] = c->RXp[2 * g0 + j];
  }
  for (int k = 0; k < K; ++k) {
    po.u[k] = c->U[g0 + k];
    po.r[k] = c->r[g0 + k];
  }
  HIPCHK(launch_lmmse_post(c->d_ch, c->nch, po, c->d_part, c->st));
  double pt[4 * MAXKG + MAXC];
  R1Args ra{};
  ra.K = K;
  if (dev_init) {
    // r1 takes alpha2 from the device-reduced Tr(Sigma2): the update is queued
    // before the host reads the sums (which it computes alpha2 from as well)
    CHK(reduce_dev(c, 4 * MAXKG + MAXC, c->d_ch_begin, identity_map(), c->d_tot));
    ra.trs = c->d_tot;
    ra.Mtot = (double)c->Mtot;
    ra.rho = rho;
    ra.damp = lmmse_damp;
    for (int k = 0; k < K; ++k) {
      ra.X[k] = c->X[2 * g0 + (2 * k)];
      ra.r2[k] = c->r2[g0 + k];
      ra.r1[k] = c->r1[g0 + k];
      ra.gam2[k] = gam2[k];
      ra.alpha2_prev[k] = alpha2_prev[k];
    }
    HIPCHK(launch_r1_update(c->d_ch, c->nch, ra, c->st));   // :348
    HIPCHK(launch_copy_f64(c->h_tot, c->d_tot, 4 * MAXKG + MAXC, c->st));
    CHK(stream_wait(c));
    resolve_timers(c);
    std::memcpy(pt, c->h_tot, sizeof(pt));
  } else {
    CHK(reduce_host(c, 4 * MAXKG + MAXC, c->d_ch_begin, pt));
  }
  for (int j = 0; j < ncol; ++j) c->xnz[2 * g0 + j] = pt[2 * MAXKG + j] > 0.0;

  for (int k = 0; k < K; ++k) {
    const double TrSigma2 = pt[k];
    double a2 = gam2[k] * TrSigma2 / (double)c->Mtot;              // :340
    if (lmmse_damp) a2 = rho * a2 + (1 - rho) * alpha2_prev[k];    // :345-346
    const double g1 = gam2[k] * (1 - a2) / a2;                    // :347
    double* o = out + (size_t)k * SGV_LMMSE_NOUT;
    o[SGV_O_TRSIGMA2] = TrSigma2;
    o[SGV_O_ALPHA2] = a2;
    o[SGV_O_GAM1] = g1;
    o[SGV_O_XR] = pt[MAXKG + k];
    o[SGV_O_Z] = 0.0;
    o[SGV_O_TRRSIGMA2] = 0.0;
    o[SGV_O_XRX] = 0.0;
    o[SGV_O_GAMW] = gamw[k];
    ra.X[k] = c->X[2 * g0 + (2 * k)];
    ra.r2[k] = c->r2[g0 + k];
    ra.r1[k] = c->r1[g0 + k];
    ra.alpha2[k] = a2;
    cg_out[4 * k + 0] = iters[2 * k];
    cg_out[4 * k + 1] = info[2 * k];
    cg_out[4 * k + 2] = iters[2 * k + 1];
    cg_out[4 * k + 3] = info[2 * k + 1];
  }
  if (!dev_init) HIPCHK(launch_r1_update(c->d_ch, c->nch, ra, c->st));   // :348

  if (learn_gamw && c->rs_rec) {  // :350-363 from the carried products: no pass
    for (int k = 0; k < K; ++k) {
      const double N = c->Ncoh[g0 + k];
      double* o = out + (size_t)k * SGV_LMMSE_NOUT;
      const double xRx = pt[2 * MAXKG + MAXC + k];
      const double TrRSigma2 = pt[3 * MAXKG + MAXC + k];
      double z = N - 2 * o[SGV_O_XR] + xRx;                        // :352
      if (z < 0) z = 0;                                            // :353-354
      o[SGV_O_Z] = z;
      o[SGV_O_XRX] = xRx;
      o[SGV_O_TRRSIGMA2] = TrRSigma2;
      o[SGV_O_GAMW] = 1 / (z / N + TrRSigma2 / N);                 // :363
    }
  } else if (learn_gamw) {  // :350-363; R_s [xhat2, Sigma2_u] is also the next warm start's R_s x0
    for (int ld = 0; ld < c->nld; ++ld) {
      PassArgs pa{};
      Map16 map = identity_map();
      int nc = 0;
      for (int j = 0; j < ncol; ++j) {
        const int k = j / 2;
        if (c->ld_of[g0 + k] != ld) continue;
        pa.in[nc] = c->X[2 * g0 + j];
        pa.out[nc] = c->RX0[2 * g0 + j];
        pa.dot[nc] = (j % 2 == 0) ? c->X[2 * g0 + j] : c->U[g0 + k];
        pa.c1[nc] = 1.0 - s;
        pa.c2[nc] = s;
        map.d[nc] = j;
        ++nc;
        c->rx0_valid[2 * g0 + j] = 1;
      }
      if (!nc) continue;
      CHK(ld_pass(c, ld, nc, pa));
      ++passes;
      double gt[MAXC];
      CHK(reduce_dev(c, nc, ld_parts(c, ld), map, c->h_tot));
      CHK(stream_wait(c));
      resolve_timers(c);
      std::memcpy(gt, c->h_tot, sizeof(double) * ncol);
      for (int k = 0; k < K; ++k) {
        if (c->ld_of[g0 + k] != ld) continue;
        const double N = c->Ncoh[g0 + k];
        double* o = out + (size_t)k * SGV_LMMSE_NOUT;
        const double xRx = gt[2 * k];
        const double TrRSigma2 = gt[2 * k + 1];
        double z = N - 2 * o[SGV_O_XR] + xRx;                      // :352
        if (z < 0) z = 0;                                          // :353-354
        o[SGV_O_Z] = z;
        o[SGV_O_XRX] = xRx;
        o[SGV_O_TRRSIGMA2] = TrRSigma2;
        o[SGV_O_GAMW] = 1 / (z / N + TrRSigma2 / N);               // :363
      }
    }
  } else {
    CHK(stream_wait(c));
  }
  if (passes_out) *passes_out = passes;
  return SGV_OK;
}

extern "C" int sgv_lmmse(sgv_ctx* c, int it, const double* gamw, const double* gam2,
                         const double* alpha1, const double* alpha2_prev, const int8_t* probes,
                         int cg_maxit, double rtol, int lmmse_damp, double rho, int learn_gamw,
                         double* out, int* cg_out, int* passes_out) {
  ENTER(c);
  (void)it;
  if (!gamw || !gam2 || !alpha1 || !alpha2_prev || !probes || !out || !cg_out || cg_maxit < 0)
    return fail(c, SGV_ERR_ARG, "sgv_lmmse: bad arguments");
  const int K = c->K;

  // probes u_k (:326), int8 +-1 -> f64; uploaded at the start of sgv_step, or now
  int ps = c->pref_slot;
  if (ps < 0 || c->pref_src != probes) CHK(probe_upload(c, probes, &ps));
  c->pref_slot = -1;
  c->pref_src = nullptr;
  HIPCHK(hipStreamWaitEvent(c->st, c->ev_probe[ps], 0));
  for (int k = 0; k < K; ++k)
    HIPCHK(launch_unpack_i8(c->d_ch, c->nch, c->d_ch_doff,
                            c->d_probe + ps * c->probe_cap + (size_t)k * c->Mloc, c->U[k], c->st));
  HIPCHK(hipEventRecord(c->ev_unpk[ps], c->st));

  // cohorts in groups of MAXKG (2 MAXKG = MAXC CG columns per LD pass): the
  // LMMSE of a cohort touches only its own vectors and the shared xhat1, so the
  // groups run one after another with the same per-cohort arithmetic
  int passes = 0;
  for (int g0 = 0; g0 < K; g0 += MAXKG) {
    const int Kg = std::min(MAXKG, K - g0);
    int gp = 0;
    CHK(lmmse_group(c, g0, Kg, gamw + g0, gam2 + g0, alpha1 + g0, alpha2_prev + g0, cg_maxit, rtol,
                    lmmse_damp, rho, learn_gamw, out + (size_t)g0 * SGV_LMMSE_NOUT, cg_out + 4 * g0,
                    &gp));
    passes += gp;
  }
  if (passes_out) *passes_out = passes;
  return SGV_OK;
}

extern "C" int sgv_metrics(sgv_ctx* c, double* out4) {
  ENTER(c);
  if (!out4) return fail(c, SGV_ERR_ARG, "out4 is null");
  HIPCHK(launch_metrics(c->d_ch, c->nch, c->xhat1, c->x0, c->d_part, c->st));
  return reduce_host(c, 4, c->d_ch_begin, out4);
}

// The same sums, queued without a host wait (xhat1 and x0 are not written
// again before sgv_metrics_end); the ordered totals land in pinned memory.
// With the host exchange the reduction itself waits, so begin completes it.
extern "C" int sgv_metrics_begin(sgv_ctx* c) {
  ENTER(c);
  if (!c->h_met) {
    HIPCHK(hipHostMalloc(&c->h_met, sizeof(double) * 4, hipHostMallocCoherent));
    HIPCHK(hipEventCreateWithFlags(&c->ev_met, hipEventDisableTiming));
  }
  HIPCHK(launch_metrics(c->d_ch, c->nch, c->xhat1, c->x0, c->d_part, c->st));
  CHK(reduce_dev(c, 4, c->d_ch_begin, identity_map(), c->h_met));
  HIPCHK(hipEventRecord(c->ev_met, c->st));
  c->met_pending = 1;
  return SGV_OK;
}

extern "C" int sgv_metrics_end(sgv_ctx* c, double* out4) {
  ENTER(c);
  if (!out4) return fail(c, SGV_ERR_ARG, "out4 is null");
  if (!c->met_pending) return fail(c, SGV_ERR_ARG, "sgv_metrics_end without sgv_metrics_begin");
  hipError_t e;
  while ((e = hipEventQuery(c->ev_met)) == hipErrorNotReady) __builtin_ia32_pause();
  if (e != hipSuccess) return fail(c, SGV_ERR_HIP, "metrics wait: %s", hipGetErrorString(e));
  std::memcpy(out4, c->h_met, sizeof(double) * 4);
  c->met_pending = 0;
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// operator seam (tests): R_s v and a batched CG on (c1 R_s + c2 I)
// ---------------------------------------------------------------------------
extern "C" int sgv_ld_matvec(sgv_ctx* c, int ld, int ncol, const double* v, double* y) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || ncol < 1 || ncol > MAXC || !v || !y)
    return fail(c, SGV_ERR_ARG, "sgv_ld_matvec: bad arguments");
  PassArgs pa{};
  for (int j = 0; j < ncol; ++j) {
    CHK(upload_vec(c, v + (size_t)j * c->Mloc, c->S[j]));
    pa.in[j] = c->S[j];
    pa.out[j] = c->S[MAXC + j];
    pa.dot[j] = nullptr;
    pa.c1[j] = 1.0 - c->s;
    pa.c2[j] = c->s;
  }
  CHK(ld_pass(c, ld, ncol, pa));
  for (int j = 0; j < ncol; ++j) CHK(download_vec(c, c->S[MAXC + j], y + (size_t)j * c->Mloc));
  resolve_timers(c);
  return SGV_OK;
}

extern "C" int sgv_cg_solve(sgv_ctx* c, int ld, int ncol, const double* c1, const double* c2,
                            const double* b, double* x, int maxiter, double rtol, int* iters_out,
                            int* info_out) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || ncol < 1 || ncol > MAXC || !c1 || !c2 || !b || !x ||
      !iters_out || !info_out || maxiter < 0)
    return fail(c, SGV_ERR_ARG, "sgv_cg_solve: bad arguments");
  double* SB[MAXC];
  CgCols cc;
  cc.ncol = ncol;
  int warm[MAXC];
  for (int j = 0; j < ncol; ++j) {
    SB[j] = c->S[j];
    cc.X[j] = c->S[MAXC + j];
    cc.Rr[j] = c->S[2 * MAXC + j];
    cc.P[j] = c->S[3 * MAXC + j];
    cc.Q[j] = c->S[4 * MAXC + j];
    cc.col_ld[j] = ld;
    cc.c1[j] = c1[j] * (1.0 - c->s);
    cc.c2[j] = c1[j] * c->s + c2[j];
    CHK(upload_vec(c, b + (size_t)j * c->Mloc, SB[j]));
    CHK(upload_vec(c, x + (size_t)j * c->Mloc, cc.X[j]));
    warm[j] = host_any(x + (size_t)j * c->Mloc, c->Mloc);
  }
  // r = b - A x0 if x0.any() else b (iterative.py:392)
  PassArgs pa{};
  int nc = 0;
  AxpbyArgs ax{};
  for (int j = 0; j < ncol; ++j) {
    HIPCHK(hipMemcpyAsync(cc.Rr[j], SB[j], sizeof(double) * c->Mpad, hipMemcpyDeviceToDevice, c->st));
    ax.y[j] = cc.Rr[j];
    ax.x[j] = cc.Q[j];
    ax.a[j] = 1.0;
    ax.b[j] = warm[j] ? -1.0 : 0.0;
    if (!warm[j]) continue;
    pa.in[nc] = cc.X[j];
    pa.out[nc] = cc.Q[j];
    pa.dot[nc] = nullptr;
    pa.c1[nc] = cc.c1[j];
    pa.c2[nc] = cc.c2[j];
    ++nc;
  }
  ax.ncol = ncol;
  if (nc) CHK(ld_pass(c, ld, nc, pa));
  // map back: the pass wrote Q for warm columns in order; non-warm Q unused (b = 0 weight)
  HIPCHK(launch_axpby(c->d_ch, c->nch, ax, c->st));
  DotsArgs da{};
  da.ncol = 2 * ncol;
  for (int j = 0; j < ncol; ++j) {
    da.x[j] = SB[j];
    da.y[j] = SB[j];
    da.x[ncol + j] = cc.Rr[j];
    da.y[ncol + j] = cc.Rr[j];
    HIPCHK(hipMemcpyAsync(cc.P[j], cc.Rr[j], sizeof(double) * c->Mpad, hipMemcpyDeviceToDevice,
                          c->st));
  }
  if (2 * ncol > MAXC) return fail(c, SGV_ERR_ARG, "sgv_cg_solve: ncol <= %d", MAXC / 2);
  HIPCHK(launch_dots(c->d_ch, c->nch, da, c->d_part, c->st));
  double tot[MAXC];
  CHK(reduce_host(c, MAXC, c->d_ch_begin, tot));
  double rho[MAXC], atol[MAXC];
  int active[MAXC];
  for (int j = 0; j < ncol; ++j) {
    const double bn = std::sqrt(tot[j]);
    atol[j] = std::max(0.0, rtol * bn);
    rho[j] = tot[ncol + j];
    active[j] = 1;
    if (bn == 0.0) {
      HIPCHK(hipMemcpyAsync(cc.X[j], SB[j], sizeof(double) * c->Mpad, hipMemcpyDeviceToDevice, c->st));
      active[j] = 0;
    }
  }
  CHK(cg_run(c, cc, rho, atol, maxiter, active, iters_out, info_out, nullptr));
  for (int j = 0; j < ncol; ++j) CHK(download_vec(c, cc.X[j], x + (size_t)j * c->Mloc));
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// one outer iteration in the shim (src/sgvamp.py:222-387 minus the files and
// logs): the host returns to the caller once, not between the phases
// ---------------------------------------------------------------------------
static int step_impl(sgv_ctx* c, int it, int flags, int em_maxit, int nslab,
                     const double* sigmas, const double* a, double* lam_io, double* omegas_io,
                     const double* gam1s, double rho, const double* gamw,
                     const double* alpha1_prev, const double* alpha2_prev,
                     const int8_t* probes, int cg_maxit, double rtol, int out_slot,
                     double* res, int* ires, double* out, int* cg_out, int staged) {
  if (!sigmas || !a || !lam_io || !omegas_io || !gam1s || !gamw || !alpha1_prev ||
      !alpha2_prev || !probes || !res || !ires || !out || !cg_out || out_slot >= NOUT_SLOTS)
    return fail(c, SGV_ERR_ARG, "sgv_step: bad arguments");
  const int K = c->K;
  c->chain.valid = 0;   // a step chained behind this one fails unless this one completes
  res[0] = 0.0;
  ires[0] = 0;
  // this step's probes go up now, behind nothing: the copy overlaps EM/denoiser
  // (a step begun behind another had its host copy made by sgv_step_begin)
  if (staged >= 0) CHK(probe_issue(c, staged, &c->pref_slot));
  else CHK(probe_upload(c, probes, &c->pref_slot));
  c->pref_src = probes;
  if (flags & SGV_STEP_EM) {   // :250-257
    CHK(sgv_em(c, gam1s, a, nslab, sigmas, em_maxit, lam_io, omegas_io, &ires[0], &res[0]));
  } else if (flags & SGV_STEP_MLE) {   // :244-247
    CHK(sgv_mle_update(c, gam1s, a, nslab, sigmas, lam_io, omegas_io, &c->mle_gam, &ires[0]));
    res[0] = c->mle_gam;
  }
  if (nslab < 1 || nslab > MAXL) return fail(c, SGV_ERR_ARG, "sgv_step: nslab=%d", nslab);
  // denoiser (:270-291); the output copies and metrics (:281-283, 379-387) are
  // queued behind it before the host waits for the derivative sums
  bool met_fused = false;
  CHK(denoise_enqueue(c, gam1s, a, *lam_io, nslab, omegas_io, sigmas, rho,
                      (flags & SGV_STEP_DENOISE_DAMP) ? 1 : 0, (flags & SGV_STEP_METRICS) != 0,
                      &met_fused));
  HIPCHK(hipEventRecord(c->ev_den, c->st));
  if (out_slot >= 0) CHK(sgv_outputs_begin(c, out_slot));
  if ((flags & SGV_STEP_METRICS) && !met_fused) CHK(sgv_metrics_begin(c));
  CHK(event_spin(c, c->ev_den));
  std::vector<double> der(c->h_tot, c->h_tot + K), alpha1(K), gam2(K);
  if (met_fused)   // the metrics' ordered sums (sgv_metrics order), long done
    for (int j = 0; j < 4; ++j) res[1 + 2 * K + j] = c->h_tot[K + j];
  for (int k = 0; k < K; ++k) {
    double a1 = der[k] / (double)c->Mtot;                           // np.mean (:285)
    if (flags & SGV_STEP_ALPHA1_DAMP) a1 = rho * a1 + (1 - rho) * alpha1_prev[k];   // :290-291
    alpha1[k] = a1;
    gam2[k] = gam1s[k] * (1 - a1) / a1;                             // :305
    res[1 + k] = a1;
    res[1 + K + k] = gam2[k];
  }
  int passes = 0;
  CHK(sgv_lmmse(c, it, gamw, gam2.data(), alpha1.data(), alpha2_prev, probes, cg_maxit, rtol,
                (flags & SGV_STEP_LMMSE_DAMP) ? 1 : 0, rho, (flags & SGV_STEP_LEARN_GAMW) ? 1 : 0,
                out, cg_out, &passes));
  ires[1] = passes;
  if ((flags & SGV_STEP_METRICS) && !met_fused) CHK(sgv_metrics_end(c, res + 1 + 2 * K));
  // inputs of a chained next step: src/sgvamp.py:347, 363-374 (gamw clamped to
  // >= 1 after it is logged, as Python's max(gamw, 1.0))
  sgv_ctx::Chain& ch = c->chain;
  for (int k = 0; k < K; ++k) {
    const double* o = out + (size_t)k * SGV_LMMSE_NOUT;
    ch.gam1[k] = o[SGV_O_GAM1];
    const double gw = (flags & SGV_STEP_LEARN_GAMW) ? o[SGV_O_GAMW] : gamw[k];
    ch.gamw[k] = (1.0 > gw) ? 1.0 : gw;
    ch.alpha1[k] = alpha1[k];
    ch.alpha2[k] = o[SGV_O_ALPHA2];
  }
  ch.lam = *lam_io;
  for (int l = 0; l < nslab; ++l) ch.om[l] = omegas_io[l];
  ch.valid = 1;
  return SGV_OK;
}

extern "C" int sgv_step(sgv_ctx* c, int it, int flags, int em_maxit, int nslab,
                        const double* sigmas, const double* a, double* lam_io, double* omegas_io,
                        const double* gam1s, double rho, const double* gamw,
                        const double* alpha1_prev, const double* alpha2_prev,
                        const int8_t* probes, int cg_maxit, double rtol, int out_slot,
                        double* res, int* ires, double* out, int* cg_out) {
  ENTER(c);
  return step_impl(c, it, flags, em_maxit, nslab, sigmas, a, lam_io, omegas_io, gam1s, rho, gamw,
                   alpha1_prev, alpha2_prev, probes, cg_maxit, rtol, out_slot, res, ires, out,
                   cg_out, -1);
}

// Hand-offs spin (a futex wake costs tens of microseconds, the GPU idles for
// it): the worker spins up to ~2 ms for the next step before it blocks, and
// sgv_step_end spins for the step it waits on.  Steps run in begin order.
static void worker_main(sgv_ctx* c) {
  (void)hipSetDevice(c->dev);
  for (;;) {
    sgv_ctx::Job& j = c->jobs[c->job_run % 2];
    const auto t0 = std::chrono::steady_clock::now();
    while (j.state.load(std::memory_order_acquire) != 1 && !c->worker_quit.load()) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
        std::unique_lock<std::mutex> lk(c->wmu);
        c->wcv.wait(lk, [&] { return j.state.load() == 1 || c->worker_quit.load(); });
      }
    }
    if (j.state.load(std::memory_order_acquire) != 1) return;   // quit
    j.state.store(2);
    j.rc = j.fn();
    ++c->job_run;
    j.state.store(3, std::memory_order_release);
  }
}

extern "C" int sgv_step_begin(sgv_ctx* c, int it, int flags, int em_maxit, int nslab,
                              const double* sigmas, const double* a, double* lam_io,
                              double* omegas_io, const double* gam1s, double rho,
                              const double* gamw, const double* alpha1_prev,
                              const double* alpha2_prev, const int8_t* probes, int cg_maxit,
                              double rtol, int out_slot, double* res, int* ires, double* out,
                              int* cg_out) {
  if (!c) return fail(nullptr, SGV_ERR_ARG, "null context");
  if (nslab < 1 || nslab > MAXL || !sigmas || !a || !gam1s || !gamw || !alpha1_prev ||
      !alpha2_prev || !lam_io || !omegas_io)
    return fail(c, SGV_ERR_ARG, "sgv_step_begin: bad arguments");
  sgv_ctx::Job& j = c->jobs[c->job_begun % 2];
  if (j.state.load() != 0) return fail(c, SGV_ERR_ARG, "sgv_step_begin: two steps already queued");
  // the K- and L-length inputs are copied (a chained step takes gam1, gamw,
  // alpha1, alpha2, lam and omegas from the step before it when it starts);
  // lam_io/omegas_io, probes and the outputs stay the caller's until sgv_step_end
  const int K = c->K;
  std::vector<double> v_sig(sigmas, sigmas + nslab), v_a(a, a + K), v_g1(gam1s, gam1s + K),
      v_gw(gamw, gamw + K), v_a1(alpha1_prev, alpha1_prev + K), v_a2(alpha2_prev, alpha2_prev + K);
  // the probes' host copy is made here, while the step ahead runs on the GPU,
  // so the worker starts this step with the device copy alone (the buffers
  // come from the first step's upload; until then the worker stages them)
  int staged = -1;
  if (probes && c->probe_cap.load(std::memory_order_acquire) >= std::max<size_t>((size_t)K * c->Mloc, 8)) {
    staged = probe_stage(c, probes);
    if (staged < 0) return SGV_ERR_HIP;
  }
  j.fn = [=]() mutable {
    if (flags & SGV_STEP_CHAIN) {
      const sgv_ctx::Chain& ch = c->chain;
      if (!ch.valid) return fail(c, SGV_ERR_ARG, "chained step without a completed step");
      for (int k = 0; k < K; ++k) {
        v_g1[k] = ch.gam1[k];
        v_gw[k] = ch.gamw[k];
        v_a1[k] = ch.alpha1[k];
        v_a2[k] = ch.alpha2[k];
      }
      *lam_io = ch.lam;
      for (int l = 0; l < nslab; ++l) omegas_io[l] = ch.om[l];
    }
    ENTER(c);
    return step_impl(c, it, flags & ~SGV_STEP_CHAIN, em_maxit, nslab, v_sig.data(), v_a.data(),
                     lam_io, omegas_io, v_g1.data(), rho, v_gw.data(), v_a1.data(), v_a2.data(),
                     probes, cg_maxit, rtol, out_slot, res, ires, out, cg_out, staged);
  };
  {
    std::lock_guard<std::mutex> lk(c->wmu);   // a worker about to block sees the job
    j.state.store(1, std::memory_order_release);
  }
  ++c->job_begun;
  if (!c->worker.joinable()) c->worker = std::thread(worker_main, c);
  c->wcv.notify_all();
  return SGV_OK;
}

extern "C" int sgv_step_end(sgv_ctx* c) {
  if (!c) return fail(nullptr, SGV_ERR_ARG, "null context");
  if (c->job_ended == c->job_begun) return fail(c, SGV_ERR_ARG, "sgv_step_end without sgv_step_begin");
  sgv_ctx::Job& j = c->jobs[c->job_ended % 2];
  while (j.state.load(std::memory_order_acquire) != 3) __builtin_ia32_pause();
  const int rc = j.rc;
  j.fn = nullptr;
  j.state.store(0);
  ++c->job_ended;
  return rc;
}
