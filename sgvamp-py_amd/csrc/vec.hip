// Marker-wise kernels of the sgVAMP outer iteration and the ordered reductions.
// Compiled with -ffp-contract=off so expressions round like the reference's
// NumPy code (one rounding per operation, reference operand order).
//
// Every kernel walks "chunks" (<= CHUNK markers inside one LD block) and writes
// one partial per chunk; launch_reduce_* turn those into per-block sums and
// the global total in block order (bitwise independent of the GPU count).
#include "common.h"

namespace sgv {

#define CHUNK_LOOP(ch)                                                  \
  for (int t = threadIdx.x; t < (ch).len; t += VTHREADS)

// Latency-bound vector kernels: a thread owns markers t, t + 256, t + 512,
// t + 768 of its chunk (the CHUNK_LOOP order, so every per-thread sum adds in
// the same order), and all of their loads are issued before the first store.
// Pointers taken from argument structs may alias as far as the compiler
// knows, so in a CHUNK_LOOP each store fences the next marker's loads: a chain
// of MPT x (columns) dependent HBM round trips (~24 us for k_cg_xr whatever M).
// Independent columns / cohorts run as grid.y, one per workgroup.
constexpr int MPT = CHUNK / VTHREADS;
static_assert(CHUNK % VTHREADS == 0, "markers per thread");

// one value summed over the workgroup like block_reduce_store (wave butterfly,
// waves 0..3 in order), stored by thread 0 at *out
template <int NV>
__device__ __forceinline__ void block_reduce_slots(double (&v)[NV], double* __restrict__ base,
                                                   const int (&slot)[NV]) {
  __shared__ double sm[VTHREADS / WAVE][NV];
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = wave_sum(v[k]);
    if (lane == 0) sm[wid][k] = s;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k)
    if ((int)threadIdx.x == k) base[slot[k]] = ((sm[0][k] + sm[1][k]) + sm[2][k]) + sm[3][k];
}

// block y == 0 of a chunk zeroes the partial slots whose owner (column or
// cohort) has no workgroup (owner >= n), as the one-workgroup-per-chunk kernels
// did by summing zeros
template <class F>
__device__ __forceinline__ void zero_unowned(double* __restrict__ base, int nv, int n, F owner) {
  if (blockIdx.y != 0) return;
  for (int t = threadIdx.x; t < nv; t += VTHREADS)
    if (owner(t) >= n) base[t] = 0.0;
}

// ---------------------------------------------------------------------------
// denoiser_meta + der_denoiser_meta, src/sgvamp.py:93-114, per marker (:273,285)
// ---------------------------------------------------------------------------
// KM: cohort bound of the instantiation (registers: vr holds MPT x KM values);
// partials [k] at stride K (+ 4 with the metrics: [K .. K + 3])
template <int KM>
__global__ __launch_bounds__(VTHREADS) void k_denoise(const ChunkDesc* __restrict__ chs,
                                                      DenoiseArgs a,
                                                      double* __restrict__ part) {
  const ChunkDesc ch = chs[blockIdx.x];
  const bool met = a.x0 != nullptr;   // uniform
  double acc[KM + 4];
#pragma unroll
  for (int k = 0; k < KM + 4; ++k) acc[k] = 0.0;
  // loads of the thread's MPT markers first (see MPT), then the markers in order
  double vr[MPT][KM], vxo[MPT], vx0[MPT];
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      const int64_t i = ch.voff + t;
      if (a.inner) {
        vr[j][0] = a.inner[i];
      } else {
#pragma unroll
        for (int k = 0; k < KM; ++k)
          if (k < a.K) vr[j][k] = a.r1[k][i];
      }
      if (a.damp && a.write_x) vxo[j] = a.xhat1[i];
      if (met) vx0[j] = a.x0[i];
    }
  }
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t >= ch.len) continue;
    const int64_t i = ch.voff + t;
    // np.inner(rs, a*gam1s) (:96)
    double inner = 0.0;
    if (a.inner) {
      inner = vr[j][0];
    } else {
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k < a.K) inner = (k == 0) ? vr[j][0] * a.ag[0] : inner + vr[j][k] * a.ag[k];
    }
    double mu[MAXL];
    int m = 0;
    double best = 0.0;
#pragma unroll
    for (int l = 0; l < MAXL; ++l)
      if (l < a.nslab) {
        mu[l] = inner * a.s2[l];
        const double ratio = mu[l] * mu[l] / a.s2[l];   // :97
        if (l == 0 || ratio > best) {                   // argmax: first maximum
          best = ratio;
          m = l;
        }
      }
    double s2m = a.s2[0], mum = mu[0];
#pragma unroll
    for (int l = 1; l < MAXL; ++l)
      if (l < a.nslab && l == m) {
        s2m = a.s2[l];
        mum = mu[l];
      }
    double EXP[MAXL];
    double sumN = 0.0, sumD = 0.0;
#pragma unroll
    for (int l = 0; l < MAXL; ++l)
      if (l < a.nslab) {
        EXP[l] = exp(0.5 * (mu[l] * mu[l] * s2m - mum * mum * a.s2[l]) / (a.s2[l] * s2m));  // :98
        const double tn = a.omegas[l] * EXP[l] * mu[l] * a.sq[l];                           // :99
        const double td = a.omegas[l] * EXP[l] * a.sq[l];                                   // :101
        sumN = (l == 0) ? tn : sumN + tn;
        sumD = (l == 0) ? td : sumD + td;
      }
    const double Num = a.lam * sumN;
    const double EXP2 = exp(-0.5 * (mum * mum / s2m));   // :100
    const double Den = (1 - a.lam) * EXP2 + a.lam * sumD;
    if (a.write_x) {
      double x = Num / Den;
      if (a.damp) x = a.rho * x + (1 - a.rho) * vxo[j];   // :275-276
      a.xhat1[i] = x;
      if (met) {   // k_metrics' sums of this marker, same order (:381-382)
        const double b = vx0[j], d = x - b;
        acc[KM + 0] += x * b;
        acc[KM + 1] += x * x;
        acc[KM + 2] += d * d;
        acc[KM + 3] += b * b;
      }
    }
    // der_denoiser_meta for every cohort k (:112-114 with a[k]*gam1s[k])
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < a.K) {
        double dn = 0.0, dd = 0.0;
#pragma unroll
        for (int l = 0; l < MAXL; ++l)
          if (l < a.nslab) {
            const double tn = a.omegas[l] * EXP[l] * (mu[l] * mu[l] + a.s2[l]) * a.a[k] *
                              a.gam1[k] * a.sq[l];
            const double td = a.omegas[l] * mu[l] * EXP[l] * a.a[k] * a.gam1[k] * a.sq[l];
            dn = (l == 0) ? tn : dn + tn;
            dd = (l == 0) ? td : dd + td;
          }
        const double DerNum = a.lam * dn;
        const double DerDen = a.lam * dd;
        acc[k] += (DerNum * Den - DerDen * Num) / (Den * Den);
      }
  }
  // the workgroup's sums as block_reduce_store (wave butterfly, waves in order):
  // derivative sum k -> slot k, metric j -> slot K + j
  {
    __shared__ double sm[VTHREADS / WAVE][KM + 4];
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
#pragma unroll
    for (int k = 0; k < KM + 4; ++k) {
      if (k >= KM ? !met : k >= a.K) continue;   // uniform
      const double s = wave_sum(acc[k]);
      if (lane == 0) sm[wid][k] = s;
    }
    __syncthreads();
    const int nv = a.K + (met ? 4 : 0);
    double* out = part + (int64_t)blockIdx.x * nv;
    const int t = threadIdx.x;
    if (t < nv) {
      const int k = t < a.K ? t : KM + (t - a.K);
      out[t] = ((sm[0][k] + sm[1][k]) + sm[2][k]) + sm[3][k];
    }
  }
}

hipError_t launch_denoise(const ChunkDesc* d_ch, int nch, const DenoiseArgs& a, double* d_part,
                          hipStream_t st) {
#define L_DEN(KM) hipLaunchKernelGGL(k_denoise<KM>, dim3(nch), dim3(VTHREADS), 0, st, d_ch, a, d_part)
  if (a.K < 1 || a.K > MAXK) return hipErrorInvalidValue;   // cohorts
  if (a.K <= 1) L_DEN(1);
  else if (a.K <= 2) L_DEN(2);
  else if (a.K <= 4) L_DEN(4);
  else if (a.K <= 8) L_DEN(8);
  else if (a.K <= 16) L_DEN(16);
  else L_DEN(MAXK);
#undef L_DEN
  return hipGetLastError();
}

__global__ __launch_bounds__(VTHREADS) void k_den_inner(const ChunkDesc* __restrict__ chs,
                                                        DenoiseArgs a, double* __restrict__ inner,
                                                        int first) {
  const ChunkDesc ch = chs[blockIdx.x];
  CHUNK_LOOP(ch) {
    const int64_t i = ch.voff + t;
    double s = first ? a.r1[0][i] * a.ag[0] : inner[i] + a.r1[0][i] * a.ag[0];
    for (int k = 1; k < a.K; ++k) s = s + a.r1[k][i] * a.ag[k];
    inner[i] = s;
  }
}

hipError_t launch_den_inner(const ChunkDesc* d_ch, int nch, const DenoiseArgs& a, double* inner,
                            int first, hipStream_t st) {
  if (a.K < 1 || a.K > MAXK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_den_inner, dim3(nch), dim3(VTHREADS), 0, st, d_ch, a, inner, first);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// prior_update_em, src/sgvamp.py:116-136 (one EM step)
// ---------------------------------------------------------------------------
// One workgroup per chunk with one marker per thread (EM_THREADS = CHUNK): the
// step is latency-bound (exp, sqrt and divisions per marker and slab), and
// four markers in sequence per thread made it 13-16 us at any M.  A thread's
// sums take its marker's K cohorts in order; the workgroup adds them by wave
// butterfly, then the 16 waves in order.  false: the device loop has stopped
// (no-op step; uniform over the grid).
constexpr int EM_THREADS = CHUNK;
template <int KM, int LM>
__device__ __forceinline__ bool em_partials(const ChunkDesc* __restrict__ chs, const EmArgs& a,
                                            double* __restrict__ part) {
  const ChunkDesc ch = chs[blockIdx.x];
  double lam = a.lam, om[MAXL];
#pragma unroll
  for (int l = 0; l < MAXL; ++l) om[l] = a.omegas[l];
  if (a.st) {   // device EM loop
    if (a.st->done) return false;
    lam = a.st->lam;
#pragma unroll
    for (int l = 0; l < MAXL; ++l) om[l] = a.st->om[l];
  }
  double acc[EM_NV];
#pragma unroll
  for (int v = 0; v < EM_NV; ++v) acc[v] = 0.0;
  const int t = threadIdx.x;
  __shared__ double tab[KM * EM_TAB];
  for (int q = t; q < a.K * EM_TAB; q += EM_THREADS) tab[q] = a.tab[q];
  __syncthreads();
  if (t < ch.len) {
    double vr[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < a.K) vr[k] = a.r1[k][ch.voff + t];
    double avg = 0.0;   // sum_k pi_k a_k (np.average numerator, sequential over k)
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < a.K) {
        const double r = vr[k];
        const double r2 = r * r;                  // np.power(r1s, 2)
        const double* tb = tab + k * EM_TAB;      // gam1invs and its sums/roots (k_em_prep)
        double tl[LM];
        double emax = 0.0;
#pragma unroll
        for (int l = 0; l < LM; ++l)
          if (l < a.nslab) {
            tl[l] = -r2 / 2 / tb[2 + l];                     // :127
            emax = (l == 0 || tl[l] > emax) ? tl[l] : emax;
          }
        double xi[LM];
        double sum_xi = 0.0;
#pragma unroll
        for (int l = 0; l < LM; ++l)
          if (l < a.nslab) {
            xi[l] = lam * om[l] * exp(tl[l] - emax) / tb[2 + MAXL + l];                 // :128
            sum_xi = (l == 0) ? xi[l] : sum_xi + xi[l];                                   // :129
          }
        const double pi =
            1.0 / (1.0 + (1 - lam) * exp(-r2 / 2 * a.gam1[k] - emax) / tb[1] / sum_xi);   // :131
        const double pa = pi * a.a[k];
        avg = (k == 0) ? pa : avg + pa;
        // compile-time accumulator indices (a runtime acc[1 + nslab] puts the
        // array in scratch memory)
#pragma unroll
        for (int v = 1; v < LM + 2; ++v) {
          const int l = v - 1;
          if (l < a.nslab)
            acc[v] += pi * (xi[l] / sum_xi) * a.a[k];   // :136 numerator
          else if (l == a.nslab)
            acc[v] += pa;                               // :136 denominator
        }
      }
    acc[0] += avg / a.scl;   // np.average(pi, axis=0, weights=a)  (:134)
  }
  __shared__ double sm[EM_THREADS / WAVE][EM_NV];
  const int lane = t & (WAVE - 1), w = t / WAVE;
#pragma unroll
  for (int v = 0; v < EM_NV; ++v) {
    const double x = wave_sum(acc[v]);
    if (lane == 0) sm[w][v] = x;
  }
  __syncthreads();
  if (t < EM_NV) {
    double x = sm[0][t];
#pragma unroll
    for (int q = 1; q < EM_THREADS / WAVE; ++q) x += sm[q][t];
    double* dst = part + (int64_t)blockIdx.x * EM_NV + t;
    *dst = a.accum ? *dst + x : x;
  }
  return true;
}

template <int KM, int LM>
__global__ __launch_bounds__(EM_THREADS) void k_em(const ChunkDesc* __restrict__ chs, EmArgs a,
                                                   double* __restrict__ part) {
  em_partials<KM, LM>(chs, a, part);
}

// instantiations by cohort / slab count (registers: the fully unrolled
// MAXK x MAXL body spills at 1024 threads)
#define EM_DISPATCH(K, L, LAUNCH)                                             \
  do {                                                                        \
    if ((K) <= 1 && (L) <= 2) { LAUNCH(1, 2); }                               \
    else if ((K) <= 4 && (L) <= 2) { LAUNCH(4, 2); }                          \
    else if ((K) <= 8 && (L) <= 2) { LAUNCH(8, 2); }                          \
    else if ((K) <= 4) { LAUNCH(4, MAXL); }                                   \
    else if ((K) <= 8) { LAUNCH(8, MAXL); }                                   \
    else if ((K) <= 16 && (L) <= 2) { LAUNCH(16, 2); }                        \
    else if ((K) <= 16) { LAUNCH(16, MAXL); }                                 \
    else if ((L) <= 2) { LAUNCH(MAXK, 2); }                                   \
    else { LAUNCH(MAXK, MAXL); }                                              \
  } while (0)

__global__ __launch_bounds__(WAVE) void k_em_prep(EmArgs a, double* __restrict__ tab) {
  for (int k = threadIdx.x; k < a.K; k += WAVE) {
    double* tb = tab + k * EM_TAB;
    const double ginv = 1.0 / a.gam1[k];      // gam1invs (:125)
    tb[0] = ginv;
    tb[1] = sqrt(ginv);                       // np.sqrt(gam1invs) (:131)
    for (int l = 0; l < MAXL; ++l) {
      tb[2 + l] = l < a.nslab ? a.sigmas[l] + ginv : 1.0;               // (:127)
      tb[2 + MAXL + l] = l < a.nslab ? sqrt(ginv + a.sigmas[l]) : 1.0;   // (:128)
    }
  }
}

hipError_t launch_em_prep(const EmArgs& a, double* tab, hipStream_t st) {
  if (a.K < 1 || a.K > MAXK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_em_prep, dim3(1), dim3(WAVE), 0, st, a, tab);
  return hipGetLastError();
}

hipError_t launch_em(const ChunkDesc* d_ch, int nch, const EmArgs& a, double* d_part,
                     hipStream_t st) {
  if (!a.tab) return hipErrorInvalidValue;
#define L_EM(KM, LM) \
  hipLaunchKernelGGL((k_em<KM, LM>), dim3(nch), dim3(EM_THREADS), 0, st, d_ch, a, d_part)
  EM_DISPATCH(a.K, a.nslab, L_EM);
#undef L_EM
  return hipGetLastError();
}

// the host loop's update and test (capi.hip sgv_em), same expressions in the
// same order: -ffp-contract=off and correctly rounded division and sqrt give
// the same bits, so the same step count.  One thread.
__device__ void em_ctl_update(EmState* __restrict__ s, EmState* mirror,
                              const double* __restrict__ tot, int nslab, double Mtot, int it,
                              int maxit) {
  if (!s->done) {
    const double lam = s->lam;
    const double lam_new = tot[0] / Mtot;                 // np.mean (:134)
    double om_new[MAXL];
    double dn = 0.0, on = 0.0;
    for (int l = 0; l < nslab; ++l) {
      om_new[l] = tot[1 + l] / tot[1 + nslab];            // :136
      const double d = om_new[l] - s->om[l];
      dn += d * d;
      on += s->om[l] * s->om[l];
    }
    const double om_err = sqrt(dn) / sqrt(on);            // :254
    const double lam_err = fabs(lam_new - lam) / lam_new; // :255
    s->lam = lam_new;
    for (int l = 0; l < nslab; ++l) s->om[l] = om_new[l];
    s->steps = it + 1;
    s->err = (om_err < lam_err) ? lam_err : om_err;       // std::max
    if ((om_err < 1e-6 && lam_err < 1e-6) || it + 1 >= maxit) s->done = 1;   // :256
  }
  if (mirror) {
    mirror->lam = s->lam;
    for (int l = 0; l < MAXL; ++l) mirror->om[l] = s->om[l];
    mirror->err = s->err;
    mirror->steps = s->steps;
    mirror->done = s->done;
  }
}

__global__ __launch_bounds__(WAVE) void k_em_ctl(EmState* __restrict__ s, EmState* mirror,
                                                const double* __restrict__ tot, int nslab,
                                                double Mtot, int it, int maxit) {
  if (threadIdx.x == 0) em_ctl_update(s, mirror, tot, nslab, Mtot, it, maxit);
}

hipError_t launch_em_ctl(EmState* d_st, EmState* mirror, const double* d_tot, int nslab,
                         double Mtot, int it, int maxit, hipStream_t st) {
  hipLaunchKernelGGL(k_em_ctl, dim3(1), dim3(WAVE), 0, st, d_st, mirror, d_tot, nslab, Mtot, it,
                     maxit);
  return hipGetLastError();
}

// ---- one-workgroup reduction + EM control (one rank) -----------------------
// k_reduce_local (nv workgroups) followed by k_em_ctl (one wave) cost two
// launches per EM step; here one 1024-thread workgroup forms all EM_NV totals
// exactly as k_reduce_local does -- per LD block b, lane l adds parts
// begin[b] + l, + 64, ... in order, wave butterfly; then the blocks in order --
// and applies the update and stop test.  Same bits, one launch less per step.
// (A last-workgroup-done epilogue in k_em itself was measured slower: each
// workgroup's device-scope release fence writes back the XCD's L2.)
// Waves take the (block, value) pairs LB_U at a time, all their loads first.
constexpr int LB_U = 8;

__device__ void lb_reduce(const double* __restrict__ part, int nv, const int* __restrict__ begin,
                          int nblk, double* bs /* LDS, nv * nblk */, double* tot /* LDS, nv */) {
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  const int nw = blockDim.x / WAVE, npairs = nv * nblk;
  for (int q0 = w * LB_U; q0 < npairs; q0 += nw * LB_U) {
    double s[LB_U];
#pragma unroll
    for (int u = 0; u < LB_U; ++u) {
      s[u] = 0.0;
      const int q = q0 + u;
      if (q < npairs) {
        const int b = q / nv, v = q - b * nv;
        const int p1 = begin[b + 1];
        for (int p = begin[b] + lane; p < p1; p += WAVE) s[u] += part[(int64_t)p * nv + v];
      }
    }
#pragma unroll
    for (int u = 0; u < LB_U; ++u) {
      const double t = wave_sum(s[u]);
      if (lane == 0 && q0 + u < npairs) bs[q0 + u] = t;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < nv) {
    const int v = threadIdx.x;
    double t = 0.0;
    for (int b = 0; b < nblk; ++b) t = (b == 0) ? bs[v] : t + bs[b * nv + v];
    tot[v] = t;
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void k_em_reduce_ctl(const double* __restrict__ part,
                                                        EmState* __restrict__ s, EmCtl f) {
  __shared__ double bs[EM_CTL_MAXBLK * EM_NV];
  __shared__ double tot[EM_NV];
  if (s->done) {   // past the stop (k_em was a no-op): mirror the state only
    if (threadIdx.x == 0) em_ctl_update(s, f.mirror, nullptr, f.nslab, f.Mtot, f.it, f.maxit);
    return;
  }
  lb_reduce(part, EM_NV, f.begin, f.nblk, bs, tot);
  if (threadIdx.x == 0) em_ctl_update(s, f.mirror, tot, f.nslab, f.Mtot, f.it, f.maxit);
}

hipError_t launch_em_reduce_ctl(const double* d_part, EmState* d_st, const EmCtl& f,
                                hipStream_t st) {
  if (f.nblk < 1 || f.nblk > EM_CTL_MAXBLK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_em_reduce_ctl, dim3(1), dim3(1024), 0, st, d_part, d_st, f);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// LMMSE set-up, src/sgvamp.py:305-313 + scipy cg prologue (iterative.py:375-392)
// partials: [c] = |b_c|^2, [MAXC + c] = |r0_c|^2
// ---------------------------------------------------------------------------
constexpr int INIT_NV = 2 * MAXC;
// grid (nch, K): workgroup (chunk, k) does cohort k's two columns 2k, 2k + 1
__global__ __launch_bounds__(VTHREADS) void k_lmmse_init(const ChunkDesc* __restrict__ chs,
                                                         InitArgs a,
                                                         double* __restrict__ part) {
  const ChunkDesc ch = chs[blockIdx.x];
  const int k = blockIdx.y;
  double* pb = part + (int64_t)blockIdx.x * INIT_NV;
  zero_unowned(pb, INIT_NV, a.K, [](int t) { return (t < MAXC ? t : t - MAXC) / 2; });
  const double* __restrict__ xh = a.xhat1;
  const double* __restrict__ r1 = a.cp.r1[k];
  const double* __restrict__ rk = a.cp.r[k];
  const double* __restrict__ uk = a.cp.u[k];
  double* __restrict__ r2o = a.cp.r2[k];
  const double al = a.alpha1[k], gw = a.gamw[k], g2 = a.gam2[k];
  const int c0 = 2 * k;
  const bool w0 = a.warm[c0], w1 = a.warm[c0 + 1];
  const bool sx = a.save_x0, sxr = sx && a.col.RXp[c0];
  double vx[MPT], vr1[MPT], vr[MPT], vu[MPT], vrx[2][MPT], vxc[2][MPT];
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      const int64_t i = ch.voff + t;
      vx[j] = xh[i];
      vr1[j] = r1[i];
      vr[j] = rk[i];
      vu[j] = uk[i];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool w = h ? w1 : w0;
        vrx[h][j] = (w || (h == 0 && sxr)) ? a.col.RX0[c0 + h][i] : 0.0;
        vxc[h][j] = (w || (h == 0 && sx)) ? a.col.X[c0 + h][i] : 0.0;
      }
    }
  }
  double acc[4] = {0.0, 0.0, 0.0, 0.0};   // |b_c|^2, |b_c+1|^2, |r0_c|^2, |r0_c+1|^2
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      const int64_t i = ch.voff + t;
      const double r2 = (vx[j] - al * vr1[j]) / (1 - al);   // :310
      r2o[i] = r2;
      const double b1 = gw * vr[j] + g2 * r2;               // :313
      const double b2 = vu[j];                              // :326
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = c0 + h;
        const double b = h == 0 ? b1 : b2;
        double r = b;
        if (h ? w1 : w0) {
          // r = b - A x0, A x0 = gamw (R_s x0) + gam2 x0 (:312; R_s x0 carried)
          const double ax = gw * vrx[h][j] + g2 * vxc[h][j];
          r = b - ax;
        }
        a.col.Rr[c][i] = r;
        a.col.P[c][i] = r;
        acc[h] += b * b;
        acc[2 + h] += r * r;
      }
      if (sx) {
        a.col.X0[c0][i] = vxc[0][j];
        if (sxr) a.col.RXp[c0][i] = vrx[0][j];
      }
    }
  }
  const int slot[4] = {c0, c0 + 1, MAXC + c0, MAXC + c0 + 1};
  block_reduce_slots<4>(acc, pb, slot);
}

hipError_t launch_lmmse_init(const ChunkDesc* d_ch, int nch, const InitArgs& a, double* d_part,
                             hipStream_t st) {
  if (a.K < 1 || a.K > MAXKG) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_lmmse_init, dim3(nch, a.K), dim3(VTHREADS), 0, st, d_ch, a, d_part);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// CG update (iterative.py:412-415): alpha = rho / (p.q); x += alpha p;
// r -= alpha q; partial rho_new = r.r  (partials [c], stride MAXC)
// ---------------------------------------------------------------------------
// grid (nch, ncol): workgroup (chunk, c) updates column c
__global__ __launch_bounds__(VTHREADS) void k_cg_xr(const ChunkDesc* __restrict__ chs, XrArgs a,
                                                    double* __restrict__ part) {
  const ChunkDesc ch = chs[blockIdx.x];
  const int c = blockIdx.y;
  double* pb = part + (int64_t)blockIdx.x * MAXC;
  bool on = (a.mask >> c) & 1u;
  double rc = a.rho[c];
  if (a.st) {   // device-side control: the columns still active after this iteration's test
    const int any = a.st->any, act = a.st->active[c];
    rc = a.st->rho[c];
    if (!any) return;   // no-op iteration (its r.r partials are never read)
    on = on && act;
  }
  zero_unowned(pb, MAXC, a.ncol, [](int t) { return t; });
  double acc[1] = {0.0};
  if (on) {
    const double alpha = rc / a.pq[c];
    double* __restrict__ X = a.X[c];
    double* __restrict__ Rr = a.Rr[c];
    double* __restrict__ RX = a.RX[c];
    const double* __restrict__ P = a.P[c];
    const double* __restrict__ Q = a.Q[c];
    const double* __restrict__ Y = a.Y[c];
    double vx[MPT], vp[MPT], vr[MPT], vq[MPT], vrx[MPT], vy[MPT];
#pragma unroll
    for (int j = 0; j < MPT; ++j) {
      const int t = threadIdx.x + j * VTHREADS;
      if (t < ch.len) {
        const int64_t i = ch.voff + t;
        vx[j] = X[i];
        vp[j] = P[i];
        vr[j] = Rr[i];
        vq[j] = Q[i];
        if (RX) {
          vrx[j] = RX[i];
          vy[j] = Y[i];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < MPT; ++j) {
      const int t = threadIdx.x + j * VTHREADS;
      if (t < ch.len) {
        const int64_t i = ch.voff + t;
        X[i] = vx[j] + alpha * vp[j];
        if (RX) RX[i] = vrx[j] + alpha * vy[j];   // R_s x carried
        const double r = vr[j] - alpha * vq[j];
        Rr[i] = r;
        acc[0] += r * r;
      }
    }
  }
  const int slot[1] = {c};
  block_reduce_slots<1>(acc, pb, slot);
}

hipError_t launch_cg_xr(const ChunkDesc* d_ch, int nch, const XrArgs& a, double* d_part,
                        hipStream_t st) {
  if (a.ncol < 1 || a.ncol > MAXC) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cg_xr, dim3(nch, a.ncol), dim3(VTHREADS), 0, st, d_ch, a, d_part);
  return hipGetLastError();
}

// p = beta p + r   (iterative.py:405-407: p *= beta; p += z); grid (nch, ncol)
__global__ __launch_bounds__(VTHREADS) void k_cg_p(const ChunkDesc* __restrict__ chs, PArgs a) {
  const ChunkDesc ch = chs[blockIdx.x];
  const int c = blockIdx.y;
  bool on = (a.mask >> c) & 1u;
  double beta = a.beta[c];
  if (a.st) {
    const int any = a.st->any, act = a.st->active[c];
    beta = a.st->beta[c];
    if (!any) return;
    on = on && act;
  }
  if (!on) return;
  double* __restrict__ P = a.P[c];
  const double* __restrict__ Rr = a.Rr[c];
  double vp[MPT], vr[MPT];
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      vp[j] = P[ch.voff + t];
      vr[j] = Rr[ch.voff + t];
    }
  }
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) P[ch.voff + t] = vp[j] * beta + vr[j];
  }
}

hipError_t launch_cg_p(const ChunkDesc* d_ch, int nch, const PArgs& a, hipStream_t st) {
  if (a.ncol < 1 || a.ncol > MAXC) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cg_p, dim3(nch, a.ncol), dim3(VTHREADS), 0, st, d_ch, a);
  return hipGetLastError();
}

// Device-side CG control, one wave (thread j = column j); same expressions
// as the host loop (correctly rounded sqrt and division: the same decisions
// and the same beta bit for bit).
// by one wave (lane j = column j)
__device__ __forceinline__ void cg_ctl_body(CgState* __restrict__ s, CgState* mirror,
                                            const double* rho_new, int it, int ncol, int final_it) {
  const int j = threadIdx.x;
  int act = 0;
  if (j < ncol) {
    act = s->active[j];
    if (final_it >= 0) {                     // for-loop exhausted (iterative.py:420-422)
      if (act) {
        s->iters[j] = final_it;
        s->info[j] = final_it;
      }
      act = 0;
    } else if (act) {
      if (it > 0) {                          // rho_prev = rho_cur; rho_cur = r.r (:412-415)
        s->rho_prev[j] = s->rho[j];
        s->rho[j] = rho_new[j];
      }
      if (sqrt(s->rho[j]) < s->atol[j]) {   // iterative.py:398 (strict <)
        act = 0;
        s->active[j] = 0;
        s->iters[j] = it;
        s->info[j] = 0;
      } else if (it > 0) {
        s->beta[j] = s->rho[j] / s->rho_prev[j];   // :405
      }
    }
  }
  const int any = __any(act) ? 1 : 0;
  if (j == 0) {
    s->any = any;
    s->it = it;
  }
  if (mirror && j < MAXC) {
    mirror->rho[j] = s->rho[j];
    mirror->active[j] = j < ncol ? (final_it >= 0 ? 0 : s->active[j]) : 0;
    mirror->iters[j] = s->iters[j];
    mirror->info[j] = s->info[j];
  }
  if (mirror && j == 0) {
    mirror->any = any;
    mirror->it = it;
  }
}

__global__ __launch_bounds__(WAVE) void k_cg_ctl(CgState* __restrict__ s, CgState* mirror,
                                                const double* __restrict__ rho_new, int it, int ncol,
                                                int final_it) {
  cg_ctl_body(s, mirror, rho_new, it, ncol, final_it);
}

// One rank: the r.r reduction of iteration it - 1 (k_cg_xr's partials, formed
// as k_reduce_local forms them) and the control of iteration it in one
// single-workgroup launch -- same bits as k_reduce_local + k_cg_ctl.
__global__ __launch_bounds__(1024) void k_cg_reduce_ctl(const double* __restrict__ part,
                                                        const int* __restrict__ begin, int nblk,
                                                        CgState* __restrict__ s, CgState* mirror,
                                                        int it, int ncol) {
  __shared__ double bs[EM_CTL_MAXBLK * MAXC];
  __shared__ double tot[MAXC];
  lb_reduce(part, MAXC, begin, nblk, bs, tot);
  if (threadIdx.x < WAVE) cg_ctl_body(s, mirror, tot, it, ncol, -1);
}

hipError_t launch_cg_reduce_ctl(const double* d_part, const int* d_begin, int nblk,
                                CgState* d_st, CgState* mirror, int it, int ncol,
                                hipStream_t st) {
  if (nblk < 1 || nblk > EM_CTL_MAXBLK || it < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cg_reduce_ctl, dim3(1), dim3(1024), 0, st, d_part, d_begin, nblk, d_st,
                     mirror, it, ncol);
  return hipGetLastError();
}

__global__ __launch_bounds__(WAVE) void k_cg_init(CgState* __restrict__ s,
                                                 const double* __restrict__ tot, double rtol,
                                                 int ncol) {
  const int j = threadIdx.x;
  int act = 0;
  if (j < MAXC) {
    double rho = 0.0, atol = 0.0;
    int zero = 0;
    if (j < ncol) {
      const double bn = sqrt(tot[j]);        // bnrm2 (iterative.py:376)
      const double v = rtol * bn;
      atol = (0.0 < v) ? v : 0.0;            // std::max(0.0, v)
      rho = tot[MAXC + j];
      zero = bn == 0.0;
      act = !zero;
    }
    s->rho[j] = rho;
    s->rho_prev[j] = 0.0;
    s->beta[j] = 0.0;
    s->atol[j] = atol;
    s->active[j] = act;
    s->iters[j] = 0;
    s->info[j] = 0;
    s->zero[j] = zero;
  }
  const int any = __any(act) ? 1 : 0;
  if (j == 0) {
    s->any = any;
    s->it = 0;
  }
}

struct ZeroCols {
  double* X[MAXC];
  double* RX[MAXC];
};
// grid (nch, ncol): X[c] = 0 and R_s X[c] = 0 where the state says |b_c| == 0
__global__ __launch_bounds__(VTHREADS) void k_cg_zero(const ChunkDesc* __restrict__ chs,
                                                     const CgState* __restrict__ s, ZeroCols z) {
  const int c = blockIdx.y;
  if (!s->zero[c]) return;
  const ChunkDesc ch = chs[blockIdx.x];
  CHUNK_LOOP(ch) {
    z.X[c][ch.voff + t] = 0.0;
    if (z.RX[c]) z.RX[c][ch.voff + t] = 0.0;
  }
}

hipError_t launch_cg_init(CgState* d_st, const double* d_tot, double rtol, int ncol,
                          const ChunkDesc* d_ch, int nch, double* const* X, double* const* RX,
                          hipStream_t st) {
  if (ncol < 1 || ncol > MAXC) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cg_init, dim3(1), dim3(WAVE), 0, st, d_st, d_tot, rtol, ncol);
  ZeroCols z{};
  for (int j = 0; j < ncol; ++j) {
    z.X[j] = X[j];
    z.RX[j] = RX[j];
  }
  hipLaunchKernelGGL(k_cg_zero, dim3(nch, ncol), dim3(VTHREADS), 0, st, d_ch, d_st, z);
  return hipGetLastError();
}

__global__ void k_copy_f64(double* dst, const double* __restrict__ src, int n) {
  const int t = threadIdx.x;
  if (t < n) dst[t] = src[t];
}
hipError_t launch_copy_f64(double* dst, const double* src, int n, hipStream_t st) {
  if (n < 1 || n > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_copy_f64, dim3(1), dim3(n), 0, st, dst, src, n);
  return hipGetLastError();
}

hipError_t launch_cg_ctl(CgState* d_st, CgState* mirror, const double* d_rho_new, int it, int ncol,
                         int final_it, hipStream_t st) {
  hipLaunchKernelGGL(k_cg_ctl, dim3(1), dim3(WAVE), 0, st, d_st, mirror, d_rho_new, it, ncol,
                     final_it);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// after both CG solves (src/sgvamp.py:322-338,352,359):
//   xhat2 damping; partials [k] = u.Sigma2_u, [MAXKG + k] = xhat2.r,
//   [2 MAXKG + c] = count(x_c != 0)  (next iteration's x0.any()),
//   with the carried products (rs): [2 MAXKG + MAXC + k] = xhat2.R_s xhat2,
//   [3 MAXKG + MAXC + k] = u.R_s Sigma2_u
// ---------------------------------------------------------------------------
constexpr int POST_NV = 4 * MAXKG + MAXC;
static_assert(POST_NV <= MAXNV, "post partials");
// grid (nch, K): workgroup (chunk, k) does cohort k
__global__ __launch_bounds__(VTHREADS) void k_lmmse_post(const ChunkDesc* __restrict__ chs,
                                                         PostArgs a,
                                                         double* __restrict__ part) {
  const ChunkDesc ch = chs[blockIdx.x];
  const int k = blockIdx.y;
  double* pb = part + (int64_t)blockIdx.x * POST_NV;
  zero_unowned(pb, POST_NV, a.K, [](int t) {
    return t < 2 * MAXKG ? t % MAXKG : t < 2 * MAXKG + MAXC ? (t - 2 * MAXKG) / 2 : (t - 2 * MAXKG - MAXC) % MAXKG;
  });
  double* __restrict__ X0 = a.X[2 * k];
  const double* __restrict__ X1 = a.X[2 * k + 1];
  const double* __restrict__ Xp = a.X0[2 * k];
  double* __restrict__ RX0 = a.RX[2 * k];
  const double* __restrict__ RX1 = a.RX[2 * k + 1];
  const double* __restrict__ RXp = a.RXp[2 * k];
  const double* __restrict__ U = a.u[k];
  const double* __restrict__ Rk = a.r[k];
  const bool damp = a.damp, rs = a.rs;
  const double rho = a.rho;
  double vx[MPT], vxp[MPT], vs[MPT], vu[MPT], vr[MPT], vrx[MPT], vrxp[MPT], vrx1[MPT];
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      const int64_t i = ch.voff + t;
      vx[j] = X0[i];
      vs[j] = X1[i];
      vu[j] = U[i];
      vr[j] = Rk[i];
      if (damp) vxp[j] = Xp[i];
      if (rs) {
        vrx[j] = RX0[i];
        vrx1[j] = RX1[i];
        if (damp) vrxp[j] = RXp[i];
      }
    }
  }
  // [u.S2u, x2.r, nnz x2, nnz S2u, x2.R_s x2, u.R_s S2u]
  double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      const int64_t i = ch.voff + t;
      double x2 = vx[j];
      if (damp) {
        x2 = rho * x2 + (1 - rho) * vxp[j];   // :322-323
        X0[i] = x2;
      }
      const double s2u = vs[j];
      const double uk = vu[j];
      acc[0] += uk * s2u;                       // :338
      acc[1] += x2 * vr[j];                     // :352
      if (rs) {
        double rx = vrx[j];
        if (damp) {                             // R_s is linear: damp with x
          rx = rho * rx + (1 - rho) * vrxp[j];
          RX0[i] = rx;
        }
        acc[4] += x2 * rx;                      // :352 xhat2^T R_s xhat2
        acc[5] += uk * vrx1[j];                 // :359 u^T R_s Sigma2_u
      }
      acc[2] += (x2 != 0.0) ? 1.0 : 0.0;
      acc[3] += (s2u != 0.0) ? 1.0 : 0.0;
    }
  }
  const int slot[6] = {k, MAXKG + k, 2 * MAXKG + 2 * k, 2 * MAXKG + 2 * k + 1, 2 * MAXKG + MAXC + k,
                       3 * MAXKG + MAXC + k};
  block_reduce_slots<6>(acc, pb, slot);
}

hipError_t launch_lmmse_post(const ChunkDesc* d_ch, int nch, const PostArgs& a, double* d_part,
                             hipStream_t st) {
  if (a.K < 1 || a.K > MAXKG) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_lmmse_post, dim3(nch, a.K), dim3(VTHREADS), 0, st, d_ch, a, d_part);
  return hipGetLastError();
}

// r1 = (xhat2 - alpha2 r2) / (1 - alpha2)   (src/sgvamp.py:348)
// grid (nch, K)
__global__ __launch_bounds__(VTHREADS) void k_r1_update(const ChunkDesc* __restrict__ chs,
                                                        R1Args a) {
  const ChunkDesc ch = chs[blockIdx.x];
  const int k = blockIdx.y;
  const double* __restrict__ X = a.X[k];
  const double* __restrict__ r2 = a.r2[k];
  double* __restrict__ r1 = a.r1[k];
  double al = a.alpha2[k];
  if (a.trs) {   // same expressions as the host's (capi.hip sgv_lmmse)
    al = a.gam2[k] * a.trs[k] / a.Mtot;                                   // :340
    if (a.damp) al = a.rho * al + (1 - a.rho) * a.alpha2_prev[k];         // :345-346
  }
  double vx[MPT], vr[MPT];
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      vx[j] = X[ch.voff + t];
      vr[j] = r2[ch.voff + t];
    }
  }
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) r1[ch.voff + t] = (vx[j] - al * vr[j]) / (1 - al);
  }
}

hipError_t launch_r1_update(const ChunkDesc* d_ch, int nch, const R1Args& a, hipStream_t st) {
  if (a.K < 1 || a.K > MAXKG) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_r1_update, dim3(nch, a.K), dim3(VTHREADS), 0, st, d_ch, a);
  return hipGetLastError();
}

// metrics (src/sgvamp.py:381-382): <x,x0>, |x|^2, |x-x0|^2, |x0|^2
__global__ __launch_bounds__(VTHREADS) void k_metrics(const ChunkDesc* __restrict__ chs,
                                                      const double* __restrict__ x,
                                                      const double* __restrict__ x0,
                                                      double* __restrict__ part) {
  const ChunkDesc ch = chs[blockIdx.x];
  double va[MPT], vb[MPT];
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      va[j] = x[ch.voff + t];
      vb[j] = x0[ch.voff + t];
    }
  }
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < MPT; ++j) {
    const int t = threadIdx.x + j * VTHREADS;
    if (t < ch.len) {
      const double a = va[j], b = vb[j], d = a - b;
      acc[0] += a * b;
      acc[1] += a * a;
      acc[2] += d * d;
      acc[3] += b * b;
    }
  }
  block_reduce_store<4>(acc, part + (int64_t)blockIdx.x * 4, 4);
}

hipError_t launch_metrics(const ChunkDesc* d_ch, int nch, const double* xhat1, const double* x0,
                          double* d_part, hipStream_t st) {
  hipLaunchKernelGGL(k_metrics, dim3(nch), dim3(VTHREADS), 0, st, d_ch, xhat1, x0, d_part);
  return hipGetLastError();
}

__global__ __launch_bounds__(VTHREADS) void k_dots(const ChunkDesc* __restrict__ chs, DotsArgs a,
                                                   double* __restrict__ part) {
  const ChunkDesc ch = chs[blockIdx.x];
  double acc[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) acc[c] = 0.0;
  CHUNK_LOOP(ch) {
    const int64_t i = ch.voff + t;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (c < a.ncol) acc[c] += a.x[c][i] * a.y[c][i];
  }
  block_reduce_store<MAXC>(acc, part + (int64_t)blockIdx.x * MAXC, MAXC);
}

hipError_t launch_dots(const ChunkDesc* d_ch, int nch, const DotsArgs& a, double* d_part,
                       hipStream_t st) {
  hipLaunchKernelGGL(k_dots, dim3(nch), dim3(VTHREADS), 0, st, d_ch, a, d_part);
  return hipGetLastError();
}

__global__ __launch_bounds__(VTHREADS) void k_axpby(const ChunkDesc* __restrict__ chs,
                                                    AxpbyArgs a) {
  const ChunkDesc ch = chs[blockIdx.x];
  CHUNK_LOOP(ch) {
    const int64_t i = ch.voff + t;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (c < a.ncol) a.y[c][i] = a.a[c] * a.y[c][i] + a.b[c] * a.x[c][i];
  }
}

hipError_t launch_axpby(const ChunkDesc* d_ch, int nch, const AxpbyArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_axpby, dim3(nch), dim3(VTHREADS), 0, st, d_ch, a);
  return hipGetLastError();
}

// dense <-> padded layout ----------------------------------------------------
__global__ __launch_bounds__(VTHREADS) void k_unpack(const ChunkDesc* __restrict__ chs,
                                                     const int64_t* __restrict__ doff,
                                                     const double* __restrict__ src,
                                                     double* __restrict__ dst) {
  const ChunkDesc ch = chs[blockIdx.x];
  const int64_t o = doff[blockIdx.x];
  CHUNK_LOOP(ch) dst[ch.voff + t] = src[o + t];
}
__global__ __launch_bounds__(VTHREADS) void k_unpack_i8(const ChunkDesc* __restrict__ chs,
                                                        const int64_t* __restrict__ doff,
                                                        const int8_t* __restrict__ src,
                                                        double* __restrict__ dst) {
  const ChunkDesc ch = chs[blockIdx.x];
  const int64_t o = doff[blockIdx.x];
  CHUNK_LOOP(ch) dst[ch.voff + t] = (double)src[o + t];
}
__global__ __launch_bounds__(VTHREADS) void k_pack(const ChunkDesc* __restrict__ chs,
                                                   const int64_t* __restrict__ doff,
                                                   const double* __restrict__ src,
                                                   double* __restrict__ dst) {
  const ChunkDesc ch = chs[blockIdx.x];
  const int64_t o = doff[blockIdx.x];
  CHUNK_LOOP(ch) dst[o + t] = src[ch.voff + t];
}

hipError_t launch_unpack(const ChunkDesc* d_ch, int nch, const int64_t* d_doff,
                         const double* src, double* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_unpack, dim3(nch), dim3(VTHREADS), 0, st, d_ch, d_doff, src, dst);
  return hipGetLastError();
}
hipError_t launch_unpack_i8(const ChunkDesc* d_ch, int nch, const int64_t* d_doff,
                            const int8_t* src, double* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_unpack_i8, dim3(nch), dim3(VTHREADS), 0, st, d_ch, d_doff, src, dst);
  return hipGetLastError();
}
hipError_t launch_pack(const ChunkDesc* d_ch, int nch, const int64_t* d_doff, const double* src,
                       double* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_pack, dim3(nch), dim3(VTHREADS), 0, st, d_ch, d_doff, src, dst);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ordered reductions
// ---------------------------------------------------------------------------
// grid (nblk, nv), one wave: bsum[b * ostride + ooff + v] = sum (op 0) or min
// (op 1) of parts [begin[b], begin[b+1])
__global__ __launch_bounds__(WAVE) void k_reduce_blocks(const double* __restrict__ part, int nv,
                                                        const int* __restrict__ begin,
                                                        double* __restrict__ bsum, int op,
                                                        int ostride, int ooff) {
  const int b = blockIdx.x, v = blockIdx.y, lane = threadIdx.x;
  const int p0 = begin[b], p1 = begin[b + 1];
  double* out = bsum + (int64_t)b * ostride + ooff + v;
  if (op == 0) {
    double s = 0.0;
    for (int p = p0 + lane; p < p1; p += WAVE) s += part[(int64_t)p * nv + v];
    s = wave_sum(s);
    if (lane == 0) *out = s;
  } else {
    double s = __builtin_inf();
    for (int p = p0 + lane; p < p1; p += WAVE) s = fmin(s, part[(int64_t)p * nv + v]);
    for (int o = 32; o > 0; o >>= 1) s = fmin(s, __shfl_xor(s, o, WAVE));
    if (lane == 0) *out = s;
  }
}

hipError_t launch_reduce_blocks(const double* d_part, int nv, const int* d_begin, int nblk,
                                double* d_bsum, hipStream_t st, int op, int ostride, int ooff) {
  hipLaunchKernelGGL(k_reduce_blocks, dim3(nblk, nv), dim3(WAVE), 0, st, d_part, nv, d_begin,
                     d_bsum, op, ostride > 0 ? ostride : nv, ooff);
  return hipGetLastError();
}

// total[v] = sum over ranks r, local blocks b < counts[r] (global block order)
__global__ void k_reduce_total(const double* __restrict__ bsum_all, int nranks, int nbmax, int nv,
                               const int* __restrict__ counts, Map16 map,
                               double* __restrict__ dst, int op) {
  const int v = threadIdx.x;
  if (v >= nv) return;
  double s = 0.0;
  bool first = true;
  for (int r = 0; r < nranks; ++r) {
    const int nb = counts[r];
    for (int b = 0; b < nb; ++b) {
      const double x = bsum_all[((int64_t)r * nbmax + b) * nv + v];
      s = first ? x : (op == 0 ? s + x : fmin(s, x));
      first = false;
    }
  }
  dst[map.d[v]] = s;
}

// One rank, no exchange: both steps in one launch.  Wave v computes every
// block's sum exactly as k_reduce_blocks does (same lane stride, same
// wave_sum) and folds them in block order exactly as k_reduce_total does, so
// the result is bitwise the two-kernel one.
// one rank: per-block sums (each by one wave, lanes strided over the block's
// parts, butterfly -- the order k_reduce_blocks uses) computed by 16 waves in
// parallel, then added in block order by one thread: the same sums as a
// single wave walking the blocks one after another, without its chain of
// nblk dependent loads (~42 us at 64 blocks)
constexpr int RL_WAVES = 16;
constexpr int RL_BATCH = 1024;
__global__ __launch_bounds__(WAVE * RL_WAVES) void k_reduce_local(
    const double* __restrict__ part, int nv, const int* __restrict__ begin, int nblk, Map16 map,
    double* __restrict__ dst, int op) {
  __shared__ double bs[RL_BATCH];
  const int v = blockIdx.x, lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  double tot = 0.0;
  for (int b0 = 0; b0 < nblk; b0 += RL_BATCH) {
    const int nb = min(RL_BATCH, nblk - b0);
    for (int bb = w; bb < nb; bb += RL_WAVES) {
      const int p0 = begin[b0 + bb], p1 = begin[b0 + bb + 1];
      double s;
      if (op == 0) {
        s = 0.0;
        for (int p = p0 + lane; p < p1; p += WAVE) s += part[(int64_t)p * nv + v];
        s = wave_sum(s);
      } else {
        s = __builtin_inf();
        for (int p = p0 + lane; p < p1; p += WAVE) s = fmin(s, part[(int64_t)p * nv + v]);
        for (int o = 32; o > 0; o >>= 1) s = fmin(s, __shfl_xor(s, o, WAVE));
      }
      if (lane == 0) bs[bb] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int bb = 0; bb < nb; ++bb) {
        const double s = bs[bb];
        tot = (b0 + bb == 0) ? s : (op == 0 ? tot + s : fmin(tot, s));
      }
    __syncthreads();
  }
  if (threadIdx.x == 0) dst[map.d[v]] = tot;
}

hipError_t launch_reduce_local(const double* d_part, int nv, const int* d_begin, int nblk,
                               const Map16& map, double* d_dst, hipStream_t st, int op) {
  hipLaunchKernelGGL(k_reduce_local, dim3(nv), dim3(WAVE * RL_WAVES), 0, st, d_part, nv, d_begin,
                     nblk, map, d_dst, op);
  return hipGetLastError();
}

hipError_t launch_reduce_total(const double* d_bsum_all, int nranks, int nbmax, int nv,
                               const int* d_counts, const Map16& map, double* d_dst,
                               hipStream_t st, int op) {
  hipLaunchKernelGGL(k_reduce_total, dim3(1), dim3(64), 0, st, d_bsum_all, nranks, nbmax, nv,
                     d_counts, map, d_dst, op);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// MLE prior update (src/sgvamp.py:139-160, Lagrangian_der)
// ---------------------------------------------------------------------------
// min over markers of r1_k^2 per cohort (partials [k], stride MAXK; min reduce).
// The reference's exp_max = max_{k,m,l} (-r1_km^2 / 2) / v_kl is monotone in
// r1^2 (also in floating point), so it is attained at min_m r1_km^2.
__global__ __launch_bounds__(VTHREADS) void k_mle_minsq(const ChunkDesc* __restrict__ chs,
                                                        MleArgs a, double* __restrict__ part) {
  __shared__ double sm[VTHREADS / WAVE][MAXK];
  const ChunkDesc ch = chs[blockIdx.x];
  double mn[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) mn[k] = __builtin_inf();
  CHUNK_LOOP(ch) {
    const int64_t i = ch.voff + t;
#pragma unroll
    for (int k = 0; k < MAXK; ++k)
      if (k < a.K) {
        const double r = a.r1[k][i];
        mn[k] = fmin(mn[k], r * r);
      }
  }
  const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    double v = mn[k];
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, WAVE));
    if (lane == 0) sm[wid][k] = v;
  }
  __syncthreads();
  if ((int)threadIdx.x < MAXK) {
    const int k = threadIdx.x;
    part[(int64_t)blockIdx.x * MAXK + k] = fmin(fmin(sm[0][k], sm[1][k]), fmin(sm[2][k], sm[3][k]));
  }
}

hipError_t launch_mle_minsq(const ChunkDesc* d_ch, int nch, const MleArgs& a, double* d_part,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_mle_minsq, dim3(nch), dim3(VTHREADS), 0, st, d_ch, a, d_part);
  return hipGetLastError();
}

// S_l = sum_{k,m} a_k p_kml / Den_km with p_kml = exp(-r1^2/2/v_kl - exp_max) / sqrt(v_kl),
// Den_km = sum_l p_kml omega_l (:153-158; the same operation order per element)
constexpr int MLE_NV = MAXL + 1;
static_assert(MLE_NV <= MAXNV, "mle partials");
__global__ __launch_bounds__(VTHREADS) void k_mle_terms(const ChunkDesc* __restrict__ chs,
                                                        MleArgs a, double* __restrict__ part) {
  const ChunkDesc ch = chs[blockIdx.x];
  double acc[MLE_NV];
#pragma unroll
  for (int l = 0; l < MLE_NV; ++l) acc[l] = 0.0;
  CHUNK_LOOP(ch) {
    const int64_t i = ch.voff + t;
#pragma unroll
    for (int k = 0; k < MAXK; ++k)
      if (k < a.K) {
        const double r = a.r1[k][i];
        const double nr2 = -(r * r);
        double p[MLE_NV];
        double den = 0.0;
#pragma unroll
        for (int l = 0; l < MLE_NV; ++l)
          if (l < a.L) {
            const double v = a.sigma2[l] + a.ginv[k];       // prior_vars0 + gam1invs
            p[l] = exp(nr2 / 2.0 / v - a.exp_max) / sqrt(v);
            den = (l == 0) ? p[l] * a.omega[l] : den + p[l] * a.omega[l];
          }
#pragma unroll
        for (int l = 0; l < MLE_NV; ++l)
          if (l < a.L) acc[l] += a.a[k] * p[l] / den;
      }
  }
  block_reduce_store<MLE_NV>(acc, part + (int64_t)blockIdx.x * MLE_NV, MLE_NV);
}

hipError_t launch_mle_terms(const ChunkDesc* d_ch, int nch, const MleArgs& a, double* d_part,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_mle_terms, dim3(nch), dim3(VTHREADS), 0, st, d_ch, a, d_part);
  return hipGetLastError();
}

}  // namespace sgv
