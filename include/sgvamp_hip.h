/*
 * sgvamp_hip.h -- C ABI of the MI355X-native sgVAMP hot path (libsgvamp_hip.so).
 *
 * The reference (medical-genomics-group/sgVAMP-py) has no FFI layer; its hot path
 * sits behind the class seam VAMP(...)/VAMP.infer(...) (src/sgvamp.py:15,196) and
 * the operator seam con_grad(A, b, maxiter, x0) -> (x, info) (src/sgvamp.py:7,316,332).
 * Every entry point below names the reference code it replaces.  The Python host
 * (sgvamp-py_amd/sgvamp.py) binds them with ctypes; INTEGRATION.md shows the stub.
 *
 * Conventions
 *  - Return 0 on success, a negative SGV_ERR_* code on failure; the message is in
 *    sgv_last_error(ctx) (ctx may be NULL for errors raised before a ctx exists).
 *    No C++ exception crosses the ABI.
 *  - Host arrays are caller-owned, C-contiguous, borrowed for the call only.
 *    Vectors are f64 in the rank-local DENSE marker order (the rank's blocks
 *    concatenated).  Device memory is owned by the ctx.
 *  - One ctx per process and GPU; one host thread drives it; not re-entrant.
 *  - Markers are partitioned into LD blocks (block-diagonal LD).  A rank owns a
 *    contiguous range of global blocks [blk0, blk0 + nblk).  All K cohorts of a
 *    marker live on the same rank.  Every M-length reduction is summed per LD
 *    block in a fixed order and then over blocks in global block order, so runs
 *    on 1/2/4/8 GPUs give bit-identical results.
 */
#ifndef SGVAMP_HIP_H
#define SGVAMP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGV_OK 0
#define SGV_ERR_HIP (-1)
#define SGV_ERR_ARG (-2)
#define SGV_ERR_RCCL (-3)
#define SGV_ERR_STATE (-4)

/* ABI revision of this header.  2: sgv_timers / sgv_exchange_stats take the
 * caller's buffer length (cap), sgv_comm_info added.  An integrator checks
 * sgv_abi_version() == SGV_ABI_VERSION before binding the rest. */
#define SGV_ABI_VERSION 2
int sgv_abi_version(void);

#define SGV_MAX_COHORTS 1024 /* cohorts per context (the reference's K is its MPI
                                world size); the LMMSE batches them 8 at a time
                                (16 CG right-hand sides per LD pass), the marker
                                kernels (denoiser, EM, MLE) 32 per launch          */
#define SGV_MAX_SLABS 8     /* L - 1 slab components of the prior      */

/* vector ids for sgv_set_vector / sgv_get_vector */
#define SGV_VEC_R 0       /* r_k = X_k^T y_k            (src/main.py:176-191,266)   */
#define SGV_VEC_R1 1      /* r1_k, denoiser input        (src/sgvamp.py:204,348)     */
#define SGV_VEC_XHAT1 2   /* xhat1 (shared)              (src/sgvamp.py:273-276)     */
#define SGV_VEC_XHAT2 3   /* xhat2_k                     (src/sgvamp.py:316-323)     */
#define SGV_VEC_SIG2U 4   /* Sigma2_u_k                  (src/sgvamp.py:332-333)     */
#define SGV_VEC_X0 5      /* true signal for metrics     (src/main.py:268-285)       */

/* sgv_lmmse per-cohort outputs, out[k * SGV_LMMSE_NOUT + i] */
#define SGV_LMMSE_NOUT 8
#define SGV_O_TRSIGMA2 0  /* u^T Sigma2 u                 src/sgvamp.py:338 */
#define SGV_O_ALPHA2 1    /* alpha2 (after damping)       :340,345-346      */
#define SGV_O_GAM1 2      /* gam2 (1-alpha2)/alpha2       :347              */
#define SGV_O_Z 3         /* z (clamped at 0)             :352-354          */
#define SGV_O_TRRSIGMA2 4 /* u^T R Sigma2 u               :359              */
#define SGV_O_GAMW 5      /* 1/(z/N + TrRSigma2/N), not yet clamped at 1 :363 */
#define SGV_O_XR 6        /* xhat2^T r                    :352              */
#define SGV_O_XRX 7       /* xhat2^T R xhat2              :352              */

typedef struct sgv_ctx sgv_ctx;

/* ---- lifetime ------------------------------------------------------------ */

/* Per-rank setup; replaces src/main.py:79-97 (K, N lists), :143 (M), :287 (a)
 * and VAMP.__init__ src/sgvamp.py:15-31 for the device side.
 *   device          HIP device ordinal this rank drives
 *   K               cohorts (1..SGV_MAX_COHORTS)
 *   nld             distinct LD matrices; ld_of[k] in [0, nld)
 *   nblk, blk_sizes LD blocks owned by this rank, in marker order
 *   blk0            global index of this rank's first block
 *   nblk_global     total blocks over all ranks
 *   M_total         total markers over all ranks (np.mean denominators) */
int sgv_create(int device, int K, int nld, const int* ld_of, int nblk,
               const int64_t* blk_sizes, int blk0, int nblk_global, int64_t M_total,
               sgv_ctx** out);
void sgv_destroy(sgv_ctx* ctx);
const char* sgv_last_error(const sgv_ctx* ctx);

/* ---- multi-GPU (RCCL over xGMI) ----------------------------------------- */

/* Replaces mpi4py COMM_WORLD (src/main.py:16-18) and the per-iteration K x M
 * bcast all-gather (src/sgvamp.py:228-233), which disappears because all cohorts
 * of a marker are co-located.  What remains are ordered reductions of per-block
 * partial sums (ncclAllGather).  id: 128 bytes (ncclUniqueId) from rank 0.
 * nranks may be 1: a real one-rank communicator then carries the same gather
 * (rehearses the RCCL calls on a single GPU; results bitwise unchanged). */
int sgv_comm_unique_id(char* id_out /* 128 bytes */);
int sgv_comm_init(sgv_ctx* ctx, int nranks, int rank, const char* id /* 128 bytes */,
                  const int* nblk_per_rank /* [nranks] */);
/* Host-side exchange instead of RCCL (same ordered reductions, bitwise the same
 * results): the library copies its per-block partials to host memory and calls
 * fn(user, send, recv, count) which must all-gather `count` doubles from every
 * rank into recv[nranks][count] in rank order and return 0.  For ranks that
 * RCCL cannot connect (several ranks on one device, hosts without xGMI peers)
 * and for testing the sharded path with a host communicator. */
typedef int (*sgv_allgather_fn)(void* user, const double* send, double* recv, int64_t count);
int sgv_comm_init_host(sgv_ctx* ctx, int nranks, int rank, const int* nblk_per_rank,
                       sgv_allgather_fn fn, void* user);

/* ---- inputs -------------------------------------------------------------- */

/* Upload one dense LD block (row-major n x n, host row stride ld_host elements).
 * Replaces the R loaders src/main.py:199-202 (dense .npy / CSR .npz blocks). */
int sgv_set_ld_block(sgv_ctx* ctx, int ld, int blk_local, const double* rowmajor,
                     int64_t ld_host);
/* Upload one symmetric LD block from the CSR arrays of its upper triangle
 * (diagonal included; block-relative column indices >= the row; duplicates are
 * summed).  Replaces the sparse loaders src/main.py:199-200 (.npz CSR of any
 * sparsity) and :251-257 (PLINK .ld pairs assembled into CSR): a block whose
 * entries lie within j - i <= bw is stored as a packed BAND -- panel g (rows
 * 256g ..) keeps columns 256g .. 256g + round_up(256 + bw, 256) - 1 -- so
 * windowed LD over a whole chromosome needs n * (bw + 256..511) doubles instead
 * of n^2 / 2.  Blocks whose band is as wide as the triangle are stored as the
 * packed triangle.  Never allocates n x n on the host. */
int sgv_set_ld_block_csr(sgv_ctx* ctx, int ld, int blk_local, const int64_t* indptr /* n+1 */,
                         const int64_t* indices, const double* data);
/* R_s xhat2 and R_s Sigma2_u for gamw learning (src/sgvamp.py:352,359) and the
 * next warm start's R_s x0 (scipy iterative.py:392): on (default), carried
 * through both CG solves -- x_k = x_0 + sum a_i p_i, so R_s x_k = R_s x_0 +
 * sum a_i R_s p_i with R_s p_i written by the pass the CG makes anyway -- which
 * saves one LD pass per outer iteration; off, computed by a separate pass as
 * the reference does.  Same values in exact arithmetic; measured against the
 * reference fixtures the carried form agrees as closely (tests/). */
int sgv_set_rs_recurrence(sgv_ctx* ctx, int on);
/* Packed passes with at least nc_min right-hand sides run on the f64 matrix
 * cores (v_mfma_f64_16x16x4f64); fewer run on the VALU.  0 = never.  Default 3
 * (env SGV_MFMA_MIN).  Results agree to rounding, not bitwise, across the two. */
int sgv_set_mfma_min(sgv_ctx* ctx, int nc_min);
/* CG and EM-loop drivers (scipy iterative.py:397-422; src/sgvamp.py:250-257):
 * on (default) the CG's stop test, beta and alpha, and the EM prior loop's
 * update and convergence test run on the device, and iteration i+1 is enqueued
 * while iteration i runs (no host round trip between iterations); off, the
 * host tests every iteration.  Same iterates and counts; env SGV_CG_PIPE=0
 * sets the default off.  Column sets of the pipelined CG: see sgv_set_cg_exact. */
int sgv_set_cg_pipeline(sgv_ctx* ctx, int on);
/* Column sets of the pipelined CG's passes.  mode 1 ("exact"): a pass over an
 * LD matrix shared by >= 3 columns carries only the columns still active after
 * its own stop test (the host reads the test while the p update runs); mode 0:
 * one iteration of look-ahead (a column stopping at that test rides along
 * unused).  The two modes can round differently where the narrower set runs
 * another pass kernel, so every rank of a run must use the same mode -- it is
 * the run's choice, not a rank's: Python's Engine sets it from the GLOBAL LD
 * size (>= 24 GB packed-triangle bytes), identical for 1 and N ranks.  mode -1
 * (default): by this rank's stored bytes at one rank, look-ahead with a
 * communicator.  SGV_CG_EXACT=0/1 (with SGV_AB=1) overrides every mode. */
int sgv_set_cg_exact(sgv_ctx* ctx, int mode);
/* Storage of LD blocks set or generated from now on: mode 1 (default) stores a
 * block that is exactly symmetric as packed upper-triangle panels (about half
 * the bytes per pass: the LD matrix of src/main.py:199-265 is symmetric by
 * construction, R = X^T X); mode 0 always stores the full square. */
int sgv_set_ld_packing(sgv_ctx* ctx, int mode);
/* fmt_out: 0 dense, 1 packed symmetric (triangle), 2 packed band, -1 not set. */
int sgv_ld_block_format(sgv_ctx* ctx, int ld, int blk_local, int* fmt_out);
/* Bytes one pass over LD matrix ld reads from this rank's blocks that are set
 * (dense n^2*8, packed triangle / band: the stored panels).  Python's Engine
 * sums it over ranks to pick the run's CG column-set mode (sgv_set_cg_exact). */
int sgv_ld_stored_bytes(sgv_ctx* ctx, int ld, double* bytes_out);
/* Coupling between consecutive band pieces gb and gb + 1 (global block
 * indices) of LD matrix ld: C = R[last nr rows of gb][first nc columns of gb+1],
 * nr x nc row-major.  A band block too long for one GPU (one chromosome of
 * windowed LD: src/main.py:199-200,251-257) is cut into pieces that ranks own
 * like LD blocks; a pass then adds C p_{gb+1}[head] to gb's last rows and
 * C^T p_gb[tail] to gb+1's first rows, in a fixed order on every rank (results
 * bitwise independent of the rank count), the halo of a coupling that spans two
 * ranks exchanged per pass.  Every rank calls this for EVERY coupling (C may be
 * NULL where the rank owns neither piece): the exchange is collective.  Pieces
 * must be stored packed (sgv_set_ld_block_csr). */
int sgv_set_ld_coupling(sgv_ctx* ctx, int ld, int gb, int nr, int nc, const double* C);
/* Download one LD block (row-major n x n into a host array of row stride ld_host). */
int sgv_get_ld_block(sgv_ctx* ctx, int ld, int blk_local, double* rowmajor, int64_t ld_host);
/* Start a new VAMP.infer on this context (src/sgvamp.py:198-217 restarts from
 * r1 = r, xhat2 = 0, Sigma2_u_prev = 0 on every call): zeroes every solver
 * vector except r, r1 and x0 and clears the warm-start and chained-step state.
 * LD blocks, ridge and cohort sizes are kept.  Fails while a step is queued. */
int sgv_reset_solver(sgv_ctx* ctx);
/* R_s = (1 - s) R + s I, applied inside every LD pass (src/main.py:265). */
int sgv_set_ridge(sgv_ctx* ctx, double s);
/* Cohort sample size N_k (src/main.py:83-85; used by gamw learning :352,363). */
int sgv_set_cohort_n(sgv_ctx* ctx, int k, double N);

int sgv_set_vector(sgv_ctx* ctx, int which, int k, const double* host_local);
int sgv_get_vector(sgv_ctx* ctx, int which, int k, double* host_local);

/* ---- synthetic data on device (simulation/sim_gen_phen_mult.py:36-55) ------
 * Genotypes x_{in} ~ Binomial(2, 0.4) from a counter-based hash of
 * (geno_seed, global marker index, sample n); standardised per marker over the
 * Nsamp samples (population std), X_std; G = X_std / sqrt(Nsamp).
 * marker0 = global index of this rank's first marker (keys the hash, so the
 * data does not depend on how blocks are spread over ranks).
 * Step 1: for every owned block b: if ld >= 0 store R_b = G_b G_b^T into LD
 *         matrix `ld`; write g_b[n] = sum_{i in b} X_std[i][n] beta_i to
 *         g_blocks_out[b * Nsamp + n] (host, nblk x Nsamp).
 * Step 2 (after the host forms y = sum_b g_b + w): r_k,b = G_b y. */
int sgv_synth_ld_g(sgv_ctx* ctx, int ld, uint64_t geno_seed, int64_t marker0, int Nsamp,
                   const double* beta_local, double* g_blocks_out);
int sgv_synth_r(sgv_ctx* ctx, int k, uint64_t geno_seed, int64_t marker0, int Nsamp,
                const double* y);

/* ---- Hutchinson probes (host only, no device) ----------------------------
 * src/sgvamp.py:326 u = np.random.binomial(p=1/2, n=1, size=n)*2-1 from a legacy
 * numpy RandomState (MT19937) whose state is key[624], *pos (as
 * RandomState.get_state() returns them): advances the stream by n samples and
 * writes the +-1 values of samples [lo, hi) to out[0 .. hi-lo).  Bit for bit
 * numpy's stream and values; replaces the draw each reference rank makes. */
int sgv_probe_draw(uint32_t* key, int32_t* pos, int64_t n, int64_t lo, int64_t hi,
                   int8_t* out);

/* ---- the hot path -------------------------------------------------------- */

/* One VAMP outer iteration, src/sgvamp.py:222-387 without the output files and
 * logs, with no return to the caller between its phases:
 *   flags & SGV_STEP_EM:  sgv_em (lam_io, omegas_io updated; ires[0] = steps,
 *                         res[0] = final error);
 *   sgv_denoise (damping iff SGV_STEP_DENOISE_DAMP);
 *   out_slot 0/1/2:      sgv_outputs_begin(out_slot) (xhat1, r1 for the files);
 *   SGV_STEP_METRICS:    the metric sums of xhat1 (:381-382) in res[1 + 2K .. + 4);
 *   alpha1 = der_sum / M_total, damped with alpha1_prev iff SGV_STEP_ALPHA1_DAMP
 *   (:285-291), gam2 = gam1 (1 - alpha1) / alpha1 (:305): res[1 + k], res[1 + K + k];
 *   sgv_lmmse (damping iff SGV_STEP_LMMSE_DAMP, gamw learning iff
 *   SGV_STEP_LEARN_GAMW): out, cg_out as sgv_lmmse; ires[1] = LD passes.
 * res holds 1 + 2K + 4 doubles, ires 2 ints.
 * flags & SGV_STEP_MLE: sgv_mle_update instead of sgv_em (lam_io, omegas_io and the
 *                        context's gam updated; ires[0] = its status, res[0] = gam
 *                        after it, NaN while the reference's is None); the context's
 *                        gam starts as None (sgv_create) and is set by sgv_set_mle_gam.
 * SGV_STEP_CHAIN (sgv_step_begin only): gam1s, gamw (clamped to >= 1, :374),
 * alpha1_prev, alpha2_prev, *lam_io and omegas_io are taken, when the step
 * starts, from the results of the step queued before it -- so a step can be
 * queued while the previous one runs. */
#define SGV_STEP_EM 1
#define SGV_STEP_DENOISE_DAMP 2
#define SGV_STEP_ALPHA1_DAMP 4
#define SGV_STEP_LMMSE_DAMP 8
#define SGV_STEP_LEARN_GAMW 16
#define SGV_STEP_METRICS 32
#define SGV_STEP_CHAIN 64
#define SGV_STEP_MLE 128
int sgv_step(sgv_ctx* ctx, int it, int flags, int em_maxit, int nslab, const double* sigmas,
             const double* a, double* lam_io, double* omegas_io, const double* gam1s,
             double rho, const double* gamw, const double* alpha1_prev,
             const double* alpha2_prev, const int8_t* probes, int cg_maxit, double rtol,
             int out_slot, double* res, int* ires, double* out, int* cg_out);
/* sgv_step on the context's host worker thread: returns at once; at most two
 * steps are queued and they run in order.  The caller may run host work
 * (files, logs, the next probes) that does not touch the context
 * (sgv_outputs_wait excepted) until sgv_step_end, which waits for the oldest
 * queued step and returns its status.  lam_io, omegas_io, probes and the
 * outputs must stay valid until then; the other arrays are copied. */
int sgv_step_begin(sgv_ctx* ctx, int it, int flags, int em_maxit, int nslab,
                   const double* sigmas, const double* a, double* lam_io, double* omegas_io,
                   const double* gam1s, double rho, const double* gamw,
                   const double* alpha1_prev, const double* alpha2_prev, const int8_t* probes,
                   int cg_maxit, double rtol, int out_slot, double* res, int* ires, double* out,
                   int* cg_out);
int sgv_step_end(sgv_ctx* ctx);

/* Meta denoiser + derivative over all markers: src/sgvamp.py:93-114 applied at
 * :270-291.  xhat1 <- denoiser_meta(r1s, gam1s); if damp: xhat1 <- rho*xhat1 +
 * (1-rho)*xhat1_prev.  der_sum_out[k] = sum_j der_denoiser_meta_k(r1s[:, j])
 * (the host divides by M_total: np.mean, :285). */
int sgv_denoise(sgv_ctx* ctx, const double* gam1s, const double* a, double lam,
                int nslab, const double* omegas, const double* sigmas, double rho,
                int damp, double* der_sum_out);

/* EM prior update loop: src/sgvamp.py:116-136 driven as :250-257 (stop when the
 * relative change of omegas and lam are both < 1e-6, at most maxit steps). */
int sgv_em(sgv_ctx* ctx, const double* gam1s, const double* a, int nslab,
           const double* sigmas, int maxit, double* lam_io, double* omegas_io,
           int* steps_out, double* final_err_out);

/* LMMSE step for all cohorts: src/sgvamp.py:301-364.  For every cohort k:
 *   r2 = (xhat1 - alpha1 r1)/(1 - alpha1); mu2 = gamw r + gam2 r2;
 *   CG #1: (gamw R_s + gam2 I) xhat2 = mu2, warm start xhat2_prev   (:316)
 *   damping of xhat2 if lmmse_damp                                 (:322-323)
 *   CG #2: (gamw R_s + gam2 I) Sigma2_u = u, warm start Sigma2_u_prev (:332)
 *   alpha2, gam1, r1 update                                        (:338-348)
 *   if learn_gamw: z, TrRSigma2, new gamw                          (:350-363)
 * Both CG solves of all cohorts run batched: one pass over each LD matrix per
 * CG iteration serves every right-hand side still iterating.  The CG is
 * scipy 1.15.3's (iterative.py:375-422): rtol, atol 0, strict '<' stop test.
 *   per-cohort inputs [K]: gamw, gam2, alpha1, alpha2_prev
 *   probes: [K][M_local] int8 of +-1 (the host draws u, :326)
 *   out: [K][SGV_LMMSE_NOUT]; cg_out: [K][4] = iters1, info1, iters2, info2
 *   ld_passes_out: LD passes (full sweeps over all owned LD bytes) performed */
/* MLE prior update (--prior-update mle, src/sgvamp.py:139-194).  The host runs
 * the reference's scipy.optimize.fsolve on Lagrangian_der; these two calls
 * compute its device-side parts over all markers and cohorts (the current r1
 * vectors).  L = mixture components including the spike, sigma2[L] the
 * component variances (sigma2[0] = 1e-16, :169-171).
 * exp_max (:152): max over (k, m, l) of (-r1_km^2 / 2) / (sigma2_l + 1/gam1_k).
 * sums[l] (:155-158): sum over k, m of a_k p_kml / sum_l' p_kml' omega_l', with
 * p_kml = exp((-r1_km^2 / 2) / v_kl - exp_max) / sqrt(v_kl). */
int sgv_mle_exp_max(sgv_ctx* ctx, const double* gam1s /* K */, int L, const double* sigma2,
                    double* exp_max);
int sgv_mle_terms(sgv_ctx* ctx, const double* a /* K */, const double* gam1s /* K */, int L,
                  const double* sigma2 /* L */, const double* omega /* L */, double exp_max,
                  double* sums /* L */);
/* The whole MLE prior update in the library, src/sgvamp.py:162-194: x0 from
 * lam, omegas (nslab of them) and gam (*gam_io NaN = the reference's None: x0[-1]
 * = 1), sgv_fsolve on Lagrangian_der (:139-160, the sums from sgv_mle_terms),
 * then the reference's acceptance tests and normalisation.  *status_out: 0 =
 * lam_io, omegas_io, gam_io updated; SGV_MLE_NOT_CONVERGED (fsolve's ier != 1)
 * or SGV_MLE_NEGATIVE (a non-positive mixture weight): nothing changed, the
 * reference's "No prior update!" cases. */
#define SGV_MLE_NOT_CONVERGED 1
#define SGV_MLE_NEGATIVE 2
int sgv_mle_update(sgv_ctx* ctx, const double* gam1s /* K */, const double* a /* K */, int nslab,
                   const double* sigmas /* nslab */, double* lam_io, double* omegas_io,
                   double* gam_io, int* status_out);

/* scipy.optimize.fsolve(fcn, x0, full_output=True) with its defaults (MINPACK
 * hybrd: xtol 1.49012e-08, maxfev 200 (n + 1), forward-difference Jacobian with
 * epsfcn = machine epsilon, factor 100, automatic scaling), host only: fcn
 * writes F(x) to fvec and returns 0, or a negative value to stop the solver.
 * x_io: x0 in, the last accepted iterate out; fvec_out (may be null): F there;
 * *nfev_out (may be null): function evaluations.  Returns MINPACK's info
 * (1 = converged, 2-5 = the other terminations, < 0 = fcn's stop value, 0 =
 * bad arguments) -- the reference's `ier` (src/sgvamp.py:179-181). */
/* The MLE update's Lagrange multiplier that SGV_STEP_MLE steps use and update
 * (the reference's self.gam, src/sgvamp.py:31,178,194; NaN = None). */
int sgv_set_mle_gam(sgv_ctx* ctx, double gam);

typedef int (*sgv_fsolve_fn)(void* user, int n, const double* x, double* fvec);
int sgv_fsolve(int n, sgv_fsolve_fn fcn, void* user, double* x_io, double* fvec_out,
               int* nfev_out);

/* The per-iteration output vectors without a host wait (src/sgvamp.py:281,283):
 * sgv_outputs_begin queues this rank's slices of xhat1 and r1[0..K-1] (unscaled,
 * marker order) into pinned slot 0, 1 or 2; sgv_outputs_wait -- callable from a
 * writer thread -- waits for that copy and returns the slot's buffer
 * [(K + 1) x M_local] doubles, valid until the slot is begun again. */
int sgv_outputs_begin(sgv_ctx* ctx, int slot);
int sgv_outputs_wait(sgv_ctx* ctx, int slot, double** data);

int sgv_lmmse(sgv_ctx* ctx, int it, const double* gamw, const double* gam2,
              const double* alpha1, const double* alpha2_prev, const int8_t* probes,
              int cg_maxit, double rtol, int lmmse_damp, double rho, int learn_gamw,
              double* out, int* cg_out, int* ld_passes_out);

/* Metrics src/sgvamp.py:379-387: out[0] = <xhat1, x0>, out[1] = |xhat1|^2,
 * out[2] = |xhat1 - x0|^2, out[3] = |x0|^2 (global sums). */
int sgv_metrics(sgv_ctx* ctx, double* out4);
/* Split form of sgv_metrics: begin queues the kernel and the ordered reduction
 * (call after sgv_denoise; xhat1/x0 must not change before end), end waits for
 * it and returns the same 4 sums.  Lets the host skip a sync per iteration. */
int sgv_metrics_begin(sgv_ctx* ctx);
int sgv_metrics_end(sgv_ctx* ctx, double* out4);

/* ---- operator seam, exposed for tests ------------------------------------ */

/* y = R_s v for LD matrix `ld` over the rank's blocks (one LD pass, up to 16
 * columns).  v, y: [ncol][M_local] host, dense.  Replaces A.matvec inside
 * scipy cg (src/sgvamp.py:316,332) and R @ x (:352,359). */
int sgv_ld_matvec(sgv_ctx* ctx, int ld, int ncol, const double* v, double* y);

/* Batched scipy-1.15.3 CG on (c1 R_s + c2 I) x = b for ncol columns sharing LD
 * `ld` (operator seam con_grad, src/sgvamp.py:7).  x: in = x0, out = solution.
 * iters_out/info_out [ncol]. */
int sgv_cg_solve(sgv_ctx* ctx, int ld, int ncol, const double* c1, const double* c2,
                 const double* b, double* x, int maxiter, double rtol, int* iters_out,
                 int* info_out);

/* ---- timing -------------------------------------------------------------- */
/* Summed over LD passes since the last reset (HIP events on the ctx stream):
 * t[0] = kernel time (ms), t[1] = passes, t[2] = LD bytes read (the stored
 * bytes: n^2*8 dense, sum over panels H*(n - r0)*8 packed), t[3] = RHS bytes
 * (2 * ncol * M_local * 8), t[4] = dense-equivalent LD bytes (n^2*8),
 * t[5] = packed-pass partial-buffer bytes (written + read), t[6] = the passes'
 * algorithmic flops (2 per multiply-add: each column's row part over every
 * stored element, and its transpose part over the packed elements right of
 * each panel's diagonal block), t[7] / t[8] / t[9] = flops / kernel ms / passes
 * of the 9..16-column passes (f64 16x16x4 MFMA: their bound is the matrix core).
 * Writes min(cap, SGV_TIMERS_N) values (a caller built against a shorter list
 * passes its own length and gets that prefix); cap < 0 is an error.
 * reset != 0 zeroes. */
#define SGV_TIMERS_N 10
int sgv_timers(sgv_ctx* ctx, double* t, int cap, int reset);
/* Cross-rank exchange counters since the last reset (the bcast/all-gather of
 * src/sgvamp.py:228-233 and the CG/EM scalar reductions that replace it):
 * out[0] = all-gathers issued, out[1] = ms spent in them (RCCL: HIP events
 * around each ncclAllGather on the ctx stream, the wait for the slowest peer
 * included; host exchange: wall time of the callback), out[2] = bytes this rank
 * contributed, out[3] = the last EM prior loop's mode (1 replicated: r1
 * all-gathered once per loop; 0 one exchange per EM step; -1 no communicator or
 * no loop yet), out[4] = the per-all-gather latency (us) the EM cost model uses,
 * out[5] = 1 RCCL, 2 host exchange, 0 none, out[6] / out[7] = EM loops run
 * replicated / per step, out[8] / out[9] = the last decision's predicted cost
 * (us) of the replicated / per-step loop, out[10] = the steps it predicted,
 * out[11] = ms the device idled between an exact-CG iteration's p update and
 * its passes, which the host enqueues once it has read the stop test (HIP
 * events), out[12] = the latency's source (0 default 25 us, 1 env
 * SGV_XCHG_LAT_US of rank 0, 2 sgv_exchange_probe), out[13] = 1 if the
 * replicated loop can run (K <= 32, <= 128 blocks in all), out[14] / out[15] =
 * ms / count of the device-driven EM prior loops (HIP events from the loop's
 * first enqueue to its last step: the cost the model predicts in out[8..9]).
 * Writes min(cap, SGV_EXCHANGE_STATS_N) values; cap < 0 is an error.  reset != 0
 * zeroes out[0..2], out[6..7], out[11] and out[14..15]. */
#define SGV_EXCHANGE_STATS_N 16
int sgv_exchange_stats(sgv_ctx* ctx, double* out, int cap, int reset);

/* Who this context's exchange talks to, for a launch to prove its topology:
 * out[0] = transport (0 none, 1 RCCL, 2 host exchange), out[1] = ranks in the
 * communicator (RCCL: ncclCommCount; host: the nranks given), out[2] = this
 * rank in it (RCCL: ncclCommUserRank), out[3] = the HIP device the context runs
 * on (RCCL: ncclCommCuDevice), out[4] = the nranks the context was given.
 * Writes min(cap, SGV_COMM_INFO_N) values; pci_bus_id (if not null) receives
 * the device's PCI bus id ("0000:xx:00.0", NUL-terminated, at most pci_len
 * bytes). */
#define SGV_COMM_INFO_N 5
int sgv_comm_info(sgv_ctx* ctx, int* out, int cap, char* pci_bus_id, int pci_len);

/* Measure the per-all-gather latency of this job's exchange (the CG's ordered
 * reduction of 16 values: per-block sums, all-gather, ordered total; `reps`
 * times on the ctx stream) and make the maximum over ranks the EM cost model's
 * latency on every rank.  Collective (every rank, between steps); *us_out =
 * the agreed latency in us (0 without a communicator).  The probe's
 * all-gathers are not counted in sgv_exchange_stats. */
int sgv_exchange_probe(sgv_ctx* ctx, int reps, double* us_out);

/* The EM exchange cost model alone (host arithmetic, no device): predicted us
 * of one EM loop of `steps` enqueued steps over `cohort_markers` = K x M on
 * `nranks` ranks with a per-all-gather latency of `latency_us`; out2[0] =
 * replicated (one r1 all-gather, the loop over all markers on every rank;
 * src/sgvamp.py:228-259), out2[1] = one exchange per EM step.  The library
 * runs the cheaper (sgv_exchange_stats out[3], out[8..10]). */
int sgv_em_cost_model(double cohort_markers, int nranks, double latency_us, double steps,
                      double* out2);

/* Synchronise the ctx stream. */
int sgv_sync(sgv_ctx* ctx);

/* The device's streaming-read rate (context for the LD passes' roofline): a
 * temporary buffer of `bytes` (rounded down to 256 KiB) read once per repeat,
 * every workgroup its own contiguous 256 KiB with 16-B nontemporal loads; the
 * best of `reps` repeats in GB/s (1e9 B/s) -> *gbps. */
int sgv_read_bw(sgv_ctx* ctx, int64_t bytes, int reps, double* gbps);

#ifdef __cplusplus
}
#endif
#endif /* SGVAMP_HIP_H */
