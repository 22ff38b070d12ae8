"""Shard-aware wrapper over one sgv_ctx: this rank's LD blocks, all cohorts.

An Engine owns the rank-local slice [marker0, marker0 + Mloc) of every
marker-length vector; every M-length reduction inside the library is ordered
by global LD block, so the scalars it returns are identical on every rank and
for any number of ranks.
"""
import ctypes
import os

import numpy as np

import hip_backend as hb
from partition import marker_offsets, partition_blocks

CG_EXACT_MIN_BYTES = 24e9   # capi.hip: exact CG column sets from passes of this size
SYM_H = 256                 # rows per packed panel (common.h)


def cg_exact_mode(block_sizes):
    """The run's CG column-set mode (sgv_set_cg_exact) from the GLOBAL LD: exact
    sets when a pass streams >= 24 GB of packed triangle, else look-ahead.  A
    function of the global block sizes only, so every rank of a run and every
    rank count make the same choice (the modes can round differently).  The
    estimate before any LD is stored; Engine.update_cg_exact refines it from the
    bytes actually stored (band blocks store far less than the triangle)."""
    tri = sum(float(n) * (n + SYM_H) / 2.0 * 8.0 for n in block_sizes)
    return 1 if tri >= CG_EXACT_MIN_BYTES else 0


def cg_exact_from_stored(global_bytes_per_ld, ld_of):
    """The same choice from the global stored bytes of each LD matrix: exact when
    a matrix shared by >= 2 cohorts (>= 4 CG columns: the MFMA pass, where a
    narrower column set is cheaper) streams >= 24 GB per pass."""
    shared = [l for l in set(ld_of) if list(ld_of).count(l) >= 2]
    big = max((global_bytes_per_ld[l] for l in shared), default=0.0)
    return 1 if big >= CG_EXACT_MIN_BYTES else 0


class Engine:
    def __init__(self, block_sizes, K, ld_of=None, comm=None, device=None, exchange=None):
        """block_sizes: global LD block sizes (marker order).  ld_of[k]: index of
        the LD matrix cohort k uses (cohorts sharing an LD share LD passes).
        exchange: "rccl" (default) or "host" (the communicator's allgather_f64
        carries the per-block partials; env SGV_EXCHANGE overrides the default).
        With one rank no communicator is made unless `exchange` is passed
        explicitly (a one-rank RCCL/host exchange: same results, used to rehearse
        the exchange on one GPU)."""
        from comm import SingleComm

        self.comm = comm or SingleComm()
        self.rank = self.comm.Get_rank()
        self.nranks = self.comm.Get_size()
        self.block_sizes = [int(b) for b in block_sizes]
        self.K = int(K)
        self.ld_of = list(ld_of) if ld_of is not None else [0] * self.K
        if len(self.ld_of) != self.K:
            raise ValueError("ld_of must have K entries")
        # canonical LD ids 0..nld-1 in order of first use
        remap = {}
        for l in self.ld_of:
            remap.setdefault(l, len(remap))
        self.ld_of = [remap[l] for l in self.ld_of]
        self.nld = len(remap)
        self.ranges = partition_blocks(self.block_sizes, self.nranks)
        self.b0, self.b1 = self.ranges[self.rank]
        offs = marker_offsets(self.block_sizes)
        self.M = int(offs[-1])
        self.marker0 = int(offs[self.b0])
        self.Mloc = int(offs[self.b1] - offs[self.b0])
        self.local_sizes = self.block_sizes[self.b0:self.b1]
        self.sl = slice(self.marker0, self.marker0 + self.Mloc)
        if device is None:   # one process per GPU: the node-local rank (comm.launch_from_env)
            device = int(getattr(self.comm, "local_rank", 0)) if self.nranks > 1 else 0
        self.ctx = hb.Context(device, self.K, self.ld_of, self.local_sizes, self.b0,
                              len(self.block_sizes), self.M)
        self.cg_exact = cg_exact_mode(self.block_sizes)
        self.ctx.sgv_set_cg_exact(self.cg_exact)    # an SGV_CG_EXACT A/B override wins
        self.exchange = exchange or os.environ.get("SGV_EXCHANGE", "rccl")
        if self.exchange not in ("rccl", "host"):
            raise ValueError("exchange must be 'rccl' or 'host', got %r" % self.exchange)
        self._ag_cb = None
        if self.nranks > 1 or exchange is not None:
            counts = np.array([r1 - r0 for r0, r1 in self.ranges], dtype=np.int32)
            if self.exchange == "host":
                self._ag_cb = hb.make_allgather(self.comm, self.nranks)
                self.ctx.sgv_comm_init_host(self.nranks, self.rank, hb.iptr(counts),
                                            ctypes.cast(self._ag_cb, ctypes.c_void_p), None)
            else:
                uid = hb.unique_id() if self.rank == 0 else None
                uid = self.comm.bcast(uid, root=0)
                self.ctx.sgv_comm_init(self.nranks, self.rank, uid, hb.iptr(counts))
            # this job's all-gather latency, the EM loop's cost-model parameter.
            # The probe is collective, so the decision must be the same on every
            # rank: the library took rank 0's SGV_XCHG_LAT_US (if any) at
            # communicator set-up, and its latency source -- rank 0's, identical
            # on every rank -- says whether to probe ("default": rank 0 set no
            # value) or keep rank 0's setting.  A rank's own environment decides
            # nothing here.
            if self.exchange_stats()["latency_source"] == "default":
                self.exchange_probe(10)

    # ---- inputs ----------------------------------------------------------
    def set_ld_block(self, ld, b_global, block):
        """Upload LD block b_global of LD matrix `ld` if this rank owns it."""
        if not (self.b0 <= b_global < self.b1):
            return
        B = np.ascontiguousarray(block, dtype=np.float64)
        n = self.block_sizes[b_global]
        if B.shape != (n, n):
            raise ValueError("LD block %d has shape %s, expected (%d, %d)" % (b_global, B.shape, n, n))
        self.ctx.sgv_set_ld_block(ld, b_global - self.b0, hb.dptr(B), n)

    def set_ld_block_csr(self, ld, b_global, upper):
        """Upload LD block b_global from the scipy CSR of its upper triangle
        (block-relative, diagonal included) if this rank owns it; stored as a
        packed band when the entries stay near the diagonal (sgv_set_ld_block_csr)."""
        if not (self.b0 <= b_global < self.b1):
            return
        n = self.block_sizes[b_global]
        if upper.shape != (n, n):
            raise ValueError("LD block %d has shape %s, expected (%d, %d)" % (b_global, upper.shape, n, n))
        indptr = np.ascontiguousarray(upper.indptr, dtype=np.int64)
        indices = np.ascontiguousarray(upper.indices, dtype=np.int64)
        data = np.ascontiguousarray(upper.data, dtype=np.float64)
        self.ctx.sgv_set_ld_block_csr(ld, b_global - self.b0, indptr.ctypes.data_as(hb._c_i64_p),
                                      indices.ctypes.data_as(hb._c_i64_p), hb.dptr(data))

    def set_ld_coupling(self, ld, gb, nr, nc, C):
        """Coupling between band pieces gb and gb + 1 (global indices) of LD matrix
        ld: C = R[last nr rows of gb][first nc columns of gb + 1] (dense or
        scipy sparse).  Called on every rank for every coupling; the matrix is
        densified and sent only where this rank owns one of the two pieces."""
        own = self.b0 <= gb < self.b1 or self.b0 <= gb + 1 < self.b1
        ptr = None
        if own:
            D = C.toarray() if hasattr(C, "toarray") else np.asarray(C)
            D = np.ascontiguousarray(D, dtype=np.float64)
            if D.shape != (nr, nc):
                raise ValueError("coupling %d has shape %s, expected (%d, %d)" % (gb, D.shape, nr, nc))
            ptr = hb.dptr(D)
        self.ctx.sgv_set_ld_coupling(int(ld), int(gb), int(nr), int(nc), ptr)

    def stored_bytes(self, ld):
        """Bytes one pass over LD matrix ld reads on this rank (blocks set so far)."""
        out = np.zeros(1)
        self.ctx.sgv_ld_stored_bytes(int(ld), hb.dptr(out))
        return float(out[0])

    def update_cg_exact(self):
        """Once every rank's LD blocks are stored: the run's CG column-set mode
        from the GLOBAL stored bytes (summed over ranks in rank order, so every
        rank makes the same choice for any rank count).  Collective."""
        local = np.array([self.stored_bytes(l) for l in range(self.nld)], dtype=np.float64)
        if self.nranks > 1:
            parts = self.comm.allgather(local)
            tot = np.zeros(self.nld)
            for p in parts:
                tot = tot + np.asarray(p, dtype=np.float64)
        else:
            tot = local
        self.cg_exact = cg_exact_from_stored(list(tot), self.ld_of)
        self.ctx.sgv_set_cg_exact(self.cg_exact)    # an SGV_CG_EXACT A/B override wins
        return self.cg_exact

    def get_ld_block(self, ld, b_global):
        n = self.block_sizes[b_global]
        out = np.empty((n, n), dtype=np.float64)
        self.ctx.sgv_get_ld_block(ld, b_global - self.b0, hb.dptr(out), n)
        return out

    def set_mfma_min(self, nc_min):
        """Packed LD passes with >= nc_min right-hand sides use the f64 MFMA kernel."""
        self.ctx.sgv_set_mfma_min(int(nc_min))

    def set_cg_pipeline(self, on):
        """Device-side CG control with the next iteration enqueued ahead (default)
        or the host-side stop test per iteration."""
        self.ctx.sgv_set_cg_pipeline(1 if on else 0)

    def set_rs_recurrence(self, on):
        """Carry R_s x through the CG (default) instead of a gamw LD pass."""
        self.ctx.sgv_set_rs_recurrence(1 if on else 0)

    def reset_solver(self):
        """Zero the solver state for a new infer() (src/sgvamp.py:198-217)."""
        self.ctx.sgv_reset_solver()

    def set_ridge(self, s):
        self.ctx.sgv_set_ridge(float(s))

    def set_cohort_n(self, k, N):
        self.ctx.sgv_set_cohort_n(k, float(N))

    def set_vector(self, which, k, full_or_local):
        v = np.asarray(full_or_local, dtype=np.float64).ravel()
        if v.shape[0] == self.M and self.M != self.Mloc:
            v = v[self.sl]
        v = np.ascontiguousarray(v)
        if v.shape[0] != self.Mloc:
            raise ValueError("vector length %d != local M %d" % (v.shape[0], self.Mloc))
        self.ctx.sgv_set_vector(which, k, hb.dptr(v))

    def get_vector(self, which, k=0):
        out = np.empty(self.Mloc, dtype=np.float64)
        self.ctx.sgv_get_vector(which, k, hb.dptr(out))
        return out

    # ---- synthetic inputs (device generator) -------------------------------
    def synth_ld_g(self, ld, geno_seed, nsamp, beta_full):
        beta = np.ascontiguousarray(np.asarray(beta_full, dtype=np.float64)[self.sl])
        g = np.empty((len(self.local_sizes), nsamp), dtype=np.float64)
        self.ctx.sgv_synth_ld_g(int(ld), int(geno_seed), self.marker0, int(nsamp), hb.dptr(beta),
                                hb.dptr(g))
        return g

    def synth_r(self, k, geno_seed, nsamp, y):
        y = np.ascontiguousarray(y, dtype=np.float64)
        self.ctx.sgv_synth_r(int(k), int(geno_seed), self.marker0, int(nsamp), hb.dptr(y))

    # ---- hot path ------------------------------------------------------------
    def denoise(self, gam1s, a, lam, omegas, sigmas, rho, damp):
        out = np.zeros(self.K)
        om = hb.f64(omegas)
        sg = hb.f64(sigmas)
        self.ctx.sgv_denoise(hb.dptr(hb.f64(gam1s)), hb.dptr(hb.f64(a)), float(lam), len(sg),
                             hb.dptr(om), hb.dptr(sg), float(rho), int(bool(damp)), hb.dptr(out))
        return out

    def em(self, gam1s, a, sigmas, maxit, lam, omegas):
        lam_io = np.array([lam], dtype=np.float64)
        om = hb.f64(np.array(omegas, dtype=np.float64).copy())
        sg = hb.f64(sigmas)
        steps = np.zeros(1, dtype=np.int32)
        err = np.zeros(1)
        self.ctx.sgv_em(hb.dptr(hb.f64(gam1s)), hb.dptr(hb.f64(a)), len(sg), hb.dptr(sg),
                        int(maxit), hb.dptr(lam_io), hb.dptr(om), hb.iptr(steps), hb.dptr(err))
        return float(lam_io[0]), om, int(steps[0]), float(err[0])

    def outputs_begin(self, slot):
        """Queue xhat1 and r1[k] (this rank's slice) into pinned slot 0/1 (no wait)."""
        self.ctx.sgv_outputs_begin(int(slot))

    def outputs_wait(self, slot):
        """Wait for slot's copy (any thread); returns a (K + 1, Mloc) view of the
        pinned buffer, valid until the slot is begun again."""
        p = hb._c_dbl_p()
        rc = self.ctx.lib.sgv_outputs_wait(self.ctx.h, int(slot), ctypes.byref(p))
        if rc != hb.SGV_OK:
            raise hb.HipError("sgv_outputs_wait failed (%d)" % rc)
        return np.ctypeslib.as_array(p, shape=(self.K + 1, max(self.Mloc, 1)))[:, :self.Mloc]

    def mle_exp_max(self, gam1s, sigma2):
        """max over (k, m, l) of (-r1_km^2 / 2) / (sigma2_l + 1/gam1_k) (src/sgvamp.py:152)."""
        out = np.zeros(1)
        sg = hb.f64(sigma2)
        self.ctx.sgv_mle_exp_max(hb.dptr(hb.f64(gam1s)), len(sg), hb.dptr(sg), hb.dptr(out))
        return float(out[0])

    def mle_terms(self, a, gam1s, sigma2, omega, exp_max):
        """The L marker sums of Lagrangian_der (src/sgvamp.py:153-157)."""
        sg = hb.f64(sigma2)
        out = np.zeros(len(sg))
        self.ctx.sgv_mle_terms(hb.dptr(hb.f64(a)), hb.dptr(hb.f64(gam1s)), len(sg), hb.dptr(sg),
                               hb.dptr(hb.f64(omega)), float(exp_max), hb.dptr(out))
        return out

    def set_mle_gam(self, gam):
        """The Lagrange multiplier SGV_STEP_MLE steps start from (None = the reference's)."""
        self.ctx.sgv_set_mle_gam(float("nan") if gam is None else float(gam))

    def mle_update(self, gam1s, a, sigmas, lam, omegas, gam):
        """The whole MLE prior update in the library (sgv_mle_update,
        src/sgvamp.py:162-194): returns (status, lam, omegas, gam); status 0 =
        updated, hb.MLE_NOT_CONVERGED / hb.MLE_NEGATIVE = the reference's "No prior
        update!" cases (inputs returned unchanged).  gam None = the reference's."""
        sg = hb.f64(sigmas)
        lam_io = np.array([lam], dtype=np.float64)
        om = np.array(omegas, dtype=np.float64).copy()
        g = np.array([np.nan if gam is None else gam], dtype=np.float64)
        st = np.zeros(1, dtype=np.int32)
        self.ctx.sgv_mle_update(hb.dptr(hb.f64(gam1s)), hb.dptr(hb.f64(a)), len(sg), hb.dptr(sg),
                                hb.dptr(lam_io), hb.dptr(om), hb.dptr(g), hb.iptr(st))
        return int(st[0]), float(lam_io[0]), om, (None if np.isnan(g[0]) else float(g[0]))

    def lmmse(self, it, gamw, gam2, alpha1, alpha2_prev, probes_local, cg_maxit, lmmse_damp, rho,
              learn_gamw, rtol=1e-5):
        K = self.K
        out = np.zeros((K, hb.LMMSE_NOUT))
        cg = np.zeros((K, 4), dtype=np.int32)
        passes = np.zeros(1, dtype=np.int32)
        pr = np.ascontiguousarray(probes_local, dtype=np.int8)
        if pr.shape != (K, self.Mloc):
            raise ValueError("probes must be (K, Mloc) int8")
        self.ctx.sgv_lmmse(int(it), hb.dptr(hb.f64(gamw)), hb.dptr(hb.f64(gam2)),
                           hb.dptr(hb.f64(alpha1)), hb.dptr(hb.f64(alpha2_prev)),
                           pr.ctypes.data_as(hb._c_i8_p), int(cg_maxit), float(rtol),
                           int(bool(lmmse_damp)), float(rho), int(bool(learn_gamw)), hb.dptr(out),
                           hb.iptr(cg), hb.iptr(passes))
        return out, cg, int(passes[0])

    def step_begin(self, it, flags, em_maxit, sigmas, a, lam, omegas, gam1s, rho, gamw,
                   alpha1_prev, alpha2_prev, probes_local, cg_maxit, out_slot, rtol=1e-5):
        """One outer iteration (sgv_step) on the library's worker thread; returns a
        handle for step_end.  Until then only host work that does not touch the
        context may run (outputs_wait excepted).  With hb.STEP_CHAIN in flags the
        scalar inputs come from the step queued before this one."""
        K = self.K
        sg = hb.f64(sigmas)
        pr = np.ascontiguousarray(probes_local, dtype=np.int8)
        if pr.shape != (K, self.Mloc):
            raise ValueError("probes must be (K, Mloc) int8")
        h = dict(lam=np.array([lam], dtype=np.float64),
                 om=np.array(omegas, dtype=np.float64).copy(),
                 pr=pr, res=np.zeros(1 + 2 * K + 4), ires=np.zeros(2, dtype=np.int32),
                 out=np.zeros((K, hb.LMMSE_NOUT)), cg=np.zeros((K, 4), dtype=np.int32))
        self.ctx.sgv_step_begin(int(it), int(flags), int(em_maxit), len(sg), hb.dptr(sg),
                                hb.dptr(hb.f64(a)), hb.dptr(h["lam"]), hb.dptr(h["om"]),
                                hb.dptr(hb.f64(gam1s)), float(rho), hb.dptr(hb.f64(gamw)),
                                hb.dptr(hb.f64(alpha1_prev)), hb.dptr(hb.f64(alpha2_prev)),
                                pr.ctypes.data_as(hb._c_i8_p), int(cg_maxit), float(rtol),
                                int(out_slot), hb.dptr(h["res"]), hb.iptr(h["ires"]),
                                hb.dptr(h["out"]), hb.iptr(h["cg"]))
        return h

    def step_end(self, h):
        """Wait for the oldest queued step; returns dict(lam, omegas, em_steps,
        em_err, alpha1, gam2, metrics, out, cg, passes) (see sgv_step)."""
        self.ctx.sgv_step_end()
        K = self.K
        return dict(lam=float(h["lam"][0]), omegas=h["om"], em_steps=int(h["ires"][0]),
                    em_err=float(h["res"][0]), mle_status=int(h["ires"][0]),
                    mle_gam=(None if np.isnan(h["res"][0]) else float(h["res"][0])),
                    alpha1=h["res"][1:1 + K].tolist(),
                    gam2=h["res"][1 + K:1 + 2 * K].tolist(), metrics=h["res"][1 + 2 * K:],
                    out=h["out"], cg=h["cg"], passes=int(h["ires"][1]))

    def metrics(self):
        out = np.zeros(4)
        self.ctx.sgv_metrics(hb.dptr(out))
        return out

    def metrics_begin(self):
        """Queue the metric sums behind the denoiser (no host wait)."""
        self.ctx.sgv_metrics_begin()

    def metrics_end(self):
        out = np.zeros(4)
        self.ctx.sgv_metrics_end(hb.dptr(out))
        return out

    # ---- operator seam (tests) ------------------------------------------------
    def ld_matvec(self, ld, V_local):
        V = np.ascontiguousarray(np.atleast_2d(V_local), dtype=np.float64)
        Y = np.empty_like(V)
        self.ctx.sgv_ld_matvec(int(ld), V.shape[0], hb.dptr(V), hb.dptr(Y))
        return Y

    def cg_solve(self, ld, c1, c2, B_local, X0_local, maxiter, rtol=1e-5):
        B = np.ascontiguousarray(np.atleast_2d(B_local), dtype=np.float64)
        X = np.ascontiguousarray(np.atleast_2d(X0_local), dtype=np.float64).copy()
        n = B.shape[0]
        it = np.zeros(n, dtype=np.int32)
        info = np.zeros(n, dtype=np.int32)
        self.ctx.sgv_cg_solve(int(ld), n, hb.dptr(hb.f64(c1)), hb.dptr(hb.f64(c2)), hb.dptr(B),
                              hb.dptr(X), int(maxiter), float(rtol), hb.iptr(it), hb.iptr(info))
        return X, it, info

    def timers(self, reset=False):
        t = np.zeros(hb.TIMERS_N)
        self.ctx.sgv_timers(hb.dptr(t), len(t), int(bool(reset)))
        return dict(ld_ms=t[0], ld_launches=int(t[1]), ld_bytes=t[2], rhs_bytes=t[3],
                    dense_bytes=t[4], aux_bytes=t[5], ld_flops=t[6], wide_flops=t[7],
                    wide_ms=t[8], wide_launches=int(t[9]))

    def exchange_stats(self, reset=False):
        """Cross-rank exchange counters (sgv_exchange_stats): all-gathers issued,
        ms in them, bytes contributed, the EM loops' modes and the cost model's
        last decision, the exact-CG host waits."""
        t = np.zeros(hb.EXCHANGE_STATS_N)
        self.ctx.sgv_exchange_stats(hb.dptr(t), len(t), int(bool(reset)))
        return dict(allgathers=int(t[0]), ms=float(t[1]), bytes=float(t[2]),
                    em_mode={1: "replicated", 0: "per-step", -1: None}[int(t[3])],
                    latency_us=float(t[4]),
                    latency_source={0: "default", 1: "env SGV_XCHG_LAT_US",
                                    2: "measured (sgv_exchange_probe)"}[int(t[12])],
                    transport={1: "rccl", 2: "host", 0: None}[int(t[5])],
                    em_loops_replicated=int(t[6]), em_loops_per_step=int(t[7]),
                    em_pred_replicated_us=float(t[8]), em_pred_per_step_us=float(t[9]),
                    em_pred_steps=float(t[10]), host_wait_ms=float(t[11]),
                    em_replicated_possible=bool(t[13]), em_ms=float(t[14]),
                    em_loops_timed=int(t[15]))

    def comm_info(self):
        """Who the exchange talks to (sgv_comm_info): transport, ranks in the
        communicator and this rank in it (RCCL's own ncclCommCount /
        ncclCommUserRank), the HIP device and its PCI bus id."""
        t = np.zeros(hb.COMM_INFO_N, dtype=np.int32)
        pci = ctypes.create_string_buffer(64)
        self.ctx.sgv_comm_info(hb.iptr(t), len(t), pci, len(pci))
        return dict(transport={1: "rccl", 2: "host", 0: None}[int(t[0])], comm_ranks=int(t[1]),
                    comm_rank=int(t[2]), device=int(t[3]), nranks=int(t[4]),
                    pci_bus_id=pci.value.decode(errors="replace"))

    def exchange_probe(self, reps=20):
        """Measure the exchange's per-all-gather latency (collective) and make the
        maximum over ranks the EM cost model's parameter; returns it in us."""
        us = np.zeros(1)
        self.ctx.sgv_exchange_probe(int(reps), hb.dptr(us))
        return float(us[0])

    def set_ld_packing(self, packed):
        """True: symmetric blocks set/generated from now on are stored packed."""
        self.ctx.sgv_set_ld_packing(int(bool(packed)))

    def ld_block_format(self, ld, b_global):
        f = np.zeros(1, dtype=np.int32)
        self.ctx.sgv_ld_block_format(int(ld), b_global - self.b0, hb.iptr(f))
        return int(f[0])

    def sync(self):
        self.ctx.sgv_sync()

    def read_bw(self, nbytes=8 << 30, reps=5):
        """The device's streaming-read rate in GB/s (sgv_read_bw), best of reps."""
        out = np.zeros(1)
        self.ctx.sgv_read_bw(int(nbytes), int(reps), hb.dptr(out))
        return float(out[0])

    def close(self):
        self.ctx.close()
