"""ORACLE -- CPU restatement of the reference sgVAMP hot path (TEST INFRASTRUCTURE).

This module is a checker, never a product path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The shipped path (``sgvamp-py_amd/``) never imports anything from
``oracle/`` and fails loudly when its HIP library is missing.

Parity pinning
--------------
Pinned against the golden fixtures in ``tests/golden/*.npz``; those were
produced by importing the reference (/root/reference/src/sgvamp.py) in the build
container with ``tests/golden/make_golden.py``.  ``tests/test_oracle_golden.py``
checks this restatement against every fixture.

What it restates (reference file:line)
---------------------------------------
* ``VAMP.__init__``  src/sgvamp.py:15-31     (lam, sigmas*Nt, omegas)
* ``denoiser_meta``  src/sgvamp.py:93-102    vectorised over markers
* ``der_denoiser_meta`` src/sgvamp.py:104-114 vectorised, all K cohorts at once
* ``prior_update_em`` src/sgvamp.py:116-136  + driver loop :247-259
* ``Lagrangian_der`` / ``prior_update_mle`` src/sgvamp.py:139-194 (scipy
  ``optimize.fsolve``, MINPACK hybrd, as the reference calls it)
* ``VAMP.infer``      src/sgvamp.py:196-389  all K cohort ranks in one process
* scipy 1.15.3 ``cg`` scipy/sparse/linalg/_isolve/iterative.py:305-422 (the
  reference's ``con_grad``, src/sgvamp.py:7,316,332): rtol 1e-5, atol 0,
  strict ``<`` stop test, warm-start residual only when ``x0.any()``.

Arithmetic is IEEE f64 and follows the reference's operation order where that
is cheap (builtin ``sum`` over slabs is sequential, ``np.mean`` for alpha1).
The LD product uses ``A p = gamw*(R_s p) + gam2*p`` instead of materialising
``A = gamw*R_s + gam2*I`` (src/sgvamp.py:312): same math, different rounding.

Two reduction modes for the M-length dot products:
* ``"numpy"``   np.dot / np.linalg.norm, as the reference (default);
* ``"blocked"`` per-LD-block partial sums added in block order -- the order the
  HIP path uses so that 1/2/4/8-GPU runs agree bit for bit.  ``BlockedComm``
  lets a sharded run (each rank owning a contiguous range of blocks) exchange
  per-block partials (tests/test_dist_gloo.py).
"""
import numpy as np


# ----------------------------------------------------------------------------
# element-wise pieces
# ----------------------------------------------------------------------------
def _seqsum_last(x):
    """Python builtin sum() over the last axis: ((0 + x0) + x1) + ...
    (src/sgvamp.py:95,99,101 use builtin sum over the L-1 slabs)."""
    acc = x[..., 0].copy()
    for l in range(1, x.shape[-1]):
        acc = acc + x[..., l]
    return acc


def _seqsum(v):
    acc = v[0]
    for t in v[1:]:
        acc = acc + t
    return acc


def denoiser_terms(r1s, gam1s, a, lam, omegas, sigmas):
    """Shared sub-expressions of denoiser_meta / der_denoiser_meta
    (src/sgvamp.py:95-101 and :105-111), vectorised over markers.

    r1s (K, M); returns dict of (M, L-1) / (M,) arrays."""
    ag = a * gam1s                                        # (K,)
    sum_ag = _seqsum(list(ag))                            # builtin sum, :95
    s2 = 1.0 / (sum_ag + 1.0 / sigmas)                    # (L-1,)  :95
    inner = r1s[0] * ag[0]                                # np.inner(rs, a*gam1s) :96,
    for k in range(1, r1s.shape[0]):                      # sequential over k (the HIP
        inner = inner + r1s[k] * ag[k]                    # kernel's order)
    mu = inner[:, None] * s2[None, :]                     # (M, L-1)
    ratio = mu * mu / s2[None, :]                         # :97
    m = np.argmax(ratio, axis=1)                          # first max, as ndarray.argmax
    rows = np.arange(mu.shape[0])
    s2m = s2[m]
    mum = mu[rows, m]
    EXP = np.exp(0.5 * (mu * mu * s2m[:, None] - (mum * mum)[:, None] * s2[None, :])
                 / (s2[None, :] * s2m[:, None]))          # :98
    sq = np.sqrt(s2 / sigmas)                             # (L-1,)
    Num = lam * _seqsum_last(omegas * EXP * mu * sq)      # :99
    EXP2 = np.exp(-0.5 * (mum ** 2 / s2m))                # :100
    Den = (1 - lam) * EXP2 + lam * _seqsum_last(omegas * EXP * sq)   # :101
    return dict(s2=s2, mu=mu, EXP=EXP, sq=sq, Num=Num, Den=Den)


def denoiser_meta(r1s, gam1s, a, lam, omegas, sigmas):
    """xhat1 (M,) -- src/sgvamp.py:93-102 applied per marker (:273)."""
    t = denoiser_terms(r1s, gam1s, a, lam, omegas, sigmas)
    return t["Num"] / t["Den"]


def der_denoiser_meta(r1s, gam1s, a, lam, omegas, sigmas):
    """(K, M) derivative for every cohort k -- src/sgvamp.py:104-114, with the
    rank's factor a[rank]*gam1s[rank] (:112-113) taken for each k."""
    t = denoiser_terms(r1s, gam1s, a, lam, omegas, sigmas)
    s2, mu, EXP, sq, Num, Den = (t[k] for k in ("s2", "mu", "EXP", "sq", "Num", "Den"))
    out = np.empty((len(a), mu.shape[0]))
    for k in range(len(a)):
        DerNum = lam * _seqsum_last(omegas * EXP * (mu * mu + s2) * a[k] * gam1s[k] * sq)
        DerDen = lam * _seqsum_last(omegas * mu * EXP * a[k] * gam1s[k] * sq)
        out[k] = (DerNum * Den - DerDen * Num) / (Den * Den)
    return out


def prior_update_em(r1s, gam1s, a, lam, omegas, sigmas, red=None, M_total=None):
    """One EM step -- src/sgvamp.py:116-136.  Returns (lam, omegas).
    With a "blocked" reducer the marker sums go through it (sharded runs)."""
    K, M = r1s.shape
    Lm1 = len(sigmas)
    prior_vars0 = sigmas.reshape(1, 1, Lm1)
    gam1s_rs = gam1s.reshape(K, 1, 1)
    gam1invs = 1.0 / gam1s_rs
    r1s_rs = r1s.reshape(K, M, 1)
    r2 = np.power(r1s_rs, 2)
    exp_max = (-r2 / 2 / (prior_vars0 + gam1invs)).max(axis=2).reshape(K, M, 1)   # :127
    xi = lam * omegas.reshape(1, 1, Lm1) * np.exp(-r2 / 2 / (prior_vars0 + gam1invs) - exp_max) \
        / np.sqrt(gam1invs + prior_vars0)                                        # :128
    sum_xi = xi.sum(axis=2).reshape(K, M, 1)                                     # :129
    xi_tilde = xi / sum_xi                                                       # :130
    pi = 1.0 / (1.0 + (1 - lam) * np.exp(-r2 / 2 * gam1s_rs - exp_max) / np.sqrt(gam1invs) / sum_xi)  # :131
    if red is None or red.mode == "numpy":
        lam_new = np.mean(np.average(pi, axis=0, weights=a))                     # :134
        omegas_new = np.sum(pi * xi_tilde * a.reshape(K, 1, 1), axis=(0, 1)) \
            / np.sum(pi * a.reshape(K, 1, 1), axis=(0, 1))                       # :136
        return lam_new, omegas_new
    ones = np.ones(M)
    avg = np.average(pi, axis=0, weights=a).ravel()
    lam_new = red.dot(avg, ones) / M_total
    num = (pi * xi_tilde * a.reshape(K, 1, 1)).sum(axis=0)                      # (M, L-1)
    den = (pi * a.reshape(K, 1, 1)).sum(axis=0).ravel()
    omegas_new = np.array([red.dot(num[:, l], ones) for l in range(Lm1)]) / red.dot(den, ones)
    return lam_new, omegas_new


def lagrangian_der(x, omega0, sigma2, r1s, gam1s, a, exp_max, red=None):
    """src/sgvamp.py:139-160 (Lagrangian_der).  ``exp_max`` (:152) depends only
    on r1s, gam1s and sigma2, so it is computed once per update (mle_exp_max).
    With a "blocked" reducer the marker sums go through it (sharded runs)."""
    K, M = r1s.shape
    L = len(sigma2)
    y = np.zeros(L + 1)
    omega = x[:L]
    gam = x[L]
    prior_vars0 = sigma2.reshape(1, 1, L)
    gam1invs = 1.0 / gam1s.reshape(K, 1, 1)
    r1s_rs = r1s.reshape(K, M, 1)
    probs = np.exp(-np.power(r1s_rs, 2) / 2 / (prior_vars0 + gam1invs) - exp_max) \
        / np.sqrt(prior_vars0 + gam1invs)                                        # :153
    Num = a.reshape(K, 1, 1) * probs                                             # :154
    Den = np.sum(probs * omega.reshape(1, 1, L), axis=2).reshape(K, M, 1)        # :155
    if red is None or red.mode == "numpy":
        S = np.sum(Num / Den, axis=(0, 1))                                       # :157
    else:
        T = Num / Den
        t = T[0]
        for k in range(1, K):
            t = t + T[k]
        ones = np.ones(M)
        S = np.array([red.dot(t[:, l], ones) for l in range(L)])
    y[:L] = S + (omega0 - 1) / omega + gam                                       # :157
    y[L] = sum(omega) - 1.0                                                      # :158
    return y


def mle_exp_max(r1s, gam1s, sigma2, red=None):
    """src/sgvamp.py:152: max over (k, m, l) of (-r1^2 / 2) / (sigma2_l + 1/gam1_k)."""
    K, M = r1s.shape
    L = len(sigma2)
    v = sigma2.reshape(1, 1, L) + 1.0 / gam1s.reshape(K, 1, 1)
    local = (-np.power(r1s.reshape(K, M, 1), 2) / 2 / v).max()
    if red is not None and red.comm is not None:
        return float(np.max(red.comm.allgather_blocks(np.array([local]))))
    return local


def prior_update_mle(r1s, gam1s, a, lam, omegas, sigmas, gam, red=None):
    """src/sgvamp.py:162-194.  Returns (lam, omegas, gam, warning or None)."""
    from scipy import optimize

    L = len(sigmas) + 1
    omega0 = np.zeros(L)
    omega0[0] = 1 - lam
    omega0[1:] = lam * omegas
    sigma2 = np.zeros(L)
    sigma2[0] = 1e-16
    sigma2[1:] = sigmas
    x0 = np.zeros(L + 1)
    x0[:-1] = omega0
    x0[-1] = 1 if gam is None else gam
    em = mle_exp_max(r1s, gam1s, sigma2, red)
    x, _, ier, _ = optimize.fsolve(func=lagrangian_der, x0=x0,
                                   args=(omega0, sigma2, r1s, gam1s, a, em, red), full_output=True)
    if ier != 1:                                                                 # :183-186
        return lam, omegas, gam, "WARNING: fsolve not converged. No prior update!"
    if any(s <= 0 for s in x[:-1]):                                              # :187-190
        return lam, omegas, gam, "WARNING: Negative values in MLE. No prior update!"
    x[:-1] /= sum(x[:-1])                                                        # :191
    lam = 1 - x[0]
    omegas = np.array([w / sum(x[1:-1]) for w in x[1:-1]])
    return lam, omegas, x[L], None


# ----------------------------------------------------------------------------
# reductions
# ----------------------------------------------------------------------------
class Reducer:
    """M-length dot products.  mode "numpy" = np.dot; mode "blocked" = per-block
    partial sums (block = LD block of the marker partition) added in global
    block order.  A sharded run owns blocks [b0, b1) of ``bounds`` and hands
    its per-block partials to ``comm.allgather_blocks`` (None = single rank)."""

    def __init__(self, mode="numpy", bounds=None, comm=None):
        self.mode, self.bounds, self.comm = mode, bounds, comm

    def dot(self, x, y):
        if self.mode == "numpy":
            return np.dot(x, y)
        part = np.array([np.dot(x[s0:s1], y[s0:s1])
                         for s0, s1 in zip(self.bounds[:-1], self.bounds[1:])])
        if self.comm is not None:
            part = self.comm.allgather_blocks(part)
        return _seqsum(list(part)) if len(part) else 0.0

    def norm(self, x):
        return np.sqrt(self.dot(x, x))     # numpy/linalg/_linalg.py: sqrt(dot(x, x))

    def mean(self, x, n_total):
        if self.mode == "numpy":
            return np.mean(x)
        return self.dot(x, np.ones_like(x)) / n_total


# ----------------------------------------------------------------------------
# LD operator and CG
# ----------------------------------------------------------------------------
class BlockLD:
    """Block-diagonal LD matrix R (the build's storage model): dense f64 blocks
    on the diagonal.  ``s`` applies R_s = (1-s) R + s I (src/main.py:265)."""

    def __init__(self, blocks, s=0.0):
        self.blocks = [np.ascontiguousarray(b, dtype=np.float64) for b in blocks]
        self.bounds = np.cumsum([0] + [b.shape[0] for b in self.blocks])
        self.s = s

    def matvec_R(self, v):
        out = np.empty_like(v)
        for (s0, s1), B in zip(zip(self.bounds[:-1], self.bounds[1:]), self.blocks):
            out[s0:s1] = B @ v[s0:s1]
        return out

    def matvec_Rs(self, v):
        if self.s == 0.0:
            return self.matvec_R(v)
        return (1 - self.s) * self.matvec_R(v) + self.s * v

    def matmat_Rs(self, V):
        """Column by column (each column exactly its matvec_Rs: the batched
        reference algebra, cg_scipy_batch, then equals cg_scipy bit for bit)."""
        V = np.asarray(V, dtype=np.float64)
        return np.stack([self.matvec_Rs(np.ascontiguousarray(V[:, i])) for i in range(V.shape[1])],
                        axis=1)


class CoupledLD:
    """Band pieces with corner couplings: the layout that lets ranks share one
    band block (one chromosome of windowed LD, src/main.py:199-200,251-257;
    the build's sgv_set_ld_coupling).  This rank holds pieces gb0 .. gb0 +
    len(pieces) - 1 (CSR, diagonal blocks of the band) and knows every
    coupling {gb: (nr, nc, C)}, C = R[last nr rows of gb][first nc columns of
    gb + 1].  R v = per-piece products, then the couplings added to the rows
    they reach (gb's tail: C v_{gb+1}[:nc], gb + 1's head: C^T v_gb[-nr:]);
    with a communicator the neighbours' head / tail rows come from an all-
    gather, so 1 and N ranks add the same terms in the same order."""

    def __init__(self, pieces, couplings, gb0=0, comm=None, s=0.0):
        self.pieces = [P.tocsr() for P in pieces]
        self.couplings = dict(couplings)
        self.gb0 = gb0
        self.comm = comm
        self.s = s
        self.sizes = [P.shape[0] for P in self.pieces]
        self.bounds = np.cumsum([0] + self.sizes)
        self.hmax = max([max(nr, nc) for nr, nc, _ in self.couplings.values()] or [0])

    def matvec_R(self, v):
        out = np.empty_like(v)
        nb = len(self.pieces)
        for k, P in enumerate(self.pieces):
            out[self.bounds[k]:self.bounds[k + 1]] = P @ v[self.bounds[k]:self.bounds[k + 1]]
        head = {self.gb0 + k: v[self.bounds[k]:self.bounds[k] + self.hmax] for k in range(nb)}
        tail = {self.gb0 + k: v[max(self.bounds[k], self.bounds[k + 1] - self.hmax):self.bounds[k + 1]]
                for k in range(nb)}
        if self.comm is not None:   # the neighbours' pieces next to this rank's
            first, last = self.gb0, self.gb0 + nb - 1
            got = self.comm.allgather((first, head[first], last, tail[last]))
            for f, h, l_, t in got:
                head.setdefault(f, h)
                tail.setdefault(l_, t)
        for gb in sorted(self.couplings):
            nr, nc, C = self.couplings[gb]
            k = gb - self.gb0
            if 0 <= k < nb:                  # gb's tail rows
                out[self.bounds[k + 1] - nr:self.bounds[k + 1]] += C @ head[gb + 1][:nc]
            if 0 <= k + 1 < nb:              # gb + 1's head rows
                out[self.bounds[k + 1]:self.bounds[k + 1] + nc] += C.T @ tail[gb][-nr:]
        return out

    def matvec_Rs(self, v):
        if self.s == 0.0:
            return self.matvec_R(v)
        return (1 - self.s) * self.matvec_R(v) + self.s * v


_PANEL_LIB = []


def _panel_lib():
    """oracle/libpanel_ld.so (oracle/panel_ld.c, built by oracle/Makefile): the
    same block product in C, ~3x NumPy's tall-skinny GEMMs per core; None when
    it is not built (the NumPy form below is the same operator)."""
    if not _PANEL_LIB:
        import ctypes
        import os

        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpanel_ld.so")
        lib = None
        if os.path.exists(path) and os.environ.get("SGV_ORACLE_NUMPY") != "1":
            lib = ctypes.CDLL(path)
            lib.oracle_panel_block_matmat.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                                      ctypes.c_int, ctypes.c_void_p,
                                                      ctypes.c_void_p]
            lib.oracle_panel_block_matmat.restype = ctypes.c_int
            lib.oracle_panel_range_matmat.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                                      ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                                      ctypes.c_void_p, ctypes.c_void_p]
            lib.oracle_panel_range_matmat.restype = ctypes.c_int
        _PANEL_LIB.append(lib)
    return _PANEL_LIB[0]


def _oracle_workers():
    """Threads for the host panel products: the job's CPU share
    (OMP_NUM_THREADS: 16 on the MI355X pool, where os.cpu_count() shows the
    whole machine), at most 16; SGV_ORACLE_THREADS overrides."""
    import os

    v = os.environ.get("SGV_ORACLE_THREADS") or os.environ.get("OMP_NUM_THREADS")
    try:
        n = int(v) if v else (os.cpu_count() or 1)
    except ValueError:
        n = 1
    return max(1, min(16, n))


class _blas_single_thread:
    """One BLAS thread per call while the pool runs (threadpoolctl when present;
    otherwise BLAS keeps its own setting -- the sums are the same, only slower)."""

    def __enter__(self):
        try:
            from threadpoolctl import threadpool_limits

            self._cm = threadpool_limits(limits=1, user_api="blas")
            self._cm.__enter__()
        except Exception:
            self._cm = None
        return self

    def __exit__(self, *exc):
        if self._cm is not None:
            self._cm.__exit__(*exc)
        return False


class PanelLD:
    """Block-diagonal LD held as the upper triangle of each block in panels of
    ``H`` rows -- panel g of a block stores rows r0 = H*g .. r0+h-1 over columns
    r0 .. n-1, its h x h diagonal block in full (the device's packed layout,
    DESIGN.md section 3) -- so a full-size configuration (M = 1e6: 63.5 GB
    instead of 125 GB dense) fits the test host.  Same operator as BlockLD on
    the same blocks (R_s = (1-s) R + s I, src/main.py:265); only the summation
    order of the products differs.  ``matmat_R`` takes several columns at once
    (one BLAS call per panel and part, not per column)."""

    def __init__(self, s=0.0, H=256):
        self.s, self.H = s, H
        self.blocks = []          # (offset, n, [panel arrays])
        self.sizes = []
        self._inner_pool = None

    @property
    def bounds(self):
        return np.cumsum([0] + self.sizes)

    def add_block(self, B):
        """Append the next diagonal block (a dense symmetric n x n array; only
        its upper triangle is kept)."""
        n = B.shape[0]
        off = int(sum(self.sizes))
        panels = [np.ascontiguousarray(B[r0:min(r0 + self.H, n), r0:], dtype=np.float64)
                  for r0 in range(0, n, self.H)]
        self.blocks.append((off, n, panels))
        self.sizes.append(n)

    RANGE = 16   # panels per task of the C product (a fixed cut: sums do not depend on threads)

    def _block_product(self, blk, V, Y):
        off, n, panels = blk
        Vb, Yb = V[off:off + n], Y[off:off + n]
        lib = _panel_lib()
        if lib is not None and V.shape[1] <= 16:
            import ctypes

            Vc = np.ascontiguousarray(Vb)
            ptrs = (ctypes.c_void_p * len(panels))(*[P.ctypes.data for P in panels])
            # the block's panels in fixed ranges, each into its own partial, the
            # partials added in range order; the ranges of a block with few
            # blocks in the product run on the pool too (C3: 8 blocks, 16 cores)
            cuts = list(range(0, len(panels), self.RANGE)) + [len(panels)]
            parts = [np.empty_like(Vc) for _ in cuts[:-1]]

            def run(i):
                rc = lib.oracle_panel_range_matmat(n, self.H, ptrs, cuts[i], cuts[i + 1],
                                                   Vc.shape[1], Vc.ctypes.data, parts[i].ctypes.data)
                if rc != 0:
                    raise RuntimeError("oracle_panel_range_matmat failed")

            if len(parts) > 1 and self._inner_pool is not None:
                list(self._inner_pool.map(run, range(len(parts))))
            else:
                for i in range(len(parts)):
                    run(i)
            acc = parts[0]
            for q in parts[1:]:
                acc += q
            Yb[...] = acc
            return
        for g, P in enumerate(panels):
            r0 = g * self.H
            h = P.shape[0]
            Yb[r0:r0 + h] += P @ Vb[r0:]                     # rows of the panel
            if P.shape[1] > h:
                Yb[r0 + h:] += P[:, h:].T @ Vb[r0:r0 + h]    # their transposes

    def matmat_R(self, V):
        """Blocks are independent (each writes only its own rows), so they run
        on a thread pool (numpy releases the GIL in BLAS), one BLAS thread per
        call: the order of the additions inside a block does not depend on the
        worker count.  A full-size pass over 63.5 GB then streams at the host's
        memory rate instead of one core's (the north-star gate in the driver's
        GPU suite)."""
        V = np.asarray(V, dtype=np.float64)
        Y = np.zeros_like(V)
        nw = _oracle_workers()
        self._inner_pool = None
        if nw <= 1 or len(self.blocks) < 2:
            for blk in self.blocks:
                self._block_product(blk, V, Y)
            return Y
        from concurrent.futures import ThreadPoolExecutor

        with _blas_single_thread(), ThreadPoolExecutor(nw) as ex:
            if len(self.blocks) < nw:   # few big blocks: their panel ranges on a second pool
                with ThreadPoolExecutor(nw) as inner:
                    self._inner_pool = inner
                    list(ex.map(lambda blk: self._block_product(blk, V, Y), self.blocks))
                    self._inner_pool = None
            else:
                list(ex.map(lambda blk: self._block_product(blk, V, Y), self.blocks))
        return Y

    def matvec_R(self, v):
        return self.matmat_R(np.asarray(v)[:, None])[:, 0]

    def matmat_Rs(self, V):
        if self.s == 0.0:
            return self.matmat_R(V)
        return (1 - self.s) * self.matmat_R(V) + self.s * V

    def matvec_Rs(self, v):
        return self.matmat_Rs(np.asarray(v)[:, None])[:, 0]


class CsrLD:
    """A general sparse LD matrix R (scipy CSR, any sparsity pattern): the
    reference's own operator for .npz and PLINK .ld inputs (src/main.py:199-200,
    251-257), whose products are CSR mat-vecs inside scipy's cg
    (src/sgvamp.py:312-316,332).  ``s`` as in BlockLD."""

    def __init__(self, A, s=0.0):
        self.A = A.tocsr()
        self.s = s

    def matvec_R(self, v):
        return self.A @ v

    def matvec_Rs(self, v):
        if self.s == 0.0:
            return self.matvec_R(v)
        return (1 - self.s) * self.matvec_R(v) + self.s * v


def banded_ld(n, bw, seed=0, decay=None, taps=40):
    """Test input: an exactly symmetric, positive semi-definite LD-like matrix
    with unit diagonal whose entries vanish for |i - j| > bw (CSR), bandwidth
    exactly bw.  R = B B^T with B lower-banded -- row i mixes the "haplotype
    factors" i - k for k in a fixed set of `taps` offsets that includes 0 and bw
    -- scaled to unit diagonal: the shape of windowed LD (PLINK --ld-window)
    without its truncation artefacts, cheap to build at any n."""
    import scipy.sparse

    rs = np.random.RandomState(seed)
    decay = decay or max(bw / 3.0, 1.0)
    offs = {0, bw}
    if bw > 1:
        offs |= set(rs.choice(np.arange(1, bw), min(bw - 1, taps), replace=False).tolist())
    rows, cols, vals = [], [], []
    for k in sorted(offs):
        i = np.arange(k, n)
        rows.append(i)
        cols.append(i - k)
        vals.append(rs.normal(size=n - k) * np.exp(-k / decay) + (1.0 if k == 0 else 0.0))
    B = scipy.sparse.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                                shape=(n, n))
    R = (B @ B.T).tocsr()
    d = 1.0 / np.sqrt(R.diagonal())
    R = scipy.sparse.diags(d) @ R @ scipy.sparse.diags(d)
    R = ((R + R.T) * 0.5).tocsr()
    R.sum_duplicates()
    R.sort_indices()
    return R


def cg_scipy(matvec, b, x0, maxiter, red, rtol=1e-5):
    """scipy 1.15.3 cg (iterative.py:375-422), with counters.
    Returns (x, info, n_iter, n_matvec)."""
    x = np.array(x0, dtype=np.float64).ravel().copy()
    b = np.asarray(b, dtype=np.float64).ravel()
    bnrm2 = red.norm(b)
    atol = max(0.0, rtol * bnrm2)
    if bnrm2 == 0:
        return b.copy(), 0, 0, 0
    nmv = 0
    if x.any():
        r = b - matvec(x)
        nmv += 1
    else:
        r = b.copy()
    rho_prev, p = None, None
    for it in range(maxiter):
        if red.norm(r) < atol:
            return x, 0, it, nmv
        rho_cur = red.dot(r, r)
        if it > 0:
            beta = rho_cur / rho_prev
            p *= beta
            p += r
        else:
            p = r.copy()
        q = matvec(p)
        nmv += 1
        alpha = rho_cur / red.dot(p, q)
        x += alpha * p
        r -= alpha * q
        rho_prev = rho_cur
    return x, maxiter, maxiter, nmv


def cg_track(matvec_rs, gw, gam2, b, x0, rsx0, maxiter, red, rtol=1e-5):
    """cg_scipy with A = gw*R_s + gam2*I that also carries R_s x along the
    iterates: x_k = x_0 + sum alpha_i p_i  =>  R_s x_k = R_s x_0 + sum alpha_i (R_s p_i),
    and every iteration's pass computes R_s p_i anyway.  The warm-start residual
    uses the carried R_s x_0 (no extra pass).  Same iterates as cg_scipy in exact
    arithmetic; rounding differs from a direct product.  Returns
    (x, rsx, info, n_iter, n_matvec)."""
    x = np.array(x0, dtype=np.float64).ravel().copy()
    rsx = np.array(rsx0, dtype=np.float64).ravel().copy()
    b = np.asarray(b, dtype=np.float64).ravel()
    bnrm2 = red.norm(b)
    atol = max(0.0, rtol * bnrm2)
    if bnrm2 == 0:
        return b.copy(), np.zeros_like(b), 0, 0, 0
    nmv = 0
    if x.any():
        r = b - (gw * rsx + gam2 * x)
    else:
        r = b.copy()
    rho_prev, p = None, None
    for it in range(maxiter):
        if red.norm(r) < atol:
            return x, rsx, 0, it, nmv
        rho_cur = red.dot(r, r)
        if it > 0:
            beta = rho_cur / rho_prev
            p *= beta
            p += r
        else:
            p = r.copy()
        y = matvec_rs(p)
        q = gw * y + gam2 * p
        nmv += 1
        alpha = rho_cur / red.dot(p, q)
        x += alpha * p
        rsx += alpha * y
        r -= alpha * q
        rho_prev = rho_cur
    return x, rsx, maxiter, maxiter, nmv


def cg_scipy_batch(ld_cols, gws, gam2s, B, X0, maxiter, red, rtol=1e-5):
    """cg_scipy on A_j = gws[j]*R_s + gam2s[j]*I for several columns in lockstep
    -- the reference's own algebra (src/sgvamp.py:312-316,332: one con_grad per
    column, the warm start's residual from a direct product, no carried R_s x)
    with the products of the columns still iterating on one LD matrix taken
    together.  An LD object whose matmat_Rs gives each column the bits it gives
    alone (PanelLD with oracle/panel_ld.c) makes every column exactly its
    cg_scipy run.  Returns (X, info, n_iter, n_matvec) per column."""
    nc = len(B)
    X = [np.array(x, dtype=np.float64).ravel().copy() for x in X0]
    Bv = [np.asarray(b, dtype=np.float64).ravel() for b in B]
    info, n_it, n_mv = [maxiter] * nc, [maxiter] * nc, [0] * nc
    atol, R, P, rho_prev, active = [0.0] * nc, [None] * nc, [None] * nc, [None] * nc, []
    warm = []
    for j in range(nc):
        bnrm2 = red.norm(Bv[j])
        atol[j] = max(0.0, rtol * bnrm2)
        if bnrm2 == 0:
            X[j], info[j], n_it[j] = Bv[j].copy(), 0, 0
            continue
        if X[j].any():
            warm.append(j)
        else:
            R[j] = Bv[j].copy()
        active.append(j)

    def products(js, vecs):
        out = {}
        for ld, cols in ld_cols:
            cols = [j for j in cols if j in js]
            if cols:
                Y = ld.matmat_Rs(np.stack([vecs[j] for j in cols], axis=1))
                for i, j in enumerate(cols):
                    out[j] = gws[j] * Y[:, i] + gam2s[j] * vecs[j]
        return out

    for j, q in products(warm, X).items():          # r = b - A x0 (iterative.py:392)
        R[j] = Bv[j] - q
        n_mv[j] += 1
    for it in range(maxiter):
        still = []
        for j in active:
            if red.norm(R[j]) < atol[j]:
                info[j], n_it[j] = 0, it
                continue
            rho_cur = red.dot(R[j], R[j])
            if it > 0:
                P[j] *= rho_cur / rho_prev[j]
                P[j] += R[j]
            else:
                P[j] = R[j].copy()
            rho_prev[j] = rho_cur
            still.append(j)
        active = still
        if not active:
            break
        for j, q in products(active, P).items():
            n_mv[j] += 1
            alpha = rho_prev[j] / red.dot(P[j], q)
            X[j] += alpha * P[j]
            R[j] -= alpha * q
    return X, info, n_it, n_mv


def cg_track_batch(ld_cols, gws, gam2s, B, X0, RSX0, maxiter, red, rtol=1e-5):
    """cg_track on several columns in lockstep: every column runs scipy 1.15.3's
    cg (iterative.py:375-422) with its own stop test, scalars and iteration
    count, exactly as alone; only the LD products of the columns still iterating
    on one LD matrix are taken together, Y = R_s P, one multi-column product per
    LD matrix and iteration (``ld_cols``: list of (ld, [column indices]) with an
    ``ld.matmat_Rs``).  Returns (X, RSX, info, n_iter, n_matvec) per column."""
    nc = len(B)
    X = [np.array(x, dtype=np.float64).ravel().copy() for x in X0]
    RSX = [np.array(x, dtype=np.float64).ravel().copy() for x in RSX0]
    Bv = [np.asarray(b, dtype=np.float64).ravel() for b in B]
    info, n_it, n_mv = [maxiter] * nc, [maxiter] * nc, [0] * nc
    atol, R, P, rho_prev, active = [0.0] * nc, [None] * nc, [None] * nc, [None] * nc, []
    for j in range(nc):
        bnrm2 = red.norm(Bv[j])
        atol[j] = max(0.0, rtol * bnrm2)
        if bnrm2 == 0:
            X[j], RSX[j], info[j], n_it[j] = Bv[j].copy(), np.zeros_like(Bv[j]), 0, 0
            continue
        R[j] = Bv[j] - (gws[j] * RSX[j] + gam2s[j] * X[j]) if X[j].any() else Bv[j].copy()
        active.append(j)
    for it in range(maxiter):
        still = []
        for j in active:
            if red.norm(R[j]) < atol[j]:
                info[j], n_it[j] = 0, it
                continue
            rho_cur = red.dot(R[j], R[j])
            if it > 0:
                P[j] *= rho_cur / rho_prev[j]
                P[j] += R[j]
            else:
                P[j] = R[j].copy()
            rho_prev[j] = rho_cur
            still.append(j)
        active = still
        if not active:
            break
        for ld, cols in ld_cols:
            cols = [j for j in cols if j in active]
            if not cols:
                continue
            Y = ld.matmat_Rs(np.stack([P[j] for j in cols], axis=1))
            for i, j in enumerate(cols):
                y = Y[:, i]
                q = gws[j] * y + gam2s[j] * P[j]
                n_mv[j] += 1
                alpha = rho_prev[j] / red.dot(P[j], q)
                X[j] += alpha * P[j]
                RSX[j] += alpha * y
                R[j] -= alpha * q
    return X, RSX, info, n_it, n_mv


# ----------------------------------------------------------------------------
# probe vectors (the reference's global RNG, seeded per cohort rank)
# ----------------------------------------------------------------------------
class ProbeStream:
    """u = binomial(p=1/2, n=1, size=M)*2-1 from RandomState(seed + k):
    identical to the stream src/sgvamp.py:326 sees after np.random.seed(seed+k)."""

    def __init__(self, seed, K):
        self.rs = [np.random.RandomState(seed + k) for k in range(K)]

    def draw(self, k, M):
        return self.rs[k].binomial(p=1 / 2, n=1, size=M) * 2 - 1


# ----------------------------------------------------------------------------
# the outer loop
# ----------------------------------------------------------------------------
def infer(lds, ld_of, r_list, N_list, iterations, *, rho=0.5, gamw=5.0, gam1=1e-6,
          prior_vars=(0.0, 1.0), prior_probs=(0.99, 0.01), x0=None, cg_maxit=500,
          em_prior_maxit=100, learn_gamw=True, lmmse_damp=False, prior_update="em",
          update_prior_from=1, seed=0, reducer=None, M_total=None, probe=None,
          rs_recurrence=False, batched=False, progress=None):
    """All K cohorts of src/sgvamp.py:196-389 in one process.

    batched: run the 2K CG solves of an iteration in lockstep (cg_track_batch:
    each column exactly scipy's cg, the LD products of the columns on one LD
    matrix taken together) -- the same per-column arithmetic apart from the
    products' summation order, at the cost of max(CG iterations) LD sweeps
    instead of their sum; LD objects with matmat_Rs.  With rs_recurrence off
    (the reference's algebra) the columns run cg_scipy_batch and gamw's R_s
    products are direct, taken together per LD matrix.
    For full-size configurations (tests/test_gpu_configs.py).

    rs_recurrence: carry R_s x through both CG solves (cg_track) instead of the
    direct products of the warm start and gamw learning (:352, :359) -- the
    build's pass-saving variant; exact in exact arithmetic.

    lds: list of BlockLD; ld_of[k]: which LD cohort k uses; r_list[k]: (M,)
    x0: true signal in reference scale (beta*sqrt(N_0)) or None.
    Sharded use: pass the local marker slice of everything, ``reducer`` with a
    comm, ``M_total`` the global M and ``probe`` a callable (k, it) -> local u.
    Returns a dict with per-iteration trajectories."""
    K = len(r_list)
    M = len(r_list[0])
    M_tot = M if M_total is None else M_total
    red = reducer or Reducer()
    Nt = sum(N_list)
    a = np.array(N_list, dtype=np.float64) / sum(N_list)                 # main.py:287
    lam = 1 - prior_probs[0]                                             # sgvamp.py:26
    sigmas = np.array(prior_vars[1:]) * Nt                              # :27
    omegas = np.array([p / sum(prior_probs[1:]) for p in prior_probs[1:]])   # :28
    probes = probe or (lambda k, it, _s=ProbeStream(seed, K): _s.draw(k, M))

    r = [np.asarray(v, dtype=np.float64).ravel() for v in r_list]
    r1 = [v.copy() for v in r]                                           # :204
    xhat1 = np.zeros(M)
    xhat2 = [np.zeros(M) for _ in range(K)]
    sig2u_prev = [np.zeros(M) for _ in range(K)]
    rs_x2 = [np.zeros(M) for _ in range(K)]       # R_s xhat2 (rs_recurrence)
    rs_s2u = [np.zeros(M) for _ in range(K)]      # R_s Sigma2_u
    gam1_k = [gam1] * K
    gamw_k = [gamw] * K
    alpha1_k = [0] * K
    alpha2_k = [0] * K
    traj = dict(xhat=[], r1=[], csv=[[] for _ in range(K)], metrics=[], cg_iters=[],
                cg_info=[], em_steps=[], gamws=[[] for _ in range(K)], ld_passes=[],
                mle_warnings=[])
    gam_mle = None                                                       # :31 self.gam

    for it in range(iterations):
        if progress is not None:   # test harness heartbeat (long full-size runs)
            progress(it)
        gam1s = np.array(gam1_k, dtype=np.float64)                      # :228-233
        r1s = np.stack(r1)
        if it >= update_prior_from and prior_update == "em":            # :242-259
            for em_it in range(em_prior_maxit):
                old_omegas, old_lam = omegas, lam
                lam, omegas = prior_update_em(r1s, gam1s, a, lam, omegas, sigmas, red, M_tot)
                om_err = np.linalg.norm(omegas - old_omegas) / np.linalg.norm(old_omegas)
                lam_err = np.abs(lam - old_lam) / lam
                if om_err < 1e-6 and lam_err < 1e-6:
                    break
            traj["em_steps"].append(em_it + 1)
        elif it >= update_prior_from and prior_update == "mle":          # :244-246
            lam, omegas, gam_mle, warn = prior_update_mle(r1s, gam1s, a, lam, omegas, sigmas,
                                                          gam_mle, red)
            if warn:
                traj["mle_warnings"].append(warn)

        xhat1_prev = xhat1
        xhat1 = denoiser_meta(r1s, gam1s, a, lam, omegas, sigmas)       # :273
        if it > 0:
            xhat1 = rho * xhat1 + (1 - rho) * xhat1_prev                # :275-276
        traj["xhat"].append(xhat1 / np.sqrt(Nt))                        # :281
        traj["r1"].append([v / np.sqrt(Nt) for v in r1])                # :283
        der = der_denoiser_meta(r1s, gam1s, a, lam, omegas, sigmas)     # :285
        it_cg, it_info, passes = [], [], 0
        if batched:
            pre = []
            for k in range(K):                     # :285-313 for every cohort first
                alpha1 = red.mean(der[k], M_tot)
                if it > 0:
                    alpha1 = rho * alpha1 + (1 - rho) * alpha1_k[k]
                alpha1_k[k] = alpha1
                gam2 = gam1_k[k] * (1 - alpha1) / alpha1
                r2 = (xhat1 - alpha1 * r1[k]) / (1 - alpha1)
                mu2 = gamw_k[k] * r[k] + gam2 * r2
                pre.append((alpha1, gam2, r2, mu2, probes(k, it)))   # :326 (own stream)
            cols = {}
            for k in range(K):
                cols.setdefault(ld_of[k], []).extend([2 * k, 2 * k + 1])
            ldc = [(lds[l], c) for l, c in cols.items()]
            gws2 = [gamw_k[k] for k in range(K) for _ in (0, 1)]
            g2s = [pre[k][1] for k in range(K) for _ in (0, 1)]
            Bs = [v for k in range(K) for v in (pre[k][3], pre[k][4])]
            X0s = [v for k in range(K) for v in (xhat2[k], sig2u_prev[k])]
            if rs_recurrence:
                X, RSX, info, nit, nmv = cg_track_batch(
                    ldc, gws2, g2s, Bs, X0s,
                    [v for k in range(K) for v in (rs_x2[k], rs_s2u[k])], cg_maxit, red)
            else:   # the reference's algebra, columns in lockstep (cg_scipy_batch)
                X, info, nit, nmv = cg_scipy_batch(ldc, gws2, g2s, Bs, X0s, cg_maxit, red)
                RSX = [None] * (2 * K)
            xs_new = []
            for k in range(K):
                x2 = X[2 * k]
                if lmmse_damp:                                          # :322-323
                    x2 = rho * x2 + (1 - rho) * xhat2[k]
                xs_new.append(x2)
            if not rs_recurrence and learn_gamw:
                # gamw learning's R_s xhat2 and R_s Sigma2_u as direct products
                # (:352,359), every cohort's taken together per LD matrix
                for l, c in cols.items():
                    ks = sorted({j // 2 for j in c})
                    V = np.stack([xs_new[k] for k in ks] + [X[2 * k + 1] for k in ks], axis=1)
                    Y = lds[l].matmat_Rs(V)
                    for i, k in enumerate(ks):   # contiguous, as a matvec's result
                        RSX[2 * k] = np.ascontiguousarray(Y[:, i])
                        RSX[2 * k + 1] = np.ascontiguousarray(Y[:, len(ks) + i])
                        nmv[2 * k] += 1
                        nmv[2 * k + 1] += 1
            for k in range(K):
                alpha1, gam2, r2, _, u = pre[k]
                x2, rx2, s2u, rs2 = xs_new[k], RSX[2 * k], X[2 * k + 1], RSX[2 * k + 1]
                if lmmse_damp and rs_recurrence:                        # :322-323
                    rx2 = rho * rx2 + (1 - rho) * rs_x2[k]
                rs_x2[k], xhat2[k] = rx2, x2
                sig2u_prev[k], rs_s2u[k] = s2u, rs2
                uf = u.astype(np.float64)
                TrSigma2 = red.dot(uf, s2u)                             # :338
                alpha2 = gam2 * TrSigma2 / M_tot                        # :340
                if lmmse_damp:
                    alpha2 = rho * alpha2 + (1 - rho) * alpha2_k[k]     # :345-346
                alpha2_k[k] = alpha2
                gam1_k[k] = gam2 * (1 - alpha2) / alpha2                # :347
                r1[k] = (x2 - alpha2 * r2) / (1 - alpha2)               # :348
                gw = gamw_k[k]
                if learn_gamw:                                          # :350-364
                    N = N_list[k]
                    z = N - 2 * red.dot(x2, r[k]) + red.dot(x2, rx2)
                    if z < 0:
                        z = 0
                    TrRSigma2 = red.dot(uf, rs2)
                    gw = 1 / (z / N + TrRSigma2 / N)
                traj["gamws"][k].append(gw)                             # :373
                gamw_k[k] = max(gw, 1.0)                                # :374
                traj["csv"][k].append([it, gamw_k[k], gam1_k[k], gam2, alpha1, alpha2, lam])
                it_cg.append((nit[2 * k], nit[2 * k + 1]))
                it_info.append((info[2 * k], info[2 * k + 1]))
                passes += nmv[2 * k] + nmv[2 * k + 1]
        for k in range(0 if batched else K):
            alpha1 = red.mean(der[k], M_tot)
            if it > 0:
                alpha1 = rho * alpha1 + (1 - rho) * alpha1_k[k]         # :290-291
            alpha1_k[k] = alpha1
            gam2 = gam1_k[k] * (1 - alpha1) / alpha1                    # :305
            r2 = (xhat1 - alpha1 * r1[k]) / (1 - alpha1)                # :310
            L = lds[ld_of[k]]
            gw = gamw_k[k]

            def A(p, L=L, gw=gw, gam2=gam2):                            # :312
                return gw * L.matvec_Rs(p) + gam2 * p
            mu2 = gw * r[k] + gam2 * r2                                 # :313
            x2_prev = xhat2[k]
            if rs_recurrence:
                x2, rx2, info1, n1, m1 = cg_track(L.matvec_Rs, gw, gam2, mu2, x2_prev, rs_x2[k],
                                                  cg_maxit, red)
                if lmmse_damp:
                    rx2 = rho * rx2 + (1 - rho) * rs_x2[k]
                rs_x2[k] = rx2
            else:
                x2, info1, n1, m1 = cg_scipy(A, mu2, x2_prev, cg_maxit, red)    # :316
            if lmmse_damp:
                x2 = rho * x2 + (1 - rho) * x2_prev                     # :322-323
            xhat2[k] = x2
            u = probes(k, it)                                           # :326
            if rs_recurrence:
                s2u, rs2, info2, n2, m2 = cg_track(L.matvec_Rs, gw, gam2, u, sig2u_prev[k],
                                                   rs_s2u[k], cg_maxit, red)
                rs_s2u[k] = rs2
            else:
                s2u, info2, n2, m2 = cg_scipy(A, u, sig2u_prev[k], cg_maxit, red)   # :332
            sig2u_prev[k] = s2u
            uf = u.astype(np.float64)
            TrSigma2 = red.dot(uf, s2u)                                 # :338
            alpha2 = gam2 * TrSigma2 / M_tot                            # :340
            if lmmse_damp:
                alpha2 = rho * alpha2 + (1 - rho) * alpha2_k[k]         # :345-346
            alpha2_k[k] = alpha2
            gam1_k[k] = gam2 * (1 - alpha2) / alpha2                    # :347
            r1[k] = (x2 - alpha2 * r2) / (1 - alpha2)                   # :348
            if learn_gamw:                                              # :350-364
                N = N_list[k]
                rx = rs_x2[k] if rs_recurrence else L.matvec_Rs(x2)
                z = N - 2 * red.dot(x2, r[k]) + red.dot(x2, rx)
                if z < 0:
                    z = 0
                TrRSigma2 = red.dot(uf, rs_s2u[k] if rs_recurrence else L.matvec_Rs(s2u))
                gw = 1 / (z / N + TrRSigma2 / N)
            traj["gamws"][k].append(gw)                                 # :373
            gamw_k[k] = max(gw, 1.0)                                    # :374
            traj["csv"][k].append([it, gamw_k[k], gam1_k[k], gam2, alpha1, alpha2, lam])   # :377
            it_cg.append((n1, n2))
            it_info.append((info1, info2))
            passes += m1 + m2 + (2 if learn_gamw else 0)
        traj["cg_iters"].append(it_cg)
        traj["cg_info"].append(it_info)
        traj["ld_passes"].append(passes)
        if x0 is not None:                                              # :379-387
            x0v = np.asarray(x0, dtype=np.float64).ravel()
            nx = red.norm(xhat1)
            n0 = red.norm(x0v)
            alignment = red.dot(xhat1, x0v) / nx / n0
            l2 = red.norm(xhat1 - x0v) / n0
            traj["metrics"].append([it, alignment, l2])
    traj["final"] = dict(lam=lam, omegas=omegas, gamw=gamw_k, gam1=gam1_k, xhat2=xhat2,
                         sig2u=sig2u_prev)
    return traj
