"""sgVAMP for summary statistics on MI355X -- drop-in for the reference's
``src/sgvamp.py`` class seam (``VAMP(...)``, ``VAMP.infer(...)``).

Same constructor and ``infer`` arguments, same log lines, same output files
(names, headers, delimiters, value formatting).  Differences by design:

* one process drives all K cohorts of its marker range (the reference runs one
  MPI rank per cohort and all-gathers K x M vectors every iteration,
  src/sgvamp.py:228-233); ``comm`` is the communicator of GPU ranks that each
  own a contiguous range of LD blocks.  Hence ``N`` is the list of per-cohort
  sample sizes (a scalar is accepted for K = 1), and ``R``/``r`` hold every
  cohort (``R``: one ``BlockLD`` shared by all cohorts, or a list of K);
* the LD matrix is handed over as its block-diagonal structure (``BlockLD``:
  dense blocks, or sparse blocks stored as packed bands on the device, so
  windowed/banded LD of any size is accepted); ``R_s = (1 - s) R + s I`` is
  applied inside the LD pass;
* the Hutchinson probes come from ``RandomState(seed + k)`` per cohort, the
  stream the reference draws after ``np.random.seed(seed + rank)``
  (src/sgvamp.py:326; the reference itself never seeds);
* all vector arithmetic runs in libsgvamp_hip.so; there is no CPU fallback.
"""
import csv
import gc
import logging
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import hip_backend as hb
from engine import Engine
from partition import coarsen_blocks, detect_blocks_csr, detect_blocks_dense


# Largest LD block densified on the host (n x n f64).  Symmetric CSR blocks never
# are (they go up as CSR and are stored as a packed band or triangle); this
# bounds non-symmetric sparse blocks and the dense-storage mode.
DENSE_BLOCK_LIMIT = int(os.environ.get("SGV_DENSE_BLOCK_LIMIT", str(16 << 30)))


# Band pieces: a symmetric sparse LD block of at least 2 BAND_PIECE markers
# whose entries stay within BAND_PIECE / 4 of the diagonal (windowed LD over a
# whole chromosome) is cut into pieces of BAND_PIECE markers (the last one up
# to twice that) that ranks own like LD blocks, consecutive pieces coupled by the
# band's corner (sgv_set_ld_coupling).  The cut depends on the matrix only, never
# on the rank count, so 1 and N ranks compute the same sums.  SGV_BAND_PIECE
# (a multiple of 1024) changes the piece length, 0 disables the cut.
BAND_PIECE = int(os.environ.get("SGV_BAND_PIECE", "65536"))
# widest band cut into pieces: a coupling is a dense bw x bw corner on each of
# the two ranks (128 MB at 4,096); wider bands stay one block
BAND_CUT_MAX_BW = 4096


def csr_bandwidth(U, chunk=1 << 16):
    """max(j - i) over the entries (i, j) of a CSR matrix (rows in chunks)."""
    bw = 0
    n = U.shape[0]
    ip, ix = U.indptr, U.indices
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        a, b = int(ip[r0]), int(ip[r1])
        if a == b:
            continue
        rows = np.repeat(np.arange(r0, r1, dtype=np.int64), np.diff(ip[r0:r1 + 1]))
        bw = max(bw, int((ix[a:b].astype(np.int64) - rows).max()))
    return bw


def _dense_guard(n, why):
    need = 8.0 * n * n
    if need > DENSE_BLOCK_LIMIT:
        raise ValueError(
            "LD block of %d markers would be densified (%s): %.1f GB exceeds the dense-block "
            "limit of %.1f GB (SGV_DENSE_BLOCK_LIMIT).  Symmetric sparse/banded LD is stored as "
            "a packed band instead; check that the LD matrix is symmetric and dense storage is "
            "not forced." % (n, why, need / 1e9, DENSE_BLOCK_LIMIT / 1e9))


class BlockLD:
    """Block-diagonal LD matrix: diagonal blocks in marker order, each from a
    dense loader or (sparse sources) a CSR loader.

    Dense blocks go to the device as they are; a symmetric CSR block goes up as
    the CSR of its upper triangle and is stored as a packed band when its entries
    stay near the diagonal (windowed LD: the reference's .npz / PLINK .ld paths,
    src/main.py:199-200,251-257), without ever being densified.  ``s`` is the
    ridge of src/main.py:265 (R_s = (1-s) R + s I); it is applied on the device,
    the blocks stay unregularised."""

    def __init__(self, blocks=None, block_sizes=None, loader=None, s=0.0, csr_loader=None):
        if blocks is not None:
            self._blocks = [np.asarray(b, dtype=np.float64) for b in blocks]
            self.block_sizes = [b.shape[0] for b in self._blocks]
            self._loader = None
        else:
            if block_sizes is None or (loader is None and csr_loader is None):
                raise ValueError("BlockLD needs blocks, or block_sizes and a loader")
            self._blocks = None
            self.block_sizes = [int(b) for b in block_sizes]
            self._loader = loader
        self._csr_loader = csr_loader
        # from_csr: the whole matrix and the block offsets, so pieces and
        # couplings are sliced from it directly (no per-block copies)
        self._csr_src = None
        self._sym = {}
        self.s = float(s)

    @property
    def M(self):
        return int(sum(self.block_sizes))

    def block(self, b):
        """Block b as a dense array."""
        if self._blocks is not None:
            return self._blocks[b]
        if self._loader is None:
            _dense_guard(self.block_sizes[b], "dense block requested")
            return self._csr_loader(b).toarray()
        return np.asarray(self._loader(b), dtype=np.float64)

    def block_csr(self, b):
        """Block b as scipy CSR, or None for a dense source."""
        return None if self._csr_loader is None else self._csr_loader(b).tocsr()

    def symmetric(self, b, A=None):
        """Whether CSR block b is exactly symmetric (cached: one transpose per block)."""
        if b not in self._sym:
            A = self.block_csr(b) if A is None else A
            self._sym[b] = A is not None and (A != A.T).nnz == 0
        return self._sym[b]

    def upload(self, eng, ld, b, packed=True):
        """Put block b of this matrix into LD slot `ld` of the engine."""
        A = self.block_csr(b) if packed else None
        if A is not None:
            if self.symmetric(b, A):
                import scipy.sparse

                U = scipy.sparse.triu(A, format="csr")
                U.sum_duplicates()
                U.sort_indices()
                eng.set_ld_block_csr(ld, b, U)
                return
            _dense_guard(self.block_sizes[b], "the block is not symmetric")
        elif self._csr_loader is not None:
            _dense_guard(self.block_sizes[b], "dense LD storage requested")
        eng.set_ld_block(ld, b, self.block(b))

    def band_width(self, b):
        """Bandwidth of block b (max j - i over its entries), None for a dense
        source or a non-symmetric block."""
        cache = self.__dict__.setdefault("_bw", {})
        if b not in cache:
            A = self.block_csr(b)
            # symmetric: the upper bandwidth is max(j - i) over all entries
            # (straight from indptr / indices: no transpose, no triangle copy)
            cache[b] = csr_bandwidth(A) if A is not None and self.symmetric(b, A) else None
        return cache[b]

    def pieces(self, cuts):
        """The same matrix on a finer partition that cuts band blocks into pieces:
        cuts[b] = the piece sizes of block b (one entry = not cut).  Returns the
        piece-partitioned BlockLD (each piece the diagonal CSR block) and its
        couplings {gb: C} between consecutive pieces of one block (gb = global
        index of the upper piece, C = R[last nr rows of gb][first nc columns of
        gb + 1], nr = min(bw, n_gb), nc = min(bw, n_gb+1))."""
        import scipy.sparse

        sizes, origin = [], []
        for b, ps in enumerate(cuts):
            o = 0
            for n in ps:
                sizes.append(int(n))
                origin.append((b, o))
                o += n
        if len(sizes) == len(self.block_sizes):
            return self, {}
        src = self
        if self._csr_src is not None:
            # slices of the whole matrix: a rank loads only the pieces it owns
            # and no block is copied whole
            Afull, boffs = self._csr_src

            def region(b, r0, r1, c0, c1):
                g = int(boffs[b])
                return Afull[g + r0:g + r1, g + c0:g + c1]
        else:
            last = {}   # the original block last sliced (pieces are loaded in order)

            def region(b, r0, r1, c0, c1):
                if last.get("b") != b:
                    last.clear()
                    last.update(b=b, A=src.block_csr(b))
                return last["A"][r0:r1, c0:c1]

        def loader(k):
            b, o = origin[k]
            return region(b, o, o + sizes[k], o, o + sizes[k])

        L = BlockLD(block_sizes=sizes, s=self.s, csr_loader=loader)
        couplings = {}
        k = 0
        for b, ps in enumerate(cuts):
            if len(ps) > 1:
                bw = max(1, src.band_width(b) or 1)
                o = 0
                for i in range(len(ps) - 1):
                    cut = o + ps[i]
                    nr, nc = min(bw, ps[i]), min(bw, ps[i + 1])
                    C = region(b, cut - nr, cut, cut, cut + nc)
                    couplings[k + i] = (nr, nc, C)   # sparse; densified on upload
                    o = cut
            k += len(ps)
        return L, couplings

    @classmethod
    def from_dense(cls, R, block_sizes=None, s=0.0):
        """A dense M x M LD matrix (the reference's .npy path, src/main.py:201-202);
        block structure detected from its zero pattern unless given."""
        R = np.asarray(R, dtype=np.float64)
        sizes = block_sizes or coarsen_blocks(detect_blocks_dense(R))
        offs = np.concatenate([[0], np.cumsum(sizes)])
        return cls(block_sizes=sizes, loader=lambda b: R[offs[b]:offs[b + 1], offs[b]:offs[b + 1]],
                   s=s)

    @classmethod
    def from_csr(cls, A, block_sizes=None, s=0.0):
        """A scipy sparse LD matrix (the reference's .npz path, src/main.py:199-200,
        and the PLINK .ld assembly, :251-257), any sparsity pattern: blocks are the
        finest block-diagonal partition of its pattern, each kept sparse."""
        A = A.tocsr()
        M = A.shape[0]
        sizes = block_sizes or coarsen_blocks(detect_blocks_csr(A.indptr, A.indices, M))
        offs = np.concatenate([[0], np.cumsum(sizes)])
        if len(sizes) == 1:   # one block: the matrix itself, not a copy
            L = cls(block_sizes=sizes, csr_loader=lambda b: A, s=s)
        else:
            L = cls(block_sizes=sizes,
                    csr_loader=lambda b: A[offs[b]:offs[b + 1], offs[b]:offs[b + 1]], s=s)
        L._csr_src = (A, offs)
        return L

    def regroup(self, sizes):
        """The same matrix on a coarser partition (every boundary of ``sizes`` must
        be a boundary of this matrix)."""
        if list(sizes) == list(self.block_sizes):
            return self
        mine = np.concatenate([[0], np.cumsum(self.block_sizes)])
        theirs = np.concatenate([[0], np.cumsum(sizes)])
        if not set(theirs.tolist()) <= set(mine.tolist()):
            raise ValueError("partition is not a coarsening of the LD block structure")

        def parts(b):
            s0, s1 = theirs[b], theirs[b + 1]
            return [j for j in range(len(self.block_sizes)) if mine[j] >= s0 and mine[j + 1] <= s1]

        if self._csr_loader is not None:
            import scipy.sparse

            return BlockLD(block_sizes=sizes, s=self.s, csr_loader=lambda b: scipy.sparse.block_diag(
                [self.block_csr(j) for j in parts(b)], format="csr"))

        def load(b):
            s0, s1 = theirs[b], theirs[b + 1]
            out = np.zeros((s1 - s0, s1 - s0))
            for j in parts(b):
                o = mine[j] - s0
                n = self.block_sizes[j]
                out[o:o + n, o:o + n] = self.block(j)
            return out

        return BlockLD(block_sizes=sizes, loader=load, s=self.s)


def band_cuts(lds, sizes, piece=None):
    """Piece sizes per block of the common partition (see BAND_PIECE): a block is
    cut when every LD matrix holds it as a symmetric sparse band of bandwidth <=
    min(piece / 4, BAND_CUT_MAX_BW) and it spans at least two pieces.  A function
    of the matrices only (the same for every rank count)."""
    piece = BAND_PIECE if piece is None else int(piece)
    out = []
    for b, n in enumerate(sizes):
        n = int(n)
        if piece <= 0 or n < 2 * piece:
            out.append([n])
            continue
        bws = [L.band_width(b) for L in lds]
        if any(w is None or w > min(piece // 4, BAND_CUT_MAX_BW) for w in bws):
            out.append([n])
            continue
        k = n // piece
        out.append([piece] * (k - 1) + [n - piece * (k - 1)])
    return out


def common_partition(size_lists):
    """Coarsest partition on which every LD matrix is block-diagonal: the
    boundaries shared by all of them."""
    sets = [set(np.concatenate([[0], np.cumsum(s)]).tolist()) for s in size_lists]
    common = sorted(set.intersection(*sets))
    return [int(b - a) for a, b in zip(common[:-1], common[1:])]


class VAMP:
    def __init__(self, N, Nt, M, K, rho, gamw, gam1, a, prior_vars, prior_probs, out_dir,
                 out_name, comm=None, seed=None, device=None, write_files=True, ld_packing=True,
                 exchange=None, mfma_min=None, rs_recurrence=None):
        # src/sgvamp.py:15-31
        self.eps = 1e-32
        self.K = int(K)
        if np.ndim(N) == 0:
            if self.K != 1:
                raise ValueError("N must list the sample size of every cohort when K > 1")
            N = [N]
        self.N_list = [float(n) for n in N]
        if len(self.N_list) != self.K:
            raise ValueError("len(N) != K")
        self.N = self.N_list[0]
        self.Nt = Nt
        self.M = M
        self.L = len(prior_probs)
        if self.L - 1 > hb.MAX_SLABS:
            raise ValueError("at most %d slab components" % hb.MAX_SLABS)
        self.rho = rho
        self.gamw = gamw
        self.gam1 = gam1
        self.a = np.asarray(a, dtype=np.float64)
        self.lam = 1 - prior_probs[0]
        self.sigmas = np.array(prior_vars[1:]) * Nt
        self.omegas = np.array([p / sum(prior_probs[1:]) for p in prior_probs[1:]])
        from comm import SingleComm

        self.comm = comm or SingleComm()
        self.rank = self.comm.Get_rank()
        self.seed = seed
        self.device = device
        self.exchange = exchange
        self.write_files = write_files
        self.ld_packing = ld_packing   # packed symmetric LD storage for symmetric blocks
        self.mfma_min = mfma_min       # None: library default (f64 MFMA pass from 3 RHS)
        self.rs_recurrence = rs_recurrence   # None: library default (R_s x carried, no gamw pass)
        self.gam = None
        self.engine = None
        self.history = []
        self.setup_io(out_dir, out_name)

    # ---- output files (src/sgvamp.py:33-76) -----------------------------------
    def setup_io(self, out_dir, out_name):
        self.out_dir = out_dir
        self.out_name = out_name
        if not self.write_files or self.rank != 0:
            return
        for i in range(self.K):
            with open(os.path.join(self.out_dir, "%s_cohort_%d.csv" % (self.out_name, i + 1)), "w",
                      newline="") as f:
                csv.writer(f, delimiter="\t").writerow(
                    ["it", "gamw", "gam1", "gam2", "alpha1", "alpha2", "lam"])
        with open(os.path.join(self.out_dir, "%s_metrics.csv" % self.out_name), "w", newline="") as f:
            csv.writer(f, delimiter="\t").writerow(["it", "alignment", "l2"])

    def write_params_to_file(self, params, cohort_idx):
        with open(os.path.join(self.out_dir, "%s_cohort_%d.csv" % (self.out_name, cohort_idx + 1)),
                  "a", newline="") as f:
            csv.writer(f, delimiter="\t").writerow(params)

    def write_metrics_to_file(self, metrics):
        with open(os.path.join(self.out_dir, "%s_metrics.csv" % self.out_name), "a", newline="") as f:
            csv.writer(f, delimiter="\t").writerow(metrics)

    def _write_slice(self, fname, local):
        """Native-endian f64, M values, no header.  Each rank writes its marker
        slice at its byte offset, so no gather is needed."""
        path = os.path.join(self.out_dir, fname)
        # written from the array's buffer: .tobytes() would copy under the GIL
        # (writer threads stalled the iteration loop by up to a switch interval)
        buf = memoryview(np.ascontiguousarray(local, dtype=np.float64)).cast("B")
        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            if self.rank == 0:
                os.ftruncate(fd, self.M * 8)
            off, pos = self.engine.marker0 * 8, 0
            while pos < len(buf):
                pos += os.pwrite(fd, buf[pos:], off + pos)
        finally:
            os.close(fd)

    def write_xhat_to_file(self, it, xhat_local):
        self._write_slice("%s_xhat_it_%d.bin" % (self.out_name, it), xhat_local)

    def write_r1_to_file(self, it, r1_local, k):
        self._write_slice("%s_r1_cohort_%d_it_%d.bin" % (self.out_name, k, it), r1_local)

    # ---- set-up ----------------------------------------------------------------
    def _setup(self, R, r, x0):
        K = self.K
        lds = list(R) if isinstance(R, (list, tuple)) else [R] * K
        if len(lds) != K:
            raise ValueError("R must be one BlockLD or a list of K")
        uniq, ld_of = [], []
        for L in lds:
            for j, U in enumerate(uniq):
                if U is L:
                    ld_of.append(j)
                    break
            else:
                uniq.append(L)
                ld_of.append(len(uniq) - 1)
        s_vals = {L.s for L in uniq}
        if len(s_vals) != 1:
            raise ValueError("all LD matrices must use the same ridge s")
        sizes = common_partition([L.block_sizes for L in uniq])
        if sum(sizes) != self.M:
            raise ValueError("LD matrices cover %d markers, M = %d" % (sum(sizes), self.M))
        uniq = [L.regroup(sizes) for L in uniq]
        couplings = [{} for _ in uniq]
        if self.ld_packing:   # band blocks too long for one GPU: coupled pieces
            cuts = band_cuts(uniq, sizes)
            if any(len(c) > 1 for c in cuts):
                split = [L.pieces(cuts) for L in uniq]
                uniq = [x[0] for x in split]
                couplings = [x[1] for x in split]
                sizes = [n for c in cuts for n in c]
        nranks = self.comm.Get_size()
        if len(sizes) < nranks:   # ranks own whole blocks / band pieces
            raise ValueError(
                "%d LD block(s) cannot be spread over %d ranks: run on at most %d GPU(s)%s"
                % (len(sizes), nranks, len(sizes),
                   ", or cut windowed LD into shorter pieces (SGV_BAND_PIECE, a multiple of "
                   "1024, now %d)" % BAND_PIECE if self.ld_packing else ""))
        self.engine = eng = Engine(sizes, K, ld_of, comm=self.comm, device=self.device,
                                          exchange=self.exchange)
        eng.set_ld_packing(self.ld_packing)
        if self.mfma_min is not None:
            eng.set_mfma_min(self.mfma_min)
        if self.rs_recurrence is not None:
            eng.set_rs_recurrence(self.rs_recurrence)
        eng.set_ridge(s_vals.pop())
        for l, L in enumerate(uniq):
            for b in range(eng.b0, eng.b1):
                L.upload(eng, l, b, packed=self.ld_packing)
            for gb in sorted(couplings[l]):   # every rank, every coupling (collective)
                nr, nc, C = couplings[l][gb]
                eng.set_ld_coupling(l, gb, nr, nc, C)
        eng.update_cg_exact()   # the run's CG column sets from the bytes stored (collective)
        rr = np.asarray(r, dtype=np.float64)
        rr = rr.reshape(K, -1) if rr.size == K * self.M else rr
        for k in range(K):
            eng.set_vector(hb.VEC_R, k, rr[k].ravel())
            eng.set_vector(hb.VEC_R1, k, rr[k].ravel())       # r1 = r (:204)
            eng.set_cohort_n(k, self.N_list[k])
        if x0 is not None:
            eng.set_vector(hb.VEC_X0, 0, np.asarray(x0, dtype=np.float64).ravel())

    def _probe_streams(self):
        seed = self.seed
        if seed is None and self.comm.Get_size() > 1:
            seed = self.comm.bcast(int(np.random.SeedSequence().entropy % (2 ** 31))
                                   if self.rank == 0 else None, root=0)
        if seed is None:
            return [np.random.RandomState() for _ in range(self.K)]
        return [np.random.RandomState(seed + k) for k in range(self.K)]

    def attach_engine(self, engine, x0=None):
        """Use an Engine whose LD blocks and r vectors are already on the device
        (e.g. generated there); sets r1 = r (src/sgvamp.py:204) and N_k."""
        self.engine = engine
        self._begun = False
        engine.update_cg_exact()   # collective: every rank attaches its engine
        for k in range(self.K):
            engine.set_vector(hb.VEC_R1, k, engine.get_vector(hb.VEC_R, k))
            engine.set_cohort_n(k, self.N_list[k])
        if x0 is not None:
            engine.set_vector(hb.VEC_X0, 0, np.asarray(x0, dtype=np.float64).ravel())
        self._has_x0 = x0 is not None

    # ---- the outer loop (src/sgvamp.py:196-389) --------------------------------
    def infer(self, R, r, iterations, x0, cg_maxit=500, em_prior_maxit=100, learn_gamw=True,
              lmmse_damp=True, prior_update=None, update_prior_from=1, return_xhat=True):
        self.begin(R, r, x0, cg_maxit=cg_maxit, em_prior_maxit=em_prior_maxit,
                   learn_gamw=learn_gamw, lmmse_damp=lmmse_damp, prior_update=prior_update,
                   update_prior_from=update_prior_from, return_xhat=return_xhat,
                   iterations=iterations)
        for it in range(iterations):
            self.step(it)
        self.finish()
        self.gamws = self._st["gamws"]
        return self._st["xhat1s"]

    def begin(self, R=None, r=None, x0=None, cg_maxit=500, em_prior_maxit=100, learn_gamw=True,
              lmmse_damp=True, prior_update=None, update_prior_from=1, return_xhat=True,
              iterations=None):
        """Initialisation of src/sgvamp.py:198-220 (uploads R, r, x0 unless an
        engine was attached).  `iterations`: the number of step() calls that will
        follow (0, 1, ...); when known, step(it) queues step it + 1 behind it."""
        self._n_iter = iterations
        self._queued = None
        self._xhat_loc = {}        # iteration -> local xhat1 (return_xhat with files)
        self._writes = []          # (iteration, future) of the output-file writers
        self._unwritten = []       # finished iterations whose files are not started
        if self.engine is None:
            self._setup(R, r, x0)
            self._ld_src = R
            self._has_x0 = x0 is not None
        elif getattr(self, "_begun", False):
            self._restart(R, r, x0)
        self._begun = True
        # MLE steps chained behind a non-MLE one start fsolve from the context's
        # gam: make it this object's (a rebuilt engine starts with none, and a
        # drained step may have moved it), as the reference's self.gam carries
        # over between infer() calls (src/sgvamp.py:170-176)
        self.engine.set_mle_gam(self.gam)
        K = self.K
        self._st = dict(gam1=[self.gam1] * K, gamw=[self.gamw] * K, alpha1=[0] * K,
                        alpha2=[0] * K, gamws=[[] for _ in range(K)], xhat1s=[],
                        probes=[hb.ProbeStream(rs) for rs in self._probe_streams()],
                        cg_maxit=cg_maxit,
                        em_prior_maxit=em_prior_maxit, learn_gamw=learn_gamw,
                        lmmse_damp=lmmse_damp, prior_update=prior_update,
                        update_prior_from=update_prior_from, return_xhat=return_xhat)
        # host work that overlaps the GPU: the next iteration's probes are drawn
        # (in stream order) while the current one runs; output files are written
        # by a writer thread (at most one iteration in flight).
        # one thread per cohort stream (numpy's legacy binomial releases the GIL),
        # writers in parallel per file
        self._probe_pool = ThreadPoolExecutor(max_workers=self.K)
        self._write_pool = ThreadPoolExecutor(max_workers=self.K + 1)
        self._out_pool = ThreadPoolExecutor(max_workers=1)   # waits for the output copies
        # per-iteration CSV rows, appended in order off the main thread (the GPU
        # would otherwise idle through each open/append/close).  Rows are handed
        # to the writer just before the LMMSE call, while the main thread waits in
        # C with the GIL released, so the writer's Python never delays a launch.
        self._csv_pool = ThreadPoolExecutor(max_workers=1)
        self._csv_futs = []
        self._csv_rows = []
        self._next_probes = self._submit_probes()
        self._pending_write = None
        # everything allocated so far (imports, LD upload) lives for the whole run:
        # keep it out of the cyclic collector's scans, whose full passes otherwise
        # stall an iteration for milliseconds at a time
        gc.freeze()
        if self.rank == 0:
            logging.debug(f"a = {self.a}")

    def _restart(self, R, r, x0):
        """A further infer()/begin() on this object starts over as the reference's
        infer does (src/sgvamp.py:198-217: r1 = r, xhat1 = xhat2 = Sigma2_u_prev
        = 0); lam/omegas/gam carry over, as they are attributes there too.  A
        different R rebuilds the engine; the same R keeps its LD on the device."""
        if R is not None and R is not getattr(self, "_ld_src", None):
            self.engine.close()
            self.engine = None
            self._setup(R, r, x0)
            self._ld_src = R
            self._has_x0 = x0 is not None
            return
        eng = self.engine
        eng.reset_solver()
        if r is not None:
            rr = np.asarray(r, dtype=np.float64)
            rr = rr.reshape(self.K, -1) if rr.size == self.K * self.M else rr
            for k in range(self.K):
                eng.set_vector(hb.VEC_R, k, rr[k].ravel())
        for k in range(self.K):
            eng.set_vector(hb.VEC_R1, k, eng.get_vector(hb.VEC_R, k))
        if x0 is not None:
            eng.set_vector(hb.VEC_X0, 0, np.asarray(x0, dtype=np.float64).ravel())
            self._has_x0 = True
        elif R is not None or r is not None:   # a new problem without a true signal
            eng.set_vector(hb.VEC_X0, 0, np.zeros(self.M))
            self._has_x0 = False

    def _draw_probe(self, k):
        """u_k = binomial(p=1/2, n=1, size=M)*2-1 (src/sgvamp.py:326), local slice:
        the cohort's RandomState stream, drawn in C (hip_backend.ProbeStream)."""
        sl = self.engine.sl
        return self._st["probes"][k].draw(self.M, sl.start, sl.stop)

    def _submit_probes(self):
        # each cohort's stream is drawn in its own task; the next iteration's draws
        # are submitted only after this iteration's are consumed (stream order kept)
        return [self._probe_pool.submit(self._draw_probe, k) for k in range(self.K)]

    def _write_outputs(self, it, slot):
        """Writer side of one iteration's files: wait for the pinned copy queued by
        sgv_outputs_begin, then write xhat1 and every r1, one file per task."""
        Nt = self.Nt
        out = self.engine.outputs_wait(slot)
        if self._st["return_xhat"] and not hb.ab_env("SGV_STEP") == "phases":
            self._xhat_loc[it] = out[0].copy()   # gathered in order by drain()
        futs = [self._write_pool.submit(lambda: self.write_xhat_to_file(
            it, out[0] / np.sqrt(Nt)))]                                              # :281
        for k in range(self.K):
            futs.append(self._write_pool.submit(
                lambda k=k: self.write_r1_to_file(it, out[k + 1] / np.sqrt(Nt), k + 1)))   # :283
        for f in futs:
            f.result()

    def flush(self):
        """Wait for the output files of every finished iteration."""
        if getattr(self, "_pending_write", None) is not None:
            self._pending_write.result()
            self._pending_write = None
        if getattr(self, "_unwritten", None):
            self._submit_writers()
        for _, f in getattr(self, "_writes", []):
            f.result()
        self._writes = []

    def _queue_csv(self, fn, *args):
        if getattr(self, "_csv_pool", None) is None:
            fn(*args)
            return
        self._csv_rows.append((fn, args))

    def _submit_csv(self):
        if not getattr(self, "_csv_rows", None):
            return
        rows, self._csv_rows = self._csv_rows, []
        keep = []
        for f in self._csv_futs:   # finished appends: re-raise a failure, then drop
            if f.done():
                f.result()
            else:
                keep.append(f)
        self._csv_futs = keep
        self._csv_futs.append(self._csv_pool.submit(lambda: [fn(*a) for fn, a in rows]))

    def drain(self):
        """Wait for every output of the finished iterations: .bin files and CSV rows."""
        if getattr(self, "_queued", None) is not None:   # a step queued past the last call
            self.engine.step_end(self._queued["h"])
            self._queued = None
            # its MLE update (if any) is thrown away: the context's gam follows Python's
            self.engine.set_mle_gam(self.gam)
        self._submit_csv()
        self.flush()
        xl = getattr(self, "_xhat_loc", None)
        if xl:                         # return_xhat with files: xhat1 of every iteration
            for it in sorted(xl):
                full = xl[it]
                if self.comm.Get_size() > 1:
                    full = np.concatenate(self.comm.allgather(full))
                self._st["xhat1s"].append(full.reshape((self.M, 1)))
            xl.clear()
        for f in getattr(self, "_csv_futs", []):
            f.result()                    # re-raise a failed append
        self._csv_futs = []

    def finish(self):
        self.drain()
        for pool in ("_probe_pool", "_write_pool", "_out_pool", "_csv_pool"):
            if getattr(self, pool, None) is not None:
                getattr(self, pool).shutdown(wait=True)
                setattr(self, pool, None)

    def set_iterations(self, iterations):
        """Change the iteration horizon (see begin); call between steps."""
        self._n_iter = iterations

    def _flags(self, it):
        """sgv_step flags of iteration it (the prior update, EM or MLE, runs inside
        the step: src/sgvamp.py:242-259)."""
        st = self._st
        flags = 0
        if it >= st["update_prior_from"]:                             # :242-259
            if st["prior_update"] == "mle":
                flags |= hb.STEP_MLE
            elif st["prior_update"] == "em":
                flags |= hb.STEP_EM
        if it > 0:
            flags |= hb.STEP_DENOISE_DAMP | hb.STEP_ALPHA1_DAMP       # :275-276, 290-291
        if st["lmmse_damp"]:
            flags |= hb.STEP_LMMSE_DAMP
        if st["learn_gamw"]:
            flags |= hb.STEP_LEARN_GAMW
        if self._has_x0:
            flags |= hb.STEP_METRICS                                  # :379-387
        return flags

    def _take_probes(self, rec):
        """This step's probes (drawn in the background, stream order); the next
        step's draws are submitted."""
        t0 = time.perf_counter()
        fs = self._next_probes
        u = fs[0].result()[None] if self.K == 1 else np.stack([f.result() for f in fs])   # :326
        rec["wait_probes_ms"] = (time.perf_counter() - t0) * 1e3
        self._next_probes = self._submit_probes()
        return u

    def _flush_until(self, last, rec=None):
        """Wait for the file writers of iterations <= last (their pinned output
        slot is reused by iteration last + OUT_SLOTS)."""
        t0 = time.perf_counter()
        keep = []
        for i, f in self._writes:
            if i <= last:
                f.result()
            else:
                keep.append((i, f))
        self._writes = keep
        if rec is not None:
            rec["wait_write_ms"] = rec.get("wait_write_ms", 0.0) + (time.perf_counter() - t0) * 1e3

    def _submit_writers(self):
        for i in self._unwritten:
            self._writes.append((i, self._out_pool.submit(self._write_outputs, i,
                                                          i % hb.OUT_SLOTS)))
        self._unwritten = []

    def _can_chain(self, nxt):
        st = self._st
        return (self._n_iter is not None and nxt < self._n_iter
                and not (st["return_xhat"] and not self.write_files)
                and hb.ab_env("SGV_STEP") != "nochain")

    def _begin_step(self, it, flags, u, chain):
        st = self._st
        return self.engine.step_begin(
            it, flags | (hb.STEP_CHAIN if chain else 0), st["em_prior_maxit"], self.sigmas,
            self.a, self.lam, self.omegas, np.array(st["gam1"], dtype=np.float64), self.rho,
            st["gamw"], st["alpha1"], st["alpha2"], u, st["cg_maxit"],
            it % hb.OUT_SLOTS if self.write_files else -1)

    def step(self, it):
        """One outer iteration, src/sgvamp.py:222-387.  The device phases (EM
        loop, denoiser, LMMSE) run as one sgv_step on the library's worker
        thread.  While it runs this thread queues the next iteration's step behind
        it (sgv_step's inputs chained from this one's results, when the iteration
        count is known), starts the file writers of finished iterations and hands
        the CSV rows to their writer -- so the GPU does not wait for Python
        between iterations.  Logs follow the step in the reference's order."""
        if hb.ab_env("SGV_STEP") == "phases":
            return self._step_phases(it)
        st = self._st
        eng = self.engine
        K, M, Nt, rho, rank = self.K, self.M, self.Nt, self.rho, self.rank
        gam1, gamw, alpha1, alpha2 = st["gam1"], st["gamw"], st["alpha1"], st["alpha2"]
        t_it = time.perf_counter()
        rec = dict(it=it)
        # lazy %-arguments: nothing is formatted unless the level is enabled
        if rank == 0:
            logging.info("\n -----ITERATION %s -----", it)
        gam1s = np.array(gam1, dtype=np.float64)                      # :228-233
        if rank == 0:
            logging.debug("gam1s=%s", gam1s)
            logging.info("...Data from all ranks collected")

        q = self._queued
        if q is not None:             # queued by the previous step(), already running
            if q["it"] != it:
                raise RuntimeError("step(%d) called, step(%d) was queued" % (it, q["it"]))
            self._queued = None
            h, flags = q["h"], q["flags"]
            rec.update(q["rec"])
        else:
            flags = self._flags(it)
            if flags & hb.STEP_MLE:
                eng.set_mle_gam(self.gam)   # the step chain carries it on from here
            u = self._take_probes(rec)
            if self.write_files:
                self._flush_until(it - hb.OUT_SLOTS, rec)
            h = self._begin_step(it, flags, u, chain=False)
        # host work overlapping the step (touches no device state)
        self._submit_writers()
        self._submit_csv()            # previous iterations' rows
        if self._can_chain(it + 1):
            rec1 = {}
            flags1 = self._flags(it + 1)
            u1 = self._take_probes(rec1)
            if self.write_files:
                self._flush_until(it + 1 - hb.OUT_SLOTS, rec1)
            self._queued = dict(it=it + 1, h=self._begin_step(it + 1, flags1, u1, chain=True),
                                flags=flags1, rec=rec1)
        try:
            r = eng.step_end(h)
        except Exception:
            # the step queued behind a failed one fails too (its chained inputs are
            # gone): collect it so no later drain() completes it, then re-raise
            if self._queued is not None:
                try:
                    eng.step_end(self._queued["h"])
                except Exception:  # noqa: BLE001 -- the first error is the one raised
                    pass
                self._queued = None
            raise
        if self.write_files:
            self._unwritten.append(it)

        if flags & hb.STEP_EM:
            self.lam, self.omegas = r["lam"], r["omegas"]
            rec["em_steps"] = r["em_steps"]
            if rank == 0:
                logging.info("...Updating prior parameters using EM")
                logging.info("... prior-learning EM algorithm performed %s steps "
                             "and had final relative error = %0.9f", r["em_steps"], r["em_err"])
        elif flags & hb.STEP_MLE:                                     # :244-247
            if rank == 0:
                logging.info("...Updating prior parameters using MLE")
            warn = self._mle_result(r["mle_status"], r["lam"], r["omegas"], r["mle_gam"])
            if warn:
                rec["mle_warning"] = warn
        if rank == 0:
            logging.debug("lam=%s", self.lam)
            logging.debug("omegas=%s", self.omegas)
            logging.debug("sigmas=%s", self.sigmas)
            logging.info("...Denoising")
        if st["return_xhat"] and not self.write_files:
            xhat_loc = eng.get_vector(hb.VEC_XHAT1)    # LMMSE leaves xhat1 as denoised
            full = xhat_loc
            if self.comm.Get_size() > 1:
                full = np.concatenate(self.comm.allgather(xhat_loc))
            st["xhat1s"].append(full.reshape((M, 1)))
        # (with files, the writer keeps xhat1 from the output copy: see _write_outputs)
        gam2 = r["gam2"]
        for k in range(K):
            alpha1[k] = r["alpha1"][k]
        if rank == 0:
            logging.debug("[rank = %s] alpha1 = %s", rank, alpha1[0])
            logging.debug("[rank = %s] gam2 = %s", rank, gam2[0])
        for k in range(K):
            logging.info("...LMMSE cohort %s", k)
        out, cg, passes = r["out"], r["cg"], r["passes"]
        rec.update(cg_iters=cg[:, [0, 2]].tolist(), cg_info=cg[:, [1, 3]].tolist(),
                   ld_passes=passes)
        for k in range(K):
            if cg[k, 1] > 0:
                logging.info("Rank %s WARNING: CG 1 convergence after %s "
                             "iterations not achieved!", k, cg[k, 1])
            if cg[k, 3] > 0:
                logging.info("Rank %s WARNING: CG 2 convergence after %s "
                             "iterations not achieved!", k, cg[k, 3])
            alpha2[k] = out[k, hb.O_ALPHA2]
            gam1[k] = out[k, hb.O_GAM1]
            if st["learn_gamw"]:
                gamw[k] = float(out[k, hb.O_GAMW])                    # :363-364
        if rank == 0:
            logging.debug("[rank = %s] alpha2 = %s", rank, alpha2[0])
            logging.debug("gamw = %0.9f \n", gamw[0])
        for k in range(K):
            st["gamws"][k].append(gamw[k])                            # :373
            gamw[k] = max(gamw[k], 1.0)                               # :374
            if rank == 0 and self.write_files:
                self._queue_csv(self.write_params_to_file,
                                [it, gamw[k], gam1[k], gam2[k], alpha1[k], alpha2[k],
                                 self.lam], k)                        # :377
        if self._has_x0:                                              # :379-387
            s = r["metrics"]
            alignment = s[0] / np.sqrt(s[1]) / np.sqrt(s[3])
            l2 = np.sqrt(s[2]) / np.sqrt(s[3])
            rec["metrics"] = (alignment, l2)
            if rank == 0:
                logging.debug("Alignment(xhat1, x0) = %0.9f \n", alignment)
                logging.debug("L2_error(xhat1, x0) = %0.9f \n", l2)
                if self.write_files:
                    self._queue_csv(self.write_metrics_to_file, [it, alignment, l2])
        rec.update(gamw=list(gamw), gam1=list(gam1), gam2=gam2, alpha1=list(alpha1),
                   alpha2=list(alpha2), lam=self.lam, wall_s=time.perf_counter() - t_it)
        self.history.append(rec)
        return rec

    def _step_phases(self, it):
        """One outer iteration, src/sgvamp.py:222-387, one host call per phase
        (SGV_STEP=phases: the A/B reference for step(); same results)."""
        st = self._st
        eng = self.engine
        K, M, Nt, rho, rank = self.K, self.M, self.Nt, self.rho, self.rank
        gam1, gamw, alpha1, alpha2 = st["gam1"], st["gamw"], st["alpha1"], st["alpha2"]
        t_it = time.perf_counter()
        rec = dict(it=it)
        # lazy %-arguments: nothing is formatted unless the level is enabled
        if rank == 0:
            logging.info("\n -----ITERATION %s -----", it)
        gam1s = np.array(gam1, dtype=np.float64)                      # :228-233
        if rank == 0:
            logging.debug("gam1s=%s", gam1s)
            logging.info("...Data from all ranks collected")

        if it >= st["update_prior_from"]:                             # :242-259
            if st["prior_update"] == "mle":
                if rank == 0:
                    logging.info("...Updating prior parameters using MLE")
                warn = self.prior_update_mle(gam1s)
                if warn:
                    rec["mle_warning"] = warn
            elif st["prior_update"] == "em":
                if rank == 0:
                    logging.info("...Updating prior parameters using EM")
                self.lam, self.omegas, steps, err = eng.em(
                    gam1s, self.a, self.sigmas, st["em_prior_maxit"], self.lam, self.omegas)
                rec["em_steps"] = steps
                if rank == 0:
                    logging.info("... prior-learning EM algorithm performed %s steps "
                                 "and had final relative error = %0.9f", steps, err)
        if rank == 0:
            logging.debug("lam=%s", self.lam)
            logging.debug("omegas=%s", self.omegas)
            logging.debug("sigmas=%s", self.sigmas)
            logging.info("...Denoising")

        alpha1_prev = list(alpha1)
        der_sum = eng.denoise(gam1s, self.a, self.lam, self.omegas, self.sigmas, rho,
                              damp=it > 0)                            # :273-276, 285
        if self.write_files:
            # the previous iteration's files are written (its pinned slot is free),
            # then this iteration's copies are queued without a wait
            t0 = time.perf_counter()
            self.flush()
            rec["wait_write_ms"] = (time.perf_counter() - t0) * 1e3
            eng.outputs_begin(it % 2)
            self._pending_write = self._out_pool.submit(self._write_outputs, it, it % 2)
        if self._has_x0:
            eng.metrics_begin()       # of xhat1, read back at the end (:379-387)
        if st["return_xhat"]:
            xhat_loc = eng.get_vector(hb.VEC_XHAT1)
            full = xhat_loc
            if self.comm.Get_size() > 1:
                full = np.concatenate(self.comm.allgather(xhat_loc))
            st["xhat1s"].append(full.reshape((M, 1)))
        gam2 = [0.0] * K
        for k in range(K):
            a1 = der_sum[k] / M                                       # np.mean (:285)
            if it > 0:
                a1 = rho * a1 + (1 - rho) * alpha1_prev[k]            # :290-291
            alpha1[k] = a1
            gam2[k] = gam1[k] * (1 - a1) / a1                         # :305
        if rank == 0:
            logging.debug("[rank = %s] alpha1 = %s", rank, alpha1[0])
            logging.debug("[rank = %s] gam2 = %s", rank, gam2[0])
        for k in range(K):
            logging.info("...LMMSE cohort %s", k)
        t0 = time.perf_counter()
        u = np.stack([f.result() for f in self._next_probes])        # :326
        rec["wait_probes_ms"] = (time.perf_counter() - t0) * 1e3
        self._next_probes = self._submit_probes()
        self._submit_csv()            # previous iteration's rows, written during the LMMSE
        out, cg, passes = eng.lmmse(it, gamw, gam2, alpha1, alpha2, u, st["cg_maxit"],
                                    st["lmmse_damp"], rho, st["learn_gamw"])
        rec.update(cg_iters=cg[:, [0, 2]].tolist(), cg_info=cg[:, [1, 3]].tolist(),
                   ld_passes=passes)
        for k in range(K):
            if cg[k, 1] > 0:
                logging.info("Rank %s WARNING: CG 1 convergence after %s "
                             "iterations not achieved!", k, cg[k, 1])
            if cg[k, 3] > 0:
                logging.info("Rank %s WARNING: CG 2 convergence after %s "
                             "iterations not achieved!", k, cg[k, 3])
            alpha2[k] = out[k, hb.O_ALPHA2]
            gam1[k] = out[k, hb.O_GAM1]
            if st["learn_gamw"]:
                gamw[k] = float(out[k, hb.O_GAMW])                    # :363-364
        if rank == 0:
            logging.debug("[rank = %s] alpha2 = %s", rank, alpha2[0])
            logging.debug("gamw = %0.9f \n", gamw[0])
        for k in range(K):
            st["gamws"][k].append(gamw[k])                            # :373
            gamw[k] = max(gamw[k], 1.0)                               # :374
            if rank == 0 and self.write_files:
                self._queue_csv(self.write_params_to_file,
                                [it, gamw[k], gam1[k], gam2[k], alpha1[k], alpha2[k],
                                 self.lam], k)                        # :377
        if self._has_x0:                                              # :379-387
            s = eng.metrics_end()
            alignment = s[0] / np.sqrt(s[1]) / np.sqrt(s[3])
            l2 = np.sqrt(s[2]) / np.sqrt(s[3])
            rec["metrics"] = (alignment, l2)
            if rank == 0:
                logging.debug("Alignment(xhat1, x0) = %0.9f \n", alignment)
                logging.debug("L2_error(xhat1, x0) = %0.9f \n", l2)
                if self.write_files:
                    self._queue_csv(self.write_metrics_to_file, [it, alignment, l2])
        rec.update(gamw=list(gamw), gam1=list(gam1), gam2=gam2, alpha1=list(alpha1),
                   alpha2=list(alpha2), lam=self.lam, wall_s=time.perf_counter() - t_it)
        self.history.append(rec)
        return rec

    MLE_WARNINGS = {hb.MLE_NOT_CONVERGED: "WARNING: fsolve not converged. No prior update!",
                    hb.MLE_NEGATIVE: "WARNING: Negative values in MLE. No prior update!"}

    def _mle_result(self, status, lam, omegas, gam):
        """Take an MLE prior update's outcome (src/sgvamp.py:180-194): the new
        lam/omegas/gam, or the reference's warning and no update."""
        if status:
            msg = self.MLE_WARNINGS[status]
            if self.rank == 0:
                logging.info(msg)
            return msg
        self.lam, self.omegas, self.gam = lam, np.array(omegas), gam
        return None

    def prior_update_mle(self, gam1s):
        """src/sgvamp.py:162-194 in one library call (sgv_mle_update): scipy's
        fsolve (MINPACK hybrd, restated in csrc/hybrd.cpp) on Lagrangian_der
        (:139-160), whose K x M x L marker sums run on the device."""
        status, lam, omegas, gam = self.engine.mle_update(gam1s, self.a, self.sigmas, self.lam,
                                                          self.omegas, self.gam)
        warn = self._mle_result(status, lam, omegas, gam)
        self.engine.set_mle_gam(self.gam)   # a later chained MLE step starts from it
        return warn
