"""Golden fixtures generated from the reference (see make_golden.py)."""
import glob
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def exact_ld(X, blocks):
    """Block-diagonal LD of genotypes X (N x M, values 0/1/2) exactly as
    G^T G with G = (X - mean) / (std * sqrt(N)) (the simulation recipe,
    simulation/sim_gen_phen_mult.py:40,53-55), formed so every machine gets the
    same bits: the integer Gram S = X^T X is exact in f64 BLAS (integer partial
    sums < 2^53, any order), column sums and N*sum(x^2) - (sum x)^2 are exact
    integers, and R_ij = (N S_ij - s_i s_j) / (sqrt(v_i) sqrt(v_j)) uses only
    correctly rounded operations.  Returns the dense M x M matrix."""
    X = np.asarray(X, dtype=np.float64)
    N, M = X.shape
    s1 = X.sum(axis=0).astype(np.int64)                      # exact (integers)
    s2 = (X * X).sum(axis=0).astype(np.int64)
    v = N * s2 - s1 * s1                                     # N^2 var, exact
    sq = np.sqrt(v.astype(np.float64))
    R = np.zeros((M, M))
    o = 0
    for n in blocks:
        Xb = X[:, o:o + n]
        S = np.rint(Xb.T @ Xb).astype(np.int64)              # exact integer Gram
        num = N * S - np.outer(s1[o:o + n], s1[o:o + n])     # exact
        R[o:o + n, o:o + n] = num.astype(np.float64) / np.outer(sq[o:o + n], sq[o:o + n])
        o += n
    return R


def ld_checksum(R, blocks):
    import hashlib

    h = hashlib.sha256()
    o = 0
    for n in blocks:
        h.update(np.ascontiguousarray(R[o:o + n, o:o + n]).tobytes())
        o += n
    return h.hexdigest()


def regen_inputs(flags):
    """The LD of an exact-recipe fixture, regenerated from its seed (the draws of
    make_golden.make_inputs in the same order)."""
    rs = np.random.RandomState(flags["seed"])
    M, Ns, blocks = flags["M"], flags["N"], flags["blocks"]
    lam_sim = flags.get("lam_sim", None)
    cm = flags["_cm"]
    rs.choice(M, cm, replace=False)
    rs.normal(0, 1.0, cm)
    Rs = []
    for k, N in enumerate(Ns):
        X = rs.binomial(2, 0.4, size=(N, M)).astype(np.float64)
        if flags["distinct_ld"] or k == 0:
            Rs.append(exact_ld(X, blocks))
        if not flags["distinct_ld"]:
            break
        rs.normal(0.0, 1.0, size=N)                           # the noise draw of cohort k
    del lam_sim
    return Rs


_REGEN = {}   # regenerated LD of the exact-recipe fixtures, per process


def case_names():
    return sorted(os.path.splitext(os.path.basename(p))[0]
                  for p in glob.glob(os.path.join(HERE, "*.npz")))


class Case:
    """One fixture: inputs (LD blocks, r, N, flags, beta) and the reference's
    recorded outputs (xhat/r1 per iteration, cohort/metrics CSV, CG/EM counts)."""

    def __init__(self, name):
        d = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
        self.name = name
        self.flags = json.loads(str(d["flags"]))
        f = self.flags
        self.K = len(f["N"])
        self.M = f["M"]
        self.N = list(f["N"])
        self.block_sizes = list(f["blocks"])
        self.beta = d["beta"]
        self.r = d["r"]
        sizes2 = [n * n for n in self.block_sizes]
        offs = np.cumsum([0] + sizes2)
        self.ld_blocks = []
        if "R_blocks" in d.files:
            for row in d["R_blocks"]:
                self.ld_blocks.append([row[offs[b]:offs[b + 1]].reshape(n, n)
                                       for b, n in enumerate(self.block_sizes)])
        elif name in _REGEN:
            self.ld_blocks = _REGEN[name]
        else:                         # exact recipe: regenerate, check the checksum
            f["_cm"] = int(np.count_nonzero(self.beta))
            want = [str(x) for x in d["R_sha256"]]
            bounds = np.cumsum([0] + self.block_sizes)
            for l, R in enumerate(regen_inputs(f)):
                got = ld_checksum(R, self.block_sizes)
                if got != want[l]:
                    raise RuntimeError("%s: regenerated LD %d checksum %s != fixture %s"
                                       % (name, l, got, want[l]))
                self.ld_blocks.append([R[bounds[b]:bounds[b + 1], bounds[b]:bounds[b + 1]].copy()
                                       for b in range(len(self.block_sizes))])
            del f["_cm"]
            _REGEN[name] = self.ld_blocks
        self.ld_of = list(range(self.K)) if f["distinct_ld"] else [0] * self.K
        self.xhat = d["xhat"]
        self.r1 = d["r1"]
        self.cohort_csv = d["cohort_csv"]
        self.cohort_csv_text = [str(t) for t in d["cohort_csv_text"]]
        self.metrics_csv = d["metrics_csv"]
        self.metrics_csv_text = str(d["metrics_csv_text"])
        self.cg_iters = d["cg_iters"]
        self.cg_info = d["cg_info"]
        self.em_steps = d["em_steps"]
        self.lam0_repr = str(d["lam0_repr"])
        # the reference's "WARNING: ..." log lines (MLE: fsolve not converged / negative weights)
        self.warnings = json.loads(str(d["warnings"])) if "warnings" in d.files else []

    @property
    def x0(self):
        # main.py:276/279 -- rank 0's metrics use beta * sqrt(N_0)
        return self.beta * np.sqrt(self.N[0])

    def dense_R(self, l):
        M = self.M
        R = np.zeros((M, M))
        o = 0
        for B in self.ld_blocks[l]:
            n = B.shape[0]
            R[o:o + n, o:o + n] = B
            o += n
        return R

    def kwargs(self):
        f = self.flags
        return dict(rho=f["rho"], gamw=f["gamw"], gam1=f["gam1"], prior_vars=f["prior_vars"],
                    prior_probs=f["prior_probs"], cg_maxit=f["cg_maxit"],
                    em_prior_maxit=f["em_prior_maxit"], learn_gamw=f["learn_gamw"],
                    lmmse_damp=f["lmmse_damp"], prior_update=f["prior_update"],
                    update_prior_from=f["update_prior_from"], seed=f["seed"])
