"""Golden fixtures generated from the reference (see make_golden.py)."""
import glob
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


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
        for row in d["R_blocks"]:
            self.ld_blocks.append([row[offs[b]:offs[b + 1]].reshape(n, n)
                                   for b, n in enumerate(self.block_sizes)])
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
