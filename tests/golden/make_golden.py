"""Generate golden fixtures by running the REFERENCE sgVAMP implementation.

Run ONLY in the build container (it needs /root/reference, which never travels
to the GPU box):

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

What it does
------------
* Builds small seeded synthetic problems following the reference's own recipe
  (simulation/sim_gen_phen_mult.py:28-55): X ~ Binomial(2, 0.4), standardised,
  divided by sqrt(N); y = X beta + noise; r = X^T y; R = X^T X (optionally
  block-diagonal, i.e. R = blockdiag(X_b^T X_b)).
* Restates the plumbing of src/main.py that cannot run here (mpi4py is absent):
  a = N/sum(N) (main.py:287), R <- (1-s)R + s*I (main.py:265), r reshape
  (main.py:266), x0 = beta*sqrt(N_rank) (main.py:276/279).
* Imports /root/reference/src/sgvamp.py and runs VAMP.infer once per cohort
  rank.  K > 1 uses K forked processes with a queue-backed fake comm that
  implements the only two methods the reference calls (Get_rank, bcast).
  Each rank seeds numpy's global RNG with seed + rank before infer (the
  reference never seeds; the build exposes --seed with the same stream).
* Records per-iteration outputs exactly as the reference wrote them to disk
  (xhat_it_*.bin, r1_cohort_*_it_*.bin, cohort CSVs, metrics CSV), plus CG
  iteration counts (scipy callback) and EM step counts (rank-0 log line).

The fixtures are DATA (inputs and expected outputs); no reference source is
copied into the repository.
"""
import json
import logging
import multiprocessing as mp
import os
import re
import sys
import tempfile

import numpy as np
import scipy.sparse

REF_SRC = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# synthetic inputs (simulation/sim_gen_phen_mult.py:28-55, seeded)
# --------------------------------------------------------------------------
def make_inputs(seed, M, Ns, blocks, lam_sim=0.5, h2=0.8, distinct_ld=False, exact=False):
    """Each cohort k has its own genotypes X_k (sim_gen_phen_mult.py:36-39) and
    r_k = X_k^T y_k.  R_k = blockdiag(X_k,b^T X_k,b).  With shared LD every
    cohort is given R_0 (cohort 0's LD used as the reference panel).

    exact=True: R is formed by tests.golden.exact_ld (bit-reproducible on any
    IEEE machine, so the fixture stores a checksum instead of the matrix and
    the tests regenerate it); everything else is the same recipe."""
    rs = np.random.RandomState(seed)
    cm = max(1, int(M * lam_sim))
    idx = rs.choice(M, cm, replace=False)
    beta = np.zeros(M)
    beta[idx] = rs.normal(0, np.sqrt(h2 / cm), cm)
    bounds = np.cumsum([0] + list(blocks))
    rvecs, Rs = [], []
    for k, N in enumerate(Ns):
        X = rs.binomial(2, 0.4, size=(N, M)).astype(np.float64)
        if exact and (distinct_ld or k == 0):
            sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
            from tests.golden import exact_ld

            Rs.append(exact_ld(X, blocks))
        X = (X - X.mean(axis=0)) / X.std(axis=0)          # :40
        g = X @ beta                                      # :44 (before /sqrt(N))
        w = rs.normal(0.0, np.sqrt(1 - h2), size=N)       # :46
        y = g + w
        X /= np.sqrt(N)                                   # :53
        rvecs.append(X.T @ y)                             # :54
        if exact:
            if not (distinct_ld or k == 0):
                Rs.append(Rs[0])
        elif distinct_ld or k == 0:
            R = np.zeros((M, M))
            for b in range(len(blocks)):
                s0, s1 = bounds[b], bounds[b + 1]
                R[s0:s1, s0:s1] = X[:, s0:s1].T @ X[:, s0:s1]   # :55, per block
            Rs.append(R)
        else:
            Rs.append(Rs[0])
    return beta, rvecs, Rs


# --------------------------------------------------------------------------
# fake MPI comm (only what src/sgvamp.py uses: Get_rank, bcast)
# --------------------------------------------------------------------------
class QueueComm:
    def __init__(self, rank, size, queues):
        self.rank, self.size, self.q = rank, size, queues

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def bcast(self, obj, root=0):
        if self.size == 1:
            return obj
        if self.rank == root:
            for d in range(self.size):
                if d != root:
                    self.q[root][d].put(obj)
            return obj
        return self.q[root][self.rank].get()


class _Capture(logging.Handler):
    def __init__(self):
        super().__init__(level=logging.INFO)
        self.em_steps, self.warnings = [], []

    def emit(self, record):
        msg = record.getMessage()
        m = re.search(r"prior-learning EM algorithm performed (\d+) steps", msg)
        if m:
            self.em_steps.append(int(m.group(1)))
        if "WARNING" in msg:
            self.warnings.append(msg)


def _rank_main(rank, cfg, queues, out_dir, result_q):
    sys.path.insert(0, REF_SRC)
    import sgvamp  # the reference module

    root = logging.getLogger()
    root.handlers[:] = []
    cap = _Capture()
    root.addHandler(cap)
    root.setLevel(logging.INFO)

    cg_counts = []
    orig_cg = sgvamp.con_grad

    def counting_cg(A, b, **kw):
        n = [0]

        def cb(xk):
            n[0] += 1

        x, info = orig_cg(A, b, callback=cb, **kw)
        cg_counts.append((n[0], int(info)))
        return x, info

    sgvamp.con_grad = counting_cg

    K = cfg["K"]
    Ns = cfg["N"]
    M = cfg["M"]
    s = cfg["s"]
    Nt = sum(Ns)
    N = Ns[rank]
    R = np.load(cfg["R_paths"][rank])
    if cfg["sparse"]:
        R = scipy.sparse.csr_matrix(R)
    # main.py:265 (dense .npy -> np.matrix; CSR stays CSR)
    R = (1 - s) * R + s * scipy.sparse.identity(M)
    r = np.load(cfg["r_paths"][rank]).reshape((M, 1))
    x0 = None
    if cfg["x0_path"] is not None:
        x0 = np.load(cfg["x0_path"]).reshape((M, 1)) * np.sqrt(N)
    a = np.array(Ns) / sum(Ns)
    comm = QueueComm(rank, K, queues)
    v = sgvamp.VAMP(N=N, Nt=Nt, M=M, K=K, rho=cfg["rho"], gam1=cfg["gam1"],
                    gamw=cfg["gamw"], a=a, prior_vars=cfg["prior_vars"],
                    prior_probs=cfg["prior_probs"], out_dir=out_dir,
                    out_name=cfg["name"], comm=comm)
    lam0 = v.lam
    np.random.seed(cfg["seed"] + rank)
    v.infer(R, r, cfg["iterations"], x0=x0, cg_maxit=cfg["cg_maxit"],
            em_prior_maxit=cfg["em_prior_maxit"], learn_gamw=cfg["learn_gamw"],
            lmmse_damp=cfg["lmmse_damp"], prior_update=cfg["prior_update"],
            update_prior_from=cfg["update_prior_from"])
    result_q.put((rank, cg_counts, cap.em_steps, cap.warnings, repr(lam0)))


def run_reference(cfg, workdir):
    K = cfg["K"]
    out_dirs = [os.path.join(workdir, "rank%d" % k) for k in range(K)]
    for d in out_dirs:
        os.makedirs(d, exist_ok=True)
    ctx = mp.get_context("fork")
    queues = [[ctx.Queue() for _ in range(K)] for _ in range(K)]
    result_q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(k, cfg, queues, out_dirs[k], result_q))
             for k in range(K)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(K):
        rank, cg, em, warn, lam0 = result_q.get(timeout=600)
        results[rank] = (cg, em, warn, lam0)
    for p in procs:
        p.join()
        assert p.exitcode == 0, "reference rank failed"
    return out_dirs, results


def read_bin(path):
    return np.fromfile(path, dtype=np.float64)


def read_tsv(path):
    with open(path) as f:
        text = f.read()
    lines = text.splitlines()
    rows = [[float(x) for x in ln.split("\t")] for ln in lines[1:]]
    return text, np.array(rows, dtype=np.float64)


# prior="auto": a spike-and-slab prior matched to the simulated scale.  With
# r = X^T y and X = X_std/sqrt(N), cohort k's signal is x = sqrt(N_k)*beta, so
# var(x) ~ h2/cm * N_k; the reference scales slab variances by Nt
# (sgvamp.py:27), hence prior_var = h2/cm * mean(N)/Nt.
CASES = {
    # K=1, one dense LD block, every CLI default (prior 0,1 / 0.99,0.01: the
    # slab variance is Nt, far above the simulated effect size)
    "k1_defaults": dict(seed=11, M=320, N=[1200], blocks=[320], iterations=6),
    # K=1, one dense LD block (C1 shape, scaled down), matched prior
    "k1_dense": dict(seed=21, M=400, N=[1500], blocks=[400], iterations=12,
                     prior="auto", lam_sim=0.1),
    # K=1, block-diagonal LD as CSR (.npz path), ridge s and LMMSE damping
    "k1_blocks_csr_s_damp": dict(seed=12, M=600, N=[2000], blocks=[200, 250, 150],
                                 iterations=10, sparse=True, s=0.1, lmmse_damp=1,
                                 prior="auto", lam_sim=0.1),
    # K=2 cohorts sharing one LD, EM prior on (C3-like)
    "k2_shared": dict(seed=13, M=450, N=[1500, 2500], blocks=[150, 150, 150],
                      iterations=10, prior="auto", lam_sim=0.1),
    # K=2 cohorts with distinct LD matrices
    "k2_distinct": dict(seed=14, M=240, N=[1000, 1400], blocks=[240], iterations=8,
                        distinct_ld=True, prior="auto", lam_sim=0.15),
    # K=1, no prior learning, fixed gamw
    "k1_noem_fixgamw": dict(seed=15, M=350, N=[1000], blocks=[350], iterations=8,
                            prior_update="none", learn_gamw=0, prior="auto", lam_sim=0.1),
    # K=1, three-component prior (two slabs) -> multi-slab denoiser + EM omegas
    "k1_L3": dict(seed=16, M=400, N=[1500], blocks=[200, 200], iterations=10,
                  prior="auto3", lam_sim=0.1),
    # MLE prior update (src/sgvamp.py:139-194, scipy fsolve), K=1 two components
    "k1_mle": dict(seed=18, M=400, N=[1500], blocks=[200, 200], iterations=8,
                   prior="auto", lam_sim=0.1, prior_update="mle"),
    # MLE, K=2 shared LD, three components (two slabs)
    "k2_mle_L3": dict(seed=19, M=360, N=[1200, 1800], blocks=[180, 180], iterations=8,
                      prior="auto3", lam_sim=0.1, prior_update="mle"),
    # MLE with the CLI default prior (slab variance far above the effect size)
    "k1_mle_defaults": dict(seed=20, M=300, N=[1000], blocks=[300], iterations=6,
                            prior_update="mle"),
    # K=4 shared LD, s>0, damping on, EM from iteration 2 (C5-like, small)
    "k4_shared_s_damp": dict(seed=17, M=320, N=[1000, 1200, 1400, 1600],
                             blocks=[160, 160], iterations=8, s=0.05, lmmse_damp=1,
                             update_prior_from=2, prior="auto", lam_sim=0.1),
    # --- the north star's accuracy gate (xhat within 1e-5 after 50 iterations),
    # pinned to the reference itself; R regenerated by the tests (exact=True) ---
    # (rho = 0.3: with the default 0.5 these runs blow up to NaN within 15-45
    # iterations -- in the reference as in the oracle -- which would gate nothing)
    # K=1, three blocks, ridge, damping, EM: 50 iterations
    "k1_long50": dict(seed=41, M=2400, N=[4000], blocks=[800, 900, 700], iterations=50,
                      s=0.02, lmmse_damp=1, rho=0.3, prior="auto", lam_sim=0.1, exact=True),
    # K=4 cohorts sharing one LD (MFMA pass), ridge, damping, EM: 50 iterations
    "k4_long50": dict(seed=42, M=2000, N=[3000, 3500, 4000, 4500], blocks=[1000, 1000],
                      iterations=50, s=0.02, lmmse_damp=1, rho=0.3, prior="auto", lam_sim=0.1,
                      exact=True),
    # more than 8 cohorts (the LMMSE runs them in groups of 8 CG column pairs):
    # K=10 sharing one LD with ridge + damping + EM, K=11 with distinct LDs
    "k10_shared": dict(seed=51, M=300, N=[800 + 100 * k for k in range(10)], blocks=[150, 150],
                       iterations=6, s=0.05, lmmse_damp=1, prior="auto", lam_sim=0.1),
    "k11_distinct": dict(seed=52, M=200, N=[700 + 50 * k for k in range(11)], blocks=[200],
                         iterations=6, distinct_ld=True, prior="auto", lam_sim=0.15),
    # C1 (BASELINE.json configs[0]): K=1, M=5000, N=10000, one dense block, 20
    # iterations; the simulation recipe's 50 % causal markers, matched prior
    "c1": dict(seed=43, M=5000, N=[10000], blocks=[5000], iterations=20, prior="auto",
               lam_sim=0.5, exact=True),
}

DEFAULTS = dict(rho=0.5, gamw=5.0, gam1=1e-6, prior_vars=[0.0, 1.0],
                prior_probs=[0.99, 0.01], cg_maxit=500, em_prior_maxit=100,
                learn_gamw=1, lmmse_damp=0, s=0.0, prior_update="em",
                update_prior_from=1, sparse=False, distinct_ld=False, exact=False)


def make_case(name, spec, workdir):
    cfg = dict(DEFAULTS)
    cfg.update(spec)
    cfg["name"] = name
    K = len(cfg["N"])
    cfg["K"] = K
    lam_sim = cfg.get("lam_sim", 0.5)
    beta, rvecs, Rs = make_inputs(cfg["seed"], cfg["M"], cfg["N"], cfg["blocks"],
                                  lam_sim=lam_sim, distinct_ld=cfg["distinct_ld"],
                                  exact=cfg["exact"])
    prior = cfg.get("prior")
    if prior in ("auto", "auto3"):
        cm = max(1, int(cfg["M"] * lam_sim))
        v = 0.8 / cm * np.mean(cfg["N"]) / sum(cfg["N"])
        if prior == "auto":
            cfg["prior_vars"] = [0.0, v]
            cfg["prior_probs"] = [1 - lam_sim, lam_sim]
        else:
            cfg["prior_vars"] = [0.0, 0.3 * v, 3.0 * v]
            cfg["prior_probs"] = [1 - lam_sim, 0.6 * lam_sim, 0.4 * lam_sim]
    cfg["R_paths"], cfg["r_paths"] = [], []
    for k in range(K):
        pR = os.path.join(workdir, "R%d.npy" % k)
        pr = os.path.join(workdir, "r%d.npy" % k)
        np.save(pR, Rs[k])
        np.save(pr, rvecs[k])
        cfg["R_paths"].append(pR)
        cfg["r_paths"].append(pr)
    cfg["x0_path"] = os.path.join(workdir, "beta.npy")
    np.save(cfg["x0_path"], beta)
    # learn_gamw/lmmse_damp as main.py parses them: bool(int(x)) (main.py:69-70)
    cfg["learn_gamw"] = bool(int(cfg["learn_gamw"]))
    cfg["lmmse_damp"] = bool(int(cfg["lmmse_damp"]))

    out_dirs, results = run_reference(cfg, workdir)
    its = cfg["iterations"]
    M = cfg["M"]
    xhat = np.stack([read_bin(os.path.join(out_dirs[0], "%s_xhat_it_%d.bin" % (name, it)))
                     for it in range(its)])
    r1 = np.stack([np.stack([read_bin(os.path.join(out_dirs[k], "%s_r1_cohort_%d_it_%d.bin"
                                                   % (name, k + 1, it)))
                             for it in range(its)]) for k in range(K)])
    csv_text, csv_rows = [], []
    for k in range(K):
        t, rows = read_tsv(os.path.join(out_dirs[k], "%s_cohort_%d.csv" % (name, k + 1)))
        csv_text.append(t)
        csv_rows.append(rows)
    mt, mrows = read_tsv(os.path.join(out_dirs[0], "%s_metrics.csv" % name))
    cg = np.array([results[k][0] for k in range(K)], dtype=np.int64)  # (K, 2*its, 2)
    cg = cg.reshape(K, its, 2, 2)
    em = np.array(results[0][1], dtype=np.int64)
    flags = {k: cfg[k] for k in ["seed", "M", "N", "blocks", "iterations", "rho", "gamw",
                                 "gam1", "prior_vars", "prior_probs", "cg_maxit",
                                 "em_prior_maxit", "learn_gamw", "lmmse_damp", "s",
                                 "prior_update", "update_prior_from", "sparse",
                                 "distinct_ld", "exact"]}
    out = dict(
        flags=np.array(json.dumps(flags)),
        beta=beta,
        r=np.stack(rvecs),
        xhat=xhat, r1=r1,
        cohort_csv=np.stack(csv_rows), cohort_csv_text=np.array(csv_text),
        metrics_csv=mrows, metrics_csv_text=np.array(mt),
        cg_iters=cg[..., 0], cg_info=cg[..., 1], em_steps=em,
        lam0_repr=np.array(results[0][3]),
        warnings=np.array(json.dumps(list(results[0][2]))),
    )
    # R is block-diagonal by construction: store only the diagonal blocks,
    # concatenated row-major, one row per distinct LD matrix -- or, for the
    # exact recipe, only their checksum (the tests regenerate them).
    bounds = np.cumsum([0] + list(cfg["blocks"]))
    lds = Rs if cfg["distinct_ld"] else Rs[:1]
    if cfg["exact"]:
        sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
        from tests.golden import ld_checksum

        out["R_sha256"] = np.array([ld_checksum(Rl, cfg["blocks"]) for Rl in lds])
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **out)
        print("%-24s K=%d M=%d its=%d cg=%s em=%s -> %s (%d KB)" % (
            name, K, M, its, cg[0, :, :, 0].tolist()[:3], em.tolist()[:4],
            os.path.basename(path), os.path.getsize(path) // 1024))
        return
    for Rl in lds:
        mask = np.ones(Rl.shape, dtype=bool)
        for b in range(len(cfg["blocks"])):
            mask[bounds[b]:bounds[b + 1], bounds[b]:bounds[b + 1]] = False
        assert not Rl[mask].any()
    out["R_blocks"] = np.stack([np.concatenate([Rl[bounds[b]:bounds[b + 1], bounds[b]:bounds[b + 1]].ravel()
                                                for b in range(len(cfg["blocks"]))]) for Rl in lds])
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print("%-24s K=%d M=%d its=%d cg=%s em=%s -> %s (%d KB)" % (
        name, K, M, its, cg[0, :, :, 0].tolist()[:3], em.tolist()[:4], os.path.basename(path),
        os.path.getsize(path) // 1024))


def main():
    only = sys.argv[1:]
    for name, spec in CASES.items():
        if only and name not in only:
            continue
        with tempfile.TemporaryDirectory() as wd:
            make_case(name, spec, wd)


if __name__ == "__main__":
    main()
