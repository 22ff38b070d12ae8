"""bench.py's cpu_baseline leg on CPU with a stand-in engine (small blocks, no
GPU): the sampled oracle timing, the extrapolation check against the whole
problem, and the reference cost model fields the bench line carries."""
import argparse
import os
import sys

import numpy as np

from tests.conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


class FakeEngine:
    def __init__(self, sizes, K, distinct=False, seed=0):
        rs = np.random.RandomState(seed)
        self.block_sizes = list(sizes)
        self.K = K
        self.M = sum(sizes)
        self.ld_of = list(range(K)) if distinct else [0] * K
        self.nld = len(set(self.ld_of))
        self.blocks = []
        for _ in range(self.nld):
            bl = []
            for n in sizes:
                X = rs.binomial(2, 0.4, size=(60, n)).astype(float)
                X = (X - X.mean(0)) / (X.std(0) + 1e-9) / np.sqrt(60)
                bl.append(X.T @ X)
            self.blocks.append(bl)
        self.r = rs.normal(size=(K, self.M))

    def get_ld_block(self, ld, b):
        return self.blocks[ld][b].copy()

    def get_vector(self, which, k=0):
        return self.r[k].copy()


def _args(**kw):
    d = dict(cpu_blocks=4, cpu_iters=2, ridge=0.0, nsamp=60, seed=3)
    d.update(kw)
    return argparse.Namespace(**d)


def _flags(M):
    return dict(rho=0.5, gamw=5.0, gam1=1e-6, prior_vars=[0.0, 0.8 / (M // 2) / 2],
                prior_probs=[0.5, 0.5], cg_maxit=500, em_prior_maxit=100, learn_gamw=True,
                lmmse_damp=False, prior_update="em", update_prior_from=1)


def test_cpu_baseline_fields_and_validation(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    eng = FakeEngine([40, 50, 30, 60], K=2)
    recs = [dict(cg_iters=[(3, 4), (3, 4)], em_steps=2)] * 3
    x0 = np.random.RandomState(1).normal(size=eng.M) * 0.1
    out = bench.cpu_baseline(eng, _args(), _flags(eng.M), recs, x0)
    assert out["cores"] <= 2 and out["cores_given"] == 2 and out["kind"] == "port"
    assert out["value"] > 0 and not out["extrapolated"]
    # the whole problem fits: the two-block extrapolation is checked against it
    assert "model_error" in out and np.isfinite(out["model_error"])
    assert out["measured_step_s"] > 0
    ref = out["reference_formula"]
    assert ref["step_s"] > ref["denoiser_loops_s"] == eng.M * bench.REF_DENOISE_S_PER_MARKER
    assert abs(1.0 / ref["step_s"] - ref["value"]) < 1e-12


def test_cpu_baseline_sampled_and_distinct(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    eng = FakeEngine([40] * 6, K=2, distinct=True)
    recs = [dict(cg_iters=[(2, 3), (2, 3)], em_steps=1)] * 2
    x0 = np.random.RandomState(2).normal(size=eng.M) * 0.1
    out = bench.cpu_baseline(eng, _args(cpu_blocks=4), _flags(eng.M), recs, x0)
    # 4 blocks over 2 LD matrices: 2 blocks of each are sampled and extrapolated
    assert out["extrapolated"] and "model_error" not in out
    assert "LD blocks 0-1" in out["sample"]


def test_matvecs_per_step_counts_reference_products():
    recs = [dict(cg_iters=[(3, 4)]), dict(cg_iters=[(1, 2)])]
    # per cohort: CG #1 + CG #2 + 2 warm starts + 2 gamw products
    assert bench.matvecs_per_step(recs) == ((3 + 4 + 4) + (1 + 2 + 4)) / 2
    assert bench.matvecs_per_step(recs, learn_gamw=False) == ((3 + 4 + 2) + (1 + 2 + 2)) / 2
    assert bench._ref_em_step_s(200000, 4) == 0.034
    assert abs(bench._ref_em_step_s(1000000, 2) - 5 * (0.013 + (0.034 - 0.013) / 3)) < 1e-12
