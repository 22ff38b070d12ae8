#!/usr/bin/env python3
"""Bitwise A/B of two builds: run fixed LD passes (packed VALU/MFMA, dense, band)
and full VAMP runs of golden cases through the library at --lib, print one
SHA-256 per result.  Two builds whose lines are equal produce the same bits.

  python tools/ab_bitwise.py --lib sgvamp-py_amd/libsgvamp_hip.so > a.txt
  python tools/ab_bitwise.py --lib ab_lib/base.so > b.txt; diff a.txt b.txt"""
import argparse
import hashlib
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))
sys.path.insert(0, ROOT)


def h(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    a = ap.parse_args()
    import hip_backend
    hip_backend.load(a.lib)
    from engine import Engine
    from simulate import windowed_ld
    from sgvamp import VAMP, BlockLD
    from tests.golden import Case

    rs = np.random.RandomState(1)
    sizes = [1500, 2600, 700]
    blocks = []
    for n in sizes:
        X = rs.normal(size=(n // 2, n)) / np.sqrt(n)
        B = X.T @ X
        blocks.append((B + B.T) / 2)
    V = rs.normal(size=(16, sum(sizes)))
    for fmt in ("packed", "packed_valu", "dense"):
        eng = Engine(sizes, K=1)
        eng.set_ld_packing(fmt != "dense")
        if fmt == "packed_valu":
            eng.set_mfma_min(0)
        eng.set_ridge(0.05)
        for b, B in enumerate(blocks):
            eng.set_ld_block(0, b, B)
        for nc in (1, 2, 3, 5, 8, 12, 16):
            print("matvec %s nc=%d %s" % (fmt, nc, h(eng.ld_matvec(0, V[:nc]))))
        eng.close()
    A = windowed_ld(6000, 700, seed=3, taps=40)
    L = BlockLD.from_csr(A)
    eng = Engine(L.block_sizes, K=1)
    L.upload(eng, 0, 0)
    W = rs.normal(size=(16, 6000))
    for nc in (1, 2, 8, 16):
        print("matvec band nc=%d %s" % (nc, h(eng.ld_matvec(0, W[:nc]))))
    eng.close()
    # many blocks (> 8): the two-launch reduction + control path at one rank
    import hip_backend as hb
    sizes = [300] * 20
    M = sum(sizes)
    beta = np.zeros(M)
    beta[rs.choice(M, M // 10, replace=False)] = rs.normal(0, 0.01, M // 10)
    for K in (1, 2):
        eng = Engine(sizes, K=K)
        g = eng.synth_ld_g(0, 5, 250, beta).sum(axis=0)
        for k in range(K):
            eng.synth_r(k, 5, 250, g + np.random.RandomState(k).normal(0, 0.4, 250))
        with tempfile.TemporaryDirectory() as d:
            v = VAMP(N=[250.0] * K, Nt=250.0 * K, M=M, K=K, rho=0.5, gamw=5.0, gam1=1e-6,
                     a=[1.0 / K] * K, prior_vars=[0.0, 0.8 / (M // 10) / K],
                     prior_probs=[0.9, 0.1], out_dir=d, out_name="many", seed=3,
                     write_files=False)
            v.attach_engine(eng, x0=beta * np.sqrt(250.0))
            xh = v.infer(None, None, 5, x0=beta * np.sqrt(250.0), lmmse_damp=True,
                         prior_update="em")
            print("vamp many-blocks K=%d %s cg=%s" % (K, h(np.array(xh)),
                                                     [r["cg_iters"] for r in v.history]))
        eng.close()
    del hb
    for name in ("k1_blocks_csr_s_damp", "k4_shared_s_damp", "k10_shared", "k2_mle_L3"):
        c = Case(name)
        f = c.flags
        lds = [BlockLD(bl, s=f["s"]) for bl in c.ld_blocks]
        R = lds[0] if len(lds) == 1 else [lds[c.ld_of[k]] for k in range(c.K)]
        Nt = sum(c.N)
        with tempfile.TemporaryDirectory() as d:
            v = VAMP(N=c.N, Nt=Nt, M=c.M, K=c.K, rho=f["rho"], gamw=f["gamw"], gam1=f["gam1"],
                     a=np.array(c.N) / Nt, prior_vars=f["prior_vars"],
                     prior_probs=f["prior_probs"], out_dir=d, out_name=name, seed=f["seed"])
            xh = v.infer(R, c.r, f["iterations"], x0=c.x0, cg_maxit=f["cg_maxit"],
                         em_prior_maxit=f["em_prior_maxit"], learn_gamw=f["learn_gamw"],
                         lmmse_damp=f["lmmse_damp"], prior_update=f["prior_update"],
                         update_prior_from=f["update_prior_from"])
            print("vamp %s %s" % (name, h(np.array(xh))))
            v.engine.close()


if __name__ == "__main__":
    main()
