#!/usr/bin/env python3
"""Cost of the in-library MLE prior update (sgv_mle_update) at a given size:
r1 vectors of a spike-and-slab mixture on the device, then wall time per update
and per single function evaluation (sgv_mle_terms: one device pass + host wait).

  python tools/mle_timing.py --M 1000000 --K 4 --nslab 1"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))

import hip_backend as hb  # noqa: E402
from engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=1000000)
    ap.add_argument("--K", type=int, default=4)
    ap.add_argument("--nslab", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    nb = 64
    sizes = [a.M // nb] * nb
    M = sum(sizes)
    eng = Engine(sizes, K=a.K)
    rs = np.random.RandomState(0)
    lam = 0.3
    sig = np.sort(rs.uniform(0.5, 3.0, a.nslab))
    for k in range(a.K):
        z = rs.rand(M) < lam
        eng.set_vector(hb.VEC_R1, k, np.where(z, rs.normal(0, 1.5, M), 0.0) + rs.normal(0, 0.4, M))
    gam1s = rs.uniform(3.0, 8.0, a.K)
    w = np.full(a.K, 1.0 / a.K)
    om = np.full(a.nslab, 1.0 / a.nslab)
    sigma2 = np.concatenate([[1e-16], sig])
    omega = np.concatenate([[1 - lam], lam * om])
    em = eng.mle_exp_max(gam1s, sigma2)
    eng.mle_terms(w, gam1s, sigma2, omega, em)
    t0 = time.perf_counter()
    for _ in range(20):
        eng.mle_terms(w, gam1s, sigma2, omega, em)
    t_eval = (time.perf_counter() - t0) / 20
    res = eng.mle_update(gam1s, w, sig, lam, om, None)
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        res = eng.mle_update(gam1s, w, sig, lam, om, None)
        ts.append(time.perf_counter() - t0)
    print(json.dumps(dict(M=M, K=a.K, nslab=a.nslab, eval_ms=t_eval * 1e3,
                          update_ms=float(np.median(ts)) * 1e3,
                          evals_per_update_est=float(np.median(ts)) / t_eval,
                          status=res[0], lam=res[1])), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
