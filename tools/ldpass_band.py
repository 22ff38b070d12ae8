#!/usr/bin/env python3
"""LD-pass microbenchmark for sparse / windowed LD stored as packed bands
(sgv_set_ld_block_csr): one band of M markers and bandwidth bw built on the host
(simulate.windowed_ld, a few taps so it is cheap at any size), uploaded as
CSR, then kernel time per pass (HIP events) for 1..16 right-hand sides.  The
stored bytes are the band's panels (round_up(256 + bw, 256) columns per 256-row
panel); the "csr_equiv" rate counts the 12 B per stored nonzero (8-B value +
4-B index) a CSR mat-vec would stream instead.

  python tools/ldpass_band.py --M 200000 --bw 2000 --ncols 1,2,8,16"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=200000)
    ap.add_argument("--bw", type=int, default=2000)
    ap.add_argument("--taps", type=int, default=12)
    ap.add_argument("--fill", choices=["taps", "dense"], default="taps",
                    help="dense: every entry within bw non-zero, genotype-LD-like values "
                         "(N(0, 0.02^2) off the diagonal, 1 on it; a mat-vec study, not PSD)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ncols", default="1,2,8,16")
    ap.add_argument("--lib", default=None, help="A/B of builds: load this libsgvamp_hip.so")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    if a.lib:
        import hip_backend
        hip_backend.load(a.lib, strict=False)
    from engine import Engine
    from simulate import windowed_ld
    from sgvamp import BlockLD

    t0 = time.time()
    if a.fill == "dense":
        import scipy.sparse
        rs0 = np.random.RandomState(1)
        offs = list(range(1, a.bw + 1))
        U = scipy.sparse.diags([rs0.normal(0.0, 0.02, a.M - k) for k in offs], offs,
                               shape=(a.M, a.M), format="csr")
        A = (U + U.T + scipy.sparse.identity(a.M, format="csr")).tocsr()
        A.sort_indices()
    else:
        A = windowed_ld(a.M, a.bw, seed=1, taps=a.taps)
    L = BlockLD.from_csr(A)
    eng = Engine(L.block_sizes, K=1)
    for b in range(len(L.block_sizes)):
        L.upload(eng, 0, b)
    fmts = sorted({eng.ld_block_format(0, b) for b in range(len(L.block_sizes))})
    print("[band] M=%d bw=%d nnz=%d blocks=%d formats=%s setup %.1f s" % (
        a.M, a.bw, A.nnz, len(L.block_sizes), fmts, time.time() - t0), file=sys.stderr)
    rs = np.random.RandomState(0)
    for nc in [int(x) for x in a.ncols.split(",")]:
        V = rs.normal(size=(nc, a.M))
        Y = eng.ld_matvec(0, V)
        eng.timers(reset=True)
        for _ in range(a.reps):
            eng.ld_matvec(0, V)
        t = eng.timers()
        ms = t["ld_ms"] / t["ld_launches"]
        print(json.dumps(dict(tag=a.tag, M=a.M, bw=a.bw, ncol=nc, ms_per_pass=ms,
                              stored_GB=t["ld_bytes"] / t["ld_launches"] / 1e9,
                              stored_GBs=t["ld_bytes"] / t["ld_launches"] / ms / 1e6,
                              frac_of_8TBs=t["ld_bytes"] / t["ld_launches"] / ms / 1e6 / 8000.0,
                              csr_equiv_GBs=12.0 * A.nnz / ms / 1e6,
                              sha=hashlib.sha256(Y.tobytes()).hexdigest()[:16])), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
