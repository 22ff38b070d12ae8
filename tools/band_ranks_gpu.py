#!/usr/bin/env python3
"""One chromosome of windowed LD over N ranks on ONE GPU (host exchange): a
single band block (simulate.windowed_ld) cut into coupled pieces
(SGV_BAND_PIECE), the pieces spread over the ranks, VAMP run for a few
iterations; rank 0 reruns on one rank and requires every output file to be
bitwise identical (one block no longer means one GPU).

  RANK=r WORLD_SIZE=2 ... SGV_EXCHANGE=host python tools/band_ranks_gpu.py [K]
Exit code 0 iff the N-rank files equal the one-rank files."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))

from comm import SingleComm, world_from_env  # noqa: E402
from simulate import windowed_ld  # noqa: E402
from sgvamp import VAMP, BlockLD  # noqa: E402

M, BW, N, ITS = 100000, 600, 5000, 5


def problem(K):
    A = windowed_ld(M, BW, seed=7, taps=12)
    rs = np.random.RandomState(3)
    beta = np.zeros(M)
    idx = rs.choice(M, M // 20, replace=False)
    beta[idx] = rs.normal(0, np.sqrt(0.5 / len(idx)), len(idx))
    x0 = beta * np.sqrt(N)
    r = np.stack([A @ x0 + rs.normal(0, np.sqrt(1.0), M) for _ in range(K)])
    return A, r, x0, len(idx)


def run(comm, K, out, prior_update="em"):
    A, r, x0, cm = problem(K)
    L = BlockLD.from_csr(A)
    v = VAMP(N=[N] * K, Nt=N * K, M=M, K=K, rho=0.5, gamw=5.0, gam1=1e-6, a=[1.0 / K] * K,
             prior_vars=[0.0, 0.5 / cm * N / (N * K)], prior_probs=[0.95, 0.05], out_dir=out,
             out_name="band", seed=11, comm=comm, device=0)
    v.infer(L, r, ITS, x0=x0, cg_maxit=500, em_prior_maxit=100, learn_gamw=True,
            lmmse_damp=False, prior_update=prior_update, update_prior_from=1)
    comm.barrier()
    info = dict(pieces=len(v.engine.block_sizes), local=(v.engine.b0, v.engine.b1),
                cg=[h["cg_iters"] for h in v.history])
    v.engine.close()
    return info


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    pu = sys.argv[2] if len(sys.argv) > 2 else "em"   # prior update: em / mle
    comm = world_from_env()
    rank = comm.Get_rank()
    out = comm.bcast(tempfile.mkdtemp(prefix="band_ranks_") if rank == 0 else None)
    info = run(comm, K, out, pu)
    print("[band_ranks] rank %d of %d: pieces %d, local %s, cg %s" % (
        rank, comm.Get_size(), info["pieces"], info["local"], info["cg"]), flush=True)
    ok = True
    if rank == 0:
        solo = tempfile.mkdtemp(prefix="band_one_")
        info1 = run(SingleComm(), K, solo, pu)
        assert info1["pieces"] == info["pieces"] and info["pieces"] > comm.Get_size(), info
        files = sorted(f for f in os.listdir(solo))
        assert files == sorted(os.listdir(out)), (files, os.listdir(out))
        for f in files:
            a = open(os.path.join(out, f), "rb").read()
            b = open(os.path.join(solo, f), "rb").read()
            if a != b:
                print("[band_ranks] MISMATCH %s" % f, flush=True)
                ok = False
        print("[band_ranks] K=%d %s %d ranks vs one rank: %d files %s" % (
            K, pu, comm.Get_size(), len(files), "bitwise equal -> OK" if ok else "DIFFER"), flush=True)
    comm.barrier()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
