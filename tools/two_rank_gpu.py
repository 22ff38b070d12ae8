#!/usr/bin/env python3
"""Multi-rank HIP path on ONE GPU: N ranks (torchrun) all on device 0.  RCCL
refuses two ranks on one device, so run with SGV_EXCHANGE=host (the library's
host exchange carries the per-block partials over gloo).  Rank 0 checks the
merged output files against the golden fixture of each case.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29531 tools/two_rank_gpu.py k2_shared k1_blocks_csr_s_damp
Rank 0 then reruns each case on one rank (same device) and requires the output
files to be bitwise identical: the ordered per-block reductions make the
trajectory independent of the number of ranks.
Exit code 0 iff every case matches (golden bar, and bitwise vs one rank)."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))

from comm import world_from_env  # noqa: E402
from sgvamp import VAMP, BlockLD  # noqa: E402
from tests.golden import Case  # noqa: E402


def maxrel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def main():
    comm = world_from_env()
    rank = comm.rank
    ok = True
    for name in sys.argv[1:] or ["k2_shared"]:
        c = Case(name)
        f = c.flags
        out = comm.bcast(tempfile.mkdtemp(prefix="two_rank_") if rank == 0 else None)
        lds = [BlockLD(blocks, s=f["s"]) for blocks in c.ld_blocks]
        R = lds[0] if len(lds) == 1 else [lds[c.ld_of[k]] for k in range(c.K)]
        Nt = sum(c.N)
        v = VAMP(N=c.N, Nt=Nt, M=c.M, K=c.K, rho=f["rho"], gamw=f["gamw"], gam1=f["gam1"],
                 a=np.array(c.N) / Nt, prior_vars=f["prior_vars"], prior_probs=f["prior_probs"],
                 out_dir=out, out_name=name, seed=f["seed"], comm=comm, device=0)
        v.infer(R, c.r, f["iterations"], x0=c.x0, cg_maxit=f["cg_maxit"],
                em_prior_maxit=f["em_prior_maxit"], learn_gamw=f["learn_gamw"],
                lmmse_damp=f["lmmse_damp"], prior_update=f["prior_update"],
                update_prior_from=f["update_prior_from"])
        comm.barrier()
        v.engine.close()
        if rank == 0:
            from comm import SingleComm

            solo = tempfile.mkdtemp(prefix="one_rank_")
            v1 = VAMP(N=c.N, Nt=Nt, M=c.M, K=c.K, rho=f["rho"], gamw=f["gamw"], gam1=f["gam1"],
                      a=np.array(c.N) / Nt, prior_vars=f["prior_vars"],
                      prior_probs=f["prior_probs"], out_dir=solo, out_name=name, seed=f["seed"],
                      comm=SingleComm(), device=0)
            v1.infer(R, c.r, f["iterations"], x0=c.x0, cg_maxit=f["cg_maxit"],
                     em_prior_maxit=f["em_prior_maxit"], learn_gamw=f["learn_gamw"],
                     lmmse_damp=f["lmmse_damp"], prior_update=f["prior_update"],
                     update_prior_from=f["update_prior_from"])
            v1.engine.close()
            bitwise = True
            for it in range(f["iterations"]):
                names = ["%s_xhat_it_%d.bin" % (name, it)] + [
                    "%s_r1_cohort_%d_it_%d.bin" % (name, k + 1, it) for k in range(c.K)]
                for fn in names:
                    with open(os.path.join(out, fn), "rb") as fa, open(os.path.join(solo, fn), "rb") as fb:
                        bitwise &= fa.read() == fb.read()
            worst = 0.0
            for it in range(f["iterations"]):
                xb = np.fromfile(os.path.join(out, "%s_xhat_it_%d.bin" % (name, it)))
                worst = max(worst, maxrel(xb, c.xhat[it]))
            cg = np.array([h["cg_iters"] for h in v.history]).transpose(1, 0, 2)
            same_cg = bool(np.array_equal(cg, c.cg_iters))
            em = [h["em_steps"] for h in v.history if "em_steps" in h]
            good = worst < 1e-8 and same_cg and em == list(c.em_steps) and bitwise
            ok &= good
            print("[two_rank] %s ranks=%d blocks/rank=%s maxrel_xhat=%.3e cg_equal=%s em_equal=%s "
                  "bitwise_vs_1rank=%s -> %s"
                  % (name, comm.size, v.engine.local_sizes, worst, same_cg, em == list(c.em_steps),
                     bitwise, "OK" if good else "FAIL"), flush=True)
        comm.barrier()
    ok = comm.bcast(ok)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
