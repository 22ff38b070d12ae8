"""Sharded (N > 1 ranks) HIP path on one GPU.

RCCL refuses two ranks on one device, so these ranks use the library's host
exchange (sgv_comm_init_host, gloo all-gather of the per-block partials).  All
other code is the sharded product path: LD block ranges per rank, rank-local
vectors, the ordered cross-rank reduction (bitwise the same scalars as one
rank), rank-sliced output files.  tools/two_rank_gpu.py checks the merged files
against the reference's golden outputs (maxrel < 1e-8, identical CG and EM
counts) and, rerun on one rank, bitwise against the one-rank output files."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("world,cases,em", [
    (2, ["k2_shared", "k1_blocks_csr_s_damp", "k4_shared_s_damp", "k1_L3", "k1_mle"], "auto"),
    (3, ["k2_shared", "k1_blocks_csr_s_damp"], "auto"),
    (2, ["k2_shared", "k4_shared_s_damp", "k10_shared"], "per-step"),
    (2, ["k4_shared_s_damp", "k10_shared", "k4_long50"], "cg-exact"),
])
def test_sharded_ranks_match_golden(world, cases, em):
    """em: "auto" = the size rule (these small cases: replicated EM, r1 gathered
    once per loop); "per-step" forces one exchange per EM step (the rule's choice
    above about a million cohort-markers, e.g. the north star); "cg-exact" forces
    the exact CG column sets (the global-size rule's choice for >= 24 GB of LD,
    e.g. the north star and C5), so one rank and two ranks must agree bitwise in
    that mode too (tools/two_rank_gpu.py reruns each case on one rank)."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SGV_EXCHANGE="host")
        if em == "per-step":
            env.update(SGV_AB="1", SGV_EM_REP="0")
        if em == "cg-exact":
            env.update(SGV_AB="1", SGV_CG_EXACT="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "two_rank_gpu.py")]
                                      + cases, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, "rank %d failed:\n%s" % (r, out[-4000:])
    assert outs[0].count("-> OK") == len(cases), outs[0]


def _run_case_files(name, out, exchange):
    """One-rank run of golden case `name`; returns {file name: bytes}."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))
    from sgvamp import VAMP, BlockLD
    from tests.golden import Case

    c = Case(name)
    f = c.flags
    lds = [BlockLD(blocks, s=f["s"]) for blocks in c.ld_blocks]
    R = lds[0] if len(lds) == 1 else [lds[c.ld_of[k]] for k in range(c.K)]
    Nt = sum(c.N)
    v = VAMP(N=c.N, Nt=Nt, M=c.M, K=c.K, rho=f["rho"], gamw=f["gamw"], gam1=f["gam1"],
             a=np.array(c.N) / Nt, prior_vars=f["prior_vars"], prior_probs=f["prior_probs"],
             out_dir=str(out), out_name=name, seed=f["seed"], device=0, exchange=exchange)
    v.infer(R, c.r, f["iterations"], x0=c.x0, cg_maxit=f["cg_maxit"],
            em_prior_maxit=f["em_prior_maxit"], learn_gamw=f["learn_gamw"],
            lmmse_damp=f["lmmse_damp"], prior_update=f["prior_update"],
            update_prior_from=f["update_prior_from"])
    info = v.engine.comm_info()
    _short_buffers(v.engine)
    v.engine.close()
    files = {fn: open(os.path.join(out, fn), "rb").read() for fn in sorted(os.listdir(out))
             if fn.endswith(".bin")}
    return files, info


def _short_buffers(eng):
    """ABI revision 2: a caller built against a shorter list
    passes its own length and the library writes that prefix only."""
    import numpy as np

    import hip_backend as hb

    for fn, n in (("sgv_exchange_stats", hb.EXCHANGE_STATS_N), ("sgv_timers", hb.TIMERS_N)):
        full = np.zeros(n)
        getattr(eng.ctx, fn)(hb.dptr(full), n, 0)
        buf = np.full(n + 4, -7.25)
        getattr(eng.ctx, fn)(hb.dptr(buf), 6, 0)          # round 5's 6-double buffer
        assert (buf[6:] == -7.25).all(), fn
        np.testing.assert_array_equal(buf[:6], full[:6])
    with pytest.raises(hb.HipError):
        eng.ctx.sgv_timers(hb.dptr(np.zeros(1)), -1, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["k2_shared", "k1_blocks_csr_s_damp"])
def test_one_rank_exchange_rehearsal_bitwise(name, tmp_path):
    """The RCCL exchange on one GPU: a real one-rank communicator (ncclCommInitRank,
    ncclAllGather on the library stream) carries the ordered per-block partials;
    the host exchange likewise.  Both must leave every output file bitwise
    identical to the run without a communicator."""
    (tmp_path / "none").mkdir()
    base, info = _run_case_files(name, tmp_path / "none", None)
    assert info["transport"] is None and info["comm_ranks"] == 1
    for ex in ("rccl", "host"):
        d = tmp_path / ex
        d.mkdir()
        got, info = _run_case_files(name, d, ex)
        assert got.keys() == base.keys() and len(base) > 0
        for fn in base:
            assert got[fn] == base[fn], (ex, fn)
        # the communicator's own view: RCCL counts one rank (ncclCommCount), this
        # rank is its rank 0 on HIP device 0, whose PCI bus id is reported
        assert info["transport"] == ex and info["comm_ranks"] == 1 and info["comm_rank"] == 0, info
        assert info["device"] == 0 and info["nranks"] == 1 and len(info["pci_bus_id"]) >= 7, info


@pytest.mark.gpu
@pytest.mark.parametrize("world,K,prior", [(2, 1, "em"), (3, 2, "em"), (4, 4, "em"), (2, 2, "mle")])
def test_single_band_block_over_ranks(world, K, prior):
    """One band block (one chromosome of windowed LD, M = 100,000) cut into
    coupled pieces of 16,384 markers and spread over `world` ranks (host
    exchange on one GPU): every output file bitwise identical to the one-rank
    run (tools/band_ranks_gpu.py), for K = 1 (VALU passes) and K = 2 (MFMA),
    with the EM prior update and with the MLE one (fsolve over the sharded sums)."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SGV_EXCHANGE="host",
                   SGV_BAND_PIECE="16384")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "band_ranks_gpu.py"),
                                       str(K), prior], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, "rank %d failed:\n%s" % (r, out[-4000:])
    assert "bitwise equal -> OK" in outs[0], outs[0][-3000:]
