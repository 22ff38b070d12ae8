"""N > 1 path on CPU: world_size 2, over the product's host communicator
(comm.SocketComm, the torch-free TCP rendezvous) and over torch.distributed
gloo (test-side reference transport only; the product never imports torch).

* the host communicator (RCCL-id bootstrap, barrier, allgather) and the block
  partition agree across ranks;
* the sharded decomposition the GPU path uses -- each rank owns a contiguous
  range of LD blocks for all cohorts, every M-length sum is a per-block partial
  exchanged by all-gather and added in global block order -- reproduces the
  single-rank run BIT FOR BIT (checked with the oracle's restatement, the
  same algorithm the HIP kernels implement).
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from oracle import vamp_oracle as vo
from tests.golden import Case


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _TestGlooComm:
    """torch.distributed gloo with the comm.SocketComm interface (test only)."""

    def __init__(self):
        import torch.distributed as dist

        self.dist = dist
        dist.init_process_group(backend="gloo", init_method="env://")
        self.rank, self.size = dist.get_rank(), dist.get_world_size()

    def bcast(self, obj, root=0):
        box = [obj]
        self.dist.broadcast_object_list(box, src=root)
        return box[0]

    def allgather(self, obj):
        out = [None] * self.size
        self.dist.all_gather_object(out, obj)
        return out

    def barrier(self):
        self.dist.barrier()


class _GlooBlocks:
    def __init__(self, comm):
        self.comm = comm

    def allgather_blocks(self, part):
        return np.concatenate(self.comm.allgather(np.asarray(part)))


def _rank(rank, world, port, case_name, q, kind):
    try:
        if kind == "mpirun":   # only what Open MPI's mpirun -np 2 sets (src/main.py:16-18)
            for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
                os.environ.pop(k, None)
            os.environ.update(OMPI_COMM_WORLD_RANK=str(rank), OMPI_COMM_WORLD_SIZE=str(world),
                              OMPI_COMM_WORLD_LOCAL_RANK=str(rank),
                              OMPI_COMM_WORLD_LOCAL_SIZE=str(world),
                              OMPI_MCA_ess_base_jobid="job%d" % port, SGV_COMM_PORT=str(port))
        else:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                              WORLD_SIZE=str(world), SGV_COMM_PORT=str(port))
        from comm import world_from_env
        from partition import marker_offsets, partition_blocks

        comm = world_from_env() if kind in ("socket", "mpirun") else _TestGlooComm()
        if kind == "mpirun":
            assert (comm.Get_rank(), comm.Get_size(), comm.local_rank) == (rank, world, rank)
        uid = comm.bcast(b"\x01" * 128 if rank == 0 else None, root=0)
        assert uid == b"\x01" * 128
        c = Case(case_name)
        ranges = partition_blocks(c.block_sizes, world)
        assert comm.allgather(ranges) == [ranges] * world
        b0, b1 = ranges[rank]
        offs = marker_offsets(c.block_sizes)
        sl = slice(offs[b0], offs[b1])
        lds = [vo.BlockLD(blocks[b0:b1], s=c.flags["s"]) for blocks in c.ld_blocks]
        red = vo.Reducer("blocked", bounds=lds[0].bounds, comm=_GlooBlocks(comm))
        streams = vo.ProbeStream(c.flags["seed"], c.K)
        probe = lambda k, it: streams.draw(k, c.M)[sl]     # same stream on every rank
        with np.errstate(all="ignore"):
            t = vo.infer(lds, c.ld_of, [v[sl] for v in c.r], c.N, c.flags["iterations"],
                         x0=c.x0[sl], reducer=red, M_total=c.M, probe=probe, **c.kwargs())
        comm.barrier()
        q.put((rank, np.array(t["xhat"]), np.array(t["csv"]), np.array(t["cg_iters"]),
               list(t["em_steps"]), np.array(t["metrics"])))
    except Exception as e:  # surface the failure in the parent
        import traceback

        q.put((rank, "ERROR", traceback.format_exc(), None, None, None))


def _single(case_name):
    c = Case(case_name)
    lds = [vo.BlockLD(b, s=c.flags["s"]) for b in c.ld_blocks]
    red = vo.Reducer("blocked", bounds=lds[0].bounds)
    with np.errstate(all="ignore"):
        return vo.infer(lds, c.ld_of, list(c.r), c.N, c.flags["iterations"], x0=c.x0,
                        reducer=red, **c.kwargs())


@pytest.mark.parametrize("kind", ["socket", "gloo", "mpirun"])
@pytest.mark.parametrize("case_name", ["k2_shared", "k1_blocks_csr_s_damp", "k4_shared_s_damp",
                                       "k1_mle", "k2_mle_L3"])
def test_two_rank_sharded_run_is_bit_identical(case_name, kind):
    """kind "mpirun": the ranks see only Open MPI's variables -- the reference's
    own launch becomes one job of two GPU ranks with the same partition and the
    one-rank result bit for bit (not two one-rank jobs writing the same files)."""
    world = 2
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, case_name, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=300)
        assert not isinstance(item[1], str), item[2]
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _single(case_name)
    xh = np.concatenate([res[r][1] for r in range(world)], axis=1)
    np.testing.assert_array_equal(xh, np.array(ref["xhat"]))
    for r in range(world):
        np.testing.assert_array_equal(res[r][2], np.array(ref["csv"]))
        np.testing.assert_array_equal(res[r][3], np.array(ref["cg_iters"]))
        assert res[r][4] == list(ref["em_steps"])
        np.testing.assert_array_equal(res[r][5], np.array(ref["metrics"]))


def _comm_rank(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), SGV_COMM_PORT=str(port))
        import sys

        from comm import SocketComm, world_from_env

        comm = world_from_env()
        assert isinstance(comm, SocketComm) and "torch" not in sys.modules
        out = {}
        out["bcast"] = comm.bcast(("id", 7) if rank == 1 else None, root=1)
        out["ag"] = comm.allgather({"r": rank})
        out["f64"] = comm.allgather_f64(np.arange(3, dtype=np.float64) + 10 * rank)
        out["empty"] = comm.allgather_f64(np.zeros(0))
        big = np.random.RandomState(rank).normal(size=200_000)
        out["big"] = float(comm.allgather_f64(big).sum())
        comm.barrier()
        comm.close()
        q.put((rank, out))
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_socket_comm_collectives(world):
    """comm.SocketComm alone: rank order, bcast from a non-zero root, empty and
    multi-MB payloads; torch is never imported."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    want_big = sum(float(np.random.RandomState(r).normal(size=200_000).sum()) for r in range(world))
    for r in range(world):
        out = res[r]
        assert isinstance(out, dict), out
        assert out["bcast"] == ("id", 7)
        assert out["ag"] == [{"r": i} for i in range(world)]
        np.testing.assert_array_equal(out["f64"], np.concatenate(
            [np.arange(3.0) + 10 * i for i in range(world)]))
        assert out["empty"].shape == (0,)
        assert abs(out["big"] - want_big) < 1e-6


# ---- one band block over two ranks (coupled pieces) -----------------------------------
_BAND = dict(M=70000, bw=600, N=5000, its=4, piece=16384)


def _band_problem():
    import scipy.sparse

    from sgvamp import BlockLD, band_cuts

    A = vo.banded_ld(_BAND["M"], _BAND["bw"], seed=9, taps=12)
    L = BlockLD.from_csr(A)
    cuts = band_cuts([L], L.block_sizes, piece=_BAND["piece"])
    P, cpl = L.pieces(cuts)
    pieces = [P.block_csr(k) for k in range(len(P.block_sizes))]
    cpl = {gb: (nr, nc, C.toarray() if scipy.sparse.issparse(C) else C)
           for gb, (nr, nc, C) in cpl.items()}
    rs = np.random.RandomState(4)
    M, N = _BAND["M"], _BAND["N"]
    beta = np.zeros(M)
    idx = rs.choice(M, M // 20, replace=False)
    beta[idx] = rs.normal(0, np.sqrt(0.5 / len(idx)), len(idx))
    x0 = beta * np.sqrt(N)
    r = A @ x0 + rs.normal(0, 1.0, M)
    kw = dict(rho=0.5, gamw=5.0, gam1=1e-6, prior_vars=[0.0, 0.5 / len(idx)],
              prior_probs=[0.95, 0.05], seed=5)
    return pieces, cpl, r, x0, kw


def _band_rank(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), SGV_COMM_PORT=str(port))
        from comm import world_from_env
        from partition import partition_blocks

        comm = world_from_env()
        pieces, cpl, r, x0, kw = _band_problem()
        sizes = [P.shape[0] for P in pieces]
        ranges = partition_blocks(sizes, world)
        b0, b1 = ranges[rank]
        offs = np.cumsum([0] + sizes)
        sl = slice(offs[b0], offs[b1])
        L = vo.CoupledLD(pieces[b0:b1], cpl, gb0=b0, comm=comm)
        red = vo.Reducer("blocked", bounds=L.bounds, comm=_GlooBlocks(comm))
        streams = vo.ProbeStream(kw["seed"], 1)
        probe = lambda k, it: streams.draw(k, _BAND["M"])[sl]
        t = vo.infer([L], [0], [r[sl]], [_BAND["N"]], _BAND["its"], x0=x0[sl], reducer=red,
                     M_total=_BAND["M"], probe=probe, **kw)
        comm.barrier()
        q.put((rank, np.array(t["xhat"]), np.array(t["cg_iters"]), (b0, b1)))
    except Exception:  # surface the failure in the parent
        import traceback

        q.put((rank, "ERROR", traceback.format_exc(), None))


def test_band_block_over_two_ranks_is_bit_identical():
    """One band block cut into coupled pieces (the product's band_cuts /
    BlockLD.pieces), two socket ranks owning two pieces each: the sharded
    oracle -- pieces' products plus the corner couplings, the neighbour's head /
    tail rows all-gathered -- is bitwise the one-rank run (VERDICT round 3,
    item 6: one chromosome no longer means one GPU)."""
    world = 2
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=300)
        assert not isinstance(item[1], str), item[2]
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][3] == (0, 2) and res[1][3] == (2, 4)     # two pieces each
    pieces, cpl, r, x0, kw = _band_problem()
    L = vo.CoupledLD(pieces, cpl)
    t = vo.infer([L], [0], [r], [_BAND["N"]], _BAND["its"], x0=x0,
                 reducer=vo.Reducer("blocked", bounds=L.bounds), **kw)
    xh = np.concatenate([res[k][1] for k in range(world)], axis=1)
    np.testing.assert_array_equal(xh, np.array(t["xhat"]))
    np.testing.assert_array_equal(res[0][2], np.array(t["cg_iters"]))
    # and the pieces with their couplings are the band itself
    A = vo.banded_ld(_BAND["M"], _BAND["bw"], seed=9, taps=12)
    v = np.random.RandomState(0).normal(size=_BAND["M"])
    np.testing.assert_allclose(L.matvec_R(v), A @ v, rtol=0, atol=1e-12)
