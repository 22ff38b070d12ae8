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
@pytest.mark.parametrize("world,cases", [
    (2, ["k2_shared", "k1_blocks_csr_s_damp", "k4_shared_s_damp", "k1_L3", "k1_mle"]),
    (3, ["k2_shared", "k1_blocks_csr_s_damp"]),
])
def test_sharded_ranks_match_golden(world, cases):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SGV_EXCHANGE="host")
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
