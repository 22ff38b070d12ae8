"""Launch paths on CPU: the rank model read from every launcher the reference
or a cluster uses (src/main.py:16-18: ``mpirun -np K``), ``--gpus N``
self-launch, and the host communicator's hardening (no unpickling, stray and
unauthenticated connections dropped)."""
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from tests.conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "sgvamp-py_amd"))
import comm as cm  # noqa: E402
import launch  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ---- launcher detection ---------------------------------------------------------------

def test_no_launcher_is_one_rank():
    info = cm.launch_from_env({})
    assert (info["rank"], info["size"], info["source"]) == (0, 1, "none")
    assert isinstance(cm.world_from_env({}), cm.SingleComm)


def test_torchrun_style_env():
    env = dict(RANK="3", LOCAL_RANK="1", WORLD_SIZE="4", MASTER_ADDR="10.0.0.5", MASTER_PORT="1234")
    info = cm.launch_from_env(env)
    assert (info["rank"], info["size"], info["local_rank"]) == (3, 4, 1)
    assert (info["addr"], info["port"], info["source"]) == ("10.0.0.5", 1235, "env")


def test_openmpi_single_node_maps_to_gpu_ranks():
    env = dict(OMPI_COMM_WORLD_RANK="1", OMPI_COMM_WORLD_SIZE="2", OMPI_COMM_WORLD_LOCAL_RANK="1",
               OMPI_COMM_WORLD_LOCAL_SIZE="2", OMPI_MCA_ess_base_jobid="4242")
    a = cm.launch_from_env(env)
    b = cm.launch_from_env(dict(env, OMPI_COMM_WORLD_RANK="0", OMPI_COMM_WORLD_LOCAL_RANK="0"))
    assert (a["rank"], a["size"], a["local_rank"], a["source"]) == (1, 2, 1, "openmpi")
    assert a["addr"] == "127.0.0.1"
    # both ranks derive the same rendezvous port and token from the job id
    assert a["port"] == b["port"] and 20000 <= a["port"] < 40000 and a["token"] == b["token"]
    c = cm.launch_from_env(dict(env, OMPI_MCA_ess_base_jobid="4243"))
    assert c["port"] != a["port"] or c["token"] != a["token"]


def test_openmpi_multi_node_needs_master_addr():
    env = dict(OMPI_COMM_WORLD_RANK="0", OMPI_COMM_WORLD_SIZE="16", OMPI_COMM_WORLD_LOCAL_RANK="0",
               OMPI_COMM_WORLD_LOCAL_SIZE="8")
    with pytest.raises(RuntimeError, match="MASTER_ADDR"):
        cm.launch_from_env(env)
    info = cm.launch_from_env(dict(env, MASTER_ADDR="node0"))
    assert (info["addr"], info["size"], info["local_rank"]) == ("node0", 16, 0)


def test_hydra_and_srun_envs():
    hy = cm.launch_from_env(dict(PMI_RANK="2", PMI_SIZE="4", MPI_LOCALRANKID="2",
                                 MPI_LOCALNRANKS="4", PMI_KVSNAME="kvs_77"))
    assert (hy["rank"], hy["size"], hy["local_rank"], hy["source"]) == (2, 4, 2, "pmi")
    sl = cm.launch_from_env(dict(SLURM_PROCID="5", SLURM_STEP_NUM_TASKS="8", SLURM_LOCALID="5",
                                 SLURM_STEP_NUM_NODES="1", SLURM_JOB_ID="99", SLURM_STEP_ID="0"))
    assert (sl["rank"], sl["size"], sl["local_rank"], sl["source"]) == (5, 8, 5, "slurm")
    # a batch script in an 8-task allocation is ONE process: not a world of 8
    batch = cm.launch_from_env(dict(SLURM_PROCID="0", SLURM_NTASKS="8", SLURM_JOB_ID="99"))
    assert batch["size"] == 1


def test_bad_launch_env_fails_fast():
    with pytest.raises(RuntimeError):
        cm.launch_from_env(dict(RANK="4", WORLD_SIZE="4"))
    with pytest.raises(RuntimeError, match="LOCAL_RANK"):
        cm.launch_from_env(dict(OMPI_COMM_WORLD_RANK="0", OMPI_COMM_WORLD_SIZE="4",
                                MASTER_ADDR="h"))


# ---- self-launch ----------------------------------------------------------------------

def test_rank_envs():
    envs = launch.rank_envs(3, base={"PATH": "/bin"}, port=5555, token="t")
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (
            str(r), str(r), "3", "3")
        assert (e["MASTER_ADDR"], e["SGV_COMM_PORT"], e["SGV_COMM_TOKEN"]) == ("127.0.0.1", "5555", "t")
        assert e["PATH"] == "/bin"
        info = cm.launch_from_env(e)
        assert (info["rank"], info["size"], info["port"], info["token"]) == (r, 3, 5555, "t")


def test_gpus_must_match_external_world():
    with pytest.raises(SystemExit, match="must agree"):
        launch.relaunch(2, environ=dict(RANK="0", WORLD_SIZE="4", LOCAL_RANK="0"))
    assert launch.relaunch(4, environ=dict(RANK="0", WORLD_SIZE="4", LOCAL_RANK="0")) is None
    assert launch.relaunch(None, environ={}) is None
    assert launch.relaunch(1, environ={}) is None


def _clean_env():
    env = {k: v for k, v in os.environ.items()
           if not k.startswith(("OMPI_", "PMI_", "SLURM_", "MPI_LOCAL"))
           and k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                         "MASTER_PORT", "SGV_COMM_PORT", "SGV_COMM_TOKEN")}
    return env


def test_bench_gpus_2_self_launch_dry_run():
    """bench.py --gpus 2 (no launcher): the parent starts two child ranks with
    the world set up, rank 0's line is relayed, no GPU is touched."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--dry-run"], env=_clean_env(), capture_output=True, text=True,
                         timeout=120, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["dry_run"] and d["n_gpus"] == 2
    ranks = d["ranks"]
    assert [r["rank"] for r in ranks] == [0, 1]
    assert [r["device"] for r in ranks] == [0, 1]
    assert all(r["env"]["SGV_LAUNCHED_BY"] == "sgvamp.launch" for r in ranks)
    assert len({r["pid"] for r in ranks}) == 2


def test_bench_under_simulated_mpirun_dry_run():
    """Two processes with only Open MPI's variables (what ``mpirun -np 2``
    sets): one job of two GPU ranks, not two one-rank jobs."""
    job = str(os.getpid())
    procs = []
    for r in range(2):
        env = dict(_clean_env(), OMPI_COMM_WORLD_RANK=str(r), OMPI_COMM_WORLD_SIZE="2",
                   OMPI_COMM_WORLD_LOCAL_RANK=str(r), OMPI_COMM_WORLD_LOCAL_SIZE="2",
                   OMPI_MCA_ess_base_jobid=job, SGV_COMM_PORT=str(_free_port()) if r == 0 else "")
        procs.append(env)
    procs[1]["SGV_COMM_PORT"] = procs[0]["SGV_COMM_PORT"]
    ps = [subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"], env=e,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT)
          for e in procs]
    outs = [p.communicate(timeout=120) for p in ps]
    assert all(p.returncode == 0 for p in ps), [o[1][-2000:] for o in outs]
    assert outs[1][0].strip() == ""                    # only rank 0 prints
    d = json.loads(outs[0][0])
    assert d["n_gpus"] == 2 and [r["local_rank"] for r in d["ranks"]] == [0, 1]
    assert d["ranks"][1]["env"]["OMPI_COMM_WORLD_RANK"] == "1"


def test_spawn_propagates_failure():
    code = "import os,sys; sys.exit(3 if os.environ['RANK']=='1' else 0)"
    assert launch.spawn(2, [sys.executable, "-c", code], base=_clean_env()) == 3
    slow = "import os,sys,time; r=os.environ['RANK']; time.sleep(60 if r=='0' else 0); sys.exit(int(r)*5)"
    t = time.monotonic()
    assert launch.spawn(2, [sys.executable, "-c", slow], base=_clean_env()) == 5
    assert time.monotonic() - t < 30                   # rank 0 was stopped, not waited for


def test_rank_dying_in_a_collective_ends_the_job(tmp_path):
    """A rank that dies mid-run while its peer waits in a collective: the parent
    exits non-zero within a bounded time and leaves no rank blocked (the
    waiting rank is stopped, not waited for)."""
    code = ("import os, sys, time\n"
            "sys.path.insert(0, %r)\n"
            "from comm import world_from_env\n"
            "c = world_from_env()\n"
            "c.barrier()\n"
            "open(os.path.join(%r, 'pid%%d' %% c.Get_rank()), 'w').write(str(os.getpid()))\n"
            "if c.Get_rank() == 1:\n"
            "    os._exit(7)\n"
            "time.sleep(0.5)\n"
            "c.allgather(b'x')\n"
            "time.sleep(600)\n") % (os.path.join(ROOT, "sgvamp-py_amd"), str(tmp_path))
    t = time.monotonic()
    rc = launch.spawn(2, [sys.executable, "-c", code], base=_clean_env())
    assert rc == 7
    assert time.monotonic() - t < 60
    for r in range(2):
        pid = int((tmp_path / ("pid%d" % r)).read_text())
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)


def test_sigterm_to_parent_stops_every_rank(tmp_path):
    """a SIGTERM to the self-launching parent alone (a scheduler
    or `timeout` signalling its PID) stops the N ranks before the parent exits
    (128 + 15), instead of leaving them holding their GPUs and the port."""
    child = ("import os, time; open(os.path.join(%r, 'pid' + os.environ['RANK']), 'w')"
             ".write(str(os.getpid())); time.sleep(600)") % str(tmp_path)
    parent = ("import sys; sys.path.insert(0, %r); import launch; "
              "sys.exit(launch.spawn(2, [sys.executable, '-c', %r]))") % (
                  os.path.join(ROOT, "sgvamp-py_amd"), child)
    p = subprocess.Popen([sys.executable, "-c", parent], env=_clean_env())
    deadline = time.monotonic() + 60
    while time.monotonic() < deadline and not all(
            (tmp_path / ("pid%d" % r)).exists() for r in range(2)):
        time.sleep(0.1)
    pids = [int((tmp_path / ("pid%d" % r)).read_text()) for r in range(2)]
    p.send_signal(15)
    assert p.wait(timeout=60) == 128 + 15
    for pid in pids:
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)


# ---- host communicator hardening ----------------------------------------------------------

def test_codec_roundtrip_and_refusals():
    obj = {"a": (1, 2.5, None, True), 3: [b"\x00\x01", "s"], "arr": np.arange(6.0).reshape(2, 3),
           "i": np.int64(2 ** 40), "f": float("inf"), "neg": -0.0}
    back = cm.decode(cm.encode(obj))
    assert back["a"] == (1, 2.5, None, True) and back[3] == [b"\x00\x01", "s"]
    np.testing.assert_array_equal(back["arr"], obj["arr"])
    assert back["i"] == 2 ** 40 and back["f"] == float("inf")
    assert str(back["neg"]) == "-0.0"
    with pytest.raises(TypeError):
        cm.encode(np.array([object()], dtype=object))
    with pytest.raises(TypeError):
        cm.encode({1, 2})
    bad = cm.encode(np.zeros(2)).replace(b'"<f8"', b'"|O8"')
    with pytest.raises((ValueError, TypeError)):
        cm.decode(bad)


def _rank_thread(rank, size, port, token, out):
    try:
        c = cm.SocketComm(rank, size, "127.0.0.1", port, timeout=30, token=token)
        out[rank] = c.allgather(rank * 10)
        c.close()
    except Exception as e:  # noqa: BLE001
        out[rank] = e


def test_rendezvous_drops_stray_and_unauthenticated_peers():
    port = _free_port()
    out = {}
    t0 = threading.Thread(target=_rank_thread, args=(0, 2, port, "secret", out))
    t0.start()
    time.sleep(0.3)
    stray = socket.create_connection(("127.0.0.1", port))        # says nothing
    impostor = socket.create_connection(("127.0.0.1", port))     # wrong token
    fake = cm.SocketComm.__new__(cm.SocketComm)
    fake.size = 2
    import hashlib
    fake._key = hashlib.sha256(b"sgvamp-comm|wrong").digest()
    impostor.sendall(cm._HELLO.pack(1, 2, fake._mac(1)))
    t1 = threading.Thread(target=_rank_thread, args=(1, 2, port, "secret", out))
    t1.start()
    t0.join(60)
    t1.join(60)
    stray.close()
    impostor.close()
    assert out[0] == [0, 10] and out[1] == [0, 10], out


def test_env_launch_requires_rank_and_local_rank():
    """a RANK/WORLD_SIZE launch without RANK is refused (every
    process would be rank 0); LOCAL_RANK falls back to the global rank only on a
    one-node world (LOCAL_WORLD_SIZE == WORLD_SIZE, or no LOCAL_WORLD_SIZE and
    the ranks meeting on this host)."""
    import comm as cm

    with pytest.raises(RuntimeError, match="RANK is not set"):
        cm.launch_from_env(dict(WORLD_SIZE="2", LOCAL_RANK="0"))
    assert cm.launch_from_env(dict(WORLD_SIZE="1"))["rank"] == 0
    one = cm.launch_from_env(dict(RANK="1", WORLD_SIZE="2", LOCAL_WORLD_SIZE="2"))
    assert one["local_rank"] == 1
    assert cm.launch_from_env(dict(RANK="1", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1"))["local_rank"] == 1
    with pytest.raises(RuntimeError, match="LOCAL_RANK"):     # two nodes of 4 GPUs
        cm.launch_from_env(dict(RANK="5", WORLD_SIZE="8", LOCAL_WORLD_SIZE="4", MASTER_ADDR="10.0.0.5"))
    with pytest.raises(RuntimeError, match="LOCAL_RANK"):     # remote rendezvous, node size unknown
        cm.launch_from_env(dict(RANK="5", WORLD_SIZE="8", MASTER_ADDR="10.0.0.5"))
    # a MASTER_ADDR naming this host (its name, or an address one of its
    # interfaces holds) is a one-node launch -- if the world
    # fits this node's GPUs; otherwise (a multi-node job whose
    # rendezvous is here) LOCAL_RANK stays required
    import socket
    host = socket.gethostname()
    try:
        socket.getaddrinfo(host, None)
        resolvable = True
    except OSError:
        resolvable = False
    if resolvable:
        two = dict(RANK="1", WORLD_SIZE="2", MASTER_ADDR=host, HIP_VISIBLE_DEVICES="0,1")
        assert cm.launch_from_env(two)["local_rank"] == 1
        with pytest.raises(RuntimeError, match="LOCAL_RANK"):  # 16 ranks, 8 GPUs here
            cm.launch_from_env(dict(RANK="9", WORLD_SIZE="16", MASTER_ADDR=host,
                                    ROCR_VISIBLE_DEVICES="0,1,2,3,4,5,6,7"))
    # no device count known: a non-loopback address never implies one node
    assert cm._local_gpu_count(dict(HIP_VISIBLE_DEVICES="3,5,")) == 2
