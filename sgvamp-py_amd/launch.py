"""One process per GPU on this node, started by the program itself.

``bench.py --gpus N`` and ``main.py --gpus N`` call ``relaunch`` before they
touch the GPU: when no launcher has set up a world (``comm.launch_from_env``
finds none) and N > 1, the parent starts N copies of the same command line as
child processes -- never an exec -- with RANK, LOCAL_RANK, WORLD_SIZE,
LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free SGV_COMM_PORT and a random
SGV_COMM_TOKEN set, waits for them and exits with the first failing child's
status (the others are then stopped).  Rank 0 keeps the parent's stdout, so its
one JSON line / log goes where the parent's would; the other ranks' stdout goes
to stderr.  Under an external launcher ``--gpus`` must equal its world size.

This replaces the reference's ``mpirun -np K`` (src/main.py:16-18) for the
one-node case; MPI launches are still accepted (comm.launch_from_env).
"""
import os
import secrets
import signal
import socket
import subprocess
import sys
import time


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_envs(n, base=None, port=None, token=None):
    """The environment of each of n local ranks (list of dicts)."""
    base = dict(os.environ if base is None else base)
    port = _free_port() if port is None else int(port)
    token = secrets.token_hex(16) if token is None else token
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SGV_COMM_PORT=str(port),
                 SGV_COMM_TOKEN=token, SGV_LAUNCHED_BY="sgvamp.launch")
        out.append(e)
    return out


class _Signalled(BaseException):
    def __init__(self, signum):
        super().__init__(signum)
        self.signum = signum


def _pdeathsig():
    """Child side, between fork and exec (nothing has touched a GPU): the kernel
    sends the rank SIGTERM if the parent dies without stopping it (SIGKILL)."""
    try:
        import ctypes

        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl(1, signal.SIGTERM, 0, 0, 0)      # PR_SET_PDEATHSIG
    except Exception:  # noqa: BLE001 -- best effort (non-Linux)
        pass


def spawn(n, argv, base=None, poll_s=0.05):
    """Run argv as n local ranks; returns the exit status (0 when all succeed,
    else the first failing rank's).  A SIGTERM / SIGHUP / SIGINT to this parent
    (a scheduler or timeout signalling only its PID) stops every rank before the
    parent exits with 128 + the signal; a parent killed outright takes the ranks
    with it (PR_SET_PDEATHSIG)."""
    procs = []
    old = {}

    def on_signal(signum, _frame):
        raise _Signalled(signum)

    for sig in (signal.SIGTERM, signal.SIGHUP):
        try:
            old[sig] = signal.signal(sig, on_signal)
        except ValueError:   # not the main thread: leave the handlers alone
            pass
    try:
        for r, env in enumerate(rank_envs(n, base)):
            procs.append(subprocess.Popen(argv, env=env, preexec_fn=_pdeathsig,
                                          stdout=None if r == 0 else sys.stderr.fileno()))
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                _stop(procs)
                return bad[0] if bad[0] > 0 else 128 - bad[0]
            if all(c == 0 for c in codes):
                return 0
            time.sleep(poll_s)
    except _Signalled as e:
        _stop(procs)
        return 128 + int(e.signum)
    except BaseException:
        _stop(procs)
        raise
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)


def _stop(procs, grace=10.0):
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t = time.monotonic() + grace
    for p in procs:
        while p.poll() is None and time.monotonic() < t:
            time.sleep(0.05)
        if p.poll() is None:
            p.kill()
            p.wait()


def relaunch(gpus, argv=None, environ=None):
    """Called first thing by a --gpus N entry point.  Returns None when this
    process is (one rank of) the run; otherwise runs the N ranks as children
    and returns their exit status for the caller to exit with."""
    from comm import launch_from_env

    info = launch_from_env(environ)
    if info["source"] != "none":
        if gpus is not None and int(gpus) != info["size"]:
            raise SystemExit("--gpus %d but the launcher (%s) started %d rank(s): they must agree"
                             % (int(gpus), info["source"], info["size"]))
        return None
    if gpus is None or int(gpus) <= 1:
        return None
    argv = list(sys.argv if argv is None else argv)
    return spawn(int(gpus), [sys.executable] + argv, environ)
