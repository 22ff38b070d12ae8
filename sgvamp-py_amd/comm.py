"""Host-side communicators (bootstrap, barriers, timing) -- no third-party deps.

The data-path reductions of the solver run inside libsgvamp_hip.so over RCCL.
These objects exchange the RCCL unique id, synchronise ranks and combine
scalars for logging/benchmarking; ``allgather_f64`` also serves as the
library's host exchange (``sgv_comm_init_host``) when RCCL cannot connect the
ranks (e.g. several ranks on one device).  They mirror the subset of the
mpi4py API the reference uses (src/main.py:16-18; src/sgvamp.py:202,232-233):
Get_rank, Get_size, bcast -- plus allgather and barrier.

The rank model is one process per GPU.  ``launch_from_env`` reads it from
whichever launcher started the process:

* ``RANK``/``WORLD_SIZE``/``LOCAL_RANK`` (this build's own ``--gpus N``
  launcher, ``launch.py``, and any one-process-per-GPU launcher);
* Open MPI's ``mpirun`` (``OMPI_COMM_WORLD_{RANK,SIZE,LOCAL_RANK,LOCAL_SIZE}``),
  the reference's own launch (``mpirun -np K python main.py``, src/main.py:16-18);
* MPICH / Intel MPI Hydra (``PMI_RANK``/``PMI_SIZE``, ``MPI_LOCALRANKID``/
  ``MPI_LOCALNRANKS``);
* Slurm ``srun`` (``SLURM_PROCID``/``SLURM_STEP_NUM_TASKS``/``SLURM_LOCALID``).

Under an MPI or Slurm launch without ``MASTER_ADDR`` the ranks meet on
127.0.0.1 when they all run on one node; a multi-node launch must name rank 0's
host in ``MASTER_ADDR`` (there is no MPI library to ask), and is refused with
that message otherwise.  The rendezvous port is ``SGV_COMM_PORT``, else
``MASTER_PORT + 1`` (a launcher's own store may hold ``MASTER_PORT``), else one
derived from the launcher's job id.

Multi-rank runs use ``SocketComm``: a TCP star on that address.  Peers prove
they belong to the job with an HMAC of a shared token (``SGV_COMM_TOKEN``, set
by ``launch.py``; otherwise derived from the launch itself), a connection that
does not say hello correctly within a few seconds is dropped, and payloads are
encoded as JSON plus raw array bytes -- nothing received is ever unpickled.
"""
import hashlib
import hmac
import json
import os
import socket
import struct
import time
import zlib

import numpy as np


class SingleComm:
    """World of one rank (the K=1 / one-GPU case)."""

    local_rank = 0

    def Get_rank(self):
        return 0

    def Get_size(self):
        return 1

    def bcast(self, obj, root=0):
        return obj

    def allgather(self, obj):
        return [obj]

    def allgather_f64(self, arr):
        return np.array(arr, dtype=np.float64, copy=True)

    def barrier(self):
        pass

    def close(self):
        pass


_LEN = struct.Struct("<Q")
_HELLO = struct.Struct("<QQ32s")    # rank, size, HMAC-SHA256


def _send(sock, data):
    sock.sendall(_LEN.pack(len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed the connection")
        got += k
    return bytes(buf)


def _recv(sock):
    (n,) = _LEN.unpack(_recv_exact(sock, _LEN.size))
    return _recv_exact(sock, n)


# ---- payload codec: JSON for the structure, raw bytes for arrays ------------------
# Types the solver exchanges: None, bool, int, float, str, bytes, list, tuple,
# dict, numpy arrays of numeric dtype and numpy scalars.  Anything else raises
# on the sending side; the receiving side only ever builds these types.

_NUMERIC_KINDS = "biufc"


def encode(obj):
    bufs = []

    def enc(o):
        if o is None or isinstance(o, (bool, str)):
            return o
        if isinstance(o, (int, np.integer)) and not isinstance(o, bool):
            return {"$i": str(int(o))}
        if isinstance(o, (float, np.floating)):
            return {"$f": float(o).hex()}          # exact, including inf/nan
        if isinstance(o, (bytes, bytearray)):
            bufs.append(bytes(o))
            return {"$b": len(bufs) - 1}
        if isinstance(o, np.ndarray):
            if o.dtype.kind not in _NUMERIC_KINDS:
                raise TypeError("comm: arrays of dtype %s are not exchanged" % o.dtype)
            a = np.ascontiguousarray(o)
            bufs.append(a.tobytes())
            return {"$a": len(bufs) - 1, "dtype": a.dtype.str, "shape": list(a.shape)}
        if isinstance(o, tuple):
            return {"$t": [enc(x) for x in o]}
        if isinstance(o, list):
            return [enc(x) for x in o]
        if isinstance(o, dict):
            return {"$d": [[enc(k), enc(v)] for k, v in o.items()]}
        raise TypeError("comm: cannot exchange objects of type %s" % type(o).__name__)

    head = json.dumps(enc(obj), separators=(",", ":")).encode()
    out = [_LEN.pack(len(head)), head, _LEN.pack(len(bufs))]
    for b in bufs:
        out += [_LEN.pack(len(b)), b]
    return b"".join(out)


def decode(blob):
    pos = 0

    def take(n):
        nonlocal pos
        if pos + n > len(blob):
            raise ValueError("comm: truncated payload")
        v = blob[pos:pos + n]
        pos += n
        return v

    (hn,) = _LEN.unpack(take(_LEN.size))
    head = json.loads(take(hn).decode())
    (nb,) = _LEN.unpack(take(_LEN.size))
    bufs = []
    for _ in range(nb):
        (n,) = _LEN.unpack(take(_LEN.size))
        bufs.append(take(n))

    def dec(o):
        if isinstance(o, list):
            return [dec(x) for x in o]
        if not isinstance(o, dict):
            return o
        if "$i" in o:
            return int(o["$i"])
        if "$f" in o:
            return float.fromhex(o["$f"])
        if "$b" in o:
            return bufs[o["$b"]]
        if "$a" in o:
            dt = np.dtype(o["dtype"])
            if dt.kind not in _NUMERIC_KINDS:
                raise ValueError("comm: refused array dtype %s" % dt)
            return np.frombuffer(bufs[o["$a"]], dtype=dt).reshape(o["shape"]).copy()
        if "$t" in o:
            return tuple(dec(x) for x in o["$t"])
        if "$d" in o:
            return {dec(k): dec(v) for k, v in o["$d"]}
        raise ValueError("comm: malformed payload")

    return dec(head)


class SocketComm:
    """TCP star: every rank holds one connection to rank 0; a collective is
    gather-to-0 then send-back (payloads are a few KB to a few MB: latency,
    not bandwidth, matters).  All collectives are blocking and must be called
    by every rank in the same order (MPI semantics)."""

    HELLO_TIMEOUT = 5.0

    def __init__(self, rank, size, addr="127.0.0.1", port=29500, timeout=300.0, token=None,
                 local_rank=None):
        self.rank, self.size = int(rank), int(size)
        self.local_rank = self.rank if local_rank is None else int(local_rank)
        self.peers = {}
        self.sock = None
        key = (token if token is not None else "%s:%d:%d" % (addr, port, self.size)).encode()
        self._key = hashlib.sha256(b"sgvamp-comm|" + key).digest()
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            self._accept_peers(addr, port, deadline)
        else:
            self._connect(addr, port, deadline)

    def _mac(self, rank):
        return hmac.new(self._key, b"hello|%d|%d" % (rank, self.size), hashlib.sha256).digest()

    def _accept_peers(self, addr, port, deadline):
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind((addr, port))
        srv.listen(max(self.size, 8))
        try:
            while len(self.peers) < self.size - 1:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError("rendezvous: %d of %d ranks joined %s:%d"
                                       % (len(self.peers) + 1, self.size, addr, port))
                srv.settimeout(left)
                try:
                    conn, _ = srv.accept()
                except socket.timeout:
                    continue
                # the hello is read under a short timeout; a connection that is
                # silent, malformed or unauthenticated is dropped, not fatal
                try:
                    conn.settimeout(self.HELLO_TIMEOUT)
                    r, n, mac = _HELLO.unpack(_recv_exact(conn, _HELLO.size))
                    ok = (n == self.size and 0 < r < self.size and r not in self.peers
                          and hmac.compare_digest(mac, self._mac(r)))
                except (OSError, ConnectionError, struct.error):
                    ok = False
                if not ok:
                    conn.close()
                    continue
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                conn.settimeout(None)
                self.peers[int(r)] = conn
        finally:
            srv.close()

    def _connect(self, addr, port, deadline):
        while True:
            try:
                s = socket.create_connection((addr, port), timeout=5.0)
                break
            except OSError:
                if time.monotonic() > deadline:
                    raise TimeoutError("rendezvous with rank 0 at %s:%d timed out" % (addr, port))
                time.sleep(0.05)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.settimeout(None)
        s.sendall(_HELLO.pack(self.rank, self.size, self._mac(self.rank)))
        self.sock = s

    @classmethod
    def from_env(cls, environ=None):
        info = launch_from_env(environ)
        return cls(info["rank"], info["size"], info["addr"], info["port"], token=info["token"],
                   local_rank=info["local_rank"])

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def allgather_bytes(self, payload):
        """Every rank's bytes, in rank order, on every rank."""
        payload = bytes(payload)
        if self.size == 1:
            return [payload]
        if self.rank == 0:
            parts = [payload] + [_recv(self.peers[r]) for r in range(1, self.size)]
            blob = b"".join(_LEN.pack(len(p)) for p in parts) + b"".join(parts)
            for r in range(1, self.size):
                _send(self.peers[r], blob)
        else:
            _send(self.sock, payload)
            blob = _recv(self.sock)
        lens = [_LEN.unpack_from(blob, _LEN.size * i)[0] for i in range(self.size)]
        out, pos = [], _LEN.size * self.size
        for n in lens:
            out.append(blob[pos:pos + n])
            pos += n
        return out

    def allgather(self, obj):
        return [decode(b) for b in self.allgather_bytes(encode(obj))]

    def bcast(self, obj, root=0):
        parts = self.allgather_bytes(encode(obj) if self.rank == root else b"")
        return decode(parts[root])

    def allgather_f64(self, arr):
        """All-gather a float64 array of the same length from every rank, in rank
        order (size * len(arr) doubles)."""
        a = np.ascontiguousarray(arr, dtype=np.float64)
        parts = self.allgather_bytes(a.tobytes())
        if any(len(p) != a.nbytes for p in parts):
            raise ValueError("allgather_f64: ranks passed arrays of different lengths")
        return np.frombuffer(b"".join(parts), dtype=np.float64).copy()

    def barrier(self):
        self.allgather_bytes(b"")

    def close(self):
        for s in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = {}, None


# ---- launcher detection --------------------------------------------------------------

def _int(env, *names):
    for n in names:
        v = env.get(n)
        if v not in (None, ""):
            return int(v)
    return None


def _job_port(job):
    """A rendezvous port derived from a launcher's job id (20000-39999)."""
    return 20000 + zlib.crc32(job.encode()) % 20000


def launch_from_env(environ=None):
    """The rank model of this process: dict(rank, size, local_rank, local_size,
    addr, port, token, source).  size 1 when no launcher is detected."""
    env = os.environ if environ is None else environ
    job = None
    if _int(env, "WORLD_SIZE") is not None:
        source = "env"
        rank, size = _int(env, "RANK"), _int(env, "WORLD_SIZE")
        if rank is None:
            if size > 1:   # every process would take rank 0 and bind the rendezvous port
                raise RuntimeError("WORLD_SIZE=%d but RANK is not set: a launcher of %d ranks "
                                   "must give each its RANK" % (size, size))
            rank = 0
        local_rank = _int(env, "LOCAL_RANK")
        local_size = _int(env, "LOCAL_WORLD_SIZE")
    elif _int(env, "OMPI_COMM_WORLD_SIZE") is not None:
        source = "openmpi"
        rank, size = _int(env, "OMPI_COMM_WORLD_RANK"), _int(env, "OMPI_COMM_WORLD_SIZE")
        local_rank = _int(env, "OMPI_COMM_WORLD_LOCAL_RANK")
        local_size = _int(env, "OMPI_COMM_WORLD_LOCAL_SIZE")
        job = env.get("OMPI_MCA_ess_base_jobid") or env.get("PMIX_NAMESPACE") or \
            env.get("OMPI_MCA_orte_ess_jobid")
    elif _int(env, "PMI_SIZE") is not None:
        source = "pmi"
        rank, size = _int(env, "PMI_RANK"), _int(env, "PMI_SIZE")
        local_rank = _int(env, "MPI_LOCALRANKID", "PMI_LOCAL_RANK")
        local_size = _int(env, "MPI_LOCALNRANKS", "PMI_LOCAL_SIZE")
        job = env.get("PMI_KVSNAME") or env.get("PMI_ID")
    elif _int(env, "SLURM_STEP_NUM_TASKS") is not None and _int(env, "SLURM_PROCID") is not None:
        # srun sets the step's task count; a batch script alone (one process
        # in an allocation of many tasks) does not, and stays one rank
        source = "slurm"
        rank, size = _int(env, "SLURM_PROCID"), _int(env, "SLURM_STEP_NUM_TASKS")
        local_rank = _int(env, "SLURM_LOCALID")
        nnodes = _int(env, "SLURM_STEP_NUM_NODES", "SLURM_NNODES")
        local_size = size if nnodes == 1 else None
        job = "%s.%s" % (env.get("SLURM_JOB_ID", ""), env.get("SLURM_STEP_ID", ""))
    else:
        return dict(rank=0, size=1, local_rank=0, local_size=1, addr="127.0.0.1", port=None,
                    token=None, source="none")
    if rank is None or size is None or not 0 <= rank < size:
        raise RuntimeError("launcher environment (%s): rank %r of world size %r" % (source, rank, size))
    if local_rank is None:
        # the global rank is the node-local one only on a one-node world: the
        # launcher says so (node-local size = world size), or -- RANK/WORLD_SIZE
        # launches that set no LOCAL_WORLD_SIZE -- the ranks meet on this host
        # -- a loopback rendezvous, or one on an address of this host when the
        # whole world fits this node's GPUs (in a multi-node job
        # whose MASTER_ADDR names this host, the ranks here must not take
        # rank = local rank while the other nodes' ranks fail; the device count
        # is checked before any name lookup)
        maddr = env.get("MASTER_ADDR", "127.0.0.1")
        ngpu = _local_gpu_count(env) if maddr not in _LOOPBACK else None
        one_node = (local_size == size or size == 1 or
                    (source == "env" and local_size is None and
                     (maddr in _LOOPBACK or
                      (ngpu is not None and size <= ngpu and _is_local_addr(maddr)))))
        local_rank = rank if one_node else None
    if local_rank is None:
        raise RuntimeError("launcher environment (%s) gives no node-local rank: set LOCAL_RANK "
                           "(it selects this rank's GPU)" % source)
    addr = env.get("MASTER_ADDR")
    if not addr:
        if size > 1 and local_size != size and source != "env":
            raise RuntimeError(
                "%d ranks launched by %s over more than one node (or the node-local world size "
                "is unknown): set MASTER_ADDR to rank 0's host -- the ranks meet there (this "
                "build runs one process per GPU and needs no MPI library to do so)" % (size, source))
        addr = "127.0.0.1"
    if env.get("SGV_COMM_PORT"):
        port = int(env["SGV_COMM_PORT"])
    elif env.get("MASTER_PORT"):
        port = int(env["MASTER_PORT"]) + 1
    elif job:
        port = _job_port(job)
    else:
        port = 29501
    token = env.get("SGV_COMM_TOKEN") or ("%s|%s" % (source, job) if job else None)
    return dict(rank=int(rank), size=int(size), local_rank=int(local_rank),
                local_size=local_size, addr=addr, port=int(port), token=token, source=source)


_LOOPBACK = ("127.0.0.1", "localhost", "::1")


def _local_gpu_count(env):
    """GPUs this process may use on this node, without initialising HIP: the
    count of a *_VISIBLE_DEVICES list if one is set (the smallest), else the
    KFD topology's GPU nodes (gfx_target_version != 0); None if unknown."""
    counts = []
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(k)
        if v is not None:
            counts.append(len([x for x in v.split(",") if x.strip()]))
    if counts:
        return min(counts)
    import glob

    n = 0
    for path in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(path) as f:
                for line in f:
                    if line.startswith("gfx_target_version") and int(line.split()[1]) != 0:
                        n += 1
                        break
        except (OSError, ValueError, IndexError):
            continue
    return n or None


def _is_local_addr(addr):
    """True if `addr` (a name or a literal) is this host: a loopback name, or an
    address some local interface holds (a socket can be bound to it)."""
    if addr in _LOOPBACK:
        return True
    try:
        infos = socket.getaddrinfo(addr, None)
    except OSError:
        return False
    for fam, _, _, _, sa in infos:
        try:
            with socket.socket(fam, socket.SOCK_DGRAM) as s:
                s.bind((sa[0], 0))
            return True
        except OSError:
            continue
    return False


def world_from_env(environ=None):
    """SingleComm unless the launcher started more than one rank, then SocketComm."""
    info = launch_from_env(environ)
    if info["size"] > 1:
        return SocketComm(info["rank"], info["size"], info["addr"], info["port"],
                          token=info["token"], local_rank=info["local_rank"])
    return SingleComm()
