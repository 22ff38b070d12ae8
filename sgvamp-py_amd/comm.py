"""Host-side communicators (bootstrap, barriers, timing) -- no third-party deps.

The data-path reductions of the solver run inside libsgvamp_hip.so over RCCL.
These objects exchange the RCCL unique id, synchronise ranks and combine
scalars for logging/benchmarking; ``allgather_f64`` also serves as the
library's host exchange (``sgv_comm_init_host``) when RCCL cannot connect the
ranks (e.g. several ranks on one device).  They mirror the subset of the
mpi4py API the reference uses (src/main.py:16-18; src/sgvamp.py:202,232-233):
Get_rank, Get_size, bcast -- plus allgather and barrier.

Multi-rank runs use ``SocketComm``: a TCP star rendezvous read from the
environment any one-process-per-GPU launcher sets (RANK, WORLD_SIZE,
MASTER_ADDR, MASTER_PORT; LOCAL_RANK picks the device).  The launcher's own
store may already listen on MASTER_PORT, so rank 0 listens on
``SGV_COMM_PORT`` (default MASTER_PORT + 1).
"""
import os
import pickle
import socket
import struct
import time

import numpy as np


class SingleComm:
    """World of one rank (the K=1 / one-GPU case)."""

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


class SocketComm:
    """TCP star: every rank holds one connection to rank 0; a collective is
    gather-to-0 then send-back (payloads are a few KB to a few MB: latency,
    not bandwidth, matters).  All collectives are blocking and must be called
    by every rank in the same order (MPI semantics)."""

    def __init__(self, rank, size, addr="127.0.0.1", port=29500, timeout=300.0):
        self.rank, self.size = int(rank), int(size)
        self.peers = {}
        self.sock = None
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.size)
            srv.settimeout(max(1.0, deadline - time.monotonic()))
            try:
                while len(self.peers) < self.size - 1:
                    conn, _ = srv.accept()
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    conn.settimeout(None)
                    (r,) = _LEN.unpack(_recv_exact(conn, _LEN.size))
                    if not 0 < r < self.size or r in self.peers:
                        conn.close()
                        raise RuntimeError("rendezvous: unexpected rank %d" % r)
                    self.peers[int(r)] = conn
            finally:
                srv.close()
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise TimeoutError("rendezvous with rank 0 at %s:%d timed out"
                                           % (addr, port))
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(None)
            s.sendall(_LEN.pack(self.rank))
            self.sock = s

    @classmethod
    def from_env(cls):
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("SGV_COMM_PORT") or int(os.environ.get("MASTER_PORT", "29500")) + 1)
        return cls(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), addr, port)

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
        return [pickle.loads(b) for b in self.allgather_bytes(pickle.dumps(obj))]

    def bcast(self, obj, root=0):
        parts = self.allgather_bytes(pickle.dumps(obj) if self.rank == root else b"")
        return pickle.loads(parts[root])

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


def world_from_env():
    """SingleComm unless WORLD_SIZE > 1 (one process per GPU), then SocketComm."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return SocketComm.from_env()
    return SingleComm()
