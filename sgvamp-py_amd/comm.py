"""Host-side communicators (bootstrap, barriers, timing).

The data-path reductions of the solver run inside libsgvamp_hip.so over RCCL.
These objects exchange the RCCL unique id, synchronise ranks and combine
scalars for logging/benchmarking; ``allgather_f64`` also serves as the
library's host exchange (``sgv_comm_init_host``) when RCCL cannot connect the
ranks (e.g. several ranks on one device).  They mirror the subset of the
mpi4py API the reference uses (src/main.py:16-18; src/sgvamp.py:202,232-233):
Get_rank, Get_size, bcast -- plus allgather and barrier.
"""
import os


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
        return arr.copy()

    def barrier(self):
        pass


class TorchGlooComm:
    """torch.distributed (gloo, CPU) as bootstrap plumbing for one-process-per-GPU
    runs launched by torchrun.  Rendezvous from MASTER_ADDR/MASTER_PORT/RANK/
    WORLD_SIZE (env://)."""

    def __init__(self):
        import torch.distributed as dist

        self.dist = dist
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group(backend="gloo", init_method="env://")
        self.rank = dist.get_rank()
        self.size = dist.get_world_size()

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def bcast(self, obj, root=0):
        box = [obj]
        self.dist.broadcast_object_list(box, src=root)
        return box[0]

    def allgather(self, obj):
        out = [None] * self.size
        self.dist.all_gather_object(out, obj)
        return out

    def allgather_f64(self, arr):
        """All-gather a float64 array of the same length from every rank, in rank
        order (size * len(arr) doubles)."""
        import torch

        t = torch.from_numpy(arr)
        out = [torch.empty_like(t) for _ in range(self.size)]
        self.dist.all_gather(out, t)
        return torch.cat(out).numpy()

    def barrier(self):
        self.dist.barrier()


def world_from_env():
    """SingleComm unless WORLD_SIZE > 1 (torchrun), then TorchGlooComm."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return TorchGlooComm()
    return SingleComm()
