"""Host-side communicators (bootstrap, barriers, timing) -- never on the data path.

The data-path reductions of the solver run inside libsgvamp_hip.so over RCCL.
These objects only exchange the RCCL unique id, synchronise ranks and
combine scalars for logging/benchmarking.  They mirror the subset of the
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

    def barrier(self):
        self.dist.barrier()


def world_from_env():
    """SingleComm unless WORLD_SIZE > 1 (torchrun), then TorchGlooComm."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return TorchGlooComm()
    return SingleComm()
