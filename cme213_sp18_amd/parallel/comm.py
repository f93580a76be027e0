"""Communicators for the data-parallel trainer.

The reference synchronises gradients with four blocking ``MPI_Allreduce``
calls on HOST buffers after copying every gradient device->host
(fpcode/neural_network.cpp:496-536).  Here gradients never leave the GPU:

* :class:`TorchDistComm` -- one process per GPU, ``torch.distributed`` with
  backend ``"nccl"`` (= RCCL on ROCm, xGMI between the GPUs of a node).  The
  whole gradient bucket is ONE flat device tensor ``[dW1|db1|dW2|db2]``, so a
  step issues a single all-reduce (optionally split into row chunks that are
  issued as soon as each chunk is final).  Collectives are stream-ordered and
  can be captured into a HIP graph together with the kernels.
* :class:`NullComm` -- world_size == 1: no communicator, no overhead.
* :class:`LoopbackComm` -- in-process threads sharing host buffers; exercises
  the bucketing / sharding plumbing with no cluster (tests).

Process-group bootstrap lives in :mod:`cme213_sp18_amd.parallel.launcher`.
"""
from __future__ import annotations

import threading

import torch


class Communicator:
    rank: int = 0
    world_size: int = 1
    graph_capturable: bool = True

    def allreduce_(self, t: torch.Tensor) -> None:  # in-place SUM
        raise NotImplementedError

    def allreduce_scalar(self, v: float, op: str = "sum") -> float:
        raise NotImplementedError

    def barrier(self) -> None:
        pass

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        raise NotImplementedError

    @property
    def name(self) -> str:
        return type(self).__name__


class NullComm(Communicator):
    """world_size == 1 fast path."""

    def allreduce_(self, t):
        return None

    def allreduce_scalar(self, v, op="sum"):
        return float(v)

    def broadcast_(self, t, src=0):
        return None


class TorchDistComm(Communicator):
    """RCCL (backend "nccl") or gloo through the default torch.distributed group."""

    def __init__(self, group=None):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised; use parallel.launcher.init_distributed()")
        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.graph_capturable = self.backend == "nccl"

    def allreduce_(self, t):
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM, group=self.group)

    def allreduce_scalar(self, v, op="sum"):
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        x = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        rop = {"sum": self._dist.ReduceOp.SUM, "max": self._dist.ReduceOp.MAX, "min": self._dist.ReduceOp.MIN}[op]
        self._dist.all_reduce(x, op=rop, group=self.group)
        return float(x.item())

    @property
    def name(self) -> str:
        """"rccl" (the nccl backend on ROCm) or the gloo backend's name: what the record's allreduce reports."""
        return "rccl" if self.backend == "nccl" else str(self.backend)

    def barrier(self):
        if self.backend == "nccl":
            self._dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            self._dist.barrier(group=self.group)

    def broadcast_(self, t, src=0):
        self._dist.broadcast(t, src=src, group=self.group)


class _LoopbackHub:
    def __init__(self, world_size: int):
        self.world_size = world_size
        self.barrier = threading.Barrier(world_size)
        self.slots: list = [None] * world_size
        self.lock = threading.Lock()


class LoopbackComm(Communicator):
    """Thread-based communicator: ``world_size`` ranks in one process (CPU tensors).

    Reduction order is rank order, so results are deterministic.
    """
    graph_capturable = False

    def __init__(self, hub: _LoopbackHub, rank: int):
        self.hub = hub
        self.rank = rank
        self.world_size = hub.world_size

    @staticmethod
    def create(world_size: int) -> list["LoopbackComm"]:
        hub = _LoopbackHub(world_size)
        return [LoopbackComm(hub, r) for r in range(world_size)]

    def allreduce_(self, t):
        h = self.hub
        h.slots[self.rank] = t.detach().to("cpu", copy=True)
        h.barrier.wait()
        acc = h.slots[0].clone()
        for r in range(1, h.world_size):
            acc += h.slots[r]
        h.barrier.wait()
        t.copy_(acc.to(t.device))

    def allreduce_scalar(self, v, op="sum"):
        x = torch.tensor([float(v)], dtype=torch.float64)
        if op == "sum":
            self.allreduce_(x)
            return float(x.item())
        h = self.hub
        h.slots[self.rank] = float(v)
        h.barrier.wait()
        vals = list(h.slots)
        h.barrier.wait()
        return float(max(vals) if op == "max" else min(vals))

    def barrier(self):
        self.hub.barrier.wait()

    def broadcast_(self, t, src=0):
        h = self.hub
        if self.rank == src:
            h.slots[src] = t.detach().to("cpu", copy=True)
        h.barrier.wait()
        val = h.slots[src]
        h.barrier.wait()
        t.copy_(val.to(t.device))
