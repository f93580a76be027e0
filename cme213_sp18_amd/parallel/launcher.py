"""Process-group bootstrap: one process per GPU, no MPI.

The reference uses ``MPI_Init`` + ``cudaSetDevice(rank)`` (fpcode/main.cpp:37-50),
which maps the GLOBAL rank to a device id (breaks multi-node) and only warns
when there are fewer GPUs than ranks.  Here:

* ranks come from the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE /
  MASTER_ADDR / MASTER_PORT); the device is ``LOCAL_RANK``;
* the backend is ``"nccl"`` (RCCL over xGMI) when a GPU is present, ``gloo``
  otherwise (CPU tests);
* a rank with no GPU to bind to is an error, not a warning.

Launch: ``python -m torch.distributed.run --nproc-per-node N --master-addr
127.0.0.1 -m cme213_sp18_amd.train ...`` (or :func:`spawn` for tests).
"""
from __future__ import annotations

import datetime
import os
import socket

import torch

from .comm import Communicator, NullComm, TorchDistComm


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init_distributed(backend: str | None = None, timeout_s: float = 600.0) -> tuple[Communicator, torch.device]:
    """Initialise the process group from env vars; returns (communicator, device)."""
    rank, local_rank, world = env_world()
    if os.environ.get("CME_SHARED_GPU") == "1":
        # rehearsal mode: every rank on cuda:0 with a gloo group (RCCL refuses two ranks on one GPU);
        # exercises the multi-rank GPU code paths (xGMI peer kernel, sharding, bench) on a 1-GPU box
        torch.cuda.set_device(0)
        device, backend, use_gpu = torch.device("cuda", 0), "gloo", False
    elif (use_gpu := torch.cuda.is_available() and backend != "gloo"):
        ndev = torch.cuda.device_count()
        if local_rank >= ndev:
            raise RuntimeError(f"LOCAL_RANK {local_rank} has no GPU to bind to ({ndev} visible)")
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    if world == 1:
        return NullComm(), device
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    if not dist.is_initialized():
        be = backend or ("nccl" if use_gpu else "gloo")
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return TorchDistComm(), device


def shutdown() -> None:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _spawn_entry(rank, fn, world, port, backend, args):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    comm, device = init_distributed(backend)
    try:
        fn(rank, world, comm, device, *args)
    finally:
        shutdown()


def spawn(fn, world_size: int, args: tuple = (), backend: str = "gloo") -> None:
    """Run ``fn(rank, world, comm, device, *args)`` in ``world_size`` processes."""
    import torch.multiprocessing as mp

    mp.start_processes(_spawn_entry, args=(fn, world_size, free_port(), backend, args), nprocs=world_size,
                       join=True, start_method="spawn")
