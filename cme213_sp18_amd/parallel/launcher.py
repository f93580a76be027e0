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
127.0.0.1 -m cme213_sp18_amd.train ...``, or just ``--gpus N`` on the CLI /
bench.py: :func:`self_launch` then starts the N ranks itself (the reference's
``mpirun -np 4 ./main``, fpcode/run.sh:39), and :func:`verify_placement`
checks that the ranks really are N processes on N distinct GPUs.
"""
from __future__ import annotations

import datetime
import os
import socket
import subprocess
import sys

import torch

from .comm import Communicator, NullComm, TorchDistComm


class PlacementError(RuntimeError):
    """The job does not have the ranks / devices it was asked for (--gpus N)."""


def launched() -> bool:
    """True inside a rank started by a launcher (torchrun, :func:`spawn`, :func:`self_launch`)."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def self_launch(gpus: int, argv: list[str], *, module: str | None = None, script: str | None = None,
                need_gpus: bool = True) -> int | None:
    """Start ``gpus`` ranks of this same command on this node and return their exit code.

    Returns None (run in-process) when ``gpus <= 1`` or the process already is a rank.  The ranks come from
    a CHILD ``torch.distributed.run`` (never an exec of this process): the parent has made no GPU call --
    counting devices with ``torch.cuda.device_count()`` does not initialise one -- and it only waits.
    The launcher exports RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_*, so the ranks see one
    node (``xgmi.same_node``).  Refuses (PlacementError) when fewer GPUs are visible than ranks requested --
    on a GPU node, or anywhere with ``need_gpus`` -- unless CME_SHARED_GPU=1 (the several-ranks-on-one-GPU
    rehearsal); with no GPU and not ``need_gpus`` the ranks are CPU (gloo) processes."""
    if gpus <= 1 or launched():
        return None
    if os.environ.get("CME_SHARED_GPU") != "1":
        have = torch.cuda.device_count()
        if (need_gpus or have > 0) and have < gpus:
            raise PlacementError(f"--gpus {gpus} requested but only {have} GPU(s) visible on this node")
    if (module is None) == (script is None):
        raise ValueError("self_launch: exactly one of module / script")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}"]
    cmd += ["-m", module] if module is not None else [script]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd + list(argv), env=env).returncode


def device_identity(device: torch.device) -> str:
    """A node-unique name of the device this rank runs on (hostname + GPU uuid), or the CPU process."""
    host = os.uname().nodename
    if device.type != "cuda":
        return f"{host}:cpu:{os.getpid()}"
    props = torch.cuda.get_device_properties(device)
    ident = str(getattr(props, "uuid", "")) or f"{os.environ.get('HIP_VISIBLE_DEVICES', '')}:{device.index}"
    return f"{host}:{ident}"


def verify_placement(comm: Communicator, device: torch.device, gpus: int) -> dict:
    """Collective: check that the job is ``gpus`` ranks on ``gpus`` distinct GPUs; raise PlacementError on
    every rank otherwise.  Returns {"ranks_seen", "devices_distinct", "shared_gpu"}.  Processes sharing a
    GPU are accepted only under CME_SHARED_GPU=1 (and reported as such); CPU ranks (gloo tests) count as
    distinct devices."""
    shared_ok = os.environ.get("CME_SHARED_GPU") == "1"
    if comm.world_size != gpus:
        raise PlacementError(f"--gpus {gpus} but the job has {comm.world_size} rank(s)")
    if comm.world_size == 1:
        return {"ranks_seen": 1, "devices_distinct": True, "shared_gpu": False}
    import torch.distributed as dist

    ids = [None] * comm.world_size
    dist.all_gather_object(ids, device_identity(device), group=getattr(comm, "group", None))
    distinct = len(set(ids)) == len(ids)
    if not distinct and not shared_ok:
        raise PlacementError(f"ranks share GPUs ({len(set(ids))} distinct devices for {len(ids)} ranks)")
    return {"ranks_seen": comm.world_size, "devices_distinct": distinct, "shared_gpu": not distinct}


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
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
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
