#!/usr/bin/env python3
"""All-reduce latency / bandwidth sweep: RCCL (torch.distributed "nccl") vs the xGMI one-shot peer kernel.

The reference's gradient sync is 4 x MPI_Allreduce(SUM) on host buffers per batch
(fpcode/neural_network.cpp:501-536).  This bench prices the two device-side replacements the
data-parallel trainer chooses between (parallel/trainer.py, ``allreduce=auto|xgmi|rccl``) on the
bucket sizes that matter:

* the MLP gradient buckets: 784-100-10 (79,510 fp32 = 318 KB), 784-1024-10 (814,090 = 3.3 MB),
  784-4096-10 (3,256,330 = 13 MB);
* a power-of-4 sweep from 4 KB to 64 MB.

Launch one rank per GPU:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/allreduce_bench.py

Per size and path, rank 0 prints one JSON line: microseconds per call (``--iters`` back-to-back calls
on one stream, as in the training step; the loop is bracketed by barrier + synchronize and the max
over ranks is taken), ``algbw`` = bytes / time and ``busbw`` = algbw * 2 (R-1) / R (the
ring-equivalent bytes per rank, the nccl-tests convention).  Rehearsal on a one-GPU box:
``CME_SHARED_GPU=1`` (ranks share cuda:0 over gloo) -- then "rccl" is gloo on host memory and only
the xGMI rows say anything about the kernel.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MLP_BUCKETS = {"mlp_h100": 784 * 100 + 100 + 10 * 100 + 10,
               "mlp_h1024": 784 * 1024 + 1024 + 10 * 1024 + 10,
               "mlp_h4096": 784 * 4096 + 4096 + 10 * 4096 + 10}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--paths", nargs="*", default=["rccl", "xgmi", "xgmi-bf16"], choices=["rccl", "xgmi", "xgmi-bf16"],
                    help="xgmi-bf16: fp32 gradients over a bf16 wire (half the bytes), summed in fp32")
    ap.add_argument("--min-bytes", type=int, default=4 << 10)
    ap.add_argument("--max-bytes", type=int, default=64 << 20)
    ap.add_argument("--xgmi-max-bytes", type=int, default=16 << 20, help="largest bucket tried on the xGMI path")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--json", default=None, help="also write every record to this file (rank 0)")
    return ap.parse_args(argv)


def sizes(a) -> list[tuple[str, int]]:
    eb = 4 if a.dtype == "f32" else 8
    out = [(k, v) for k, v in MLP_BUCKETS.items() if a.min_bytes <= v * eb <= a.max_bytes]
    b = a.min_bytes
    while b <= a.max_bytes:
        out.append((f"{b}B", b // eb))
        b *= 4
    return out


def time_calls(fn, comm, device, iters: int, warmup: int) -> float:
    """Seconds per call: ``iters`` back-to-back calls bracketed by barrier + synchronize, max over ranks."""
    import torch

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(device)
    comm.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize(device)
    comm.barrier()
    dt = time.perf_counter() - t0
    return comm.allreduce_scalar(dt, op="max") / iters


def main(argv=None) -> int:
    a = parse(argv)
    import torch

    from cme213_sp18_amd.parallel.launcher import init_distributed, shutdown

    comm, device = init_distributed()
    R, rank = comm.world_size, comm.rank
    if R < 2 or device.type != "cuda":
        print("allreduce_bench: needs >= 2 GPU ranks (torch.distributed.run --nproc-per-node N)", file=sys.stderr)
        shutdown()
        return 2
    dt = torch.float32 if a.dtype == "f32" else torch.float64
    eb = 4 if a.dtype == "f32" else 8
    records = []
    for label, n in sizes(a):
        base = torch.arange(n, dtype=torch.float64, device=device).remainder_(997).to(dt)
        expect = base.double() * (R * (R + 1) / 2)
        t = base * (rank + 1)
        for path in a.paths:
            rec = {"size": label, "numel": n, "bytes": n * eb, "world": R, "path": path, "dtype": a.dtype}
            if path == "rccl":
                rec["backend"] = getattr(comm, "backend", comm.name)
                t.copy_(base * (rank + 1))
                comm.allreduce_(t)
                torch.cuda.synchronize(device)
                ok = bool(torch.allclose(t.double(), expect, rtol=1e-6))
                sec = time_calls(lambda: comm.allreduce_(t), comm, device, a.iters, a.warmup)
            else:
                if n * eb > a.xgmi_max_bytes or (path == "xgmi-bf16" and dt != torch.float32):
                    continue
                from cme213_sp18_amd.parallel.xgmi import XgmiBucket

                wire = torch.bfloat16 if path == "xgmi-bf16" else dt
                if path == "xgmi-bf16":  # what crosses the wire is bf16(base * (rank + 1)), summed in fp32
                    expect = sum((base * (r + 1)).to(torch.bfloat16).double() for r in range(R))
                    rec["wire_bytes"] = n * 2
                try:  # collective: on an IPC failure every rank skips this size together
                    xb = XgmiBucket(comm.group, rank, R, n, dt, device, self_test=False, wire=wire)
                except RuntimeError as ex:
                    rec["error"] = str(ex)
                    records.append(rec)
                    if rank == 0:
                        print(json.dumps(rec), flush=True)
                    continue
                t.copy_(base * (rank + 1))
                xb.allreduce_(t)
                torch.cuda.synchronize(device)
                ok = bool(torch.allclose(t.double(), expect, rtol=1e-6))
                sec = time_calls(lambda: xb.allreduce_(t), comm, device, a.iters, a.warmup)
                rec["peer_wait_timeouts"] = xb.error()
                ok = ok and rec["peer_wait_timeouts"] == 0
                xb.close()
                expect = base.double() * (R * (R + 1) / 2)
            rec["correct"] = comm.allreduce_scalar(0.0 if ok else 1.0, op="max") == 0.0
            rec["us"] = round(sec * 1e6, 3)
            algbw = n * eb / sec / 1e9
            rec["algbw_GBs"] = round(algbw, 3)
            rec["busbw_GBs"] = round(algbw * 2 * (R - 1) / R, 3)
            records.append(rec)
            if rank == 0:
                print(json.dumps(rec), flush=True)
    if rank == 0 and a.json:
        with open(a.json, "w") as f:
            json.dump(records, f, indent=1)
    shutdown()
    return 0 if all(r.get("correct", True) for r in records) else 1


if __name__ == "__main__":
    sys.exit(main())
