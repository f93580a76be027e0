#!/usr/bin/env python3
"""Headline benchmark: MNIST images/sec, 784-100-10 MLP, batch=800, on N MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it
runs under ``torch.distributed.run`` (one rank per GPU, RCCL) -- started by the
driver, or, when no launcher started this process, by bench.py itself (a child
launcher).  Every rank checks that the job is N ranks on N distinct GPUs and
exits non-zero WITHOUT a record otherwise (ranks_seen / devices_distinct are in
the record, with the measured all-reduce time of the step's bucket).  W untimed
warm-up steps, then EXACTLY K timed optimizer steps bracketed by barrier +
synchronize on both sides; the max time over ranks is reported; rank 0 prints
one JSON line.

What a step is (the reference's ``parallel_train`` inner loop,
fpcode/neural_network.cpp:449-555): one synchronous SGD update -- forward +
backward of the 784-100-10 MLP (random-init weights, seeded as the reference
does) on every rank, gradient all-reduce (xGMI peer kernel with the SGD
fused in, or RCCL with ``--allreduce rccl``), SGD update -- on
synthetic MNIST-shaped images resident on every GPU.  Nothing is skipped
inside the timed region.  Steps cycle over the full batches of the 54,000-image
training split and are replayed from a captured HIP graph.

Scaling (default ``weak``): every GPU processes 800 images per step, so the
global batch is 800*N (N=8 -> 6400, the BASELINE's 8-GPU batch); at N=1 this
is exactly batch=800.  ``--scaling strong`` instead splits a global batch of
800 across the N ranks (n = 800/N each), the reference's ``-b 800`` semantics.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

METRIC = "MNIST images/sec, 784-100-10 MLP batch=800 at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # BASELINE.json "published": {} -- no reference number exists


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--warmup", type=int, default=400)
    ap.add_argument("--hidden", type=int, default=100)
    ap.add_argument("--batch", type=int, default=800, help="global batch (strong) or per-GPU batch (weak)")
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64", "bf16"])
    ap.add_argument("--scaling", default="weak", choices=["strong", "weak"])
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--executor", default="auto", choices=["auto", "graph", "eager"],
                    help="auto: the native C++ step loop where a step is pure device work (one process, or the "
                         "xGMI-fused all-reduce), else captured HIP graphs; graph: always graphs")
    ap.add_argument("--allreduce", default="auto", choices=["auto", "xgmi", "xgmi2", "rccl", "host"],
                    help="gradient sync for N>1: auto (by bucket size and ranks), the xGMI one-shot peer kernel "
                         "with fused SGD (xgmi), the xGMI two-shot kernel with sharded SGD (xgmi2), RCCL, or "
                         "host-staged gloo (reference-equivalent)")
    ap.add_argument("--grad-wire", default="auto", choices=["auto", "f32", "bf16"],
                    help="element type of the gradients on the xGMI one-shot wire (bf16: opt-in, half the bytes)")
    ap.add_argument("--mode", default="optimized", choices=["optimized", "reference"],
                    help="reference: the reference's execution model on MI355X -- unfused PyTorch/hipBLAS ops, "
                         "no graphs, host-staged gradient all-reduce (for comparison only)")
    ap.add_argument("--parallel", default="dp", choices=["dp", "tp"],
                    help="dp: data parallel (the reference's scheme); tp: hidden-dimension tensor parallel "
                         "(one z2 all-reduce per step, every rank runs the whole global batch --batch; strong "
                         "scaling of a fixed model, meant for the wide configs)")
    ap.add_argument("--tune-allreduce", default="on", choices=["on", "off"],
                    help="N > 1 with --allreduce auto: time the policy's xGMI pick, the xGMI two-shot (N >= 3) and RCCL "
                         "for --tune-steps steps each before the timed region and run the fastest (the record lists "
                         "every candidate)")
    ap.add_argument("--tune-steps", type=int, default=100)
    ap.add_argument("--train-size", type=int, default=54000)
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    a = parse(argv)
    if a.mode == "reference":
        a.backend, a.no_graphs, a.allreduce = "torch", True, "host"
    from cme213_sp18_amd.parallel.launcher import PlacementError, self_launch

    # --gpus N without a launcher: start the N ranks here (a child torch.distributed.run, before any GPU
    # call in this process) and pass their exit code through; rank 0 of the child job prints the record
    try:
        rc = self_launch(a.gpus, argv, script=os.path.abspath(__file__), need_gpus=a.backend == "hip")
    except PlacementError as ex:
        print(f"error: {ex}; no record", file=sys.stderr, flush=True)
        return 2
    if rc is not None:
        return rc

    import numpy as np
    import torch

    from cme213_sp18_amd.models.mlp import NeuralNetwork
    from cme213_sp18_amd.parallel.launcher import init_distributed, shutdown, verify_placement
    from cme213_sp18_amd.parallel.trainer import DataParallelTrainer, EpochPlan
    from cme213_sp18_amd.utils.data import synthetic_mnist

    comm, device = init_distributed()
    R, rank = comm.world_size, comm.rank
    try:  # the job must be exactly --gpus ranks on --gpus distinct GPUs, or it measures nothing
        placement = verify_placement(comm, device, a.gpus)
    except PlacementError as ex:
        print(f"[rank {rank}] error: {ex}; no record", file=sys.stderr, flush=True)
        shutdown()
        return 2
    sync = (lambda: torch.cuda.synchronize(device)) if device.type == "cuda" else (lambda: None)
    if a.parallel == "tp":
        return run_tp(a, comm, device, placement, sync)
    global_batch = a.batch * R if a.scaling == "weak" else a.batch

    x, y = synthetic_mnist(a.train_size, seed=0)  # identical on every rank, no broadcast
    nn = NeuralNetwork([784, a.hidden, 10])
    lr, reg = 1e-3, 1e-4  # reference defaults (fpcode/main.cpp:58-60)

    def prepare(allreduce: str, probe_steps: int = 0):
        """Trainer + captured graphs + W warm-up steps.  Returns (trainer, timed plans, probe plans)."""
        tr = DataParallelTrainer(nn, comm=comm, device=device, dtype=a.dtype, batch_size=global_batch,
                                 backend=a.backend, use_graphs=not a.no_graphs, allreduce=allreduce,
                                 grad_wire=a.grad_wire,
                                 executor="eager" if a.no_graphs else a.executor)
        tr.load(x, y)
        full = [(s, ln) for s, ln in tr.epoch_plan().steps if ln == global_batch]
        if not full:
            raise SystemExit("training split smaller than one global batch")

        def plans_for(k: int):
            out, i = [], 0
            while i < k:
                m = min(len(full), k - i)
                out.append(EpochPlan(full[:m]))
                i += m
            return out

        warm_plans, timed_plans, probe_plans = plans_for(a.warmup), plans_for(a.steps), plans_for(probe_steps)
        native = all(tr.native_plan(p) is not None for p in warm_plans + timed_plans + probe_plans)
        if tr.use_graphs and not native:  # capture outside the timed region (graphs are cached by plan)
            try:
                for p in {tuple(p.steps): p for p in warm_plans + timed_plans + probe_plans}.values():
                    tr.capture(p, lr, reg)
            except Exception as ex:  # pragma: no cover - depends on the collective backend
                print(f"warning: HIP graph capture failed ({ex!r}); running eager steps", file=sys.stderr)
                tr.use_graphs = False
                tr._graphs.clear()
        # every rank done capturing before the first warm-up step: with the xGMI all-reduce a step waits
        # (bounded) for its peers' same step, so a rank still capturing would count against that bound
        sync()
        comm.barrier()
        for p in warm_plans:
            tr.run_plan(p, lr, reg)
        return tr, timed_plans, probe_plans

    def probe(tr, plans) -> float:
        """us/step of the probe plans on this trainer, max over ranks (inf if an xGMI wait timed out or the
        replicas diverged): the same runners and bracketing as the timed region."""
        runners = [tr.plan_runner(p, lr, reg) for p in plans]
        sync()
        comm.barrier()
        sync()
        t = time.perf_counter()
        for run in runners:
            run()
        sync()
        comm.barrier()
        sync()
        us = comm.allreduce_scalar(1e6 * (time.perf_counter() - t) / a.tune_steps, op="max")
        bad = tr.comm_failed()
        bad = bad or not tr.replicas_agree()
        return float("inf") if bad else round(us, 3)

    # --tune-allreduce: with N > 1 and --allreduce auto, the gradient sync is CHOSEN BY MEASUREMENT on this
    # node before anything is timed -- the policy's xGMI pick (cost model, docs/PERFORMANCE.md), the two-shot
    # (N >= 3) and RCCL each run --tune-steps steps, the fastest (max over ranks, agreed by every rank) runs
    # the timed region
    tuning = R > 1 and a.allreduce == "auto" and a.backend == "hip" and a.tune_allreduce == "on"
    tune = {}
    tr, timed_plans, probe_plans = prepare(a.allreduce, a.tune_steps if tuning else 0)
    sync()
    comm.barrier()
    if tr.allreduce_impl.startswith("xgmi") and a.allreduce == "auto":
        # a bounded peer wait that timed out during the warm-up (the xGMI protocol misbehaving on this
        # node) -> every rank drops to RCCL together, from the initial weights, before anything is timed
        forced = os.environ.get("CME_BENCH_TEST_FALLBACK") == "1"  # test hook: take the fallback
        failed = tr.comm_failed()
        diverged = not failed and not tr.replicas_agree()  # a stale peer read would show up here
        if failed or diverged or comm.allreduce_scalar(float(forced), op="max") > 0:
            if rank == 0:
                why = "replicas diverged" if diverged else "peer wait timed out" if failed else "forced"
                print(f"warning: xGMI all-reduce failed in warm-up ({why}); re-running on RCCL", file=sys.stderr)
            tr.close()
            tr, timed_plans, probe_plans = prepare("rccl", a.tune_steps if tuning else 0)
            tune["xgmi"] = "failed in warm-up"
    # candidates besides the policy's pick (already prepared): the xGMI two-shot from 3 ranks on (2 S / R bytes per
    # link against the one-shot's S, one more round trip), RCCL
    others = ((["xgmi2"] if R >= 3 and tr.allreduce_impl != "xgmi-2shot" else [])
              + (["rccl"] if tr.allreduce_impl.startswith("xgmi") else []))
    if tuning and others:
        modes = {tr.allreduce_impl: a.allreduce if tr.allreduce_impl.startswith("xgmi") else "rccl"}
        tune[tr.allreduce_impl] = probe(tr, probe_plans)
        last = tr.allreduce_impl
        for mode in others:
            if tr is not None:
                tr.close()  # (collective) every candidate starts from the initial weights, like every prepare
            try:
                tr, timed_plans, probe_plans = prepare(mode, a.tune_steps)
            except Exception as ex:  # noqa: BLE001 - a candidate the node cannot run (raised on every rank)
                tr, last = None, None
                tune[mode] = "unavailable"
                if rank == 0:
                    print(f"allreduce candidate {mode} unavailable: {ex}", file=sys.stderr, flush=True)
                continue
            modes[tr.allreduce_impl] = mode
            tune[tr.allreduce_impl] = probe(tr, probe_plans)
            last = tr.allreduce_impl
        nums = {k: v for k, v in tune.items() if isinstance(v, float)}
        best = min(nums, key=lambda k: (nums[k], k))  # identical floats on every rank: one decision
        if best != last:
            if tr is not None:
                tr.close()
            tr, timed_plans, _ = prepare(modes[best])  # (a failure from here on invalidates the record below)
        tune = {k: (v if v != float("inf") else "failed") for k, v in tune.items()}
        if rank == 0:
            print(f"allreduce tuned on this node: {tune} -> {tr.allreduce_impl}", file=sys.stderr, flush=True)
    native_exec = all(tr.native_plan(p) is not None for p in timed_plans)
    runners = [tr.plan_runner(p, lr, reg) for p in timed_plans]  # resolved before the clock starts
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for run in runners:
        run()
    sync()
    comm.barrier()
    if R > 1:  # an RCCL barrier is GPU work; one process has nothing left to wait for
        sync()
    dt = time.perf_counter() - t0
    dt = comm.allreduce_scalar(dt, op="max")

    # sanity, agreed by every rank: parameters finite everywhere and no xGMI peer wait timed out anywhere;
    # otherwise the record is marked invalid and every rank exits non-zero
    finite = bool(torch.isfinite(tr.engine.params).all().item())
    bad = comm.allreduce_scalar(0.0 if finite else 1.0, op="max") > 0
    comm_failed = tr.comm_failed()
    kerr = comm.allreduce_scalar(1.0 if tr.engine.kernel_error() else 0.0, op="max") > 0
    agree = tr.replicas_agree()
    ok = not bad and not comm_failed and not kerr and agree
    ar = measure_allreduce(tr, comm, sync) if ok else {}
    # strong scaling drops the remainder columns when R does not divide the batch (trainer.shard)
    images = a.steps * (global_batch // R) * R
    value = images / dt
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": R,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * dt / a.steps, 6),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": {"f32": "fp32", "f64": "fp64", "bf16": "bf16"}[a.dtype],
            "data": "synthetic (MNIST-shaped 784-dim uint8 images, random-init weights)",
            "config": {"model": f"784-{a.hidden}-10 MLP", "global_batch": global_batch, "seq_len": None,
                       "parallelism": f"dp{R}", "per_gpu_batch": global_batch // R, "backend": a.backend,
                       "mode": a.mode,
                       "hip_graphs": tr.use_graphs and not native_exec,
                       "executor": "native" if native_exec else ("graph" if tr.use_graphs else "eager"),
                       "allreduce": tr.allreduce_impl, "params_finite": not bad,
                       "comm_ok": not comm_failed, "replicas_bitwise_equal": agree, **placement, **ar,
                       "allreduce_tuning_us_per_step": tune or None},
        }
        if not ok:
            rec["invalid"] = ("non-finite parameters" if bad else "an xGMI peer wait timed out" if comm_failed
                              else "a forward+head workgroup wait timed out" if kerr
                              else "replicas diverged across ranks")
        print(json.dumps(rec), flush=True)
    shutdown()
    return 0 if ok else 1


def measure_allreduce(tr, comm, sync, iters: int = 20) -> dict:
    """After the timed run: the per-call time of the step's gradient all-reduce on its own (the same
    implementation and bucket bytes, max over ranks), so a scaling curve can be split into compute and
    communication.  The xGMI forms are timed through their one-shot kernel (the fused form runs the same
    protocol inside the wgrad launch); the overlapped RCCL backward through one whole-bucket all-reduce."""
    import torch

    if comm.world_size == 1:
        return {"allreduce_us": None}
    e = tr.engine
    buf = torch.zeros_like(e.grads)
    if tr.xgmi is not None:
        fn, wire = (lambda: tr.xgmi.allreduce_(buf)), tr.xgmi.wire
    elif tr.allreduce_mode == "host":
        import torch.distributed as dist

        def fn():
            g = buf.cpu()
            dist.all_reduce(g, group=tr._host_group)
            buf.copy_(g)
        wire = buf.dtype
    else:
        fn, wire = (lambda: comm.allreduce_(buf)), buf.dtype
    for _ in range(3):
        fn()
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    sync()
    us = comm.allreduce_scalar(1e6 * (time.perf_counter() - t0) / iters, op="max")
    nbytes = buf.numel() * torch.tensor([], dtype=wire).element_size()
    R = comm.world_size
    return {"allreduce_us": round(us, 2), "allreduce_bytes": int(nbytes),
            "allreduce_busbw_GBps": round(2 * (R - 1) / R * nbytes / (us * 1e-6) / 1e9, 2)}


def run_tp(a, comm, device, placement, sync) -> int:
    """Hidden-sharded tensor-parallel step (parallel/tensor_parallel.py): fixed model and global batch
    (strong scaling), K timed steps bracketed by barrier + synchronize, max over ranks."""
    import torch

    from cme213_sp18_amd.models.mlp import NeuralNetwork
    from cme213_sp18_amd.parallel.launcher import shutdown
    from cme213_sp18_amd.parallel.tensor_parallel import TensorParallelTrainer
    from cme213_sp18_amd.parallel.trainer import EpochPlan
    from cme213_sp18_amd.utils.data import synthetic_mnist

    R, rank = comm.world_size, comm.rank
    B = a.batch
    x, y = synthetic_mnist(a.train_size, seed=0)
    nn = NeuralNetwork([784, a.hidden, 10])
    tr = TensorParallelTrainer(nn, comm=comm, device=device, dtype=a.dtype, batch_size=B, backend=a.backend,
                               allreduce="rccl" if a.allreduce in ("rccl", "host") else a.allreduce)
    tr.load(x, y)
    full = [(s, ln) for s, ln in tr.epoch_plan().steps if ln == B]
    lr, reg = 1e-3, 1e-4

    def plans_for(k):
        out, i = [], 0
        while i < k:
            m = min(len(full), k - i)
            out.append(EpochPlan(full[:m]))
            i += m
        return out

    warm, timed = plans_for(a.warmup), plans_for(a.steps)
    graphs = tr.graphs_usable(not a.no_graphs)
    if graphs:  # every distinct plan captured outside the timed region
        for p in {tuple(p.steps): p for p in warm + timed}.values():
            tr.capture(p, lr, reg)
    for p in warm:
        tr.run_plan(p, lr, reg, use_graphs=graphs)
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for p in timed:
        tr.run_plan(p, lr, reg, use_graphs=graphs)
    sync()
    comm.barrier()
    sync()
    dt = comm.allreduce_scalar(time.perf_counter() - t0, op="max")
    ok = comm.allreduce_scalar(0.0 if bool(torch.isfinite(tr.engine.params).all().item()) else 1.0, op="max") == 0
    comm_failed = tr.comm_failed()
    ok = ok and not comm_failed
    ar = {"allreduce_us": None}
    if R > 1 and ok:  # the step's z2 all-reduce on its own (same implementation and bytes), max over ranks
        fn = (lambda: tr._xz.allreduce_(tr.z2)) if tr._xz is not None else (lambda: comm.allreduce_(tr.z2))
        for _ in range(3):
            fn()
        sync()
        comm.barrier()
        sync()
        t1 = time.perf_counter()
        for _ in range(20):
            fn()
        sync()
        us = comm.allreduce_scalar(1e6 * (time.perf_counter() - t1) / 20, op="max")
        ar = {"allreduce_us": round(us, 2), "allreduce_bytes": int(tr.z2.numel() * 4)}
    tr.close()
    value = a.steps * B / dt
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": R, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(1e3 * dt / a.steps, 6), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None,
            "dtype": {"f32": "fp32", "f64": "fp64", "bf16": "bf16"}[a.dtype],
            "data": "synthetic (MNIST-shaped 784-dim uint8 images, random-init weights)",
            "config": {"model": f"784-{a.hidden}-10 MLP", "global_batch": B, "seq_len": None,
                       "parallelism": f"tp{R}", "hidden_per_gpu": a.hidden // R, "backend": a.backend,
                       "hip_graphs": graphs, "allreduce": tr.allreduce_impl, "params_finite": ok,
                       "comm_ok": not comm_failed, **placement, **ar},
        }), flush=True)
    shutdown()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
