"""Worker entry points for the multi-process tests (must be importable by spawn)."""
import hashlib
import os

import numpy as np
import torch


def dp_train_worker(rank, world, comm, device, out_dir, H, N, batch, epochs, lr, reg, dtype, allreduce="auto"):
    torch.set_num_threads(2)
    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(N, seed=11)
    nn = NeuralNetwork([784, H, 10])
    tr = DataParallelTrainer(nn, comm=comm, device=device, dtype=dtype, batch_size=batch, backend="torch",
                             use_graphs=False, allreduce=allreduce)
    tr.load(x, y)
    st = tr.train(epochs, lr, reg, print_every=2, log=lambda *_: None)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), W0=nn.W[0], W1=nn.W[1], b0=nn.b[0], b1=nn.b[1],
             losses=np.array(st.losses), images=st.images)


def allreduce_worker(rank, world, comm, device, out_dir):
    t = torch.full((5,), float(rank + 1), dtype=torch.float64)
    comm.allreduce_(t)
    mx = comm.allreduce_scalar(rank * 10.0, op="max")
    b = torch.full((3,), float(rank), dtype=torch.float64)
    comm.broadcast_(b, src=1)
    comm.barrier()
    np.save(os.path.join(out_dir, f"ar{rank}.npy"), np.concatenate([t.numpy(), [mx], b.numpy()]))


def nccl_graph_worker(out_dir):
    """world_size=1 process group on the GPU: exercises the DP step (grads ->
    RCCL all-reduce -> flat SGD) captured in a HIP graph."""
    import datetime

    import torch.distributed as dist

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer, TorchDistComm
    from cme213_sp18_amd.utils.data import synthetic_mnist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, timeout=datetime.timedelta(seconds=120),
                            device_id=torch.device("cuda", 0))
    try:
        x, y = synthetic_mnist(4000, seed=4)
        nn = NeuralNetwork([784, 100, 10])
        ref = nn.copy()
        tr = DataParallelTrainer(nn, comm=TorchDistComm(), use_graphs=True)
        assert tr.use_graphs
        tr.load(x, y)
        tr.train(2, 0.01, 1e-4)
        t2 = DataParallelTrainer(ref, use_graphs=True)  # NullComm: fused SGD
        t2.load(x, y)
        t2.train(2, 0.01, 1e-4)
        # the overlapped RCCL backward (dW1 row chunks all-reduced on a side stream while the next chunk
        # is computed), forced at world 1 and captured in the HIP graph, against the fused single-process step
        outs = {}
        for H in (1024, 4096):
            nb = NeuralNetwork([784, H, 10])
            rb = nb.copy()
            tb = DataParallelTrainer(nb, comm=TorchDistComm(), use_graphs=True, overlap_chunks=4)
            assert tb._bucketed and tb.use_graphs and len(tb._buckets()) == 4
            tb.load(x, y)
            tb.train(1, 0.01, 1e-4)
            tr1 = DataParallelTrainer(rb, use_graphs=True)
            tr1.load(x, y)
            tr1.train(1, 0.01, 1e-4)
            a = np.concatenate([nb.W[0].ravel(), nb.W[1].ravel(), nb.b[0].ravel(), nb.b[1].ravel()])
            b = np.concatenate([rb.W[0].ravel(), rb.W[1].ravel(), rb.b[0].ravel(), rb.b[1].ravel()])
            outs[f"bucketed_rel_{H}"] = np.abs(a - b).max() / np.abs(b).max()
        np.savez(os.path.join(out_dir, "nccl.npz"), a=nn.W[0], b=ref.W[0], a1=nn.b[0], b1=ref.b[0], **outs)
    finally:
        dist.destroy_process_group()


def xgmi_worker(rank, world, comm, device, out_dir):
    """Several processes on ONE GPU: the xGMI peer all-reduce through IPC handles
    exchanged over gloo (same code path as 8 GPUs, minus the links)."""
    from cme213_sp18_amd.parallel.xgmi import XgmiBucket

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    res = {}
    # plain all-reduce: sizes around the vector / chunk / grid-stride edges, both halves, fp32 + fp64
    # (few buckets per process: every bucket is a fresh IPC export/import, and the runtime runs out
    # of them after a few dozen re-creations with several ranks on one GPU -- a training job has one)
    for dt, sizes in ((torch.float32, (3, 600 * 1024 + 3)), (torch.float64, (79_510,))):
        for n in sizes:
            xb = XgmiBucket(comm.group, rank, world, n, dt, dev)
            worst = 0.0
            base = torch.arange(n, device=dev, dtype=torch.float64) % 977
            for it in range(5):
                g = (base * 1e-3 * (rank + 1) + it).to(dt)
                xb.allreduce_(g)
                exp = sum((base * 1e-3 * (r + 1) + it).to(dt).double() for r in range(world))
                worst = max(worst, float(((g.double() - exp).abs() / exp.abs().clamp_min(1)).max()))
            torch.cuda.synchronize()
            res[f"ar_{dt}_{n}"] = worst
            res[f"ok_{dt}_{n}"] = float(xb.ok and xb.error() == 0)
            xb.close()
    # fused SGD with exact bf16 planes, replayed from a HIP graph
    n, w1n = 5000, 3136
    gen = torch.Generator(device="cpu").manual_seed(7)
    p0 = torch.randn(n, generator=gen).to(dev)
    grads = (torch.randn(n, generator=gen) * (rank + 1)).to(dev)
    params = p0.clone()
    planes = torch.zeros(3, w1n, dtype=torch.bfloat16, device=dev)
    xb = XgmiBucket(comm.group, rank, world, n, torch.float32, dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        xb.sgd_(grads, params, 0.01, planes, 3, w1n)  # eager step 1
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        xb.sgd_(grads, params, 0.01, planes, 3, w1n)
    for _ in range(4):
        graph.replay()
    torch.cuda.synchronize()
    # every rank's grads: regenerate them to build the expected update
    gsum = torch.zeros(n, dtype=torch.float64)
    for r in range(world):
        gg = torch.Generator(device="cpu").manual_seed(7)
        torch.randn(n, generator=gg)
        gsum += (torch.randn(n, generator=gg) * (r + 1)).double()
    exp = p0.double().cpu() - 5 * 0.01 * gsum
    res["sgd_err"] = float((params.double().cpu() - exp).abs().max())
    res["planes_exact"] = float(torch.equal(planes.float().sum(0), params[:w1n]))
    res["sgd_ok"] = float(xb.error() == 0)
    xb.close()
    # the trainer: xgmi fused path vs the gloo all-reduce path, same data and seeds
    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(3200, seed=3)
    out = {}
    for mode in ("xgmi", "off"):
        nn = NeuralNetwork([784, 100, 10])
        tr = DataParallelTrainer(nn, comm=comm, device=dev, batch_size=800, use_graphs=False, allreduce=mode)
        assert (tr.xgmi is not None) == (mode == "xgmi")
        tr.load(x, y)
        if mode == "xgmi":
            # all-reduce fused into the wgrad launch: on whenever every rank's tiles fit on the GPU
            # (2 ranks sharing one GPU do; 4 do not and must fall back to the separate kernel)
            res["fused_on"] = float(tr.fused_allreduce)
            if world == 2:
                res["ok_fused_enabled"] = float(tr.fused_allreduce)
        tr.train(2, 0.05, 1e-4)
        out[mode] = nn.W[0].copy(), nn.W[1].copy()
        if mode == "xgmi" and tr.fused_allreduce:  # HIP-graph replay of the fused step == eager steps
            e = tr.engine
            snap = tr._snapshot()
            for _ in range(3):
                tr.step(800, 800, 0.05, 1e-4)
            torch.cuda.synchronize()
            eager = (e.params.clone(), e.W1p.clone())
            tr._restore(snap)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                tr.step(800, 800, 0.05, 1e-4)
            for _ in range(3):
                graph.replay()
            torch.cuda.synchronize()
            res["ok_fused_graph"] = float(torch.equal(e.params, eager[0]) and torch.equal(e.W1p, eager[1]))
            res["ok_fused_err"] = float(tr._xgmi_fused.error() == 0)
        tr.close()
    res["trainer_w1_diff"] = float(np.abs(out["xgmi"][0] - out["off"][0]).max())
    res["trainer_w2_diff"] = float(np.abs(out["xgmi"][1] - out["off"][1]).max())
    # overlapped bucketed backward (dW1 row chunks all-reduced on a side stream) vs one bucket
    import cme213_sp18_amd.parallel.trainer as trmod

    trmod.BUCKET_BYTES = 256 << 10  # force several chunks (incl. a partial one)
    for H in (300, 1024):
        outs = {}
        for overlap in (True, False):
            nn = NeuralNetwork([784, H, 10])
            tr = DataParallelTrainer(nn, comm=comm, device=dev, batch_size=800, use_graphs=False, allreduce="rccl",
                                     overlap=overlap)
            assert tr._bucketed == overlap and len(tr._buckets()) > 1
            tr.load(x, y)
            tr.train(2, 0.05, 1e-4)
            outs[overlap] = np.concatenate([nn.W[0].ravel(), nn.W[1].ravel(), nn.b[0].ravel(), nn.b[1].ravel()])
        res[f"bucketed_diff_{H}"] = float(np.abs(outs[True] - outs[False]).max())
    np.savez(os.path.join(out_dir, f"xgmi{rank}.npz"), **{k: np.array(v) for k, v in res.items()})


def xgmi_spawn_main(out_dir, world):
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(xgmi_worker, world, (out_dir,), backend="gloo")


def tp_train_worker(rank, world, comm, device, out_dir, H, N, B, E, lr, reg, dtype):
    """Hidden-sharded (tensor parallel) training over gloo; saves the gathered full params + losses."""
    import numpy as np

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import TensorParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(N, seed=11)
    nn = NeuralNetwork([784, H, 10])
    tr = TensorParallelTrainer(nn, comm=comm, device="cpu", dtype=dtype, batch_size=B, backend="torch")
    tr.load(x, y)
    st = tr.train(E, lr, reg, print_every=2, log=lambda *_: None)
    np.savez(os.path.join(out_dir, f"tp{rank}.npz"), W0=nn.W[0], W1=nn.W[1], b0=nn.b[0], b1=nn.b[1],
             losses=np.array(st.losses), pred=tr.predict(x[:200]))


def xgmi_stall_worker(rank, world, comm, device, out_dir):
    """A stalled peer (rank 1 skips a step) must make rank 0's xGMI all-reduce time out WITHOUT touching
    params or bf16 planes, keep every later step a no-op on that rank, and surface as an error on EVERY
    rank through the collective check (csrc/comm/xgmi_allreduce.hip, mlp_split.hip xf_exchange)."""
    import time

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.parallel.trainer import CommFailure
    from cme213_sp18_amd.parallel.xgmi import XgmiBucket
    from cme213_sp18_amd.utils.data import synthetic_mnist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    res = {}
    # ---- A: the separate all-reduce + SGD kernel
    n, w1n = 5000, 3136
    xb = XgmiBucket(comm.group, rank, world, n, torch.float32, dev)
    params = torch.randn(n, generator=torch.Generator().manual_seed(1)).to(dev)
    planes = torch.zeros(3, w1n, dtype=torch.bfloat16, device=dev)
    grads = torch.full((n,), float(rank + 1), device=dev)
    xb.sgd_(grads, params, 0.01, planes, 3, w1n)  # one good step on both ranks
    torch.cuda.synchronize()
    res["A_first_ok"] = float(xb.error() == 0)
    comm.barrier()
    if rank == 0:  # rank 1 stalls: it never joins this step
        before = (params.clone(), planes.clone())
        t0 = time.perf_counter()
        xb.sgd_(grads, params, 0.01, planes, 3, w1n)
        torch.cuda.synchronize()
        res["A_timeout_s"] = time.perf_counter() - t0
        res["A_err"] = float(xb.error())
        res["A_untouched"] = float(torch.equal(params, before[0]) and torch.equal(planes, before[1]))
        t0 = time.perf_counter()  # a rank in error applies nothing more and does not wait again
        xb.sgd_(grads, params, 0.01, planes, 3, w1n)
        torch.cuda.synchronize()
        res["A_after_s"] = time.perf_counter() - t0
        res["A_after_untouched"] = float(torch.equal(params, before[0]))
    flag = comm.allreduce_scalar(float(xb.error()), op="max")
    res["A_collective_err"] = float(flag > 0)
    xb.close()
    # ---- B: the all-reduce fused into the weight-gradient launch, through the trainer
    x, y = synthetic_mnist(3200, seed=3)
    nn = NeuralNetwork([784, 100, 10])
    tr = DataParallelTrainer(nn, comm=comm, device=dev, batch_size=800, use_graphs=False, allreduce="xgmi")
    tr.recover = False  # (this part pins the raise; the in-process fallback: test_gpu_handoff.py)
    tr.load(x, y)
    res["B_fused"] = float(tr.fused_allreduce)
    e = tr.engine
    tr.step(0, 800, 0.05, 1e-4)
    torch.cuda.synchronize()
    comm.barrier()
    if rank == 0:
        before = (e.params.clone(), e.W1p.clone())
        tr.step(800, 800, 0.05, 1e-4)  # rank 1 stalls
        torch.cuda.synchronize()
        res["B_untouched"] = float(torch.equal(e.params, before[0]) and torch.equal(e.W1p, before[1]))
    res["B_comm_failed"] = float(tr.comm_failed())
    # a whole epoch after the failure: rank 0 (in error) publishes nothing, so rank 1 times out once and
    # applies nothing either; the epoch-end check raises on BOTH ranks
    before = e.params.clone()
    try:
        tr.train(1, 0.05, 1e-4)
        res["B_raised"] = 0.0
    except CommFailure:
        res["B_raised"] = 1.0
    torch.cuda.synchronize()
    res["B_epoch_untouched"] = float(torch.equal(e.params, before))
    tr.close()
    np.savez(os.path.join(out_dir, f"stall{rank}.npz"), **{k: np.array(v) for k, v in res.items()})


def xgmi_stall_main(out_dir):
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(xgmi_stall_worker, 2, (out_dir,), backend="gloo")


# ------------------------------------------------------------------ one rank per GPU (needs >= N GPUs)
DP_MODES = (  # (name, H, trainer kwargs)
    ("xgmi-fused", 100, dict(allreduce="xgmi", fused_form="pull")),
    # the owner-tile push form of the fused all-reduce (XgmiFuse::push): bitwise the one-shot's result
    ("xgmi-push", 100, dict(allreduce="xgmi", fused_form="push")),
    # H = 32 (52 weight-gradient tiles per rank): small enough for 4 ranks' fused launches on one GPU at once
    ("xgmi-fused-h32", 32, dict(allreduce="xgmi", fused_form="pull")),
    ("xgmi-push-h32", 32, dict(allreduce="xgmi", fused_form="push")),
    ("xgmi", 100, dict(allreduce="xgmi", fuse_allreduce=False)),
    ("rccl", 100, dict(allreduce="rccl")),
    ("rccl-bucketed", 4096, dict(allreduce="rccl", overlap_chunks=4)),
    # BASELINE config 5's shape: the bf16 path's 3.3 MB fp32 gradient over a bf16 xGMI wire (1.6 MB)
    ("xgmi-bf16wire", 1024, dict(allreduce="xgmi", dtype="bf16", grad_wire="bf16")),
    # ... and exactly, through the two-shot kernel (reduce-scatter + sharded SGD + all-gather)
    ("xgmi-2shot", 1024, dict(allreduce="xgmi2", dtype="bf16")),
    ("xgmi-2shot-f32", 300, dict(allreduce="xgmi2")),
    ("host", 100, dict(allreduce="host")),
)


def multigpu_dp_worker(rank, world, comm, device, out_dir, modes, scalings, steps):
    """Every DP all-reduce path on `world` ranks, one per GPU (or sharing GPU 0 under CME_SHARED_GPU=1),
    against a single-process run of the same global batch on this rank's GPU: all replicas must be
    BITWISE identical, and the data-parallel result within fp32 reassociation of the single-process one.
    weak: global batch 800*R (800 per rank); strong: 800 split over the ranks (800/R each,
    fpcode/neural_network.cpp:458)."""
    import json

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    import torch.distributed as dist

    res = {}
    for name, H, kw in DP_MODES:
        if name not in modes:
            continue
        for scaling in scalings:
            B = 800 * world if scaling == "weak" else 800
            x, y = synthetic_mnist(B * steps, seed=5)
            nn = NeuralNetwork([784, H, 10])
            ref = nn.copy()
            tr = DataParallelTrainer(nn, comm=comm, device=device, batch_size=B, use_graphs=True, **kw)
            tr.load(x, y)
            impl = tr.allreduce_impl
            p0 = tr.engine.params.detach().double().cpu()
            tr.train(1, 0.05, 1e-4)
            got = tr.engine.params.detach().double().cpu()
            tr.close()
            single = DataParallelTrainer(ref, device=device, batch_size=B, use_graphs=True,  # one process
                                         dtype=kw.get("dtype", "f32"))
            single.load(x, y)
            single.train(1, 0.05, 1e-4)
            want = single.engine.params.detach().double().cpu()
            digests = [None] * world
            dist.all_gather_object(digests, hashlib.sha1(got.numpy().tobytes()).hexdigest(), group=comm.group)
            key = f"{name}/{scaling}"
            res[key] = {"impl": impl, "replicas_equal": len(set(digests)) == 1, "digest": digests[0],
                        "rel_vs_single": float((got - want).abs().max() / want.abs().max()),
                        "moved": float((got - p0).abs().max())}
    if rank == 0:
        with open(os.path.join(out_dir, "multigpu.json"), "w") as f:
            json.dump(res, f)


def multigpu_dp_main(out_dir, world, modes, scalings, steps, backend):
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(multigpu_dp_worker, world, (out_dir, modes, scalings, steps), backend=backend)


def handoff_timeout_dp_worker(rank, world, comm, device, out_dir, allreduce):
    """A REAL timed-out all-gather forward + head launch on rank 0 only (MlpEngine.inject_handoff_timeout)
    in data-parallel training, 2 ranks sharing GPU 0: no rank applies that step or any later one (rank 0's
    weight-gradient launch reads the sticky error word; it marks the gradient bucket's status element, which
    the all-reduce carries to every rank's SGD, or -- xGMI fused -- stops taking part so rank 1's waits time
    out), and train() raises KernelHandoffTimeout on BOTH ranks."""
    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.parallel.trainer import KernelHandoffTimeout
    from cme213_sp18_amd.utils.data import synthetic_mnist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x, y = synthetic_mnist(3200, seed=3)
    tr = DataParallelTrainer(NeuralNetwork([784, 100, 10]), comm=comm, device=dev, batch_size=1600,
                             allreduce=allreduce)
    tr.engine.set_fh_allgather(True)  # (off by default when ranks share a GPU; both launches fit here)
    tr.recover = False  # (the in-process fallback: handoff_recover_dp_worker)
    tr.load(x, y)
    res = {"impl": tr.allreduce_impl}
    tr.train(1, 0.05, 1e-4)  # a clean epoch on both ranks
    torch.cuda.synchronize()
    res["clean_err"] = float(tr.engine.kernel_error())
    comm.barrier()
    if rank == 0:
        tr.engine.inject_handoff_timeout(0, 2000)
    before = (tr.engine.params.clone(), tr.engine.W1p.clone())
    try:
        tr.train(1, 0.05, 1e-4)
        res["raised"] = 0.0
    except KernelHandoffTimeout:
        res["raised"] = 1.0
    torch.cuda.synchronize()
    res["local_err"] = float(tr.engine.kernel_error())
    res["untouched"] = float(torch.equal(tr.engine.params, before[0]) and torch.equal(tr.engine.W1p, before[1]))
    tr.close()
    np.savez(os.path.join(out_dir, f"handoff_{allreduce}_{rank}.npz"),
             **{k: np.array(v) for k, v in res.items()})


def handoff_timeout_dp_main(out_dir, allreduce):
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(handoff_timeout_dp_worker, 2, (out_dir, allreduce), backend="gloo")


def tp_xgmi_worker(rank, world, comm, device, out_dir, H):
    """Hidden-sharded training with the z2 all-reduce on the xGMI one-shot kernel (ranks sharing GPU 0),
    against single-process data-parallel training of the full model (rank 0 computes it)."""
    import json

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer, TensorParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N, B, E, lr, reg = 2000, 800, 2, 0.05, 1e-4
    x, y = synthetic_mnist(N, seed=4)
    nn = NeuralNetwork([784, H, 10])
    ref = nn.copy()
    tr = TensorParallelTrainer(nn, comm=comm, device=dev, dtype="f32", batch_size=B, allreduce="xgmi")
    tr.load(x, y)
    impl = tr.allreduce_impl
    tr.train(E, lr, reg)
    failed = tr.comm_failed()
    tr.close()
    if rank == 0:
        single = DataParallelTrainer(ref, device=dev, dtype="f32", batch_size=B)
        single.load(x, y)
        single.train(E, lr, reg)
        rel = max(float(np.abs(nn.W[i] - ref.W[i]).max() / np.abs(ref.W[i]).max()) for i in range(2))
        with open(os.path.join(out_dir, "tp_xgmi.json"), "w") as f:
            json.dump({"impl": impl, "rel": rel, "failed": bool(failed),
                       "b_err": max(float(np.abs(nn.b[i] - ref.b[i]).max()) for i in range(2))}, f)


def tp_xgmi_main(out_dir, world, H):
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(tp_xgmi_worker, world, (out_dir, H), backend="gloo")


def handoff_recover_dp_worker(rank, world, comm, device, out_dir, allreduce):
    """train()'s in-process recovery, 2 ranks sharing GPU 0: rank 0's all-gather hand-off really times out in the
    first epoch; both ranks restore the epoch-start snapshot and re-run it on the last-arriver head and the
    communicator's all-reduce.  Compared bitwise with a run that used that path from the start."""
    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x, y = synthetic_mnist(3200, seed=3)
    nn = NeuralNetwork([784, 100, 10])
    init = [p.copy() for p in nn.params]
    tr = DataParallelTrainer(nn, comm=comm, device=dev, batch_size=1600, allreduce=allreduce)
    tr.engine.set_fh_allgather(True)  # (off by default when ranks share a GPU; both launches fit here)
    tr.load(x, y)
    res = {"impl0": tr.allreduce_impl}
    if rank == 0:
        tr.engine.inject_handoff_timeout(0, 2000)
    tr.train(2, 0.05, 1e-4)
    torch.cuda.synchronize()
    res["recovered"] = float(tr.recovered is not None)
    res["impl1"] = tr.allreduce_impl
    res["agree"] = float(tr.replicas_agree())
    got = tr.engine.params.clone()
    tr.close()
    nn2 = NeuralNetwork([784, 100, 10])
    for dst, src in zip(nn2.params, init):
        dst[...] = src
    ref = DataParallelTrainer(nn2, comm=comm, device=dev, batch_size=1600, allreduce="rccl")
    ref.engine.set_fh_allgather(False)
    ref.load(x, y)
    ref.train(2, 0.05, 1e-4)
    torch.cuda.synchronize()
    res["equal_ref"] = float(torch.equal(got, ref.engine.params))
    ref.close()
    np.savez(os.path.join(out_dir, f"recover_{allreduce}_{rank}.npz"), **{k: np.array(v) for k, v in res.items()})


def handoff_recover_dp_main(out_dir, allreduce):
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(handoff_recover_dp_worker, 2, (out_dir, allreduce), backend="gloo")
