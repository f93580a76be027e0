"""Worker entry points for the multi-process tests (must be importable by spawn)."""
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
        np.savez(os.path.join(out_dir, "nccl.npz"), a=nn.W[0], b=ref.W[0], a1=nn.b[0], b1=ref.b[0])
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
