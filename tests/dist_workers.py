"""Worker entry points for the multi-process tests (must be importable by spawn)."""
import os

import numpy as np
import torch


def dp_train_worker(rank, world, comm, device, out_dir, H, N, batch, epochs, lr, reg, dtype):
    torch.set_num_threads(2)
    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    x, y = synthetic_mnist(N, seed=11)
    nn = NeuralNetwork([784, H, 10])
    tr = DataParallelTrainer(nn, comm=comm, device=device, dtype=dtype, batch_size=batch, backend="torch",
                             use_graphs=False)
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
