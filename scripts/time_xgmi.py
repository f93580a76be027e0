"""Time the xGMI fused all-reduce+SGD kernel (ranks sharing cuda:0): per-call us from a graph of K calls,
next to a plain device-local copy kernel of the same size for reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def worker(rank, world, comm, device, n, reps):
    import torch.distributed as dist

    from cme213_sp18_amd.parallel.xgmi import XgmiBucket

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    xb = XgmiBucket(comm.group, rank, world, n, torch.float32, dev)
    g = torch.randn(n, device=dev) * 1e-3
    p = torch.randn(n, device=dev)
    planes = torch.zeros(3, 78400, dtype=torch.bfloat16, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            xb.sgd_(g, p, 1e-3, planes, 3, 78400)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(reps):
            xb.sgd_(g, p, 1e-3, planes, 3, 78400)
    dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    t = torch.tensor([us])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(f"world={world} n={n} xgmi allreduce+sgd: {float(t):.2f} us/call (max over ranks, ranks share one GPU)",
              flush=True)
    xb.check()
    xb.close()


if __name__ == "__main__":
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(worker, int(sys.argv[1]), (int(sys.argv[2]), int(sys.argv[3])), backend="gloo")
