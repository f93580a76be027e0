"""Stress of the wgrad launch with the xGMI all-reduce fused in: ranks sharing cuda:0 (gloo group)
run STEPS data-parallel steps through the fused kernel and, from the same state, through the separate
all-reduce kernel; the parameters must be bitwise identical on every rank (no stale peer reads).
Usage: stress_fused.py [world=2] [steps=200]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def worker(rank, world, comm, device, steps):
    import torch.distributed as dist

    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x, y = synthetic_mnist(8000, seed=11)
    nn = NeuralNetwork([784, 100, 10])
    tr = DataParallelTrainer(nn, comm=comm, device=dev, batch_size=800, use_graphs=False, allreduce="xgmi")
    tr.load(x, y)
    on = tr.fused_allreduce
    bad = 0
    if on:
        e = tr.engine
        snap = tr._snapshot()
        plan = tr.epoch_plan().steps
        out = []
        for fused in (True, False):
            tr._restore(snap)
            tr.fused_allreduce = fused
            for k in range(steps):
                s, ln = plan[k % len(plan)]
                tr.step(s, ln, 0.05, 1e-4)
            torch.cuda.synchronize()
            out.append((e.params.clone(), e.W1p.clone()))
        tr.fused_allreduce = True
        bad = int((out[0][0] != out[1][0]).sum())
        if e.w1_planes_maintained():  # (below H = 512 no forward kernel reads the W1 planes: not refreshed)
            bad += int((out[0][1] != out[1][1]).sum())
        bad += 1000000 * int(tr._xgmi_fused.error() != 0)
    t = torch.tensor([bad, int(on)], dtype=torch.int64)
    dist.all_reduce(t, group=comm.group)
    if rank == 0:
        print(f"world={world} steps={steps} fused_ranks={int(t[1])} bad_elements={int(t[0])}", flush=True)
    tr.close()


if __name__ == "__main__":
    from cme213_sp18_amd.parallel.launcher import spawn

    w = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    spawn(worker, w, (int(sys.argv[2]) if len(sys.argv) > 2 else 200,), backend="gloo")
