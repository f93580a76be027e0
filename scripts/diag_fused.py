"""Fused wgrad + xGMI all-reduce diagnostics: 2 ranks sharing cuda:0 (gloo group) -- residency check,
bucket setup, and the separate-vs-fused parameter diff of one step, per rank."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def worker(rank, world, comm, device, _):
    from cme213_sp18_amd import NeuralNetwork
    from cme213_sp18_amd.parallel import DataParallelTrainer
    from cme213_sp18_amd.utils.data import synthetic_mnist

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x, y = synthetic_mnist(3200, seed=3)
    nn = NeuralNetwork([784, 100, 10])
    tr = DataParallelTrainer(nn, comm=comm, device=dev, batch_size=800, use_graphs=False, allreduce="xgmi")
    e = tr.engine
    print(f"rank{rank} slots={e.fused_allreduce_slots()} fused_bucket={tr._xgmi_fused is not None}", flush=True)
    tr.load(x, y)
    print(f"rank{rank} fused_on={tr.fused_allreduce}", flush=True)
    if tr._xgmi_fused is None:
        # rebuild the comparison by hand to see the diff
        from cme213_sp18_amd.parallel.xgmi import XgmiBucket

        xb = XgmiBucket(comm.group, rank, world, e.params.numel(), torch.float32, dev,
                        flag_slots=e.fused_allreduce_slots())
        snap = tr._snapshot()
        off, n = tr.shard(0, 800)
        scale, reg, lr = 1.0 / (n * world), 1e-3 / world, 0.05
        e.run(off, n, scale, reg, lr, sgd=False)
        tr._allreduce_sgd(lr)
        torch.cuda.synchronize()
        ref = e.params.clone(), e.W1p.clone()
        e.attach_xgmi(xb)
        for k in range(3):
            tr._restore(snap)
            e.run(off, n, scale, reg, lr, sgd=2)
            torch.cuda.synchronize()
            d = (e.params - ref[0]).abs()
            o = e.layout.offsets
            parts = {nm: float(d[o[i]:o[i] + e.layout.sizes[i]].max()) for i, nm in enumerate(("W1", "b1", "W2", "b2"))}
            print(f"rank{rank} try{k} err={xb.error()} diffs={parts} planes_eq={torch.equal(e.W1p, ref[1])}",
                  flush=True)
        e.attach_xgmi(None)
        xb.close()
    tr.close()


if __name__ == "__main__":
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(worker, int(sys.argv[1]) if len(sys.argv) > 1 else 2, (None,), backend="gloo")
