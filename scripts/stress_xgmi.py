"""Stress the xGMI all-reduce with several ranks sharing cuda:0: rounds x buckets x iterations, count wrong results."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def worker(rank, world, comm, device, rounds):
    from cme213_sp18_amd.parallel.xgmi import XgmiBucket

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    bad_total = calls = 0
    for dt, n in ((torch.float64, 1), (torch.float32, 79510), (torch.float64, 3000)):
        xb = XgmiBucket(comm.group, rank, world, n, dt, dev, self_test=False)
        base = torch.arange(n, device=dev, dtype=torch.float64) % 977
        if True:
            for it in range(16 * rounds):
                g = (base * 1e-3 * (rank + 1) + it).to(dt)
                xb.allreduce_(g)
                exp = sum((base * 1e-3 * (r + 1) + it).to(dt).double() for r in range(world))
                bad_total += int((((g.double() - exp).abs() / exp.abs().clamp_min(1)) > 1e-5).sum())
                calls += 1
            bad_total += 1000000 * xb.error()
            xb.close()
    t = torch.tensor([bad_total, calls], dtype=torch.int64)
    import torch.distributed as dist

    dist.all_reduce(t, group=comm.group)
    if rank == 0:
        print(f"variant={os.environ.get('CME_XGMI_VARIANT', '0')} world={world} bad_elements={int(t[0])} calls={int(t[1])}",
              flush=True)


if __name__ == "__main__":
    from cme213_sp18_amd.parallel.launcher import spawn

    spawn(worker, int(sys.argv[1]), (int(sys.argv[2]),), backend="gloo")
