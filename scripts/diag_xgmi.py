"""xGMI all-reduce diagnostics with several ranks sharing cuda:0 (gloo group): per-iteration error
report for a list of (dtype, n), optionally after creating/closing earlier buckets."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def worker(rank, world, comm, device, cases):
    from cme213_sp18_amd.parallel.xgmi import XgmiBucket

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    for dtn, n in cases:
        dt = getattr(torch, dtn)
        xb = XgmiBucket(comm.group, rank, world, n, dt, dev, self_test=False)
        # self-test style first calls, reported per rank
        base0 = torch.arange(n, dtype=torch.float64, device=dev) % 1000
        for k in range(3):
            t = ((rank + 1) * 0.25 + base0 / 1024).to(dt)
            xb.allreduce_(t)
            torch.cuda.synchronize()
            exp0 = sum(((r + 1) * 0.25 + base0 / 1024).to(dt).double() for r in range(world))
            bad0 = ((t.double() - exp0).abs() > 1e-9 * exp0.abs())
            if bad0.any():
                idx = bad0.nonzero().flatten()
                print(f"rank{rank} {dtn} n={n} first-call {k}: bad={int(bad0.sum())} err={xb.error()} "
                      f"chunks={sorted(set((idx // 1024).tolist()))[:12]} got={t[idx[0]].item()} exp={exp0[idx[0]].item()}",
                      flush=True)
        base = torch.arange(n, device=dev, dtype=torch.float64) % 977
        for it in range(8):
            g = (base * 1e-3 * (rank + 1) + it).to(dt)
            xb.allreduce_(g)
            exp = sum((base * 1e-3 * (r + 1) + it).to(dt).double() for r in range(world))
            bad = ((g.double() - exp).abs() / exp.abs().clamp_min(1)) > 1e-5
            nb = int(bad.sum())
            if nb and rank == 0:
                idx = bad.nonzero().flatten()
                print(f"{dtn} n={n} it={it} bad={nb} first={idx[:4].tolist()} last={idx[-1].item()} "
                      f"chunks={sorted(set((idx // 1024).tolist()))[:10]} got={g[idx[0]].item()} exp={exp[idx[0]].item()}",
                      flush=True)
        if rank == 0:
            print(f"{dtn} n={n} done ok={xb.ok}", flush=True)
        xb.close()


if __name__ == "__main__":
    from cme213_sp18_amd.parallel.launcher import spawn

    world = int(sys.argv[1])
    cases = [tuple(c.split(":")) for c in sys.argv[2:]]
    cases = [(a, int(b)) for a, b in cases]
    spawn(worker, world, (cases,), backend="gloo")
