"""Lookahead SGD step schedule for one process: two launches per step instead of three.

Plain SGD on the MLP is a chain  fwd1(t) -> head(t) -> wgrad(t) -> fwd1(t+1) -> ...  where every
launch waits for the previous one.  Writing the update out,

    W1' = (1 - lr*reg) W1 - lr*xs * dZ1 X^T          (xs = input scale, 1 or 1/255)
    z1' - b1' = xs W1' X'
              = xs(1 - lr*reg) * (W1 X')  -  lr*xs^2 * dZ1 (X^T X')

the next pre-activation needs W1 only through ``A' = W1 X'`` -- computable while the CURRENT head runs
-- and the rest through the Gram matrix ``G = X^T X'`` of two consecutive batches, which depends on
the data only (precomputed once per epoch plan; exact integers, held in fp32).  So one epoch step is

    L2(t): head(t)                                     ||  A(t+1) = W1(t) X(t+1)      (raw GEMM)
    L1(t): z(t+1) = c1 A(t+1) - c2 dZ1(t) G(t)^T       ||  dW1/db1/dW2/db2 + SGD of step t

with the critical path head -> combine and the weight update off it (same launch, other workgroups).
The head finishes the activation a1 = sigmoid(z + b1) itself (b1 is updated by L1).  Every SGD
update is exactly the reference's; only the evaluation order of z1 changes (fp32-class rounding).
Data parallelism keeps the plain schedule: there the next forward needs the all-reduced gradient.

Measured (MI355X, 784-100-10, batch 800): L2 9.5 us + L1 11.0 us = 21.0 us/step against 18.3 us for
the plain fwd1 / head / wgrad launches: co-scheduled roles share each CU's L2 bandwidth, and each
kernel of the plain step already uses ~175 of the 256 CUs.  Opt-in (DataParallelTrainer(lookahead=True)).
Reference loop: fpcode/neural_network.cpp:449-555 (parallel_train, one rank).
"""
from __future__ import annotations

import torch


class LookaheadRunner:
    def __init__(self, engine):
        e = engine
        if not (e.backend == "hip" and e.np and e.H <= 128 and e.XT is not None and e.XT.shape[0] == e.P + 1):
            raise ValueError("lookahead needs the hip split path, H <= 128 and the all-ones XT feature")
        self.e = e
        dev = e.device
        self.z = [torch.zeros(e.H, e.ld, dtype=torch.float32, device=dev) for _ in range(2)]
        self.A = torch.zeros(e.H, e.ld, dtype=torch.float32, device=dev)
        self._gram: dict = {}

    @staticmethod
    def plan_ok(steps) -> bool:
        """Every batch non-empty with n % 4 == 0 (16-byte fp32 rows for the Gram operand)."""
        return len(steps) > 0 and all(n > 0 and n % 4 == 0 for _, n in steps)

    @staticmethod
    def supported(engine) -> bool:
        e = engine
        return (e.backend == "hip" and bool(e.np) and e.H <= 128 and e.device.type == "cuda"
                and e.XT is not None and e.XT.shape[0] == e.P + 1)

    def gram(self, steps) -> list:
        """GT[t][j][k] = x_{t+1, j} . x_{t, k} (exact integer dot products, stored fp32), cached per plan."""
        key = tuple(steps)
        g = self._gram.get(key)
        if g is None:
            X = self.e.X
            g = []
            for (o0, n0), (o1, n1) in zip(steps[:-1], steps[1:]):
                ld = (n0 + 3) // 4 * 4  # 16-byte rows for the fp32 MFMA operand
                gt = torch.zeros(n1, ld, dtype=torch.float32, device=X.device)
                gt[:, :n0] = (X[o1:o1 + n1].double() @ X[o0:o0 + n0].double().t()).float()
                g.append(gt)
            if len(self._gram) >= 4:  # a few plans at a time (an epoch plan is reused every epoch)
                self._gram.pop(next(iter(self._gram)))
            self._gram[key] = g
        return g

    def run(self, steps, lr: float, reg: float) -> None:
        """Enqueue every step of ``steps`` [(offset, n)] on the current stream (graph-capturable)."""
        e = self.e
        st = e._hip_step()
        stream = torch.cuda.current_stream(e.device).cuda_stream
        G = self.gram(steps)
        xs = float(e.xscale)
        c1, c2 = xs * (1.0 - lr * reg), lr * xs * xs
        o0, n0 = steps[0]
        st.la_prologue(int(o0), int(n0), self.z[0].data_ptr(), stream)
        for t, (off, n) in enumerate(steps):
            zc, zn = self.z[t % 2], self.z[(t + 1) % 2]
            nxt = steps[t + 1] if t + 1 < len(steps) else None
            on, nn = (nxt if nxt is not None else (0, 0))
            st.la_l2(int(off), int(n), 1.0 / n, 0, zc.data_ptr(), int(on), int(nn), self.A.data_ptr(), stream)
            if nxt is not None:
                gt = G[t]
                st.la_l1(int(off), int(n), 1.0 / n, float(reg), float(lr), zc.data_ptr(), int(nn), gt.data_ptr(),
                         int(gt.shape[1]), self.A.data_ptr(), zn.data_ptr(), c1, c2, stream)
            else:
                st.la_l1(int(off), int(n), 1.0 / n, float(reg), float(lr), zc.data_ptr(), 0, 0, 0, 0, 0, 0.0, 0.0,
                         stream)
