"""Tensor parallelism over the hidden dimension (an extension; SURVEY §2.6 "optional stretch").

The reference only has data parallelism (fpcode/neural_network.cpp:401-575): every rank holds the whole
model and the per-batch gradient (784H + 11H + 10 values) is all-reduced.  For the WIDE configs
(784-4096-10, BASELINE config 4) that is a 13 MB fp32 all-reduce per step.  Sharding the hidden layer
instead (W1 rows / b1 / W2 columns, "column-then-row" parallel) leaves a single collective per step: the
SUM of the output pre-activations z2 (C x batch = 32 KB at batch 800), because

    z2   = sum_r W2[:, H_r] . sigmoid(W1[H_r] X + b1[H_r]) + b2     (one all-reduce)
    D    = (softmax(z2) - y) / B                                     (identical on every rank)
    dZ1  = (W2[:, H_r]^T D) .* a1_r .* (1 - a1_r)                    (local)
    dW1[H_r] = dZ1 X^T + reg W1[H_r],  db1[H_r] = dZ1 1,  dW2[:, H_r] = D a1_r^T + reg W2[:, H_r]   (local)
    db2  = D 1                                                       (identical on every rank)

so there is no gradient all-reduce at all and every rank processes the FULL global batch.  On MI355X the
z2 partials come for free out of the forward GEMM's tile epilogue (H_r >= 512), the z2 all-reduce (16 x B
fp32: 410 KB at B = 6400) goes through the xGMI one-shot kernel (parallel/xgmi.py, one launch that pulls the
R - 1 peer buffers over the point-to-point links -- latency-bound at this size, where a ring pays R - 1 hops)
or RCCL, and the head / weight-gradient kernels are the data-parallel engine's (MlpStep.tp_forward / tp_head
/ run(parts=2)).  f64 and the torch backend run the same algorithm in PyTorch ops (CPU-testable with gloo /
LoopbackComm).  This is the chosen plan for BASELINE config 4 (784-4096-10, 8 GPUs): one 410 KB all-reduce per
step instead of data parallelism's 13 MB gradient all-reduce (docs/PERFORMANCE.md, Communication policy).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .comm import Communicator, NullComm
from .engine import MlpEngine
from .trainer import EpochPlan, TrainStats


def tp_allreduce_mode(mode: str) -> str:
    """The z2 all-reduce for a data-parallel ``--allreduce`` choice, the same in every entry point (bench.py,
    train.py): the z2 sum is latency-bound (16 x batch fp32), so the xGMI two-shot form maps to the one-shot
    kernel (xgmi2 -> xgmi) and the host-staged reference form to the communicator (host -> rccl)."""
    return {"auto": "auto", "xgmi": "xgmi", "xgmi2": "xgmi", "rccl": "rccl", "host": "rccl", "off": "rccl"}[mode]


class TensorParallelTrainer:
    """Hidden-sharded training: rank r owns hidden units [r*H/R, (r+1)*H/R)."""

    def __init__(self, nn, comm: Communicator | None = None, device=None, dtype: str = "f32",
                 batch_size: int = 800, backend: str = "hip", shift: bool = True, normalize: bool = False,
                 path: str = "auto", allreduce: str = "auto"):
        self.nn = nn
        self.comm = comm or NullComm()
        self.R, self.rank = self.comm.world_size, self.comm.rank
        P, H, C = nn.H
        if H % self.R:
            raise ValueError(f"hidden size {H} is not divisible by {self.R} tensor-parallel ranks")
        self.P, self.H, self.C = P, H, C
        self.Hs = H // self.R
        self.rows = slice(self.rank * self.Hs, (self.rank + 1) * self.Hs)
        self.B = int(batch_size)
        self.normalize = normalize
        self.engine = MlpEngine((P, self.Hs, C), dtype=dtype, max_cols=self.B, device=device, backend=backend,
                                shift=shift, path=path)
        self._set_shard(*nn.params)
        e = self.engine
        # the shard's dW1 has few output tiles and K = the whole global batch (512 x 785 outputs, K = 6400 for
        # 784-4096-10 on 8 ranks): the weight-gradient launch may split K (mlp_split.hip splitk_sgd_kernel)
        e.enable_splitk(8)
        # all-reduced pre-activation z2 (without b2), [16][ld] fp32 -- the layout head_wide_kernel reads
        self.z2 = torch.zeros(16, e.ld, dtype=e.pdt if not e.np else torch.float32, device=e.device)
        self._z2part = None
        if e.backend == "hip" and e.np and e.z2buf is not None:
            self._z2part = e.z2buf
        self.iter = 0
        self._graphs: dict = {}
        self.use_graphs = True
        self.profiler = None
        # the z2 all-reduce: the xGMI one-shot kernel (allreduce auto / xgmi) when every rank is a GPU of this
        # node, else the communicator's (RCCL / gloo)
        self._xz = self._setup_xgmi(allreduce)
        self.allreduce_impl = "none" if self.R == 1 else (
            "xgmi-z2" if self._xz is not None else f"z2 all-reduce ({self.comm.name})")

    def _setup_xgmi(self, mode: str):
        from .comm import TorchDistComm

        if mode not in ("auto", "xgmi", "xgmi2", "rccl", "host", "off"):
            raise ValueError("allreduce must be auto, xgmi, xgmi2, rccl, host or off")
        mode = tp_allreduce_mode(mode)
        e = self.engine
        ok = (self.R > 1 and isinstance(self.comm, TorchDistComm) and e.device.type == "cuda" and e.backend == "hip"
              and e.np and self.z2.dtype == torch.float32)
        if mode == "rccl" or not ok:
            if mode == "xgmi" and not ok:
                raise RuntimeError("the xGMI z2 all-reduce needs >1 GPU ranks on the hip split path")
            return None
        from .xgmi import XgmiBucket, same_node

        if mode == "auto" and not same_node(self.R):
            return None
        try:
            xb = XgmiBucket(self.comm.group, self.rank, self.R, self.z2.numel(), torch.float32, e.device)
        except Exception as ex:  # every rank fails at the same point (collective set-up)
            if mode == "xgmi":
                raise
            print(f"[rank {self.rank}] xgmi z2 all-reduce unavailable ({ex}); using {self.comm.name}", flush=True)
            return None
        if not xb.ok:
            xb.close()
            if mode == "xgmi":
                raise RuntimeError("xgmi z2 all-reduce self-test failed")
            return None
        return xb

    def comm_failed(self) -> bool:
        """Collective: True on every rank when any rank's xGMI peer wait timed out."""
        local = self._xz is not None and self._xz.error() != 0
        return local if self.R == 1 else self.comm.allreduce_scalar(1.0 if local else 0.0, op="max") > 0

    def close(self) -> None:
        """Collective: release the xGMI IPC bucket (every rank must call it)."""
        if self._xz is not None:
            # the engine's cached step reads the bucket's error word as its ag_err: point it back at the engine's
            # own word (or none) before that device memory is freed
            st = self.engine._step
            if st is not None:
                e = self.engine
                st.ag_err = e.ag_err.data_ptr() if e.ag_err is not None else 0
            self._xz.close()
            self._xz = None
        self._graphs.clear()

    # ------------------------------------------------------------------ params
    def _set_shard(self, W1, b1, W2, b2):
        r = self.rows
        self.engine.set_params(np.ascontiguousarray(W1[r]), np.ascontiguousarray(b1[r]),
                               np.ascontiguousarray(W2[:, r]), np.ascontiguousarray(b2))

    def gather_params(self):
        """Full (W1, b1, W2, b2) as float64 numpy on every rank (zero-padded SUM all-reduce: exact)."""
        e = self.engine
        W1s, b1s, W2s, b2 = e.get_params()
        dev = e.device
        full = torch.zeros(self.H * self.P + self.H + self.C * self.H, dtype=torch.float64, device=dev)
        W1 = full[:self.H * self.P].view(self.H, self.P)
        b1 = full[self.H * self.P:self.H * self.P + self.H]
        W2 = full[self.H * self.P + self.H:].view(self.C, self.H)
        W1[self.rows] = torch.as_tensor(W1s, device=dev)
        b1[self.rows] = torch.as_tensor(b1s, device=dev)
        W2[:, self.rows] = torch.as_tensor(W2s, device=dev)
        if self.R > 1:
            self.comm.allreduce_(full)
        return (W1.cpu().numpy().copy(), b1.cpu().numpy().copy(), W2.cpu().numpy().copy(), np.array(b2))

    def sync_to(self, nn) -> None:
        W1, b1, W2, b2 = self.gather_params()
        nn.W[0][...] = W1
        nn.b[0][...] = b1
        nn.W[1][...] = W2
        nn.b[1][...] = b2

    # -------------------------------------------------------------------- data
    def load(self, x_train, y_train):
        self.engine.load_dataset(x_train, y_train, normalize=self.normalize)
        self.N = self.engine.num_samples

    def epoch_plan(self, N: int | None = None) -> EpochPlan:
        N = self.N if N is None else N
        nb = (N + self.B - 1) // self.B
        return EpochPlan([(b * self.B, min(self.B, N - b * self.B)) for b in range(nb)])

    # -------------------------------------------------------------------- step
    def step(self, start: int, n: int, lr: float, reg: float, with_loss: bool = False) -> None:
        """One SGD step on samples [start, start+n) (every rank sees the whole batch)."""
        e = self.engine
        if e.backend == "hip" and e.np:
            self._step_hip(start, n, lr, reg, with_loss)
        else:
            self._step_torch(start, n, lr, reg, with_loss)

    def _step_hip(self, off, n, lr, reg, with_loss):
        e = self.engine
        st = e._hip_step()
        if self._xz is not None:
            # the weight-gradient launch applies nothing once a z2 peer wait of this rank timed out (the bucket's
            # sticky error word, read like the all-gather head's: SplitStepArgs::ag_err) -- a timed-out chunk
            # leaves this rank's unreduced partial in z2, which must never reach the weights
            st.ag_err = int(self._xz.c.err_address)
        stream = torch.cuda.current_stream(e.device).cuda_stream
        zp = self._z2part
        chunks = st.tp_forward(int(off), int(n), zp.data_ptr() if zp is not None else 0, stream)
        C, ld = self.C, e.ld
        if chunks > 0:
            self.z2[:, :n] = zp[:chunks * 16 * ld].view(chunks, 16, ld)[:, :, :n].sum(0)
        else:  # narrow shard (the wave-split-K forward): z2 partial through hipBLAS
            self.z2[:C, :n] = e.W2 @ e.a1[:, :n]
        if self._xz is not None:
            self._xz.allreduce_(self.z2)
        elif self.R > 1:
            self.comm.allreduce_(self.z2)
        st.tp_head(int(off), int(n), 1.0 / n, int(bool(with_loss)), self.z2.data_ptr(), stream)
        # local weight gradients + SGD (db1 from the all-ones feature column, dW2 / db2 roles)
        st.run(int(off), int(n), 1.0 / n, float(reg), float(lr), 1, 0, stream, 2)

    def _step_torch(self, off, n, lr, reg, with_loss):
        e = self.engine
        with torch.no_grad():
            Xb = e.X[off:off + n].to(e.pdt) * e.xscale
            W1g = e.W1p.to(e.pdt).sum(0) if e.np else e.W1g.to(e.pdt)
            a1 = torch.sigmoid(Xb @ W1g.t() + e.b1)                 # [n][Hs]
            z2 = (a1 @ e.W2.t()).t().contiguous()                   # [C][n] partial
            if self.R > 1:
                self.comm.allreduce_(z2)
            z2 = z2.t() + e.b2
            if e.shift:
                z2 = z2 - z2.max(dim=1, keepdim=True).values
            ex = torch.exp(z2)
            p = ex / ex.sum(dim=1, keepdim=True)
            lab = e.labels[off:off + n].long()
            idx = torch.arange(n, device=p.device)
            if with_loss:
                e.loss_buf.zero_()
                e.loss_buf[0] = -torch.log(p[idx, lab]).sum().float()
            onehot = torch.zeros_like(p)
            onehot[idx, lab] = 1.0
            D = (p - onehot) / n
            dZ1 = (D @ e.W2) * a1 * (1 - a1)
            e.a1[:, :n] = a1.t()
            e.D[:, :n] = D.t()
            e.dZ1[:, :n] = dZ1.t()
            e.W1.sub_(lr * (dZ1.t() @ Xb + reg * e.W1))
            e.W2.sub_(lr * (D.t() @ a1 + reg * e.W2))
            e.b1.sub_(lr * dZ1.sum(0))
            e.b2.sub_(lr * D.sum(0))
            e.refresh_shadow()

    def step_loss(self, start: int, n: int, lr: float, reg: float) -> float:
        """Step + the (pre-update) global loss, reference definition (neural_network.cpp:144-154)."""
        e = self.engine
        with torch.no_grad():
            nrm = float((e.W1.double() ** 2).sum() + (e.W2.double() ** 2).sum())
        nrm = self.comm.allreduce_scalar(nrm) if self.R > 1 else nrm
        self.step(start, n, lr, reg, with_loss=True)
        return e.loss_sum() / n + 0.5 * reg * nrm  # the cross-entropy term is identical on every rank

    # ------------------------------------------------------------------ graphs
    def graphs_usable(self, use_graphs: bool = True) -> bool:
        return bool(use_graphs and self.engine.device.type == "cuda"
                    and (self.R == 1 or self.comm.graph_capturable or self._xz is not None))

    def capture(self, plan: EpochPlan, lr: float, reg: float) -> torch.cuda.CUDAGraph:
        """Capture every step of ``plan`` into one HIP graph (state-neutral warm-up first); cached."""
        key = (tuple(plan.steps), float(lr), float(reg))
        g = self._graphs.get(key)
        if g is not None:
            return g
        e = self.engine
        # every derived copy of W1 too: the bf16 shadow W1g (bf16 + mfma path) is refreshed after the
        # update, so the warm-up step leaves it one step ahead of the restored master
        snap = (e.params.clone(), (e.W1p.clone() if e.W1p is not None else None),
                (e.W1g.clone() if e.W1g is not e.W1 else None))
        side = torch.cuda.Stream(e.device)
        side.wait_stream(torch.cuda.current_stream(e.device))
        with torch.cuda.stream(side):  # warm-up (lazy kernel loads, communicator set-up)
            self.step(*plan.steps[0], lr, reg)
        torch.cuda.current_stream(e.device).wait_stream(side)
        torch.cuda.synchronize(e.device)
        e.params.copy_(snap[0])
        if snap[1] is not None:
            e.W1p.copy_(snap[1])
        if snap[2] is not None:
            e.W1g.copy_(snap[2])
        e.mark_planes_stale()
        torch.cuda.synchronize(e.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for s, ln in plan.steps:
                self.step(s, ln, lr, reg)
        torch.cuda.synchronize(e.device)
        self._graphs[key] = g
        return g

    def run_plan(self, plan: EpochPlan, lr: float, reg: float, use_graphs: bool = True) -> None:
        """All steps of ``plan``; replayed from a captured HIP graph when the communicator allows it
        (RCCL / one rank) -- the z2 all-reduce is then a graph node like the kernels around it."""
        if self.graphs_usable(use_graphs):
            self.capture(plan, lr, reg).replay()
            self.engine.mark_planes_stale()  # (a host-free replay: the lazily refreshed planes may be stale)
        else:
            for s, ln in plan.steps:
                self.step(s, ln, lr, reg)

    # ------------------------------------------------------------------- train
    def train(self, epochs: int, lr: float, reg: float, print_every: int = 0, debug: bool = False,
              outdir: str = "Outputs", log=print, on_event=None, fault=None) -> TrainStats:
        """Training loop with the data-parallel trainer's interface (loss every ``print_every`` steps,
        JSON-lines epoch events, ``fault=(rank, step)`` injection); graph-replayed epochs when no loss is
        printed.  ``debug`` (the reference's per-iteration CPU diff) is data-parallel only."""
        from .trainer import CommFailure, FaultInjected

        stats = TrainStats()
        plan = self.epoch_plan()
        dev = self.engine.device
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self.comm.barrier()
        t0 = time.perf_counter()
        for epoch in range(epochs):
            if fault is not None and fault[0] == self.rank and self.iter <= fault[1] < self.iter + len(plan.steps):
                raise FaultInjected(f"injected fault on rank {self.rank} at step {fault[1]}")
            if print_every <= 0 and self.profiler is None:
                self.run_plan(plan, lr, reg, use_graphs=self.use_graphs)
                self.iter += len(plan.steps)
                stats.steps += len(plan.steps)
                stats.images += sum(ln for _, ln in plan.steps)
            else:
                for s, ln in plan.steps:
                    if print_every > 0 and self.iter % print_every == 0:
                        l = self.step_loss(s, ln, lr, reg)
                        stats.losses.append(l)
                        if self.rank == 0:
                            log(f"Loss at iteration {self.iter} of epoch {epoch}/{epochs} = {l:.10g}")
                        if on_event is not None:
                            on_event({"event": "loss", "iter": self.iter, "epoch": epoch, "loss": l})
                    elif self.profiler is not None:
                        with self.profiler.phase("step"):
                            self.step(s, ln, lr, reg)
                    else:
                        self.step(s, ln, lr, reg)
                    self.iter += 1
                    stats.steps += 1
                    stats.images += ln
            if self._xz is not None and self.comm_failed():
                # (collective) a z2 peer wait timed out on some rank: that rank's weight-gradient launches applied
                # nothing from then on, so the shards no longer belong to one model -- every rank stops together
                raise CommFailure(f"rank {self.rank}: an xGMI z2 all-reduce peer wait timed out on some rank; "
                                  "that rank stopped updating its shard while its peers may have applied the "
                                  "step, so the shards may be inconsistent -- restart from a checkpoint")
            if on_event is not None:
                if dev.type == "cuda":
                    torch.cuda.synchronize(dev)
                el = time.perf_counter() - t0
                on_event({"event": "epoch", "epoch": epoch, "iter": self.iter, "seconds": el,
                          "images_per_s": stats.images / el if el > 0 else None})
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self.comm.barrier()
        stats.seconds = time.perf_counter() - t0
        self.sync_to(self.nn)
        return stats

    def enable_profiling(self, roctx: bool = True):
        """Per-step timing (eager steps) + roctx ranges; returns the PhaseTimer."""
        from ..utils.tracing import PhaseTimer, Roctx

        dev = self.engine.device if self.engine.device.type == "cuda" else None
        self.profiler = PhaseTimer(dev, Roctx(True) if roctx else None)
        return self.profiler

    def predict(self, x) -> np.ndarray:
        """Argmax labels with the full model in ``self.nn`` (gathered by train() / sync_to() on every rank,
        so this needs no collective and may run on one rank only)."""
        e = self.engine
        full = MlpEngine((self.P, self.H, self.C), dtype=e.dtype, max_cols=min(4096, max(1, len(x))),
                         device=e.device, backend=e.backend, shift=e.shift)
        full.set_params(*self.nn.params)
        return full.predict(x)
