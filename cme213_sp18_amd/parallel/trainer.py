"""Synchronous data-parallel SGD trainer -- the reference's ``parallel_train``.

Semantics kept from fpcode/neural_network.cpp:401-575 (so a run on R ranks
reproduces the single-process result for the same global batch):
  * every global batch of B columns is split into R contiguous shards of
    ``n = floor(min(B, N - start) / R)`` columns; the remainder columns are
    dropped, exactly like the reference (:458);
  * local gradients are pre-scaled so that their SUM over ranks is the
    global-batch gradient: D scaled by ``1/(n*R)`` and ``reg/R`` (:330-334);
  * one SUM all-reduce, then every rank applies the same SGD update (:538-541);
  * identical seeded init on every rank -> no parameter broadcast.

What changes (MI355X-first):
  * no scatter and no host staging: each rank indexes its shard of the
    device-resident dataset; gradients stay in one flat device bucket;
  * one all-reduce over RCCL (instead of 4 blocking MPI_Allreduce on host
    buffers) followed by one fused SGD kernel; world_size == 1 applies SGD
    inside the weight-gradient kernel and communicates nothing;
  * the whole epoch (3-5 launches + 1 collective per step) is captured once
    into a HIP graph and replayed, so the CPU never sits on the critical path.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .comm import Communicator, NullComm
from .engine import MlpEngine


BUCKET_BYTES = 4 << 20         # dW1 all-reduce chunk of the overlapped RCCL backward


@dataclass
class CostModel:
    """The all-reduce policy's constants (docs/PERFORMANCE.md "Communication policy"): one xGMI link per direction
    (GB/s), the fixed cost of one peer-kernel launch + hand-off (us), RCCL's fixed cost (us) and its ring's per-link
    rate (GB/s).  The defaults are planning numbers (7.5 us is the one-shot kernel with 2 ranks sharing one GPU);
    ``measure_cost_model`` replaces them with a micro-probe on the node (bench.py does at N > 1 and records them as
    ``cost_model_measured``)."""

    link_gbps: float = 64.0
    kernel_us: float = 7.5
    rccl_us: float = 25.0
    rccl_gbps: float = 64.0
    hop_us: float = 1.0  # one one-way xGMI latency (a flag or a granule store seen by the peer): planning only
    measured: bool = False

    def as_record(self) -> dict:
        return {"xgmi_link_GBps": round(self.link_gbps, 2), "xgmi_kernel_us": round(self.kernel_us, 2),
                "rccl_fixed_us": round(self.rccl_us, 2), "rccl_link_GBps": round(self.rccl_gbps, 2),
                "hop_us_planning": self.hop_us, "measured": self.measured}


COST_MODEL = CostModel()  # what the policy uses (set_cost_model replaces it)


def set_cost_model(m: CostModel | None) -> None:
    global COST_MODEL
    COST_MODEL = m if m is not None else CostModel()


def allreduce_cost_us(R: int, wire_bytes: int, shots: int, fp_bytes: int | None = None,
                      model: CostModel | None = None) -> float:
    """Predicted time of one gradient all-reduce of ``wire_bytes`` over R ranks of one node: shots 1 = the xGMI
    one-shot kernel (L + S / B: every rank pulls the R - 1 peer buckets over R - 1 links at once), 2 = the
    two-shot kernel (2 L + 2 S / (R B)), 0 = the RCCL path (L_rccl + 2 S / (R B_rccl) on the fp32 bucket
    ``fp_bytes``, minus what the bucketed backward hides behind the dW1 GEMM: up to L_rccl once the gradient
    spans more than one BUCKET_BYTES chunk -- a one-bucket gradient goes after the whole weight-gradient launch)."""
    if R <= 1:
        return 0.0
    m = model or COST_MODEL
    bw = m.link_gbps * 1e3  # bytes per us
    if shots == 1:
        return m.kernel_us + wire_bytes / bw
    if shots == 2:
        return 2 * m.kernel_us + 2 * wire_bytes / (R * bw)
    fb = wire_bytes if fp_bytes is None else fp_bytes
    ring = 2 * fb / (R * m.rccl_gbps * 1e3)
    hidden = min(m.rccl_us, ring) if fb > BUCKET_BYTES else 0.0
    return m.rccl_us + ring - hidden


def fused_exchange_us(R: int, wire_bytes: int, form: str, model: CostModel | None = None) -> float:
    """Predicted cost of the all-reduce fused into the weight-gradient launch, beyond the launch's own work
    (bench/predict_scaling.py states the same model): "pull" (the one-shot: a flag one way, then a remote read
    round trip of every peer's tile, S bytes per link) 3 hops + S / B; "push" (the owner-tile form: the tile one
    way to its owner, the update one way back, 2 S / R payload per link each way, doubled by the 8-byte tagged
    granules) 2 hops + 4 S / (R B)."""
    m = model or COST_MODEL
    bw = m.link_gbps * 1e3
    if form == "pull":
        return 3 * m.hop_us + wire_bytes / bw
    return 2 * m.hop_us + 4 * wire_bytes / (R * bw)


def auto_fused_form(R: int, wire_bytes: int, model: CostModel | None = None) -> str:
    """The fused all-reduce's form the cost model PREDICTS faster: the owner-tile push once its 4 S / R bytes per
    link and one hop fewer beat the one-shot's S (R >= 4 at 784-100-10 with the planning constants), else the pull.
    A prediction only (bench/predict_scaling.py): the hop latency is a planning constant nobody has measured across
    GPUs, so the trainer's "auto" form is the pull, and bench.py times the push next to it (dp_tune_allreduce) --
    the faster measured form is the one it runs."""
    return "push" if fused_exchange_us(R, wire_bytes, "push", model) < fused_exchange_us(R, wire_bytes, "pull",
                                                                                          model) else "pull"


def auto_allreduce_shots(R: int, wire_bytes: int, fp_bytes: int, bf16_wire: bool,
                         model: CostModel | None = None) -> int:
    """allreduce="auto" on one node: 1 = the xGMI one-shot kernel, 2 = the two-shot kernel, 0 = RCCL -- the
    candidate with the least predicted time (allreduce_cost_us).  The two-shot moves the exact gradient only (not
    the bf16 wire); RCCL always reduces the fp32 bucket.  With the planning constants: latency-bound buckets
    (318 KB at H = 100) take the one-shot at any R, 784-1024-10's 3.3 MB the one-shot at R = 2 (the two-shot and
    the ring move S per link there too) and the two-shot from R = 3, 784-4096-10's 13 MB the bucketed RCCL
    backward, whose ring hides behind the dW1 GEMM."""
    cands = {1: allreduce_cost_us(R, wire_bytes, 1, model=model),
             0: allreduce_cost_us(R, wire_bytes, 0, fp_bytes=fp_bytes, model=model)}
    if R >= 3 and not bf16_wire:
        cands[2] = allreduce_cost_us(R, wire_bytes, 2, model=model)
    return min(cands, key=lambda k: (cands[k], k))


def measure_cost_model(comm, device, small: int = 1024, large: int = 1 << 20, iters: int = 10) -> CostModel | None:
    """Collective micro-probe of the cost model's constants on this node (~1-2 s): the xGMI one-shot all-reduce and
    the communicator's (RCCL) all-reduce, each at ``small`` and ``large`` fp32 elements, max over ranks.  The small
    bucket's time is the fixed cost; the slope is the per-link rate (one-shot: t = L + S / B; ring:
    t = L + 2 (R - 1) / R S / B).  None where there is nothing to measure (one rank, no GPU, not a torch.distributed
    group); an xGMI bucket the node cannot open leaves the planning constants for the xGMI terms."""
    from .comm import TorchDistComm

    R = comm.world_size
    dev = torch.device(device)
    if R <= 1 or dev.type != "cuda" or not isinstance(comm, TorchDistComm):
        return None

    def timed(fn) -> float:
        for _ in range(3):
            fn()
        torch.cuda.synchronize(dev)
        comm.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize(dev)
        return comm.allreduce_scalar(1e6 * (time.perf_counter() - t0) / iters, op="max")

    m = CostModel(measured=True)
    plan = CostModel()
    t = {}
    for numel in (small, large):
        buf = torch.zeros(numel, dtype=torch.float32, device=dev)
        t[("rccl", numel)] = min(timed(lambda: comm.allreduce_(buf)) for _ in range(3))
    ds = 4 * (large - small)
    fixed, slope = _fit_bounded(t[("rccl", small)], t[("rccl", large)], 2 * (R - 1) / R * ds, plan.rccl_us,
                                plan.rccl_gbps)
    if fixed is None:
        m.rccl_us, m.rccl_gbps = plan.rccl_us, plan.rccl_gbps
        m.measured = False
    else:
        m.rccl_us, m.rccl_gbps = fixed, slope
    from .xgmi import XgmiBucket

    try:
        for numel in (small, large):
            xb = XgmiBucket(comm.group, comm.rank, R, numel, torch.float32, dev, self_test=False)
            buf = torch.zeros(numel, dtype=torch.float32, device=dev)
            try:
                t[("xgmi", numel)] = min(timed(lambda: xb.allreduce_(buf)) for _ in range(3))
            finally:
                xb.close()
        fixed, slope = _fit_bounded(t[("xgmi", small)], t[("xgmi", large)], ds, plan.kernel_us, plan.link_gbps)
        if fixed is None:
            m.measured = False
        else:
            m.kernel_us, m.link_gbps = fixed, slope
    except RuntimeError:  # IPC unavailable: raised on every rank together (XgmiBucket's collective setup)
        pass
    return m


def _fit_bounded(t_small: float, t_large: float, bytes_moved: float, plan_fixed_us: float, plan_gbps: float):
    """(fixed cost in us, rate in GB/s) from two timings (the min of 3 probes each, max over ranks), or (None, None)
    when the fit is not physical -- a non-positive fixed cost or slope, or a rate above 20 x the planning one (a noisy
    difference of two timings reads as hundreds of TB/s) -- so a noisy probe never replaces the planning constants
    (the caller keeps them and records measured = False).  A large fixed cost is kept: a host-staged (gloo)
    communicator really costs milliseconds, and the policy must see that.  The same decision on every rank: the
    timings are max-reduced before this is called."""
    dt = t_large - t_small
    if not (dt > 0 and t_small > 0):
        return None, None
    gbps = bytes_moved / dt / 1e3
    if gbps > 20 * plan_gbps:
        return None, None
    return t_small, gbps


class FaultInjected(RuntimeError):
    """Raised by ``train(fault=(rank, step))`` -- the failure-detection test hook."""


class CommFailure(RuntimeError):
    """Raised on every rank together when a peer-to-peer all-reduce wait timed out on any rank."""


class KernelHandoffTimeout(RuntimeError):
    """A forward + head launch in its all-gather form (H <= 128, or the fused wide head) waited past its bound
    for the other workgroups of its column tile (engine.kernel_error()): that launch's outputs are not trusted."""


@dataclass
class EpochPlan:
    steps: list  # [(start, length)]


@dataclass
class TrainStats:
    seconds: float = 0.0
    steps: int = 0
    images: int = 0
    losses: list = field(default_factory=list)

    @property
    def images_per_sec(self) -> float:
        return self.images / self.seconds if self.seconds > 0 else float("nan")


class DataParallelTrainer:
    def __init__(self, nn, comm: Communicator | None = None, device=None, dtype: str = "f32",
                 batch_size: int = 800, backend: str = "hip", shift: bool = True, use_graphs: bool = True,
                 normalize: bool = False, path: str = "auto", allreduce: str = "auto", overlap: bool = True,
                 overlap_chunks: int = 0, fuse_allreduce: bool = True, executor: str = "auto",
                 grad_wire: str = "auto", fused_form: str = "auto"):
        self.nn = nn
        # how run_plan enqueues a plan: "auto" = the native C++ step loop (MlpStep.run_steps) for plans of
        # consecutive full batches on the fused paths (pure device work), else the captured HIP graph;
        # "graph" = always the graph; "eager" = Python step by step
        if executor not in ("auto", "graph", "eager"):
            raise ValueError("executor must be auto, graph or eager")
        self.executor = executor
        # element type of the gradients on the xGMI wire: "f32" / "auto" (exact), "bf16" (opt-in: half the
        # bytes of the one-shot kernel, each rank's gradient rounded to bf16 once and summed in fp32 after the
        # pull -- data-parallel bf16 training then differs from single-GPU bf16 by that rounding; the two-shot
        # kernel moves 2 S / R bytes per link exactly, which beats it from 4 ranks on)
        if grad_wire not in ("auto", "f32", "bf16"):
            raise ValueError("grad_wire must be auto, f32 or bf16")
        self.grad_wire = grad_wire
        # the all-reduce fused into the weight-gradient launch (H <= 128): "push" = the owner-tile form (each tile
        # reduced by one rank, pushed both ways as tagged granules: 2 one-way hops, 2 S / R payload per link),
        # "pull" = the one-shot (every rank reads every peer's tile after its flag: S per link), "auto" = the pull:
        # the push is predicted faster from 4 ranks (auto_fused_form) but has not run across GPUs, and its pick
        # would rest on an unmeasured hop latency -- bench.py measures both forms on the node and runs the faster
        if fused_form not in ("push", "pull", "auto"):
            raise ValueError("fused_form must be push, pull or auto")
        self.fused_form = fused_form
        # RCCL path: dW1 row chunks all-reduced while the next chunk is computed (0: ~BUCKET_BYTES each).
        # Setting it also forces the overlapped path with ONE rank of a real process group (nccl world 1),
        # so a one-GPU box exercises the side-stream + graph-captured backward.
        self.overlap_chunks = int(overlap_chunks)
        self.comm = comm or NullComm()
        self.R = self.comm.world_size
        self.rank = self.comm.rank
        self.B = int(batch_size)
        self.dtype = dtype
        self.normalize = normalize
        self.use_graphs = bool(use_graphs) and backend == "hip" and (self.R == 1 or self.comm.graph_capturable)
        self.allreduce_mode = allreduce
        max_cols = max(1, self.B // self.R)
        self.engine = MlpEngine(nn.H, dtype=dtype, max_cols=max_cols, device=device, backend=backend, shift=shift,
                                path=path)
        self.engine.set_params(*nn.params)
        # training reads nothing of a1 after a step: the wide fused forward + head launch skips its 13 MB store
        # at H = 4096 (bench/wide_ag_ab.py: -1.4 us/step fp32, -2.1 us bf16)
        self.engine.set_store_a1(False)
        self._graphs: dict = {}
        self._sharing = None
        self.iter = 0
        # the all-gather forward + head launch waits for the other workgroups of its own launch: every
        # workgroup must be resident at once, which several processes sharing a GPU (each launch spinning
        # while the other's holds CUs) cannot promise -- one process per GPU keeps it
        from .comm import TorchDistComm

        # -- agreed by every rank (with uneven placement some ranks would otherwise take the all-gather form
        # and its epoch-end timeout check, a collective, while others do not: mismatched collectives)
        if self.R > 1 and isinstance(self.comm, TorchDistComm) and self.engine.device.type == "cuda":
            one_per_gpu = self._gpu_sharing() == 1  # (collective, like _all_true: every rank calls both)
            self.engine.set_fh_allgather(self._all_true(one_per_gpu and self.engine.fh_allgather))
        from ..utils.tracing import Roctx

        self.roctx = Roctx()       # CME_ROCTX=1: epoch / phase ranges for rocprofv3 --marker-trace
        self.profiler = None       # PhaseTimer (enable_profiling / --profile)
        self.xgmi = self._setup_xgmi(allreduce)
        # the same all-reduce fused into the wgrad launch (one kernel less per step, tiles reduced as
        # they finish): own IPC bucket with one flag slot per wgrad tile; enabled by load() once a
        # bitwise comparison with the separate-kernel step has passed on every rank
        self._xgmi_fused = None
        self.fused_allreduce = False
        if (self.xgmi is not None and fuse_allreduce and self.xgmi.wire == self.engine.params.dtype
                and self.xgmi.shots == 1):
            slots = self.engine.fused_allreduce_slots()
            if self.fused_form == "auto":
                self.fused_form = "pull"
            if slots and self.engine.params.dtype == torch.float32 and self._fused_fits(slots):
                from .xgmi import XgmiBucket

                try:
                    xb = XgmiBucket(self.comm.group, self.rank, self.R, self.engine.params.numel(),
                                    torch.float32, self.engine.device, flag_slots=slots,
                                    slab_tiles=slots if self.fused_form == "push" else 0)
                    if xb.ok:
                        self._xgmi_fused = xb
                    else:
                        xb.close()
                except RuntimeError as ex:  # raised on every rank together (collective setup)
                    print(f"[rank {self.rank}] fused xgmi bucket unavailable ({ex})", flush=True)
        if self.xgmi is not None and bool(use_graphs) and backend == "hip":
            self.use_graphs = True  # the xGMI steps are pure device work: capturable whatever the group
        # the overlapped backward only pays with >= 2 dW1 chunks; a gradient that fits ONE bucket (H=100:
        # 318 KB, H=1024: 3.3 MB) goes as ONE all-reduce on the compute stream after the whole wgrad launch
        # (two latency-bound collectives and a second graph stream would cost more than they hide)
        multi = self.R > 1 or (self.overlap_chunks > 0 and not isinstance(self.comm, NullComm))
        self._bucketed = (multi and self.xgmi is None and allreduce != "host" and overlap
                          and self.engine.supports_bucketed_wgrad and self.engine.device.type == "cuda"
                          and len(self._buckets()) > 1)
        self._comm_stream = torch.cuda.Stream(self.engine.device) if self._bucketed else None
        self.allreduce_impl = "none" if self.R == 1 else (
            ("xgmi-bf16wire" if self.xgmi.wire == torch.bfloat16 else "xgmi-2shot" if self.xgmi.shots == 2
             else "xgmi") if self.xgmi is not None
            else "host-gloo" if allreduce == "host" else self.comm.name)
        # train(): one in-process recovery from a timed-out hand-off or peer wait (the snapshot taken at the start
        # of every epoch is restored and the epoch re-run on the co-residency-free / RCCL path); False: raise
        self.recover = True
        self.recovered: str | None = None

    def _setup_xgmi(self, mode: str):
        """Peer-to-peer fused all-reduce+SGD (parallel/xgmi.py) when every rank is a GPU on this node.
        mode: auto (use it if the self-test passes), xgmi (require it), rccl/off (never)."""
        from .comm import TorchDistComm

        if mode not in ("auto", "xgmi", "xgmi2", "rccl", "off", "host"):
            raise ValueError("allreduce must be auto, xgmi, xgmi2, rccl, host or off")
        if mode == "host":
            # reference-equivalent sync: gradients staged through host memory and summed over a
            # gloo group, as the reference's MPI_Allreduce on host buffers (neural_network.cpp:496-536)
            self.use_graphs = False
            if self.R > 1:
                import torch.distributed as dist

                self._host_group = dist.new_group(backend="gloo")
            return None
        e = self.engine
        eligible = (self.R > 1 and isinstance(self.comm, TorchDistComm) and e.device.type == "cuda"
                    and e.backend == "hip" and e.params.dtype in (torch.float32, torch.float64))
        if mode in ("rccl", "off") or not eligible:
            if mode in ("xgmi", "xgmi2") and not eligible:
                raise RuntimeError("xgmi all-reduce needs >1 GPU ranks of the hip backend")
            return None
        from .xgmi import XgmiBucket, same_node

        if mode == "auto" and (not same_node(self.R) or self.R > 8):
            return None
        # one-shot / two-shot / RCCL by the cost model of auto_allreduce_shots (the bytes that count are the
        # WIRE bytes)
        fp_bytes = e.params.numel() * e.params.element_size()
        bf16_wire = e.params.dtype == torch.float32 and self.grad_wire == "bf16"
        wire = torch.bfloat16 if bf16_wire else e.params.dtype
        wire_bytes = e.params.numel() * torch.tensor([], dtype=wire).element_size()
        shots = 2 if mode == "xgmi2" else 1
        if mode == "auto":
            shots = auto_allreduce_shots(self.R, wire_bytes, fp_bytes, bf16_wire)
            if shots == 0:
                return None
        if shots == 2 and bf16_wire:
            raise ValueError("the two-shot xGMI all-reduce moves the exact gradient (grad_wire f32)")
        try:
            xb = XgmiBucket(self.comm.group, self.rank, self.R, e.params.numel(), e.params.dtype, e.device,
                            wire=wire, shots=shots)
        except Exception as ex:  # IPC unavailable: every rank sees the same failure at the same point
            if mode in ("xgmi", "xgmi2"):
                raise
            print(f"[rank {self.rank}] xgmi all-reduce unavailable ({ex}); using {self.comm.name}", flush=True)
            return None
        if not xb.ok:
            xb.close()
            if mode in ("xgmi", "xgmi2"):
                raise RuntimeError("xgmi all-reduce self-test failed")
            return None
        return xb

    def _gpu_sharing(self) -> int:
        """How many ranks of the group run on this rank's GPU (1 = one process per GPU).  Collective."""
        import torch.distributed as dist

        if self._sharing is None:
            from .launcher import device_identity

            ids = [None] * self.R
            dist.all_gather_object(ids, device_identity(self.engine.device), group=self.comm.group)
            self._sharing = sum(1 for x in ids if x == ids[self.rank])
        return self._sharing

    def _fused_fits(self, tiles: int) -> bool:
        """Every wgrad tile waits for the same tile of its peers, so all tiles of all ranks SHARING a
        GPU must be resident at once (2 workgroups of 512 threads per CU at the kernel's occupancy).
        One rank per GPU always fits (~180 tiles at H=100 on 256 CUs); the several-ranks-on-one-GPU
        rehearsal only with 2 ranks.  Collective."""
        props = torch.cuda.get_device_properties(self.engine.device)
        return self._all_true(self._gpu_sharing() * tiles <= 2 * props.multi_processor_count)

    def _all_true(self, v: bool) -> bool:
        import torch.distributed as dist

        out = [None] * self.R
        dist.all_gather_object(out, bool(v), group=self.comm.group)
        return all(out)

    def check_comm(self) -> None:
        """Raise if a peer wait of an xGMI all-reduce timed out on THIS rank (local check, no collective)."""
        for b in (self.xgmi, self._xgmi_fused):
            if b is not None:
                b.check()

    def comm_failed(self) -> bool:
        """Collective: True on EVERY rank when any rank's xGMI peer wait timed out.  A block whose wait
        timed out applied nothing (csrc/comm/xgmi_allreduce.hip), but other ranks may have applied that
        step, so the replicas can no longer be trusted to agree -- callers stop (or restart) as one."""
        local = any(b is not None and b.error() for b in (self.xgmi, self._xgmi_fused))
        if self.R == 1:
            return local
        return self.comm.allreduce_scalar(1.0 if local else 0.0, op="max") > 0

    def replicas_agree(self) -> bool:
        """Collective: True when every rank holds BITWISE the same parameters.  Every all-reduce path sums in
        a rank-independent order (xGMI: rank order on every rank; RCCL/host: one result broadcast), so
        weak- and strong-scaling replicas must agree exactly; a stale peer read in the xGMI hand-off would
        show up here as a mismatch rather than as a hang."""
        if self.R == 1:
            return True
        p = self.engine.params.detach().reshape(-1)
        w = p.view(torch.int32) if p.element_size() == 4 else p.view(torch.int16) if p.element_size() == 2 \
            else p.view(torch.int64)
        w = w.to(torch.int64)
        idx = torch.arange(1, w.numel() + 1, device=w.device, dtype=torch.int64)
        # two position-weighted sums, folded below 2^52 so they travel exactly as float64
        h = [int(w.sum().item()) % (1 << 52), int(((w % 65521) * (idx % 65519)).sum().item()) % (1 << 52)]
        return all(self.comm.allreduce_scalar(float(v), op="max") == self.comm.allreduce_scalar(float(v), op="min")
                   for v in h)

    def assert_comm_ok(self) -> None:
        """Collective: raise KernelHandoffTimeout on every rank together if any rank's all-gather forward +
        head launch timed out waiting for its tile, and CommFailure if any rank's xGMI peer wait timed out.
        Either way NO rank applied the affected update or any later one: a timed-out launch's rank stops
        updating (the weight-gradient launch reads the sticky error word) and marks its gradient bucket (the
        status element, so RCCL / host all-reduces make every rank skip the SGD) or stops taking part in the
        xGMI exchange (its peers' waits time out and apply nothing).  The hand-off check comes first: it is
        the cause when both fire."""
        if self._allgather_live():
            local = self.engine.kernel_error()
            bad = local if self.R == 1 else self.comm.allreduce_scalar(1.0 if local else 0.0, op="max") > 0
            if bad:
                raise KernelHandoffTimeout(f"rank {self.rank}: an all-gather forward + head launch timed out "
                                           "waiting for its column tile on some rank; no rank applied that step "
                                           "or any later one")
        if (self.xgmi is not None or self._xgmi_fused is not None) and self.comm_failed():
            raise CommFailure(f"rank {self.rank}: an xGMI all-reduce peer wait timed out on some rank "
                              "(a rank stalled or died); no rank applied the affected update")

    def _allgather_live(self) -> bool:
        e = self.engine
        return e.backend == "hip" and e.ag_err is not None and bool(e.fh_allgather)

    def close(self) -> None:
        """Collective: release the xGMI IPC buckets (every rank must call it)."""
        self.engine.attach_xgmi(None)
        for name in ("_xgmi_fused", "xgmi"):
            b = getattr(self, name)
            if b is not None:
                b.close()
                setattr(self, name, None)
        self.fused_allreduce = False
        self._graphs.clear()

    def _allreduce_sgd(self, lr: float) -> None:
        e = self.engine
        if self.allreduce_mode == "host":
            if self.R > 1:
                import torch.distributed as dist

                g = e.grads.cpu()
                dist.all_reduce(g, group=self._host_group)
                e.grads.copy_(g)
            e.sgd(lr)
            return
        if self.xgmi is None:
            self.comm.allreduce_(e.grads)
            e.sgd(lr)
            return
        planes, np_ = None, 0
        if e.np:  # split paths: refresh the exact bf16 planes of W1
            planes, np_ = e.W1p, e.np
        elif e.dtype == "bf16":  # bf16 path: single-rounded shadow of W1
            planes, np_ = e.W1g, 1
        self.xgmi.sgd_(e.grads, e.params, lr, planes, np_, e.H * e.P, status_index=e.status_index)
        e._w1_written()

    # ---------------------------------------------------------------- data
    def load(self, x_train, y_train):
        self.engine.load_dataset(x_train, y_train, normalize=self.normalize)
        self.N = self.engine.num_samples
        self._graphs.clear()
        if self._xgmi_fused is not None:
            self.fused_allreduce = self._check_fused()
            self.allreduce_impl = ("xgmi-push" if self.fused_form == "push" else "xgmi-fused") \
                if self.fused_allreduce else "xgmi"

    def _check_fused(self) -> bool:
        """One step from the same state through both all-reduce paths (separate xGMI kernel, and
        fused into wgrad); enable the fused one only if every rank gets bitwise-identical parameters
        and bf16 planes.  The state is restored afterwards.  Collective."""
        e = self.engine
        if e.fused_allreduce_slots() == 0 or self.N < self.R:
            e.attach_xgmi(None)
            return False
        snap = self._snapshot()
        off, n = self.shard(0, min(self.B, self.N))
        scale, reg, lr = 1.0 / (n * self.R), 1e-3 / self.R, 0.05
        e.attach_xgmi(None)
        e.run(off, n, scale, reg, lr, sgd=False)
        self._allreduce_sgd(lr)
        # (the W1 planes only where a forward kernel reads them: below H = 512 the fused update skips them)
        planes = e.w1_planes_maintained()
        ref = (e.params.clone(), e.W1p.clone() if planes else None)
        self._restore(snap)
        ok = True
        try:
            e.attach_xgmi(self._xgmi_fused, push=self.fused_form == "push")
            for _ in range(3):  # both buffer halves, and back to the first
                self._restore(snap)
                e.run(off, n, scale, reg, lr, sgd=2)
                torch.cuda.synchronize(e.device)
                ok &= bool(torch.equal(e.params, ref[0]) and (not planes or torch.equal(e.W1p, ref[1])))
            ok &= self._xgmi_fused.error() == 0 and self.xgmi.error() == 0
        except RuntimeError as ex:
            print(f"[rank {self.rank}] fused xgmi step failed: {ex}", flush=True)
            ok = False
        self._restore(snap)
        torch.cuda.synchronize(e.device)
        ok = self._all_true(ok)
        self._graphs.clear()  # (graphs captured against another attachment must not be replayed: MlpStep.set_xgmi)
        if not ok:
            e.attach_xgmi(None)
            self._xgmi_fused.close()  # collective; also drops its error flag
            self._xgmi_fused = None
            if self.rank == 0:
                print("[xgmi] fused all-reduce self-check failed; using the separate kernel", flush=True)
        return ok

    def _enqueue_plan(self, plan: EpochPlan, lr: float, reg: float) -> None:
        steps = plan.steps
        for i, (s, ln) in enumerate(steps):
            nxt = steps[i + 1] if i + 1 < len(steps) else steps[0]  # (whose pixels this step prefetches)
            self.step(s, ln, lr, reg, next_start=self.shard(*nxt)[0])

    def epoch_plan(self, N: int | None = None) -> EpochPlan:
        N = self.N if N is None else N
        nb = (N + self.B - 1) // self.B
        return EpochPlan([(b * self.B, min(self.B, N - b * self.B)) for b in range(nb)])

    # ---------------------------------------------------------------- step
    def shard(self, start: int, length: int) -> tuple[int, int]:
        n = length // self.R
        return start + self.rank * n, n

    def step(self, start: int, length: int, lr: float, reg: float, with_loss: bool = False,
             next_start: int = -1) -> None:
        """Enqueue one global SGD step on the current stream (no host sync).  next_start: this rank's first sample
        of the next step (the fused paths prefetch its pixels; -1: unknown)."""
        e = self.engine
        off, n = self.shard(start, length)
        if self.profiler is not None and n > 0:
            self._profiled_step(off, n, 1.0 / (n * self.R), reg, lr, with_loss)
            return
        if n == 0:  # fewer columns than ranks: only the regulariser contributes
            e.reg_only_grads(reg / self.R)
            self._allreduce_sgd(lr)
            return
        scale = 1.0 / (n * self.R)
        if isinstance(self.comm, NullComm) and self.allreduce_mode != "host":  # 1 process: SGD fused into wgrad
            e.run(off, n, scale, reg, lr, sgd=True, with_loss=with_loss, pf_next=next_start)
        elif self.fused_allreduce:
            e.run(off, n, scale, reg / self.R, lr, sgd=2, with_loss=with_loss, pf_next=next_start)
        elif self._bucketed:
            self._step_bucketed(off, n, scale, reg / self.R, lr, with_loss)
        else:
            e.run(off, n, scale, reg / self.R, lr, sgd=False, with_loss=with_loss)
            self._allreduce_sgd(lr)

    def _profiled_step(self, off, n, scale, reg, lr, with_loss):
        """The same step, split into timed phases (PhaseTimer events + roctx ranges; eager only)."""
        e, P = self.engine, self.profiler
        single = isinstance(self.comm, NullComm) and self.allreduce_mode != "host"
        if e.backend != "hip":
            with P.phase("step"):
                if single:
                    e.run(off, n, scale, reg, lr, sgd=True, with_loss=with_loss)
                else:
                    e.run(off, n, scale, reg / self.R, lr, sgd=False, with_loss=with_loss)
                    self._allreduce_sgd(lr)
            return
        if single or self.fused_allreduce:
            sgd, r = (True, reg) if single else (2, reg / self.R)
            with P.phase("fwd_head"):
                e.run(off, n, scale, r, lr, sgd=sgd, with_loss=with_loss, parts=1)
            with P.phase("wgrad_sgd" if single else "wgrad_allreduce_sgd"):
                e.run(off, n, scale, r, lr, sgd=sgd, with_loss=with_loss, parts=2)
            return
        r = reg / self.R
        with P.phase("fwd_head"):
            e.run(off, n, scale, r, lr, sgd=False, with_loss=with_loss, parts=1)
        with P.phase("wgrad"):
            e.run(off, n, scale, r, lr, sgd=False, with_loss=with_loss, parts=2)
            e.join()
        if self.allreduce_mode == "host" or self.xgmi is not None:
            with P.phase("allreduce_sgd"):
                self._allreduce_sgd(lr)
            return
        with P.phase("allreduce"):
            self.comm.allreduce_(e.grads)
        with P.phase("sgd"):
            e.sgd(lr)

    def enable_profiling(self, roctx: bool = True):
        """Per-phase timing (and roctx ranges) for the following train() calls: steps run eagerly and
        split into forward+head / weight-gradient / all-reduce / SGD phases (the graph-replayed
        production path has no phase boundaries to time).  Returns the PhaseTimer."""
        from ..utils.tracing import PhaseTimer, Roctx

        self.roctx = Roctx(True) if roctx else self.roctx
        dev = self.engine.device if self.engine.device.type == "cuda" else None
        self.profiler = PhaseTimer(dev, self.roctx)
        return self.profiler

    def _buckets(self):
        """dW1 row chunks of ~BUCKET_BYTES (multiples of 128 rows, the blocked-GEMM tile)."""
        e = self.engine
        w1_bytes = e.H * e.P * e.params.element_size()
        k = self.overlap_chunks if self.overlap_chunks > 0 else max(1, min(8, -(-w1_bytes // BUCKET_BYTES)))
        rows = -(-e.H // k)
        rows = -(-rows // 128) * 128
        return [(r0, min(rows, e.H - r0)) for r0 in range(0, e.H, rows)]

    def _step_bucketed(self, off, n, scale, reg, lr, with_loss):
        """Backward with the gradient all-reduce overlapped (RCCL path): every dW1 row
        chunk is all-reduced on a side stream as soon as its GEMM has finished, while the next chunk
        is still being computed; the small [b1|W2|b2] bucket follows the last chunk."""
        e = self.engine
        cur = torch.cuda.current_stream(e.device)
        cs = self._comm_stream
        e.run_forward_head(off, n, scale, with_loss)
        e.run_wgrad(off, n, scale, reg, parts=2)
        w1n = e.H * e.P
        # dW1 row chunks first (each all-reduced while the next is computed); the small tail bucket
        # [b1|W2|b2] last, because db1 comes out of the dW1 GEMMs (all-ones feature column)
        pieces = [(e.grads[r0 * e.P:(r0 + rows) * e.P], (r0, rows)) for r0, rows in self._buckets()]
        pieces.append((e.grads[w1n:], None))
        for view, rng in pieces:
            if rng is not None:
                e.run_wgrad(off, n, scale, reg, parts=1, row0=rng[0], rows=rng[1])
            ev = torch.cuda.Event()
            ev.record(cur)
            cs.wait_event(ev)
            with torch.cuda.stream(cs):
                self.comm.allreduce_(view)
        cur.wait_stream(cs)
        e.sgd(lr)

    def step_loss(self, start: int, length: int, lr: float, reg: float) -> float:
        """One step that also returns the (pre-update) global loss -- reference
        ``loss()`` definition (neural_network.cpp:144-154)."""
        e = self.engine
        with torch.no_grad():
            nrm = float((e.W1.double() ** 2).sum() + (e.W2.double() ** 2).sum())
        self.step(start, length, lr, reg, with_loss=True)
        _, n = self.shard(start, length)
        ce = self.comm.allreduce_scalar(e.loss_sum()) if n > 0 else 0.0
        return ce / max(1, n * self.R) + 0.5 * reg * nrm

    # -------------------------------------------------------------- graphs
    def _snapshot(self):
        e = self.engine
        e.join()
        return (e.params.clone(), (e.W1g.clone() if e.W1g is not e.W1 else None),
                (e.W1p.clone() if e.W1p is not None else None))

    def _restore(self, snap):
        e = self.engine
        e.params.copy_(snap[0])
        if snap[1] is not None:
            e.W1g.copy_(snap[1])
        if snap[2] is not None:
            e.W1p.copy_(snap[2])
        e.mark_planes_stale()

    def capture(self, plan: EpochPlan, lr: float, reg: float) -> torch.cuda.CUDAGraph:
        """Capture every step of ``plan`` into one HIP graph (state-neutral warm-up first)."""
        key = (tuple(plan.steps), float(lr), float(reg))
        g = self._graphs.get(key)
        if g is not None:
            return g
        snap = self._snapshot()
        side = torch.cuda.Stream(self.engine.device)
        side.wait_stream(torch.cuda.current_stream(self.engine.device))
        with torch.cuda.stream(side):  # warm-up: lazy kernel loads, communicator init
            self._enqueue_plan(EpochPlan(plan.steps[:1]), lr, reg)
        torch.cuda.current_stream(self.engine.device).wait_stream(side)
        torch.cuda.synchronize(self.engine.device)
        self._restore(snap)
        torch.cuda.synchronize(self.engine.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._enqueue_plan(plan, lr, reg)
        torch.cuda.synchronize(self.engine.device)
        self._graphs[key] = g
        return g

    def native_plan(self, plan: EpochPlan):
        """(gstart0, count) when ``plan`` runs on the native step loop: executor "auto", the hip backend,
        a fused step (one process, or the xGMI all-reduce fused into wgrad) and consecutive full global
        batches (wrapping to 0 at the end of the dataset); else None."""
        e = self.engine
        if (self.executor != "auto" or e.backend != "hip" or self.profiler is not None or not plan.steps
                or not ((isinstance(self.comm, NullComm) and self.allreduce_mode != "host") or self.fused_allreduce)):
            return None
        g0 = plan.steps[0][0]
        gs = g0
        for s0, ln in plan.steps:
            if gs + self.B > self.N:
                gs = 0
            if s0 != gs or ln != self.B:
                return None
            gs += self.B
        return g0, len(plan.steps)

    def plan_runner(self, plan: EpochPlan, lr: float, reg: float):
        """A zero-argument callable that enqueues ``plan`` with everything resolved up front (the native
        loop's arguments bound, or the graph captured): the least host time between a timer start and the
        first kernel, for short timed runs (bench.py)."""
        nat = self.native_plan(plan)
        if nat is not None:
            e = self.engine
            n = self.B // self.R
            sgd, r = (1, reg) if isinstance(self.comm, NullComm) else (2, reg / self.R)
            args = (nat[0], nat[1], self.B, self.rank * n, n, self.N, 1.0 / (n * self.R), r, lr, sgd,
                    torch.cuda.current_stream(e.device).cuda_stream)
            fn = e._hip_step().run_steps
            return lambda: fn(*args)
        if self.use_graphs and self.executor != "eager":
            g = self.capture(plan, lr, reg)

            def replay():
                g.replay()
                # a replay runs host-free: the lazily refreshed W1 planes (MlpStep.planes_stale) may be stale again
                self.engine.mark_planes_stale()
            return replay
        return lambda: self._enqueue_plan(plan, lr, reg)

    def run_plan(self, plan: EpochPlan, lr: float, reg: float) -> None:
        nat = self.native_plan(plan)
        if nat is not None:
            e = self.engine
            n = self.B // self.R
            sgd, r = (1, reg) if isinstance(self.comm, NullComm) else (2, reg / self.R)
            e._hip_step().run_steps(nat[0], nat[1], self.B, self.rank * n, n, self.N, 1.0 / (n * self.R), r, lr,
                                    sgd, torch.cuda.current_stream(e.device).cuda_stream)
        elif self.use_graphs and self.executor != "eager":
            self.capture(plan, lr, reg).replay()
            self.engine.mark_planes_stale()  # (the replay's in-place updates skipped the plane refresh)
        else:
            self._enqueue_plan(plan, lr, reg)

    # ------------------------------------------------------------- recovery
    def _fall_back_to_comm(self) -> None:
        """Collective: drop the xGMI all-reduce (its sticky error word and per-tile epochs can no longer be trusted
        after a timed-out peer wait) and use the communicator's all-reduce (RCCL on GPUs), bucketed and overlapped
        where the gradient spans several buckets -- the same choice __init__ makes with allreduce="rccl"."""
        self.engine.attach_xgmi(None)
        self._graphs.clear()
        for name in ("_xgmi_fused", "xgmi"):
            b = getattr(self, name)
            if b is not None:
                b.close()
                setattr(self, name, None)
        self.fused_allreduce = False
        self.allreduce_mode = "rccl"
        self._bucketed = (self.R > 1 and self.engine.supports_bucketed_wgrad and self.engine.device.type == "cuda"
                          and len(self._buckets()) > 1)
        self._comm_stream = torch.cuda.Stream(self.engine.device) if self._bucketed else None
        self.use_graphs = self.use_graphs and (self.R == 1 or self.comm.graph_capturable)
        self.allreduce_impl = self.comm.name if self.R > 1 else "none"

    def _recover_epoch(self, ex: Exception, snap) -> bool:
        """Collective (every rank raised ``ex`` together from assert_comm_ok): restore the epoch-start snapshot and
        switch to the path that cannot hit the same failure -- a timed-out all-gather forward + head launch ->
        the last-arriver form (no workgroup waits for another, mlp_fwd1_head); a timed-out xGMI peer wait -> the
        communicator's all-reduce.  Once per trainer; returns False when the failure must propagate."""
        if not self.recover or self.recovered is not None or snap is None:
            return False
        e = self.engine
        if e.device.type == "cuda":
            torch.cuda.synchronize(e.device)
        what = "hand-off" if isinstance(ex, KernelHandoffTimeout) else "peer wait"
        if isinstance(ex, KernelHandoffTimeout):
            e.set_fh_allgather(False)
            e.ag_err.zero_()
        # a rank whose forward timed out stops taking part in the xGMI exchange, so its peers' waits time out
        # too: the buckets are poisoned whichever failure was raised
        if (self.xgmi is not None or self._xgmi_fused is not None) and (isinstance(ex, CommFailure)
                                                                         or self.comm_failed()):
            self._fall_back_to_comm()
        self._restore(snap[0])
        self.iter = snap[1]
        self._graphs.clear()
        self.recovered = f"{what} timed out at epoch-start iter {snap[1]}; re-ran on " + (
            "the last-arriver forward + head" if isinstance(ex, KernelHandoffTimeout) else self.allreduce_impl)
        if self.rank == 0:
            print(f"warning: {ex} -- restored the epoch-start snapshot and continuing "
                  f"({self.recovered})", flush=True)
        return True

    # ---------------------------------------------------------------- train
    def train(self, epochs: int, lr: float, reg: float, print_every: int = 0, debug: bool = False,
              outdir: str = "Outputs", log=print, on_event=None, fault: tuple[int, int] | None = None,
              diff_file=None) -> TrainStats:
        """Full training loop (neural_network.cpp:446-555).  Eager steps where the
        host must look at a step (loss printing / debug diffs), graphs elsewhere.

        on_event(dict): structured progress records (loss, epoch) for JSON-lines logs.
        fault=(rank, step): raise FaultInjected on that rank when the global step
        counter reaches ``step`` (before it runs) -- tests that a failing rank
        takes the job down instead of leaving its peers hung.

        diff_file: an open text file for the -d CPU-vs-GPU diff rows (the caller owns it across
        several train() segments); None: this call opens Outputs/CpuGpuDiff.txt itself -- truncated
        on a fresh run (iter 0), appended to when training resumes mid-run.

        With the xGMI all-reduce, every epoch ends with a collective check of the peer-wait error flag
        (assert_comm_ok): a timed-out wait raises CommFailure on every rank before another epoch runs."""
        from ..utils.checkpoint import write_diff_gpu_cpu

        stats = TrainStats()
        plan = self.epoch_plan()
        err_file, own_file = diff_file, False
        if debug and self.rank == 0 and err_file is None:  # only rank 0 owns the diff file
            os.makedirs(outdir, exist_ok=True)
            err_file = open(os.path.join(outdir, "CpuGpuDiff.txt"), "w" if self.iter == 0 else "a")
            own_file = True
        xgmi_live = self.xgmi is not None or self._xgmi_fused is not None
        ag_live = self._allgather_live()  # all-gather forward + head launches: their timeout flag, per epoch
        host_needed = print_every > 0 or debug or self.profiler is not None
        dev = self.engine.device
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self.comm.barrier()
        t0 = time.perf_counter()
        def maybe_fault(first: int, count: int):
            if fault is not None and fault[0] == self.rank and first <= fault[1] < first + count:
                raise FaultInjected(f"injected fault on rank {self.rank} at step {fault[1]}")

        def run_epoch(epoch: int) -> None:
            if not host_needed:
                maybe_fault(self.iter, len(plan.steps))
                with self.roctx.range(f"epoch {epoch}"):
                    self.run_plan(plan, lr, reg)
                if xgmi_live or ag_live:
                    self.assert_comm_ok()  # syncs; every rank raises together
                self.iter += len(plan.steps)
                stats.steps += len(plan.steps)
                stats.images += sum((ln // self.R) * self.R for _, ln in plan.steps)
                if on_event is not None:
                    if dev.type == "cuda":
                        torch.cuda.synchronize(dev)
                    el = time.perf_counter() - t0
                    on_event({"event": "epoch", "epoch": epoch, "iter": self.iter, "seconds": el,
                              "images_per_s": stats.images / el if el > 0 else None})
                return
            for bi, (s, ln) in enumerate(plan.steps):
                it = self.iter
                maybe_fault(it, 1)
                if print_every > 0 and it % print_every == 0:
                    l = self.step_loss(s, ln, lr, reg)
                    stats.losses.append(l)
                    if self.rank == 0:
                        log(f"Loss at iteration {it} of epoch {epoch}/{epochs} = {l:.10g}")
                    if on_event is not None:
                        on_event({"event": "loss", "iter": it, "epoch": epoch, "loss": l})
                else:
                    self.step(s, ln, lr, reg)
                print_flag = (bi == 0) if print_every <= 0 else (it % print_every == 0)
                if debug and print_flag and self.rank == 0:
                    self.sync_to(self.nn)
                    write_diff_gpu_cpu(self.nn, it, err_file, outdir)
                self.iter += 1
                stats.steps += 1
                stats.images += (ln // self.R) * self.R
            if xgmi_live or ag_live:
                self.assert_comm_ok()

        try:
            for epoch in range(epochs):
                # the recovery point: parameters (+ derived planes) and the step counter at the epoch start
                can_recover = (self.recover and self.recovered is None and (xgmi_live or ag_live))
                snap = (self._snapshot(), self.iter, stats.steps, stats.images, len(stats.losses)) \
                    if can_recover else None
                try:
                    run_epoch(epoch)
                except (KernelHandoffTimeout, CommFailure) as ex:
                    if not self._recover_epoch(ex, snap):
                        raise
                    stats.steps, stats.images = snap[2], snap[3]
                    del stats.losses[snap[4]:]
                    xgmi_live = self.xgmi is not None or self._xgmi_fused is not None
                    ag_live = self._allgather_live()
                    run_epoch(epoch)  # the same epoch again on the fallback path (a second failure raises)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            if xgmi_live and not self.replicas_agree():
                # the xGMI hand-off's ordering rests on write-through stores (csrc/comm/xgmi_allreduce.hip):
                # a stale peer read would leave the replicas different -- checked bitwise once per train()
                raise CommFailure(f"rank {self.rank}: replicas differ after xGMI data-parallel training")
            self.comm.barrier()
        finally:
            if own_file:
                err_file.close()
        stats.seconds = time.perf_counter() - t0
        self.sync_to(self.nn)
        return stats

    def sync_to(self, nn) -> None:
        W1, b1, W2, b2 = self.engine.get_params()
        nn.W[0][...] = W1
        nn.b[0][...] = b1
        nn.W[1][...] = W2
        nn.b[1][...] = b2

    def predict(self, x) -> np.ndarray:
        return self.engine.predict(x)


def parallel_train(nn, X, y, learning_rate: float, reg: float = 0.0, epochs: int = 15, batch_size: int = 800,
                   grad_check: bool = False, print_every: int = -1, debug: bool = False, comm=None, device=None,
                   dtype: str = "f32", backend: str = "hip", use_graphs: bool = True, shift: bool = True,
                   outdir: str = "Outputs", normalize: bool = False, path: str = "auto",
                   allreduce: str = "auto") -> TrainStats:
    """Reference-compatible entry point (inc/neural_network.h:45-48): trains ``nn`` in place."""
    tr = DataParallelTrainer(nn, comm=comm, device=device, dtype=dtype, batch_size=batch_size, backend=backend,
                             shift=shift, use_graphs=use_graphs, normalize=normalize, path=path,
                             allreduce=allreduce)
    tr.load(X, y)
    return tr.train(epochs, learning_rate, reg, print_every=max(0, print_every), debug=debug, outdir=outdir)
