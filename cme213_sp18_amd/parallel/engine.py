"""Device-resident MLP training engine (one per rank).

Replaces the reference's per-batch host<->device shuffle
(fpcode/neural_network.cpp:484-499: X, y and ALL weights uploaded every batch,
all gradients downloaded) and its ``device_cache`` of 18 separate cudaMallocs
(fpcode/inc/gpu_func.h:49-101) with:

* the WHOLE training set uploaded once per GPU in the GEMM dtype (54,000 x 784
  fp32 = 169 MB, a rounding error of 288 GB of HBM), so a batch is a pointer
  offset -- no scatter, no H2D copies;
* one flat parameter arena ``[W1|b1|W2|b2]`` and a gradient bucket with the same
  layout, so a single all-reduce and a single fused SGD kernel cover every
  parameter;
* activations ``a1, dZ1 [H][ld]``, ``D [C][ld]`` sized once for the per-rank
  batch.

Two interchangeable compute backends execute a step:
* ``"hip"``   -- the hand-written gfx950 kernels (csrc/mlp): 3 launches per step.
* ``"torch"`` -- the same math in plain PyTorch ops; the numerics reference for
  the kernels and the backend for CPU-only (gloo) data-parallel tests.
"""
from __future__ import annotations

import numpy as np
import torch

from .._native import DTYPE_CODES, hip

_ALIGN = 64  # elements; keeps every arena segment 256-byte aligned for f32


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def fragment_order_pixels(x: torch.Tensor) -> torch.Tensor:
    """[N][P] uint8 -> the forward's fragment-ordered copy (csrc/mlp/mma_tile.h ``xs_off``): sample tile s // 16,
    64-k pair k // 64, lane ((k % 64) // 16) * 16 + s % 16, byte k % 16; zero-padded to whole tiles and pairs."""
    n, p = x.shape
    ns, npair = _round_up(n, 16), (p + 63) // 64
    xp = torch.zeros(ns, npair * 64, dtype=torch.uint8, device=x.device)
    xp[:n, :p] = x
    return xp.view(ns // 16, 16, npair, 4, 16).permute(0, 2, 3, 1, 4).contiguous().view(-1)


def fragment_rows_to_rowmajor(buf: torch.Tensor, rows: int, cols: int, kblock: int = 64) -> torch.Tensor:
    """Inverse of the fp32 fragment orders -> a [rows][cols] view.  kblock 64: csrc/mlp/mma_tile.h ``w1s_off`` (row
    tile r // 16, 64-column pair c // 64, load i = (c % 16) // 4, lane ((c % 64) // 16) * 16 + r % 16, element c % 4);
    kblock 32: csrc/mlp/rega_gemm.h ``dzr_off`` (32-column stage c // 32, load h = (c % 8) // 4, lane
    ((c % 32) // 8) * 16 + r % 16, element c % 4)."""
    rt, nb = (rows + 15) // 16, (cols + kblock - 1) // kblock
    v = buf[: rt * 16 * nb * kblock].view(rt, nb, kblock // 16, 4, 16, 4)  # [row tile][block][load][lane grp][r][e]
    return v.permute(0, 4, 1, 3, 2, 5).reshape(rt * 16, nb * kblock)[:rows, :cols]


def param_dtype(dtype: str) -> torch.dtype:
    return torch.float64 if dtype == "f64" else torch.float32


def gemm_dtype(dtype: str) -> torch.dtype:
    return {"f32": torch.float32, "f64": torch.float64, "bf16": torch.bfloat16}[dtype]


class FlatLayout:
    """Offsets of W1, b1, W2, b2 inside the flat arena (each 64-element aligned), then one STATUS element:
    in the gradient bucket it is 0 for a trusted step and 1 when this rank's forward + head launch timed out
    (csrc/mlp/mlp_split.h SplitStepArgs::gstatus); the all-reduce sums it with the gradients and the SGD
    kernels apply nothing when it is non-zero.  The parameter arena's copy stays 0."""

    def __init__(self, P: int, H: int, C: int):
        self.P, self.H, self.C = P, H, C
        sizes = [H * P, H, C * H, C, 1]
        self.offsets = []
        o = 0
        for s in sizes:
            self.offsets.append(o)
            o += _round_up(s, _ALIGN)
        self.sizes = sizes
        self.total = o
        self.status = self.offsets[4]

    def views(self, flat: torch.Tensor):
        P, H, C = self.P, self.H, self.C
        o = self.offsets
        return (flat[o[0]:o[0] + H * P].view(H, P), flat[o[1]:o[1] + H], flat[o[2]:o[2] + C * H].view(C, H),
                flat[o[3]:o[3] + C])


PATHS = ("auto", "split3", "split1", "mfma")


def resolve_path(dtype: str, path: str = "auto") -> str:
    """Compute path for a dtype.

    * ``split3`` (f32 default): fp32 parameters, GEMMs on bf16 MFMA over an EXACT
      3-plane bf16 split of the fp32 operands (csrc/mlp/mlp_split.h); needs inputs
      that are exact in bf16 (raw 0..255 pixels).  2 kernels per step.
    * ``split1`` (bf16 default): the same kernels with single bf16 planes (mixed precision).
    * ``mfma``: plain f32 / f64 MFMA kernels (csrc/mlp/mlp_kernels.hip); the f64 parity
      path and the f32 path for non-integer (normalised) inputs.  3 kernels per step.
    """
    if path not in PATHS:
        raise ValueError(f"path must be one of {PATHS}")
    if path == "auto":
        return {"f32": "split3", "bf16": "split1", "f64": "mfma"}[dtype]
    if path.startswith("split") and dtype == "f64":
        raise ValueError("the split-bf16 path has fp32 parameters; use path='mfma' for f64")
    return path


class MlpEngine:
    def __init__(self, H=(784, 100, 10), dtype: str = "f32", max_cols: int = 800, device=None,
                 backend: str = "hip", shift: bool = True, feature_major_copy: bool = True, path: str = "auto"):
        if dtype not in DTYPE_CODES:
            raise ValueError(f"dtype must be one of {list(DTYPE_CODES)}")
        self.P, self.H, self.C = (int(h) for h in H)
        self.dtype = dtype
        self.path = resolve_path(dtype, path)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        if backend == "hip" and self.device.type != "cuda":
            raise RuntimeError("the 'hip' backend needs a GPU; use backend='torch' on CPU")
        self.backend = backend
        self.shift = bool(shift)
        self.pdt = param_dtype(dtype)
        self.layout = FlatLayout(self.P, self.H, self.C)
        dev = self.device
        self.params = torch.zeros(self.layout.total, dtype=self.pdt, device=dev)
        self.grads = torch.zeros(self.layout.total, dtype=self.pdt, device=dev)
        self.W1, self.b1, self.W2, self.b2 = self.layout.views(self.params)
        self.gW1, self.gb1, self.gW2, self.gb2 = self.layout.views(self.grads)
        self.status_index = self.layout.status  # the gradient bucket's status element (FlatLayout)
        self.X = None
        self.Xw = self.XTw = None  # wide-layer bf16 copies (load_dataset)
        self.XT = None
        self.Xs = None  # the pixels in the forward's fragment order (load_dataset)
        self.labels = None
        self._normalize = False
        self.xscale = 1.0
        # keep a second, feature-major copy of the dataset ([P][N]) so the dW1 GEMM
        # reads its B operand K-contiguous (16-byte loads); +1x dataset bytes, which
        # is nothing next to 288 GB of HBM.
        self.feature_major_copy = bool(feature_major_copy) or self.path.startswith("split")
        self._configure_path()
        self._alloc_acts(max_cols)
        self._step = None
        self._xgmi_fuse = None
        # H <= 128 split path: the forward + head launch in its all-gather form (every workgroup of the
        # launch must be resident at once; DataParallelTrainer turns it off when processes share a GPU)
        self.fh_allgather = True
        self.store_a1 = True
        # wide split3 layers: the in-place W1 update skips the W1-plane refresh when no forward reads the planes
        # (MlpStep.lazy_planes; they are re-split before one that does)
        # (measured at 784-4096-10 fp32: step 58.0 -> 55.2 us, profiles/wide_ag_ab_lazy_planes_r3.jsonl)
        self.lazy_planes = True
        self._ag_test_skip, self._ag_wait_us = -1, 50_000  # inject_handoff_timeout (tests); 50 ms default
        self.kpart = None  # split-K dW1 slabs (enable_splitk)

    def _configure_path(self):
        dev = self.device
        self.np = {"split3": 3, "split1": 1}.get(self.path, 0)
        if self.np:
            self.gdt = torch.bfloat16
            self.W1p = torch.zeros(self.np, self.H, self.P, dtype=torch.bfloat16, device=dev)
            self.W1g = self.W1  # the torch backend reads the (exact) fp32 master
        else:
            self.gdt = gemm_dtype(self.dtype)
            self.W1p = None
            self.W1g = (torch.zeros(self.H, self.P, dtype=torch.bfloat16, device=dev)
                        if self.dtype == "bf16" else self.W1)

    # ------------------------------------------------------------------ setup
    def _alloc_acts(self, max_cols: int):
        self.ld = _round_up(max(int(max_cols), 1), 16)
        dev, H, C, ld = self.device, self.H, self.C, self.ld
        self.a1 = torch.zeros(H, ld, dtype=self.pdt, device=dev)
        self.dZ1 = torch.zeros(H, ld, dtype=self.pdt, device=dev)
        self.D = torch.zeros(C, ld, dtype=self.pdt, device=dev)
        if self.np:
            self.dZ1p = torch.zeros(self.np, H, ld, dtype=torch.bfloat16, device=dev)
            self.dZ1g = self.dZ1
        else:
            self.dZ1p = None
            self.dZ1g = torch.zeros(H, ld, dtype=torch.bfloat16, device=dev) if self.dtype == "bf16" else self.dZ1
        # wide layers: scratch for the split-H z2 partial sums of the two-kernel head
        self.z2buf = self.dw2buf = None
        if self.backend == "hip" and H >= 512 and self.pdt == torch.float32:
            self.z2buf = torch.zeros(int(hip().head_big_scratch_floats(H, ld)), dtype=torch.float32, device=dev)
            # dW2 partials the wide head leaves per 32-column tile ([tile][16][H]) for the weight-gradient launch
            self.dw2buf = torch.zeros((ld + 31) // 32 * 16 * H, dtype=torch.float32, device=dev)
        elif self.backend == "hip" and self.np and H <= 128 and C <= 16:
            # ... and the H <= 128 all-gather forward + head (MlpStep.head_dw2: two 16-column partials per tile)
            self.dw2buf = torch.zeros((ld + 31) // 32 * 2 * 16 * H, dtype=torch.float32, device=dev)
        nblk = (ld + 15) // 16
        self.loss_buf = torch.zeros(max(nblk, 1), dtype=torch.float32, device=dev)
        # split path, H <= 128: forward GEMM + head in one launch (mlp_fwd1_head); one uint32
        # counter per 32-column a1 tile tells the last row-tile workgroup to run the head
        self.fh_counters = None
        self.ag_counters = self.ag_slabs = self.ag_err = self.ag_gran = self.W1s = self.dZ1s = None
        if self.backend == "hip" and self.np and H <= 128 and C <= 16:
            tiles = (ld + 31) // 32
            self.fh_counters = torch.zeros(tiles, dtype=torch.int32, device=dev)
            # all-gather form (mlp_fwd1_head_ag): monotonic uint64 tile counters (the launch epoch), z2 partial
            # granules {value, epoch} [tile][8 row tiles][16 classes][32 columns], and the timed-out-poll word
            self.ag_counters = torch.zeros(tiles * 32, dtype=torch.int64, device=dev)  # one 256-B line each
            self.ag_slabs = torch.zeros(tiles * 8 * 16 * 32, dtype=torch.int64, device=dev)
            self.ag_err = torch.zeros(1, dtype=torch.int32, device=dev)
            if self.np == 3:  # the forward's fragment-ordered fp32 copy of W1 (MlpStep.w1_swz)
                self.W1s = torch.zeros(int(hip().mlp_split_w1s_floats(H, self.P)), dtype=torch.float32, device=dev)
                # ... and dZ1 in the weight-gradient GEMM's fragment order (MlpStep.dz_swz)
                self.dZ1s = torch.zeros(int(hip().mlp_split_w1s_floats(H, ld)), dtype=torch.float32, device=dev)
        elif self.backend == "hip" and self.np and H >= 512 and C <= 16 and self.dw2buf is not None:
            # wide layers: the all-gather head fused into the forward launch (mlp_fwd1_wide_ag) uses one
            # monotonic counter per column tile -- a separate array per tiling (128 x 128 / 64 x 64) -- and
            # the timed-out-wait word
            tiles = (ld + 31) // 32
            if self.np == 3:  # fp32 dZ1 in the A-in-registers dW1 K loop's fragment order (MlpStep.dz_swz)
                self.dZ1s = torch.zeros((H + 15) // 16 * 16 * ((ld + 31) // 32 * 32), dtype=torch.float32, device=dev)
            self.ag_counters = torch.zeros(2 * tiles * 32, dtype=torch.int64, device=dev)
            self.ag_err = torch.zeros(1, dtype=torch.int32, device=dev)
            # its hand-off granules: 8-byte {value, epoch} z2 partials [H/64][16][ld] and D [16][ld] (tags only
            # grow, so the buffer is never re-zeroed)
            self.ag_gran = torch.zeros(((H + 63) // 64 * 16 + 16) * ld, dtype=torch.int64, device=dev)
        self._step = None

    def load_dataset(self, x, labels, normalize: bool = False):
        """Upload the training set once ([N][P] uint8 or float) and keep it resident.

        Split paths keep the RAW uint8 pixels (1 byte/element; widened to bf16
        exactly inside the GEMM kernels, normalisation folded into the epilogues
        as ``xscale``), plus a feature-major uint8 copy for the dW1 GEMM.  The
        mfma path stores the (optionally normalised) values in the GEMM dtype.
        """
        x = torch.as_tensor(np.ascontiguousarray(x) if isinstance(x, np.ndarray) else x)
        if x.ndim != 2 or x.shape[1] != self.P:
            raise ValueError(f"expected [N][{self.P}] samples, got {tuple(x.shape)}")
        xd = x.to(self.device)
        self._normalize = bool(normalize)
        if self.np:
            raw = xd.to(torch.float32)
            exact = bool(((raw == raw.round()) & (raw >= 0) & (raw <= 255)).all().item())
            if not exact:  # the split kernels need raw 0..255 pixels; fall back to the plain MFMA path
                self.path = "mfma"
                self._configure_path()
                self._alloc_acts(self.ld)
        if self.np:
            self.xscale = 1.0 / 255.0 if normalize else 1.0
            self.X = raw.to(torch.uint8).contiguous()
        else:
            self.xscale = 1.0
            xd = xd.to(torch.float64 if self.dtype == "f64" else torch.float32)
            if normalize:
                xd = xd / 255.0
            self.X = xd.to(self.gdt).contiguous()
        if self.feature_major_copy and self.np:
            # + an all-ones feature row: the dW1 GEMM's extra column is db1 (no separate bias reduction)
            self.XT = torch.cat([self.X.t(), torch.ones(1, self.X.shape[0], dtype=self.X.dtype, device=self.device)])
            self.XT = self.XT.contiguous()
        else:
            self.XT = self.X.t().contiguous() if self.feature_major_copy else None
        # wide layers on the hip backend: bf16 copies of both layouts for the direct-to-LDS GEMM engine
        # (csrc/mlp/glds_gemm.h streams operands global -> LDS unconverted; 2 B/pixel, ~170 MB for the
        # 54k-image training split -- nothing next to 288 GB of HBM)
        self.Xw = self.XTw = None
        # H <= 128 split3: the pixels again, in the forward's fragment order (MlpStep.x_swz; mma_tile.h xs_off):
        # [cdiv(N, 16)][cdiv(P, 64)][4 lane groups][16 samples][16 B], zero-padded -- a wave's 16-byte load
        # instruction reads 1 KB of contiguous memory instead of 16 rows x 64 B (~47 MB for 60k images)
        self.Xs = None
        if self.np == 3 and self.backend == "hip" and self.H <= 128 and self.XT is not None:
            self.Xs = fragment_order_pixels(self.X)
        if self.np and self.backend == "hip" and self.H >= 512 and self.XT is not None:
            self.Xw = self.X.to(torch.bfloat16).contiguous()
            self.XTw = self.XT.to(torch.bfloat16).contiguous()
        self.labels = torch.as_tensor(np.asarray(labels, dtype=np.int32)).to(self.device).contiguous()
        self.num_samples = int(self.X.shape[0])
        self._step = None
        self.refresh_shadow()

    def set_params(self, W1, b1, W2, b2):
        self.join()
        with torch.no_grad():
            for dst, src in ((self.W1, W1), (self.b1, b1), (self.W2, W2), (self.b2, b2)):
                dst.copy_(torch.as_tensor(np.asarray(src)).to(dst.dtype))
            self.refresh_shadow()

    def dz1(self) -> torch.Tensor:
        """The last step's dZ1 as [H][ld] row-major.  A whole hip step with fp32 dZ1 leaves it only in the
        weight-gradient GEMM's fragment order (MlpStep.dz_swz, csrc/mlp/mma_tile.h w1s_off over [H][ld]); this view
        undoes that order (diagnostics and tests; the training step never reads dZ1 back)."""
        st = self._step
        if self.backend != "hip" or st is None or not st.dz_left_swz:
            return self.dZ1
        return fragment_rows_to_rowmajor(self.dZ1s, self.H, self.ld, 64 if st.dz_left_swz == 1 else 32)

    def _w1_written(self) -> None:
        """W1 changed outside the step's own in-place update: the forward's fragment-ordered copy (MlpStep.w1_swz)
        is rebuilt before the next forward that reads it."""
        if self._step is not None:
            self._step.swz_stale = True

    def refresh_shadow(self):
        """Re-derive the low-precision copies of W1 (bf16 shadow or bf16 planes)."""
        self.join()
        self._w1_written()
        with torch.no_grad():
            if self.np:
                if self.backend == "hip":
                    hip().split_planes(self.W1.data_ptr(), self.W1p.data_ptr(), self.H * self.P, self.np,
                                       torch.cuda.current_stream(self.device).cuda_stream)
                else:
                    r = self.W1.clone()
                    for p in range(self.np):
                        self.W1p[p] = r.to(torch.bfloat16)
                        r -= self.W1p[p].to(torch.float32)
            elif self.dtype == "bf16":
                self.W1g.copy_(self.W1.to(torch.bfloat16))

    def set_fh_allgather(self, on: bool) -> None:
        self.fh_allgather = bool(on)
        if self._step is not None:
            self._step.fh_allgather = int(self.fh_allgather)

    def enable_splitk(self, max_split: int = 8) -> None:
        """Let the wide weight-gradient launch split K (the batch) over up to ``max_split`` slices when its output
        tiles alone cannot fill the chip and K is long -- the tensor-parallel shard at a large global batch
        (784-4096-10 at global batch 6400 on 8 GPUs: 512 x 785 outputs, K = 6400).  Allocates the fp32 partial
        slabs [max_split][H][P + 1]; a second kernel sums them in slab order and applies the update."""
        if self.backend != "hip" or not self.np or max_split < 2:
            return
        self.kpart = torch.zeros(int(max_split) * self.H * (self.P + 1), dtype=torch.float32, device=self.device)
        self._step = None

    def set_store_a1(self, on: bool) -> None:
        """Split layers with the head fused into the forward launch: False skips the a1 store whenever that launch
        also leaves the dW2 partials (no kernel of the training step reads a1 then: dZ1 and the partials come out
        of the same launch).  Wide layers: always; H <= 128: from n = 768 columns (MlpStep.head_dw2 auto), where
        the weight-gradient launch's dW2 GEMM over the whole batch was that launch's critical path
        (bench/stamps_roles.py: roles end 5.99 -> 3.74 us at n = 800; below, the partials cost the forward more
        than they save -- profiles/r5/)."""
        self.store_a1 = bool(on)
        if self._step is not None:
            self._step.store_a1 = int(self.store_a1)

    def w1_planes_maintained(self) -> bool:
        """True when the W1 bf16 planes track the fp32 master after every update.  Below H = 512 the split3
        forward kernels read fp32 W1 and split it in registers, so the update stops refreshing the planes
        (csrc/mlp/mlp_split.hip mlp_split_w1_planes_read); at H = 4096 the 128 x 128 forward does too, and with
        lazy_planes the in-place update leaves them stale until a forward that reads them (MlpStep.planes_stale).
        refresh_w1_planes() rebuilds them on demand."""
        if not (self.np and self.backend == "hip"):
            return False
        s = self._hip_step()
        return bool(s.w1_planes_read()) and not s.lazy_planes_apply()

    def refresh_w1_planes(self) -> None:
        """Rebuild the W1 planes from the fp32 master (exact split3 / rounded split1)."""
        if self.np and self.backend == "hip":
            hip().split_planes(self.W1.data_ptr(), self.W1p.data_ptr(), self.W1.numel(), self.np,
                               torch.cuda.current_stream(self.device).cuda_stream)
            if self._step is not None:
                self._step.planes_stale = False

    def inject_handoff_timeout(self, row_tile: int = 0, wait_us: int = 2000) -> None:
        """TEST HOOK: from the next step on, row tile ``row_tile`` of column tile 0 withholds its hand-off
        granules in every all-gather forward + head launch, so that tile's wait really times out (after
        ``wait_us`` microseconds of wall time; the production bound is 50 ms).  ``row_tile=-1`` turns the
        withholding off (the bound stays).  A timed-out launch sets the sticky error word: this engine then
        applies no further update (kernel_error(), KernelHandoffTimeout) -- make a new engine afterwards."""
        self._ag_test_skip, self._ag_wait_us = int(row_tile), int(wait_us)
        if self._step is not None:
            self._step.ag_test_skip, self._step.ag_wait_us = self._ag_test_skip, self._ag_wait_us

    def kernel_error(self) -> bool:
        """True if a forward + head launch's wait for the workgroups of its column tile timed out (the
        all-gather form; its outputs were then not trusted).  Reads a device word: synchronises."""
        return self.ag_err is not None and bool(self.ag_err.item())

    def join(self):
        """Kept for API stability: every kernel of a step runs on the caller's stream, nothing to join."""

    def get_params(self):
        """Host float64 copies (W1, b1, W2, b2)."""
        self.join()
        return tuple(t.detach().to("cpu", torch.float64).numpy().copy()
                     for t in (self.W1, self.b1, self.W2, self.b2))

    # -------------------------------------------------------------- one step
    def set_lazy_planes(self, on: bool) -> None:
        self.lazy_planes = bool(on)
        if self._step is not None:
            self._step.lazy_planes = int(self.lazy_planes)

    def mark_planes_stale(self) -> None:
        """W1 / the W1 planes were overwritten from outside the step (a snapshot restore): the next forward that
        reads the planes re-splits W1 first (MlpStep.lazy_planes: the wide in-place update skips the refresh)."""
        if self._step is not None and self.W1p is not None:
            self._step.planes_stale = True
        self._w1_written()

    def _hip_step(self):
        if self._step is None:
            m = hip()
            s = m.MlpStep()
            loaded = self.X is not None
            ptr = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
            b = dict(dt=DTYPE_CODES[self.dtype], P=self.P, H=self.H, C=self.C, ld=self.ld,
                     X=ptr(self.X), labels=ptr(self.labels), XT=ptr(self.XT), Xw=ptr(self.Xw), XTw=ptr(self.XTw),
                     N=self.num_samples if loaded else 0,
                     W1=ptr(self.W1), b1=ptr(self.b1), W2=ptr(self.W2), b2=ptr(self.b2), W1g=ptr(self.W1g),
                     gW1=ptr(self.gW1), gb1=ptr(self.gb1), gW2=ptr(self.gW2), gb2=ptr(self.gb2),
                     gstatus=self.grads[self.status_index:].data_ptr(),
                     a1=ptr(self.a1), D=ptr(self.D), dZ1=ptr(self.dZ1), dZ1g=ptr(self.dZ1g), loss=ptr(self.loss_buf),
                     act=1, z2p=ptr(self.z2buf))
            if self.np:
                b.update(split=1, xscale=float(self.xscale), npw=self.np, npz=self.np, W1p=ptr(self.W1p),
                         dZ1p=ptr(self.dZ1p))
            if self.fh_counters is not None:
                b.update(fh_counters=ptr(self.fh_counters), fh_tiles=int(self.fh_counters.numel()),
                         ag_counters=ptr(self.ag_counters), ag_slabs=ptr(self.ag_slabs),
                         w1s=ptr(self.W1s), xs=ptr(self.Xs), dz1s=ptr(self.dZ1s))
            elif self.ag_gran is not None:  # the wide fused head
                b.update(fh_tiles=int(self.ag_counters.numel()) // 64,  # [2 tilings][tiles][32]
                         ag_gran=ptr(self.ag_gran), ag_gran_count=int(self.ag_gran.numel()),
                         ag_counters=ptr(self.ag_counters), dz1s=ptr(self.dZ1s))
            if self.kpart is not None:
                b.update(kpart=ptr(self.kpart), kpart_cap=int(self.kpart.numel()))
            bias_col = bool(self.np and self.XT is not None and self.XT.shape[0] == self.P + 1)
            b.update(bias_col=int(bias_col))
            s.bind(b)
            s.shift = int(self.shift)
            s.dw2p = ptr(self.dw2buf)
            if self.ag_err is not None and (self.fh_counters is not None or self.ag_gran is not None):
                s.ag_err = self.ag_err.data_ptr()
                s.fh_allgather = int(self.fh_allgather)
            if self.np:
                # a new step cannot know whether an earlier one left the planes stale: re-split once
                s.planes_stale = True
                s.lazy_planes = int(self.lazy_planes)
            s.store_a1 = int(self.store_a1)
            s.ag_test_skip, s.ag_wait_us = self._ag_test_skip, self._ag_wait_us
            if self._xgmi_fuse is not None and bias_col:
                s.set_xgmi(*self._xgmi_fuse)
            self._step = s
        return self._step

    # ------------------------------------------------ xGMI all-reduce fused into the wgrad launch
    def fused_allreduce_slots(self) -> int:
        """Flag slots (one per wgrad workgroup tile) the fused data-parallel step needs; 0 when this
        engine cannot run it (split path, H <= 128, all-ones XT feature, no head partials)."""
        bias_feature = (self.XT.shape[0] == self.P + 1 if self.XT is not None   # loaded, or will be
                        else self.feature_major_copy)
        if not (self.backend == "hip" and self.np and self.H <= 128 and self.device.type == "cuda"
                and bias_feature):
            return 0
        return max(0, int(hip().mlp_split_fused_tiles(self.P, self.H, 1 << 30)))

    def attach_xgmi(self, bucket, push: bool = False) -> None:
        """Bind an open XgmiBucket (created with flag_slots >= fused_allreduce_slots()) to the step;
        ``None`` detaches.  run(..., sgd=2) then all-reduces and applies SGD inside the wgrad launch: the one-shot
        pull (every rank reads every peer's tile), or with ``push`` the owner-tile form (XgmiFuse::push: tile t
        reduced and applied by rank t % world, pushed both ways as tagged granules; the bucket needs
        slab_tiles >= fused_allreduce_slots())."""
        if bucket is None:
            self._xgmi_fuse = None
            if self._step is not None:
                self._step.set_xgmi(0, 0, 0, 0, 0)
            return
        o = self.layout.offsets
        self._xgmi_fuse = (int(bucket.c.desc_address), int(bucket.c.nblocks), int(o[1]), int(o[2]), int(o[3]),
                           int(bool(push)))
        self._hip_step().set_xgmi(*self._xgmi_fuse)

    def run(self, off: int, n: int, scale: float, reg: float, lr: float, sgd, with_loss: bool = False,
            parts: int = 3, pf_next: int = -1):
        """Forward + backward on samples [off, off+n).  sgd=True: update params in
        place; False: write pre-scaled gradients into ``self.grads``; 2: all-reduce over the attached
        xGMI bucket and update inside the wgrad launch (attach_xgmi).  parts (hip backend): bit0 forward +
        head, bit1 weight gradients / update -- the per-phase profiler runs the two halves separately.
        pf_next >= 0: the next step's first sample, whose pixels this step's prefetch workgroups pull into L2."""
        if self.X is None:
            raise RuntimeError("load_dataset() first")
        if n > self.ld:
            raise ValueError(f"batch slice {n} exceeds activation capacity {self.ld}")
        if off < 0 or off + n > self.num_samples:
            raise IndexError("batch slice outside the resident dataset")
        if self.backend == "hip":
            st = self._hip_step()
            st.run(int(off), int(n), float(scale), float(reg), float(lr), 2 if sgd == 2 else int(bool(sgd)),
                   int(bool(with_loss)),
                   torch.cuda.current_stream(self.device).cuda_stream, int(parts), int(pf_next))
        elif parts & 1:  # the torch backend always runs the whole step
            self._torch_step(off, n, scale, reg, lr, sgd, with_loss)

    def run_forward_head(self, off: int, n: int, scale: float, with_loss: bool = False):
        """Forward + head only (a1, D, dZ1 and its planes); the weight gradients follow via run_wgrad."""
        self._hip_step().run(int(off), int(n), float(scale), 0.0, 0.0, 0, int(bool(with_loss)),
                             torch.cuda.current_stream(self.device).cuda_stream, 1)

    def run_wgrad(self, off: int, n: int, scale: float, reg: float, parts: int, row0: int = 0, rows: int = -1):
        """Gradient pieces into ``self.grads`` (split paths): parts bit0 = dW1 rows [row0, row0+rows),
        bit1 = dW2 + bias gradients."""
        self._hip_step().run_wgrad(int(off), int(n), float(scale), float(reg), 0.0, 0, int(parts), int(row0),
                                   int(rows), torch.cuda.current_stream(self.device).cuda_stream)

    @property
    def supports_bucketed_wgrad(self) -> bool:
        return self.backend == "hip" and bool(self.np)

    def _torch_step(self, off, n, scale, reg, lr, sgd, with_loss):
        """Same math as the HIP step in PyTorch ops (param dtype accumulation)."""
        with torch.no_grad():
            Xb = self.X[off:off + n].to(self.pdt) * self.xscale
            # the weights the kernels actually multiply: sum of the bf16 planes (== W1 for split3)
            W1g = self.W1p.to(self.pdt).sum(0) if self.np else self.W1g.to(self.pdt)
            z1 = Xb @ W1g.t() + self.b1
            a1 = torch.sigmoid(z1)
            z2 = a1 @ self.W2.t() + self.b2
            if self.shift:
                z2 = z2 - z2.max(dim=1, keepdim=True).values
            e = torch.exp(z2)
            p = e / e.sum(dim=1, keepdim=True)
            lab = self.labels[off:off + n].long()
            if with_loss:
                self.loss_buf.zero_()
                self.loss_buf[0] = -torch.log(p[torch.arange(n, device=p.device), lab]).sum().float()
            onehot = torch.zeros_like(p)
            onehot[torch.arange(n, device=p.device), lab] = 1.0
            D = (p - onehot) * scale
            dZ1 = (D @ self.W2) * a1 * (1 - a1)
            self.a1[:, :n] = a1.t()
            self.D[:, :n] = D.t()
            self.dZ1[:, :n] = dZ1.t()
            gW1 = dZ1.t() @ Xb + reg * self.W1
            gW2 = D.t() @ a1 + reg * self.W2
            gb1 = dZ1.sum(0)
            gb2 = D.sum(0)
            if sgd:
                self.W1.sub_(lr * gW1)
                self.W2.sub_(lr * gW2)
                self.b1.sub_(lr * gb1)
                self.b2.sub_(lr * gb2)
                self.refresh_shadow()
            else:
                self.gW1.copy_(gW1)
                self.gW2.copy_(gW2)
                self.gb1.copy_(gb1)
                self.gb2.copy_(gb2)

    def sgd(self, lr: float):
        """params -= lr * grads over the whole flat arena (one fused kernel)."""
        self.join()
        self._w1_written()
        if self.backend == "hip" and self.np:
            hip().split_sgd(self.params.data_ptr(), self.grads.data_ptr(), self.layout.total, float(lr),
                            self.W1p.data_ptr(), self.H * self.P, self.np,
                            torch.cuda.current_stream(self.device).cuda_stream,
                            self.grads[self.status_index:].data_ptr())
        elif self.backend == "hip":
            stream = torch.cuda.current_stream(self.device).cuda_stream
            shadow = self.W1g.data_ptr() if self.dtype == "bf16" else 0
            hip().sgd_flat(DTYPE_CODES[self.dtype], self.params.data_ptr(), self.grads.data_ptr(),
                           self.layout.total, float(lr), shadow, self.H * self.P if shadow else 0, stream)
        else:
            with torch.no_grad():
                self.params.sub_(lr * self.grads)
                self.refresh_shadow()

    def reg_only_grads(self, reg: float):
        """Gradient of an EMPTY shard: reg*W for weights, 0 for biases (the
        reference's in_proc == 0 case, neural_network.cpp:458)."""
        with torch.no_grad():
            self.grads.zero_()
            self.gW1.copy_(reg * self.W1)
            self.gW2.copy_(reg * self.W2)

    def loss_sum(self) -> float:
        """Sum of -log(yhat[label]) over the last step's local samples (if requested)."""
        return float(self.loss_buf.double().sum().item())

    # --------------------------------------------------------------- predict
    def predict(self, x, chunk: int | None = None) -> np.ndarray:
        """argmax labels for samples ``x`` ([N][P], host or device); GPU forward."""
        self.join()
        xt = torch.as_tensor(np.ascontiguousarray(x) if isinstance(x, np.ndarray) else x)
        n = int(xt.shape[0])
        out = torch.empty(n, dtype=torch.int32, device=self.device)
        chunk = chunk or max(self.ld, 4096)
        a1 = torch.empty(self.H, _round_up(chunk, 16), dtype=self.pdt, device=self.device)
        if self.backend == "hip":
            self._hip_step()
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            if self.np:  # raw uint8 pixels, scaled inside the kernel
                raw = xt[s:e].to(self.device).to(torch.float32)
                if not bool(((raw == raw.round()) & (raw >= 0) & (raw <= 255)).all().item()):
                    raise ValueError("split-path predict needs raw 0..255 pixel inputs")
                xb = raw.to(torch.uint8).contiguous()
            else:
                xb = xt[s:e].to(self.device).to(torch.float64 if self.dtype == "f64" else torch.float32)
                if self._normalize:
                    xb = xb / 255.0
                xb = xb.to(self.gdt).contiguous()
            if self.backend == "hip" and self.np:
                self._hip_step().predict(xb.data_ptr(), e - s, a1.data_ptr(), a1.shape[1], out[s:e].data_ptr(),
                                         torch.cuda.current_stream(self.device).cuda_stream)
            elif self.backend == "hip":
                m = hip()
                st = torch.cuda.current_stream(self.device).cuda_stream
                dt = DTYPE_CODES[self.dtype]
                m.mlp_forward1(dt, self.W1g.data_ptr(), self.b1.data_ptr(), xb.data_ptr(), self.P, self.H, e - s,
                               a1.data_ptr(), a1.shape[1], 1, st)
                m.mlp_head(dt if self.dtype != "bf16" else 0, 1, a1.data_ptr(), a1.shape[1], self.W2.data_ptr(),
                           self.b2.data_ptr(), H=self.H, C=self.C, n=e - s, pred=out[s:e].data_ptr(), stream=st)
            else:
                with torch.no_grad():
                    W1e = self.W1p.to(self.pdt).sum(0) if self.np else self.W1g.to(self.pdt)
                    z1 = (xb.to(self.pdt) * self.xscale) @ W1e.t() + self.b1
                    z2 = torch.sigmoid(z1) @ self.W2.t() + self.b2
                    out[s:e] = z2.argmax(dim=1).to(torch.int32)
        return out.cpu().numpy()
