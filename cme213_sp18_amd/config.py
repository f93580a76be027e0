"""Training configuration: the reference's getopt flags, grade presets and the
BASELINE configs as named presets.

Reference flags (fpcode/main.cpp:58-109): ``-n num_neuron -r reg -l lr -e epochs
-b batch -g grade -p print_every -s (run sequential) -d (debug)``; grade presets
1-3 override them (fpcode/main.cpp:113-152) and grade 4 runs the GEMM benchmark
(fpcode/main.cpp:154-161).
"""
from __future__ import annotations

import argparse
import dataclasses


@dataclasses.dataclass
class TrainConfig:
    num_neuron: int = 1000      # -n  (main.cpp:63)
    reg: float = 1e-4           # -r
    learning_rate: float = 1e-3  # -l
    num_epochs: int = 20        # -e
    batch_size: int = 800       # -b
    grade: int = 0              # -g
    print_every: int = 0        # -p
    run_seq: bool = False       # -s
    debug: bool = False         # -d
    # --- MI355X engine options (not in the reference)
    dtype: str = "f32"          # f32 | f64 | bf16
    path: str = "auto"          # auto | split3 | split1 | mfma
    backend: str = "hip"        # hip (gfx950 kernels) | torch (plain PyTorch ops; CPU capable)
    data: str = "synthetic"     # synthetic | mnist
    data_dir: str = "data"
    normalize: bool = False     # reference feeds raw 0..255 pixels (mnist.cpp:26-31)
    num_train: int = 60000
    num_test: int = 10000
    seed: int = 0
    outdir: str = "Outputs"
    ckpt_dir: str = ""
    resume: str = ""
    use_graphs: bool = True
    softmax_shift: bool = True
    ckpt_precision: int = 12
    allreduce: str = "auto"     # auto | xgmi (one-shot peer kernel, SGD fused) | xgmi2 (two-shot, sharded SGD) | rccl
    comm_timeout: float = 300.0  # seconds before a stuck collective fails the job
    fault_inject: str = ""      # "rank:step" -- raise on that rank at that step (failure-detection test hook)
    log_json: str = ""          # rank-0 JSON-lines event log
    ckpt_every: int = 0         # epochs between checkpoints (needs --ckpt-dir); 0 = only at the end
    profile: bool = False       # per-phase event timing + roctx ranges (eager steps), summary at the end
    overlap_chunks: int = 0     # RCCL path: dW1 all-reduce row chunks overlapped with the backward (0 = auto)
    parallel: str = "dp"        # dp (reference scheme) | tp (hidden-dimension tensor parallel, wide layers)
    gpus: int = 0               # ranks (one per GPU); 0 = WORLD_SIZE of the launcher, else 1.  N > 1 without a
                                # launcher: the CLI starts the N ranks itself (parallel/launcher.self_launch)

    @property
    def H(self):
        return [784, self.num_neuron, 10]


# fpcode/main.cpp:113-152 -- "DO NOT change the following parameters"
GRADE_PRESETS = {
    1: dict(reg=1e-4, learning_rate=0.001, num_epochs=40, batch_size=800, num_neuron=100, run_seq=True,
            debug=True, print_every=0),
    2: dict(reg=1e-4, learning_rate=0.01, num_epochs=10, batch_size=800, num_neuron=100, run_seq=True,
            debug=True, print_every=0),
    3: dict(reg=1e-4, learning_rate=0.025, num_epochs=1, batch_size=800, num_neuron=100, run_seq=True,
            debug=True, print_every=1),
}

# BASELINE.json configs
NAMED_PRESETS = {
    "cpu_plumbing": dict(num_neuron=100, batch_size=800, backend="torch", dtype="f64", run_seq=True),
    "1gpu_fp32": dict(num_neuron=100, batch_size=800, dtype="f32"),
    "4gpu_rccl": dict(num_neuron=100, batch_size=800, dtype="f32", allreduce="rccl"),
    "8gpu_wide": dict(num_neuron=4096, batch_size=6400, dtype="f32"),
    "8gpu_bf16": dict(num_neuron=1024, batch_size=800, dtype="bf16"),
}


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m cme213_sp18_amd.train",
                                 description="2-layer MLP training on MI355X (CME213 final-project CLI)")
    ap.add_argument("-n", "--hidden", dest="num_neuron", type=int)
    ap.add_argument("-r", dest="reg", type=float)
    ap.add_argument("-l", dest="learning_rate", type=float)
    ap.add_argument("-e", dest="num_epochs", type=int)
    ap.add_argument("-b", dest="batch_size", type=int)
    ap.add_argument("-g", dest="grade", type=int)
    ap.add_argument("-p", dest="print_every", type=int)
    ap.add_argument("-s", dest="run_seq", action="store_true", default=None)
    ap.add_argument("-d", dest="debug", action="store_true", default=None)
    ap.add_argument("--preset", choices=sorted(NAMED_PRESETS))
    ap.add_argument("--dtype", choices=["f32", "f64", "bf16"])
    ap.add_argument("--path", choices=["auto", "split3", "split1", "mfma"])
    ap.add_argument("--backend", choices=["hip", "torch"])
    ap.add_argument("--data", choices=["synthetic", "mnist"])
    ap.add_argument("--data-dir")
    ap.add_argument("--normalize", action="store_true", default=None)
    ap.add_argument("--num-train", type=int)
    ap.add_argument("--num-test", type=int)
    ap.add_argument("--seed", type=int)
    ap.add_argument("--outdir")
    ap.add_argument("--ckpt-dir")
    ap.add_argument("--resume")
    ap.add_argument("--no-graphs", dest="use_graphs", action="store_false", default=None)
    ap.add_argument("--no-softmax-shift", dest="softmax_shift", action="store_false", default=None)
    ap.add_argument("--ckpt-precision", type=int)
    ap.add_argument("--allreduce", choices=["auto", "xgmi", "xgmi2", "rccl", "host"])
    ap.add_argument("--comm-timeout", type=float)
    ap.add_argument("--fault-inject", help="rank:step")
    ap.add_argument("--log-json")
    ap.add_argument("--ckpt-every", type=int)
    ap.add_argument("--profile", action="store_true", default=None,
                    help="time forward+head / weight gradients / all-reduce / SGD per step (eager) and emit roctx "
                         "ranges for rocprofv3 --marker-trace")
    ap.add_argument("--parallel", choices=["dp", "tp"],
                    help="dp: data parallel (default); tp: shard the hidden layer over the ranks (one z2 all-reduce "
                         "per step, every rank runs the whole global batch)")
    ap.add_argument("--gpus", type=int,
                    help="number of ranks, one per GPU (the reference's mpirun -np N); started here when no "
                         "launcher started this process")
    ap.add_argument("--overlap-chunks", type=int,
                    help="RCCL path: number of dW1 row chunks all-reduced while the backward runs (0 = auto)")
    return ap


def parse_config(argv=None) -> TrainConfig:
    a = build_parser().parse_args(argv)
    cfg = TrainConfig()
    explicit = {k: v for k, v in vars(a).items() if v is not None and k != "preset"}
    if a.preset:
        for k, v in NAMED_PRESETS[a.preset].items():
            setattr(cfg, k, v)
    for k, v in explicit.items():
        setattr(cfg, k.replace("-", "_"), v)
    if cfg.gpus <= 0:
        import os

        cfg.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if cfg.grade in GRADE_PRESETS:
        for k, v in GRADE_PRESETS[cfg.grade].items():
            setattr(cfg, k, v)
        # the grading gate is fp64-tight (max-norm rel <= 1e-7, utils/tests.cpp:39): run the
        # fp64 engine unless a dtype was requested explicitly
        if "dtype" not in explicit:
            cfg.dtype = "f64"
    return cfg
