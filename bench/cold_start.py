#!/usr/bin/env python3
"""Where the driver's short timed run loses time on a fresh process: bench.py's own preparation (trainer, W
warm-up steps), then ``--chunks`` timed runs of ``--chunk-steps`` steps each, bracketed exactly like bench.py's
timed region, each followed by a shader-clock probe (bench/micro/clockprobe.hip: s_memtime cycles over
s_memrealtime ticks on every CU).  Chunk 0 is the driver's measurement; the later chunks show how fast the same
process runs once whatever was cold has warmed up, and the clock column whether that something is the GPU clock.

    python bench/cold_start.py [--chunks 30] [--chunk-steps 20] [--warmup 5] [--prespin-ms 0]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=30)
    ap.add_argument("--chunk-steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prespin-ms", type=float, default=0.0,
                    help="spin every CU for this long (clock probe kernel) before the warm-up steps")
    ap.add_argument("--tag", default="")
    a = ap.parse_args(argv)
    t_start = time.perf_counter()
    import torch

    import bench as B
    from cme213_sp18_amd.parallel.launcher import init_distributed

    lib = ctypes.CDLL(os.path.join(ROOT, "bench", "micro", "libclockprobe.so"))
    lib.clock_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    comm, device = init_distributed()
    args = B.parse(["--steps", str(a.chunk_steps), "--warmup", str(a.warmup)])
    ctx = B.Ctx(args, comm, device, {})
    wgs = 256
    buf = torch.zeros(2 * wgs, dtype=torch.int64, device=device)

    def clock(spin_us=5):
        lib.clock_probe(torch.cuda.current_stream(device).cuda_stream, buf.data_ptr(), wgs, spin_us)
        torch.cuda.synchronize(device)
        v = buf.view(wgs, 2).double().cpu()
        mhz = 100.0 * v[:, 0] / v[:, 1].clamp_min(1)
        return round(float(mhz.median()), 1), round(float(mhz.min()), 1)

    rows = []
    c0 = clock()
    if a.prespin_ms > 0:
        lib.clock_probe(torch.cuda.current_stream(device).cuda_stream, buf.data_ptr(), wgs, int(a.prespin_ms * 1000))
        torch.cuda.synchronize(device)
    c1 = clock()
    tr, full = B.dp_prepare(ctx, 800, "auto", a.warmup)
    c2 = clock()
    print(json.dumps({"tag": a.tag, "phase": "setup", "since_start_s": round(time.perf_counter() - t_start, 2),
                      "mhz_first": c0, "mhz_after_prespin": c1, "mhz_after_warmup": c2,
                      "prespin_ms": a.prespin_ms}), flush=True)
    for i in range(a.chunks):
        runners = [tr.plan_runner(p, B.LR, B.REG) for p in B.plans_for(full, a.chunk_steps)]
        dt = B.timed(ctx, runners)
        mhz = clock()
        rows.append(1e6 * dt / a.chunk_steps)
        print(json.dumps({"tag": a.tag, "chunk": i, "us_per_step": round(rows[-1], 3), "mhz_after": mhz}), flush=True)
    print(json.dumps({"tag": a.tag, "summary": True, "first": round(rows[0], 3),
                      "median_rest": round(sorted(rows[1:])[len(rows[1:]) // 2], 3) if len(rows) > 1 else None}),
          flush=True)
    tr.close()


if __name__ == "__main__":
    main()
