#!/usr/bin/env python3
"""Where the driver form's fixed cost goes: bench.py's timed region (barrier + synchronize, K native-loop steps,
synchronize) repeated, with the host's clock (CLOCK_MONOTONIC, ns) recorded at the timer start and stop.  Run under
`rocprofv3 --kernel-trace --output-format csv` (same clock domain) and analyse with --analyse: per timed region, the
host-start -> first-kernel-start gap, the last-kernel-end -> host-stop gap, the kernels' own durations step by step
(are the first steps of a cold region slower?) and the gaps between them.  Diagnostic.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o gap -- python3 bench/driver_gap.py --out OUT/regions.json
    python3 bench/driver_gap.py --analyse OUT
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a):
    import torch

    import bench
    from cme213_sp18_amd.parallel.comm import NullComm

    args = bench.parse(["--gpus", "1", "--steps", str(a.steps), "--warmup", "5"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = bench.Ctx(args, NullComm(), dev, {})
    side = torch.cuda.Stream(dev) if a.stream else None
    if side is not None:  # everything (warm-up included) on a created stream instead of the default one
        torch.cuda.set_stream(side)
    tr, full = bench.dp_prepare(ctx, 800, "auto", args.warmup)
    regions = []
    for r in range(a.reps):
        plans = bench.plans_for(full, a.steps)
        runners = [tr.plan_runner(p, bench.LR, bench.REG) for p in plans]
        ctx.barrier_sync()
        if a.idle_us:
            time.sleep(a.idle_us * 1e-6)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.monotonic_ns()
        if a.events:
            e0.record()
        for fn in runners:
            fn()
        if a.events:
            e1.record()
        te = time.monotonic_ns()
        ctx.sync()
        t1 = time.monotonic_ns()
        regions.append({"t0": t0, "t1": t1, "us_per_step": (t1 - t0) / 1e3 / a.steps,
                        "host_enqueue_us": (te - t0) / 1e3,
                        "event_us": e0.elapsed_time(e1) * 1e3 if a.events else None})
        time.sleep(0.01)
    tr.close()
    with open(a.out, "w") as f:
        json.dump({"steps": a.steps, "regions": regions}, f)
    print(json.dumps({"us_per_step": [round(x["us_per_step"], 3) for x in regions],
                      "host_enqueue_us": [round(x["host_enqueue_us"], 1) for x in regions],
                      "event_us": [round(x["event_us"], 1) if x["event_us"] else None for x in regions]}))


def analyse(d):
    """Per timed region: host start -> first kernel start, last kernel end -> host stop, the kernels' durations and
    gaps (two-launch form: F/W per step; the XCD-local pipeline: ONE kernel per region), and -- with
    ``--hip-runtime-trace`` in the rocprofv3 run -- every HIP API call inside the region (start / end relative to the
    timer start): which part of the first-kernel gap is the host's launch path and which the device's."""
    import csv

    reg = json.load(open(glob.glob(os.path.join(d, "**", "regions.json"), recursive=True)[0]))
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = []
    for row in csv.DictReader(open(trace)):
        name = row.get("Kernel_Name", "")
        if "fwd1_head" in name or "wgrad" in name or "xstep_kernel" in name:
            ks.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]),
                       "X" if "xstep" in name else "F" if "fwd1" in name else "W"))
    ks.sort()
    api = []
    for f in glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            api.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row.get("Function", row.get("Name", ""))))
    api.sort()
    K = reg["steps"]
    for r in reg["regions"]:
        inr = [k for k in ks if r["t0"] <= k[0] <= r["t1"]]
        calls = [(round((a0 - r["t0"]) / 1e3, 2), round((a1 - r["t0"]) / 1e3, 2), nm) for a0, a1, nm in api
                 if r["t0"] <= a0 <= r["t1"]]
        if not inr or (inr[0][2] != "X" and len(inr) != 2 * K):
            print(json.dumps({"warning": f"{len(inr)} kernels in region, expected {2 * K} (or one xstep launch)"}))
            continue
        first, last = inr[0], inr[-1]
        dur = [round((k[1] - k[0]) / 1e3, 2) for k in inr]
        gaps = [round((inr[i + 1][0] - inr[i][1]) / 1e3, 2) for i in range(len(inr) - 1)]
        rec = {
            "region_us": round((r["t1"] - r["t0"]) / 1e3, 2),
            "host_start_to_first_kernel_us": round((first[0] - r["t0"]) / 1e3, 2),
            "last_kernel_end_to_host_stop_us": round((r["t1"] - last[1]) / 1e3, 2),
            "kernels_span_us": round((last[1] - first[0]) / 1e3, 2),
            "host_enqueue_us": round(r.get("host_enqueue_us", 0.0), 2),
        }
        if first[2] == "X":
            rec.update(kernels=len(inr), xstep_kernel_us=dur, xstep_us_per_step=round(dur[0] / K, 3))
        else:
            rec.update({"fwd_us_first3": dur[0:6:2], "wgrad_us_first3": dur[1:6:2],
                        "fwd_us_median": sorted(dur[0::2])[K // 2], "wgrad_us_median": sorted(dur[1::2])[K // 2],
                        "gaps_us_first6": gaps[:6], "gap_us_median": sorted(gaps)[len(gaps) // 2]})
        if calls:
            rec["hip_api_calls_us"] = calls[:12]
        print(json.dumps(rec))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--idle-us", type=float, default=0.0, help="host sleep between the barrier and the timer start")
    ap.add_argument("--out", default="regions.json")
    ap.add_argument("--events", action="store_true", help="also time the region with GPU events (marker packets)")
    ap.add_argument("--stream", action="store_true", help="run on a created stream instead of the default stream")
    ap.add_argument("--analyse", default=None, help="directory of a rocprofv3 run of this script")
    a = ap.parse_args(argv)
    if a.analyse:
        analyse(a.analyse)
    else:
        run(a)


if __name__ == "__main__":
    main()
