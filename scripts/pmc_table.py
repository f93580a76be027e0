#!/usr/bin/env python3
"""Derived per-kernel PMC table (MFMA busy, VALU busy, wave wait share, L2 hit rate, L1->L2 latency, per-wave
instruction mix) from the rocprofv3 passes of scripts/gpu_pmc_wide.sh.

    python scripts/pmc_table.py gpurun_out/pmch [--min-us 3] [--clock-ghz 2.4]

Workgroups = the launch grid (XCD padding slots that exit at once included); TCP pending stall = TCP_PENDING_STALL_CYCLES / (duration x clock x 256 CUs).  Busy % = counter cycles / (median kernel duration x clock x 1024 SIMDs); SQ_ACTIVE_INST_* count quad-cycles
(MI355X_MICROARCH.md), SQ_VALU_MFMA_BUSY_CYCLES counts cycles.  The duration is the kernel trace's median in
the PMC pass (profiled runs: a lower bound on the busy share of an unprofiled launch).
"""
import argparse
import collections
import csv
import os
import re


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=3.0)
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    a = ap.parse_args(argv)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    wgs = {}
    for f in ("l2", "waves", "lat", "lds"):
        p = os.path.join(a.dir, f + "_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for r in csv.DictReader(open(os.path.join(a.dir, f + "_kernel_trace.csv"))):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            wgs[r["Kernel_Name"]] = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    print("| kernel | median us | workgroups | MFMA busy | VALU busy | wave cycles waiting | TCP pending stall | L2 hit "
          "| L1->L2 latency (cyc) | VALU / wave | MFMA / wave | LDS bank conflicts |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, v in sorted(acc.items(), key=lambda kv: -sorted(dur[kv[0]])[len(dur[kv[0]]) // 2]):
        d = sorted(dur[k])
        t = d[len(d) // 2]
        if t < a.min_us:
            continue

        def g(c):
            x = v.get(c)
            return sum(x) / len(x) if x else float("nan")

        def div(x, y):
            return x / y if y else float("nan")

        cyc = t * 1e-6 * a.clock_ghz * 1e9 * 1024
        name = re.sub(r"\(.*$", "", k.replace("cme::(anonymous namespace)::", "").replace("void ", ""))
        cu_cyc = cyc / 4  # (256 CUs)
        print(f"| `{name[:70]}` | {t:.2f} | {wgs.get(k, 0)} | {100 * div(g('SQ_VALU_MFMA_BUSY_CYCLES'), cyc):.1f} % | "
              f"{100 * div(4 * g('SQ_ACTIVE_INST_VALU'), cyc):.1f} % | "
              f"{100 * div(g('SQ_WAIT_INST_ANY'), g('SQ_WAVE_CYCLES')):.0f} % | "
              f"{100 * div(g('TCP_PENDING_STALL_CYCLES_sum'), cu_cyc):.1f} % | "
              f"{100 * div(g('TCC_HIT_sum'), g('TCC_HIT_sum') + g('TCC_MISS_sum')):.0f} % | "
              f"{div(g('TCP_TCC_READ_REQ_LATENCY_sum'), g('TCP_TCC_READ_REQ_sum')):.0f} | "
              f"{div(g('SQ_INSTS_VALU'), g('SQ_WAVES')):.0f} | {div(g('SQ_INSTS_MFMA'), g('SQ_WAVES')):.1f} | "
              f"{g('SQ_LDS_BANK_CONFLICT'):.0f} |")


if __name__ == "__main__":
    main()
