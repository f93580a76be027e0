#!/usr/bin/env python3
"""Turn rocprofv3 CSV output into a markdown summary for profiles/.

  python scripts/prof_summary.py --stats DIR/xxx_kernel_stats.csv [--pmc DIR/xxx_counter_collection.csv]
         [--title T] [--note TEXT] -o profiles/NAME.md
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str, width: int = 90) -> str:
    name = re.sub(r"\s+", " ", name)
    name = name.replace("(anonymous namespace)::", "")
    return name if len(name) <= width else name[: width - 3] + "..."


def stats_table(path: str, top: int) -> list[str]:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0)))
    total = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
    out = ["| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---:|---:|---:|---:|---:|---:|"]
    for r in rows[:top]:
        out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                   f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                   f"{100 * float(r['TotalDurationNs']) / total:.1f} |")
    return out


def pmc_table(path: str, top: int) -> list[str]:
    acc: dict[str, dict[str, list[float]]] = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    counters = sorted({c for k in acc.values() for c in k})
    kernels = sorted(acc, key=lambda k: -len(next(iter(acc[k].values()))))[:top]
    out = ["| kernel | " + " | ".join(counters) + " |", "|---|" + "---:|" * len(counters)]
    for k in kernels:
        vals = []
        for c in counters:
            v = acc[k].get(c)
            vals.append(f"{sum(v) / len(v):.4g}" if v else "")
        out.append(f"| `{short(k, 60)}` | " + " | ".join(vals) + " |")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", action="append", default=[])
    ap.add_argument("--pmc", action="append", default=[])
    ap.add_argument("--title", default="rocprofv3 summary")
    ap.add_argument("--note", default="")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    lines = [f"# {a.title}", ""]
    if a.note:
        lines += [a.note, ""]
    for p in a.stats:
        lines += [f"## Kernel time (`{p.split('/')[-1]}`)", ""] + stats_table(p, a.top) + [""]
    for p in a.pmc:
        lines += [f"## Counters, mean per dispatch (`{p.split('/')[-1]}`)", ""] + pmc_table(p, a.top) + [""]
    open(a.out, "w").write("\n".join(lines))


if __name__ == "__main__":
    main()
