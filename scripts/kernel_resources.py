#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of a HIP translation unit (hipcc's kernel-resource-usage
remarks for gfx950), so a kernel edit can be checked for spills and occupancy changes on the CPU box.

    python scripts/kernel_resources.py csrc/mlp/mlp_split.hip [--filter rega]
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import sysconfig
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("VGPRs", "AGPRs", "SGPRs Spill", "VGPRs Spill", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]")


def resources(src: str, arch: str = "gfx950") -> list[dict]:
    import pybind11

    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", f"--offload-arch={arch}", "-O3", "-std=c++17", "-fPIC", "-c", src,
               "-o", os.path.join(d, "k.o"), f"-I{ROOT}/csrc", f"-I{pybind11.get_include()}",
               f"-I{sysconfig.get_paths()['include']}", "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-4000:])
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (Function Name|[A-Za-z \[\]/]+): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            out.append(cur)
        elif cur is not None and key in FIELDS:
            cur[key] = val
    return out


def short(name: str) -> str:
    try:
        d = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    except FileNotFoundError:
        d = name
    d = d.replace("cme::(anonymous namespace)::", "").replace("cme::", "")
    return re.sub(r"\(.*\)$", "", d)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    a = ap.parse_args(argv)
    rows = [r for r in resources(a.src) if a.filter in short(r["name"])]
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'sSpl':>5s} {'vSpl':>5s} {'occ':>4s}")
    for r in rows:
        print(f"{short(r['name'])[:70]:70s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} "
              f"{r.get('SGPRs Spill', '?'):>5s} {r.get('VGPRs Spill', '?'):>5s} {r.get('Occupancy [waves/SIMD]', '?'):>4s}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
