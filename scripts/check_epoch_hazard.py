#!/usr/bin/env python3
"""Disassembly check for the launch-epoch add (csrc/mlp/granule.h gran_epoch_add): it is inline asm, so the
compiler inserts no s_waitcnt for its result.  The contract is that nothing touches the atomic's destination
VGPRs between `global_atomic_add_x2 <dst>, ... sc0` and the next `s_waitcnt vmcnt(0)` (gran_epoch_wait) -- a
register copy, spill or AGPR move of the result placed in between would read it before the atomic returned
(a garbage epoch), and a write would be overwritten by the returning data.

Compiles the translation units that use it for gfx950 (device only), disassembles them with llvm-objdump and
checks every returning global_atomic_add_x2 of every kernel.  Exit status 1 and one line per violation.

    python scripts/check_epoch_hazard.py [csrc/mlp/mlp_kernels.hip csrc/mlp/mlp_split.hip]
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
DEFAULT = [os.path.join(ROOT, "csrc", "mlp", f) for f in ("mlp_kernels.hip", "mlp_split.hip")]
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(text: str) -> set[tuple[str, int]]:
    """Every VGPR / AGPR an instruction's operand text names, as (kind, index)."""
    out = set()
    for m in _REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def disassemble(src: str, arch: str = "gfx950") -> str:
    import pybind11

    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "k.co")
        cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", f"--offload-arch={arch}", "--cuda-device-only",
               "--no-gpu-bundle-output", "-O3", "-std=c++17", "-c", src, "-o", co, f"-I{ROOT}/csrc",
               f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise SystemExit(r.stderr[-4000:])
        r = subprocess.run([OBJDUMP, "-d", f"--mcpu={arch}", "--no-show-raw-insn", co], capture_output=True,
                           text=True)
        if r.returncode != 0:
            raise SystemExit(r.stderr[-4000:])
        return r.stdout


def check(asm: str) -> tuple[int, list[str]]:
    """(number of epoch adds checked, violations)."""
    fn, lines = "?", []
    for raw in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", raw.strip())
        if m:
            fn = m.group(1)
            continue
        s = raw.split("//")[0].strip()
        if s:
            lines.append((fn, s))
    found, bad = 0, []
    for i, (fn, ins) in enumerate(lines):
        if not ins.startswith("global_atomic_add_x2 ") or " sc0" not in ins:
            continue
        ops = ins[len("global_atomic_add_x2 "):]
        dst = regs(ops.split(",")[0])
        found += 1
        for fn2, nxt in lines[i + 1:]:
            if fn2 != fn:
                bad.append(f"{fn}: no s_waitcnt vmcnt(0) after `{ins}` before the function ends")
                break
            if nxt.startswith("s_waitcnt") and "vmcnt(0)" in nxt:
                break
            if nxt.startswith("s_waitcnt"):
                continue
            touched = regs(nxt.split(None, 1)[1] if " " in nxt else "") & dst
            if touched:
                bad.append(f"{fn}: `{nxt}` touches {sorted(touched)} of `{ins}` before the vmcnt(0) wait")
                break
    return found, bad


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="*", default=DEFAULT)
    a = ap.parse_args(argv)
    total, bad = 0, []
    for src in a.src:
        n, b = check(disassemble(src))
        total += n
        bad += b
        print(f"{os.path.relpath(src, ROOT)}: {n} epoch adds checked, {len(b)} violations")
    for line in bad:
        print("VIOLATION", line)
    return 1 if bad or total == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
