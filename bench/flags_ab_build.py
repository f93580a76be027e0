#!/usr/bin/env python3
"""Build variant copies of the package whose _hip library differs only in the compile flags of ONE translation unit
(default csrc/mlp/xstep.hip), for a process-alternated A/B on the GPU box (bench/flags_ab_run.sh):

    python bench/flags_ab_build.py name1='-mllvm -amdgpu-sched-strategy=max-ilp' name2='-O2' ...

-> bench/ab/<name>/cme213_sp18_amd (the Python package, its _cpu library and a _hip library linked from the tree's
objects with <unit> recompiled under the extra flags).  Delete bench/ab afterwards (it travels with every gpurun)."""
import os
import shlex
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from cme213_sp18_amd import _build as B  # noqa: E402


def main(argv):
    units = [ROOT / "csrc" / "mlp" / "xstep.hip"]
    specs = []
    for a in argv:
        if a.startswith("--unit="):  # (comma-separated: every listed unit gets the variant's flags)
            units = [ROOT / u for u in a.split("=", 1)[1].split(",")]
            continue
        name, flags = a.split("=", 1)
        specs.append((name, shlex.split(flags)))
    B.build(verbose=False)
    objs = [B.OBJ / f"hip_{s.stem}.o" for s in B._hip_sources()]
    for name, flags in specs:
        d = ROOT / "bench" / "ab" / name
        if d.exists():
            shutil.rmtree(d)
        pkg = d / "cme213_sp18_amd"
        shutil.copytree(ROOT / "cme213_sp18_amd", pkg, ignore=shutil.ignore_patterns("__pycache__", "*.so", "*.tmp"))
        shutil.copy2(B.PKG / f"_cpu{B.EXT}", pkg / f"_cpu{B.EXT}")
        mine = list(objs)
        for unit in units:
            obj = d / f"hip_{unit.stem}.o"
            subprocess.run(B._hip_compile_cmd(unit, obj) + flags, check=True)
            mine = [obj if o.name == obj.name else o for o in mine]
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *map(str, mine), "-o",
                        str(pkg / f"_hip{B.EXT}")], check=True)
        for unit in units:
            os.remove(d / f"hip_{unit.stem}.o")
        print(f"built {name}: {' '.join(flags)}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
