"""In-tree build of the two native extensions.

* ``_hip``  -- every gfx950 kernel (hipcc --offload-arch=gfx950) + pybind11 bindings.
* ``_cpu``  -- the native CPU runtime (g++ -O3 -fopenmp): fp64 reference
  trainer, MNIST IDX reader, raw_ascii checkpoint I/O, OpenMP radix sort, ...

The reference builds with ``mpic++`` + ``nvcc -arch=sm_20`` from a Makefile
(fpcode/Makefile:1-42); here the extensions are compiled directly with hipcc /
g++ (no hipify, no torch.utils.cpp_extension JIT) so the built ``.so`` files
live next to the Python sources and travel with the repository snapshot.

Usage: ``python -m cme213_sp18_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("CME_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _hip_sources() -> list[Path]:
    srcs = [s for d in ("mlp", "suite", "comm") for s in sorted((CSRC / d).glob("*.hip"))]
    srcs += [CSRC / "bindings_hip.cpp", CSRC / "suite" / "suite_bindings.cpp", CSRC / "comm" / "comm_bindings.cpp"]
    return srcs


def _cpu_sources() -> list[Path]:
    return sorted((CSRC / "cpu").glob("*.cpp")) + [CSRC / "bindings_cpu.cpp", CSRC / "bindings_suite_cpu.cpp"]


def _headers_mtime() -> float:
    hs = list(CSRC.rglob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _stale(src: Path, obj: Path, hdr_mtime: float) -> bool:
    if not obj.exists():
        return True
    om = obj.stat().st_mtime
    deps = [CSRC / d for d in UNIT_DEPS.get(src.name, [])]
    return om < src.stat().st_mtime or om < hdr_mtime or any(om < d.stat().st_mtime for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")


# per-translation-unit code-generation flags, each measured (process-alternated A/B of whole libraries that differ
# only in that unit's flags: bench/flags_ab_build.py + bench/flags_ab_run.sh)
UNIT_FLAGS = {
    # the XCD-local pipeline: the machine scheduler's memory-clause strategy, walking step 9.55-9.58 -> 9.46-9.50 us
    # (max-ilp 9.54-9.59, iterative-ilp 10.2-10.4, -O2 9.64-9.66; profiles/r6/flags/)
    "xstep.hip": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    # the wide fp32 A-in-registers engine (mlp_split.hip's fp32 launchers, compiled apart): max-ILP, 784-4096-10 fp32
    # walking step 57.4-58.0 -> 55.4-55.5 us; the same strategy on the whole of mlp_split.hip made the bf16 wide step
    # +3.3 us and the n = 100 two-launch step +0.4 us (profiles/r6/flags_split/)
    "mlp_wide_f32.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
}
# sources a unit includes besides the headers (its object is stale when they change)
UNIT_DEPS = {"mlp_wide_f32.hip": ["mlp/mlp_split.hip"]}


def _hip_compile_cmd(src: Path, obj: Path) -> list[str]:
    return [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", str(src), "-o",
            str(obj), f"-I{CSRC}", "-Wno-unused-result", *_pybind_includes(), *UNIT_FLAGS.get(src.name, [])]


def _cpu_compile_cmd(src: Path, obj: Path) -> list[str]:
    return [CXX, "-O3", "-march=x86-64-v2", "-std=c++17", "-fPIC", "-fopenmp", "-c", str(src), "-o", str(obj),
            f"-I{CSRC}", "-Wall", "-Wextra", "-Wno-unused-parameter", *_pybind_includes()]


# the diagnostics library (build(diag=True), `--diag`): the same kernels with the two-launch kernels' stamps compiled
# in, as module _hip_diag (loaded instead of _hip when CME_DIAG=1: cme213_sp18_amd/_native.py; bench/stamps_*.py)
DIAG_FLAGS = ["-DCME_DIAG_STAMPS=1", "-DCME_HIP_MODULE=_hip_diag"]


def build(force: bool = False, jobs: int | None = None, verbose: bool = True, diag: bool = False) -> dict[str, Path]:
    obj_dir = OBJ.parent / "obj_diag" if diag else OBJ
    obj_dir.mkdir(parents=True, exist_ok=True)
    hdr = _headers_mtime()
    jobs = jobs or min(8, os.cpu_count() or 4)
    out: dict[str, Path] = {}

    def hip_cmd(src, obj):
        return _hip_compile_cmd(src, obj) + (DIAG_FLAGS if diag else [])

    plans = {
        "_hip_diag" if diag else "_hip": (
            [(s, obj_dir / f"hip_{s.stem}.o") for s in _hip_sources()], hip_cmd,
            lambda objs, so: [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(so)]),
    }
    if not diag:
        plans["_cpu"] = ([(s, OBJ / f"cpu_{s.stem}.o") for s in _cpu_sources()], _cpu_compile_cmd,
                         lambda objs, so: [CXX, "-shared", "-fPIC", "-fopenmp", *map(str, objs), "-o", str(so)])
    todo = []
    for name, (pairs, mk, _) in plans.items():
        for src, obj in pairs:
            if force or _stale(src, obj, hdr):
                todo.append((name, src, obj, mk(src, obj)))
    if todo and verbose:
        print(f"[cme-build] compiling {len(todo)} translation unit(s) with {jobs} job(s)", flush=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(_run, cmd): (name, src) for name, src, obj, cmd in todo}
        for f in cf.as_completed(futs):
            f.result()
            if verbose:
                print(f"[cme-build]   ok {futs[f][1].relative_to(ROOT)}", flush=True)
    for name, (pairs, _, link) in plans.items():
        so = PKG / f"{name}{EXT}"
        objs = [o for _, o in pairs]
        if force or not so.exists() or any(o.stat().st_mtime > so.stat().st_mtime for o in objs):
            # linked to a temporary name and renamed into place (atomic): a snapshot of the tree taken meanwhile
            # (a GPU run's upload) sees the old library or the new one, never a half-written file
            tmp = so.with_name(so.name + ".tmp")
            _run(link(objs, tmp))
            os.replace(tmp, so)
            if verbose:
                print(f"[cme-build] linked {so.relative_to(ROOT)}", flush=True)
        out[name] = so
    return out


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--diag", action="store_true", help="the diagnostics library _hip_diag (stamps compiled in)")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, diag=a.diag)
    return 0


if __name__ == "__main__":
    sys.exit(main())
