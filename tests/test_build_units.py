"""The build's per-unit code generation (cme213_sp18_amd/_build.py UNIT_FLAGS / UNIT_DEPS) and the diagnostics-library
selection (cme213_sp18_amd/_native.py, CME_DIAG): CPU only, no compiler run."""
import os
import time
from pathlib import Path

from cme213_sp18_amd import _build, _native


def test_unit_flags_reach_only_their_units(tmp_path):
    obj = tmp_path / "x.o"
    xs = _build._hip_compile_cmd(Path("csrc/mlp/xstep.hip"), obj)
    wide = _build._hip_compile_cmd(Path("csrc/mlp/mlp_wide_f32.hip"), obj)
    other = _build._hip_compile_cmd(Path("csrc/mlp/mlp_split.hip"), obj)
    assert "-amdgpu-sched-strategy=max-memory-clause" in xs
    assert "-amdgpu-sched-strategy=max-ilp" in wide
    assert not any(a.startswith("-amdgpu-sched-strategy") for a in other)
    assert all("--offload-arch=gfx950" in c for c in (xs, wide, other))


def test_a_unit_is_stale_when_the_source_it_includes_changes(tmp_path, monkeypatch):
    csrc = tmp_path / "csrc"
    (csrc / "mlp").mkdir(parents=True)
    inc = csrc / "mlp" / "mlp_split.hip"
    unit = csrc / "mlp" / "mlp_wide_f32.hip"
    obj = tmp_path / "hip_mlp_wide_f32.o"
    for f in (inc, unit, obj):
        f.write_text("x")
    old = time.time() - 100
    os.utime(inc, (old, old))
    os.utime(unit, (old, old))
    monkeypatch.setattr(_build, "CSRC", csrc)
    assert not _build._stale(unit, obj, 0.0)
    os.utime(inc, None)  # the included source is now newer than the object
    assert _build._stale(unit, obj, 0.0)


def test_diag_library_is_selected_by_cme_diag(monkeypatch):
    seen = []
    monkeypatch.setattr(_native, "_load", lambda name: seen.append(name) or name)
    monkeypatch.delenv("CME_DIAG", raising=False)
    assert _native.hip() == "_hip"
    monkeypatch.setenv("CME_DIAG", "1")
    assert _native.hip() == "_hip_diag"
    assert seen == ["_hip", "_hip_diag"]
    assert "-DCME_DIAG_STAMPS=1" in _build.DIAG_FLAGS and "-DCME_HIP_MODULE=_hip_diag" in _build.DIAG_FLAGS
