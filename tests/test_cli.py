"""CLI / config: reference flags, grade presets, named BASELINE presets, end-to-end CPU run."""
import json
import os
import subprocess
import sys

import pytest

from cme213_sp18_amd.config import GRADE_PRESETS, parse_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_defaults_and_flags():
    c = parse_config([])
    assert (c.num_neuron, c.reg, c.learning_rate, c.num_epochs, c.batch_size) == (1000, 1e-4, 1e-3, 20, 800)
    c = parse_config(["-n", "64", "-r", "0.5", "-l", "0.1", "-e", "3", "-b", "100", "-p", "7", "-s", "-d"])
    assert (c.num_neuron, c.reg, c.learning_rate, c.num_epochs, c.batch_size, c.print_every) == (64, .5, .1, 3,
                                                                                                   100, 7)
    assert c.run_seq and c.debug


@pytest.mark.parametrize("g", [1, 2, 3])
def test_grade_presets_override_flags(g):
    c = parse_config(["-g", str(g), "-n", "1000", "-e", "99"])
    for k, v in GRADE_PRESETS[g].items():
        assert getattr(c, k) == v
    assert c.dtype == "f64"  # the grading gate is fp64-tight
    assert parse_config(["-g", str(g), "--dtype", "f32"]).dtype == "f32"


def test_named_presets():
    c = parse_config(["--preset", "8gpu_wide"])
    assert c.H == [784, 4096, 10] and c.batch_size == 6400
    assert parse_config(["--preset", "8gpu_bf16"]).dtype == "bf16"
    assert parse_config(["--preset", "1gpu_fp32", "-n", "32"]).num_neuron == 32  # flags beat presets


def test_cli_end_to_end_cpu(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "cme213_sp18_amd.train", "--preset", "cpu_plumbing", "-n", "16",
                        "-e", "2", "--num-train", "2000", "--num-test", "300", "-s", "-d", "--outdir",
                        str(tmp_path / "Outputs"), "--ckpt-dir", str(tmp_path / "ckpt")],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["correct"] is True
    assert "Correctness test failed" not in r.stdout
    pred = (tmp_path / "Outputs" / "Pred_testset.txt").read_text()
    assert len(pred) == 300 and pred.isdigit()
    assert (tmp_path / "ckpt" / "W0.mat").exists() and (tmp_path / "Outputs" / "CpuGpuDiff.txt").exists()


def test_long_flags():
    c = parse_config(["--hidden", "256", "--overlap-chunks", "3", "--profile", "--allreduce", "host"])
    assert c.num_neuron == 256 and c.overlap_chunks == 3 and c.profile and c.allreduce == "host"


def test_cli_profile_cpu(tmp_path):
    """--profile: per-phase timing summary in the JSON-lines log and in the final record."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    log = tmp_path / "run.jsonl"
    r = subprocess.run([sys.executable, "-m", "cme213_sp18_amd.train", "--preset", "cpu_plumbing", "-n", "16",
                        "-e", "1", "--num-train", "1600", "--num-test", "100", "--profile", "--log-json", str(log),
                        "--outdir", str(tmp_path / "Outputs")],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["profile"]["step"]["count"] == 2  # 1600 / 800 steps, torch backend: one phase per step
    ev = [json.loads(line) for line in log.read_text().splitlines()]
    assert any(e.get("event") == "profile" for e in ev)


def test_tracing_helpers_cpu():
    from cme213_sp18_amd.utils.tracing import PhaseTimer, Roctx

    rx = Roctx(enabled=False)
    assert not rx.enabled
    with rx.range("noop"):
        pass
    t = PhaseTimer(None, rx)
    for _ in range(3):
        with t.phase("a"):
            sum(range(1000))
    s = t.summary()
    assert s["a"]["count"] == 3 and s["a"]["total_ms"] >= 0
    assert "a=" in t.format()
