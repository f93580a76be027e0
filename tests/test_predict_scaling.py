"""The predicted strong-scaling curve's stated model (bench/predict_scaling.py), CPU only: measured per-rank steps in,
N = 1 / 2 / 4 / 8 images/s out, pull = step_xgmi1 + 3 hops + S / B, push = step_push1 + 2 hops + 4 S / (N B)."""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

import predict_scaling as ps  # noqa: E402


def test_model_arithmetic():
    rows = {800: {"step_walk_us": 14.0, "step_fused_us": 13.0},
            400: {"step_xgmi1_us": 14.0, "step_push1_us": 13.0},
            200: {"step_xgmi1_us": 13.0, "step_push1_us": 12.0},
            100: {"step_xgmi1_us": 12.0, "step_push1_us": 11.0}}
    out = ps.predict(rows, hop_us=1.0, link_gbps=64.0)
    by = {(p["N"], p["form"]): p for p in out}
    assert by[(1, "one process")]["us_per_step"] == 14.0
    s_over_b = ps.S_BYTES / 64e3
    assert abs(by[(2, "pull")]["us_per_step"] - round(14.0 + 3 + s_over_b, 2)) < 1e-9
    assert abs(by[(8, "push")]["us_per_step"] - round(11.0 + 2 + 4 * ps.S_BYTES / (8 * 64e3), 2)) < 1e-9
    # images/s: the global batch of 800 per step, in millions
    assert abs(by[(8, "push")]["images_per_s"] - round(800 / by[(8, "push")]["us_per_step"], 1)) < 0.11


def test_push_beats_pull_only_with_enough_ranks():
    rows = {n: {"step_xgmi1_us": 12.0, "step_push1_us": 12.0, "step_walk_us": 12.0} for n in (800, 400, 200, 100)}
    out = ps.predict(rows, hop_us=1.0, link_gbps=64.0)
    by = {(p["N"], p["form"]): p["us_per_step"] for p in out}
    assert by[(2, "push")] > by[(2, "pull")]  # 2 S / B of tagged payload at R = 2
    assert by[(8, "push")] < by[(8, "pull")]
