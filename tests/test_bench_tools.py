"""Bench tooling on CPU: the all-reduce sweep's size plan and its single-rank refusal."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

import allreduce_bench as ab  # noqa: E402


def test_allreduce_sizes_cover_the_mlp_buckets():
    a = ab.parse([])
    got = dict(ab.sizes(a))
    assert got["mlp_h100"] == 79510 and got["mlp_h4096"] == 3256330  # SURVEY 2.5 payloads
    sweep = [n * 4 for k, n in got.items() if k.endswith("B")]
    assert sweep[0] == 4 << 10 and sweep[-1] == 64 << 20 and all(b2 == 4 * b1 for b1, b2 in zip(sweep, sweep[1:]))
    a64 = ab.parse(["--dtype", "f64", "--max-bytes", str(1 << 20)])
    assert "mlp_h4096" not in dict(ab.sizes(a64))


def test_allreduce_bench_refuses_one_rank(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert ab.main(["--iters", "1"]) == 2
