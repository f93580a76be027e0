"""First-contact guard of the N > 1 record (bench.guard_probe) and the cost model's measured constants
(trainer.CostModel / auto_allreduce_shots).  CPU only: fake runs, no GPU, no collective.

Reference: the reference aborts the job on any MPI failure (fpcode/neural_network.cpp:9-15); here a
timed run that disagrees wildly with the probe that chose its configuration must not be reported as a clean number.
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402
from cme213_sp18_amd.parallel import trainer as T  # noqa: E402

STEPS = 200


def fake_dp(us_per_step: float, impl: str) -> dict:
    """What _run_dp_timed returns, for a run of STEPS steps at ``us_per_step``."""
    return {"ok": True, "dt": us_per_step * STEPS * 1e-6, "images": 800 * STEPS, "global_batch": 800,
            "per_gpu_batch": 200, "parallelism": "dp4", "checks": {},
            "config": {"allreduce": impl, "allreduce_tuning_us_per_step": {}}}


def test_consistent_run_is_kept_and_recorded():
    res = bench.guard_probe(fake_dp(40.0, "xgmi-fused"), STEPS, 36.0, retime=lambda: (_ for _ in ()).throw(
        AssertionError("no re-time for a consistent run")))
    assert res["ok"] and "invalid" not in res
    assert res["config"]["probe_guard"]["consistent"] is True
    assert res["config"]["probe_guard"]["timed_us_per_step"] == 40.0


def test_ten_times_off_falls_back_to_the_next_candidate():
    """The shared-GPU N = 4 rehearsal of round 4: probe 36 us, timed 15 ms.  Re-timed on RCCL, which agrees with its
    own probe: the RCCL record is reported, with both timings in probe_guard."""
    calls = []

    def retime():
        calls.append(1)
        return fake_dp(60.0, "nccl"), 55.0

    res = bench.guard_probe(fake_dp(360.0, "xgmi-fused"), STEPS, 36.0, retime)
    assert calls == [1]
    assert res["ok"] and "invalid" not in res
    assert res["config"]["allreduce"] == "nccl"
    g = res["config"]["probe_guard"]
    assert g["consistent"] is True
    assert g["first"]["what"] == "xgmi-fused" and g["first"]["timed_us_per_step"] == 360.0
    assert g["retimed"]["what"] == "nccl"


def test_still_off_after_the_retime_is_marked_invalid():
    res = bench.guard_probe(fake_dp(360.0, "xgmi-fused"), STEPS, 36.0, lambda: (fake_dp(15000.0, "nccl"), 55.0))
    assert not res["ok"]
    assert res["invalid"] == "timed run inconsistent with probe"
    assert res["config"]["probe_guard"]["consistent"] is False


def test_off_with_nothing_to_fall_back_on_is_marked_invalid():
    res = bench.guard_probe(fake_dp(360.0, "nccl"), STEPS, 36.0, None)
    assert not res["ok"] and res["invalid"] == "timed run inconsistent with probe"


def test_unprobed_or_failed_runs_are_left_alone():
    for probe in (None, "skipped: budget", "failed", float("inf")):
        res = bench.guard_probe(fake_dp(360.0, "xgmi"), STEPS, probe, None)
        assert res["ok"] and "probe_guard" not in res["config"]
    bad = fake_dp(360.0, "xgmi")
    bad["ok"] = False
    assert bench.guard_probe(bad, STEPS, 36.0, None) is bad


def test_tensor_parallel_falls_back_to_data_parallel():
    tp = {"ok": True, "dt": 1000e-6 * STEPS, "images": 0, "global_batch": 6400, "per_gpu_batch": 6400,
          "parallelism": "tp4", "checks": {}, "config": {"allreduce": "xgmi"}}
    res = bench.guard_probe(tp, STEPS, 119.0, lambda: (fake_dp(150.0, "nccl"), 140.0))
    assert res["parallelism"] == "dp4" and res["ok"]
    assert res["config"]["probe_guard"]["first"]["what"] == "tp4"


def test_cost_model_defaults_reproduce_the_planning_policy():
    T.set_cost_model(None)
    pick = T.auto_allreduce_shots
    h100, h1024, h4096 = 79_552 * 4, 814_208 * 4, 3_256_448 * 4
    assert [pick(R, h100, h100, False) for R in (2, 4, 8)] == [1, 1, 1]
    assert [pick(R, h1024, h1024, False) for R in (2, 3, 4, 8)] == [1, 2, 2, 2]
    assert [pick(R, h4096, h4096, False) for R in (2, 4, 8)] == [0, 0, 0]


def test_measured_constants_change_the_pick():
    """A node whose peer kernel is slow and whose RCCL is fast: the policy follows the measurement."""
    h100 = 79_552 * 4
    slow_peer = T.CostModel(link_gbps=20.0, kernel_us=40.0, rccl_us=8.0, rccl_gbps=100.0, measured=True)
    assert T.auto_allreduce_shots(8, h100, h100, False, model=slow_peer) == 0
    try:
        T.set_cost_model(slow_peer)
        assert T.auto_allreduce_shots(8, h100, h100, False) == 0
        assert T.allreduce_cost_us(8, h100, 1) == 40.0 + h100 / 20e3
        rec = T.COST_MODEL.as_record()
        assert rec["measured"] is True and rec["xgmi_kernel_us"] == 40.0
    finally:
        T.set_cost_model(None)
    assert T.auto_allreduce_shots(8, h100, h100, False) == 1


def test_cost_model_probe_needs_a_gpu_group():
    from cme213_sp18_amd.parallel.comm import NullComm

    assert T.measure_cost_model(NullComm(), "cpu") is None


def test_fused_form_policy_pushes_from_four_ranks():
    """The fused all-reduce's form by the cost model (planning constants): the one-shot pull at 2 ranks (the push
    form's tagged granules move 4 S / R = 2 S per link there), the owner-tile push from 4 ranks."""
    T.set_cost_model(None)
    s = 79_552 * 4
    assert T.auto_fused_form(2, s) == "pull"
    assert T.auto_fused_form(4, s) == "push" and T.auto_fused_form(8, s) == "push"
    assert T.fused_exchange_us(8, s, "push") < T.fused_exchange_us(8, s, "pull")


def test_push_form_falls_back_to_pull_then_rccl():
    """An owner-tile push run far off its probe is re-timed on the one-shot pull first; when that is off too, on
    RCCL; every timing is in the record's chain."""
    order = []

    def pull():
        order.append("pull")
        return fake_dp(500.0, "xgmi-fused"), 40.0

    def rccl():
        order.append("rccl")
        return fake_dp(60.0, "nccl"), 55.0

    res = bench.guard_probe(fake_dp(360.0, "xgmi-push"), STEPS, 36.0, [pull, rccl])
    assert order == ["pull", "rccl"]
    assert res["ok"] and res["config"]["allreduce"] == "nccl"
    g = res["config"]["probe_guard"]
    assert g["first"]["what"] == "xgmi-push"
    assert [c["what"] for c in g["chain"]] == ["xgmi-fused", "nccl"]
    # the pull agrees with its probe: RCCL is never timed
    order.clear()
    res = bench.guard_probe(fake_dp(360.0, "xgmi-push"), STEPS, 36.0, [lambda: (fake_dp(41.0, "xgmi-fused"), 40.0),
                                                                       rccl])
    assert order == [] and res["ok"] and res["config"]["allreduce"] == "xgmi-fused"


def test_fallback_chain_order_by_implementation():
    """bench.dp_fallbacks: push -> pull -> RCCL; any other xGMI form -> RCCL; RCCL and one rank -> nothing (the
    chain is built, nothing is run)."""
    from types import SimpleNamespace as NS

    class Comm:
        name = "nccl"

    ctx = NS(R=4, comm=Comm(), a=NS(warmup=1, tune_steps=1))
    assert [f.mode for f in bench.dp_fallbacks(ctx, 800, "xgmi-push", {})] == ["xgmi", "rccl"]
    assert [f.mode for f in bench.dp_fallbacks(ctx, 800, "xgmi-fused", {})] == ["rccl"]
    assert [f.mode for f in bench.dp_fallbacks(ctx, 800, "xgmi-2shot", {})] == ["rccl"]
    assert bench.dp_fallbacks(ctx, 800, "nccl", {}) == []
    assert bench.dp_fallbacks(NS(R=1, comm=Comm(), a=ctx.a), 800, "xgmi-push", {}) == []


def test_retime_keeps_the_inner_guard_record():
    inner = {"consistent": True, "timed_us_per_step": 150.0}

    def retime():
        r = fake_dp(150.0, "nccl")
        r["config"]["probe_guard"] = dict(inner)
        return r, 140.0
    tp = {"ok": True, "dt": 1000e-6 * STEPS, "images": 0, "global_batch": 6400, "per_gpu_batch": 6400,
          "parallelism": "tp4", "checks": {}, "config": {"allreduce": "xgmi"}}
    res = bench.guard_probe(tp, STEPS, 119.0, retime)
    assert res["config"]["probe_guard"]["inner"] == inner


def test_cost_model_fit_is_bounded():
    """measure_cost_model's fit: a noisy (non-positive or absurd) slope keeps the planning constants; a large fixed
    cost (a host-staged gloo communicator) is kept."""
    plan = T.CostModel()
    fixed, gbps = T._fit_bounded(10.0, 30.0, 4 * (1 << 20), plan.kernel_us, plan.link_gbps)
    assert fixed == 10.0 and abs(gbps - 4 * (1 << 20) / 20.0 / 1e3) < 1e-9
    assert T._fit_bounded(10.0, 9.0, 4e6, plan.kernel_us, plan.link_gbps) == (None, None)       # slope < 0
    assert T._fit_bounded(10.0, 10.0001, 4e6, plan.kernel_us, plan.link_gbps) == (None, None)   # 40 TB/s
    assert T._fit_bounded(0.0, 20.0, 4e6, plan.kernel_us, plan.link_gbps) == (None, None)       # no fixed cost
    assert T._fit_bounded(4500.0, 9000.0, 4e6, plan.rccl_us, plan.rccl_gbps)[0] == 4500.0      # gloo: kept
