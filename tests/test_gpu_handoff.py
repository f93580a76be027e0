"""Failure semantics of the in-launch hand-offs (the all-gather forward + head launches) on the GPU.

The forward + head launch waits, inside the kernel, for the other workgroups of its column tile (H <= 128:
csrc/mlp/fha_body.h; wide layers: mlp_split.hip wide_head_ag).  A wait that outlasts its bound sets a sticky
error word; the weight-gradient launch reads that word and APPLIES NOTHING, and train() raises
KernelHandoffTimeout -- on every rank (a failing rank must take the job down, not leave it hung
or let the replicas diverge; the reference only ``exit(1)``s, fpcode/neural_network.cpp:9-15).  Here the
timeout is REAL: MlpEngine.inject_handoff_timeout makes one workgroup of column tile 0 withhold its hand-off
granules (the z2 partial at H <= 128, the column tile's D in the wide fused head), so that tile's polls expire.  Also pinned: the wide fused head's counters stay consistent when a partial
batch switches the launch between its 128 x 128 and 64 x 64 tilings (each tiling has its own counters).
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd.parallel import DataParallelTrainer, MlpEngine
from cme213_sp18_amd.parallel.trainer import KernelHandoffTimeout
from cme213_sp18_amd.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (dtype, H, n): the H <= 128 form, the 128 x 128 wide form (H = 4096, n = 800), the 64 x 64 wide form
CASES = [("f32", 100, 800), ("bf16", 100, 800), ("f32", 100, 37), ("f32", 4096, 800), ("bf16", 1024, 800),
         ("f32", 4096, 200)]


def _engine(dt, H, n, N=None):
    x, y = synthetic_mnist(N or 3 * n + 64, seed=H + n)
    nn = NeuralNetwork([784, H, 10])
    e = MlpEngine(nn.H, dtype=dt, max_cols=n, device="cuda")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    e.set_store_a1(False)  # the trainer's setting: the wide fused head's measured form
    return e


@pytest.mark.parametrize("dt,H,n", CASES)
def test_forced_handoff_timeout_applies_nothing(dt, H, n):
    """A step whose forward + head launch really timed out leaves params and the W1 planes bitwise as they
    were (sgd=1: the fused update is skipped); so does every later step (the error word is sticky); in
    gradient mode (sgd=0) the bucket's status element is 1 and the separate SGD kernel changes nothing."""
    e = _engine(dt, H, n)
    e.run(0, n, 1.0 / n, 1e-4, 0.05, sgd=True)  # one good step
    torch.cuda.synchronize()
    assert not e.kernel_error()
    moved = e.params.clone()
    e.run(n, n, 1.0 / n, 1e-4, 0.05, sgd=False)
    torch.cuda.synchronize()
    assert float(e.grads[e.status_index]) == 0.0  # a trusted step's status
    before = (e.params.clone(), e.W1p.clone())
    assert torch.equal(before[0], moved)
    e.inject_handoff_timeout(0, 2000)
    e.run(n, n, 1.0 / n, 1e-4, 0.05, sgd=True)
    torch.cuda.synchronize()
    assert e.kernel_error(), "the forced hand-off did not time out"
    assert torch.equal(e.params, before[0]) and torch.equal(e.W1p, before[1])
    e.inject_handoff_timeout(-1)
    e.run(2 * n, n, 1.0 / n, 1e-4, 0.05, sgd=True)  # sticky: nothing after the timeout is applied either
    e.run(0, n, 1.0 / n, 1e-4, 0.05, sgd=False)
    torch.cuda.synchronize()
    assert torch.equal(e.params, before[0]) and torch.equal(e.W1p, before[1])
    assert float(e.grads[e.status_index]) == 1.0
    e.sgd(0.05)  # the separate SGD kernel honours the status element
    torch.cuda.synchronize()
    assert torch.equal(e.params, before[0]) and torch.equal(e.W1p, before[1])


@pytest.mark.parametrize("H", [100, 4096])
def test_real_timeout_raises_in_train_and_freezes_params(H):
    """train() (native step loop) after a real timed-out hand-off: KernelHandoffTimeout at the end of the
    epoch, and not one of the epoch's steps changed a parameter."""
    x, y = synthetic_mnist(3200, seed=2)
    tr = DataParallelTrainer(NeuralNetwork([784, H, 10]), dtype="f32", batch_size=800)
    tr.recover = False  # (the in-process fallback is pinned by the next test)
    tr.load(x, y)
    tr.train(1, 0.01, 1e-4)
    assert tr._allgather_live() and not tr.engine.kernel_error()
    tr.engine.inject_handoff_timeout(1, 2000)
    before = tr.engine.params.clone()
    with pytest.raises(KernelHandoffTimeout):
        tr.train(1, 0.01, 1e-4)
    assert torch.equal(tr.engine.params, before)


@pytest.mark.parametrize("H", [100, 4096])
def test_train_recovers_from_handoff_timeout_bitwise(H):
    """train() survives a REAL timed-out all-gather hand-off in its first epoch: the epoch-start snapshot is
    restored, the forward + head switches to the last-arriver form (no workgroup waits for another) and the epoch
    re-runs, with one warning.  The result is BITWISE the run that used that form from the start."""
    x, y = synthetic_mnist(3200, seed=4)
    nn = NeuralNetwork([784, H, 10])
    init = [p.copy() for p in nn.params]
    tr = DataParallelTrainer(nn, dtype="f32", batch_size=800)
    tr.load(x, y)
    tr.engine.inject_handoff_timeout(1, 2000)
    st = tr.train(2, 0.01, 1e-4)
    assert tr.recovered is not None and "hand-off" in tr.recovered, tr.recovered
    assert not tr._allgather_live() and not tr.engine.kernel_error()
    assert st.steps == 2 * 4 and tr.iter == 8
    nn2 = NeuralNetwork([784, H, 10])
    for dst, src in zip(nn2.params, init):
        dst[...] = src
    ref = DataParallelTrainer(nn2, dtype="f32", batch_size=800)
    ref.engine.set_fh_allgather(False)
    ref.load(x, y)
    ref.train(2, 0.01, 1e-4)
    assert torch.equal(tr.engine.params, ref.engine.params)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_wide_head_counters_survive_tiling_switch(dt):
    """One engine alternating per-GPU batches that take the 128 x 128 tiling (n = 800) and the 64 x 64
    tiling (n = 200) of the wide fused head, H = 4096: every step agrees with the plain forward + head
    launches (to fp32 rounding of the dW2 partial sums) and no poll timed out -- each tiling keeps its own
    epoch counters (with ONE shared array a round-2 64 x 64 launch after an 800-column launch computed its
    wait target from the other tiling's count and read unpublished partials: ADVICE r2)."""
    H, N = 4096, 2400
    x, y = synthetic_mnist(N, seed=17)
    nn = NeuralNetwork([784, H, 10])
    outs = []
    for ag in (True, False):
        e = MlpEngine(nn.H, dtype=dt, max_cols=800, device="cuda")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        e.set_store_a1(False)
        e.set_fh_allgather(ag)
        e._hip_step().ag_tiles64 = 1
        for off, n in ((0, 800), (800, 200), (1000, 800), (1800, 200), (0, 200), (200, 800)):
            e.run(off, n, 1.0 / n, 1e-4, 0.05, sgd=True)
        torch.cuda.synchronize()
        if ag:
            assert not e.kernel_error()
            c = e.ag_counters.view(2, -1, 32)[:, :, 0]
            t128, t64 = (800 + 127) // 128, (800 + 63) // 64
            assert c[0, :t128].tolist() == [32 * 3] * t128  # three 800-column launches, tm = 32 epoch adds each
            assert c[1, :(200 + 63) // 64].tolist() == [64 * 3] * ((200 + 63) // 64)  # tm = 64
            assert int(c[1, (200 + 63) // 64:t64].sum()) == 0
        outs.append(e.params.clone())
    rel = float((outs[0] - outs[1]).abs().max() / outs[1].abs().max())
    # (bf16: the two heads' dW2 partial sums round differently in fp32, and over 6 steps the bf16 rounding of
    # D / dZ1 turns some of those last-bit differences into bf16-ulp ones: 4e-4 .. 1.5e-3 measured)
    assert rel < (1e-5 if dt == "f32" else 3e-3), rel


@pytest.mark.parametrize("allreduce", ["xgmi"])
def test_dp_recovers_from_one_ranks_handoff_timeout(tmp_path, allreduce):
    """2 data-parallel ranks sharing the GPU on the xGMI-fused all-reduce; rank 0's hand-off really times out in
    the first epoch.  Both ranks raise together, restore the epoch-start snapshot, drop to the last-arriver head and
    the communicator's all-reduce (the poisoned xGMI buckets are closed) and finish: replicas bitwise equal, and
    bitwise the run that used that path from the start."""
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); from tests.dist_workers import handoff_recover_dp_main; "
            f"handoff_recover_dp_main({str(tmp_path)!r}, {allreduce!r})")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    z = [dict(np.load(tmp_path / f"recover_{allreduce}_{rank}.npz")) for rank in range(2)]
    for rank in range(2):
        assert str(z[rank]["impl0"]).startswith("xgmi"), z[rank]["impl0"]
        assert float(z[rank]["recovered"]) == 1.0 and not str(z[rank]["impl1"]).startswith("xgmi"), z[rank]
        assert float(z[rank]["equal_ref"]) == 1.0, rank
    assert float(z[0]["agree"]) == 1.0


@pytest.mark.parametrize("allreduce", ["rccl", "xgmi"])
def test_handoff_timeout_on_one_rank_stops_every_rank(tmp_path, allreduce):
    """2 data-parallel ranks sharing the GPU, rank 0's hand-off really times out: both ranks raise
    KernelHandoffTimeout and neither applied a step of that epoch.  rccl here is the gloo all-reduce of the
    gradient bucket (its status element carries the failure to the other rank's SGD); xgmi is the all-reduce
    fused into the weight-gradient launch (the failed rank stops taking part, rank 1's waits time out)."""
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); from tests.dist_workers import handoff_timeout_dp_main; "
            f"handoff_timeout_dp_main({str(tmp_path)!r}, {allreduce!r})")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    z = [dict(np.load(tmp_path / f"handoff_{allreduce}_{rank}.npz")) for rank in range(2)]
    if allreduce == "xgmi":
        assert str(z[0]["impl"]).startswith("xgmi"), z[0]["impl"]
    for rank in range(2):
        assert float(z[rank]["clean_err"]) == 0.0
        assert float(z[rank]["raised"]) == 1.0, (rank, z[rank])
        assert float(z[rank]["untouched"]) == 1.0, (rank, z[rank])
    assert float(z[0]["local_err"]) == 1.0 and float(z[1]["local_err"]) == 0.0


@pytest.mark.parametrize("H", [100, 4096])
def test_partial_residency_times_out_and_applies_nothing(H):
    """The hazard the bounded polls exist for, forced for real: a side stream holds all but 8 CUs (one
    160 KB-LDS workgroup per CU, sleeping ~50 ms, csrc/mlp/occupy.hip) while the step's all-gather forward + head
    launch starts, so most of its column tiles' workgroups are NOT resident.  The resident ones' polls must time out
    (no hang), the error word must be set, and the weight-gradient launch must apply nothing."""
    import time

    from cme213_sp18_amd._native import hip

    n = 800
    e = _engine("f32", H, n)
    e.run(0, n, 1.0 / n, 1e-4, 0.05, sgd=True)
    torch.cuda.synchronize()
    assert not e.kernel_error()
    e.inject_handoff_timeout(-1, 500)  # no withheld granules: only a short wall-time bound (500 us)
    # (the column-tile placement: a column tile's row-tile workgroups share an XCD.  Under the XCD-row placement
    # (MlpStep.xcd_rows) they sit on different XCDs and are dispatched together, so with the 8 free CUs spread one
    # per XCD each column tile runs complete and in turn -- correct, and no wait to time out.)
    e._hip_step().xcd_rows = 0
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    # The step must run BESIDE the holder, i.e. on another hardware queue.  HIP spreads streams over its few
    # hardware queues, so a new stream may share the holder's queue; then the step simply runs after the holder (and
    # completes normally) -- detected by its duration, and retried on the next pair of new streams.
    for _attempt in range(8):
        side, work = torch.cuda.Stream(), torch.cuda.Stream()
        work.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        before = e.params.clone()
        running = torch.zeros(1, dtype=torch.int32).pin_memory()  # set by the holder's first workgroup
        hip().occupy_cus(cus - 8, 160 * 1024, 50_000_000, side.cuda_stream, running.data_ptr())
        t0 = time.time()
        while int(running[0]) == 0:  # the holder is running before the step is queued
            assert time.time() - t0 < 5.0, "the CU holder never started"
            time.sleep(1e-4)
        time.sleep(0.002)  # (every holder workgroup dispatched)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(work):
            ev0.record()
            e.run(n, n, 1.0 / n, 1e-4, 0.05, sgd=True)
            ev1.record()
        torch.cuda.synchronize()
        if ev0.elapsed_time(ev1) > 10.0:  # it waited beside the holder: its non-resident workgroups could not start
            break
        assert not e.kernel_error()  # (it ran after the holder on the same queue: a normal step)
    else:
        pytest.fail("no stream pair ran the step beside the CU holder")
    assert e.kernel_error(), "most of the grid was not resident: the hand-off polls should have timed out"
    assert torch.equal(e.params, before)
