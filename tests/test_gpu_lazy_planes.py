"""Lazy W1-plane refresh of the wide split3 step (MlpStep.lazy_planes, MlpEngine.lazy_planes).

At 784-4096-10 the 128 x 128 forward reads fp32 W1 (split into its exact bf16 planes in registers), so the weight
update no longer re-splits W1 into the stored planes (3 bf16 stores per weight, ~3 us of a 58 us step); the step
marks them stale and re-splits W1 right before a forward that DOES read them (the 64 x 64 tiling of a partial batch,
predict, the tensor-parallel forward) and after a snapshot restore.  The planes are an exact function of W1, so
every result must be BITWISE what the eager-refresh engine computes.
"""
import pytest
import torch

from cme213_sp18_amd import NeuralNetwork
from cme213_sp18_amd.parallel import DataParallelTrainer, MlpEngine
from cme213_sp18_amd.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu


def test_lazy_planes_bitwise_equal_across_tilings():
    """n = 800 (128 x 128, fp32 W1) and n = 200 (64 x 64, reads the planes) steps interleaved, with and without
    the all-gather head: params bitwise equal to the eager-refresh engine after every step, and the planes equal
    once refreshed."""
    H, N = 4096, 2400
    x, y = synthetic_mnist(N, seed=5)
    nn = NeuralNetwork([784, H, 10])
    for ag in (True, False):
        engines = []
        for lazy in (False, True):
            e = MlpEngine(nn.H, dtype="f32", max_cols=800, device="cuda")
            e.set_lazy_planes(lazy)
            e.set_params(*nn.params)
            e.load_dataset(x, y)
            e.set_store_a1(False)
            e.set_fh_allgather(ag)
            e._hip_step().ag_tiles64 = 1
            engines.append(e)
        plan = ((0, 800), (800, 800), (1600, 200), (1600, 800), (0, 200), (200, 200), (400, 800))
        for i, (off, n) in enumerate(plan):
            for e in engines:
                e.run(off, n, 1.0 / n, 1e-4, 0.05, sgd=True)
            torch.cuda.synchronize()
            assert torch.equal(engines[0].params, engines[1].params), (ag, i, off, n)
        s = engines[1]._hip_step()
        assert s.planes_stale, "the last 800-column step should have left the planes stale"
        s.refresh_planes(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert not s.planes_stale
        assert torch.equal(engines[0].W1p, engines[1].W1p)
        assert not any(e.kernel_error() for e in engines)


def test_lazy_planes_trainer_graphs_and_predict():
    """DataParallelTrainer at H = 4096 with captured HIP graphs over an epoch whose last batch is partial (the
    64 x 64 tiling), then predict(): identical to the eager-refresh trainer, bitwise."""
    H = 4096
    x, y = synthetic_mnist(2200, seed=9)
    outs = []
    for lazy in (False, True):
        tr = DataParallelTrainer(NeuralNetwork([784, H, 10]), dtype="f32", batch_size=800, use_graphs=True,
                                 executor="graph")
        tr.engine.set_lazy_planes(lazy)
        tr.load(x, y)
        tr.train(2, 0.01, 1e-4)
        pred = tr.engine.predict(x[:500])
        torch.cuda.synchronize()
        outs.append((tr.engine.params.clone(), pred))
    assert torch.equal(outs[0][0], outs[1][0])
    assert (outs[0][1] == outs[1][1]).all()
