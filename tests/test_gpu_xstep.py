"""The XCD-local step pipeline (csrc/mlp/xstep.hip: a whole native-loop plan in ONE persistent launch, XCD-local
barriers, the z2 all-gather the only cross-XCD hand-off) against the two-launch step it replaces: parameters
BITWISE equal over whole epochs (the same arithmetic and summation orders), across launches (the control banks
alternate, the granule tags continue), mixed with two-launch steps, and a forced hand-off timeout that applies
nothing.  The reference's hot loop: fpcode/neural_network.cpp:449-555."""
import pytest
import torch

from cme213_sp18_amd.models.mlp import NeuralNetwork
from cme213_sp18_amd.parallel.engine import MlpEngine
from cme213_sp18_amd.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu

LR, REG = 0.05, 1e-4


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _pair(H, n, N, seed, forms=(0, -1)):
    """Engines with the same weights and data: [0] the two-launch step (xstep = 0), [1] the pipeline
    (auto); the head's dW2 partials on below 768 columns too (the pipeline always takes them, and [1]'s own
    two-launch steps must then match [0]'s)."""
    x, y = synthetic_mnist(N, seed=seed)
    nn = NeuralNetwork([784, H, 10])
    out = []
    for xs in forms:
        e = MlpEngine(nn.H, "f32", max_cols=n, device="cuda", path="split3")
        e.set_params(*nn.params)
        e.load_dataset(x, y)
        e.set_store_a1(False)
        e._hip_step().xstep = xs
        e._hip_step().head_dw2 = 1
        out.append(e)
    return out


def _plan(e, g0, count, n, N):
    e._hip_step().run_steps(g0, count, n, 0, n, N, 1.0 / n, REG, LR, 1, _stream())


@pytest.mark.parametrize("H,n", [(100, 800), (128, 800), (64, 960), (100, 784), (100, 400), (128, 512)])
def test_xstep_is_bitwise_the_two_launch_step(H, n):
    """Two epochs (with the wrap to sample 0) as one plan, then plans from other start batches (the other control
    bank, then the first again), then a two-launch step and a plan again: parameters bitwise equal throughout."""
    N = 5 * n + 48  # (a partial batch at the end: the walk wraps before it)
    engines = _pair(H, n, N, seed=H + n)

    def both(fn):
        for e in engines:
            fn(e)
        torch.cuda.synchronize()
        assert torch.equal(engines[0].params, engines[1].params)

    both(lambda e: _plan(e, 0, 2 * (N // n), n, N))
    assert engines[1]._hip_step().xstep_used == 1, engines[1]._hip_step().xstep_reason
    assert engines[0]._hip_step().xstep_used == 0
    both(lambda e: _plan(e, 2 * n, 3, n, N))
    both(lambda e: _plan(e, n, 7, n, N))
    both(lambda e: e.run(16, n, 1.0 / n, REG, LR, sgd=True))  # a two-launch step between plans
    both(lambda e: _plan(e, 3 * n, 1, n, N))
    both(lambda e: _plan(e, 0, 4, n, N))
    assert torch.equal(engines[0].dz1()[:, :n], engines[1].dz1()[:, :n])
    for e in engines:
        assert not e.kernel_error()


@pytest.mark.parametrize("H,n,g0", [(100, 100, 0), (128, 100, 0), (100, 104, 0), (64, 200, 4), (100, 256, 0),
                                    (100, 800, 8)])
def test_xstep_row_major_form_is_bitwise_the_two_launch_step(H, n, g0):
    """Steps off the 16-sample grid (n = 100: three batches in four; a plan starting at sample 8) or below 257
    columns run the pipeline's row-major form (row-major pixels, fp32 dZ1 row-major, read with sc1 loads; dW1 as 2 x
    16-byte vectors for n % 8 == 0, the same with the tail past n zeroed in registers for n % 4 == 0, 16-byte pixel
    pairs on the grid at n % 16 == 0) -- bitwise the two-launch step that takes fp32 dZ1
    (a_fp32 = 3; at n = 100 the default two-launch step takes dZ1 planes instead).  A one-step plan is first checked
    against the torch backend's fp32 step (raw 0-255 pixels at lr 0.05 amplify rounding differences over steps, so
    only the bitwise comparison runs longer)."""
    N = 5 * n + 48
    engines = _pair(H, n, N, seed=H + n + g0)
    for e in engines:
        e._hip_step().a_fp32 = 3
    ref = MlpEngine([784, H, 10], "f32", max_cols=n, device="cuda", backend="torch")
    ref.set_params(*(t.cpu().numpy() for t in (engines[0].W1, engines[0].b1, engines[0].W2, engines[0].b2)))
    ref.load_dataset(*synthetic_mnist(N, seed=H + n + g0))

    def both(fn, stage=""):
        for e in engines:
            fn(e)
        torch.cuda.synchronize()
        diff = {k: float((getattr(engines[0], k) - getattr(engines[1], k)).abs().max()) for k in ("W1", "b1", "W2", "b2")}
        assert torch.equal(engines[0].params, engines[1].params), (stage, diff)

    both(lambda e: _plan(e, g0, 1, n, N), "one-step plan")
    ref.run(g0, n, 1.0 / n, REG, LR, sgd=True)
    torch.cuda.synchronize()
    assert engines[1]._hip_step().xstep_used == 1, engines[1]._hip_step().xstep_reason
    err = (engines[1].params - ref.params).abs().max() / ref.params.abs().max()
    assert err < 2e-5, float(err)
    # (n = 800 from sample 8: no wrap to sample 0, where the two-launch step would take the fragment-ordered forms)
    both(lambda e: _plan(e, g0, 2 * (N // n) if g0 % 16 == 0 else N // n - 1, n, N), "two epochs")
    assert engines[1]._hip_step().xstep_used == 1, engines[1]._hip_step().xstep_reason
    assert engines[1]._hip_step().dz_left_swz == 0
    both(lambda e: _plan(e, 2 * n + g0, 2, n, N))
    both(lambda e: e.run(16, n, 1.0 / n, REG, LR, sgd=True))  # a two-launch step between plans
    both(lambda e: _plan(e, n + g0, 3, n, N))
    assert torch.equal(engines[0].dz1()[:, :n], engines[1].dz1()[:, :n])
    for e in engines:
        assert not e.kernel_error()


def test_xstep_falls_back_where_it_does_not_apply():
    """Plans the pipeline does not take run the two-launch loop (bitwise the same as xstep = 0): steps off 4-byte
    aligned pixel columns, the head's dW2 partials off; xstep = 1 (required) then raises."""
    n, N = 800, 3 * 800 + 48
    engines = _pair(100, n, N, seed=7)
    for e in engines:
        _plan(e, 2, 2, n, N)  # (first sample 2: the dW1 tiles' pixel loads need 4-byte aligned columns)
    torch.cuda.synchronize()
    assert engines[1]._hip_step().xstep_used == 0
    assert "4-byte" in engines[1]._hip_step().xstep_reason
    assert torch.equal(engines[0].params, engines[1].params)
    st = engines[1]._hip_step()
    st.xstep = 1
    with pytest.raises(ValueError, match="xstep"):
        _plan(engines[1], 2, 1, n, N)
    small = _pair(100, 400, 2000, seed=8)
    for e in small:
        e._hip_step().head_dw2 = 0
        _plan(e, 0, 3, 400, 2000)
    torch.cuda.synchronize()
    assert small[1]._hip_step().xstep_used == 0
    assert "dW2 partials" in small[1]._hip_step().xstep_reason
    assert torch.equal(small[0].params, small[1].params)


@pytest.mark.parametrize("bar", [0, 1, 2])
def test_xstep_barrier_forms_give_the_same_bits(bar):
    """The XCD-local barrier forms (MlpStep.xstep_bar: 0 an atomic counter, 1 a flag line in the XCD's L2, 2 the flag
    line with the first barrier fine-grained per dW1 wave, 3 both barriers fine-grained -- the forward's waves wait
    for their own dW1 tiles, the default) order the same work: the same bits as the default form, over launches that
    alternate the control banks."""
    n, N = 800, 4 * 800
    engines = _pair(100, n, N, seed=11)
    engines[0]._hip_step().xstep = -1
    engines[0]._hip_step().xstep_bar = bar
    for g0, k in ((0, 9), (n, 3), (2 * n, 5)):
        for e in engines:
            _plan(e, g0, k, n, N)
        torch.cuda.synchronize()
        assert all(e._hip_step().xstep_used for e in engines), [e._hip_step().xstep_reason for e in engines]
        assert torch.equal(engines[0].params, engines[1].params)


@pytest.mark.parametrize("bar", [1, 3])
def test_xstep_handoff_timeout_applies_nothing(bar):
    """A z2 hand-off that never completes (row tile 3 of column tile 0 withholds its granules): every XCD's
    workgroup of that column tile times out, arrives 'bad' at the first barrier, and the launch stops before any
    update -- the parameters are bitwise those before the plan and the sticky error word is set.  (The withholding
    hook exists only in the diagnostics build of the kernel, barrier forms 1 and 3; the waits, bad arrivals and stop
    are the production code.)"""
    n, N = 800, 4 * 800
    x, y = synthetic_mnist(N, seed=3)
    nn = NeuralNetwork([784, 100, 10])
    e = MlpEngine(nn.H, "f32", max_cols=n, device="cuda", path="split3")
    e.set_params(*nn.params)
    e.load_dataset(x, y)
    e.set_store_a1(False)
    e._hip_step().xstep_bar = bar
    _plan(e, 0, 2, n, N)  # a good plan first (launch 0)
    torch.cuda.synchronize()
    assert e._hip_step().xstep_used == 1, e._hip_step().xstep_reason
    assert not e.kernel_error()
    before = e.params.clone()
    e.inject_handoff_timeout(row_tile=3, wait_us=2000)
    _plan(e, 0, 3, n, N)
    torch.cuda.synchronize()
    assert e._hip_step().xstep_used == 1
    assert e.kernel_error()
    assert torch.equal(e.params, before)
