"""GPU parity: Delaybank HIP engine vs the restatement -- BIT-EXACT (np.array_equal):
delay indexing is integer work and the kernel rounds every product/sum as the reference
(FP contraction off)."""
import numpy as np
import pytest

from oracle import golden_names, load_golden
from oracle_delay import OracleDelaybank, bank_from_golden

pytestmark = pytest.mark.gpu


def _pair(lines, S, time, dtype):
    from huygens_amd import Delaybank
    return Delaybank(lines, S, time, dtype), OracleDelaybank(lines, S, time, dtype)


@pytest.mark.parametrize("name", golden_names("dly_"))
@pytest.mark.parametrize("split", [0, 1, 2])
def test_golden(gpu_lib, name, split):
    from huygens_amd import Delaybank
    g = load_golden(name)
    b = bank_from_golden(Delaybank, g)
    b.set_split(split)
    y = b.process(g["x"])
    assert np.array_equal(y, g["y"])
    assert b.origin() == int(g["origin"])
    if "mix" in g:
        b2 = bank_from_golden(Delaybank, g)
        assert np.array_equal(b2.process(g["x"], mix=True), g["mix"])


@pytest.mark.parametrize("split", [0, 1, 2])
def test_c5_bank(gpu_lib, split):
    """C5: Delaybank<float,64>(3, 2 SR), fwd {(0,1)}, fb {(10000+37k,.5),(20000+53k,.5)},
    streamed in 1024-sample calls then one long call (ring committed across calls)."""
    g, o = _pair(64, 3, 2 * 48000, np.float32)
    for k in range(64):
        fwd, back = [(0, 1.0)], [(10000 + 37 * k, 0.5), (20000 + 53 * k, 0.5)]
        g.coefficients(k, fwd, back)
        o.coefficients(k, fwd, back)
    g.set_split(split)
    assert g.info() == (10000, 96001)
    rng = np.random.default_rng(5)
    for n in (1024, 1024, 1000, 30000, 70000):
        x = (0.1 * rng.standard_normal(n)).astype(np.float32)
        assert np.array_equal(g.process(x), o.process(x))
    x = (0.1 * rng.standard_normal(4096)).astype(np.float32)
    assert np.array_equal(g.process(x, mix=True), o.process(x, mix=True))
    assert g.origin() == o.origin()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_streamed_mix_calls(gpu_lib, dtype):
    """Streamed mixed calls (C5's pattern): bit-exact against the restatement across calls,
    incl. an age-0 feedback tap (delay = ring size: the partial sum), per-line input, a call
    longer than the shortest feedback age (serial sub-blocks) and one-sample calls."""
    rng = np.random.default_rng(11)
    N, S, time = 70, 3, 3000
    g, o = _pair(N, S, time, dtype)
    for k in range(N):
        fwd = [(int(rng.integers(0, 1800)), float(rng.uniform(-1, 1))) for _ in range(S)]
        back = [(int(rng.integers(1100, 1900)), float(rng.uniform(-0.3, 0.3))) for _ in range(S - 1)]
        if k == 5:
            back[1] = (time + 1, 0.25)   # age 0: reads the sample's own partial sum
        g.coefficients(k, fwd, back)
        o.coefficients(k, fwd, back)
    for i, n in enumerate([1024, 1024, 1000, 64, 1, 1024, 2500, 1024]):
        x = rng.standard_normal((N, n) if i % 3 == 2 else n).astype(dtype)
        assert np.array_equal(g.process(x, mix=True), o.process(x, mix=True)), (i, n)
    assert g.origin() == o.origin()
    x = rng.standard_normal(1024).astype(dtype)   # the per-line outputs after fused calls
    assert np.array_equal(g.process(x), o.process(x))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_random_taps_wrap_and_short_feedback(gpu_lib, dtype):
    """Random taps incl. delays longer than the ring (uint wrap), feedback age 1 (serial
    sub-blocks), zero-time feedback, per-line input, calls longer than the ring."""
    rng = np.random.default_rng(7)
    N, S, time = 9, 4, 300
    g, o = _pair(N, S, time, dtype)
    for k in range(N):
        fwd = [(int(rng.integers(0, 700)), float(rng.uniform(-1, 1))) for _ in range(S)]
        back = [(int(rng.integers(0, 900)), float(rng.uniform(-0.2, 0.2))) for _ in range(S - 1)]
        if k == 3:
            back[0] = (1, 0.3)
        g.coefficients(k, fwd, back)
        o.coefficients(k, fwd, back)
    assert g.info()[0] == 1
    for n in (100, 301, 1500, 7):
        x = rng.standard_normal((N, n)).astype(dtype)
        assert np.array_equal(g.process(x), o.process(x))
    assert g.origin() == o.origin()


def test_modulate_between_calls(gpu_lib):
    g, o = _pair(3, 2, 5000, np.float64)
    for k in range(3):
        for b in (g, o):
            b.coefficients(k, [(0, 1.0), (11 * k, 0.5)], [(800 + k, 0.4)])
    rng = np.random.default_rng(3)
    for step in range(4):
        x = rng.standard_normal(2000)
        assert np.array_equal(g.process(x), o.process(x))
        for b in (g, o):
            b.modulate_forward(1, 1, (100 * step + 3, -0.25))
            b.modulate_back(2, 0, (50 + step, 0.2))
            b.modulate_back(0, 1, (0, 0.7))   # zero-time feedback -> {0,0}


def test_single_delay_and_device_pointers(gpu_lib):
    import torch
    from huygens_amd import Delay
    d = Delay(10, 2 * 48000)
    o = OracleDelaybank(1, 10, 2 * 48000)
    d.coefficients([(0, 1.0)], [(20000, 0.5), (10000, 0.5)])   # tests/delay.cpp:41
    o.coefficients(0, [(0, 1.0)], [(20000, 0.5), (10000, 0.5)])
    x = np.zeros(50000)
    x[0] = 1.0
    ref = o.process(x)[0]
    xt = torch.from_numpy(x).cuda()
    yt = torch.empty_like(xt)
    d.process_device(xt.data_ptr(), yt.data_ptr(), x.size)
    d.synchronize()
    assert np.array_equal(yt.cpu().numpy(), ref)
    assert list(np.flatnonzero(ref)[:4]) == [0, 10000, 20000, 30000]


def test_errors(gpu_lib):
    from huygens_amd import HZError, Delaybank
    b = Delaybank(2, 2, 100)
    with pytest.raises(HZError):
        b.coefficients(0, [(2 ** 31, 1.0)], [])
    with pytest.raises(HZError):
        b.modulate_forward(5, 0, (1, 1.0))
    with pytest.raises(HZError):
        Delaybank(0, 2, 100)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_bare_ticks(gpu_lib, dtype):
    """tick() without operator() (delay.h:92-97) only moves both rings' origins: the skipped slots
    keep the samples written `size` ticks earlier and later reads see those stale values, exactly
    as the reference (round-2 advisor: the drop-in used to run a zero-input sample instead)."""
    rng = np.random.default_rng(13)
    g, o = _pair(5, 3, 700, dtype)
    for k in range(5):
        fwd, back = [(0, 1.0), (350 + k, 0.5)], [(300 + 7 * k, 0.4), (701, 0.2)]
        g.coefficients(k, fwd, back)
        o.coefficients(k, fwd, back)
    for n, ticks in ((900, 3), (1, 1), (250, 700), (1, 0), (1200, 1401), (64, 5)):
        x = (0.1 * rng.standard_normal(n)).astype(dtype)
        assert np.array_equal(g.process(x), o.process(x))
        g.tick(ticks)
        o.tick(ticks)
        assert g.origin() == o.origin()
    x = (0.1 * rng.standard_normal(2000)).astype(dtype)
    assert np.array_equal(g.process(x), o.process(x))
