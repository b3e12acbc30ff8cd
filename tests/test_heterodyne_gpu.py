"""GPU parity: the heterodyne-chain HIP engine vs the restatement (oracle/hz_oracle_het.c).

Every channel's state (oscillator phasors, Slidebank stages, RMS sums and history, latch
flags, Stickbank outputs) is bit-exact: the kernel evaluates each channel without FMA
contraction in the reference's operation order.  The output differs only by the order of
the channel sum (Mixer) and device vs libm atan: |gpu - oracle| <= TOL (the output is an
atan limiter, |y| < 1)."""

import numpy as np
import pytest

from oracle_het import OracleHet

pytestmark = pytest.mark.gpu
TOL = 1e-12


def bursty(n, seed, amp=0.2):
    """Noise plus a chirp under an on/off envelope, so the latches engage and release."""
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    env = (np.sin(2 * np.pi * t / 1500.0) > 0.2).astype(float)
    return amp * env * (np.sin(2 * np.pi * (200 + 0.05 * t) * t / 48000) + 0.3 * rng.standard_normal(n))


def make_pair(N, order=4, width=240, sorder=1, srad=-0.9, thresh=0.0005, ratio=0.2, dry=0.1, gain=3.0, seed=0,
              imag=0.0, active=1.0):
    from huygens_amd import Heterodyne
    rng = np.random.default_rng(seed)
    radii = np.zeros(2 * N)
    radii[0::2] = rng.uniform(0.95, 0.999, N)
    radii[1::2] = imag * rng.standard_normal(N)
    args = (N, order, radii, thresh, ratio, width, sorder, srad, dry, gain)
    g, o = Heterodyne(*args), OracleHet(*args)
    fa = rng.uniform(40, 6000, N) * np.where(rng.random(N) < 0.5, -1, 1)
    fs = -2 * fa
    idx = np.arange(N)
    acts = [idx[rng.random(N) < active] for _ in range(2)]
    for h in (g, o):
        h.freqmod(0, idx, fa)
        h.freqmod(1, idx, fs)
        for b in (0, 1):
            h.activate(b, acts[b])
    return g, o


def assert_states_equal(g, o):
    for what in range(7):
        a, b = g.state(what), o.state(what)
        assert np.array_equal(a, b), f"state {what}: max diff {np.max(np.abs(a - b))}"


def assert_close(gy, oy):
    """|gy - oy| <= TOL; a chain that diverges (an unstable Stickbank) must do so at the same samples."""
    assert np.array_equal(np.isfinite(gy), np.isfinite(oy))
    f = np.isfinite(oy)
    assert np.max(np.abs(gy[f] - oy[f]), initial=0.0) <= TOL


@pytest.mark.parametrize("N,order,width,sorder,imag,active", [(1, 1, 48, 1, 0.0, 1.0), (96, 4, 2400, 1, 0.0, 1.0),
                                                              (300, 3, 100, 2, 0.01, 0.6), (513, 8, 33, 4, 0.0, 0.9),
                                                              (64, 2, 4, 3, 0.02, 1.0), (7, 5, 9, 1, 0.0, 0.5)])
def test_chain_vs_oracle(gpu_lib, N, order, width, sorder, imag, active):
    # Stickbank(order, rad) is stable for these radii (its feedback is (z + rad)^order read backwards)
    srad = {1: -0.9, 2: -0.2, 3: -0.2, 4: -0.1}[sorder]
    g, o = make_pair(N, order=order, width=width, sorder=sorder, srad=srad, imag=imag, active=active, seed=N)
    x = bursty(9000, N)
    for a, b in [(0, 1), (1, 4000), (4000, 4031), (4031, 9000)]:   # ragged calls, a one-sample call
        assert_close(g.process(x[a:b]), o.process(x[a:b]))
    assert_states_equal(g, o)


def test_harmbank_instrument(gpu_lib):
    """tests/harmbank.cpp's 96-channel instrument: both banks open, order 4, SR/20 RMS."""
    from huygens_amd import Heterodyne, harmbank
    n, fa, fs, radii = harmbank()
    args = (n, 4, radii, 0.0005, 0.2, 2400, 1, -0.9, 0.0, 3.0)
    g, o = Heterodyne(*args), OracleHet(*args)
    for h in (g, o):
        h.freqmod(0, np.arange(n), fa)
        h.freqmod(1, np.arange(n), fs)
        h.open(0)
        h.open(1)
    x = bursty(12000, 7, amp=0.3)
    gy, oy = g.process(x), o.process(x)
    assert np.max(np.abs(oy)) > 1e-3
    assert_close(gy, oy)
    assert_states_equal(g, o)


def test_reconfigure_between_calls(gpu_lib):
    """freqmod, deactivate and Slidebank::setup between calls (setup zeroes the stages)."""
    N = 200
    g, o = make_pair(N, order=3, width=64, seed=3)
    x = bursty(6000, 3)
    assert_close(g.process(x[:2000]), o.process(x[:2000]))
    idx = np.random.default_rng(4).choice(N, 50, replace=False)
    hz = np.random.default_rng(5).uniform(100, 300, 50)
    for h in (g, o):
        h.freqmod(1, idx, hz)
        h.activate(0, idx[:20], on=False)
    assert_close(g.process(x[2000:4000]), o.process(x[2000:4000]))
    radii = np.zeros(2 * N)
    radii[0::2] = 0.97
    for h in (g, o):
        h.setup(5, radii)
        h.open(1, on=False)
    assert_close(g.process(x[4000:]), o.process(x[4000:]))
    assert_states_equal(g, o)


def test_launch_splits(gpu_lib, monkeypatch):
    """A call split over several launches (HZ_HET_CHUNK) equals one call."""
    monkeypatch.setenv("HZ_HET_CHUNK", "777")
    g, o = make_pair(500, order=4, width=300, sorder=2, srad=-0.2, seed=9)
    x = bursty(5000, 9)
    assert_close(g.process(x), o.process(x))
    assert_states_equal(g, o)


def test_unstable_stickbank_diverges_alike(gpu_lib):
    """Stickbank(2, -0.9) is unstable (root 1.8): both blow up to inf / NaN at the same samples."""
    g, o = make_pair(32, order=2, width=50, sorder=2, srad=-0.9, seed=13)
    x = bursty(4000, 13)
    gy, oy = g.process(x), o.process(x)
    assert not np.isfinite(oy).all()
    assert_close(gy, oy)


def test_device_pointers(gpu_lib):
    import torch
    g, o = make_pair(128, seed=11)
    x = bursty(3000, 11)
    xt = torch.from_numpy(x).cuda()
    yt = torch.empty_like(xt)
    g.set_stream(torch.cuda.current_stream().cuda_stream)
    g.process_device(xt.data_ptr(), yt.data_ptr(), x.size)
    torch.cuda.synchronize()
    assert_close(yt.cpu().numpy(), o.process(x))


def test_wide_bank_channel_states(gpu_lib):
    """65536 channels: a random subset's states equal a restatement of just those channels
    (channels are independent up to the mix), and the full mix matches the restatement."""
    from huygens_amd import Heterodyne
    N, n = 65536, 2048
    rng = np.random.default_rng(12)
    radii = np.zeros(2 * N)
    radii[0::2] = rng.uniform(0.95, 0.999, N)
    fa = rng.uniform(40, 8000, N)
    args = dict(thresh=0.0005, ratio=0.2, width=240, stick_order=1, stick_rad=-0.9, dry=0.0, gain=3.0 / 256)
    g = Heterodyne(N, 4, radii, **args)
    g.freqmod(0, np.arange(N), fa)
    g.freqmod(1, np.arange(N), -2 * fa)
    g.open(0)
    g.open(1)
    x = bursty(n, 12)
    gy = g.process(x)
    sub = np.sort(rng.choice(N, 64, replace=False))
    rs = np.zeros(128)
    rs[0::2] = radii[0::2][sub]
    o = OracleHet(64, 4, rs, 0.0005, 0.2, 240, 1, -0.9, 0.0, 3.0 / 256)
    o.freqmod(0, np.arange(64), fa[sub])
    o.freqmod(1, np.arange(64), -2 * fa[sub])
    o.open(0)
    o.open(1)
    o.process(x)
    for what, width in [(0, 2), (1, 2), (2, 8), (3, 1), (4, 2), (5, 2)]:
        assert np.array_equal(g.state(what).reshape(N, width)[sub], o.state(what).reshape(64, width))
    full = OracleHet(N, 4, radii, 0.0005, 0.2, 240, 1, -0.9, 0.0, 3.0 / 256)
    full.freqmod(0, np.arange(N), fa)
    full.freqmod(1, np.arange(N), -2 * fa)
    full.open(0)
    full.open(1)
    assert_close(gy, full.process(x))


def test_errors(gpu_lib):
    from huygens_amd import Heterodyne, HZError
    r = np.zeros(8)
    with pytest.raises(HZError):
        Heterodyne(4, 9, r)        # Slidebank order > 8
    with pytest.raises(HZError):
        Heterodyne(4, 2, r, stick_order=5)
    with pytest.raises(HZError):
        Heterodyne(4, 2, r, width=0)
    with pytest.raises(ValueError):
        Heterodyne(4, 2, np.zeros(6))
    g = Heterodyne(4, 2, r)
    with pytest.raises(HZError):
        g.freqmod(2, [0], [1.0])
    with pytest.raises(HZError):
        g.setup(9, r)
    assert g.process(np.zeros(0)).size == 0
