"""Gain setters while the bank streams (the reference demos retarget mix() on
every MIDI note, /root/reference/tests/filterbank.cpp:217-252, smoothed by src/filterbank.h:173).

The gain smoothers share s_g, so after mix() the mixdown is the stationary convolution with the new
targets' response plus s_g^(t - dref) times a convolution with the transient response
h_D = sum_n D_n r_n (hz_fb_stream.hip fb_stream_gain_setter): the streaming engine keeps running, a
second launch per block adds the transient term, and both responses are updated per setter from the
per-band responses kept in HBM.  Every 1024-sample block against the restatement (which runs the
reference recurrence sample by sample through the same setters), per-block bound 1e-7 as the C2
streaming tests."""
import numpy as np
import pytest

from golden.spec_numpy import resonant_coefficients
from oracle import OracleFilterbank
from test_c2_pinned_gpu import block_errors

pytestmark = pytest.mark.gpu
B = 1024


def _pair(N, kp=0.1, kg=1.0):
    from huygens_amd import Filterbank
    fwd, back = resonant_coefficients(N, 0.999, 1.0)
    g, o = Filterbank(2, N, kp, kg), OracleFilterbank(2, N, kp, kg)
    for fb in (g, o):
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
        fb.boost(np.ones(N))
        fb.open()
    g.tune_response(0, 1)   # (small test bank: stationary whenever legal)
    return g, o


def _stationary(g, o, rng):
    from huygens_amd._lib import HZ_FB_PATH_RESPONSE
    for _ in range(8):
        x = rng.uniform(-1, 1, 60000)
        err, _ = block_errors(g.process(x), o.process(x))
        assert err.max() <= 1e-7
        if g.last_path() == HZ_FB_PATH_RESPONSE:
            return
    raise AssertionError(g.last_path())


@pytest.mark.parametrize("N", [512, 1024])
def test_mix_churn_streams(gpu_lib, N):
    from huygens_amd._lib import HZ_FB_PATH_STREAM
    g, o = _pair(N)
    rng = np.random.default_rng(N)
    _stationary(g, o, rng)
    worst, streamed = 0.0, 0
    calls0 = g.stream_info()[2]
    for blk in range(150):
        if blk < 80 and blk % 5 == 2:   # 9 bands retuned every ~100 ms (tests/filterbank.cpp:217-252)
            bands = rng.choice(N, 9, replace=False)
            vals = rng.uniform(0.3, 1.7, 9)
            for b, v in zip(bands, vals):
                g.mix(int(b), float(v))
                o.mix(int(b), float(v))
        if blk == 40:   # one all-band setter too (Filterbank::mix(vector))
            v = rng.uniform(0.8, 1.2, N)
            g.mix(v)
            o.mix(v)
        x = rng.uniform(-1, 1, B)
        yg, yo = g.process(x), o.process(x)
        err, _ = block_errors(yg, yo)
        worst = max(worst, float(err.max()))
        streamed += g.last_path() == HZ_FB_PATH_STREAM
    assert worst <= 1e-7, worst
    # every block streamed: the setters did not send the bank back to the per-band engines
    assert streamed == 150 and g.stream_info()[2] - calls0 == 150
    # then a long call (the per-band / stationary engines take over from the streamed state)
    x = rng.uniform(-1, 1, 30000)
    err, _ = block_errors(g.process(x), o.process(x))
    assert err.max() <= 1e-7
    st_g, st_o = g.get_state(), o.get_state()
    assert np.max(np.abs(st_g - st_o)) <= 1e-8 * max(1.0, np.max(np.abs(st_o)))


def test_mix_churn_then_boost(gpu_lib):
    """a boost() (pre-amps) while a gain transient streams falls back to the per-band engines, exactly"""
    g, o = _pair(256)
    rng = np.random.default_rng(5)
    _stationary(g, o, rng)
    for blk in range(30):
        if blk == 3:
            g.mix(10, 0.5)
            o.mix(10, 0.5)
        if blk == 12:
            g.boost(20, 1.5)
            o.boost(20, 1.5)
        x = rng.uniform(-1, 1, B)
        err, _ = block_errors(g.process(x), o.process(x))
        assert err.max() <= 1e-7, blk
