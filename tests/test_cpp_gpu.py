"""GPU: the C++ drop-in headers end to end -- tests/cpp/dropin.cpp (reference-style demo
code over include/soundmath/*.h) runs on the device and every output is replayed through
the oracle (tolerances as in the per-engine tests; Delay bit-exact)."""
import os
import subprocess

import numpy as np
import pytest
import scipy.fft

from oracle import OracleFilterbank, OracleOscbank, rel_err
from oracle_bowl import OracleBowl
from oracle_delay import OracleDelaybank
from oracle_osc import OracleAdditive, OracleSinusoids
from oracle_stft import OracleSTFT
from test_cpp_cpu import EXE, build_dropin

pytestmark = pytest.mark.gpu
PI = 3.14159265359


def x_input(n):
    t = np.arange(n)
    return np.sin(0.01 * t) + 0.5 * (((t * 7919) % 13) - 6) / 6.0


@pytest.fixture(scope="module")
def outputs(tmp_path_factory):
    r = build_dropin()
    assert r.returncode == 0, r.stderr[-3000:]
    d = tmp_path_factory.mktemp("dropin")
    p = subprocess.run([EXE, str(d)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "dropin ok" in p.stdout, p.stdout + p.stderr

    def load(name, dtype=np.float64):
        return np.fromfile(os.path.join(d, name + ".bin"), dtype=dtype)
    load.dir = str(d)
    return load


def test_filterbank(outputs):
    """Per-sample operator()/tick() with two bare ticks after t = 40 and 41, then process()."""
    o = OracleFilterbank(2, 16)
    for i in range(16):
        g, R, th = 0.01 * (i + 1), 0.99, 2 * PI * (i + 1) / 40.0
        o.coefficients(i, [g, 0, -g], [-2 * R * np.cos(th), R * R])
    o.boost(np.ones(16))
    o.open()
    x = x_input(1000)
    want = np.empty(1000)
    for t in range(100):
        want[t] = o(x[t])
        o.tick()
        if t in (40, 41):
            o.tick()
    want[100:700] = o.process(x[100:700])
    for t in range(700, 800):
        want[t] = o(x[t])
        o.tick()
    want[800:] = o.process(x[800:])
    assert rel_err(outputs("filterbank"), want) < 1e-9


def test_ffilterbank(outputs):
    """FFilterbank<double, 16, 2>: the same bank in one process() call."""
    o = OracleFilterbank(2, 16)
    for i in range(16):
        g, R, th = 0.01 * (i + 1), 0.99, 2 * PI * (i + 1) / 40.0
        o.coefficients(i, [g, 0, -g], [-2 * R * np.cos(th), R * R])
    o.boost(np.ones(16))
    o.open()
    assert rel_err(outputs("ffilterbank"), o.process(x_input(1000))) < 1e-9


def test_subtractive_resonant_stream(outputs):
    """Filterbank::process_resonant: every band retuned every sample (hz_fb_process_tv)."""
    o = OracleFilterbank(2, 16)
    o.boost(np.ones(16))
    o.open()
    t, b = np.arange(1000)[:, None], np.arange(16)[None, :]
    fr = 110.0 * (b + 1) * (1 + 0.02 * np.sin(0.003 * t + b))
    assert rel_err(outputs("subtractive"), o.process_tv(x_input(1000), 1, fr, 0.999)) < 1e-10   # host sin of the tracks may differ by an ulp


def test_delay_bit_exact(outputs):
    """Per-sample operator()/tick() for 10 samples, two ticks without operator() (the rings move,
    nothing is written: delay.h:92-97), then one block."""
    o = OracleDelaybank(1, 10, 2 * 48000)
    o.coefficients(0, [(0, 1.0)], [(20000, 0.5), (10000, 0.5)])
    x = np.zeros(50000)
    x[0] = 1.0
    y = outputs("delay")
    want = np.concatenate([o.process(x[:10])[0], (o.tick(2), o.process(x[10:])[0])[1]])
    assert np.array_equal(y, want)
    assert list(np.flatnonzero(y)[:3]) == [0, 9998, 19998]


def test_bowl_float(outputs):
    f = [np.float32(100.0) * np.float32(i + 1) * np.float32(1.01) for i in range(8)]
    a = [np.float32(0.01) * np.float32(i + 1) for i in range(8)]
    d = [np.float32(0.5) * np.float32(i + 1) for i in range(8)]
    o = OracleBowl(8, np.float64(f), np.float64(a), np.float64(d), np.float32)
    assert rel_err(outputs("bowl", np.float32), o.fill(2048)) < 1e-5


def test_fourier_host_processor_and_static(outputs):
    """Fourier per sample with the reference's state machine: alternating write/read, a stretch of
    two writes per read, writes alone, reads alone; a host processor of the reference's type."""
    x = x_input(1000)
    o = OracleSTFT(64, 4, 0, 3)   # the C++ hilbert64 callback == the built-in half-band
    yr, yi = [], []
    w = 0
    for t in range(900):
        o.write(x[w]); w += 1
        if 300 <= t < 340:
            o.write(x[w]); w += 1
        if 500 <= t < 540:
            continue
        r, i = o.read(); yr.append(r); yi.append(i)
        if 600 <= t < 640:
            r, i = o.read(); yr.append(r); yi.append(i)
    orr, oi = np.array(yr), np.array(yi)
    assert rel_err(outputs("fourier_re"), orr) < 1e-10
    assert np.max(np.abs(outputs("fourier_im") - oi)) <= 1e-10 * np.max(np.abs(oi))
    s = OracleSTFT(64, 4, 1, 1)
    assert rel_err(outputs("static_re"), s.process_block(x)[0]) < 1e-10


def synth_reference(n, f, phi=0.0, k=2.0 / 48000, shape=lambda p: np.sin(2 * PI * p), events=()):
    """Oscillator<T>::tick (src/oscillator.h:27-38) and Synth::operator() (synth.h:16-17) in plain
    Python floats, op for op (abs taken as fabs)."""
    import math
    s = 0.0 if k == 0 else 2.0 ** (math.log2(2.220446049250313e-16) / (max(0.0, k) * 48000))
    freq = abs(f); tf = freq; ph = max(0.0, phi); tp = ph
    out = []
    ev = dict(events)
    for t in range(n):
        if t in ev:
            kind, v = ev[t]
            if kind == "f":
                tf = v
            else:
                tp += v; tp -= int(tp); tp += 1; tp -= int(tp)
        out.append((shape(ph), ph))
        ph += freq / 48000
        tp += freq / 48000
        freq = tf * (1 - s) + freq * s
        w = (1 - s) * math.sin(2 * PI * (2 * abs(tp - ph) + 0.25))
        ph = w * tp + (1 - w) * ph
        ph -= int(ph)
        tp -= int(tp)
    return out


def test_synth_and_oscillator(outputs):
    """Synth<double>(&cycle, 220) with freqmod / phasemod, Oscillator<double>(3, 0.25, 0.01) and a
    saw Synth: the host classes are exact restatements (bit-identical to the Python replay)."""
    y = outputs("synth")
    a = synth_reference(3000, 220.0, events={1000: ("f", 330.0), 2000: ("p", 0.5)}.items())
    m = synth_reference(3000, 3.0, 0.25, 0.01)
    want = np.array([v for (sa, _), (_, pm) in zip(a, m) for v in (sa, pm)])
    saw = synth_reference(500, 100.0, 0.1, shape=lambda p: 2 * p - 1)
    want = np.concatenate([want, [v for v, _ in saw]])
    assert y.shape == want.shape
    assert np.max(np.abs(y - want)) <= 1e-15 * 8, np.max(np.abs(y - want))


def test_cosine(outputs):
    y = outputs("cosine")
    x = x_input(64)
    assert rel_err(y[:64], scipy.fft.dct(x, type=2)) < 1e-13
    assert rel_err(y[64:], 128 * x) < 1e-13


def test_oscbank(outputs):
    o = OracleOscbank(8)
    for i in range(8):
        o.freqmod(i, 110.0 * (i + 1))
    o.open()
    ref = []
    for _ in range(10):
        z3 = o.phases()[3]
        m = o.fill(1)[0]
        ref += [m.real, m.imag, z3.real]
    mix = o.fill(100)
    ref += list(np.stack([mix.real, mix.imag], -1).reshape(-1))
    assert rel_err(outputs("oscbank"), np.array(ref)) < 1e-9


def test_additive_and_sinusoids(outputs):
    o = OracleAdditive(4, 8, 0.75, 1.0)
    o.makenote(48, 1.0)
    o.makenote(55, 0.5)
    assert rel_err(outputs("additive"), o.fill(2000)) < 1e-8
    s = OracleSinusoids(220.0, 6, 0.8)
    assert rel_err(outputs("sinusoids"), s.fill(1000)) < 1e-8


def test_granulator(outputs):
    """Granulator<double> + Buffer<double>: per-sample write/granny()/request/tick, then process()."""
    from oracle_gran import OracleGranulator
    o = OracleGranulator(3000, 16)
    reqs = [(t, 0.001 * (t % 7), 0.002 + 0.0005 * (t % 11), 0.5 + 0.25 * (t % 5), 0.3, 0.0)
            for t in range(4000) if t % 97 == 0]
    y, voices = o.process(x_input(4000), reqs)
    assert rel_err(outputs("granulator"), y) < 1e-12
    assert list(outputs("granulator_voices").astype(int)) == list(voices)


def test_freezer(outputs):
    """Freezer<64>(4, 1): per-sample operator() with freeze()/unfreeze(), then process()."""
    from oracle_frz import OracleFreezer, libc_srand
    o = OracleFreezer(64, 4, 1.0)
    libc_srand(11)
    y = o.process(x_input(3000), [(400, 1), (900, 0), (1300, 1), (2500, 0)])
    assert np.max(np.abs(outputs("freezer") - y)) <= 1e-9 * np.max(np.abs(y))


def test_heterodyne(outputs):
    """Heterodyne<96> (tests/harmbank.cpp instrument): per-sample operator(), then process()."""
    from huygens_amd import harmbank
    from oracle_het import OracleHet
    n, fa, fs, radii = harmbank()
    o = OracleHet(n, 4, radii, 0.0005, 0.2, 2400, 1, -0.9, 0.0, 3.0)
    o.freqmod(0, np.arange(n), fa)
    o.freqmod(1, np.arange(n), fs)
    o.open(0)
    o.open(1)
    y = o.process(0.3 * x_input(4000))
    assert np.max(np.abs(y)) > 1e-3
    assert np.max(np.abs(outputs("heterodyne") - y)) <= 1e-12


def test_offline_audio_engine(outputs):
    """Heterodyne<96> as the process() callback of the offline Audio engine (src/audio.h
    stand-in): float32 WAV in -> float32 WAV out equals the restatement on the same floats."""
    from huygens_amd import harmbank
    from oracle_het import OracleHet
    from test_audio_cpu import read_f32
    y, rate = read_f32(os.path.join(outputs.dir, "audio_out.wav"))
    n, fa, fs, radii = harmbank()
    o = OracleHet(n, 4, radii, 0.0005, 0.2, 2400, 1, -0.9, 0.0, 3.0)
    o.freqmod(0, np.arange(n), fa)
    o.freqmod(1, np.arange(n), fs)
    o.open(0)
    o.open(1)
    x = (0.3 * x_input(1000)).astype(np.float32).astype(np.float64)
    want = o.process(x).astype(np.float32)
    assert rate == 48000 and y.shape == (1000, 1)
    assert np.max(np.abs(y[:, 0] - want)) <= 1e-6
