"""GPU parity of the per-sample Fourier / StaticSTFT API (hz_stft_write / read / forward /
backward / process_slot): the reference's own slot state machine (src/fourier.h:102-177) with the
slot transforms and device processors on the GPU, against the restatement's write / read, in any
order and number -- two writes before a read, reads without writes, direct forward(i) /
process(i) / backward(i) calls -- and the stateful host processor of tests/demo.cpp.
Tolerance as tests/test_stft_gpu.py (device FFT vs the oracle's long double DFT)."""
import time

import numpy as np
import pytest

from oracle_stft import OracleSTFT

pytestmark = pytest.mark.gpu
TOL = 1e-10


def pair(N, laps, window, proc, callback=None, ocallback=None):
    from huygens_amd import Fourier
    g = Fourier(callback if callback is not None else proc, N, laps, window)
    o = OracleSTFT(N, laps, window, proc, callback=ocallback)
    return g, o


def c4_like(n, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 48000.0
    x = 0.1 * rng.standard_normal(n)
    for k in range(1, 5):
        x += 0.5 * np.sin(2 * np.pi * 900 * k ** 1.5 * t)
    return x


def lockstep(g, o, ops, xs):
    """ops: 'w' write, 'r' read, ('f'|'b'|'p', slot); returns the max error of the reads"""
    outs_g, outs_o = [], []
    k = 0
    for op in ops:
        if op == 'w':
            g.write(xs[k].real, xs[k].imag)
            o.write(xs[k].real, xs[k].imag)
            k += 1
        elif op == 'r':
            outs_g.append(g.read())
            outs_o.append(o.read())
        else:
            kind, slot = op
            getattr(g, {"f": "forward", "b": "backward", "p": "process"}[kind])(slot)
            getattr(o, {"f": "forward", "b": "backward", "p": "process"}[kind])(slot)
    a, b = np.array(outs_g), np.array(outs_o)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)) if len(b) else 0.0


@pytest.mark.parametrize("N,laps,window,proc", [(64, 4, 0, 0), (64, 4, 1, 1), (256, 8, 0, 2), (128, 2, 0, 3),
                                                (1024, 8, 0, 0)])
def test_alternating_write_read(gpu_lib, N, laps, window, proc):
    g, o = pair(N, laps, window, proc)
    n = 5 * N + 17
    x = c4_like(n, N) + 0.01j * np.random.default_rng(N).standard_normal(n)
    err = lockstep(g, o, ['w', 'r'] * n, x)
    assert err < TOL, err


def test_irregular_calls(gpu_lib):
    """Writes and reads in any number: the two heads run independently (a slot turns to reading
    on its N-th write and back on its N-th read), as in the reference."""
    N, laps = 64, 4
    g, o = pair(N, laps, 0, 0)
    rng = np.random.default_rng(3)
    ops = []
    writes = 0
    for _ in range(600):
        r = rng.random()
        if r < 0.15:
            ops += ['w', 'w']
            writes += 2
        elif r < 0.25:
            ops += ['r']
        else:
            ops += ['w', 'r']
            writes += 1
    x = rng.standard_normal(writes) + 1j * rng.standard_normal(writes)
    err = lockstep(g, o, ops, x)
    assert err < TOL, err


def test_direct_slot_operations(gpu_lib):
    """forward(i) / process(i) / backward(i) called by the user between samples act on the
    slot buffers the state machine uses (fourier.h:130-144 are public)."""
    N, laps = 64, 2
    g, o = pair(N, laps, 1, 1)
    rng = np.random.default_rng(4)
    x = rng.standard_normal(2000) + 0j
    ops = []
    for t in range(1000):
        ops += ['w', 'r']
        if t % 97 == 5:
            ops += [('f', t % (2 * laps)), ('p', t % (2 * laps))]
        if t % 131 == 7:
            ops += [('b', (t + 1) % (2 * laps))]
    err = lockstep(g, o, ops, x)
    assert err < TOL, err


def test_stateful_host_processor(gpu_lib):
    """A host processor with state between frames (tests/demo.cpp:49-80 shape), per sample."""
    N, laps = 128, 4
    state_g, state_o = {"k": 0}, {"k": 0}

    def gate_g(a, b):   # keep the bins above the running frame count's threshold (state)
        state_g["k"] += 1
        thr = 0.05 * (1 + state_g["k"] % 3)
        m = np.abs(a) > thr * np.max(np.abs(a))
        b[:] = np.where(m, a, 0)
        return 0

    def gate_o(pin, pout):
        state_o["k"] += 1
        a = np.ctypeslib.as_array(pin, shape=(2 * N,)).view(np.complex128)
        b = np.ctypeslib.as_array(pout, shape=(2 * N,)).view(np.complex128)
        thr = 0.05 * (1 + state_o["k"] % 3)
        m = np.abs(a) > thr * np.max(np.abs(a))
        b[:] = np.where(m, a, 0)
        return 0

    g, o = pair(N, laps, 0, 4, callback=gate_g, ocallback=gate_o)
    x = c4_like(6 * N, 5) + 0j
    err = lockstep(g, o, ['w', 'r'] * len(x), x)
    assert state_g["k"] == state_o["k"] > 10
    assert err < 1e-9, err


def test_modes_exclusive(gpu_lib):
    """An object runs per sample or by blocks: the other kind is refused with HZ_E_STATE."""
    from huygens_amd import Fourier
    from huygens_amd._lib import HZError
    f = Fourier(0, 64, 4)
    f.write(1.0)
    with pytest.raises(HZError, match="HZ_E_STATE"):
        f.process_block(np.ones(10))
    g = Fourier(0, 64, 4)
    g.process_block(np.ones(10))
    with pytest.raises(HZError, match="HZ_E_STATE"):
        g.write(1.0)
    with pytest.raises(HZError, match="HZ_E_RANGE"):
        f.forward(8)


def test_spectral_cpp_rate(gpu_lib):
    """tests/spectral.cpp's configuration (N = 8192, laps = 32, the 625 gate) per sample through
    the C ABI: above 48,000 samples/s (real time)."""
    from huygens_amd import Fourier
    f = Fourier(2, 8192, 32)
    x = c4_like(48000, 6)
    for v in x[:2000]:
        f.write(v)
        f.read()
    t0 = time.perf_counter()
    for v in x[2000:]:
        f.write(v)
        f.read()
    rate = 46000 / (time.perf_counter() - t0)
    print(f"spectral.cpp per-sample: {rate:.0f} samples/s")
    assert rate > 48000, rate
