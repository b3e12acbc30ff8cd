"""CPU: the per-sample coefficient restatement (orc_fb_process_tv, oracle/hz_oracle.c) --
SURVEY.md 8(f) row 4, Subtractive ALLINONE / ONEPERVOICE (src/subtractive.h:215-228, 300-317).

The stream path is the pinned Filterbank restatement (orc_fb_sample / tick) with every band's
coefficients set before each sample, so it is checked against that path driven by per-sample
coefficients() calls; resonant() (subtractive.h:240-249) against Python's complex arithmetic
(the same Smith quotient as libgcc's __divdc3, abs = hypot).  Parity unpinned by reference
fixtures (the reference holds none for Subtractive)."""
import math

import numpy as np
import pytest

from huygens_amd._lib import header_symbols
from oracle import OracleFilterbank

PI = 3.14159265359
SR = 48000


def coeff_stream(n, N, O, seed):
    """[n][2O+1][N]: slowly gliding stable resonators (poles radius < 1)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n)[:, None]
    f0 = rng.uniform(100, 5000, N)[None, :] * (1 + 0.3 * np.sin(2 * np.pi * t / max(n, 1) + rng.uniform(0, 6, N)))
    R = 0.995
    st = np.zeros((n, 2 * O + 1, N))
    if O == 0:
        st[:, 0, :] = rng.uniform(0.1, 1, N)
        return st
    st[:, 0, :] = 1 - R
    if O >= 2:
        st[:, 2, :] = -(1 - R)
        st[:, O + 1, :] = -2 * R * np.cos(2 * np.pi * f0 / SR)
        st[:, O + 2, :] = R * R
    else:
        st[:, O + 1, :] = -R * np.cos(2 * np.pi * f0 / SR)
    for k in range(3, O + 1):
        st[:, k, :] = 0.01 * k
    return st


def make(O, N, seed):
    fb = OracleFilterbank(O, N, 0.1, 1.0)
    rng = np.random.default_rng(seed)
    fb.boost(list(rng.uniform(0.5, 1.5, N)))
    fb.open()
    return fb


@pytest.mark.parametrize("O", [0, 1, 2, 3, 4])
def test_stream_equals_per_sample_coefficient_calls(O):
    N, n = 7, 300
    st = coeff_stream(n, N, O, O)
    x = np.random.default_rng(O).standard_normal(n)
    a, b = make(O, N, 1), make(O, N, 1)
    ya = a.process_tv(x, 0, st)
    yb = np.zeros(n)
    for t in range(n):
        for band in range(N):
            b.coefficients(band, st[t, :O + 1, band], st[t, O + 1:, band])
        yb[t] = b.process(x[t:t + 1])[0]
    assert np.array_equal(ya, yb)


def test_constant_stream_is_the_plain_filterbank():
    O, N, n = 2, 9, 500
    st = np.repeat(coeff_stream(1, N, O, 5), n, axis=0)
    x = np.random.default_rng(5).standard_normal(n)
    a, b = make(O, N, 2), make(O, N, 2)
    for band in range(N):
        b.coefficients(band, st[0, :O + 1, band], st[0, O + 1:, band])
    assert np.array_equal(a.process_tv(x, 0, st), b.process(x))


@pytest.mark.parametrize("f,Q", [(440.0, 0.99999), (30.0, 0.999), (12000.0, 0.9), (23999.0, 0.99)])
def test_resonant_matches_complex_arithmetic(f, Q):
    from oracle import lib
    c2, s2 = math.cos(4 * PI * f / SR), math.sin(4 * PI * f / SR)
    maximum = 1.0 / (Q - 1) - 1.0 / (Q - complex(c2, 0) - 1j * s2)
    want = 1 / math.sqrt(abs(maximum))
    assert lib().orc_resonant(f, Q) == pytest.approx(want, rel=1e-15)


def test_resonant_stream_sets_subtractive_coefficients():
    import ctypes as C
    from oracle import lib
    f, R = 523.25, 0.9999
    fwd, back = (C.c_double * 3)(), (C.c_double * 2)()
    lib().orc_fb_resonant_coefficients(f, R, fwd, back)
    g = lib().orc_resonant(f, R)
    assert list(fwd) == [g, 0.0, -g]
    assert list(back) == [-2 * R * math.cos(2 * PI * f / SR), R * R]


def test_abi_declares_tv():
    syms = header_symbols()
    assert "hz_fb_process_tv" in syms and "hz_fb_process_tv_device" in syms
