"""CPU: the Granulator restatement (oracle/hz_oracle_gran.c) against closed forms and an
independent pure-Python restatement of src/granulator.h:51-104 + src/buffer.h:33-47.

Parity status: the reference holds no fixtures or known answers for Granulator; these
checks pin the restatement by hand-derived cases (grain lifetime, voice allocation, the
uint32 ring wrap) and by a second, independently written per-sample model."""
import math

import numpy as np
import pytest

from huygens_amd._lib import header_symbols
from oracle_gran import OracleGranulator

PI = 3.14159265359   # src/includes.h:30
SR = 48000


class PyGranulator:
    """Pure-Python per-sample Granulator<double> + Buffer<double> (small cases only)."""

    def __init__(self, size, polyphony):
        self.size = size + (1 if size == 0 else 0)
        self.data = [0.0] * self.size
        self.origin = 0
        self.P = polyphony
        self.active = [False] * polyphony
        self.ticks = [0] * polyphony
        self.par = [None] * polyphony

    def request(self, offset, size, speed, gain, pan=0.0):
        if size == 0:
            return -1
        lo = size * (speed - 1)
        offset = lo if offset < lo else offset
        for v in range(self.P):
            if not self.active[v]:
                self.par[v] = (SR * offset, SR * size, speed, gain)
                self.active[v] = True
                self.ticks[v] = 0
                return v
        return -1

    def read(self, position):
        center = int(position)          # C truncation toward zero
        before = center + 1
        disp = position - center
        i0 = ((self.origin - center) % (1 << 32) + self.size) % (1 << 32) % self.size
        i1 = ((self.origin - before) % (1 << 32) + self.size) % (1 << 32) % self.size
        return self.data[i0] * (1 - disp) + self.data[i1] * disp

    def sample(self):
        out = 0.0
        for v in range(self.P):
            if self.active[v]:
                offs, sizes, speed, gain = self.par[v]
                t = self.ticks[v]
                phase = float(t) / sizes
                out += gain * self.read(offs + (1 - speed) * t) * (0.5 * (1 - math.cos(2 * PI * phase)))
                if t >= sizes:
                    self.active[v] = False
        return out

    def tick(self):
        self.origin = (self.origin + 1) % self.size
        for v in range(self.P):
            if self.active[v]:
                self.ticks[v] += 1


def test_single_grain_closed_form():
    """Constant input 1, speed 1: y = gain * hann(ticks / sizes) for ticks 0..ceil(sizes)."""
    o = OracleGranulator(1000, 4)
    size = 10.5 / SR
    assert o.request(0.0, size, 1.0, 0.5) == 0
    y, _ = o.process(np.ones(20))
    sizes = SR * size
    expect = [0.5 * 1.0 * (0.5 * (1 - math.cos(2 * PI * (k / sizes)))) for k in range(12)] + [0.0] * 8
    assert np.array_equal(y, np.array(expect))
    assert o.activity() == 0


def test_voice_allocation_and_reuse():
    o = OracleGranulator(100, 2)
    assert o.request(0, 2.0 / SR, 1, 1) == 0
    assert o.request(0, 5.0 / SR, 1, 1) == 1
    assert o.request(0, 1.0 / SR, 1, 1) == -1           # polyphony exhausted
    assert o.request(0, 0.0, 1, 1) == -1                # size == 0 (granulator.h:53-54)
    # voice 0 reads ticks 0, 1, 2 (deactivated at the third read), so it is free after sample 2
    _, v = o.process(np.zeros(4), [(1, 0, 1.0 / SR, 1, 1, 0), (2, 0, 1.0 / SR, 1, 1, 0)])
    assert list(v) == [-1, 0]


def test_offset_clamp():
    """offset = max(offset, size (speed - 1)) so the read never looks into the future."""
    o, p = OracleGranulator(64, 1), PyGranulator(64, 1)
    x = np.arange(1, 41, dtype=float)
    assert o.request(0.0, 8.0 / SR, 3.0, 1.0) == p.request(0.0, 8.0 / SR, 3.0, 1.0) == 0
    ref = []
    for xi in x:
        p.data[p.origin] = xi
        ref.append(p.sample())
        p.tick()
    assert np.array_equal(o.process(x)[0], np.array(ref))


@pytest.mark.parametrize("size,P,seed", [(37, 4, 0), (100, 8, 1), (5, 3, 2)])
def test_restatement_vs_python(size, P, seed):
    """Random grains (negative speeds, reads past the ring: the uint32 wrap) bit for bit."""
    rng = np.random.default_rng(seed)
    n = 400
    x = rng.standard_normal(n)
    reqs = []
    for i in sorted(rng.integers(0, n, 30)):
        reqs.append((int(i), float(rng.uniform(0, 3 * size / SR)), float(rng.uniform(1, 40) / SR),
                     float(rng.uniform(-2, 3)), float(rng.uniform(0, 1)), 0.0))
    o, p = OracleGranulator(size, P), PyGranulator(size, P)
    y, voices = o.process(x, reqs)
    ref, rv, k = [], [], 0
    for i in range(n):
        p.data[p.origin] = x[i]
        ref.append(p.sample())
        while k < len(reqs) and reqs[k][0] == i:
            rv.append(p.request(*reqs[k][1:]))
            k += 1
        p.tick()
    assert list(voices) == rv
    assert np.array_equal(y, np.array(ref))


def test_abi_declares_granulator():
    syms = header_symbols()
    for s in ("hz_gran_create", "hz_gran_request", "hz_gran_process", "hz_gran_process_device",
              "hz_gran_activity", "hz_gran_destroy"):
        assert s in syms
