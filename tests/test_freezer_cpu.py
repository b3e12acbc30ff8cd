"""CPU: the Freezer restatement (oracle/hz_oracle_frz.c) against closed forms and an
independent numpy restatement of src/fourier.h:236-562 (FFrame, IFrame, DFrame, Freezer).

Parity status: the reference holds no fixtures for Freezer; these checks pin the
restatement (the dry Delay path exactly, the frozen path against a second model to 1e-12)."""
import ctypes as C

import numpy as np
import pytest

from huygens_amd._lib import header_symbols
from oracle_frz import OracleFreezer, libc_srand

PI = 3.14159265359
_libc = C.CDLL(None)


def halfhann(p):
    return np.sqrt(0.5 * (1 - np.cos(2 * PI * p)))


class PyFreezer:
    """numpy restatement, per sample (small N only); rand() from libc like the reference."""

    def __init__(self, N, laps, width):
        width, laps = max(width, 1.0), max(laps, 2)
        self.N, self.stride = N, N // laps
        self.M = int(width * laps) + 1
        self.size = self.M * self.stride
        M = self.M
        self.data = np.zeros((M, N), complex)
        self.norms = np.zeros((M, N))
        self.phases = np.zeros((M, N))
        self.dn = np.zeros((M, N))
        self.dp = np.zeros((M, N))
        self.idata = np.zeros((M, N), complex)
        self.iqueue = [0] * M
        self.iindex = self.origin = self.readhead = self.excluded = 0
        self.frozen = False
        self.din = np.zeros(N + 1)
        self.dorigin = 0
        self.win = halfhann(np.arange(N) / N)

    def write(self, x):
        for i in range(self.M):
            spot = (self.origin - i * self.stride) % self.size
            if spot < self.N:
                self.data[i, spot] = complex(self.win[spot] * x, self.win[spot] * 0.0)
            if spot == 0:
                j = (i - 1) % self.M
                X = np.fft.fft(self.data[j])
                self.norms[j] = X.real ** 2 + X.imag ** 2
                self.phases[j] = np.arctan2(X.imag, X.real)
        self.origin = (self.origin + 1) % self.size

    def freeze(self):
        if not self.frozen:
            self.excluded = self.origin // self.stride
            for i in range(1, self.M - 1):
                d = (self.excluded + i) % self.M
                s = (d + 1) % self.M
                self.dn[d] = self.norms[s]
                self.dp[d] = self.phases[s] - self.phases[d]
        self.readhead = 0
        self.frozen = True

    def unfreeze(self):
        self.frozen = False

    def sample(self, x):
        self.write(x)
        out = 0.0
        if self.frozen:
            for i in range(self.M):
                spot = (self.readhead - i * self.stride) % self.size
                if spot < self.N:
                    out += self.idata[self.iqueue[i], spot].real * self.win[spot]
                if spot == 0:
                    nxt = _libc.rand() % (self.M - 2)
                    if nxt >= self.excluded:
                        nxt += 2
                    self.iindex = (self.iindex + 1) % self.M
                    self.iqueue[self.iindex] = nxt
                    voc = np.fmod(self.dp[nxt], 2 * PI)
                    r = np.sqrt(self.dn[nxt])
                    self.idata[nxt] = np.fft.ifft(r * np.cos(voc) + 1j * r * np.sin(voc)) * self.N
            self.readhead = (self.readhead + 1) % self.size
            out /= self.N
        else:
            o = self.dorigin
            self.din[o] = x
            out = self.din[(o + 1) % (self.N + 1)]
        self.dorigin = (self.dorigin + 1) % (self.N + 1)
        return out

    def process(self, x, events=()):
        ev = list(events)
        y, k = np.zeros(len(x)), 0
        for i, xi in enumerate(x):
            while k < len(ev) and ev[k][0] == i:
                self.freeze() if ev[k][1] else self.unfreeze()
                k += 1
            y[i] = self.sample(xi)
        return y


def test_dry_path_is_an_n_sample_delay():
    o = OracleFreezer(64, 4, 1.0)
    x = np.random.default_rng(0).standard_normal(500)
    assert np.array_equal(o.process(x), np.r_[np.zeros(64), x[:-64]])


def test_dry_path_after_a_freeze_reads_the_stale_ring():
    """While frozen the Delay's input ring is not written (fourier.h:528-533), only ticked."""
    N = 16
    o = OracleFreezer(N, 2, 1.0)
    x = np.arange(1, 301, dtype=float)
    libc_srand(3)
    y = o.process(x, [(100, 1), (130, 0)])
    unfrozen = np.ones(300, bool)
    unfrozen[100:130] = False
    for t in range(130, 180):   # closed form of the ring read (t + 1) mod (N + 1)
        tau = t - N
        while tau >= 0 and not unfrozen[tau]:
            tau -= N + 1
        assert y[t] == (x[tau] if tau >= 0 else 0.0)


@pytest.mark.parametrize("N,laps,width,seed", [(8, 2, 1.0, 1), (16, 4, 1.0, 2), (32, 3, 2.5, 3), (16, 2, 3.0, 4)])
def test_restatement_vs_numpy(N, laps, width, seed):
    rng = np.random.default_rng(seed)
    n = 900
    x = rng.standard_normal(n)
    events = [(37, 1), (150, 1), (211, 0), (212, 0), (400, 1), (777, 0), (778, 1)]
    o, p = OracleFreezer(N, laps, width), PyFreezer(N, laps, width)
    libc_srand(seed)
    yo = o.process(x, events)
    libc_srand(seed)
    yp = p.process(x, events)
    assert np.max(np.abs(yo - yp)) <= 1e-12 * max(1.0, np.max(np.abs(yp)))


def test_abi_declares_freezer():
    syms = header_symbols()
    for s in ("hz_frz_create", "hz_frz_process", "hz_frz_process_device", "hz_frz_freeze", "hz_frz_unfreeze"):
        assert s in syms
