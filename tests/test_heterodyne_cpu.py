"""CPU: the heterodyne-chain restatement (oracle/hz_oracle_het.c) against closed forms and an
independent numpy restatement of tests/harmbank.cpp:77-101 (src/oscbank.h, modbank.h,
slidebank.h, rmsbank.h, latchbank.h, stickbank.h, mixer.h).

Parity status: the reference holds no fixtures for this chain and is unbuildable here
(Eigen absent); these checks pin the restatement -- per-channel state bit-exact against the
numpy model (both without FMA, in the reference's operation order), the mix to 1e-13."""
import math

import numpy as np
import pytest

from huygens_amd._lib import header_symbols
from huygens_amd.heterodyne import harmbank
from oracle_het import OracleHet

PI = 3.14159265359
SR = 48000


class PyHet:
    """numpy restatement over real arrays (no complex128 kernels: their FMA use is unspecified)."""

    def __init__(self, N, order, radii, thresh, ratio, width, sorder, srad, dry, gain):
        self.N, self.O, self.W, self.S = N, max(1, order), width, max(1, sorder)
        self.rr, self.ri = radii[0::2].copy(), radii[1::2].copy()
        self.thresh, self.ratio, self.dry, self.gain = thresh, ratio, dry, gain
        self.z = {b: [np.ones(N), np.zeros(N)] for b in (0, 1)}
        self.w = {b: [np.ones(N), np.zeros(N)] for b in (0, 1)}
        self.act = {b: np.zeros(N, bool) for b in (0, 1)}
        self.sl = [[np.zeros(N), np.zeros(N)] for _ in range(self.O)]
        self.hist = np.zeros((width + 1, N))   # |s|^2, row = time mod (width + 1)
        self.t = 0
        self.rsum = np.zeros(N)
        self.armed, self.engaged = np.zeros(N, bool), np.zeros(N, bool)
        # stickbank coefficients of (z + rad)^order, ascending, without the leading 1
        self.back = np.poly(np.full(self.S, -srad))[::-1][:-1].copy()
        self.sgain = (1 + srad) ** self.S
        self.y = [[np.zeros(N), np.zeros(N)] for _ in range(self.S)]

    def freqmod(self, bank, i, hz):
        self.w[bank][0][i] = math.cos(2 * PI * hz / SR)   # libm, like the engine's host code
        self.w[bank][1][i] = math.sin(2 * PI * hz / SR)

    def sample(self, x):
        zr, zi = self.z[0]
        ir, ii = x * zr, x * zi
        cr, ci = 1.0 - self.rr, 0.0 - self.ri
        for q in range(self.O):
            o_r, o_i = self.sl[q]
            nr = (cr * ir - ci * ii) + (self.rr * o_r - self.ri * o_i)
            ni = (cr * ii + ci * ir) + (self.rr * o_i + self.ri * o_r)
            ir, ii = o_r, o_i
            self.sl[q] = [nr, ni]
        sr, si = self.sl[-1]
        a2 = sr * sr + si * si
        W1 = self.W + 1
        old = self.hist[(self.t - self.W) % W1]
        self.hist[self.t % W1] = a2
        self.rsum = (a2 - old) + self.rsum
        rms = np.sqrt(self.rsum / self.W)
        lo, hi = self.thresh * self.ratio, self.thresh * (1 - self.ratio)
        armed = self.armed | (rms < lo)
        t1 = self.engaged & (rms < lo)
        t2 = ~self.engaged & (rms > hi) & armed
        self.engaged = (self.engaged & ~t1) | t2
        self.armed = armed & ~t1
        eg = self.engaged.astype(float)
        lr, li = sr * eg, si * eg
        accr, acci = np.zeros(self.N), np.zeros(self.N)
        for k in range(self.S):
            accr = accr + (self.y[k][0] * self.back[k] - self.y[k][1] * 0.0)
            acci = acci + (self.y[k][0] * 0.0 + self.y[k][1] * self.back[k])
        yr, yi = self.sgain * lr - accr, self.sgain * li - acci
        self.y = [[yr, yi]] + self.y[:-1]
        szr, szi = self.z[1]
        d = szr * yr - szi * yi
        mix = 0.0
        for v in d:   # Mixer: channel order
            mix += v
        out = 2.0 / PI * np.arctan(self.dry * x + self.gain * mix)
        for b in (0, 1):
            zr, zi = self.z[b]
            wr, wi = self.w[b]
            r, m = zr * wr - zi * wi, zr * wi + zi * wr
            nrm = (1.0 + (r * r + m * m)) / 2
            a = self.act[b]
            self.z[b] = [np.where(a, r / nrm, zr), np.where(a, m / nrm, zi)]
        self.t += 1
        return out

    def process(self, x):
        return np.array([self.sample(v) for v in x])


def configure(objs, N, seed, active_frac=1.0):
    rng = np.random.default_rng(seed)
    fa = rng.uniform(40, 4000, N) * np.where(rng.random(N) < 0.5, -1, 1)
    fs = rng.uniform(40, 4000, N)
    act = [np.flatnonzero(rng.random(N) < active_frac) for _ in range(2)]
    for o in objs:
        for i in range(N):
            if isinstance(o, PyHet):
                o.freqmod(0, i, fa[i])
                o.freqmod(1, i, fs[i])
            else:
                o.freqmod(0, [i], [fa[i]])
                o.freqmod(1, [i], [fs[i]])
        for b in (0, 1):
            if isinstance(o, PyHet):
                o.act[b][act[b]] = True
            else:
                o.activate(b, act[b])


def radii_for(N, seed, imag=0.0):
    rng = np.random.default_rng(seed)
    r = np.zeros(2 * N)
    r[0::2] = rng.uniform(0.9, 0.999, N)
    r[1::2] = imag * rng.standard_normal(N)
    return r


def test_stick_coefficients_are_z_plus_rad_power():
    """stickbank.h:197-217 with zeros {rad} x order builds (z + rad)^order."""
    p = PyHet(1, 1, np.zeros(2), 0, 0, 4, 3, -0.9, 0, 1)
    assert np.allclose(p.back, [(-0.9) ** 3, 3 * 0.81, 3 * -0.9])


@pytest.mark.parametrize("N,order,width,sorder,srad,thresh,seed",
                         [(8, 4, 64, 1, -0.9, 0.0005, 1), (5, 1, 16, 2, -0.5, 0.002, 2), (12, 3, 100, 3, 0.3, 0.0, 3),
                          (7, 8, 9, 4, -0.2, 0.01, 4)])
def test_restatement_vs_numpy(N, order, width, sorder, srad, thresh, seed):
    radii = radii_for(N, seed, imag=0.01 if seed % 2 else 0.0)
    args = (N, order, radii, thresh, 0.2, width, sorder, srad, 0.25, 3.0)
    o, p = OracleHet(*args), PyHet(*args)
    configure([o, p], N, seed, active_frac=0.7)
    x = np.random.default_rng(seed).standard_normal(700) * 0.1
    yo, yp = o.process(x), p.process(x)
    assert np.max(np.abs(yo - yp)) <= 1e-13
    assert np.array_equal(o.state(0).reshape(N, 2), np.stack(p.z[0], 1))
    assert np.array_equal(o.state(1).reshape(N, 2), np.stack(p.z[1], 1))
    sl = o.state(2).reshape(N, order, 2)
    for q in range(order):
        assert np.array_equal(sl[:, q, 0], p.sl[q][0]) and np.array_equal(sl[:, q, 1], p.sl[q][1])
    assert np.array_equal(o.state(3), p.rsum)
    lat = o.state(4).reshape(N, 2)
    assert np.array_equal(lat[:, 0] != 0, p.armed) and np.array_equal(lat[:, 1] != 0, p.engaged)
    st = o.state(5).reshape(N, sorder, 2)
    for k in range(sorder):
        assert np.array_equal(st[:, k, 0], p.y[k][0])


def test_unengaged_latch_passes_only_dry():
    """thresh so high that rms never exceeds thresh (1 - ratio): out = limiter(dry x)."""
    N = 6
    o = OracleHet(N, 2, radii_for(N, 5), thresh=1e9, ratio=0.2, width=32, dry=0.7, gain=3.0)
    configure([o], N, 5)
    x = np.random.default_rng(5).standard_normal(500)
    assert np.array_equal(o.process(x), [2.0 / PI * math.atan(0.7 * v) for v in x])   # libm atan
    assert not o.state(4).reshape(N, 2)[:, 1].any()


def test_history_and_running_sum():
    """RMSbank: the ring holds |s|^2 newest first; the running sum tracks its total."""
    N, W = 4, 20
    o = OracleHet(N, 1, radii_for(N, 6), width=W)
    configure([o], N, 6)
    o.process(np.random.default_rng(6).standard_normal(333))
    hist = o.state(6).reshape(N, W)
    assert np.allclose(hist.sum(1), o.state(3), rtol=1e-12, atol=1e-15)
    assert (hist >= 0).all()


def test_closed_oscillators_stay_at_one():
    """Closed banks never tick: phases stay 1 (setOnes) and the chain is a real filterbank."""
    N = 3
    o = OracleHet(N, 1, radii_for(N, 7), width=8)
    o.process(np.random.default_rng(7).standard_normal(50))
    assert np.array_equal(o.state(0).reshape(N, 2), np.tile([1.0, 0.0], (N, 1)))


def test_harmbank_config():
    """tests/harmbank.cpp: 96 channels, +-partials, synthesis an octave up and reversed."""
    n, fa, fs, radii = harmbank()
    assert n == 96
    assert np.allclose(fs, -2 * fa)
    assert np.all(fa[0::2] > 0) and np.all(fa[1::2] < 0)
    assert np.all((radii[0::2] > 0.9) & (radii[0::2] <= 0.999)) and not radii[1::2].any()


def test_abi_declares_heterodyne():
    syms = header_symbols()
    for s in ("hz_het_create", "hz_het_process", "hz_het_process_device", "hz_het_freqmod", "hz_het_activate",
              "hz_het_open", "hz_het_setup", "hz_het_state"):
        assert s in syms
