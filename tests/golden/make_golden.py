"""Generate the golden fixtures in tests/golden/ (run: python tests/golden/make_golden.py).

TEST INFRASTRUCTURE.  This is a second, independent restatement of the
reference semantics written in numpy (vectorised over bands, per-sample loop in
time), deliberately not sharing code with oracle/hz_oracle.c.  Every fixture is
additionally cross-checked against an independent implementation of the
underlying maths where one exists here (scipy.signal.lfilter for the IIR
recurrences, numpy.fft for FFTW's DFT conventions, scipy.fft.dct for REDFT10/01).

The reference (amcerbu/huygens) cannot be built in this image and its own tests
hold no golden data, so these fixtures pin the oracle to the reference's
*semantics as read from its source*, not to outputs of the reference binary.

Fixtures are small .npz files (inputs + expected outputs, float64).
"""
from __future__ import annotations

import os
import zlib
import sys

import numpy as np
from scipy import signal

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from spec_numpy import (  # noqa: E402
    PI, SR, relaxation, filterbank_run, resonant_coefficients, white_noise_f32, oscbank_run,
)


def check_fb_against_lfilter(fwd, back, pre_seq_fn, x, y_bands):
    """Fold the time-varying pre-amp into the input and compare every band
    against scipy.signal.lfilter (exact recurrence equivalence)."""
    for n in range(fwd.shape[0]):
        conv = signal.lfilter(fwd[n], [1.0], x)
        u = pre_seq_fn(n) * conv
        y = signal.lfilter([1.0], np.concatenate(([1.0], back[n])), u)
        err = np.max(np.abs(y - y_bands[:, n])) / max(1e-300, np.max(np.abs(y)))
        assert err < 1e-11, (n, err)


def make_filterbank():
    out = {}
    rng_cases = [
        # name, order, N, R, nsamp, dist, dist_param, kp, kg
        ("fb_o2_n16_r0999", 2, 16, 0.999, 4096, 0, 0.0, 0.1, 1.0),
        ("fb_o2_n16_r09999_softclip", 2, 16, 0.9999, 4096, 1, 0.125, 0.1, 1.0),
        ("fb_o2_n7_fast", 2, 7, 0.99, 3001, 0, 0.0, 0.0, 0.001),
        ("fb_o1_n9", 1, 9, 0.9, 2500, 0, 0.0, 0.1, 1.0),
        ("fb_o3_n5", 3, 5, 0.95, 2048, 3, 0.0, 0.05, 0.5),
    ]
    for name, order, N, R, nsamp, dist, dparam, kp, kg in rng_cases:
        x = white_noise_f32(nsamp, seed=zlib.crc32(name.encode()) % 1000 + 1)
        if order == 2:
            fwd, back = resonant_coefficients(N, R)
        else:
            rng = np.random.default_rng(7 + order)
            fwd = rng.uniform(-1, 1, size=(N, order + 1))
            # stable all-pole part: poles inside radius R
            back = np.zeros((N, order))
            for n in range(N):
                roots = R * np.exp(1j * rng.uniform(0, np.pi, size=order))
                if order % 2 == 1:
                    roots[-1] = R * rng.uniform(-1, 1)
                if order >= 2:
                    roots[1] = np.conj(roots[0])
                poly = np.real(np.poly(roots))
                back[n] = poly[1:]
        boost = np.ones(N)
        mix = np.ones(N)
        # setter schedule: (sample index, kind, band or -1, value)
        sched = [(0, "boost_all", boost), (0, "open", None)]
        if name == "fb_o2_n7_fast":
            sched += [(1000, "boost", (3, 0.25)), (2000, "mix", (1, -2.0))]
        y_mix, y_bands, pre_hist = filterbank_run(order, N, kp, kg, fwd, back, x, sched, dist, dparam)
        if dist == 0 and not any(s[1] in ("boost", "mix") for s in sched):
            check_fb_against_lfilter(fwd, back, lambda n: pre_hist[:, n], x, y_bands)
        out[name] = dict(order=order, N=N, kp=kp, kg=kg, fwd=fwd, back=back, x=x,
                         dist=dist, dist_param=dparam, y=y_mix,
                         sched_t=np.array([s[0] for s in sched]),
                         sched_kind=np.array([s[1] for s in sched]),
                         sched_band=np.array([(-1 if s[2] is None or isinstance(s[2], np.ndarray) else s[2][0]) for s in sched]),
                         sched_val=np.array([(np.nan if s[2] is None or isinstance(s[2], np.ndarray) else s[2][1]) for s in sched]))
    # known answer: impulse response of one biquad with constant pre-amp after
    # convergence (k_p = 0 -> relaxation 0 -> pre = target immediately)
    N = 1
    fwd = np.array([[0.5, 0.25, -0.125]])
    back = np.array([[-1.2, 0.5]])
    x = np.zeros(64)
    x[0] = 1.0
    sched = [(0, "boost_all", np.ones(1)), (0, "open", None)]
    y_mix, _, _ = filterbank_run(2, N, 0.0, 0.0, fwd, back, x, sched, 0, 0.0)
    ref = signal.lfilter(fwd[0], [1.0, -1.2, 0.5], x)
    assert np.allclose(y_mix, ref, rtol=0, atol=1e-15)
    # hand-computed first samples: y0 = b0, y1 = b1 - a1*y0, y2 = b2 - a1*y1 - a2*y0
    y0 = 0.5
    y1 = 0.25 + 1.2 * y0
    y2 = -0.125 + 1.2 * y1 - 0.5 * y0
    assert abs(y_mix[0] - y0) < 1e-15 and abs(y_mix[1] - y1) < 1e-15 and abs(y_mix[2] - y2) < 1e-15
    out["fb_impulse_known"] = dict(order=2, N=1, kp=0.0, kg=0.0, fwd=fwd, back=back, x=x, dist=0,
                                   dist_param=0.0, y=y_mix, sched_t=np.array([0, 0]),
                                   sched_kind=np.array(["boost_all", "open"]),
                                   sched_band=np.array([-1, -1]), sched_val=np.array([np.nan, np.nan]))
    return out


def osc_events_to_arrays(events):
    """Encode an event list as flat arrays for the .npz (no pickles)."""
    kinds = {"freqmod": 0, "activate": 1, "deactivate": 2, "open": 3, "close": 4}
    t, k, i, v = [], [], [], []
    for (tt, kind, arg) in events:
        if kind == "freqmod":
            t.append(tt); k.append(0); i.append(arg[0]); v.append(arg[1])
        elif kind in ("activate", "deactivate"):
            for ii in arg:
                t.append(tt); k.append(kinds[kind]); i.append(ii); v.append(0.0)
        else:
            t.append(tt); k.append(kinds[kind]); i.append(-1); v.append(0.0)
    return dict(ev_t=np.array(t), ev_kind=np.array(k), ev_index=np.array(i), ev_value=np.array(v))


def make_oscbank():
    out = {}
    rng = np.random.default_rng(21)
    # 1. N = 32 partials, all open, harmonic frequencies, 4096 samples; check the
    #    phasor trajectory against the exact rotation e^{i 2 PI f t / SR}
    N, n = 32, 4096
    freqs = 110.0 * (1 + np.arange(N))
    ev = [(0, "freqmod", (i, float(freqs[i]))) for i in range(N)] + [(0, "open", None)]
    mix, z = oscbank_run(N, ev, n)
    t = np.arange(n)[:, None]
    exact = np.exp(1j * 2 * PI * freqs[None, :] * t / SR).sum(axis=1)
    assert np.max(np.abs(mix - exact)) / N < 1e-9
    out["osc_n32_open"] = dict(N=N, n=n, mix=mix, z_final=z, **osc_events_to_arrays(ev))
    # 2. N = 64, partial activation, deactivation and freqmod changes mid-stream,
    #    out-of-range indices ignored (oscbank.h:51, multichannel.h:87-100)
    N, n = 64, 3000
    ev = [(0, "freqmod", (i, float(rng.uniform(20, 20000)))) for i in range(N)]
    ev += [(0, "activate", sorted(rng.choice(N, 20, replace=False).tolist()) + [N + 3, -1])]
    ev += [(700, "freqmod", (5, 1234.5)), (700, "freqmod", (N, 99.0)), (700, "activate", [5, 6, 7])]
    ev += [(1500, "deactivate", [5, 6, 40, 41]), (2222, "open", None), (2600, "close", None),
           (2700, "activate", [0, 63])]
    mix, z = oscbank_run(N, ev, n)
    out["osc_n64_events"] = dict(N=N, n=n, mix=mix, z_final=z, **osc_events_to_arrays(ev))
    return out


def main():
    fixtures = make_filterbank()
    fixtures.update(make_oscbank())
    for name, d in fixtures.items():
        np.savez(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name, {k: (v.shape if hasattr(v, "shape") else v) for k, v in d.items() if k in ("x", "y")})


if __name__ == "__main__":
    main()
