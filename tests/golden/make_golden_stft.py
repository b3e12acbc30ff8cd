"""Golden fixtures for Fourier / StaticSTFT / Cosine (run: python tests/golden/make_golden_stft.py).

TEST INFRASTRUCTURE.  Independent restatement of src/fourier.h:50-234 and
src/staticSTFT.h:10-177 that does NOT replay the slot state machine: it uses the closed-form
schedule derived from it -- frame f = c*2*laps + i of slot i starts at
s = stride*i + c*(2N-1), covers input [s, s+N-1] and emits IFFT sample k at t = s+N-1+k --
with numpy.fft (unnormalised forward e^{-}, ifft*N for FFTW BACKWARD) and scipy.fft.dct
type 2 / 3 for REDFT10 / REDFT01.  Overlap-add sums the slots in slot order in np.longdouble
and divides by the int N*laps/2.  Each gated case records the smallest relative distance of
any bin from its gate threshold (`margin`): decisions closer than ~1e-12 could legitimately
flip between FFT implementations.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import scipy.fft

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from spec_numpy import PI  # noqa: E402


def window(kind, N):
    p = np.arange(N) / float(N)
    h = 0.5 * (1 - np.cos(2 * PI * p))
    return h if kind == "hann" else np.sqrt(h)


def proc_static_gate(X, N):
    mag = np.sqrt(X.real * X.real + X.imag * X.imag) / N
    average = np.add.accumulate(mag)[-1]                     # sequential, as the C loop
    nrm = X.real * X.real + X.imag * X.imag
    thr = 100 * average * average
    Y = np.where(nrm < thr, X * 0.1, X)
    return Y, np.min(np.abs(nrm - thr) / thr)


def proc_gate_keep(X, N):
    average = np.longdouble(0)
    for v in np.hypot(X.real, X.imag):
        average += np.longdouble(v)
    average /= N
    nrm = (X.real * X.real + X.imag * X.imag).astype(np.longdouble)
    thr = 625 * average * average
    Y = np.where(nrm > thr, X, 0)
    return Y, float(np.min(np.abs(nrm - thr) / thr))


def proc_hilbert(X, N):
    Y = X.copy()
    Y[N // 2:] = 0
    return Y, np.inf


def stft_run(x, N, laps, wkind, proc):
    n = len(x)
    stride = N // laps
    S = 2 * laps
    w = window(wkind, N)
    acc = np.zeros((S, n), dtype=np.clongdouble)   # per-slot contributions, summed in slot order
    starts, margin = [], np.inf
    c = 0
    while True:
        any_frame = False
        for i in range(S):
            s = stride * i + c * (2 * N - 1)
            if s + N - 1 >= n:
                continue
            any_frame = True
            starts.append(s)
            frame = w * x[s:s + N]
            X = np.fft.fft(frame)
            Y, m = proc(X, N)
            margin = min(margin, m)
            y = np.fft.ifft(Y) * N
            k = np.arange(N)
            t = s + N - 1 + k
            ok = t < n
            acc[i, t[ok]] += (w[k[ok]] * y.real[k[ok]]) + 1j * (w[k[ok]] * y.imag[k[ok]])
        if not any_frame:
            break
        c += 1
    tot = np.zeros(n, dtype=np.clongdouble)
    for i in range(S):
        tot += acc[i]
    tot /= (N * laps // 2)
    return tot.real.astype(np.float64), tot.imag.astype(np.float64), np.array(sorted(starts)), margin


def signal(n, seed, complex_in=False, N=64):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    x = 0.1 * rng.standard_normal(n)
    for k in (3, 7, 12):                       # bin-centred tones so some bins pass a gate
        x = x + 0.5 * np.sin(2 * np.pi * k * t / N + k)
    if complex_in:
        x = x + 1j * (0.1 * rng.standard_normal(n))
    return x


def main():
    out = {}
    cases = [
        ("stft_static_n64", 64, 4, "hann", proc_static_gate, 1, False, 1),
        ("stft_gate_n64", 64, 4, "halfhann", proc_gate_keep, 2, False, 2),
        ("stft_id_n16_cplx", 16, 4, "halfhann", lambda X, N: (X, np.inf), 0, True, 3),
        ("stft_hilbert_n32_l8", 32, 8, "halfhann", proc_hilbert, 3, False, 4),
    ]
    for name, N, laps, wk, proc, pid, cplx, seed in cases:
        n = 3 * (2 * N - 1)
        x = signal(n, seed, cplx, N)
        if pid == 2:
            # spectral.cpp's 625 gate (|X| > 25 mean|X|) passes only a near-pure one-sided tone:
            # with the sqrt-hann window sum|X| ~ 2 peak for e^{2 pi i k t/N}
            t = np.arange(n)
            x = 0.5 * np.exp(2j * np.pi * 5 * t / N) + 0.001 * np.random.default_rng(seed).standard_normal(n)
            cplx = True
        yr, yi, starts, margin = stft_run(x, N, laps, wk, proc)
        out[name] = dict(N=N, laps=laps, window=int(wk == "hann"), proc=pid, x_re=x.real.copy(),
                         x_im=(x.imag.copy() if cplx else np.zeros(n)), y_re=yr, y_im=yi, starts=starts,
                         margin=margin)
        hops = np.diff(starts)
        print(name, "frames", len(starts), "hops", sorted(set(hops.tolist())), "margin %.3g" % margin,
              "|y|max %.3g" % np.max(np.abs(yr)))
    rng = np.random.default_rng(9)
    x = rng.standard_normal(64)
    y2 = scipy.fft.dct(x, type=2)
    y3 = scipy.fft.dct(y2, type=3)
    out["dct_n64"] = dict(N=64, x=x, redft10=y2, roundtrip=y3)
    for name, d in out.items():
        np.savez(os.path.join(HERE, name + ".npz"), **d)


if __name__ == "__main__":
    main()
