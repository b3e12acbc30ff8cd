"""Independent numpy restatement of the reference semantics (TEST INFRASTRUCTURE).

Used only by tests/golden/make_golden.py to produce fixtures and by CPU tests.
Written from /root/reference/src/*.h directly; shares no code with oracle/.
"""
from __future__ import annotations

import math

import numpy as np

PI = 3.14159265359          # src/includes.h:30 (truncated, not math.pi)
E = 2.718281828459045       # src/includes.h:31
SR = 48000                  # src/includes.h:32 (int)


def relaxation(k: float) -> float:
    """src/includes.h:43-48: 2^(log2(eps) / (max(0,k) * SR)), 0 for k == 0."""
    if k == 0:
        return 0.0
    return 2.0 ** (math.log2(np.finfo(np.float64).eps) / (max(0.0, k) * SR))


def white_noise_f32(n: int, seed: int = 1) -> np.ndarray:
    """uniform[-1,1) generated as float32 (PortAudio delivers float) then widened."""
    rng = np.random.default_rng(seed)
    return rng.uniform(-1.0, 1.0, size=n).astype(np.float32).astype(np.float64)


def transfer(frequency: float, r: float, f: float) -> complex:
    """tests/resynthesis.cpp:23-27 band-pass transfer function."""
    z = complex(math.cos(2 * PI * f / SR), -math.sin(2 * PI * f / SR))
    return (1.0 - z * z) / (1.0 - 2 * r * math.cos(2 * PI * frequency / SR) * z + r * r * z * z)


def resonant_coefficients(N: int, R: float, centre_offset: float = 1.0):
    """tests/resynthesis.cpp:48-54 coefficient recipe.  centre_offset=1 is the
    reference's f_i = 0.5 (i+1) SR / N (whose last band sits on Nyquist);
    centre_offset=0.5 gives the balanced variant used by some parity tests."""
    fwd = np.zeros((N, 3))
    back = np.zeros((N, 2))
    for i in range(N):
        frequency = 0.5 * (i + centre_offset) * SR / N
        cosine = math.cos(2 * PI * frequency / SR)
        gain = abs(transfer(frequency, R, frequency))
        fwd[i] = [1.0 / gain, 0.0, -1.0 / gain]
        back[i] = [-2 * R * cosine, R * R]
    return fwd, back


def dist(id_: int, v: np.ndarray, param: float) -> np.ndarray:
    """Distortions: tests/filterbank.cpp:158-176 (softclip, saturate), src/wave.h:150 (limiter)."""
    if id_ == 0:
        return v
    if id_ == 1:
        width = param
        sign = np.sign(v)
        gap = v - sign * width
        clipped = sign * width + (1 - width) * 2.0 / PI * np.arctan(PI * gap / (2 * (1 - width)))
        return np.where(np.abs(v) < width, v, clipped)
    if id_ == 2:
        return 2.0 / PI * np.arctan(2 * PI * v / 2.0)
    if id_ == 3:
        return 2.0 / PI * np.arctan(v)
    raise ValueError(id_)


def filterbank_run(order, N, kp, kg, fwd, back, x, sched, dist_id=0, dist_param=0.0):
    """Filterbank<double>: src/filterbank.h:36-187, driven by the demo block
    loop out[i] = F(in[i]); F.tick() (tests/resynthesis.cpp:35-39).

    sched: list of (sample index, kind, arg) applied before that sample:
    kind in {boost_all(vec), mix_all(vec), open(None), boost((n,v)), mix((n,v))}.
    Returns (mix output, per-band y [T, N], pre-amp history [T, N])."""
    sp, sg = relaxation(kp), relaxation(kg)
    F = np.zeros((N, order + 1))
    B = np.zeros((N, order))
    F[:, :] = fwd[:, : order + 1]
    B[:, :] = back[:, :order]
    pin = np.zeros(N)
    gin = np.zeros(N)
    pre = np.zeros(N)
    g = np.zeros(N)
    xh = np.zeros(order + 1)      # x[t], x[t-1], ...
    yh = np.zeros((order, N))     # y[t-1], y[t-2], ...
    T = len(x)
    out = np.zeros(T)
    yb = np.zeros((T, N))
    ph = np.zeros((T, N))
    si = 0
    sched = sorted(sched, key=lambda s: s[0])
    for t in range(T):
        while si < len(sched) and sched[si][0] == t:
            _, kind, arg = sched[si]
            if kind == "boost_all":
                pin[: min(N, len(arg))] = arg[: min(N, len(arg))]
            elif kind == "mix_all":
                gin[: min(N, len(arg))] = arg[: min(N, len(arg))]
            elif kind == "open":
                gin[:] = 1.0
            elif kind == "boost":
                pin[arg[0]] = arg[1]
            elif kind == "mix":
                gin[arg[0]] = arg[1]
            si += 1
        pre = (1 - sp) * pin + sp * pre
        g = (1 - sg) * gin + sg * g
        xh = np.roll(xh, 1)
        xh[0] = x[t]
        ff = F[:, 0] * xh[0]
        for i in range(1, order + 1):
            ff = ff + F[:, i] * xh[i]
        fbk = np.zeros(N)
        for k in range(order):
            fbk = fbk + B[:, k] * yh[k]
        y = ff * pre - fbk
        if order > 0:
            yh = np.roll(yh, 1, axis=0)
            yh[0] = y
        yb[t] = y
        ph[t] = pre
        out[t] = np.sum(dist(dist_id, y * g, dist_param))
    return out, yb, ph


def oscbank_run(N, events, n):
    """Oscbank<double,N> (src/oscbank.h:37-90) driven by
    n x { mix[t] = mixdown(); tick(); } with setter events applied before sample t.
    events: list of (t, kind, arg): freqmod((i, hz)), activate([i...]), deactivate([i...]),
    open(None), close(None).  Returns (mix [n] complex, final phases [N] complex)."""
    z = np.ones(N, dtype=np.complex128)
    w = np.ones(N, dtype=np.complex128)
    active = np.zeros(N, dtype=bool)
    mix = np.zeros(n, dtype=np.complex128)
    ev = sorted(events, key=lambda e: e[0])
    ei = 0
    for t in range(n):
        while ei < len(ev) and ev[ei][0] == t:
            _, kind, arg = ev[ei]
            if kind == "freqmod":
                i, hz = arg
                if 0 <= i < N:
                    w[i] = complex(math.cos(2 * PI * hz / SR), math.sin(2 * PI * hz / SR))
            elif kind == "activate":
                for i in arg:
                    if 0 <= i < N:
                        active[i] = True
            elif kind == "deactivate":
                for i in arg:
                    if 0 <= i < N:
                        active[i] = False
            elif kind == "open":
                active[:] = True
            elif kind == "close":
                active[:] = False
            ei += 1
        idx = np.nonzero(active)[0]           # `where`, ascending
        mix[t] = np.sum(z[idx]) if len(idx) else 0.0
        zz = z[idx] * w[idx]
        z[idx] = zz / ((1.0 + (zz.real ** 2 + zz.imag ** 2)) / 2)
    return mix, z
