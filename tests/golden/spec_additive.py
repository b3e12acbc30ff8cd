"""Independent numpy restatement of Oscillator / Additive / Sinusoids (TEST INFRASTRUCTURE).

Written from /root/reference/src/{oscillator,additive,sinusoids,minimizer}.h; shares no
code with oracle/.  Vectorised over oscillators, per-sample loop in time.
"""
from __future__ import annotations

import math

import numpy as np

from spec_numpy import PI, SR, relaxation


def mtof(m):
    return 440.0 * 2.0 ** ((m - 69) / 12)


def ftom(f):
    return 69 + math.log2(f / 440.0) * 12


class OscBankSpec:
    """A vector of Oscillator<double> (src/oscillator.h:12-71), phasemod never used."""

    def __init__(self, n, f, k):
        self.freq = np.abs(np.asarray(f, dtype=np.float64) * np.ones(n))
        self.target = self.freq.copy()
        self.phase = np.zeros(n)
        self.tphase = np.zeros(n)
        self.s = relaxation(k)

    def tick(self, mask=None):
        idx = slice(None) if mask is None else mask
        s = self.s
        ph, tp, f = self.phase[idx], self.tphase[idx], self.freq[idx]
        ph = ph + f / SR
        tp = tp + f / SR
        f = self.target[idx] * (1 - s) + f * s
        w = (1 - s) * np.sin(2 * PI * (2 * np.abs(tp - ph) + 0.25))
        ph = w * tp + (1 - w) * ph
        ph = ph - np.trunc(ph)
        tp = tp - np.trunc(tp)
        self.phase[idx], self.tphase[idx], self.freq[idx] = ph, tp, f


def additive_run(V, O, decay, harm, k, events, n):
    """Additive<double>(&cycle, V, O, decay, harm, k) driven by
    n x { out[t] = A(); A.tick(); }; events (t, 'makenote'|'endnote'|'request'|'release', args)."""
    attack = relaxation(k)
    norm = (1 - decay ** O) / (1 - decay) if decay != 1 else O
    osc = OscBankSpec(V * O, 0.0, 0.0001)
    amps = np.zeros(V)
    active = np.zeros(V)
    pitches = np.zeros(V)
    guide = np.zeros(V)
    position = np.zeros(V * O)
    out = np.zeros(n)
    dec = decay ** np.arange(O)

    def request(fundamental, amplitude):
        voice = -1
        for i in range(V):
            if not active[i]:
                voice = i
                break
        if voice < 0:
            pitch = ftom(fundamental)
            best, dist = -1, 0.0
            for i in range(V):
                off = (pitch - guide[i]) ** 2
                if best < 0 or off < dist:
                    best, dist = i, off
            voice = best
        active[voice] = amplitude
        guide[voice] = ftom(fundamental)
        for j in range(O):
            freq = fundamental * (1 + math.pow(j / (O - 1), harm) * (O - 1))
            position[voice * O + j] = ftom(freq)
        return voice

    ev = sorted(events, key=lambda e: e[0])
    ei = 0
    for t in range(n):
        while ei < len(ev) and ev[ei][0] == t:
            _, kind, arg = ev[ei]
            if kind == "makenote":
                v = request(mtof(arg[0]), arg[1])
                pitches[v] = arg[0]
            elif kind == "endnote":
                for j in range(V):
                    if pitches[j] == arg[0]:
                        active[j] = 0
            elif kind == "request":
                request(arg[0], arg[1])
            elif kind == "release":
                if arg[0] >= 0:
                    active[arg[0]] = 0
                else:
                    active[:] = 0
            ei += 1
        s = 0.0
        for i in range(V):
            if amps[i]:
                s += np.sum(amps[i] * dec * np.sin(2 * PI * osc.phase[i * O:(i + 1) * O]) / (V * norm))
        out[t] = s
        amps[:] = (1 - attack) * active + attack * amps
        for i in range(V):
            if active[i] or amps[i]:
                sl = slice(i * O, (i + 1) * O)
                osc.target[sl] = mtof(position[sl])
                osc.tick(np.arange(i * O, (i + 1) * O))
    return out


def sinusoids_run(fundamental, O, decay, harm, k, events, n):
    """Sinusoids<double>(&cycle, ...) driven by n x { out[t] = S(); S.tick(); };
    events (t, 'fundmod'|'decaymod'|'harmmod', value)."""
    tf, td, th = fundamental, decay, harm
    f, d, h = fundamental, decay, harm
    s = relaxation(k)
    osc = OscBankSpec(O, 0.0, 2.0 / SR)
    osc.freq = np.abs(fundamental * (np.arange(O) + 1.0) ** harm)
    osc.target = osc.freq.copy()
    norm = (1 - d ** O) / (1 - d) if d != 1 else O
    out = np.zeros(n)
    ev = sorted(events, key=lambda e: e[0])
    ei = 0
    for t in range(n):
        while ei < len(ev) and ev[ei][0] == t:
            _, kind, v = ev[ei]
            if kind == "fundmod":
                tf = v
            elif kind == "decaymod":
                td = v
            elif kind == "harmmod":
                th = v
            ei += 1
        out[t] = np.sum(d ** np.arange(O) * np.sin(2 * PI * osc.phase) / norm)
        f = tf * (1 - s) + f * s
        d = td * (1 - s) + d * s
        h = th * (1 - s) + h * s
        osc.target = f * (np.arange(O) + 1.0) ** h
        osc.tick()
        norm = (1 - d ** O) / (1 - d) if d != 1 else O
    return out
