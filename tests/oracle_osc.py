"""ctypes binding of the Additive / Sinusoids restatement (oracle/hz_oracle_osc.c).
TEST INFRASTRUCTURE."""
from __future__ import annotations

import ctypes as C

import numpy as np

from oracle import D, I, L, PD, VP, _bind, _p

_SIGS = {
    "orc_add_create": (VP, [I, I, D, D, D]),
    "orc_add_destroy": (None, [VP]),
    "orc_add_request": (I, [VP, D, D]),
    "orc_add_release": (None, [VP, I]),
    "orc_add_makenote": (I, [VP, D, D]),
    "orc_add_endnote": (None, [VP, D]),
    "orc_add_fill": (None, [VP, PD, L]),
    "orc_sin_create": (VP, [D, I, D, D, D]),
    "orc_sin_destroy": (None, [VP]),
    "orc_sin_fundmod": (None, [VP, D]),
    "orc_sin_decaymod": (None, [VP, D]),
    "orc_sin_harmmod": (None, [VP, D]),
    "orc_sin_fill": (None, [VP, PD, L]),
}


class OracleAdditive:
    def __init__(self, voices, overtones, decay, harmonicity=1.0, k=0.1):
        self.l = _bind(_SIGS)
        self.h = self.l.orc_add_create(voices, overtones, decay, harmonicity, k)

    def __del__(self):
        try:
            self.l.orc_add_destroy(self.h)
        except Exception:
            pass

    def request(self, fundamental, amplitude=0.0):
        return self.l.orc_add_request(self.h, fundamental, amplitude)

    def release(self, voice):
        self.l.orc_add_release(self.h, voice)

    def makenote(self, pitch, amplitude):
        return self.l.orc_add_makenote(self.h, pitch, amplitude)

    def endnote(self, pitch):
        self.l.orc_add_endnote(self.h, pitch)

    def fill(self, n):
        out = np.zeros(n)
        self.l.orc_add_fill(self.h, _p(out), n)
        return out


class OracleSinusoids:
    def __init__(self, fundamental, overtones, decay, harmonicity=1.0, k=2.0 / 48000):
        self.l = _bind(_SIGS)
        self.h = self.l.orc_sin_create(fundamental, overtones, decay, harmonicity, k)

    def __del__(self):
        try:
            self.l.orc_sin_destroy(self.h)
        except Exception:
            pass

    def fundmod(self, v):
        self.l.orc_sin_fundmod(self.h, v)

    def decaymod(self, v):
        self.l.orc_sin_decaymod(self.h, v)

    def harmmod(self, v):
        self.l.orc_sin_harmmod(self.h, v)

    def fill(self, n):
        out = np.zeros(n)
        self.l.orc_sin_fill(self.h, _p(out), n)
        return out


def run_note_events(obj, g):
    """Drive an Additive- or Sinusoids-like object through a fixture's events,
    splitting fill() at every event time."""
    n = int(g["n"])
    t_ev, kind, ea, eb = g["ev_t"], g["ev_kind"], g["ev_a"], g["ev_b"]
    out = np.zeros(n)
    pos = 0
    for t in sorted(set(t_ev.tolist())) + [n]:
        if t > pos:
            out[pos:t] = obj.fill(t - pos)
            pos = t
        if t >= n:
            break
        for e in range(len(t_ev)):
            if t_ev[e] != t:
                continue
            k = int(kind[e])
            if k == 0:
                obj.makenote(float(ea[e]), float(eb[e]))
            elif k == 1:
                obj.endnote(float(ea[e]))
            elif k == 2:
                obj.request(float(ea[e]), float(eb[e]))
            elif k == 3:
                obj.release(int(ea[e]))
            elif k == 10:
                obj.fundmod(float(ea[e]))
            elif k == 11:
                obj.decaymod(float(ea[e]))
            elif k == 12:
                obj.harmmod(float(ea[e]))
    return out
