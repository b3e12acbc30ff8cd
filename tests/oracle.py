"""ctypes binding of the CPU restatement oracle/hz_oracle.c (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "oracle", "_build", "libhz_oracle.so")

D, I, L, VP = C.c_double, C.c_int, C.c_long, C.c_void_p
PD = C.POINTER(C.c_double)

_SIGS = {
    "orc_relaxation": (D, [D]),
    "orc_mtof": (D, [D]),
    "orc_ftom": (D, [D]),
    "orc_dist": (D, [I, D, D]),
    "orc_fb_create": (VP, [I, I, D, D]),
    "orc_fb_destroy": (None, [VP]),
    "orc_fb_coefficients": (None, [VP, I, PD, I, PD, I]),
    "orc_fb_boost": (None, [VP, I, D]),
    "orc_fb_boost_all": (None, [VP, PD, I]),
    "orc_fb_mix": (None, [VP, I, D]),
    "orc_fb_mix_all": (None, [VP, PD, I]),
    "orc_fb_open": (None, [VP]),
    "orc_fb_sample": (D, [VP, D, I, D]),
    "orc_fb_tick": (None, [VP]),
    "orc_fb_process": (None, [VP, PD, PD, L, I, D]),
    "orc_fb_get_state": (None, [VP, PD]),
    "orc_fb_process_tv": (None, [VP, PD, PD, L, I, PD, D, I, D]),
    "orc_resonant": (D, [D, D]),
    "orc_fb_resonant_coefficients": (None, [D, D, PD, PD]),
}

_lib = None


def lib():
    """The oracle library: oracle/_build/libhz_oracle.so, or HZ_ORACLE_SO (bench.py's
    cpu_baseline points it at a -O3 -march=native build of the same sources)."""
    global _lib
    if _lib is None:
        so = os.environ.get("HZ_ORACLE_SO") or SO
        if not os.path.exists(so):
            import subprocess
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
            so = SO
        _lib = C.CDLL(so)
        for name, (res, args) in _SIGS.items():
            fn = getattr(_lib, name)
            fn.restype = res
            fn.argtypes = args
    return _lib


def _p(a):
    return a.ctypes.data_as(PD)


class OracleFilterbank:
    """CPU restatement of Filterbank<double> (src/filterbank.h:16-188)."""

    def __init__(self, order, N, k_p=0.1, k_g=1.0):
        self.l = lib()
        self.h = self.l.orc_fb_create(order, N, k_p, k_g)
        self.order, self.N = order, N
        self.dist = (0, 0.0)

    def __del__(self):
        try:
            self.l.orc_fb_destroy(self.h)
        except Exception:
            pass

    def coefficients(self, n, fwd, back):
        f = np.ascontiguousarray(fwd, dtype=np.float64)
        b = np.ascontiguousarray(back, dtype=np.float64)
        self.l.orc_fb_coefficients(self.h, n, _p(f), len(f), _p(b), len(b))

    def boost(self, n_or_values, value=None):
        if value is None:
            v = np.ascontiguousarray(n_or_values, dtype=np.float64)
            self.l.orc_fb_boost_all(self.h, _p(v), len(v))
        else:
            self.l.orc_fb_boost(self.h, n_or_values, value)

    def mix(self, n_or_values, value=None):
        if value is None:
            v = np.ascontiguousarray(n_or_values, dtype=np.float64)
            self.l.orc_fb_mix_all(self.h, _p(v), len(v))
        else:
            self.l.orc_fb_mix(self.h, n_or_values, value)

    def open(self):
        self.l.orc_fb_open(self.h)

    def distortion(self, dist_id, param=None):
        # param None: the reference's default (softclip: width 0.125, tests/filterbank.cpp:168-171)
        self.dist = (dist_id, (0.125 if dist_id == 1 else 0.0) if param is None else param)

    def process(self, x):
        xi = np.ascontiguousarray(x, dtype=np.float64)
        out = np.empty_like(xi)
        self.l.orc_fb_process(self.h, _p(xi), _p(out), len(xi), self.dist[0], self.dist[1])
        return out

    def get_state(self):
        """[x history (O)] [y history (N O)] [pre, gain (2 N)] -- hz_fb_get_state's layout"""
        buf = np.zeros(self.order + self.N * self.order + 2 * self.N)
        self.l.orc_fb_get_state(self.h, _p(buf))
        return buf

    def __call__(self, sample):
        """operator()(T) (filterbank.h:125-131), cached until tick()."""
        return self.l.orc_fb_sample(self.h, float(sample), self.dist[0], self.dist[1])

    def tick(self):
        """tick() (filterbank.h:142-148): origin moves; no compute if operator() was not called."""
        self.l.orc_fb_tick(self.h)

    def process_tv(self, x, kind, stream, param=0.0):
        xi = np.ascontiguousarray(x, dtype=np.float64)
        st = np.ascontiguousarray(stream, dtype=np.float64)
        out = np.empty_like(xi)
        self.l.orc_fb_process_tv(self.h, _p(xi), _p(out), len(xi), kind, _p(st), param, self.dist[0], self.dist[1])
        return out


def run_schedule(fb, x, sched_t, sched_kind, sched_band, sched_val, fwd=None, back=None):
    """Drive a Filterbank-like object (oracle or GPU) through a golden fixture's
    setter schedule, splitting process() calls at every change point."""
    if fwd is not None:
        for n in range(fwd.shape[0]):
            fb.coefficients(n, fwd[n], back[n])
    out = np.zeros(len(x))
    pos = 0
    events = sorted(zip(sched_t.tolist(), range(len(sched_t))))
    N = fwd.shape[0] if fwd is not None else None
    for t, idx in events + [(len(x), None)]:
        if t > pos:
            out[pos:t] = fb.process(x[pos:t])
            pos = t
        if idx is None:
            break
        kind = str(sched_kind[idx])
        if kind == "boost_all":
            fb.boost(np.ones(N))
        elif kind == "mix_all":
            fb.mix(np.ones(N))
        elif kind == "open":
            fb.open()
        elif kind == "boost":
            fb.boost(int(sched_band[idx]), float(sched_val[idx]))
        elif kind == "mix":
            fb.mix(int(sched_band[idx]), float(sched_val[idx]))
    return out


def load_golden(name):
    path = os.path.join(ROOT, "tests", "golden", name + ".npz")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_names(prefix):
    d = os.path.join(ROOT, "tests", "golden")
    return sorted(f[:-4] for f in os.listdir(d) if f.startswith(prefix) and f.endswith(".npz"))


def rel_err(got, ref):
    """norm-wise parity metric of SURVEY.md 8(d): ||got-ref||_inf / ||ref||_inf (complex values
    compare as complex: both parts count)."""
    got, ref = np.asarray(got), np.asarray(ref)
    dt = np.complex128 if np.iscomplexobj(got) or np.iscomplexobj(ref) else np.float64
    got = got.astype(dt)
    ref = ref.astype(dt)
    den = np.max(np.abs(ref)) if ref.size else 0.0
    if den == 0.0:
        return float(np.max(np.abs(got))) if got.size else 0.0
    return float(np.max(np.abs(got - ref)) / den)


_OSC_SIGS = {
    "orc_osc_create": (VP, [I, D]),
    "orc_osc_destroy": (None, [VP]),
    "orc_osc_freqmod": (None, [VP, I, D]),
    "orc_osc_activate": (None, [VP, C.POINTER(C.c_int), I]),
    "orc_osc_deactivate": (None, [VP, C.POINTER(C.c_int), I]),
    "orc_osc_open": (None, [VP]),
    "orc_osc_close": (None, [VP]),
    "orc_osc_tick": (None, [VP]),
    "orc_osc_mixdown": (None, [VP, PD, PD]),
    "orc_osc_phases": (None, [VP, PD]),
    "orc_osc_active_count": (I, [VP]),
    "orc_osc_fill": (None, [VP, PD, PD, L]),
}


def _bind(sigs):
    l = lib()
    for name, (res, args) in sigs.items():
        fn = getattr(l, name)
        fn.restype = res
        fn.argtypes = args
    return l


class OracleOscbank:
    """CPU restatement of Oscbank<double,N> (src/oscbank.h:15-97)."""

    def __init__(self, N, k=2.0 / 48000):
        self.l = _bind(_OSC_SIGS)
        self.h = self.l.orc_osc_create(N, k)
        self.N = self.local_N = N

    def __del__(self):
        try:
            self.l.orc_osc_destroy(self.h)
        except Exception:
            pass

    def freqmod(self, i, hz):
        self.l.orc_osc_freqmod(self.h, int(i), float(hz))

    def activate(self, idx):
        a = np.ascontiguousarray(idx, dtype=np.int32)
        self.l.orc_osc_activate(self.h, a.ctypes.data_as(C.POINTER(C.c_int)), len(a))

    def deactivate(self, idx):
        a = np.ascontiguousarray(idx, dtype=np.int32)
        self.l.orc_osc_deactivate(self.h, a.ctypes.data_as(C.POINTER(C.c_int)), len(a))

    def open(self):
        self.l.orc_osc_open(self.h)

    def close_all(self):
        self.l.orc_osc_close(self.h)

    def active_count(self):
        return self.l.orc_osc_active_count(self.h)

    def fill(self, n, per_band=False):
        mix = np.zeros(2 * n)
        pb = np.zeros(2 * n * self.N) if per_band else None
        self.l.orc_osc_fill(self.h, _p(mix), _p(pb) if pb is not None else None, n)
        m = mix.view(np.complex128)
        if per_band:
            return m, pb.view(np.complex128).reshape(n, self.N)
        return m

    def phases(self):
        z = np.zeros(2 * self.N)
        self.l.orc_osc_phases(self.h, _p(z))
        return z.view(np.complex128)


def run_osc_events(bank, g):
    """Drive an Oscbank-like object through a golden fixture's events, splitting
    fill() at every event time."""
    t_ev, kind, index, value = g["ev_t"], g["ev_kind"], g["ev_index"], g["ev_value"]
    n = int(g["n"])
    out = np.zeros(n, dtype=np.complex128)
    pos = 0
    order = np.argsort(t_ev, kind="stable")
    times = sorted(set(t_ev.tolist())) + [n]
    for t in times:
        if t > pos:
            out[pos:t] = bank.fill(t - pos)
            pos = t
        if t >= n:
            break
        for e in order:
            if t_ev[e] != t:
                continue
            k = int(kind[e])
            if k == 0:
                bank.freqmod(int(index[e]), float(value[e]))
            elif k == 1:
                bank.activate([int(index[e])])
            elif k == 2:
                bank.deactivate([int(index[e])])
            elif k == 3:
                bank.open()
            elif k == 4:
                bank.close_all()
    return out
