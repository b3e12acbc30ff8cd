"""Filterbank<double> over the HIP engine.

Mirrors soundmath::Filterbank<T> (src/filterbank.h:16-188): the same
constructor arguments, setters and operator()/tick() pair, plus the block
method process(x) == n x {y[i] = F(x[i]); F.tick();} that runs on the GPU.
The C++ drop-in is include/soundmath/filterbank.h; this Python mirror exists
for tests and bench.py.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import HZ_DIST_NONE, HZ_DIST_SOFTCLIP, PD, check, dptr, load


TV_COEFFS, TV_RESONANT = 0, 1   # HZ_FB_TV_*


class Filterbank:
    """Filterbank(order, N=1, k_p=0.1, k_g=1) -- src/filterbank.h:36-70.

    shard=(band_begin, band_count) makes this object own only those bands of an
    N-band bank (one process per GPU, partial mixes summed over RCCL)."""

    def __init__(self, order: int, N: int = 1, k_p: float = 0.1, k_g: float = 1.0,
                 device: int = 0, shard: tuple[int, int] | None = None):
        lib = load()
        h = C.c_void_p()
        if shard is None:
            check(lib.hz_fb_create(order, N, k_p, k_g, device, C.byref(h)))
        else:
            check(lib.hz_fb_create_shard(order, N, shard[0], shard[1], k_p, k_g, device, C.byref(h)))
        self._h = h
        self._lib = lib
        self.order = order
        self.N = N
        self.shard = shard
        self._dist = (HZ_DIST_NONE, 0.0)
        self._lti_geom = 1

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_fb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- setters (filterbank.h:73-116) ------------------------------------
    def coefficients(self, n: int, forward, back):
        f = np.ascontiguousarray(forward, dtype=np.float64)
        b = np.ascontiguousarray(back, dtype=np.float64)
        check(self._lib.hz_fb_coefficients(self._h, n, dptr(f), len(f), dptr(b), len(b)))

    def boost(self, n_or_values, value: float | None = None):
        if value is None:
            v = np.ascontiguousarray(n_or_values, dtype=np.float64)
            check(self._lib.hz_fb_boost_all(self._h, dptr(v), len(v)))
        else:
            check(self._lib.hz_fb_boost(self._h, int(n_or_values), float(value)))

    def mix(self, n_or_values, value: float | None = None):
        if value is None:
            v = np.ascontiguousarray(n_or_values, dtype=np.float64)
            check(self._lib.hz_fb_mix_all(self._h, dptr(v), len(v)))
        else:
            check(self._lib.hz_fb_mix(self._h, int(n_or_values), float(value)))

    def open(self):
        check(self._lib.hz_fb_open(self._h))

    def distortion(self, dist_id: int, param: float | None = None):
        """Select the per-band T(*)(T) of operator()(T, T(*)(T)) (filterbank.h:133); param None: the
        reference's default (softclip: the one-argument overload's width 0.125, the one &softclip
        names in tests/filterbank.cpp:168-171)."""
        param = dist_default_param(dist_id) if param is None else param
        check(self._lib.hz_fb_set_distortion(self._h, dist_id, param))
        self._dist = (dist_id, param)

    def tune(self, waves: int = 0, bands_per_wave: int = 0):
        check(self._lib.hz_fb_tune(self._h, waves, bands_per_wave))

    # ---- processing ----------------------------------------------------------
    def process(self, x) -> np.ndarray:
        """n x {out[i] = F(x[i]); F.tick();} on the GPU (host buffers)."""
        xi = np.ascontiguousarray(x, dtype=np.float64)
        out = np.empty_like(xi)
        if len(xi):
            check(self._lib.hz_fb_process(self._h, dptr(xi), dptr(out), len(xi)))
        return out

    def process_host(self, x_ptr: int, out_ptr: int, n: int):
        """Host pointers (e.g. pinned buffers), synchronous: H2D + engine + D2H (hz_fb_process)."""
        check(self._lib.hz_fb_process(self._h, C.cast(C.c_void_p(x_ptr), PD), C.cast(C.c_void_p(out_ptr), PD), n))

    def process_device(self, x_ptr: int, out_ptr: int, n: int):
        """Device pointers, asynchronous on the handle's stream."""
        check(self._lib.hz_fb_process_device(self._h, C.c_void_p(x_ptr), C.c_void_p(out_ptr), n))

    def process_tv(self, x, kind: int, stream, param: float = 0.0) -> np.ndarray:
        """Per-sample coefficient streams (hz_fb_process_tv): kind TV_COEFFS with stream
        [n][2*order+1][N] (forward then back, band-minor) or TV_RESONANT with stream [n][N]
        frequencies in Hz (order 2; Subtractive's resonant filters, R = param)."""
        xi = np.ascontiguousarray(x, dtype=np.float64)
        st = np.ascontiguousarray(stream, dtype=np.float64)
        out = np.empty_like(xi)
        check(self._lib.hz_fb_process_tv(self._h, dptr(xi), dptr(out), len(xi), kind, dptr(st), float(param)))
        return out

    def process_tv_device(self, x_ptr: int, out_ptr: int, n: int, kind: int, stream_ptr: int, param: float = 0.0):
        check(self._lib.hz_fb_process_tv_device(self._h, C.c_void_p(x_ptr), C.c_void_p(out_ptr), n, kind,
                                                C.c_void_p(stream_ptr), float(param)))

    def __call__(self, sample: float) -> float:
        """T operator()(T) / operator()(T, dist) (filterbank.h:125-139) on the GPU's per-sample
        engine (hz_fb_sample): cached until tick(); the distortion is the one set by distortion()."""
        y = C.c_double()
        check(self._lib.hz_fb_sample(self._h, float(sample), int(self._dist[0]), float(self._dist[1]),
                                     C.byref(y)))
        return y.value

    def tick(self):
        """tick() (filterbank.h:142-148): recorded, applied with the next sample (or block call)."""
        check(self._lib.hz_fb_sample_tick(self._h))

    def setter_seq(self) -> int:
        """per-sample calls served when the last setter ran (it applies from that call on)"""
        v = C.c_longlong()
        check(self._lib.hz_fb_setter_seq(self._h, C.byref(v)))
        return v.value

    def sample_info(self):
        """-> (in per-sample mode, samples served, server workgroups taking part)"""
        a, n, g = C.c_int(), C.c_longlong(), C.c_int()
        check(self._lib.hz_fb_sample_info(self._h, C.byref(a), C.byref(n), C.byref(g)))
        return bool(a.value), n.value, g.value

    # ---- stream / state ------------------------------------------------------
    def set_stream(self, stream_ptr: int | None):
        check(self._lib.hz_fb_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def stream(self) -> int:
        s = C.c_void_p()
        check(self._lib.hz_fb_get_stream(self._h, C.byref(s)))
        return s.value or 0

    def synchronize(self):
        check(self._lib.hz_fb_synchronize(self._h))

    def get_state(self) -> np.ndarray:
        n = C.c_size_t()
        check(self._lib.hz_fb_state_size(self._h, C.byref(n)))
        buf = np.zeros(n.value)
        check(self._lib.hz_fb_get_state(self._h, dptr(buf), n.value))
        return buf

    def set_state(self, buf):
        b = np.ascontiguousarray(buf, dtype=np.float64)
        check(self._lib.hz_fb_set_state(self._h, dptr(b), len(b)))

    def profile(self, enable: bool, repeat: int = 1):
        """HIP-event kernel timing; repeat > 1: the stationary engine's modal-path kernels run
        `repeat` times back to back between their events (times are per launch)"""
        check(self._lib.hz_fb_profile(self._h, max(1, int(repeat)) if enable else 0))

    def profile_read(self):
        """-> (segment pre-pass ms, mix kernel ms, reduce kernel ms, launches)"""
        s, m, r, c = C.c_double(), C.c_double(), C.c_double(), C.c_long()
        check(self._lib.hz_fb_profile_read(self._h, C.byref(s), C.byref(m), C.byref(r), C.byref(c)))
        return s.value, m.value, r.value, c.value

    def set_path(self, path: int):
        """HZ_FB_PATH_AUTO (converged LTI engine when eligible) or HZ_FB_PATH_GENERAL."""
        check(self._lib.hz_fb_set_path(self._h, int(path)))

    def last_path(self) -> int:
        p = C.c_int()
        check(self._lib.hz_fb_last_path(self._h, C.byref(p)))
        return p.value

    def tune_lti(self, chunk: int = 0, bands_per_wave: int = 0, waves: int = 0):
        check(self._lib.hz_fb_tune_lti(self._h, chunk, bands_per_wave, waves))
        self._lti_geom = {16: 0, 32: 1, 64: 2, 128: 3}.get(chunk, 1)

    def lti_chunk(self) -> int:
        """Samples per lane chunk of the last LTI launch (hz_fb_lti_last_chunk; the geometry
        is picked by call length unless pinned with tune_lti)."""
        c = C.c_int()
        check(self._lib.hz_fb_lti_last_chunk(self._h, C.byref(c)))
        return c.value or {0: 16, 1: 32, 2: 64, 3: 128}.get(self._lti_geom, 32)

    def lti_plan(self):
        """-> (time segments, prepass tiles skipped per segment, fine prepass parts) of the
        last LTI launch (hz_fb_lti_plan)."""
        a, b, c = C.c_long(), C.c_long(), C.c_int()
        check(self._lib.hz_fb_lti_plan(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def set_target_groups(self, groups: int):
        check(self._lib.hz_fb_set_target_groups(self._h, groups))

    # ---- stationary engine (hz_fb_resp.hip) ---------------------------------
    def set_response(self, mode: int):
        """HZ_FB_RESP_OFF (per-band engines only), _EAGER (default: band states computed after
        every stationary call) or _LAZY (band states computed when next needed)."""
        check(self._lib.hz_fb_set_response(self._h, int(mode)))

    def tune_response(self, min_call: int = 0, bands_per_sample: int = 0):
        """(tuning) shortest stationary call and the cost-model threshold (0s = defaults)."""
        check(self._lib.hz_fb_tune_response(self._h, int(min_call), int(bands_per_sample)))

    def tune_response_engine(self, column_split: bool = True):
        """(A/B) 1 = column-split long calls, 0 = the three-kernel path (default)"""
        check(self._lib.hz_fb_tune_response_engine(self._h, 1 if column_split else 0))

    def response_engine(self):
        """-> (column split enabled, last stationary call ran it)"""
        a, b = C.c_int(), C.c_int()
        check(self._lib.hz_fb_response_engine(self._h, C.byref(a), C.byref(b)))
        return bool(a.value), b.value == 1

    def tune_modal(self, on: bool = True):
        """modal band states for banks on one pole circle (default on; off: the matrix-core pass)"""
        check(self._lib.hz_fb_tune_modal(self._h, 1 if on else 0))

    def modal_info(self):
        """-> (enabled, the bank qualifies, exceptional bands (-1: does not qualify), last stationary
        call used it)"""
        v = [C.c_int() for _ in range(4)]
        check(self._lib.hz_fb_modal_info(self._h, *[C.byref(x) for x in v]))
        return bool(v[0].value), bool(v[1].value), v[2].value, bool(v[3].value)

    def response_info(self):
        """-> (horizon K, stationary samples so far, band states implicit, stationary calls)"""
        k, r, i, c = C.c_long(), C.c_long(), C.c_int(), C.c_long()
        check(self._lib.hz_fb_response_info(self._h, C.byref(k), C.byref(r), C.byref(i), C.byref(c)))
        return k.value, r.value, bool(i.value), c.value

    def response(self, count: int) -> np.ndarray:
        """The converged bank's response h[0 .. count): sum_n gin_n (impulse response of band n
        at pre = pin_n), truncated at the horizon."""
        out = np.zeros(count)
        check(self._lib.hz_fb_get_response(self._h, dptr(out), count))
        return out

    def set_bank_response(self, h):
        """The whole bank's response (sum of the shards' response()) for time-range shards."""
        v = np.ascontiguousarray(h, dtype=np.float64)
        check(self._lib.hz_fb_set_bank_response(self._h, dptr(v), len(v)))

    def set_time_shard(self, rank: int, world: int):
        check(self._lib.hz_fb_set_time_shard(self._h, int(rank), int(world)))

    def set_time_shard_fill(self, zero_outside: bool = True):
        """zero_outside: zeros outside this rank's share (the ranks' outputs sum to the mix);
        False: the share only, the rest of the output untouched (disjoint shares)."""
        check(self._lib.hz_fb_set_time_shard_fill(self._h, 1 if zero_outside else 0))

    def stationary_ready(self, n: int) -> bool:
        """Would a call of n samples run stationary on this handle (ignoring arming)?"""
        r = C.c_int()
        check(self._lib.hz_fb_stationary_ready(self._h, int(n), C.byref(r)))
        return bool(r.value)

    def arm_time_shard(self, armed: bool = True):
        """Time-sharded handles run stationary exactly when armed (set on every rank alike:
        huygens_amd.shard.arm_when_ready)."""
        check(self._lib.hz_fb_arm_time_shard(self._h, 1 if armed else 0))

    def time_shard_info(self, n: int):
        """-> (active, first sample, count) of a stationary call of n samples on this rank"""
        a, f, c = C.c_int(), C.c_long(), C.c_long()
        check(self._lib.hz_fb_time_shard_info(self._h, C.byref(a), C.byref(f), C.byref(c), int(n)))
        return bool(a.value), f.value, c.value

    def tune_stream(self, enable: bool = True):
        """Streaming engine for 1024-sample calls of a stationary bank (hz_fb_stream.hip) on / off."""
        check(self._lib.hz_fb_tune_stream(self._h, 1 if enable else 0))

    def stream_info(self):
        """-> (enabled, call length, streamed calls, history in the ring)"""
        e, b, c, r = C.c_int(), C.c_long(), C.c_long(), C.c_int()
        check(self._lib.hz_fb_stream_info(self._h, C.byref(e), C.byref(b), C.byref(c), C.byref(r)))
        return bool(e.value), b.value, c.value, bool(r.value)


def dist_default_param(dist_id: int) -> float:
    """HZ_DIST_DEFAULT_PARAM: softclip's width 0.125 (tests/filterbank.cpp:168-171), else 0"""
    return 0.125 if dist_id == HZ_DIST_SOFTCLIP else 0.0


def sample_many(banks, x, dist: int = HZ_DIST_NONE, param: float | None = None) -> np.ndarray:
    """One sample of several Filterbanks in one per-sample server request (hz_fb_sample_many):
    y[i] = banks[i](x[i], dist) -- each bank's tick() stays separate (tests/filterbanks.cpp:191-211)."""
    n = len(banks)
    lib = banks[0]._lib
    hs = (C.c_void_p * n)(*[b._h for b in banks])
    xs = np.ascontiguousarray(x, dtype=np.float64)
    if xs.shape != (n,):
        raise ValueError(f"sample_many: x must hold one value per bank ({n}), got shape {xs.shape}")
    ys = np.empty(n)
    param = dist_default_param(dist) if param is None else param
    check(lib.hz_fb_sample_many(hs, n, xs.ctypes.data_as(PD), int(dist), float(param), ys.ctypes.data_as(PD)))
    return ys
