"""Fourier / StaticSTFT / Cosine over the HIP engine.

Fourier(processor, N, laps)   src/fourier.h:50-194 (halfhann windows)
StaticSTFT(N, laps)           src/staticSTFT.h:10-177 (hann windows, built-in gate)
Cosine(N)                     src/fourier.h:197-234 (REDFT10 forward, REDFT01 backward)

process_block(re, im) == n x { write(re[t], im[t]); read(&re_out, &im_out); }.
A processor is a built-in id (PROC_*) or a Python callable f(inp, out) over complex128
arrays of length N, run per frame in frame order (host path).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dptr, load

WIN_HALFHANN, WIN_HANN = 0, 1
PROC_IDENTITY, PROC_STATIC_GATE, PROC_GATE_KEEP, PROC_HILBERT, PROC_HOST = 0, 1, 2, 3, 4
_PARAMS = {PROC_STATIC_GATE: (100.0, 0.1), PROC_GATE_KEEP: (625.0, 0.0)}
PROC_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double))


class Fourier:
    def __init__(self, processor=PROC_IDENTITY, N: int = 4096, laps: int = 4, window: int = WIN_HALFHANN,
                 device: int = 0):
        lib = load()
        builtin = processor if isinstance(processor, int) else PROC_HOST
        p0, p1 = _PARAMS.get(builtin, (0.0, 0.0))
        h = C.c_void_p()
        check(lib.hz_stft_create(N, laps, window, builtin, p0, p1, device, C.byref(h)))
        self._h, self._lib, self.N, self.laps = h, lib, N, laps
        self._cb = None
        if builtin == PROC_HOST:
            user = processor

            def tramp(inp, out):
                a = np.ctypeslib.as_array(inp, shape=(2 * N,)).view(np.complex128)
                b = np.ctypeslib.as_array(out, shape=(2 * N,)).view(np.complex128)
                r = user(a, b)
                return int(r or 0)

            self._cb = PROC_FN(tramp)
            check(lib.hz_stft_set_processor(h, C.cast(self._cb, C.c_void_p)))

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_stft_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process_block(self, re, im=None):
        re = np.ascontiguousarray(re, dtype=np.float64)
        n = re.size
        imv = None if im is None else np.ascontiguousarray(im, dtype=np.float64)
        yr, yi = np.zeros(n), np.zeros(n)
        if n:
            check(self._lib.hz_stft_process_block(self._h, dptr(re), dptr(imv) if imv is not None else None,
                                                  dptr(yr), dptr(yi), n))
        return yr, yi

    def process_block_device(self, re_ptr, im_ptr, ore_ptr, oim_ptr, n):
        check(self._lib.hz_stft_process_block_device(self._h, C.c_void_p(re_ptr), C.c_void_p(im_ptr or 0),
                                                     C.c_void_p(ore_ptr), C.c_void_p(oim_ptr or 0), n))

    def frames(self):
        f, t = C.c_long(), C.c_long()
        check(self._lib.hz_stft_frames(self._h, C.byref(f), C.byref(t)))
        return f.value, t.value

    # ---- per-sample operator API (fourier.h:102-177), exact state machine -----------------
    def write(self, re: float, im: float = 0.0):
        check(self._lib.hz_stft_write(self._h, float(re), float(im)))

    def read(self):
        r, i = C.c_double(), C.c_double()
        check(self._lib.hz_stft_read(self._h, C.byref(r), C.byref(i)))
        return r.value, i.value

    def forward(self, slot: int):
        check(self._lib.hz_stft_forward(self._h, int(slot)))

    def backward(self, slot: int):
        check(self._lib.hz_stft_backward(self._h, int(slot)))

    def process(self, slot: int):
        check(self._lib.hz_stft_process_slot(self._h, int(slot)))

    def set_frame_shard(self, rank: int, world: int, block: int):
        """Time-range shard: compute frame f iff (f // block) % world == rank
        (hz_stft_set_frame_shard); the ranks' outputs sum to the unsharded output."""
        check(self._lib.hz_stft_set_frame_shard(self._h, int(rank), int(world), int(block)))

    def set_stream(self, stream_ptr):
        check(self._lib.hz_stft_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        check(self._lib.hz_stft_synchronize(self._h))

    def profile(self, enable: bool, repeat: int = 1):
        """Event-time the frame / overlap-add kernels; repeat > 1 launches each block's frame
        kernel `repeat` times back to back (per-launch time without the event overhead)."""
        check(self._lib.hz_stft_profile(self._h, max(1, int(repeat)) if enable else 0))

    def profile_read(self):
        a, b, c = C.c_double(), C.c_double(), C.c_long()
        check(self._lib.hz_stft_profile_read(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value


def frames_before(N: int, laps: int, samples: int) -> int:
    """Frames completing within the first `samples` samples (hz_stft_frames_before)."""
    f = C.c_long()
    check(load().hz_stft_frames_before(N, laps, int(samples), C.byref(f)))
    return f.value


class StaticSTFT(Fourier):
    def __init__(self, N: int = 4096, laps: int = 4, device: int = 0):
        super().__init__(PROC_STATIC_GATE, N, laps, WIN_HANN, device)


class Cosine:
    """Cosine(N, &in, &out): `inp` / `out` are numpy views of the handle's pinned buffers."""

    def __init__(self, N: int, device: int = 0):
        lib = load()
        h = C.c_void_p()
        check(lib.hz_dct_create(N, device, C.byref(h)))
        pi, po = C.POINTER(C.c_double)(), C.POINTER(C.c_double)()
        check(lib.hz_dct_buffers(h, C.byref(pi), C.byref(po)))
        self._h, self._lib, self.N = h, lib, N
        self.inp = np.ctypeslib.as_array(pi, shape=(N,))
        self.out = np.ctypeslib.as_array(po, shape=(N,))

    def close(self):
        if getattr(self, "_h", None):
            self.inp = self.out = None
            self._lib.hz_dct_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def forward(self):
        check(self._lib.hz_dct_forward(self._h))

    def backward(self):
        check(self._lib.hz_dct_backward(self._h))

    def forward_device(self, in_ptr, out_ptr, batch=1):
        check(self._lib.hz_dct_forward_device(self._h, C.c_void_p(in_ptr), C.c_void_p(out_ptr), batch))

    def backward_device(self, in_ptr, out_ptr, batch=1):
        check(self._lib.hz_dct_backward_device(self._h, C.c_void_p(in_ptr), C.c_void_p(out_ptr), batch))
