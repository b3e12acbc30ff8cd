"""ctypes binding of the Fourier/StaticSTFT/Cosine restatement (oracle/hz_oracle_stft.c).
TEST INFRASTRUCTURE."""
from __future__ import annotations

import ctypes as C

import numpy as np

from oracle import D, I, L, PD, VP, _bind, _p

CB = C.CFUNCTYPE(C.c_int, PD, PD)
_SIGS = {
    "orc_stft_create": (VP, [I, I, I, I, D, D]),
    "orc_stft_set_callback": (None, [VP, CB]),
    "orc_stft_destroy": (None, [VP]),
    "orc_stft_write": (None, [VP, D, D]),
    "orc_stft_read": (None, [VP, PD, PD]),
    "orc_stft_process_block": (None, [VP, PD, PD, PD, PD, L]),
    "orc_stft_frames": (L, [VP]),
    "orc_stft_forward": (None, [VP, I]),
    "orc_stft_backward": (None, [VP, I]),
    "orc_stft_process_slot": (None, [VP, I]),
    "orc_dft": (None, [PD, PD, I, I]),
    "orc_dct": (None, [PD, PD, I, I]),
}

PROC_PARAMS = {0: (0.0, 0.0), 1: (100.0, 0.1), 2: (625.0, 0.0), 3: (0.0, 0.0)}


class OracleSTFT:
    """window 0 = halfhann (Fourier), 1 = hann (StaticSTFT); proc per ORC_PROC_*."""

    def __init__(self, N, laps, window=0, proc=0, callback=None):
        self.l = _bind(_SIGS)
        p0, p1 = PROC_PARAMS.get(proc, (0.0, 0.0))
        self.h = self.l.orc_stft_create(N, laps, window, proc, p0, p1)
        self._cb = None
        if callback is not None:
            self._cb = CB(callback)
            self.l.orc_stft_set_callback(self.h, self._cb)

    def __del__(self):
        try:
            self.l.orc_stft_destroy(self.h)
        except Exception:
            pass

    def process_block(self, re, im=None):
        re = np.ascontiguousarray(re, dtype=np.float64)
        n = re.size
        im_ = None if im is None else np.ascontiguousarray(im, dtype=np.float64)
        yr, yi = np.zeros(n), np.zeros(n)
        self.l.orc_stft_process_block(self.h, _p(re), _p(im_) if im_ is not None else None, _p(yr), _p(yi), n)
        return yr, yi

    def frames(self):
        return self.l.orc_stft_frames(self.h)

    def write(self, re, im=0.0):           # fourier.h:102-128
        self.l.orc_stft_write(self.h, float(re), float(im))

    def read(self):                          # fourier.h:147-177
        r, i = C.c_double(), C.c_double()
        self.l.orc_stft_read(self.h, C.byref(r), C.byref(i))
        return r.value, i.value

    def forward(self, slot):
        self.l.orc_stft_forward(self.h, slot)

    def backward(self, slot):
        self.l.orc_stft_backward(self.h, slot)

    def process(self, slot):
        self.l.orc_stft_process_slot(self.h, slot)


def oracle_dct(x, kind):
    l = _bind(_SIGS)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.zeros_like(x)
    l.orc_dct(_p(x), _p(y), x.size, kind)
    return y


def oracle_dft(x, sign):
    l = _bind(_SIGS)
    xi = np.ascontiguousarray(np.stack([np.real(x), np.imag(x)], -1).reshape(-1), dtype=np.float64)
    y = np.zeros_like(xi)
    l.orc_dft(_p(xi), _p(y), np.size(x), sign)
    return y[0::2] + 1j * y[1::2]
