"""BASELINE config C1: tests/resynthesis.cpp's 128-band Filterbank<double>
on 48 kHz mono, 1024-sample blocks -- the plumbing case the reference runs on the CPU.

Recipe (tests/resynthesis.cpp:23-27, 48-54): f_i = 0.5 (i+1) SR / 128, R = 0.999,
fwd {1/g, 0, -1/g}, back {-2 R cos theta_i, R^2}, g = |H(f_i)|, plus boost(1...) and open()
(the demo as written is silent); 2^16 samples of float32 white noise.

CPU: the C restatement against an independent model built from scipy.signal.lfilter: per band
u[t] = pre[t] (b . x)[t] (the pre-amp multiplies the whole feed-forward sum, filterbank.h:178),
y = lfilter([1], [1, a1, a2], u), out = sum_n gain[t] y_n[t], with the smoothers'
closed form pre[t] = 1 - s_p^(t+1), gain[t] = 1 - s_g^(t+1) (includes.h:43-48).
GPU: the HIP engine against the restatement over the same 64 blocks."""
import numpy as np
import pytest
import scipy.signal

from golden.spec_numpy import resonant_coefficients, white_noise_f32
from oracle import OracleFilterbank, rel_err

N, R, B, NB = 128, 0.999, 1024, 64
SR = 48000


def relaxation(k):
    return 0.0 if k == 0 else 2.0 ** (np.log2(np.finfo(np.float64).eps) / (max(0.0, k) * SR))


def setup(fb, fwd, back):
    for n in range(N):
        fb.coefficients(n, fwd[n], back[n])
    fb.boost(np.ones(N))
    fb.open()


def lfilter_model(fwd, back, x, k_p=0.1, k_g=1.0):
    t = np.arange(len(x), dtype=np.float64)
    pre = 1.0 - relaxation(k_p) ** (t + 1)
    gain = 1.0 - relaxation(k_g) ** (t + 1)
    out = np.zeros(len(x))
    for n in range(N):
        ff = scipy.signal.lfilter(fwd[n], [1.0], x)
        out += gain * scipy.signal.lfilter([1.0], [1.0, back[n][0], back[n][1]], pre * ff)
    return out


def test_c1_restatement_vs_lfilter_blocks():
    fwd, back = resonant_coefficients(N, R)
    x = white_noise_f32(B * NB, seed=1)
    o = OracleFilterbank(2, N, 0.1, 1.0)
    setup(o, fwd, back)
    y = np.concatenate([o.process(x[i * B:(i + 1) * B]) for i in range(NB)])
    ref = lfilter_model(fwd, back, x)
    assert np.max(np.abs(ref)) > 1.0
    assert rel_err(y, ref) < 1e-9


@pytest.mark.gpu
def test_c1_hip_vs_restatement_blocks(gpu_lib):
    from huygens_amd import Filterbank
    fwd, back = resonant_coefficients(N, R)
    x = white_noise_f32(B * NB, seed=1)
    g, o = Filterbank(2, N, 0.1, 1.0), OracleFilterbank(2, N, 0.1, 1.0)
    setup(g, fwd, back)
    setup(o, fwd, back)
    yg = np.concatenate([g.process(x[i * B:(i + 1) * B]) for i in range(NB)])
    yo = np.concatenate([o.process(x[i * B:(i + 1) * B]) for i in range(NB)])
    assert rel_err(yg, yo) < 1e-9
