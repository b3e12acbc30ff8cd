"""The streaming stationary engine's algebra (tests/stream_model.py, restating
hz_fb_stream.hip) against a direct truncated convolution: out[t] = sum_{tau < K} h[tau]
x[t - tau], on the CPU."""
import numpy as np

from stream_model import COLS, F, P, StreamModel, col_forward, col_inverse, final_stage


def test_column_transform_is_the_dft():
    rng = np.random.default_rng(0)
    win = rng.standard_normal(F)
    X = np.fft.fft(win)
    for c in range(COLS):
        got = col_forward(win, c)
        np.testing.assert_allclose(got, X[c + 64 * np.arange(32)], rtol=0, atol=1e-11)


def test_inverse_columns_and_final_stage():
    rng = np.random.default_rng(1)
    y = rng.standard_normal(F)
    Y = np.fft.fft(y)
    Cs = [col_inverse(Y[c + 64 * np.arange(32)], c) for c in range(COLS)]
    # unnormalised inverse: F * y, last P samples
    np.testing.assert_allclose(final_stage(Cs), F * y[P:], rtol=0, atol=1e-9)


def test_stream_blocks_equal_truncated_convolution():
    rng = np.random.default_rng(2)
    K = 8 * P
    h = rng.standard_normal(K) * np.exp(-np.arange(K) / 2000.0)
    hist = rng.standard_normal(K)
    m = StreamModel(h)
    m.prime(hist)
    xs = rng.standard_normal(4 * P)
    full = np.concatenate([hist, xs])
    for b in range(4):
        out = m.block(xs[b * P:(b + 1) * P])
        t0 = K + b * P
        ref = np.array([np.dot(h, full[t - K + 1:t + 1][::-1]) for t in range(t0, t0 + P)])
        np.testing.assert_allclose(out, ref, rtol=0, atol=1e-10 * np.abs(ref).max())
