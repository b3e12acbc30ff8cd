"""The column-split schedule of the stationary engine (tests/resp_col_model.py) against a direct
convolution: index algebra, the radix-4 unit split, the conjugate columns and the overlap-save
output half, before the HIP kernels that follow it run on a GPU."""
import numpy as np

import resp_col_model as m


def test_units_cover_columns_once():
    cols = [c for _, cl in m.units() for c in cl]
    canon = sorted(min(c, 64 - c) if c else 0 for c in cols)
    assert canon == list(range(33))


def test_stage1_unit_is_the_column_dft():
    rng = np.random.default_rng(1)
    seg = rng.standard_normal(m.P)
    U = seg.reshape(32, 64)
    for c0 in (0, 3, 8):
        D = m.stage1_unit(seg, c0)
        for i in range(4):
            c = c0 + 16 * i
            ref = (U * m.w(64, np.arange(32) * c)[:, None]).sum(0)
            assert np.allclose(D[i], ref, atol=1e-12)


def test_column_forward_is_the_window_spectrum():
    rng = np.random.default_rng(2)
    segs = rng.standard_normal((3, m.P))
    for c in (0, 5, 32, 47):
        D = np.array([(s.reshape(32, 64) * m.w(64, np.arange(32) * c)[:, None]).sum(0) for s in segs])
        Z = m.column_forward(segs, c, D)
        for j in range(2):
            X = np.fft.fft(np.concatenate([segs[j], segs[j + 1]]))
            assert np.allclose(Z[j], X[c + 64 * np.arange(64)], atol=1e-9)


def test_convolution_matches_direct():
    rng = np.random.default_rng(3)
    K, n = 4 * m.P, 3 * m.P + 777
    h = rng.standard_normal(K) * np.exp(-np.arange(K) / 2000.0)
    u = rng.standard_normal(K + n)
    y = m.convolve(u, h, K, n)
    ref = m.direct(u, h, K, n)
    assert np.max(np.abs(y - ref)) <= 1e-11 * np.max(np.abs(ref))
