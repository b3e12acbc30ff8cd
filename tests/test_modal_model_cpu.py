"""The modal band-state pass (tests/modal_model.py, the schedule hz_fb_modal.h follows) against the
sequential restatement on the CPU: the four-step DFT against numpy's, and the band states of
resonator banks on one pole circle (the recipe's Nyquist band through the direct sum) against the
restatement's state after a long run."""
import numpy as np
import pytest

import modal_model as mm
from golden.spec_numpy import resonant_coefficients
from oracle import OracleFilterbank


def test_four_step_is_the_dft():
    rng = np.random.default_rng(1)
    F = rng.standard_normal(mm.L)
    ref = np.fft.ifft(F) * mm.L          # sum_r e^(+2 pi i m r / L) F[r]
    assert np.allclose(mm.four_step(F), ref, rtol=0, atol=1e-10 * np.abs(ref).max())


def test_plan_recipe_and_off_grid():
    fwd, back = resonant_coefficients(1024, 0.999, 1.0)
    m, c, p, exc, Rg = mm.plan(back[:, 0], back[:, 1], 49152)
    assert list(np.nonzero(exc)[0]) == [1023]               # the Nyquist double pole
    assert list(m[:4]) == [4, 8, 12, 16]                    # theta = pi (i + 1) / 1024 = 2 pi 4 (i + 1) / 8192
    back2 = back.copy()
    back2[5, 0] *= 1 + 1e-9                                 # one band off the grid
    assert mm.plan(back2[:, 0], back2[:, 1], 49152) is None


@pytest.mark.parametrize("N,R,centre", [(512, 0.999, 1.0), (512, 0.99, 0.5)])
def test_states_against_restatement(N, R, centre):
    K = 49152
    fwd, back = resonant_coefficients(N, R, centre)
    x = np.random.default_rng(5).uniform(-1, 1, K + 8000).astype(np.float32).astype(np.float64)
    o = OracleFilterbank(2, N, 0.1, 1.0)
    for b in range(N):
        o.coefficients(b, fwd[b], back[b])
    o.boost(np.ones(N))
    o.open()
    o.process(x)
    ys = o.get_state()[2:2 + 2 * N].reshape(N, 2)
    s, exc = mm.states(x[-K:], fwd, back, np.ones(N))
    ne = ~exc
    assert np.max(np.abs(s[ne] - ys[ne])) <= 1e-11 * np.max(np.abs(ys[ne]))
    if exc.any():
        assert np.max(np.abs(s[exc] - ys[exc])) <= 1e-11 * np.max(np.abs(ys[exc]))
