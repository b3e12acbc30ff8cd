"""Modal band states (hz_fb_modal.h) on the GPU: banks on one pole circle get a stationary call's
band states from a fold and one 8192-point DFT instead of the matrix-core pass.  Checked against
the matrix-core pass (a twin handle with hz_fb_tune_modal(0)) and against the restatement; the
bank's next, per-band call continues from those states.  Model and CPU checks:
tests/modal_model.py, tests/test_modal_model_cpu.py."""
import numpy as np
import pytest

import modal_model as mm
from golden.spec_numpy import resonant_coefficients
from oracle import OracleFilterbank
from test_c2_pinned_gpu import block_errors

pytestmark = pytest.mark.gpu


def _bank(N, fwd, back, k_p=0.1, k_g=1.0, modal=True, bps=0):
    from huygens_amd import Filterbank
    g = Filterbank(2, N, k_p, k_g)
    for n in range(N):
        g.coefficients(n, fwd[n], back[n])
    g.boost(np.ones(N))
    g.open()
    g.tune_modal(modal)
    if bps:
        g.tune_response(bands_per_sample=bps)
    return g


def _to_stationary(gs, rng, n, calls=8):
    from huygens_amd._lib import HZ_FB_PATH_RESPONSE
    xs = []
    for _ in range(calls):
        x = rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64)
        xs.append(x)
        ys = [g.process(x) for g in gs]
        if all(g.last_path() == HZ_FB_PATH_RESPONSE for g in gs):
            return xs, ys
    raise AssertionError([g.last_path() for g in gs])


def test_modal_plan_flags(gpu_lib):
    fwd, back = resonant_coefficients(4096, 0.999, 1.0)
    g = _bank(4096, fwd, back)
    rng = np.random.default_rng(3)
    _to_stationary([g], rng, 200_000)
    on, ok, exc, last = g.modal_info()
    assert (on, ok, exc, last) == (True, True, 1, True)      # the Nyquist band: a direct sum
    assert g.response_engine() == (False, False)
    g.close()
    # a bank off the grid: the matrix-core pass
    rng2 = np.random.default_rng(9)
    th = np.sort(rng2.uniform(0.01, 3.1, 512))
    back2 = np.stack([-2 * 0.999 * np.cos(th), np.full(512, 0.999 ** 2)], 1)
    fwd2 = np.tile([0.01, 0.0, -0.01], (512, 1))
    g2 = _bank(512, fwd2, back2, bps=1)
    _to_stationary([g2], rng, 200_000)
    assert g2.modal_info()[1:] == (False, -1, False)
    g2.close()


@pytest.mark.parametrize("N,R,centre,n", [(4096, 0.999, 1.0, 200_000), (2048, 0.999, 0.5, 200_000),
                                          (4096, 0.9999, 1.0, 600_000),
                                          # calls shorter than the horizon (K = 507,904): the modal
                                          # window is the history's tail plus the call (round 6)
                                          (4096, 0.9999, 1.0, 480_000), (1024, 0.999, 1.0, 30_000)])
def test_modal_matches_matrix_core_pass(gpu_lib, N, R, centre, n):
    fwd, back = resonant_coefficients(N, R, centre)
    gm, gc = _bank(N, fwd, back, modal=True), _bank(N, fwd, back, modal=False)
    rng = np.random.default_rng(11)
    xs, ys = _to_stationary([gm, gc], rng, n)
    assert gm.modal_info()[3] and not gc.modal_info()[3]
    # outputs: the same convolution; states: modal against the matrix-core pass
    assert np.array_equal(ys[0], ys[1])
    sm, sc = gm.get_state()[2:2 + 2 * N], gc.get_state()[2:2 + 2 * N]
    exc = np.zeros(N, bool)
    if centre == 1.0:
        exc[-1] = True
    reg = np.repeat(~exc, 2)
    scale = np.max(np.abs(sc[reg]))
    # both against the numpy model of the modal pass (itself within 3e-13 of the restatement:
    # tests/test_modal_model_cpu.py) over the call's last K inputs
    K = gm.response_info()[0]
    win = np.concatenate(xs)[-K:]   # the last K inputs (across calls when the call is shorter)
    assert len(win) == K
    ref, _ = mm.states(win, fwd, back, np.ones(N), exc_direct=False)
    ref = ref.reshape(-1)
    em = np.max(np.abs(sm[reg] - ref[reg])) / scale
    ec = np.max(np.abs(sc[reg] - ref[reg])) / scale
    assert em <= 1e-11, (em, ec)
    assert ec <= 1e-8, (em, ec)   # the matrix-core pass: its FP64 MFMA chains over the window
    if exc.any():   # the direct sums against the model's (long-double response, numpy dot)
        e = np.repeat(exc, 2)
        dref = mm.direct(win, fwd[-1], back[-1], 1.0)
        es = np.max(np.abs(sm[e] - dref)) / np.max(np.abs(dref))
        ecx = np.max(np.abs(sc[e] - dref)) / np.max(np.abs(dref))
        assert es <= 1e-10, (es, ecx)
        assert ecx <= 1e-6, (es, ecx)
    # the next call on the per-band engines continues from them
    x = rng.uniform(-1, 1, 3000)
    gm.set_response(0)
    gc.set_response(0)
    y1, y2 = gm.process(x), gc.process(x)
    err, _ = block_errors(y1, y2)
    # (R = 0.9999: the matrix-core pass's Nyquist-band state is ~5e-8 off, see above)
    assert err.max() <= (1e-9 if R < 0.9999 else 1e-6)
    gm.close()
    gc.close()


def test_modal_states_against_restatement(gpu_lib):
    """a 256-band recipe bank (cost model opened up), states and the following blocks per block
    against the restatement"""
    N = 256
    fwd, back = resonant_coefficients(N, 0.999, 1.0)
    g = _bank(N, fwd, back, bps=1)
    o = OracleFilterbank(2, N, 0.1, 1.0)
    for b in range(N):
        o.coefficients(b, fwd[b], back[b])
    o.boost(np.ones(N))
    o.open()
    rng = np.random.default_rng(21)
    from huygens_amd._lib import HZ_FB_PATH_RESPONSE
    stationary = 0
    for _ in range(8):
        x = rng.uniform(-1, 1, 100_000).astype(np.float32).astype(np.float64)
        yg, yc = g.process(x), o.process(x)
        err, _ = block_errors(yg, yc)
        assert err.max() <= 1e-9, err.max()
        if g.last_path() == HZ_FB_PATH_RESPONSE:
            stationary += 1
            assert g.modal_info()[3]
            st_g, st_c = g.get_state(), o.get_state()
            d = np.abs(st_g[2:2 + 2 * N] - st_c[2:2 + 2 * N])
            assert d[:-2].max() <= 1e-10 * np.abs(st_c[2:2 * N]).max()
            # the Nyquist double pole (direct sum): the sequential recurrence itself carries ~1e-9 of
            # its state there
            assert d[-2:].max() <= 1e-8 * np.abs(st_c[2 * N:2 + 2 * N]).max()
    assert stationary >= 2
    for _ in range(4):   # short calls after stationary ones: the per-band engines from these states
        x = rng.uniform(-1, 1, 1500)
        err, _ = block_errors(g.process(x), o.process(x))
        assert err.max() <= 1e-9
    g.close()
