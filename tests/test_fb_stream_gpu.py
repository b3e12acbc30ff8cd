"""Streaming calls of a stationary bank (hz_fb_stream.hip, HZ_FB_PATH_STREAM): 1024-sample
blocks -- the reference's audio callback, tests/resynthesis.cpp:33-42 over
src/filterbank.h:125-148 -- one launch each, against the C restatement PER BLOCK, across the
switches between the per-band, stationary and streaming engines, through setters, get_state,
long calls, ragged calls and the per-sample path.

Criterion: ||y_gpu - y_cpu||_inf <= 1e-5 ||y_cpu||_inf per 1024-sample block
(north star); the tests hold the engines to 1e-7 (the Nyquist double pole of the reference
recipe is an ill-conditioned recurrence in any summation order)."""
import numpy as np
import pytest

from golden.spec_numpy import resonant_coefficients
from oracle import OracleFilterbank
from test_c2_pinned_gpu import NORTH_STAR, TIGHT, ThreadedOracle, block_errors

pytestmark = pytest.mark.gpu

B = 1024


def _bank(N, R=0.999, k_p=0.1, k_g=1.0):
    from huygens_amd import Filterbank
    fwd, back = resonant_coefficients(N, R, 1.0)
    g = Filterbank(2, N, k_p, k_g)
    o = OracleFilterbank(2, N, k_p, k_g)
    for fb in (g, o):
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
        fb.boost(np.ones(N))
        fb.open()
    return g, o


def _check(yg, yc, tol=TIGHT):
    err, _ = block_errors(yg, yc)
    assert err.max() <= tol, (err.max(), int(err.argmax()))
    return float(err.max())


def test_stream_small_bank_switches(gpu_lib):
    from huygens_amd._lib import HZ_FB_PATH_LTI, HZ_FB_PATH_RESPONSE, HZ_FB_PATH_STREAM
    N = 256
    g, o = _bank(N, R=0.99, k_p=0.01, k_g=0.01)
    g.tune_response(0, 1)   # long calls of this small bank stationary too (cost model off)
    rng = np.random.default_rng(5)

    def run(n):
        x = rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64)
        yg, yc = g.process(x), o.process(x)
        _check(yg, yc)
        return g.last_path()

    # per-band 1024-sample calls until converged for K: they keep the history, then stream
    paths = [run(B) for _ in range(40)]
    K = g.response_info()[0]
    assert 0 < K <= 65536, K
    assert HZ_FB_PATH_STREAM in paths, paths
    first = paths.index(HZ_FB_PATH_STREAM)
    assert all(p == HZ_FB_PATH_STREAM for p in paths[first:]), paths
    assert g.stream_info()[3]   # history in the ring
    # band states after streamed calls (materialised on demand)
    st_g, st_c = g.get_state(), o.get_state()
    sc = np.max(np.abs(st_c[2:2 + 2 * N]))
    assert np.max(np.abs(st_g[2:2 + 2 * N] - st_c[2:2 + 2 * N])) <= TIGHT * sc
    assert np.array_equal(st_g[:2], st_c[:2])
    assert np.max(np.abs(st_g[2 + 2 * N:] - st_c[2 + 2 * N:])) <= 1e-12
    # streaming resumes after get_state without a gap
    assert run(B) == HZ_FB_PATH_STREAM
    # a long call: stationary engine from the ring's history, then streaming again
    assert run(40000) == HZ_FB_PATH_RESPONSE
    assert [run(B) for _ in range(3)] == [HZ_FB_PATH_STREAM] * 3
    # a ragged call restarts the history: per-band until K more 1024-sample calls
    assert run(1000) != HZ_FB_PATH_STREAM
    p2 = [run(B) for _ in range(K // B + 2)]
    assert p2[0] == HZ_FB_PATH_LTI and p2[-1] == HZ_FB_PATH_STREAM, p2
    # a setter: smoothers move (general), converge (LTI), K later stream again
    g.boost(np.full(N, 0.5))
    o.boost(np.full(N, 0.5))
    p3 = [run(B) for _ in range(K // B + 12)]
    assert p3[0] != HZ_FB_PATH_STREAM and p3[-1] == HZ_FB_PATH_STREAM, p3
    # the per-sample path after streamed calls (states materialised for the resident kernel)
    xs = rng.uniform(-1, 1, 64)
    yg = np.array([(g(v), g.tick())[0] for v in xs])
    yc = np.array([(o(v), o.tick())[0] for v in xs])
    assert np.max(np.abs(yg - yc)) <= TIGHT * max(1e-300, np.max(np.abs(yc)))
    # and block calls after it
    assert run(B) != HZ_FB_PATH_STREAM
    g.close()


def test_stream_disabled_and_impulse_zeros(gpu_lib):
    """tune_stream(False) keeps 1024-sample calls on the per-band engines (same outputs); an
    impulse followed by silence past the horizon streams exact zeros (the truncation)."""
    from huygens_amd._lib import HZ_FB_PATH_STREAM
    N = 128
    g, o = _bank(N, R=0.99, k_p=0.01, k_g=0.01)
    g2, _ = _bank(N, R=0.99, k_p=0.01, k_g=0.01)
    g2.tune_stream(False)
    rng = np.random.default_rng(6)
    for i in range(40):
        x = rng.uniform(-1, 1, B)
        y1, y2, yc = g.process(x), g2.process(x), o.process(x)
        _check(y1, yc)
        _check(y2, yc)
        assert g2.last_path() != HZ_FB_PATH_STREAM
    assert g.last_path() == HZ_FB_PATH_STREAM
    K = g.response_info()[0]
    x = np.zeros(B)
    x[17] = 1.0
    outs_g, outs_c = [], []
    for i in range(K // B + 4):
        outs_g.append(g.process(x))
        outs_c.append(o.process(x))
        assert g.last_path() == HZ_FB_PATH_STREAM
        x = np.zeros(B)
    yg, yc = np.concatenate(outs_g), np.concatenate(outs_c)
    peak = np.max(np.abs(yc))
    err, bpeak = block_errors(yg, yc)
    live = bpeak > 2.0 ** -40 * peak
    assert err[live].max() <= NORTH_STAR
    for b in np.flatnonzero(~live):
        assert np.max(np.abs(yg[b * B:(b + 1) * B] - yc[b * B:(b + 1) * B])) <= 2.0 ** -50 * peak, b
    # past the horizon (+ the window of the impulse's block): exact zeros
    t_dead = 17 + K + 2 * B
    assert np.all(yg[t_dead:] == 0.0)
    g.close()
    g2.close()


def test_stream_c2_exact_config_per_block(gpu_lib):
    """The BASELINE C2 config streamed: Filterbank<double>(2, 4096), reference recipe (R = 0.999,
    Nyquist double pole), k_p 0.1, k_g 1, white noise float32 -> double; two 10 s calls make it
    stationary, then 1024-sample calls: streaming engine, per block against the restatement,
    through a boost setter (general -> LTI -> per-band 1024 calls keeping the history -> streaming
    again) and a get_state."""
    from huygens_amd import Filterbank
    from huygens_amd._lib import HZ_FB_PATH_GENERAL, HZ_FB_PATH_LTI, HZ_FB_PATH_STREAM
    N = 4096
    fwd, back = resonant_coefficients(N, 0.999, 1.0)
    g = Filterbank(2, N, 0.1, 1.0)
    for n in range(N):
        g.coefficients(n, fwd[n], back[n])
    g.boost(np.ones(N))
    g.open()
    o = ThreadedOracle(fwd, back)
    rng = np.random.default_rng(1234)
    for _ in range(2):
        x = rng.uniform(-1, 1, 480_000).astype(np.float32).astype(np.float64)
        _check(g.process(x), o.process(x))
    paths, worst = [], 0.0

    def block():
        nonlocal worst
        x = rng.uniform(-1, 1, B).astype(np.float32).astype(np.float64)
        yg, yc = g.process(x), o.process(x)
        e = _check(yg, yc)
        assert e <= NORTH_STAR
        worst = max(worst, e)
        paths.append(g.last_path())

    for _ in range(40):
        block()
    assert paths == [HZ_FB_PATH_STREAM] * 40, paths
    st_g, st_c = g.get_state(), o.state()
    sc = np.max(np.abs(st_c[2:2 + 2 * N]))
    assert np.max(np.abs(st_g[2:2 + 2 * N] - st_c[2:2 + 2 * N])) <= TIGHT * sc
    assert np.array_equal(st_g[:2], st_c[:2])
    # boost setter mid-stream (the reference's MIDI thread: tests/filterbank.cpp:236-244)
    g.boost(np.full(N, 0.75))
    for _, _, sh in o.shards:
        sh.boost(np.full(sh_count(sh), 0.75))
    for _ in range(120):
        block()
    after = paths[40:]
    assert after[0] == HZ_FB_PATH_GENERAL, after[:4]
    assert HZ_FB_PATH_LTI in after and after[-1] == HZ_FB_PATH_STREAM, after
    print("C2 streamed blocks: worst per-block error %.3e, paths after the setter %s" % (worst, after))
    g.close()


def sh_count(o):
    return o.N


def test_stream_horizon_shrinks_after_coefficients(gpu_lib):
    """ a bank streamed with a long horizon, then coefficients with a shorter one: the
    partition-spectra rows past the new Q must be zeros again (they held the old response's
    spectra), so every streamed block after the change still matches the restatement."""
    from huygens_amd._lib import HZ_FB_PATH_STREAM
    N = 128
    g, o = _bank(N, R=0.999, k_p=0.01, k_g=0.01)
    rng = np.random.default_rng(11)

    def run():
        x = rng.uniform(-1, 1, B).astype(np.float32).astype(np.float64)
        _check(g.process(x), o.process(x))
        return g.last_path()

    K1 = None
    for _ in range(120):
        if run() == HZ_FB_PATH_STREAM:
            K1 = g.response_info()[0]
            break
    assert K1 is not None
    for _ in range(8):
        assert run() == HZ_FB_PATH_STREAM
    fwd, back = resonant_coefficients(N, 0.99, 1.0)
    for fb in (g, o):
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
    log = []
    for _ in range(40):
        x = rng.uniform(-1, 1, B).astype(np.float32).astype(np.float64)
        err, _ = block_errors(g.process(x), o.process(x))
        log.append((g.last_path(), float(err.max())))
    assert max(e for _, e in log) <= TIGHT, log
    paths = [p for p, _ in log]
    K2 = g.response_info()[0]
    assert 0 < K2 < K1, (K1, K2)
    assert paths[-1] == HZ_FB_PATH_STREAM, paths
    assert sum(p == HZ_FB_PATH_STREAM for p in paths) >= 10, paths
    g.close()


def test_stream_mix_mid_stream(gpu_lib):
    """ mix() after streamed blocks: the gain smoothers glide from the gains the
    streamed samples ran with (their lazy upkeep is applied before the new targets are
    uploaded), per block against the restatement; the same for a one-band mix(n, v)."""
    from huygens_amd._lib import HZ_FB_PATH_STREAM
    N = 128
    g, o = _bank(N, R=0.99, k_p=0.01, k_g=0.001)
    rng = np.random.default_rng(12)

    def run():
        x = rng.uniform(-1, 1, B).astype(np.float32).astype(np.float64)
        _check(g.process(x), o.process(x))
        return g.last_path()

    paths = [run() for _ in range(60)]
    assert paths[-1] == HZ_FB_PATH_STREAM, paths
    gains = rng.uniform(0.2, 1.5, N)
    g.mix(gains)
    o.mix(gains)
    for _ in range(6):
        run()
    for _ in range(20):
        run()
    g.mix(5, 0.1)
    o.mix(5, 0.1)
    for _ in range(6):
        run()
    g.close()


def test_stream_high_q_tail(gpu_lib):
    """ a horizon past the head's 2^17 samples (R = 0.9999: K ~ 0.4-0.5 M): the
    1024-sample calls stream in one launch each, the response tail h[K1, K) added from per-epoch
    (16384-sample) convolutions issued ahead on a side stream -- per block against the restatement
    over several epochs, through a long call, a setter and get_state."""
    from huygens_amd._lib import HZ_FB_PATH_RESPONSE, HZ_FB_PATH_STREAM
    N = 64
    g, o = _bank(N, R=0.9999, k_p=0.01, k_g=0.01)
    g.tune_response(bands_per_sample=1)   # a 64-band bank: let the cost model pick the engines
    rng = np.random.default_rng(31)

    def run(n, tol=1e-6):
        x = rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64)
        yg, yc = g.process(x), o.process(x)
        err, _ = block_errors(yg, yc)
        assert err.max() <= tol, (n, g.last_path(), err.max())
        return g.last_path()

    # long calls until stationary (the horizon needs K converged samples)
    paths = [run(200_000) for _ in range(6)]
    K = g.response_info()[0]
    assert K > 1 << 17, K
    assert paths[-1] == HZ_FB_PATH_RESPONSE, paths
    bp = [run(B) for _ in range(70)]   # > 4 epochs of 16 blocks
    assert all(p == HZ_FB_PATH_STREAM for p in bp), bp
    st_g, st_c = g.get_state(), o.get_state()
    sc = np.max(np.abs(st_c[2:2 + 2 * N]))
    assert np.max(np.abs(st_g[2:2 + 2 * N] - st_c[2:2 + 2 * N])) <= 1e-6 * sc
    assert [run(B) for _ in range(20)] == [HZ_FB_PATH_STREAM] * 20
    assert run(50_000) == HZ_FB_PATH_RESPONSE
    assert [run(B) for _ in range(40)] == [HZ_FB_PATH_STREAM] * 40
    g.close()
