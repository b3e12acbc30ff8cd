"""GPU parity of the stationary Filterbank engine (huygens_amd/csrc/hz_fb_resp.hip).

Once a converged bank (pre = pin, gain = gin) has kept its coefficients for K samples -- K its
horizon, ||M^K||_inf < 2^-53 for every band, rounded up to a multiple of 8192 (49,152 samples at
C2; inputs older than K reach an output below 2^-53 of their own scale, the bound
tests/test_c2_pinned_gpu.py::test_impulse_then_silence_horizon_bound asserts as 2^-50 of the
peak) -- long calls run as ONE partitioned FFT convolution of
the input with the bank response h = sum_n gin_n r_n (src/filterbank.h:130,178-179 summed over
bands), and the band states at the call end are the zero-start response of the last K inputs.
Every test drives the GPU object and the CPU restatement (oracle/hz_oracle.c) through the same
calls (mix bound 1e-9 of the mix, as for the other engines) and asserts which engine ran
(last_path); band states are compared with a twin handle that keeps the per-band LTI engine.
"""
import os

import numpy as np
import pytest

from golden.spec_numpy import resonant_coefficients, white_noise_f32
from oracle import OracleFilterbank, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-9


def paths():
    from huygens_amd import _lib
    return _lib


def make(order, N, fwd, back, kp=0.001, kg=0.001, boost=None, gains=None, mode=None, oracle=True,
         force=True):
    from huygens_amd import Filterbank
    L = paths()
    g = Filterbank(order, N, kp, kg)
    g.set_response(L.HZ_FB_RESP_EAGER if mode is None else mode)
    if force:   # small test banks: stationary whenever it is legal (cost model off)
        g.tune_response(0, 1)
    objs = [g]
    o = None
    if oracle:
        o = OracleFilterbank(order, N, kp, kg)
        objs.append(o)
    for fb in objs:
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
        fb.boost(np.ones(N) if boost is None else boost)
        if gains is None:
            fb.open()
        else:
            fb.mix(gains)
    return g, o


def states_close(a, b, tol=1e-9):
    return np.max(np.abs(a - b)) <= tol * max(1.0, np.max(np.abs(b)))


def test_c2_recipe_paths_and_parity(gpu_lib):
    """C2 coefficient recipe on 1024 bands: general (smoothers moving) -> LTI while the history
    fills -> stationary, ragged lengths, a short call (LTI; history restarts), back to
    stationary; the band states equal the per-band LTI twin's after each call."""
    L = paths()
    N = 1024
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make(2, N, fwd, back)
    t, _ = make(2, N, fwd, back, mode=L.HZ_FB_RESP_OFF, oracle=False)
    K = None
    rng = np.random.default_rng(5)
    lengths = [3000, 40000, 30000, 100000, 70001, 16384, 5000, 30000, 30000, 40000]
    for i, n in enumerate(lengths):
        x = rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64)
        yg, yo, yt = g.process(x), o.process(x), t.process(x)
        assert rel_err(yg, yo) < TOL, (i, n, rel_err(yg, yo))
        assert rel_err(yt, yo) < TOL, (i, n)
        K, run, implicit, calls = g.response_info()
        assert not implicit
        assert K > 0 or i == 0   # computed once the bank converged
        p = g.last_path()
        if i in (3, 4, 5, 9):
            assert p == L.HZ_FB_PATH_RESPONSE, (i, n, p, run, K)
        else:
            assert p != L.HZ_FB_PATH_RESPONSE, (i, n, p, run, K)
        assert states_close(g.get_state(), t.get_state()), i
    assert 40960 <= K <= 65536, K   # R = 0.999: 45056
    assert g.response_info()[3] == 4


def test_lazy_matches_eager(gpu_lib):
    """LAZY leaves the band states implicit after a stationary call; get_state, a setter and the
    next (general) call materialise them with the same result as EAGER."""
    L = paths()
    N = 512
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    e, o = make(2, N, fwd, back)
    z, _ = make(2, N, fwd, back, mode=L.HZ_FB_RESP_LAZY, oracle=False)
    rng = np.random.default_rng(8)
    for i, n in enumerate([4000, 60000, 20000, 30000]):
        x = rng.uniform(-1, 1, n)
        ye, yz, yo = e.process(x), z.process(x), o.process(x)
        assert rel_err(ye, yo) < TOL and rel_err(yz, yo) < TOL, i
    assert z.last_path() == L.HZ_FB_PATH_RESPONSE and e.last_path() == L.HZ_FB_PATH_RESPONSE
    assert z.response_info()[2]   # implicit
    x = rng.uniform(-1, 1, 25000)
    ye, yz, yo = e.process(x), z.process(x), o.process(x)
    assert rel_err(yz, yo) < TOL
    assert states_close(z.get_state(), e.get_state())
    assert not z.response_info()[2]
    # a setter after a stationary call: the next call restarts from the exact band states
    z.process(x[:20000]), e.process(x[:20000]), o.process(x[:20000])
    assert z.response_info()[2]
    for fb in (e, z, o):
        fb.boost(17, 2.5)
    x = rng.uniform(-1, 1, 9000)
    ye, yz, yo = e.process(x), z.process(x), o.process(x)
    assert z.last_path() != L.HZ_FB_PATH_RESPONSE
    assert rel_err(yz, yo) < TOL and rel_err(ye, yo) < TOL


@pytest.mark.parametrize("order,N,seed", [(1, 200, 1), (2, 300, 2), (3, 100, 3), (4, 77, 4)])
def test_orders_random_banks(gpu_lib, order, N, seed):
    """Random stable banks of every order, per-band pre-amps and signed gains."""
    from test_filterbank_lti_gpu import random_bank
    L = paths()
    fwd, back = random_bank(order, N, seed=500 + seed, radius=(0.5, 0.998))
    rng = np.random.default_rng(seed)
    g, o = make(order, N, fwd, back, boost=rng.uniform(0.2, 2.0, N), gains=rng.uniform(-1, 1, N))
    K = None
    got = []
    for i, n in enumerate([2000, 40000, 40000, 33333, 65536]):
        x = rng.uniform(-1, 1, n)
        yg, yo = g.process(x), o.process(x)
        assert rel_err(yg, yo) < TOL, (i, n, rel_err(yg, yo))
        got.append(g.last_path())
        K = g.response_info()[0]
    assert K > 0
    assert got[-1] == L.HZ_FB_PATH_RESPONSE, (got, K)


def test_bank_response_vs_lfilter(gpu_lib):
    """h = sum_n gin_n lfilter(pin_n F_n, [1, B_n], delta): an independent restatement of the
    reference recurrence (scipy), over the whole horizon."""
    sig = pytest.importorskip("scipy.signal")
    N = 64
    fwd, back = resonant_coefficients(N, 0.99, 0.5)
    rng = np.random.default_rng(12)
    pin, gin = rng.uniform(0.5, 1.5, N), rng.uniform(-1, 1, N)
    g, _ = make(2, N, fwd, back, boost=pin, gains=gin, oracle=False)
    K = 16384
    h = g.response(K)
    d = np.zeros(K)
    d[0] = 1.0
    ref = sum(gin[n] * sig.lfilter(pin[n] * fwd[n], np.concatenate([[1.0], back[n]]), d) for n in range(N))
    Kh = g.response_info()[0]
    assert 0 < Kh <= K
    assert np.max(np.abs(h - ref)) <= 1e-12 * np.max(np.abs(ref))


def test_no_horizon_stays_per_band(gpu_lib):
    """Poles this close to the unit circle need more than 2^18 samples to forget: no horizon,
    the per-band engines keep running and stay exact."""
    L = paths()
    N = 256
    fwd, back = resonant_coefficients(N, 0.99999, 0.5)
    g, o = make(2, N, fwd, back)
    rng = np.random.default_rng(2)
    for n in [3000, 70000, 70000, 70000, 70000]:
        x = rng.uniform(-1, 1, n)
        assert rel_err(g.process(x), o.process(x)) < TOL
        assert g.last_path() != L.HZ_FB_PATH_RESPONSE
    assert g.response_info()[0] == -1


def test_distortion_and_stationary_history(gpu_lib):
    """A distortion functor forces the general engine; the history keeps counting (the band
    states do not depend on the functor), so the first call without it is stationary."""
    L = paths()
    N = 256
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make(2, N, fwd, back)
    rng = np.random.default_rng(4)
    x = rng.uniform(-1, 1, 2000)
    assert rel_err(g.process(x), o.process(x)) < TOL
    for fb in (g, o):
        fb.distortion(3, 0.0)
    for n in [30000, 30000]:
        x = rng.uniform(-1, 1, n)
        assert rel_err(g.process(x), o.process(x)) < TOL
        assert g.last_path() == L.HZ_FB_PATH_GENERAL
    for fb in (g, o):
        fb.distortion(0, 0.0)
    x = rng.uniform(-1, 1, 20000)
    assert rel_err(g.process(x), o.process(x)) < TOL
    assert g.last_path() == L.HZ_FB_PATH_RESPONSE


def test_shards_sum(gpu_lib):
    """Each shard convolves with its own bands' response: the shard mixes sum to the full mix."""
    from huygens_amd import Filterbank
    L = paths()
    N = 300
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    _, o = make(2, N, fwd, back, oracle=True)
    shards = []
    for b0, cnt in [(0, 128), (128, 100), (228, 72)]:
        s = Filterbank(2, N, 0.001, 0.001, shard=(b0, cnt))
        s.tune_response(0, 1)
        for n in range(N):
            s.coefficients(n, fwd[n], back[n])
        s.boost(np.ones(N))
        s.open()
        shards.append(s)
    rng = np.random.default_rng(6)
    for n in [1500, 60000, 40000, 17000]:
        x = rng.uniform(-1, 1, n)
        ref = o.process(x)
        ys = sum(s.process(x) for s in shards)
        assert rel_err(ys, ref) < TOL
    assert all(s.last_path() == L.HZ_FB_PATH_RESPONSE for s in shards)


def test_c2_full_size_against_lti(gpu_lib):
    """BASELINE C2 at full size (4096 bands, 10 s calls): stationary vs per-band LTI engine on
    the same input, outputs and band states (a size-independent property; the oracle checks
    the LTI engine elsewhere)."""
    L = paths()
    N = 4096
    fwd, back = resonant_coefficients(N, 0.999, 1.0)
    g, _ = make(2, N, fwd, back, kp=0.1, kg=1.0, oracle=False, force=False)
    t, _ = make(2, N, fwd, back, kp=0.1, kg=1.0, mode=L.HZ_FB_RESP_OFF, oracle=False, force=False)
    for i in range(4):
        x = white_noise_f32(480000, seed=100 + i)
        yg, yt = g.process(x), t.process(x)
        assert rel_err(yg, yt) < 1e-7, (i, rel_err(yg, yt))   # Nyquist double pole: TOL_STIFF
    assert g.last_path() == L.HZ_FB_PATH_RESPONSE
    assert states_close(g.get_state(), t.get_state(), 1e-7)


def test_time_range_shards(gpu_lib):
    """Multi-GPU layout on one device: three band shards, each given the whole bank's response
    (sum of the shards' responses) and a time share; their outputs (zeros outside their share)
    sum to the restatement's mix, calls of any length; a setter clears the bank response and
    the shards fall back to full-length outputs of their own bands (still summing right)."""
    from huygens_amd import Filterbank
    from huygens_amd.shard import set_time_shards, time_share
    L = paths()
    N = 300
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    _, o = make(2, N, fwd, back, oracle=True)
    cuts = [(0, 128), (128, 100), (228, 72)]
    shards = []
    for b0, cnt in cuts:
        s = Filterbank(2, N, 0.001, 0.001, shard=(b0, cnt))
        s.tune_response(0, 1)
        for n in range(N):
            s.coefficients(n, fwd[n], back[n])
        s.boost(np.ones(N))
        s.open()
        shards.append(s)
    # the all-reduces by hand: the largest horizon, every shard's response over it, summed
    for s in shards:
        s.response(8192)
    K_all = max(s.response_info()[0] for s in shards)
    full = sum(s.response(K_all) for s in shards)
    for r, s in enumerate(shards):
        # (set_time_shards' second all-reduce is the failure flag: 0 on every rank here)
        assert set_time_shards(s, r, 3, lambda h, full=full: full, lambda k, K_all=K_all: K_all if k > 1 else k)
        assert s.response_info()[0] == K_all
    rng = np.random.default_rng(11)
    for n in [1500, 60000, 40000, 17000, 100003]:
        # the collective arming of shard.arm_when_ready, by hand: stationary on every shard or none
        ready = all(s.stationary_ready(n) for s in shards)
        for s in shards:
            s.arm_time_shard(ready)
        x = rng.uniform(-1, 1, n)
        ref = o.process(x)
        outs = [s.process(x) for s in shards]
        assert rel_err(sum(outs), ref) < TOL, n
        if shards[0].last_path() == L.HZ_FB_PATH_RESPONSE:
            act = [s.time_shard_info(n) for s in shards]
            assert all(a[0] for a in act)
            assert [(f, c) for _, f, c in act] == [time_share(r, 3, n) for r in range(3)]
            assert sum(a[2] for a in act) == n and act[0][1] == 0
            for (a, f, c), y in zip(act, outs):   # zeros outside the share
                assert not np.any(y[:f]) and not np.any(y[f + c:])
    assert all(s.last_path() == L.HZ_FB_PATH_RESPONSE for s in shards)
    for fb in shards + [o]:
        fb.mix(5, 0.25)
    for n in [3000, 70000, 30000]:
        x = rng.uniform(-1, 1, n)
        ref = o.process(x)
        assert rel_err(sum(s.process(x) for s in shards), ref) < TOL
    assert not shards[0].time_shard_info(1000)[0]


@pytest.mark.parametrize("lazy", [False, True])
def test_stream_and_per_sample_after_stationary(gpu_lib, lazy):
    """After stationary calls: a per-sample coefficient stream (hz_fb_process_tv reads the band
    states, then leaves new coefficients), per-sample operator()/tick() and long calls again --
    every path picks up the exact band states (LAZY: materialised on the way)."""
    L = paths()
    N = 256
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make(2, N, fwd, back, mode=L.HZ_FB_RESP_LAZY if lazy else L.HZ_FB_RESP_EAGER)
    rng = np.random.default_rng(21)
    for n in [2000, 50000, 30000]:
        x = rng.uniform(-1, 1, n)
        assert rel_err(g.process(x), o.process(x)) < TOL
    assert g.last_path() == L.HZ_FB_PATH_RESPONSE
    assert g.response_info()[2] == lazy
    if os.environ.get("HZ_TEST_STATE_FIRST"):   # (diagnostic) the band states before the stream call
        st_g, st_o = g.get_state(), o.get_state()
        assert np.max(np.abs(st_g - st_o)) <= 1e-8 * max(1.0, np.max(np.abs(st_o))), np.argmax(np.abs(st_g - st_o))
    # resonant retuning stream over 3000 samples (Subtractive ALLINONE), order 2
    x = rng.uniform(-1, 1, 3000)
    fr = np.tile(np.linspace(200.0, 4000.0, N), (3000, 1)) * (1.0 + 0.1 * np.sin(np.arange(3000) / 300.0))[:, None]
    assert rel_err(g.process_tv(x, 1, fr, 0.999), o.process_tv(x, 1, fr, 0.999)) < TOL
    assert not g.response_info()[2]
    # the stream left new coefficients: long calls run per-band, then stationary again
    for n in [40000, 60000, 20000]:
        x = rng.uniform(-1, 1, n)
        assert rel_err(g.process(x), o.process(x)) < TOL
    assert g.last_path() == L.HZ_FB_PATH_RESPONSE
    # per-sample operator() / tick() after a stationary call
    x = rng.uniform(-1, 1, 40)
    ref = o.process(x)
    got = []
    for v in x:
        got.append(g(v))
        g.tick()
    assert rel_err(np.array(got), ref) < TOL


@pytest.mark.parametrize("R,centre,order", [(0.999, 1.0, 2), (0.9985, 0.5, 2), (0.997, 0.5, 2), (0.999, 0.5, 4)])
def test_column_split_vs_three_kernel(gpu_lib, R, centre, order):
    """The long-call convolution's two structures (hz_fb_col.h column split, opt-in; the
    three-kernel path, the default) on the same calls: both against the
    restatement, ragged lengths, band states equal; horizons of 8 / 16 / 24 partitions take the
    column split."""
    from test_filterbank_lti_gpu import random_bank
    L = paths()
    N = 512
    if order == 2:
        fwd, back = resonant_coefficients(N, R, centre)
    else:
        fwd, back = random_bank(order, N, seed=77, radius=(0.5, R))
    g, o = make(order, N, fwd, back)
    g.tune_response_engine(True)
    t, _ = make(order, N, fwd, back, oracle=False)
    t.tune_response_engine(False)
    t.tune_modal(False)   # the same (matrix-core) band-state pass on both: this compares the convolutions
    rng = np.random.default_rng(21)
    col_calls = 0
    for i, n in enumerate([3000, 60000, 60000, 50001, 2048 * 30, 100000, 16384, 99999]):
        x = rng.uniform(-1, 1, n)
        yg, yt, yo = g.process(x), t.process(x), o.process(x)
        tol = 1e-7 if centre == 1.0 else TOL
        assert rel_err(yg, yo) < tol, (i, n, rel_err(yg, yo))
        assert rel_err(yt, yo) < tol, (i, n)
        assert g.last_path() == t.last_path()
        if g.last_path() == L.HZ_FB_PATH_RESPONSE:
            assert not t.response_engine()[1]
            col_calls += g.response_engine()[1]
            assert states_close(g.get_state(), t.get_state(), 1e-9)
    K = g.response_info()[0]
    if K // 2048 in (8, 16, 24):
        assert col_calls >= 3, (K, col_calls)
    print("horizon", K, "column-split calls", col_calls)


@pytest.mark.parametrize("fill", [True, False])
def test_time_range_shards_modal(gpu_lib, fill):
    """The N > 1 value path of bench.py on one device: band shards of a bank
    on one pole circle at grid angles (the C2 recipe with N = 512: m = 8 (i + 1), the last band the
    Nyquist double pole) time-split with the whole bank's response.  Their band states come from
    the MODAL pass (hz_fb_modal.h, now allowed under time shards: every rank holds the whole call's
    input), equal to the restatement's; fill=True: zeros outside each share, outputs summing to the
    mix; fill=False (hz_fb_set_time_shard_fill(h, 0)): each share written, the rest untouched, the
    shares assembled by range equal to the mix.  The shard without any band in a phase-2 bin range
    skips it (early exit): states still exact."""
    import torch
    from huygens_amd import Filterbank
    from huygens_amd.shard import set_time_shards
    L = paths()
    N, O = 512, 2
    fwd, back = resonant_coefficients(N, 0.999, 1.0)
    _, o = make(2, N, fwd, back, oracle=True)
    cuts = [(0, 200), (200, 256), (456, 56)]
    shards = []
    for b0, cnt in cuts:
        s = Filterbank(2, N, 0.001, 0.001, shard=(b0, cnt))
        s.tune_response(0, 1)
        for n in range(N):
            s.coefficients(n, fwd[n], back[n])
        s.boost(np.ones(N))
        s.open()
        shards.append(s)
    for s in shards:
        s.response(8192)
    K_all = max(s.response_info()[0] for s in shards)
    full = sum(s.response(K_all) for s in shards)
    for r, s in enumerate(shards):
        assert set_time_shards(s, r, 3, lambda h, full=full: full, lambda k, K_all=K_all: K_all if k > 1 else k)
        s.set_time_shard_fill(fill)
    rng = np.random.default_rng(12)
    modal_calls = 0
    for n in [60000, 60000, 70001, 52000, 100003]:
        ready = all(s.stationary_ready(n) for s in shards)
        for s in shards:
            s.arm_time_shard(ready)
        x = rng.uniform(-1, 1, n)
        ref = o.process(x)
        outs = []
        xd = torch.from_numpy(x).cuda()
        for s in shards:   # device buffers (process_device): the untouched samples are observable
            yd = torch.full((n,), 7.0, dtype=torch.float64, device="cuda")
            s.process_device(xd.data_ptr(), yd.data_ptr(), n)
            s.synchronize()
            outs.append(yd.cpu().numpy())
        if shards[0].last_path() == L.HZ_FB_PATH_RESPONSE:
            assert all(s.modal_info()[3] for s in shards), [s.modal_info() for s in shards]
            modal_calls += 1
            if fill:
                got = sum(outs)
            else:
                got = np.zeros(n)
                for s, y in zip(shards, outs):
                    _, f, c = s.time_shard_info(n)
                    assert np.all(y[:f] == 7.0) and np.all(y[f + c:] == 7.0)   # outside: untouched
                    got[f:f + c] = y[f:f + c]
        else:
            got = sum(outs)
        assert rel_err(got, ref) < TOL, n
        st = o.get_state()
        for (b0, cnt), s in zip(cuts, shards):
            gs = s.get_state()
            assert states_close(gs[O:O + cnt * O], st[O + b0 * O:O + (b0 + cnt) * O]), (n, b0)
    assert modal_calls >= 2
    assert shards[2].modal_info()[2] == 1 and shards[0].modal_info()[2] == 0   # the Nyquist band: shard 2
