"""GPU parity: Fourier / StaticSTFT / Cosine HIP engines vs the restatement.

Tolerance: 1e-10 of the output's peak (the north star allows 1e-5); the FFTs round
differently from the oracle's long double DFT (~1e-15) and the overlap-add replaces
long double with double-double.  Gate decisions must agree: every gated input here has
its closest bin >= 1e-6 (relative) from the threshold (the fixtures record `margin`)."""
import numpy as np
import pytest
import scipy.fft

from oracle import golden_names, load_golden
from oracle_stft import OracleSTFT

pytestmark = pytest.mark.gpu
TOL = 1e-10


def peak_err(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


def c4_signal(n, seed=3):
    """C4: white noise (sigma 0.1) + 8 sinusoids (amp 0.5, f = 220 k^1.5 Hz)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 48000.0
    x = 0.1 * rng.standard_normal(n)
    for k in range(1, 9):
        x += 0.5 * np.sin(2 * np.pi * 220 * k ** 1.5 * t)
    return x


def make(N, laps, window, proc, callback=None):
    from huygens_amd import Fourier
    g = Fourier(callback if callback is not None else proc, N, laps, window)
    o = OracleSTFT(N, laps, window, proc, callback=None)
    return g, o


@pytest.mark.parametrize("name", golden_names("stft_"))
def test_golden(gpu_lib, name):
    from huygens_amd import Fourier
    g = load_golden(name)
    f = Fourier(int(g["proc"]), int(g["N"]), int(g["laps"]), int(g["window"]))
    yr, yi = f.process_block(g["x_re"], g["x_im"])
    scale = max(np.max(np.abs(g["y_re"])), np.max(np.abs(g["y_im"])))
    assert np.max(np.abs(yr - g["y_re"])) <= TOL * scale
    assert np.max(np.abs(yi - g["y_im"])) <= TOL * scale
    assert f.frames()[0] == len(g["starts"])


@pytest.mark.parametrize("N,laps", [(4, 1), (8, 2), (16, 16), (64, 4), (256, 8), (1024, 4), (2048, 32)])
@pytest.mark.parametrize("window", [0, 1])
def test_identity_vs_oracle_blocks(gpu_lib, N, laps, window):
    """Irregular block sizes carry the slot schedule and history across calls."""
    g, o = make(N, laps, window, 0)
    rng = np.random.default_rng(N + laps)
    for n in (1, 3 * N + 5, 1000, 2 * N - 1, 7):
        re, im = rng.standard_normal(n), rng.standard_normal(n)
        gr, gi = g.process_block(re, im)
        orr, oi = o.process_block(re, im)
        assert peak_err(gr, orr) < TOL and peak_err(gi, oi) < TOL
    assert g.frames()[0] == o.frames()


@pytest.mark.parametrize("N,laps", [(64, 4), (4096, 4)])
def test_real_then_complex_calls(gpu_lib, N, laps):
    """Real-only calls skip the Im history plane; a complex call must switch it back on for
    every frame that reads one of its samples, including frames straddling later real calls."""
    g, o = make(N, laps, 0, 0)
    rng = np.random.default_rng(7)
    for n, cplx in ((3 * N + 1, False), (N // 2 + 3, True), (5, False), (4 * N, False), (N + 9, True), (3 * N, False)):
        re = rng.standard_normal(n)
        im = rng.standard_normal(n) if cplx else None
        gr, gi = g.process_block(re, im)
        orr, oi = o.process_block(re, im)
        scale = max(np.max(np.abs(orr)), np.max(np.abs(oi)), 1e-300)   # Im of a real call is ~0: use one scale
        assert np.max(np.abs(gr - orr)) < TOL * scale and np.max(np.abs(gi - oi)) < TOL * scale
    assert g.frames()[0] == o.frames()


@pytest.mark.parametrize("N,laps,proc", [(64, 4, 2), (4096, 4, 2), (512, 4, 1)])
def test_gate_real_then_complex_calls(gpu_lib, N, laps, proc):
    """Gated frames of real calls run two per transform (stft_pair_kernel), whose frames leave the
    ring's Im plane unwritten (the overlap-add takes their Im part as 0); complex calls in
    between run one frame per transform and write it -- the Im output must match the
    restatement across every switch, including switches closer together than 2 laps frames."""
    g, o = make(N, laps, 0, proc)
    rng = np.random.default_rng(11)
    T = 0
    seq = ((3 * N + 1, False), (N // 2 + 3, True), (5, False), (4 * N, False), (N + 9, True), (3 * N, False),
           (2 * N + 7, True), (N // 4, False), (3, True), (5 * N, False))
    for n, cplx in seq:
        t = np.arange(T, T + n)
        z = 0.5 * np.exp(2j * np.pi * 3 * t / N) + 0.05 * rng.standard_normal(n)
        re = z.real.copy()
        im = z.imag.copy() if cplx else None
        T += n
        gr, gi = g.process_block(re, im)
        orr, oi = o.process_block(re, im)
        scale = max(np.max(np.abs(orr)), np.max(np.abs(oi)), 1e-300)
        assert np.max(np.abs(gr - orr)) < TOL * scale and np.max(np.abs(gi - oi)) < TOL * scale
    assert g.frames()[0] == o.frames()


@pytest.mark.parametrize("N,laps", [(4096, 4), (8192, 4), (512, 4), (8192, 32)])
def test_static_stft_c4(gpu_lib, N, laps):
    from huygens_amd import StaticSTFT
    g = StaticSTFT(N, laps)
    o = OracleSTFT(N, laps, 1, 1)
    x = c4_signal(6 * N)
    parts = [g.process_block(x[:N + 17])[0], g.process_block(x[N + 17:])[0]]
    ref = o.process_block(x)[0]
    assert peak_err(np.concatenate(parts), ref) < TOL


@pytest.mark.parametrize("proc", [2, 3])
def test_fourier_gates_c4(gpu_lib, proc):
    """spectral.cpp 625 gate (complex tone so bins pass) and the Hilbert half-band."""
    N, laps = 4096, 4
    g, o = make(N, laps, 0, proc)
    n = 5 * N
    t = np.arange(n)
    re = c4_signal(n)
    im = np.zeros(n)
    if proc == 2:
        z = 0.5 * np.exp(2j * np.pi * 100 * t / N) + 1e-3 * np.random.default_rng(1).standard_normal(n)
        re, im = z.real.copy(), z.imag.copy()
    gr, gi = g.process_block(re, im)
    orr, oi = o.process_block(re, im)
    assert np.max(np.abs(orr)) > 0.1
    assert peak_err(gr, orr) < TOL and peak_err(gi, oi) < TOL


@pytest.mark.parametrize("N,laps", [(4096, 4), (8192, 32), (256, 4)])
def test_gate_keep_real_pairs(gpu_lib, N, laps):
    """spectral.cpp 625 gate on real input: two frames share one transform
    (stft_pair_kernel, radix 8 and radix 16); ragged calls, odd frame counts per launch."""
    g, o = make(N, laps, 0, 2)
    n = 7 * N + 5
    x = c4_signal(n)
    if N < 1024:   # a short frame needs one dominant bin to clear 25x the average magnitude
        x = np.sin(2 * np.pi * 8 * np.arange(n) / N) + 0.01 * np.random.default_rng(5).standard_normal(n)
    cut = [0, N // 3, 3 * N + 1, n]
    parts = [g.process_block(x[a:b])[0] for a, b in zip(cut[:-1], cut[1:])]
    ref = o.process_block(x)[0]
    assert np.max(np.abs(ref)) > 0.05
    assert peak_err(np.concatenate(parts), ref) < TOL


def test_host_callback_stateful(gpu_lib):
    """A host processor runs per frame in frame order with each slot's `out` persisting
    (fourier.h:57-59): this one accumulates into out instead of overwriting it."""
    from huygens_amd import Fourier
    N, laps = 32, 4
    calls = {"g": 0}

    def acc_gpu(inp, out):
        out *= 0.5
        out += inp
        calls["g"] += 1
        return 0

    def acc_ref(inp, out):
        for i in range(2 * N):
            out[i] = 0.5 * out[i] + inp[i]
        return 0

    g = Fourier(acc_gpu, N, laps)
    o = OracleSTFT(N, laps, 0, 4, callback=acc_ref)
    rng = np.random.default_rng(2)
    for n in (50, 200, 333):
        x = rng.standard_normal(n)
        assert peak_err(g.process_block(x)[0], o.process_block(x)[0]) < TOL
    assert calls["g"] == o.frames()


def test_device_pointers(gpu_lib):
    import torch
    from huygens_amd import Fourier
    N, laps = 1024, 4
    g = Fourier(0, N, laps)
    o = OracleSTFT(N, laps, 0, 0)
    x = np.random.default_rng(4).standard_normal(5 * N)
    xt = torch.from_numpy(x).cuda()
    yr = torch.empty_like(xt)
    g.process_block_device(xt.data_ptr(), 0, yr.data_ptr(), 0, x.size)
    g.synchronize()
    assert peak_err(yr.cpu().numpy(), o.process_block(x)[0]) < TOL


@pytest.mark.parametrize("N", [4, 64, 1024, 8192])
def test_cosine(gpu_lib, N):
    from huygens_amd import Cosine
    c = Cosine(N)
    x = np.random.default_rng(N).standard_normal(N)
    c.inp[:] = x
    c.forward()
    assert peak_err(c.out, scipy.fft.dct(x, type=2)) < 1e-13
    c.backward()
    assert peak_err(c.inp, 2 * N * x) < 1e-13


def test_cosine_golden_and_batch(gpu_lib):
    import torch
    from huygens_amd import Cosine
    g = load_golden("dct_n64")
    c = Cosine(64)
    c.inp[:] = g["x"]
    c.forward()
    assert peak_err(c.out, g["redft10"]) < 1e-13
    xs = torch.from_numpy(np.random.default_rng(0).standard_normal((7, 64))).cuda()
    ys = torch.empty_like(xs)
    c.forward_device(xs.data_ptr(), ys.data_ptr(), 7)
    assert peak_err(ys.cpu().numpy(), scipy.fft.dct(xs.cpu().numpy(), type=2, axis=1)) < 1e-13


def test_errors(gpu_lib):
    from huygens_amd import Cosine, Fourier, HZError
    with pytest.raises(HZError):
        Fourier(0, 100, 4)
    with pytest.raises(HZError):
        Fourier(0, 16384, 4)
    with pytest.raises(HZError):
        Cosine(12)


@pytest.mark.parametrize("world,block,kind", [(2, 5, "static"), (3, 16, "static"), (3, 1000, "static"),
                                              (2, 3, "hilbert"), (4, 7, "gate")])
def test_time_range_shards_sum(gpu_lib, world, block, kind):
    """SURVEY.md 8(e) STFT row: frames by time range.  Runs of `block` frames rotate over
    `world` handles (hz_stft_set_frame_shard); their outputs sum to the unsharded engine's
    output across ragged calls -- a frame's overlap-add tail that lands in a later call stays
    with the rank that computed it.  static: two frames per transform (real input); hilbert:
    one frame per transform over complex input; gate: Fourier(gate625), real input."""
    from huygens_amd.stft import PROC_GATE_KEEP, PROC_HILBERT, Fourier, StaticSTFT
    N, laps = 1024, 4
    rng = np.random.default_rng(50 + world)
    x = rng.standard_normal(30000) * 0.1 + np.sin(np.arange(30000) * 0.05)
    xi = rng.standard_normal(30000) * 0.1 if kind == "hilbert" else None
    make = {"static": lambda: StaticSTFT(N, laps), "hilbert": lambda: Fourier(PROC_HILBERT, N, laps),
            "gate": lambda: Fourier(PROC_GATE_KEEP, N, laps)}[kind]
    full = make()
    shards = [make() for _ in range(world)]
    for r, sh in enumerate(shards):
        sh.set_frame_shard(r, world, block)
    t = 0
    for n in (5000, 333, 1, 12000, 12666):
        sl = slice(t, t + n)
        ref = full.process_block(x[sl], None if xi is None else xi[sl])
        got = [np.zeros(n), np.zeros(n)]
        for sh in shards:
            o = sh.process_block(x[sl], None if xi is None else xi[sl])
            got[0] += o[0]
            got[1] += o[1]
        for g, rf in zip(got, ref):
            assert np.max(np.abs(g - rf)) <= 1e-12 * max(1.0, np.max(np.abs(rf))), n
        t += n
    assert all(sh.frames() == full.frames() for sh in shards)


def test_frame_shard_args(gpu_lib):
    from huygens_amd._lib import HZ_E_INVALID, HZ_E_UNSUPPORTED, HZError
    from huygens_amd.stft import Fourier, StaticSTFT
    f = Fourier(lambda a, b: b.__setitem__(slice(None), a), 64, 4)
    with pytest.raises(HZError) as ei:
        f.set_frame_shard(0, 2, 10)
    assert ei.value.code == HZ_E_UNSUPPORTED
    f.set_frame_shard(0, 1, 10)   # one rank: every frame, allowed
    s = StaticSTFT(64, 4)
    for bad in ((2, 2, 1), (-1, 2, 1), (0, 0, 1), (0, 2, 0)):
        with pytest.raises(HZError) as ei:
            s.set_frame_shard(*bad)
        assert ei.value.code == HZ_E_INVALID
