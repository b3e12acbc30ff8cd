"""GPU parity: Filterbank with per-sample coefficient streams (hz_fb_process_tv, SURVEY.md
8(f) row 4) vs the restatement (orc_fb_process_tv).  Per-band arithmetic follows the
restatement's order without FMA; the mix order differs (and, for HZ_FB_TV_RESONANT, device
sincos / hypot vs libm), so outputs agree to rel_err <= TOL (norm-wise)."""
import numpy as np
import pytest

from oracle import OracleFilterbank, rel_err
from test_filterbank_tv_cpu import coeff_stream

pytestmark = pytest.mark.gpu
TOL = 1e-12
SR = 48000


def pair(O, N, seed, k_p=0.1, k_g=1.0):
    from huygens_amd import Filterbank
    rng = np.random.default_rng(seed)
    boost = rng.uniform(0.5, 1.5, N)
    g, o = Filterbank(O, N, k_p, k_g), OracleFilterbank(O, N, k_p, k_g)
    for fb in (g, o):
        fb.boost(list(boost))
        fb.open()
    return g, o


@pytest.mark.parametrize("O,N", [(0, 5), (1, 64), (2, 300), (3, 97), (4, 1000), (2, 1)])
def test_coefficient_stream(gpu_lib, O, N):
    g, o = pair(O, N, O + N)
    n = 3000
    st = coeff_stream(n, N, O, O)
    x = np.random.default_rng(N).standard_normal(n)
    for a, b in [(0, 1), (1, 1700), (1700, 1717), (1717, n)]:   # ragged calls incl. one sample
        assert rel_err(g.process_tv(x[a:b], 0, st[a:b]), o.process_tv(x[a:b], 0, st[a:b])) <= TOL


def subtractive_freqs(n, N, seed):
    """ALLINONE-style tracks: every band's frequency glides every sample."""
    rng = np.random.default_rng(seed)
    t = np.arange(n)[:, None]
    base = rng.uniform(60, 3000, N)[None, :]
    return base * (1 + 0.05 * np.sin(2 * np.pi * (t / 4800.0 + rng.uniform(0, 1, N)[None, :])))


@pytest.mark.parametrize("N", [96, 513])
def test_resonant_stream(gpu_lib, N):
    g, o = pair(2, N, 7)
    n = 4000
    fr = subtractive_freqs(n, N, N)
    x = np.random.default_rng(3).uniform(-1, 1, n)
    assert rel_err(g.process_tv(x[:2500], 1, fr[:2500], 0.9999), o.process_tv(x[:2500], 1, fr[:2500], 0.9999)) <= TOL
    assert rel_err(g.process_tv(x[2500:], 1, fr[2500:], 0.9999), o.process_tv(x[2500:], 1, fr[2500:], 0.9999)) <= TOL


def test_interleaved_with_plain_calls(gpu_lib):
    """process / process_tv / process share state; after a stream the last row stays staged."""
    O, N, n = 2, 200, 2000
    g, o = pair(O, N, 11)
    st = coeff_stream(n, N, O, 11)
    for fb in (g, o):
        for b in range(N):
            fb.coefficients(b, st[0, :3, b], st[0, 3:, b])
    x = np.random.default_rng(11).standard_normal(3 * n)
    assert rel_err(g.process(x[:n]), o.process(x[:n])) <= 1e-9
    assert rel_err(g.process_tv(x[n:2 * n], 0, st), o.process_tv(x[n:2 * n], 0, st)) <= TOL
    # the restatement keeps the last row as its coefficients, like the reference
    assert rel_err(g.process(x[2 * n:]), o.process(x[2 * n:])) <= 1e-9


def test_smoothers_and_distortion(gpu_lib):
    """boost / mix targets change between calls (smoothers move during the stream); softclip."""
    from huygens_amd._lib import HZ_DIST_SOFTCLIP
    O, N, n = 2, 150, 3000
    g, o = pair(O, N, 13, k_p=0.01, k_g=0.02)
    st = coeff_stream(n, N, O, 13)
    x = 3 * np.random.default_rng(13).standard_normal(n)
    for fb in (g, o):
        fb.distortion(HZ_DIST_SOFTCLIP, 0.4)
    assert rel_err(g.process_tv(x[:1000], 0, st[:1000]), o.process_tv(x[:1000], 0, st[:1000])) <= TOL
    rng = np.random.default_rng(14)
    b, m = rng.uniform(0, 2, N), rng.uniform(0, 1, N)
    for fb in (g, o):
        fb.boost(list(b))
        fb.mix(list(m))
    assert rel_err(g.process_tv(x[1000:], 0, st[1000:]), o.process_tv(x[1000:], 0, st[1000:])) <= TOL


@pytest.mark.parametrize("dist", ["HZ_DIST_SOFTCLIP", "HZ_DIST_SATURATE", "HZ_DIST_LIMITER"])
def test_resonant_stream_distortion(gpu_lib, dist):
    """Resonant streams through the producer/consumer kernel with each per-band distortion
    functor, ragged calls (tile remainders, a 1-sample call) and a bank of 130 bands (partial
    last workgroup)."""
    from huygens_amd import _lib
    N = 130
    g, o = pair(2, N, 29, k_p=0.02, k_g=0.03)
    for fb in (g, o):
        fb.distortion(getattr(_lib, dist), 0.3)
    n = 2000
    fr = subtractive_freqs(n, N, 29)
    x = 4 * np.random.default_rng(29).uniform(-1, 1, n)
    for a, b in [(0, 31), (31, 32), (32, 1500), (1500, n)]:
        assert rel_err(g.process_tv(x[a:b], 1, fr[a:b], 0.999), o.process_tv(x[a:b], 1, fr[a:b], 0.999)) <= TOL


def test_device_pointers(gpu_lib):
    import torch
    O, N, n = 2, 128, 2048
    g, o = pair(O, N, 17)
    fr = subtractive_freqs(n, N, 17)
    x = np.random.default_rng(17).standard_normal(n)
    xt, ft = torch.from_numpy(x).cuda(), torch.from_numpy(np.ascontiguousarray(fr)).cuda()
    yt = torch.empty_like(xt)
    g.set_stream(torch.cuda.current_stream().cuda_stream)
    g.process_tv_device(xt.data_ptr(), yt.data_ptr(), n, 1, ft.data_ptr(), 0.999)
    torch.cuda.synchronize()
    assert rel_err(yt.cpu().numpy(), o.process_tv(x, 1, fr, 0.999)) <= TOL


def test_errors(gpu_lib):
    from huygens_amd import Filterbank, HZError
    g = Filterbank(3, 4)
    with pytest.raises(HZError):
        g.process_tv(np.zeros(4), 1, np.zeros((4, 4)), 0.9)   # resonant needs order 2
    with pytest.raises(HZError):
        g.process_tv(np.zeros(4), 5, np.zeros((4, 28)))
    assert g.process_tv(np.zeros(0), 0, np.zeros(1)).size == 0
