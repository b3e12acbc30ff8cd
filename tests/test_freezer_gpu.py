"""GPU parity: the Freezer HIP engine vs the restatement (oracle/hz_oracle_frz.c).

Both draw libc rand() in the reference's order; each run is seeded with srand.  The dry
(Delay) path is bit-exact; frozen output agrees to 1e-9 of the peak (device FFT / atan2 /
cos rounding vs the long double DFT and libm)."""
import numpy as np
import pytest

from oracle_frz import OracleFreezer, libc_srand

pytestmark = pytest.mark.gpu
TOL = 1e-9


def peak_close(a, b):
    return np.max(np.abs(a - b), initial=0.0) <= TOL * max(np.max(np.abs(b), initial=0.0), 1e-300)


def run_both(N, laps, width, x, blocks, seed):
    """blocks: list of (length, events relative to the block)."""
    from huygens_amd import Freezer
    g, o = Freezer(N, laps, width), OracleFreezer(N, laps, width)
    ys_g, ys_o, pos = [], [], 0
    libc_srand(seed)
    for b, ev in blocks:
        ys_g.append(g.process(x[pos:pos + b], ev))
        pos += b
    pos = 0
    libc_srand(seed)
    for b, ev in blocks:
        ys_o.append(o.process(x[pos:pos + b], ev))
        pos += b
    return np.concatenate(ys_g), np.concatenate(ys_o)


@pytest.mark.parametrize("N,laps,width", [(64, 4, 1.0), (2048, 8, 1.0), (256, 3, 2.5), (16, 2, 1.0)])
def test_freeze_cycles_vs_oracle(gpu_lib, N, laps, width):
    rng = np.random.default_rng(N + laps)
    t = np.arange(40000)
    x = 0.3 * np.sin(2 * np.pi * 440 * t / 48000) + 0.05 * rng.standard_normal(t.size)
    blocks = [(5000, [(0, 0), (3000, 1)]), (7000, [(2500, 0), (2501, 1), (6000, 1)]), (1, [(0, 0)]),
              (12000, [(4000, 1), (9000, 0)]), (15999, [])]
    gy, oy = run_both(N, laps, width, x, blocks, seed=N)
    assert np.max(np.abs(oy)) > 0
    assert peak_close(gy, oy)
    assert np.array_equal(gy[:3000], oy[:3000])   # the dry path before any freeze: exact


def test_freeze_spanning_calls_and_launches(gpu_lib, monkeypatch):
    """A frozen period across calls and across a launch split (chunks of 2^18 samples here; the
    default 2^20 makes a 10 s call one launch)."""
    monkeypatch.setenv("HZ_FRZ_CHUNK", str(1 << 18))
    N, laps = 512, 4
    x = np.random.default_rng(1).standard_normal(300000 + 20000)
    blocks = [(20000, [(15000, 1)]), (300000, [(290000, 0)])]
    gy, oy = run_both(N, laps, 1.0, x, blocks, seed=7)
    assert peak_close(gy, oy)


def test_api_freeze_between_calls(gpu_lib):
    from huygens_amd import Freezer
    N, laps = 128, 4
    x = np.random.default_rng(2).standard_normal(6000)
    g, o = Freezer(N, laps), OracleFreezer(N, laps)
    libc_srand(5)
    a = g.process(x[:2000])
    g.freeze()
    b = g.process(x[2000:4000])
    g.unfreeze()
    c = g.process(x[4000:])
    libc_srand(5)
    oa = o.process(x[:2000])
    o.freeze()
    ob = o.process(x[2000:4000])
    o.unfreeze()
    oc = o.process(x[4000:])
    assert peak_close(np.r_[a, b, c], np.r_[oa, ob, oc])
    assert g.info()[2] is False


def test_device_pointers(gpu_lib):
    import torch
    from huygens_amd import Freezer
    N, laps = 256, 4
    x = np.random.default_rng(3).standard_normal(8000)
    g, o = Freezer(N, laps), OracleFreezer(N, laps)
    xt = torch.from_numpy(x).cuda()
    yt = torch.empty_like(xt)
    g.set_stream(torch.cuda.current_stream().cuda_stream)
    libc_srand(9)
    g.process_device(xt.data_ptr(), yt.data_ptr(), x.size, [(3000, 1)])
    torch.cuda.synchronize()
    libc_srand(9)
    oy = o.process(x, [(3000, 1)])
    assert peak_close(yt.cpu().numpy(), oy)


def test_errors(gpu_lib):
    from huygens_amd import Freezer, HZError
    with pytest.raises(HZError):
        Freezer(100, 4)   # N not a power of two
    g = Freezer(64, 4)
    with pytest.raises(HZError):
        g.process(np.zeros(10), [(11, 1)])
    with pytest.raises(HZError):
        g.process(np.zeros(10), [(5, 1), (2, 0)])
