"""GPU parity of the converged ("LTI") Filterbank engine (huygens_amd/csrc/hz_fb_lti.h).

Once every pre-amp and gain smoother of src/filterbank.h:172-173 has reached its
target, process() runs the LTI engine: per-chunk zero-state end states + the carry
scan + the homogeneous correction per band, and ONE bank-wide zero-state matrix
(Fmix) applied in the reduce kernel.  Every test drives the GPU object and the CPU
restatement (oracle/hz_oracle.c) through the same calls and compares the mixes
norm-wise (north-star bound 1e-5; asserted at the FP64 bounds of test_filterbank_gpu).
Small smoothing constants (k_p, k_g) make the smoothers converge within the first
call, so the later calls take the LTI engine; last_path() proves which one ran.
"""
import numpy as np
import pytest

from golden.spec_numpy import resonant_coefficients, white_noise_f32
from oracle import OracleFilterbank, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-9
TOL_STIFF = 1e-7  # Nyquist double pole (see test_filterbank_gpu.py)
LTI_GEOMS = [(16, 1, 16), (32, 1, 16), (64, 1, 16), (128, 1, 16)]


def make_pair(order, N, fwd, back, kp=0.001, kg=0.001, boost=None, gains=None):
    from huygens_amd import Filterbank
    from huygens_amd._lib import HZ_FB_RESP_OFF
    g = Filterbank(order, N, kp, kg)
    g.set_response(HZ_FB_RESP_OFF)   # the per-band LTI engine under test (test_filterbank_resp_gpu.py: the other)
    o = OracleFilterbank(order, N, kp, kg)
    for fb in (g, o):
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
        fb.boost(np.ones(N) if boost is None else boost)
        if gains is None:
            fb.open()
        else:
            fb.mix(gains)
    return g, o


def random_bank(order, N, seed, radius=(0.5, 0.995)):
    rng = np.random.default_rng(seed)
    fwd = rng.uniform(-1, 1, (N, order + 1))
    back = np.zeros((N, order))
    for n in range(N):
        roots = []
        for _ in range(order // 2):
            p = rng.uniform(*radius) * np.exp(1j * rng.uniform(0, np.pi))
            roots += [p, np.conj(p)]
        if order % 2:
            roots.append(rng.uniform(*radius) * rng.choice([-1, 1]))
        back[n] = np.real(np.poly(roots))[1:]
    return fwd, back


def run_calls(g, o, lengths, seed, expect_lti=True, tol=TOL):
    rng = np.random.default_rng(seed)
    from huygens_amd._lib import HZ_FB_PATH_GENERAL, HZ_FB_PATH_LTI
    for i, n in enumerate(lengths):
        x = rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64)
        yg, yo = g.process(x), o.process(x)
        err = rel_err(yg, yo)
        assert err < tol, (i, n, err)
        if i > 0 and expect_lti and n >= g.lti_chunk():
            assert g.last_path() == HZ_FB_PATH_LTI, (i, n)
        if i == 0:
            # the first call starts from pre = gain = 0: general engine
            assert g.last_path() == HZ_FB_PATH_GENERAL


@pytest.mark.parametrize("geom", LTI_GEOMS)
@pytest.mark.parametrize("R,centre", [(0.999, 0.5), (0.9999, 0.5), (0.999, 1.0)])
def test_c2_recipe_lti(gpu_lib, geom, R, centre):
    """C2 shape: 4096 resonant band-passes; calls of whole tiles, ragged tiles, a
    length that is not a multiple of the chunk (LTI + general tail) and one block."""
    N = 4096
    fwd, back = resonant_coefficients(N, R, centre)
    g, o = make_pair(2, N, fwd, back)
    g.tune_lti(*geom)
    run_calls(g, o, [700, 4096, 3 * 1024 + 512, 5003, 1024], seed=11,
              tol=TOL_STIFF if centre == 1.0 else TOL)


@pytest.mark.parametrize("N,order,groups", [(4096, 2, 256), (203, 2, 256), (300, 1, 16), (100, 3, 8), (77, 4, 64)])
def test_chunk128_long_calls(gpu_lib, N, order, groups):
    """Chunk 128 (8192-sample tiles, one x buffer, E operands in LDS, GEMM over 128-sample
    chunks, quarter-Fmix reduce): multi-tile and ragged calls, with time segments and the
    prepass for the small banks."""
    if order == 2:
        fwd, back = resonant_coefficients(N, 0.999, 0.5)
        g, o = make_pair(2, N, fwd, back)
    else:
        fwd, back = random_bank(order, N, seed=300 + order)
        rng = np.random.default_rng(order)
        g, o = make_pair(order, N, fwd, back, boost=rng.uniform(0.2, 2.0, N), gains=rng.uniform(-1, 1, N))
    g.tune_lti(128, 1, 16)
    g.set_target_groups(groups)
    run_calls(g, o, [700, 8192 * 3 + 128 * 5, 40000, 1024, 65536 + 300], seed=40 + order)
    assert g.lti_chunk() == 128


@pytest.mark.parametrize("shift", [1, 3])
def test_chunk128_device_pointers_unaligned(gpu_lib, shift):
    """hz_fb_process_device on x / out pointers that are only 8-byte aligned (a tensor view
    starting `shift` doubles in): the chunk-128 LDS-DMA loads 16 B per lane from x + c L + 2 l,
    which then straddles 16-byte boundaries; results must not change."""
    torch = pytest.importorskip("torch")
    N = 1024
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make_pair(2, N, fwd, back, kp=0.0, kg=0.0)
    g.tune_lti(128, 1, 16)
    rng = np.random.default_rng(70 + shift)
    for i, n in enumerate([1024, 8192 * 4 + 77, 50000]):
        x = rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64)
        buf = torch.zeros(n + 2 * shift, dtype=torch.float64, device="cuda")
        buf[shift:shift + n] = torch.from_numpy(x).cuda()
        out = torch.full((n + 2 * shift,), 7.0, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        g.process_device(buf[shift:].data_ptr(), out[shift:].data_ptr(), n)
        g.synchronize()
        yo = o.process(x)
        yg = out.cpu().numpy()
        assert rel_err(yg[shift:shift + n], yo) < TOL, (i, n)
        assert np.all(yg[:shift] == 7.0) and np.all(yg[shift + n:] == 7.0)
        if i > 0:
            assert g.lti_chunk() == 128
    from huygens_amd._lib import HZ_FB_PATH_LTI
    assert g.last_path() == HZ_FB_PATH_LTI


def test_chunk128_picked_for_c2(gpu_lib):
    """By call length: chunk 128 for long calls of banks with at most two time segments, chunk
    64 for smaller shards, chunk 16 for streaming blocks."""
    from huygens_amd import Filterbank
    for N, n, want in ((4096, 480_000, 128), (2048, 240_000, 128), (512, 480_000, 64), (4096, 1024, 16)):
        fwd, back = resonant_coefficients(N, 0.999, 0.5)
        g, _ = make_pair(2, N, fwd, back, kp=0.0, kg=0.0)
        g.process(white_noise_f32(1024, seed=1))
        g.process(white_noise_f32(n, seed=2))
        assert g.lti_chunk() == want, (N, n, g.lti_chunk())


@pytest.mark.parametrize("order", [1, 2, 3, 4])
@pytest.mark.parametrize("geom", LTI_GEOMS)
def test_orders_lti(gpu_lib, order, geom):
    N = 203
    fwd, back = random_bank(order, N, seed=200 + order)
    rng = np.random.default_rng(order)
    g, o = make_pair(order, N, fwd, back, boost=rng.uniform(0.2, 2.0, N), gains=rng.uniform(-1, 1, N))
    g.tune_lti(*geom)
    run_calls(g, o, [300, 2048, 4000, 33, 16], seed=order)


@pytest.mark.parametrize("N,groups", [(64, 1024), (512, 256), (5, 4096)])
def test_time_segments_lti(gpu_lib, N, groups):
    """Small banks split the call into time segments (segment end states, per-band
    carry, segmented mix) in the LTI engine too."""
    fwd, back = resonant_coefficients(N, 0.9995, 0.5)
    g, o = make_pair(2, N, fwd, back)
    g.set_target_groups(groups)
    run_calls(g, o, [500, 30000, 12345, 2048 * 5], seed=21)


@pytest.mark.parametrize("N,groups,calls", [(128, 16, [500, 40960, 5000]), (64, 16, [500, 98304, 700])])
def test_fine_prepass_segments_lti(gpu_lib, N, groups, calls):
    """Shard-sized banks: the segment prepass splits each segment in m fine parts (m = 2
    here) and the mix starts from every m-th carried state (hz_fb_lti.hip, fb_launch_lti)."""
    fwd, back = resonant_coefficients(N, 0.9995, 0.5)
    g, o = make_pair(2, N, fwd, back)
    g.set_target_groups(groups)
    run_calls(g, o, calls, seed=22)


@pytest.mark.parametrize("R", [0.99, 0.995])
def test_horizon_prepass_lti(gpu_lib, R):
    """Fast-decaying banks: every band forgets its state within a horizon K shorter than a
    segment (||M^K|| < 2^-64), so the segment prepass covers only each segment's last
    ceil(K / T) + 1 tiles (hz_fb_lti.hip, fb_lti_horizon)."""
    N = 64
    fwd, back = resonant_coefficients(N, R, 0.5)
    g, o = make_pair(2, N, fwd, back)
    g.set_target_groups(16)
    run_calls(g, o, [500, 98304, 2048 * 40 + 96, 3000], seed=23)
    g.process(white_noise_f32(98304, seed=24))
    nseg, skip, _ = g.lti_plan()
    assert nseg > 1 and skip > 0, (nseg, skip)


@pytest.mark.parametrize("N,n", [(2048, 240_000), (512, 480_000)])
def test_horizon_prepass_shard_shapes(gpu_lib, N, n):
    """The emulated 2-GPU (2048 bands, 2 segments) and 8-GPU (512 bands, 8 segments) shard
    shapes of C2 at R = 0.999 on 256 CUs: K = 53,248 samples (26 tiles) is shorter than a
    segment, so the prepass starts skip_tiles > 0 tiles into each segment; parity vs the
    restatement over the whole call."""
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make_pair(2, N, fwd, back)
    g.set_target_groups(256)
    x0 = white_noise_f32(500, seed=30)
    assert rel_err(g.process(x0), o.process(x0)) < TOL
    x = white_noise_f32(n, seed=31)
    err = rel_err(g.process(x), o.process(x))
    nseg, skip, fine = g.lti_plan()
    assert nseg == 4096 // N and skip > 0 and fine == 1, (nseg, skip, fine)
    assert err < TOL, err


def test_path_switches_with_setters(gpu_lib):
    """A setter change un-converges the smoothers: the next call runs the general
    engine, later calls return to LTI; the mixes stay on the oracle throughout."""
    from huygens_amd._lib import HZ_FB_PATH_GENERAL, HZ_FB_PATH_LTI
    N = 300
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make_pair(2, N, fwd, back, kp=0.002, kg=0.004)
    rng = np.random.default_rng(3)
    paths = []
    for step in range(8):
        x = rng.uniform(-1, 1, 1024)
        assert rel_err(g.process(x), o.process(x)) < TOL, step
        paths.append(g.last_path())
        if step == 3:
            for fb in (g, o):
                fb.boost(7, 3.0)
                fb.mix(11, -0.5)
                fb.coefficients(40, [0.3, 0.0, -0.3], [-1.9 * np.cos(0.2), 0.97])
    assert paths[0] == HZ_FB_PATH_GENERAL
    assert paths[2] == HZ_FB_PATH_LTI
    assert paths[4] == HZ_FB_PATH_GENERAL
    assert paths[7] == HZ_FB_PATH_LTI


def test_forced_general_matches_lti(gpu_lib):
    from huygens_amd._lib import HZ_FB_PATH_GENERAL, HZ_FB_PATH_LTI
    N = 1000
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    a, _ = make_pair(2, N, fwd, back)
    b, _ = make_pair(2, N, fwd, back)
    b.set_path(HZ_FB_PATH_GENERAL)
    x = white_noise_f32(20000, seed=5)
    a.process(x[:1000])
    b.process(x[:1000])
    ya, yb = a.process(x[1000:]), b.process(x[1000:])
    assert a.last_path() == HZ_FB_PATH_LTI and b.last_path() == HZ_FB_PATH_GENERAL
    assert rel_err(ya, yb) < TOL
    # the carried state agrees as well
    sa, sb = a.get_state(), b.get_state()
    assert np.max(np.abs(sa - sb)) <= 1e-9 * max(1.0, np.max(np.abs(sb)))


def test_distortion_keeps_general(gpu_lib):
    from huygens_amd._lib import HZ_FB_PATH_GENERAL
    N = 40
    fwd, back = resonant_coefficients(N, 0.99, 0.5)
    g, o = make_pair(2, N, fwd, back)
    for fb in (g, o):
        fb.distortion(1, 0.125)
    run_calls(g, o, [300, 2048], seed=2, expect_lti=False)
    assert g.last_path() == HZ_FB_PATH_GENERAL


def test_shards_lti(gpu_lib):
    """Each shard's Fmix covers its own bands: the shard mixes sum to the full mix."""
    from huygens_amd import Filterbank
    N = 300
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    _, o = make_pair(2, N, fwd, back)
    shards = []
    for b0, cnt in [(0, 128), (128, 100), (228, 72)]:
        s = Filterbank(2, N, 0.001, 0.001, shard=(b0, cnt))
        for n in range(N):
            s.coefficients(n, fwd[n], back[n])
        s.boost(np.ones(N))
        s.open()
        shards.append(s)
    x = white_noise_f32(9000, seed=7)
    ref = np.concatenate([o.process(x[:500]), o.process(x[500:])])
    ys = np.concatenate([sum(s.process(x[:500]) for s in shards), sum(s.process(x[500:]) for s in shards)])
    assert rel_err(ys, ref) < TOL


def test_per_sample_after_lti(gpu_lib):
    """operator()/tick() (n = 1 < chunk) after LTI calls continues the exact history."""
    N = 64
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make_pair(2, N, fwd, back)
    x = white_noise_f32(3000, seed=9)
    ref = o.process(x)
    parts = [g.process(x[:600]), g.process(x[600:2048])]
    for i in range(2048, 2080):
        parts.append(np.array([g(x[i])]))
        g.tick()
    parts.append(g.process(x[2080:]))
    assert rel_err(np.concatenate(parts), ref) < TOL
