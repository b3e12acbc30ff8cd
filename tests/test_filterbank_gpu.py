"""GPU parity: Filterbank<double> HIP engine vs the CPU restatement (oracle) and the
golden fixtures, through the C ABI.  North-star bound: ||Δ||∞/||ref||∞ ≤ 1e-5;
these tests assert a tighter FP64 bound (TOL) to catch real bugs early."""
import numpy as np
import pytest

from golden.spec_numpy import resonant_coefficients, white_noise_f32
from oracle import OracleFilterbank, golden_names, load_golden, rel_err, run_schedule

pytestmark = pytest.mark.gpu

NORTH_STAR_TOL = 1e-5   # BASELINE.json north_star: 1e-5 relative (norm-wise)
TOL = 1e-9              # FP64 reassociation of the chunked scan stays far below it
# The reference coefficient recipe puts its last band on Nyquist (f = SR/2): a double
# pole at -R with gain 1/|H| ~ 2e6 that dominates the mix.  That recurrence is
# ill-conditioned (sum |h| ~ 1/(1-R)^2), so the sequential CPU order and the chunked
# GPU order legitimately differ by ~1e-8 relative.  Still 1000x inside the bound.
TOL_STIFF = 1e-7
STIFF = {"fb_o2_n16_r0999"}


def make_pair(order, N, fwd, back, kp=0.1, kg=1.0, boost=True, opened=True, shard=None):
    from huygens_amd import Filterbank
    g = Filterbank(order, N, kp, kg, shard=shard)
    o = OracleFilterbank(order, N, kp, kg)
    for fb in (g, o):
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
        if boost:
            fb.boost(np.ones(N))
        if opened:
            fb.open()
    return g, o


@pytest.mark.parametrize("name", golden_names("fb_"))
def test_golden(gpu_lib, name):
    from huygens_amd import Filterbank
    g = load_golden(name)
    fb = Filterbank(int(g["order"]), int(g["N"]), float(g["kp"]), float(g["kg"]))
    fb.distortion(int(g["dist"]), float(g["dist_param"]))
    y = run_schedule(fb, g["x"], g["sched_t"], g["sched_kind"], g["sched_band"], g["sched_val"],
                     g["fwd"], g["back"])
    err = rel_err(y, g["y"])
    assert err < (TOL_STIFF if name in STIFF else TOL), err


@pytest.mark.parametrize("R,centre", [(0.999, 1.0), (0.999, 0.5), (0.9999, 0.5)])
def test_c2_recipe_4096_bands(gpu_lib, R, centre):
    """C2 workload shape (4096 bands, resonant band-pass) on a ragged 3 1/2-tile signal."""
    N = 4096
    fwd, back = resonant_coefficients(N, R, centre)
    g, o = make_pair(2, N, fwd, back)
    x = white_noise_f32(3 * 1024 + 517, seed=1)
    tol = TOL_STIFF if centre == 1.0 else TOL
    yg, yo = g.process(x), o.process(x)
    err = rel_err(yg, yo)
    assert err < tol, err
    # a second call continues the state (carried across calls)
    x2 = white_noise_f32(2048, seed=2)
    err2 = rel_err(g.process(x2), o.process(x2))
    assert err2 < tol, err2


@pytest.mark.parametrize("order", [0, 1, 2, 3, 4])
def test_orders_random(gpu_lib, order):
    rng = np.random.default_rng(100 + order)
    N = 37
    fwd = rng.uniform(-1, 1, (N, order + 1))
    back = np.zeros((N, max(order, 1)))
    for n in range(N):
        # conjugate pole pairs (+ one real pole for odd orders), radius 0.97
        roots = []
        for _ in range(order // 2):
            p = 0.97 * np.exp(1j * rng.uniform(0, np.pi))
            roots += [p, np.conj(p)]
        if order % 2 == 1:
            roots.append(0.97 * rng.uniform(-1, 1))
        if order:
            back[n, :order] = np.real(np.poly(roots))[1:]
    g, o = make_pair(order, N, fwd, back[:, :order], kp=0.05, kg=0.3)
    x = rng.uniform(-1, 1, 2500)
    assert rel_err(g.process(x), o.process(x)) < TOL


def test_block_split_and_per_sample(gpu_lib):
    """process() over arbitrary splits == one call; operator()/tick() per sample
    (n = 1 < order) keeps the history exact."""
    N = 64
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make_pair(2, N, fwd, back)
    x = white_noise_f32(5000, seed=4)
    ref = o.process(x)
    parts, pos = [], 0
    for L in [1, 1, 2, 3, 1021, 1024, 1, 1500]:
        parts.append(g.process(x[pos:pos + L]))
        pos += L
    # per-sample operator()/tick() with the cached-value semantics
    for i in range(pos, pos + 40):
        v = g(x[i])
        assert g(x[i]) == v  # repeated operator() before tick() returns the cached value
        g.tick()
        parts.append(np.array([v]))
    pos += 40
    parts.append(g.process(x[pos:]))
    assert rel_err(np.concatenate(parts), ref) < TOL


def test_setters_between_calls(gpu_lib):
    N = 16
    fwd, back = resonant_coefficients(N, 0.99, 0.5)
    g, o = make_pair(2, N, fwd, back, kp=0.0, kg=0.01)
    rng = np.random.default_rng(5)
    outs_g, outs_o = [], []
    for step in range(6):
        x = rng.uniform(-1, 1, 700)
        outs_g.append(g.process(x))
        outs_o.append(o.process(x))
        n = int(rng.integers(0, N))
        for fb in (g, o):
            fb.boost(n, float(step) * 0.3)
            fb.mix(n, -1.0 + step)
            fb.coefficients((n + 3) % N, [0.2, 0.1, -0.2], [-1.8 * np.cos(0.1 * step), 0.95])
    assert rel_err(np.concatenate(outs_g), np.concatenate(outs_o)) < TOL


@pytest.mark.parametrize("dist_id,param", [(1, 0.125), (2, 0.0), (3, 0.0)])
def test_distortions(gpu_lib, dist_id, param):
    N = 24
    fwd, back = resonant_coefficients(N, 0.995, 0.5)
    g, o = make_pair(2, N, fwd, back)
    g.distortion(dist_id, param)
    o.distortion(dist_id, param)
    x = 0.5 * white_noise_f32(4000, seed=6)
    assert rel_err(g.process(x), o.process(x)) < TOL


def test_shards_sum_to_full(gpu_lib):
    """Band sharding (multi-GPU partition): partial mixes of shards sum to the full mix."""
    N = 300
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    from huygens_amd import Filterbank
    full, o = make_pair(2, N, fwd, back)
    shards = []
    for b0, cnt in [(0, 128), (128, 100), (228, 72)]:
        s = Filterbank(2, N, shard=(b0, cnt))
        for n in range(N):  # setters use global indices; out-of-shard bands are ignored
            s.coefficients(n, fwd[n], back[n])
        s.boost(np.ones(N))
        s.open()
        shards.append(s)
    x = white_noise_f32(2500, seed=7)
    ref = o.process(x)
    yf = full.process(x)
    ys = sum(s.process(x) for s in shards)
    assert rel_err(yf, ref) < TOL
    assert rel_err(ys, ref) < TOL


def test_state_roundtrip(gpu_lib):
    from huygens_amd import Filterbank
    N = 50
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    a, _ = make_pair(2, N, fwd, back)
    b, _ = make_pair(2, N, fwd, back)
    x = white_noise_f32(3000, seed=8)
    a.process(x[:1234])
    b.set_state(a.get_state())
    ya = a.process(x[1234:])
    yb = b.process(x[1234:])
    assert np.array_equal(ya, yb)


def test_device_pointer_path(gpu_lib):
    torch = pytest.importorskip("torch")
    N = 512
    fwd, back = resonant_coefficients(N, 0.999, 0.5)
    g, o = make_pair(2, N, fwd, back)
    x = white_noise_f32(4096 + 100, seed=9)
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty_like(xd)
    torch.cuda.synchronize()
    g.process_device(xd.data_ptr(), yd.data_ptr(), len(x))
    g.synchronize()
    assert rel_err(yd.cpu().numpy(), o.process(x)) < TOL


def test_errors_are_reported(gpu_lib):
    from huygens_amd import Filterbank, HZError
    fb = Filterbank(2, 8)
    with pytest.raises(HZError):
        fb.coefficients(8, [1, 0, -1], [0, 0])
    with pytest.raises(HZError):
        fb.boost(-1, 1.0)
    y = fb.process(np.zeros(0))
    assert y.shape == (0,)


@pytest.mark.parametrize("N,n,groups", [(512, 20000, 256), (64, 9000, 1024), (7, 50000, 4096)])
def test_time_segments(gpu_lib, N, n, groups):
    """Small banks are split into time segments (segment end states -> per-band
    carry -> segmented mix); results must not depend on the segmentation."""
    fwd, back = resonant_coefficients(N, 0.9995, 0.5)
    g, o = make_pair(2, N, fwd, back)
    g.set_target_groups(groups)
    x = white_noise_f32(n, seed=10)
    assert rel_err(g.process(x[:n // 3]), o.process(x[:n // 3])) < TOL
    assert rel_err(g.process(x[n // 3:]), o.process(x[n // 3:])) < TOL


@pytest.mark.parametrize("waves,nb", [(4, 1), (4, 2), (4, 4), (8, 1), (8, 2), (16, 1)])
@pytest.mark.parametrize("order,N", [(2, 4096), (2, 37), (1, 9), (3, 130)])
def test_geometries(gpu_lib, waves, nb, order, N):
    """Every workgroup geometry (waves x bands per wave) on ragged banks and signals,
    with pre/gain ramps, two calls, time segments for small banks."""
    rng = np.random.default_rng(order * 1000 + N)
    fwd = rng.uniform(-0.05, 0.05, (N, order + 1))
    back = []
    for n in range(N):
        r = rng.uniform(0.5, 0.99, order)
        back.append(np.poly(r)[1:] if order else np.zeros(0))
    back = np.array(back)
    g, o = make_pair(order, N, fwd, back, boost=False)
    g.tune(waves, nb)
    boost = rng.uniform(0.5, 1.5, N)
    for fb in (g, o):
        fb.boost(boost)
    x = white_noise_f32(3000, seed=3)
    assert rel_err(g.process(x), o.process(x)) < TOL
    x2 = white_noise_f32(2100, seed=4)
    assert rel_err(g.process(x2), o.process(x2)) < TOL


@pytest.mark.parametrize("order", [1, 2, 4])
def test_tick_without_operator(gpu_lib, order):
    """tick() without operator() (filterbank.h:142-148): the ring rotates with its stale row,
    nothing is computed and the smoothers stand still (hz_fb_tick); bare ticks at the start,
    in runs and between 1-sample calls; HZ_E_STATE after a block call."""
    from huygens_amd import Filterbank
    from huygens_amd._lib import HZ_E_STATE, HZError
    rng = np.random.default_rng(40 + order)
    N = 70
    fwd = rng.uniform(-1, 1, (N, order + 1))
    back = rng.uniform(-0.3, 0.3, (N, order)) / order
    boost = rng.uniform(0.5, 1.5, N)
    g = Filterbank(order, N, 0.1, 1.0)
    o = OracleFilterbank(order, N, 0.1, 1.0)
    for fb in (g, o):
        for n in range(N):
            fb.coefficients(n, fwd[n], back[n])
        fb.boost(boost)
        fb.open()
    outs_g, outs_o = [], []
    ops = ["tick", "tick"] + list(rng.choice(["op", "tick", "op2"], 200, p=[0.6, 0.25, 0.15]))
    for op in ops:
        if op == "tick":
            g.tick()
            o.tick()
        else:
            x = float(rng.uniform(-1, 1))
            outs_g.append(g(x))
            outs_o.append(o(x))
            if op == "op2":   # repeated operator() before tick(): cached
                assert g(x + 1) == outs_g[-1]
                o(x + 1)
            g.tick()
            o.tick()
    err = rel_err(np.array(outs_g), np.array(outs_o))
    assert err < TOL, err
    # after a block call the spare ring row is not kept: the recorded tick fails at the next
    # sample (or block call) -- and at once through the direct ABI entry hz_fb_tick
    g.process(white_noise_f32(64, seed=5))
    g.tick()
    with pytest.raises(HZError) as ei:
        g(0.5)
    assert ei.value.code == HZ_E_STATE
    g2 = Filterbank(order, N, 0.1, 1.0)
    g2.process(white_noise_f32(64, seed=5))
    assert g2._lib.hz_fb_tick(g2._h) == HZ_E_STATE
