"""CPU tests: the oracle (C restatement) against the golden fixtures written by
the independent numpy restatement (tests/golden/make_golden.py), plus the
scipy/closed-form known answers.  No GPU needed."""
import math

import numpy as np
import pytest
from scipy import signal

from oracle import OracleFilterbank, golden_names, lib, load_golden, rel_err, run_schedule
from golden.spec_numpy import PI, SR, dist as spec_dist, relaxation as spec_relaxation


def test_constants_and_relaxation():
    L = lib()
    for k in [0.0, 1e-4, 0.001, 0.1, 1.0, 2.0 / SR, 50.0, -1.0]:
        if k < 0:
            # fmax(0,k) = 0 -> division by zero -> 2^-inf = 0
            assert L.orc_relaxation(k) == 0.0
            continue
        assert L.orc_relaxation(k) == spec_relaxation(k)
    # relaxation(50) = 1 - 1.5e-5 (tests/filterbank.cpp:136)
    assert abs(L.orc_relaxation(50) - (1 - 1.5e-5)) < 1e-6
    assert abs(L.orc_mtof(69) - 440.0) < 1e-12
    assert abs(L.orc_ftom(880.0) - 81.0) < 1e-12


@pytest.mark.parametrize("dist_id,param", [(0, 0), (1, 0.125), (1, 0.5), (2, 0), (3, 0)])
def test_distortions(dist_id, param):
    L = lib()
    v = np.linspace(-3, 3, 601)
    got = np.array([L.orc_dist(dist_id, float(a), param) for a in v])
    assert np.max(np.abs(got - spec_dist(dist_id, v, param))) < 1e-15


@pytest.mark.parametrize("name", golden_names("fb_"))
def test_filterbank_oracle_matches_golden(name):
    g = load_golden(name)
    fb = OracleFilterbank(int(g["order"]), int(g["N"]), float(g["kp"]), float(g["kg"]))
    fb.distortion(int(g["dist"]), float(g["dist_param"]))
    y = run_schedule(fb, g["x"], g["sched_t"], g["sched_kind"], g["sched_band"], g["sched_val"],
                     g["fwd"], g["back"])
    assert rel_err(y, g["y"]) < 1e-12


def test_filterbank_oracle_lfilter_known_answer():
    """k_p = k_g = 0: pre = gain = target immediately -> plain lfilter."""
    rng = np.random.default_rng(11)
    x = rng.uniform(-1, 1, 3000)
    b = np.array([0.3, -0.2, 0.1])
    a = np.array([-1.5, 0.7])
    fb = OracleFilterbank(2, 1, 0.0, 0.0)
    fb.coefficients(0, b, a)
    fb.boost(0, 2.0)
    fb.mix(0, 0.5)
    y = fb.process(x)
    ref = 0.5 * signal.lfilter(2.0 * b, np.concatenate(([1.0], a)), x)
    assert rel_err(y, ref) < 1e-13


def test_filterbank_oracle_silent_without_boost():
    """resynthesis.cpp as written (no boost/mix/open) is silent."""
    fb = OracleFilterbank(2, 4)
    fb.coefficients(0, [1, 0, -1], [-1.9, 0.99])
    y = fb.process(np.random.default_rng(0).uniform(-1, 1, 500))
    assert np.all(y == 0.0)


def test_filterbank_oracle_block_split_invariance():
    g = load_golden("fb_o2_n16_r0999")
    fb1 = OracleFilterbank(2, 16)
    fb2 = OracleFilterbank(2, 16)
    for fb in (fb1, fb2):
        for n in range(16):
            fb.coefficients(n, g["fwd"][n], g["back"][n])
        fb.boost(np.ones(16))
        fb.open()
    x = g["x"]
    y1 = fb1.process(x)
    parts = []
    pos = 0
    for L in [1, 2, 3, 500, 1024, 7]:
        parts.append(fb2.process(x[pos:pos + L]))
        pos += L
    parts.append(fb2.process(x[pos:]))
    assert np.array_equal(y1, np.concatenate(parts))


@pytest.mark.parametrize("order,N,n", [(2, 5, 2500), (1, 3, 1100), (3, 3, 2100), (0, 2, 1500)])
def test_kernel_algorithm_model(order, N, n):
    """The chunked-scan algebra of fb_mix_kernel (numpy lane model) == sequential oracle."""
    from kernel_model import mix_model
    rng = np.random.default_rng(order)
    fwd = rng.uniform(-1, 1, (N, order + 1))
    back = np.zeros((N, order))
    for b in range(N):
        roots = []
        for _ in range(order // 2):
            p = 0.99 * np.exp(1j * rng.uniform(0, np.pi))
            roots += [p, np.conj(p)]
        if order % 2:
            roots.append(0.99 * rng.uniform(-1, 1))
        if order:
            back[b] = np.real(np.poly(roots))[1:]
    x = rng.uniform(-1, 1, n)
    fb = OracleFilterbank(order, N, 0.1, 1.0)
    for b in range(N):
        fb.coefficients(b, fwd[b], back[b])
    fb.boost(np.ones(N))
    fb.open()
    ref = fb.process(x)
    from golden.spec_numpy import relaxation
    got = mix_model(fwd, back, relaxation(0.1), relaxation(1.0), np.ones(N), np.ones(N), x)
    assert rel_err(got, ref) < 1e-10


@pytest.mark.parametrize("order,N,L,n", [(2, 4, 32, 2 * 2048 + 32 * 5), (1, 3, 16, 1024 + 48), (3, 2, 16, 2048),
                                         (4, 2, 32, 2048 + 64)])
def test_lti_algorithm_model(order, N, L, n):
    """The converged engine's algebra (hz_fb_lti.hip: chunk end states, 64-lane DPP prefix
    with row_bcast, bank-wide zero-state matrix) == the sequential oracle once the
    smoothers have converged (k_p = k_g = 0: pre = pin and gain = gin from sample 0)."""
    from lti_model import lti_mix_model
    rng = np.random.default_rng(10 + order)
    fwd = rng.uniform(-1, 1, (N, order + 1))
    back = np.zeros((N, order))
    for b in range(N):
        roots = []
        for _ in range(order // 2):
            p = 0.98 * np.exp(1j * rng.uniform(0, np.pi))
            roots += [p, np.conj(p)]
        if order % 2:
            roots.append(0.98 * rng.uniform(-1, 1))
        back[b] = np.real(np.poly(roots))[1:]
    pin, gin = rng.uniform(0.5, 2, N), rng.uniform(-1, 1, N)
    fb = OracleFilterbank(order, N, 0.0, 0.0)
    for b in range(N):
        fb.coefficients(b, fwd[b], back[b])
    fb.boost(pin)
    fb.mix(gin)
    x = rng.uniform(-1, 1, n)
    ref = fb.process(x)
    got = lti_mix_model(fwd, back, pin, gin, x, L=L)
    assert rel_err(got, ref) < 1e-10


def _ring_model_ops(order, N, F, B, pin, gin, sp, sg, ops):
    """Pure-Python restatement of Filterbank's rings (src/filterbank.h:125-187): input ring of
    2(O+1), outputs ring of 2(O+1) x N, origin; ops = sequence of ('op', x) / ('tick',)."""
    R = order + 1
    xr = [0.0] * (2 * R)
    Y = [[0.0] * N for _ in range(2 * R)]
    pre, gain = [0.0] * N, [0.0] * N
    origin, computed, outs = 0, False, []
    for op in ops:
        if op[0] == "op":
            if not computed:
                for n in range(N):
                    pre[n] = (1 - sp) * pin[n] + sp * pre[n]
                    gain[n] = (1 - sg) * gin[n] + sg * gain[n]
                xr[origin] = xr[origin + R] = op[1]
                row = []
                for n in range(N):
                    ff = F[n][0] * xr[origin]
                    for i in range(1, order + 1):
                        ff += F[n][i] * xr[origin + i]
                    bs = 0.0
                    for k in range(order):
                        bs += B[n][k] * Y[origin + 1 + k][n]
                    row.append(ff * pre[n] - bs)
                Y[origin] = list(row)
                Y[origin + R] = list(row)
                computed = True
            s = 0.0
            for n in range(N):
                s += Y[origin][n] * gain[n]
            outs.append(s)
        else:
            origin -= 1
            if origin < 0:
                origin += R
            computed = False
    return np.array(outs)


@pytest.mark.parametrize("order", [1, 2, 3])
def test_filterbank_oracle_tick_without_operator(order):
    """tick() without operator() (filterbank.h:142-148) reuses the stale ring row: the C
    restatement follows an independent Python model of the rings on ops with bare ticks."""
    from oracle import OracleFilterbank
    rng = np.random.default_rng(7 + order)
    N = 5
    F = rng.uniform(-1, 1, (N, order + 1))
    B = rng.uniform(-0.3, 0.3, (N, order)) / order
    pin, gin = rng.uniform(0.5, 1.5, N), rng.uniform(0.5, 1.5, N)
    ops = []
    for _ in range(300):
        r = rng.uniform()
        if r < 0.25:
            ops.append(("tick",))
        elif r < 0.35:
            ops.append(("op", float(rng.uniform(-1, 1))))   # repeated operator(): cached
        else:
            ops += [("op", float(rng.uniform(-1, 1))), ("tick",)]
    o = OracleFilterbank(order, N, 0.1, 1.0)
    for n in range(N):
        o.coefficients(n, F[n], B[n])
    o.boost(pin)
    o.mix(gin)
    got = [o(op[1]) if op[0] == "op" else o.tick() for op in ops]
    got = np.array([v for v, op in zip(got, ops) if op[0] == "op"])
    want = _ring_model_ops(order, N, F, B, pin, gin, o.l.orc_relaxation(0.1), o.l.orc_relaxation(1.0), ops)
    assert np.array_equal(got, want)
