"""Per-sample operator API of the generator banks (Additive, Sinusoids, Bowl, Oscbank), served
from speculative blocks with rollback (huygens_hip.h, hz_add_fill): the reference's demos call
`y = bank(); bank.tick();` once per sample (tests/additive.cpp:27-37, tests/oscbank.cpp:102-126,
tests/bowl.cpp:49-54), with setters in between (MIDI: tests/additive.cpp:42-78).  Each test
drives the GPU bank through per-sample calls, block calls and setters at arbitrary samples, and
the C restatement through the same schedule with block fills split at the same points."""
import numpy as np
import pytest

from oracle import OracleOscbank, rel_err
from oracle_bowl import OracleBowl
from oracle_osc import OracleAdditive, OracleSinusoids

pytestmark = pytest.mark.gpu
TOL = 1e-8


def drive(g, o, schedule, per_sample, block):
    """schedule: ("s", n) n per-sample calls on the GPU bank; ("b", n) a block call on both;
    ("e", fn) a setter applied to both.  The oracle always fills in blocks."""
    outs_g, outs_o = [], []
    for kind, arg in schedule:
        if kind == "s":
            outs_g.append(np.array([per_sample(g) for _ in range(arg)]))
            outs_o.append(block(o, arg))
        elif kind == "b":
            outs_g.append(block(g, arg))
            outs_o.append(block(o, arg))
        else:
            arg(g)
            arg(o)
    return np.concatenate(outs_g), np.concatenate(outs_o)


def test_additive_per_sample_with_notes(gpu_lib):
    from huygens_amd import Additive
    from huygens_amd.additive import lookahead_info
    V, O = 10, 7   # tests/additive.cpp:23
    g, o = Additive(V, O, 0.75, 1.0), OracleAdditive(V, O, 0.75, 1.0)
    sched = [("e", lambda b: b.makenote(60, 1.0)), ("s", 700), ("e", lambda b: b.makenote(64, 0.5)),
             ("s", 1500), ("b", 3000), ("s", 37), ("e", lambda b: b.endnote(60)), ("s", 2100),
             ("e", lambda b: b.makenote(67, 0.8)), ("s", 1024), ("s", 1)]
    yg, yo = drive(g, o, sched, lambda b: b.fill(1)[0], lambda b, n: b.fill(n))
    assert rel_err(yg, yo) < TOL
    blocks, rollbacks, L = lookahead_info(g)
    assert L == 1024 and blocks >= 5 and rollbacks >= 3, (blocks, rollbacks)


def test_additive_c3_shape_per_sample(gpu_lib):
    from huygens_amd import Additive
    V, O = 64, 256
    g, o = Additive(V, O, 0.75, 1.0), OracleAdditive(V, O, 0.75, 1.0)
    for b in (g, o):
        for v in range(V):
            b.makenote(36 + v, 1.0)
    sched = [("s", 2048), ("e", lambda b: b.endnote(40)), ("s", 600)]
    yg, yo = drive(g, o, sched, lambda b: b.fill(1)[0], lambda b, n: b.fill(n))
    assert rel_err(yg, yo) < TOL


def test_sinusoids_per_sample_with_mods(gpu_lib):
    from huygens_amd import Sinusoids
    g, o = Sinusoids(220.0, 12, 0.8, 1.0), OracleSinusoids(220.0, 12, 0.8, 1.0)
    sched = [("s", 900), ("e", lambda b: b.fundmod(330.0)), ("s", 1300), ("b", 500),
             ("e", lambda b: b.decaymod(0.6)), ("s", 77), ("e", lambda b: b.harmmod(1.1)), ("s", 1100)]
    yg, yo = drive(g, o, sched, lambda b: b.fill(1)[0], lambda b, n: b.fill(n))
    assert rel_err(yg, yo) < TOL


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_bowl_per_sample_with_triggers(gpu_lib, dtype):
    from huygens_amd import Bowl
    rng = np.random.default_rng(5)
    M = 303   # tests/bowl.cpp:44
    f = np.exp(rng.uniform(np.log(20), np.log(16000), M))
    a = rng.uniform(1e-4, 5e-2, M)
    d = rng.uniform(0.05, 15, M)
    g, o = Bowl(M, f, a, d, dtype=dtype), OracleBowl(M, f, a, d, dtype=dtype)
    for b in (g, o):
        b.trigger()
    sched = [("s", 1500), ("e", lambda b: b.trigger()), ("s", 400), ("b", 2000), ("s", 1030),
             ("e", lambda b: b.trigger()), ("s", 5)]
    yg, yo = drive(g, o, sched, lambda b: b.render(1)[0], lambda b, n: b.render(n))
    assert rel_err(yg, yo) < (1e-5 if dtype == np.float32 else TOL)


def test_oscbank_per_sample_operator_mixdown_tick(gpu_lib):
    from huygens_amd import Oscbank
    N = 96
    g, o = Oscbank(N), OracleOscbank(N)
    rng = np.random.default_rng(9)
    for b in (g, o):
        for i in range(N):
            b.freqmod(i, 40.0 * (i + 1))
        b.activate(list(range(0, N, 2)))
    zs_g, mix_g, zs_o, mix_o = [], [], [], []

    def per_sample(n):
        for _ in range(n):
            zs_g.append(g.phases().copy())
            mix_g.append(g.mixdown())
            g.tick()
        m, pb = o.fill(n, per_band=True)
        zs_o.extend(pb)
        mix_o.extend(m)

    per_sample(700)
    for b in (g, o):
        b.freqmod(3, 1234.5)
        b.activate([1, 5, 7])
    per_sample(1300)
    m1, p1 = g.fill(500, per_band=True)
    m2, p2 = o.fill(500, per_band=True)
    assert rel_err(m1, m2) < TOL and rel_err(p1, p2) < TOL
    for b in (g, o):
        b.deactivate([0, 2])
    per_sample(rng.integers(50, 100))
    assert rel_err(np.array(zs_g), np.array(zs_o)) < TOL
    assert rel_err(np.array(mix_g), np.array(mix_o)) < TOL
