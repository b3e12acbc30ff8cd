"""GPU parity: Additive / Sinusoids HIP engine vs the CPU restatement and fixtures.

Bound: north-star 1e-5 (norm-wise).  The engine evaluates the oscillators' closed-form
phase instead of the per-sample recurrence, so the difference is rounding-level; the
asserted bound is 1e-8."""
import numpy as np
import pytest

from oracle import golden_names, load_golden, rel_err
from oracle_osc import OracleAdditive, OracleSinusoids, run_note_events

pytestmark = pytest.mark.gpu
TOL = 1e-8


@pytest.mark.parametrize("name", golden_names("add_"))
def test_additive_golden(gpu_lib, name):
    from huygens_amd import Additive
    g = load_golden(name)
    a = Additive(int(g["V"]), int(g["O"]), float(g["decay"]), float(g["harm"]), float(g["k"]))
    assert rel_err(run_note_events(a, g), g["y"]) < TOL


@pytest.mark.parametrize("name", golden_names("sin_"))
def test_sinusoids_golden(gpu_lib, name):
    from huygens_amd import Sinusoids
    g = load_golden(name)
    s = Sinusoids(float(g["fund"]), int(g["O"]), float(g["decay"]), float(g["harm"]), float(g["k"]))
    assert rel_err(run_note_events(s, g), g["y"]) < TOL


@pytest.mark.parametrize("V,O,n,groups", [(64, 256, 3000, 256), (8, 40, 9000, 64), (2, 3, 5000, 1)])
def test_additive_c3_shape(gpu_lib, V, O, n, groups):
    """C3 shape (64 voices x 256 partials, all sounding) and small banks with time segments."""
    from huygens_amd import Additive
    g, o = Additive(V, O, 0.75, 1.0), OracleAdditive(V, O, 0.75, 1.0)
    g.set_target_groups(groups)
    for b in (g, o):
        for v in range(V):
            b.makenote(36 + v, 1.0)
    y1g, y1o = g.fill(n), o.fill(n)
    assert rel_err(y1g, y1o) < TOL
    for b in (g, o):
        for v in range(0, V, 3):
            b.endnote(36 + v)
    assert rel_err(g.fill(n // 2), o.fill(n // 2)) < TOL


def test_additive_shards_sum(gpu_lib):
    from huygens_amd import Additive
    V, O, n = 6, 30, 4000
    o = OracleAdditive(V, O, 0.8)
    shards = [Additive(V, O, 0.8, shard=s) for s in [(0, 12), (12, 10), (22, 8)]]
    for b in [o] + shards:
        for v in range(V):
            b.makenote(50 + 2 * v, 0.5 + 0.1 * v)
    ref = o.fill(n)
    assert rel_err(sum(s.fill(n) for s in shards), ref) < TOL


def test_additive_silent_until_note(gpu_lib):
    from huygens_amd import Additive
    a = Additive(4, 4, 0.5)
    assert np.all(a.fill(2000) == 0.0)
