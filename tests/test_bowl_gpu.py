"""GPU parity: Bowl<T> HIP engine vs the CPU restatement.

T = double: rotation of decaying phasors vs the reference's direct pow/sin: 1e-9.
T = float : per-sample float-rounded phase (bit-faithful) with the sum kept in double;
the reference rounds the running sum to float after every mode, so the bound is the
north-star 1e-5 (observed ~1e-7)."""
import numpy as np
import pytest

from oracle import golden_names, load_golden, rel_err
from oracle_bowl import OracleBowl

pytestmark = pytest.mark.gpu
NORTH_STAR = 1e-5


@pytest.mark.parametrize("name", golden_names("bowl_"))
def test_golden(gpu_lib, name):
    from huygens_amd import Bowl
    g = load_golden(name)
    n = int(g["n"])
    bd = Bowl(int(g["M"]), g["f"], g["a"], g["d"], np.float64)
    assert rel_err(bd.render(n), g["y_double"]) < 1e-9
    bf = Bowl(int(g["M"]), g["f"], g["a"], g["d"], np.float32)
    assert rel_err(bf.fill(n), g["y_float"]) < NORTH_STAR


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("M,n,groups", [(2048, 5000, 256), (303, 30000, 256), (5, 7000, 1)])
def test_c5_shape(gpu_lib, dtype, M, n, groups):
    """C5 shape (2048 modes) and smaller models, several calls (phase counter carried),
    trigger() resets."""
    from huygens_amd import Bowl
    rng = np.random.default_rng(M)
    f = np.exp(rng.uniform(np.log(20.0), np.log(16000.0), M))
    a = rng.uniform(1e-4, 5e-2, M)
    d = rng.uniform(0.05, 15.0, M)
    g, o = Bowl(M, f, a, d, dtype), OracleBowl(M, f, a, d, dtype)
    g.set_target_groups(groups)
    tol = 1e-9 if dtype == np.float64 else NORTH_STAR
    parts_g, parts_o = [], []
    for L in (n // 3, 1, n - n // 3 - 1):
        parts_g.append(g.fill(L))
        parts_o.append(o.fill(L))
    assert rel_err(np.concatenate(parts_g), np.concatenate(parts_o)) < tol
    assert g.phase() == n
    g.trigger()
    o.trigger()
    assert rel_err(g.fill(1000), o.fill(1000)) < tol


def test_bowl_render_double_precision(gpu_lib):
    from huygens_amd import Bowl
    f, a, d = [440.0, 660.0, 1234.5], [0.3, 0.2, 0.1], [1.0, 3.0, 0.5]
    g, o = Bowl(3, f, a, d), OracleBowl(3, f, a, d)
    assert rel_err(g.render(20000), o.render(20000)) < 1e-9
