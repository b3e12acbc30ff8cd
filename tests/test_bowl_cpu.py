"""CPU: the Bowl<T> oracle against the golden fixtures (numpy restatement)."""
import numpy as np
import pytest

from oracle import golden_names, load_golden, rel_err
from oracle_bowl import OracleBowl


@pytest.mark.parametrize("name", golden_names("bowl_"))
def test_bowl_double_oracle(name):
    g = load_golden(name)
    b = OracleBowl(int(g["M"]), g["f"], g["a"], g["d"], np.float64)
    y = b.render(int(g["n"]))
    assert rel_err(y, g["y_double"]) < 1e-12
    b.trigger()
    yf = b.fill(int(g["n"]))              # fill() writes float
    assert np.array_equal(yf, y.astype(np.float32))


@pytest.mark.parametrize("name", golden_names("bowl_"))
def test_bowl_float_oracle(name):
    """Mixed-precision Bowl<float>: the C restatement and the numpy restatement agree
    bit-for-bit except where libm and numpy sin differ in the last ulp before the
    float rounding."""
    g = load_golden(name)
    b = OracleBowl(int(g["M"]), g["f"], g["a"], g["d"], np.float32)
    y = b.fill(int(g["n"]))
    assert rel_err(y, g["y_float"]) < 1e-6
    assert np.mean(y == g["y_float"]) > 0.95


def test_float_model_differs_from_double():
    """The float model's phase rounding is part of the reference output (not noise)."""
    g = load_golden("bowl_m32")
    assert rel_err(g["y_float"], g["y_double"]) > 1e-7


def test_bowl_pad_and_trigger():
    b = OracleBowl(4, [100.0, 200.0], [0.1, 0.2], [1.0, 2.0])   # resize(4, 0) pads modes
    y1 = b.render(100)
    b.trigger()
    y2 = b.render(100)
    assert np.array_equal(y1, y2) and y1[0] == 0.0
