"""CPU: the Delay/Delaybank restatement against the golden fixtures (bit-exact)."""
import numpy as np
import pytest

from oracle import golden_names, load_golden
from oracle_delay import OracleDelaybank, bank_from_golden


@pytest.mark.parametrize("name", golden_names("dly_"))
def test_delay_oracle_golden(name):
    g = load_golden(name)
    b = bank_from_golden(OracleDelaybank, g)
    y = b.process(g["x"])
    assert np.array_equal(y, g["y"])
    assert b.origin() == int(g["origin"])


def test_delay_mixdown_golden():
    g = load_golden("dly_bank_f")
    b = bank_from_golden(OracleDelaybank, g)
    assert np.array_equal(b.process(g["x"], mix=True), g["mix"])


def test_impulse_echo_positions():
    """tests/delay.cpp:41 pattern: echoes at every sum of 100s and 200s."""
    g = load_golden("dly_impulse")
    e = g["echoes"]
    assert e[0] == 0 and e[1] == 100 and np.all(e % 100 == 0)
    assert np.array_equal(np.flatnonzero(g["y"][0]), e)


def test_wrap_is_not_modular():
    """The uint32 wrap: a delay longer than the ring does NOT read (o - c) mod size."""
    b = OracleDelaybank(1, 1, 99, np.float64)          # ring of 100
    b.coefficients(0, [(250, 1.0)], [])
    x = np.zeros(400)
    x[10] = 1.0
    y = b.process(x)[0]
    hit = np.flatnonzero(y)
    # (250 - 2^32) mod 100 = 54 samples of age, not 50
    assert hit[0] == 10 + 54


def test_zero_time_feedback_dropped_and_per_line_input():
    b = OracleDelaybank(2, 2, 50, np.float64)
    b.coefficients(0, [(0, 1.0)], [(0, 0.9)])          # e = 0 -> {0,0}: plain copy
    b.coefficients(1, [(3, 2.0)], [])
    x = np.random.default_rng(0).standard_normal((2, 40))
    y = b.process(x)
    assert np.array_equal(y[0], x[0])
    assert np.array_equal(y[1, 3:], 2.0 * x[1, :-3]) and np.all(y[1, :3] == 0)
