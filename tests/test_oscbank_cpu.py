"""CPU: the Oscbank oracle against the golden fixtures (independent numpy restatement)."""
import numpy as np
import pytest

from oracle import OracleOscbank, golden_names, load_golden, run_osc_events


@pytest.mark.parametrize("name", golden_names("osc_"))
def test_oscbank_oracle_matches_golden(name):
    g = load_golden(name)
    o = OracleOscbank(int(g["N"]))
    mix = run_osc_events(o, g)
    assert np.max(np.abs(mix - g["mix"])) <= 1e-12 * max(1.0, np.max(np.abs(g["mix"])))
    assert np.max(np.abs(o.phases() - g["z_final"])) < 1e-12


def test_oscbank_active_set_protocol():
    o = OracleOscbank(8)
    o.activate([3, 1, 7, 1, 99, -2])     # duplicates and out-of-range ignored
    assert o.active_count() == 3
    o.deactivate([1, 5])
    assert o.active_count() == 2
    o.open()
    assert o.active_count() == 8
    o.close_all()
    assert o.active_count() == 0
    assert np.all(o.fill(5) == 0)
