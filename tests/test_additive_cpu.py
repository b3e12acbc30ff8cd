"""CPU: the Additive / Sinusoids oracle against the golden fixtures."""
import numpy as np
import pytest

from oracle import golden_names, load_golden, rel_err
from oracle_osc import OracleAdditive, OracleSinusoids, run_note_events


@pytest.mark.parametrize("name", golden_names("add_"))
def test_additive_oracle_matches_golden(name):
    g = load_golden(name)
    a = OracleAdditive(int(g["V"]), int(g["O"]), float(g["decay"]), float(g["harm"]), float(g["k"]))
    assert rel_err(run_note_events(a, g), g["y"]) < 1e-11


@pytest.mark.parametrize("name", golden_names("sin_"))
def test_sinusoids_oracle_matches_golden(name):
    g = load_golden(name)
    s = OracleSinusoids(float(g["fund"]), int(g["O"]), float(g["decay"]), float(g["harm"]), float(g["k"]))
    assert rel_err(run_note_events(s, g), g["y"]) < 1e-11


def test_released_voice_keeps_ticking():
    """A released voice's amplitude sticks at a denormal (66 * 2^-1074) and never reaches
    0 (additive.h:41-43), so its oscillators keep ticking: the phase of a voice re-used
    later depends on that.  The oracle reproduces it."""
    a = OracleAdditive(1, 2, 0.5, 1.0, 0.1)
    a.makenote(69, 1.0)
    a.fill(10)
    a.release(0)
    y = a.fill(120_000)
    assert y[-1] != 0.0 or np.any(y[-100:] != 0.0)
