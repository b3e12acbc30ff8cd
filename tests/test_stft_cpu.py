"""CPU: the Fourier/StaticSTFT/Cosine restatement against the numpy fixtures."""
import numpy as np
import pytest

from oracle import golden_names, load_golden, rel_err
from oracle_stft import OracleSTFT, oracle_dct, oracle_dft


@pytest.mark.parametrize("name", golden_names("stft_"))
def test_stft_oracle_golden(name):
    g = load_golden(name)
    o = OracleSTFT(int(g["N"]), int(g["laps"]), int(g["window"]), int(g["proc"]))
    yr, yi = o.process_block(g["x_re"], g["x_im"])
    scale = max(np.max(np.abs(g["y_re"])), np.max(np.abs(g["y_im"])), 1e-300)
    assert np.max(np.abs(yr - g["y_re"])) <= 1e-12 * scale
    assert np.max(np.abs(yi - g["y_im"])) <= 1e-12 * scale
    assert o.frames() == len(g["starts"])
    assert float(g["margin"]) > 1e-6          # no gate decision near its threshold


def test_irregular_hop():
    """Frames start at stride*i + c*(2N-1): one hop in 2*laps is stride-1."""
    g = load_golden("stft_static_n64")
    hops = np.diff(g["starts"])
    assert set(hops.tolist()) == {15, 16}
    assert np.sum(hops == 15) == len(hops) // 8


def test_identity_reconstructs():
    """halfhann^2 overlap-add with laps=4, identity processor: steady-state output is the
    input delayed by N-1, scaled by sum hann / (laps/2) ~ 1."""
    g = load_golden("stft_id_n16_cplx")
    N = int(g["N"])
    y = g["y_re"] + 1j * g["y_im"]
    x = g["x_re"] + 1j * g["x_im"]
    mid = slice(2 * N, len(x) - N)
    ratio = np.abs(y[mid]) / np.maximum(np.abs(x[mid.start - N + 1:mid.stop - N + 1]), 1e-9)
    assert 0.5 < np.median(ratio) < 1.5


def crel(a, b):
    return np.max(np.abs(np.asarray(a) - np.asarray(b))) / np.max(np.abs(np.asarray(b)))


def test_dft_and_dct_conventions():
    rng = np.random.default_rng(1)
    x = rng.standard_normal(48) + 1j * rng.standard_normal(48)   # non power of two path
    assert crel(oracle_dft(x, -1), np.fft.fft(x)) < 1e-14
    assert crel(oracle_dft(x, +1), np.fft.ifft(x) * 48) < 1e-14
    x = rng.standard_normal(64) + 1j * rng.standard_normal(64)   # radix-2 path
    assert crel(oracle_dft(x, -1), np.fft.fft(x)) < 1e-14
    g = load_golden("dct_n64")
    assert rel_err(oracle_dct(g["x"], 10), g["redft10"]) < 1e-14
    assert rel_err(oracle_dct(g["redft10"], 1), g["roundtrip"]) < 1e-14
    assert rel_err(g["roundtrip"], 128 * g["x"]) < 1e-13


def test_callback_processor_matches_builtin():
    g = load_golden("stft_hilbert_n32_l8")
    N = int(g["N"])

    def hilbert(inp, out):
        for i in range(2 * N):
            out[i] = inp[i] if i < N else 0.0
        return 0

    o = OracleSTFT(N, int(g["laps"]), 0, 4, callback=hilbert)
    yr, yi = o.process_block(g["x_re"], g["x_im"])
    b = OracleSTFT(N, int(g["laps"]), 0, 3)
    br, bi = b.process_block(g["x_re"], g["x_im"])
    assert np.array_equal(yr, br) and np.array_equal(yi, bi)
