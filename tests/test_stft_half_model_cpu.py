"""numpy model of stft_half4096_kernel's algebra (hz_stft.hip, namespace h4): one real frame as a
half-length complex transform of its even/odd samples, the per-bin split X_k = E_k + W^k O_k, the
gate on |X_k|^2 (staticSTFT.h:99-128 and the gate625 callback), the merge back into the
half-length spectrum and the unnormalised inverse -- checked against the full-length transform
the reference runs (fourier.h:110-147) on the same frame."""
import numpy as np
import pytest


def gate_full(X, p0, p1, keep):
    n = len(X)
    avg = np.sum(np.abs(X)) / n
    thr = p0 * avg * avg
    m2 = X.real ** 2 + X.imag ** 2
    if keep:
        return np.where(m2 > thr, X, 0.0)
    return np.where(m2 < thr, X * p1, X)


def half_path(frame, p0, p1, keep):
    N = len(frame)
    M = N // 2
    W = np.exp(-2j * np.pi * np.arange(N) / N)
    Z = np.fft.fft(frame[0::2] + 1j * frame[1::2])
    X = np.zeros(N, complex)
    k = np.arange(1, M // 2)
    m = M - k
    E = (Z[k] + np.conj(Z[m])) / 2
    O = (Z[k] - np.conj(Z[m])) / 2j
    t = W[k] * O
    X[k] = E + t
    X[m] = np.conj(E - t)
    X[0] = Z[0].real + Z[0].imag
    X[M] = Z[0].real - Z[0].imag
    X[M // 2] = np.conj(Z[M // 2])
    X[M + 1:] = np.conj(X[1:M][::-1])
    Xg = gate_full(X, p0, p1, keep)
    Zpp = np.zeros(M, complex)
    A = Xg[k]
    B = np.conj(Xg[m])
    S, D = A + B, A - B
    V = 1j * np.conj(W[k]) * D
    Zpp[k] = S + V
    Zpp[m] = np.conj(S - V)
    Zpp[0] = (Xg[0].real + Xg[M].real) + 1j * (Xg[0].real - Xg[M].real)
    Zpp[M // 2] = 2 * np.conj(Xg[M // 2])
    z = np.fft.ifft(Zpp) * M
    y = np.empty(N)
    y[0::2] = z.real
    y[1::2] = z.imag
    return X, y


@pytest.mark.parametrize("keep", [False, True])
@pytest.mark.parametrize("N", [64, 4096])
def test_half_length_split_gate_merge(N, keep):
    rng = np.random.default_rng(N + keep)
    w = 0.5 * (1 - np.cos(2 * np.pi * np.arange(N) / N))
    t = np.arange(N) / 48000.0
    x = 0.1 * rng.standard_normal(N) + 0.5 * np.sin(2 * np.pi * 440 * t)
    frame = w * x
    p0, p1 = (6.25, 0.0) if keep else (100.0, 0.1)
    X_ref = np.fft.fft(frame)
    y_ref = np.real(np.fft.ifft(gate_full(X_ref, p0, p1, keep))) * N
    X, y = half_path(frame, p0, p1, keep)
    assert np.max(np.abs(X - X_ref)) <= 1e-12 * np.max(np.abs(X_ref))
    assert np.max(np.abs(y - y_ref)) <= 1e-12 * np.max(np.abs(y_ref))
