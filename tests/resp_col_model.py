"""numpy model of the stationary engine's column-split convolution (hz_fb_resp.hip, column path):
the schedule and index algebra the kernels follow, checked against a direct convolution by
tests/test_resp_col_model_cpu.py before anything runs on a GPU.  TEST INFRASTRUCTURE.

Overlap-save with P = 2048-sample partitions and F = 4096-point real transforms, each transform
split four-step (F = 64 x 64):
  forward   window sample n = 64 n1 + n2, bin k = c + 64 k2 (column c):
            D_s^c[n2] = sum_{m < 32} u[s P + 64 m + n2] W64^(m c)           (segment s = u[sP, sP + P))
            A_j^c     = D_j^c + (-1)^c D_{j+1}^c                            (window j = segments j, j+1)
            Z_j[c + 64 k2] = sum_{n2} W64^(n2 k2) W4096^(n2 c) A_j^c[n2]
  unit      columns c0 + 16 i (i < 4) share their loads: D^{c0 + 16 i} = sum_{r < 4} W4^(r i) P_r,
            P_r = sum_{m = r mod 4} u_m W64^(m c0)   (a radix-4 step over the row index)
  MAC       Y_b = sum_{p < Q} H_p Z_{b + Q - 1 - p} per bin                 (H_p = FFT(h_p) / F)
  inverse   output sample n = n1 + 64 n2:
            T_b^c[n1] = W4096^(-n1 c) sum_{k2} W64^(-n1 k2) Y_b[c + 64 k2]   (per column)
            x_b[n1 + 64 n2] = sum_{c < 64} W64^(-n2 c) T_b^c[n1],  T^(64 - c) = conj T^c
            out[b P + n1 + 64 (n2 - 32)] = x_b[n1 + 64 n2] for n2 >= 32      (the window's last P)
Only columns 0..32 are computed (the input is real): the units are c0 = 1..7 (columns c0, c0 + 16
and c0 + 32 = conj of 32 - c0, c0 + 48 = conj of 16 - c0), c0 = 0 (0, 16, 32) and c0 = 8 (8, 24)."""
from __future__ import annotations

import numpy as np

P = 2048
F = 2 * P


def w(n, k):
    return np.exp(-2j * np.pi * k / n)


def units():
    """unit -> (c0, stored columns): the 33 columns 0..32 up to conjugation"""
    u = [(c0, [c0, c0 + 16, c0 + 32, c0 + 48]) for c0 in range(1, 8)]
    u.append((0, [0, 16, 32]))
    u.append((8, [8, 24]))
    return u


def stage1_unit(seg, c0):
    """the four columns c0 + 16 i of one segment (64 n2 each) from one pass over its rows"""
    U = seg.reshape(32, 64)                       # [m][n2]
    m = np.arange(32)
    Pr = np.zeros((4, 64), complex)
    for r in range(4):
        rows = m[m % 4 == r]
        Pr[r] = (U[rows] * w(64, rows * c0)[:, None]).sum(0)
    return np.array([sum(w(4, r * i) * Pr[r] for r in range(4)) for i in range(4)])   # [i][n2]


def column_forward(segs, c, D):
    """Z_j[c + 64 k2] for every window j, from the segments' D^c"""
    sgn = -1.0 if c % 2 else 1.0
    n2 = np.arange(64)
    A = D[:-1] + sgn * D[1:]                      # [j][n2]
    return np.fft.fft(A * w(F, n2 * c)[None, :], axis=1)   # sum_n2 W64^(n2 k2) (...)


def convolve(u, h, K, n):
    """out[t] = sum_{tau < K} h[tau] u[K + t - tau], t < n, by the column schedule"""
    Q, B = K // P, -(-n // P)
    nseg = Q + B
    uu = np.zeros(nseg * P)
    uu[:min(len(u), nseg * P)] = u[:nseg * P]
    segs = uu.reshape(nseg, P)
    Hf = np.array([np.fft.fft(np.concatenate([h[p * P:(p + 1) * P], np.zeros(P)])) / F for p in range(Q)])
    cols = {}
    for c0, cl in units():
        Ds = np.array([stage1_unit(s, c0) for s in segs])          # [s][i][n2]
        for i, c in enumerate([c0 + 16 * k for k in range(4)]):
            if c in cl:
                cols[c] = column_forward(segs, c, Ds[:, i, :])      # [j][k2]
    assert sorted(cols) == sorted(set(c for _, cl in units() for c in cl))
    out = np.zeros(B * P)
    n1 = np.arange(64)
    for b in range(B):
        T = {}
        for c, Z in cols.items():
            Yc = sum(Hf[p, c + 64 * np.arange(64)] * Z[b + Q - 1 - p] for p in range(Q))
            T[c] = w(F, -n1 * c) * np.fft.ifft(Yc) * 64             # sum_k2 W64^(-n1 k2) Y
        V = np.zeros((64, 64), complex)                              # [c][n1]
        for c in range(64):
            V[c] = T[c] if c in T else np.conj(T[64 - c])
        x = np.fft.ifft(V, axis=0) * 64                              # [n2][n1]
        out[b * P:(b + 1) * P] = x[32:].real.reshape(-1)             # n1 + 64 (n2 - 32)
    return out[:n]


def direct(u, h, K, n):
    y = np.convolve(u[:K + n], h[:K])
    return y[K:K + n]
