"""numpy model of the modal band-state pass (hz_fb_modal.h): the band states of a stationary call for
banks whose poles sit on one circle at angles on the 2*pi/L grid.  TEST INFRASTRUCTURE.

A second-order band y = pin (b0 x[t] + b1 x[t-1] + b2 x[t-2]) / (1 + a1 z^-1 + a2 z^-2) with complex
poles p, conj p has the impulse response g[tau] = (p^(tau+1) - conj p^(tau+1)) / (p - conj p), so

    y[t] = Im(p U(t)) / Im p,    U(t) = pin (b0 Z(t) + b1 Z(t-1) + b2 Z(t-2)),
    Z(t) = sum_{tau < K} p^tau x[t - tau],   Z(t-1) = (Z(t) - x[t]) / p      (window of K inputs)

(src/filterbank.h:178-179, the zero-start state over the call's last K samples that the MFMA pass
computes).  For p = p_g e^c with p_g = R_g e^(2 pi i m / L) on the grid and a small correction c
(the coefficients' own rounding off the grid):

    Z(T-1) = G0[m] + c G1[m] + O((c K)^2),
    G_j[m] = sum_{r < L} e^(2 pi i m r / L) F_j[r],   F_j[r] = sum_{tau = r mod L} tau^j R_g^tau x[T-1-tau]

-- one fold of the window into L bins and one length-L DFT for all bands instead of N O K
multiply-adds.  The DFT is four-step, L = 8192 = 64 x 128: r = r1 + 128 r2, m = k1 + 64 k2,

    A[k1][r1] = W^(r1 k1) sum_{r2 < 64} F[r1 + 128 r2] W64^(r2 k1)          (phase 1, per r1)
    G[k1 + 64 k2] = sum_{r1 < 128} W128^(r1 k2) A[k1][r1]                      (phase 2, per k1)

with W = e^(+2 pi i / L).  Bands whose poles nearly coincide (|Im p| tiny: the recipe's Nyquist
band, a double pole at -R) are exceptional: a direct dot product with their own response."""
from __future__ import annotations

import numpy as np

L = 8192


def poles(a1, a2):
    """radius and angle of the upper pole, in long double (the grid corrections are ~1e-13)"""
    a1 = np.asarray(a1, np.longdouble)
    a2 = np.asarray(a2, np.longdouble)
    R = np.sqrt(a2)
    phi = np.arctan2(np.sqrt(np.maximum(a2 - a1 * a1 / 4, 0)), -a1 / 2)
    return R, phi


def plan(a1, a2, K, tol=1e-6, im_min=1e-6):
    """-> (m, c, p, exceptional mask) or None when the bank is not on one circle / grid"""
    R, phi = poles(np.asarray(a1, float), np.asarray(a2, float))
    disc = a1 * a1 - 4 * a2
    exc = (disc >= 0) | (np.sin(phi) < im_min)
    Rg = R[~exc][0] if np.any(~exc) else R[0]
    m = np.rint(phi * L / (2 * np.pi)).astype(int)
    pi = np.longdouble(np.pi) + np.longdouble(1.2246467991473532e-16)   # pi to long double
    c = (np.log(R / Rg) + 1j * (phi - 2 * pi * m / L)).astype(complex)
    R, phi, Rg = R.astype(float), phi.astype(float), float(Rg)
    if np.any(np.abs(c[~exc]) * K > tol) or np.any(m[~exc] <= 0) or np.any(m[~exc] >= L // 2 + 1):
        return None
    p = R * np.exp(1j * phi)
    return m, c, p, exc, Rg


def fold(xw, Rg):
    """F0, F1 over the window xw = x[T-K .. T-1]"""
    K = len(xw)
    tau = np.arange(K)
    xr = xw[::-1]
    w = Rg ** tau.astype(float) * xr
    return np.bincount(tau % L, w, minlength=L), np.bincount(tau % L, tau * w, minlength=L)


def four_step(F):
    """G[m] = sum_r e^(2 pi i m r / L) F[r] by the two phases"""
    r1 = np.arange(128)
    r2 = np.arange(64)
    k1 = np.arange(64)
    k2 = np.arange(128)
    Fm = F.reshape(64, 128)          # [r2][r1]
    W64 = np.exp(2j * np.pi * np.outer(r2, k1) / 64)        # [r2][k1]
    A = (Fm[:, :, None] * W64[:, None, :]).sum(0)           # [r1][k1]
    A = A * np.exp(2j * np.pi * np.outer(r1, k1) / L)       # W^(r1 k1)
    W128 = np.exp(2j * np.pi * np.outer(r1, k2) / 128)      # [r1][k2]
    G = (A[:, :, None] * W128[:, None, :]).sum(0)           # [k1][k2]
    return G.T.reshape(-1)           # index k1 + 64 k2 -> [k2][k1] flattened


def states(xw, fwd, back, pin, exc_direct=True):
    """[N][2] = (y[T-1], y[T-2]) zero-start over the window, by the modal pass"""
    fwd = np.asarray(fwd, float)
    back = np.asarray(back, float)
    N, K = len(fwd), len(xw)
    a1, a2 = back[:, 0], back[:, 1]
    pl = plan(a1, a2, K)
    assert pl is not None
    m, c, p, exc, Rg = pl
    F0, F1 = fold(xw, Rg)
    G0, G1 = four_step(F0), four_step(F1)
    out = np.zeros((N, 2))
    x1, x2, x3 = xw[-1], xw[-2], xw[-3]
    for n in range(N):
        if exc[n]:
            if exc_direct:
                out[n] = direct(xw, fwd[n], back[n], pin[n])
            continue
        Z1 = G0[m[n]] + c[n] * G1[m[n]]
        Z2 = (Z1 - x1) / p[n]
        Z3 = (Z2 - x2) / p[n]
        Z4 = (Z3 - x3) / p[n]
        b0, b1, b2 = fwd[n]
        U1 = pin[n] * (b0 * Z1 + b1 * Z2 + b2 * Z3)
        U2 = pin[n] * (b0 * Z2 + b1 * Z3 + b2 * Z4)
        out[n] = [(p[n] * U1).imag / p[n].imag, (p[n] * U2).imag / p[n].imag]
    return out, exc


def response(f, b, pin, K):
    """r[tau], tau <= K: the band's zero-start response to a unit impulse (long double)"""
    r = np.zeros(K + 1, dtype=np.longdouble)
    y1 = y2 = np.longdouble(0)
    xh = [np.longdouble(0)] * 3
    for t in range(K + 1):
        xh = [np.longdouble(1 if t == 0 else 0)] + xh[:2]
        ff = sum(np.longdouble(f[q]) * xh[q] for q in range(3))
        y = np.longdouble(pin) * ff - np.longdouble(b[0]) * y1 - np.longdouble(b[1]) * y2
        y2, y1 = y1, y
        r[t] = y
    return r


def direct(xw, f, b, pin):
    K = len(xw)
    r = response(f, b, pin, K).astype(float)
    xr = xw[::-1]
    return np.array([np.dot(r[:K], xr), np.dot(r[:K - 1], xr[1:])])
