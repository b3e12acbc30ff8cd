"""Numpy model of the converged ("LTI") Filterbank engine (TEST INFRASTRUCTURE).

Mirrors huygens_amd/csrc/hz_fb_lti.hip step for step on converged smoothers
(pre = pin, gain = gin): per band, the chunk zero-state end states z = pin E x (E rows of
the chunk's zero-state response; on the device a (64 x XW) x (XW x 16 O) FP64 MFMA per
band group), the 64-lane inclusive prefix of s' = M s + z with the device's DPP schedule
(row_shr 1, 2, 4, 8 with M^(2^s), row_bcast:15 into rows 1 and 3 with M^(p+1),
row_bcast:31 into rows 2 and 3 with M^(l-31)), the chunk start states
st = Z(l-1) + M^l S (wave_shr:1), the tile end state Z(63) + M^64 S, the group correction
sum_band K[j] gin st (the device's mix MFMA), and the bank-wide zero-state term
Fmix = sum_band gin pin F applied by the reduce kernel.  It validates the algebra on the
CPU; it is neither the product nor the oracle.
"""
from __future__ import annotations

import numpy as np


def band_lti_record(b, a, L):
    """F[j][i] (zero-state chunk response to x[tc-O+i]), K[j][k] (homogeneous response to
    y[tc-1-k] = 1) and M (chunk transition of the state (y[t-1], ..., y[t-O]))."""
    O = len(a)
    XW = L + O
    F = np.zeros((L, XW))
    for i in range(XW):
        x = np.zeros(XW)
        x[i] = 1.0
        y = np.zeros(L + O)  # y[O + j] = sample j of the chunk, zero state
        for j in range(L):
            u = sum(b[q] * x[O + j - q] for q in range(O + 1))
            y[O + j] = u - sum(a[k] * y[O + j - 1 - k] for k in range(O))
        F[:, i] = y[O:]
    K = np.zeros((L, O))
    for k in range(O):
        y = np.zeros(L + O)
        y[O - 1 - k] = 1.0
        for j in range(L):
            y[O + j] = -sum(a[q] * y[O + j - 1 - q] for q in range(O))
        K[:, k] = y[O:]
    M = np.array([[K[L - 1 - r, c] for c in range(O)] for r in range(O)])
    return F, K, M


def _shift(v, src):
    """lane l <- v[src(l)] (None -> 0): the DPP moves with bound_ctrl / row masks."""
    out = np.zeros_like(v)
    for lane in range(64):
        s = src(lane)
        if s is not None:
            out[lane] = v[s]
    return out


def scan64(z, M):
    """Inclusive prefix over 64 chunk lanes with the device's DPP schedule. z: [64, O]."""
    z = z.copy()
    for s in range(4):
        d = 1 << s
        nb = _shift(z, lambda l: l - d if (l & 15) >= d else None)
        z = z + nb @ np.linalg.matrix_power(M, d).T
    nb = _shift(z, lambda l: (l & ~15) - 1 if (l >> 4) in (1, 3) else None)          # row_bcast:15
    Qa = np.stack([np.linalg.matrix_power(M, (l & 15) + 1) for l in range(64)])
    z = z + np.einsum("lrc,lc->lr", Qa, nb)
    nb = _shift(z, lambda l: 31 if l >= 32 else None)                                   # row_bcast:31
    Qb = np.stack([np.linalg.matrix_power(M, max(l - 31, 0)) for l in range(64)])
    z = z + np.einsum("lrc,lc->lr", Qb, nb)
    return z


def lti_mix_model(fwd, back, pin, gin, x, L=32, S0=None, xhist=None):
    """Mixdown of a converged bank over x (len(x) a multiple of L), one call."""
    N, O1 = fwd.shape
    O = O1 - 1
    n = len(x)
    assert n % L == 0
    T = 64 * L
    S0 = np.zeros((N, O)) if S0 is None else S0
    xhist = np.zeros(O) if xhist is None else xhist  # x[-1-k]
    ntiles = (n + T - 1) // T
    xp = np.concatenate([xhist[::-1], x, np.zeros(ntiles * T - n)])  # xp[O + t] = x[t]
    out = np.zeros(ntiles * T)
    Fmix = np.zeros((L, L + O))
    for band in range(N):
        F, K, M = band_lti_record(fwd[band], back[band, :O], L)
        Fmix += gin[band] * pin[band] * F
        S = S0[band].copy()
        for tile in range(ntiles):
            t0 = tile * T
            win = np.stack([xp[t0 + c * L: t0 + c * L + L + O] for c in range(64)])   # [64, XW]
            z = pin[band] * win @ F[L - 1 - np.arange(O)].T                             # [64, O]
            Z = scan64(z, M)
            Zs = _shift(Z, lambda l: l - 1 if l > 0 else None)                          # wave_shr:1
            Qc = np.stack([np.linalg.matrix_power(M, l) for l in range(64)])
            st = Zs + np.einsum("lrc,c->lr", Qc, S)
            S = Z[63] + np.linalg.matrix_power(M, 64) @ S
            out[t0: t0 + T] += (gin[band] * st @ K.T).reshape(-1)                       # [64, L]
    for c in range(ntiles * 64):
        out[c * L: c * L + L] += Fmix @ xp[c * L: c * L + L + O]
    return out[:n]
