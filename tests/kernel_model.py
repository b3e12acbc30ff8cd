"""Numpy model of the fb_mix_kernel algorithm (TEST INFRASTRUCTURE).

Mirrors huygens_amd/csrc/hz_filterbank.hip lane for lane: 64 lanes x 16-sample
chunks per 1024-sample tile, zero-state pass, intra-row (16-lane) DPP scan with
zero fill, wave-uniform row carries, chunk-start fix-up with Q[p] = M16^p, gain
smoothing and mixdown.  Used by CPU tests to validate the carry algebra before
it runs on a GPU; it is not the product and not the oracle.
"""
from __future__ import annotations

import numpy as np

L = 16
TILE = 64 * L


def band_record(b, a):
    """Per-band constants: homogeneous responses h[k][j], P[s] = M16^(2^s), Q[p] = M16^p."""
    O = len(a)
    h = np.zeros((O, L))
    for k in range(O):
        yh = np.zeros(O)
        yh[k] = 1.0
        for j in range(L):
            y = -np.dot(a, yh)
            yh = np.roll(yh, 1)
            yh[0] = y
            h[k, j] = y
    M = np.array([[h[c, L - 1 - r] for c in range(O)] for r in range(O)]) if O else np.zeros((0, 0))
    P = [np.linalg.matrix_power(M, 2 ** s) for s in range(6)]
    Q = [np.linalg.matrix_power(M, p) for p in range(L)]
    return h, P, Q


def row_shr(v, d):
    """DPP row_shr:d with bound_ctrl (zero fill) on a [64, ...] lane array."""
    out = np.zeros_like(v)
    for lane in range(64):
        if (lane & 15) >= d:
            out[lane] = v[lane - d]
    return out


def mix_model(fwd, back, sp, sg, pin, gin, x, S0=None, P0=None, G0=None, xhist=None):
    """Mixdown of a whole bank over x, one call, starting from the given state."""
    N, O1 = fwd.shape
    O = O1 - 1
    n = len(x)
    S0 = np.zeros((N, O)) if S0 is None else S0.copy()
    P0 = np.zeros(N) if P0 is None else P0
    G0 = np.zeros(N) if G0 is None else G0
    xhist = np.zeros(O) if xhist is None else xhist
    ntiles = (n + TILE - 1) // TILE
    out = np.zeros(ntiles * TILE)
    lanes = np.arange(64)
    for band in range(N):
        b, a = fwd[band], back[band, :O]
        h, P, Q = band_record(b, a)
        S = S0[band].copy()
        for tile in range(ntiles):
            t0 = tile * TILE
            tc = t0 + L * lanes
            # zero-state pass
            zsr = np.zeros((64, L))
            pre = pin[band] + sp ** tc * (P0[band] - pin[band])
            yh = np.zeros((64, O))
            for j in range(L):
                pre = sp * pre + (1 - sp) * pin[band]
                ff = np.zeros(64)
                for i in range(O + 1):
                    idx = tc + j - i
                    xv = np.where(idx < 0, xhist[np.clip(-idx - 1, 0, max(O - 1, 0))] if O else 0.0,
                                  np.where(idx < n, x[np.clip(idx, 0, n - 1)], 0.0))
                    ff = ff + b[i] * xv
                y = ff * pre - (yh @ a if O else 0.0)
                if O:
                    yh = np.roll(yh, 1, axis=1)
                    yh[:, 0] = y
                zsr[:, j] = y
            if O:
                z = np.stack([zsr[:, L - 1 - k] for k in range(O)], axis=1)  # [64, O]
                for s, d in enumerate((1, 2, 4, 8)):
                    z = z + row_shr(z, d) @ P[s].T
                C = [S.copy()]
                for rw in range(4):
                    C.append(z[16 * rw + 15] + P[4] @ C[rw])
                zs = row_shr(z, 1)
                st = np.stack([zs[lane] + Q[lane & 15] @ C[lane >> 4] for lane in range(64)])
                S = C[4]
            else:
                st = np.zeros((64, 0))
            g = gin[band] + sg ** tc * (G0[band] - gin[band])
            for j in range(L):
                y = zsr[:, j] + (st @ h[:, j] if O else 0.0)
                g = sg * g + (1 - sg) * gin[band]
                out[tc + j] += g * y
    return out[:n]
