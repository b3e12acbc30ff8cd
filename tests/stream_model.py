"""stream_model.py -- numpy model of the streaming stationary engine (hz_fb_stream.hip).

Test infrastructure only: restates, lane-free, the algebra the HIP kernels run, so it can be
checked against a direct convolution on the CPU before anything runs on a GPU
(tests/test_stream_model_cpu.py).

The engine: once the bank is stationary its mixdown is out[t] = sum_{tau < K}
h[tau] x[t - tau].  For 1024-sample calls it runs a uniformly partitioned overlap-save
convolution with P = 1024-sample partitions and F = 2048-point real transforms, keeping a
frequency-domain delay line (the spectra of the last K / P windows) on the device.  Each
transform is split column-wise (four-step, n = 32 n1 + n2, k = k1 + 64 k2), so one workgroup per
column k1 (0..32) computes its 32 bins of the new window's spectrum straight from the samples,
its bins of the partition MAC and its column of the inverse transform; the last workgroup to
arrive combines the 33 columns into the block's 1024 outputs (Hermitian symmetry gives columns
33..63).
"""
import numpy as np

P = 1024          # partition / call length
F = 2 * P         # window
C1, C2 = 64, 32   # k = k1 + 64 k2 (k1 < 64, k2 < 32); n = 32 n1 + n2 (n1 < 64, n2 < 32)
COLS = C1 // 2 + 1   # stored columns k1 = 0..32

W64 = np.exp(-2j * np.pi * np.arange(64) / 64)
W32 = np.exp(-2j * np.pi * np.arange(32) / 32)
W2K = np.exp(-2j * np.pi * np.arange(1024) / F)


def col_forward(win, c):
    """X[c + 64 k2], k2 < 32, of the 2048-point DFT of `win` (real), by the column's two stages:
    A[n2] = sum_n1 win[32 n1 + n2] W64^(n1 c); X = sum_n2 W32^(n2 k2) W2048^(n2 c) A[n2]."""
    w = np.asarray(win, dtype=np.float64).reshape(64, 32)          # [n1][n2]
    n1 = np.arange(64)
    A = (W64[(n1 * c) % 64][:, None] * w).sum(axis=0)             # [n2]
    A = A * W2K[(np.arange(32) * c)]
    k2 = np.arange(32)
    return (W32[(np.outer(k2, np.arange(32))) % 32] * A[None, :]).sum(axis=1)


def col_inverse(Y, c):
    """C[n2] = W2048^(-n2 c) sum_k2 Y[k2] W32^(-n2 k2) for column c."""
    n2 = np.arange(32)
    S = (np.conj(W32[np.outer(n2, np.arange(32)) % 32]) * Y[None, :]).sum(axis=1)
    return np.conj(W2K[n2 * c]) * S


def final_stage(Cs):
    """out[32 m + n2] = (window sample 1024 + 32 m + n2 of the inverse) from columns 0..32:
    C0 + (-1)^n1 C32 + 2 Re sum_{c=1}^{31} W64^(-n1 c) C[c]."""
    out = np.zeros(P)
    for m in range(32):
        n1 = 32 + m
        v = Cs[0].real + ((-1) ** n1) * Cs[32].real
        for c in range(1, 32):
            v = v + 2.0 * (np.conj(W64[(n1 * c) % 64]) * Cs[c]).real
        out[32 * m: 32 * m + 32] = v
    return out


class StreamModel:
    """The engine's state: partition spectra HS[p][c] (with 1 / F), the window spectra ring
    ZS[slot][c], the last block's samples; `prime` builds the ring from a history."""

    def __init__(self, h):
        h = np.asarray(h, dtype=np.float64)
        assert len(h) % (8 * P) == 0
        self.K = len(h)
        self.Q = self.K // P
        self.HS = np.zeros((self.Q, COLS, 32), dtype=np.complex128)
        for p in range(self.Q):
            win = np.zeros(F)
            win[:P] = h[p * P:(p + 1) * P] / F
            for c in range(COLS):
                self.HS[p, c] = col_forward(win, c)
        self.ZS = np.zeros((self.Q, COLS, 32), dtype=np.complex128)
        self.head = 0
        self.prev = np.zeros(P)

    def prime(self, hist):
        """hist = the last K inputs: windows b - p (p = 1 .. Q - 1) into slots head - p."""
        hist = np.asarray(hist, dtype=np.float64)
        assert len(hist) == self.K
        for p in range(1, self.Q):
            end = self.K - P * (p - 1)
            win = hist[end - F:end] if end - F >= 0 else np.concatenate([np.zeros(F - end), hist[:end]])
            slot = (self.head - p) % self.Q
            for c in range(COLS):
                self.ZS[slot, c] = col_forward(win, c)
        self.prev = hist[-P:].copy()

    def block(self, x):
        x = np.asarray(x, dtype=np.float64)
        assert len(x) == P
        win = np.concatenate([self.prev, x])
        Cs = []
        for c in range(COLS):
            X = col_forward(win, c)
            self.ZS[self.head, c] = X
            Y = np.zeros(32, dtype=np.complex128)
            for p in range(self.Q):
                Y += self.HS[p, c] * self.ZS[(self.head - p) % self.Q, c]
            Cs.append(col_inverse(Y, c))
        self.head = (self.head + 1) % self.Q
        self.prev = x.copy()
        return final_stage(Cs)
