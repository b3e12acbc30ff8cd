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
    """The engine's state and its pipelined schedule (hz_fb_stream.hip): launch b outputs
        y_b = head_b + tail_b,   head_b[t] = sum_{tau < P} h[tau] x[t - tau]  (direct),
        tail_b = last P samples of IFFT(Y_b),  Y_b = sum_{p >= 1} H_p Z_{b-p},
    where the tail's inverse columns C_b were computed by launch b - 1:
        Y_{b+1} = H_1 Z_b + H_2 Z_{b-1} + R_{b+1},   R_{b+2} = sum_{p >= 3} H_p Z_{b+2-p}
    (R computed one launch ahead from the ring of window spectra).  Within a launch the three
    roles (outputs, transform columns, MAC columns) share no data."""

    def __init__(self, h):
        h = np.asarray(h, dtype=np.float64)
        assert len(h) % (8 * P) == 0
        self.h = h
        self.K = len(h)
        self.Q = self.K // P
        self.HS = np.zeros((self.Q, COLS, 32), dtype=np.complex128)
        for p in range(self.Q):
            win = np.zeros(F)
            win[:P] = h[p * P:(p + 1) * P] / F
            for c in range(COLS):
                self.HS[p, c] = col_forward(win, c)
        self.ZS = np.zeros((self.Q, COLS, 32), dtype=np.complex128)
        self.head = 0            # slot of the next window spectrum Z_b
        self.prev = np.zeros(P)
        self.C = None            # inverse columns of the next block's tail
        self.R = None            # R_{b+1}

    def _z(self, p):
        """Z_{b-p} (p >= 1) from the ring, b = the next block"""
        return self.ZS[(self.head - p) % self.Q]

    def prime(self, hist):
        """hist = the last K inputs: windows b - p (p = 1 .. Q - 1) into slots head - p, then the
        first block's tail columns C_b and R_{b+1}."""
        hist = np.asarray(hist, dtype=np.float64)
        assert len(hist) == self.K
        for p in range(1, self.Q):
            end = self.K - P * (p - 1)
            win = hist[end - F:end] if end - F >= 0 else np.concatenate([np.zeros(F - end), hist[:end]])
            slot = (self.head - p) % self.Q
            for c in range(COLS):
                self.ZS[slot, c] = col_forward(win, c)
        self.prev = hist[-P:].copy()
        Y = sum(self.HS[p] * self._z(p) for p in range(1, self.Q))
        self.C = [col_inverse(Y[c], c) for c in range(COLS)]
        # R_{b+1} = sum_{p >= 3} H_p Z_{b+1-p}: Z_{b+1-p} = ring entry p - 1 back
        self.R = sum(self.HS[p] * self._z(p - 1) for p in range(3, self.Q))

    def block(self, x):
        x = np.asarray(x, dtype=np.float64)
        assert len(x) == P
        # outputs: head (direct, taps 0 .. P-1) + tail (columns from the previous launch)
        full = np.concatenate([self.prev, x])
        head = np.array([np.dot(self.h[:P], full[P + i - P + 1:P + i + 1][::-1]) for i in range(P)])
        y = head + final_stage(self.C)
        # transform columns: Z_b, then C_{b+1} from Y_{b+1} = H_1 Z_b + H_2 Z_{b-1} + R_{b+1}
        Zb = np.array([col_forward(full, c) for c in range(COLS)])
        Zb1 = self._z(1).copy()
        Y1 = self.HS[1] * Zb + self.HS[2] * Zb1 + self.R
        C1 = [col_inverse(Y1[c], c) for c in range(COLS)]
        # MAC columns: R_{b+2} = sum_{p >= 3} H_p Z_{b+2-p} (Z_{b-1} and older)
        R2 = sum(self.HS[p] * self._z(p - 2) for p in range(3, self.Q))
        self.ZS[self.head] = Zb
        self.head = (self.head + 1) % self.Q
        self.C, self.R = C1, R2
        self.prev = x.copy()
        return y
