"""CPU check of the gain-transient algebra the streaming engine uses for mix() while streaming
(hz_fb_stream.hip fb_stream_gain_setter): with every band's output y_n fixed by its (converged)
pre-amp, and the gain smoothers g_n(t+1) = (1 - s) gin_n + s g_n(t) (src/filterbank.h:173) sharing s,

    sum_n g_n(t) y_n(t) = sum_n gin_n y_n(t) + s^(t - dref) sum_n D_n y_n(t),

and per setter (bands C, new targets gin'): h += sum_C (gin' - gin) r_n, h_D = s^(t_c - dref) h_D -
sum_C (gin' - gin) r_n, dref = t_c.  Here the y_n are the band outputs themselves (the engine
convolves x with h and h_D instead), so the check is the bookkeeping of D, the rebase and the
per-sample factor, exactly as the kernels apply them."""
import numpy as np

from golden.spec_numpy import relaxation, resonant_coefficients


def test_transient_decomposition_matches_smoothed_gains():
    from scipy.signal import lfilter
    rng = np.random.default_rng(3)
    N, T = 12, 6000
    fwd, back = resonant_coefficients(N, 0.99, 1.0)
    x = rng.uniform(-1, 1, T)
    y = np.stack([lfilter(fwd[n], np.r_[1.0, back[n]], x) for n in range(N)])   # pre = pin = 1
    s = relaxation(0.02)
    gin = np.ones(N)
    g = gin.copy()                     # converged gains at t = 0
    setters = {500: [(2, 0.4), (7, 1.6)], 1900: [(2, 1.1), (3, 0.2)], 2000: [(11, 0.0)], 4100: [(0, 2.0)]}
    # reference: the smoothed gains sample by sample
    ref = np.zeros(T)
    gg = g.copy()
    tg = gin.copy()
    for t in range(T):
        for b, v in setters.get(t, []):
            tg[b] = v
        gg = (1 - s) * tg + s * gg     # compute(): smoothers first, then the output
        ref[t] = np.dot(gg, y[:, t])
    # the engine's bookkeeping: per-band "responses" are the band outputs themselves here
    base = np.dot(gin, y)              # h (targets), applied to x: sum_n gin_n y_n
    dres = np.zeros(T)                 # h_D applied to x
    dref, gin_b = 0, gin.copy()
    out = np.zeros(T)
    for t in range(T):
        if t in setters:
            delta = np.zeros(N)
            for b, v in setters[t]:
                delta[b] = v - gin_b[b]
            gin_b = gin_b + delta
            d = np.dot(delta, y)
            base = base + d
            dres = s ** (t - dref) * dres - d
            dref = t
        # the reference applies the smoother before the sample's output: the first sample after a
        # setter already carries one step, so the transient's exponent counts from dref - 1
        out[t] = base[t] + s ** (t - dref + 1) * dres[t]   # (dres is zero before the first setter)
    assert np.max(np.abs(out - ref)) <= 1e-12 * np.max(np.abs(ref))
