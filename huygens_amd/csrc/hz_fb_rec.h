// hz_fb_rec.h -- the chunked LTI band record (hz_fb_lti.hip builds it; the LTI kernels and the
// band-state pass, hz_fb_state.hip, read it).
#pragma once

namespace hz_fbi {

// LTI band record (doubles), built on the host in long double (the chunk transition and its
// powers in double-double).
template <int O, int L>
struct RecL {
    static constexpr int XW = L + O;            // chunk input window x[tc-O .. tc+L-1]
    // scalar block, read by the mix kernel every tile (kept small and contiguous so the
    // 16 bands of a CU stay resident in the scalar cache):
    static constexpr int E0 = 0;                // E[0][m], m < XW (E[k][i] = E[0][i+k], i >= O)
    static constexpr int EH = E0 + XW;          // E[k][i], k, i < O (history taps)
    static constexpr int PS = EH + O * O;       // M^1, M^2, M^4, M^8, M^64
    static constexpr int PSL = PS + 5 * O * O;  // low word of M^64 (double-double, hz_dd.h)
    static constexpr int SC_END = PSL + O * O;
    static constexpr int K = SC_END;            // K[j][k]  j<L, k<O  : homogeneous response
    static constexpr int QC = K + L * O;        // QC[e] = M^e, e <= 64 (M: chunk transition)
    static constexpr int H = QC + 65 * O * O;   // H[d], d<XW : FIR*IIR impulse response
    static constexpr int GE = H + XW;           // GE[i][j], i<O, j<L : F[j][i] (history taps)
    static constexpr int RAW = GE + O * L;
    static constexpr int SIZE = (RAW + 7) & ~7;
};

}  // namespace hz_fbi
