// hz_fb_col.h -- the stationary engine's column-split convolution (included by hz_fb_resp.hip).
//
// The same overlap-save convolution as the three-kernel path (P = 2048-sample partitions, F =
// 4096-point real transforms; hz_fb_resp.hip), with every transform split four-step, F = 64 x 64,
// so that the window spectra never leave the workgroup that computes them
// (tests/resp_col_model.py restates this schedule and checks it against a direct convolution):
//
//   resp_col_kernel   workgroup = (unit, range of kWB output blocks).  A unit is four columns
//                     c0 + 16 i (bins k = c + 64 k2) sharing one pass over the samples:
//                       stage 1  D_s^c[n2] = sum_{m<32} u[sP + 64 m + n2] W64^(mc) for the segments
//                                s of the range and its Q-partition halo (a radix-4 step over m
//                                gives the four columns from one set of loads), into LDS;
//                       stage 3  Z_j = FFT64_n2(W4096^(n2 c) (D_j + (-1)^c D_{j+1})) per window,
//                                8 x 8 points (radix-8 in registers, transposed through the
//                                window's own LDS row), eight windows per wave (wave i = column i);
//                       MAC      Y_b = sum_p H_p Z_{b+Q-1-p} per bin (lane), Z in a register ring;
//                       inverse  T_b^c[n1] = W4096^(-n1 c) IFFT64_k2(Y_b) -> HBM, [b][slot][n1]
//                                (the same 8 x 8 scheme, eight blocks per wave).
//   resp_comb_kernel  one workgroup per output block: x[n1 + 64 n2] = sum_c W64^(-n2 c) T^c[n1]
//                     (T^(64-c) = conj T^c), the block's samples n2 >= 32; its threads also do
//                     the history / smoother / x-history upkeep, and the band-state pass rides in
//                     it as extra workgroups (as in resp_inv_kernel).
// Units: c0 = 1..7 hold columns c0, c0+16, c0+32 (= conj of 32-c0), c0+48 (= conj of 16-c0);
// c0 = 0 holds 0, 16, 32 and c0 = 8 holds 8, 24: the 33 columns 0..32 up to conjugation.
#pragma once

namespace hz_col {

constexpr int kP = 2048;
constexpr int kUnits = 9;
constexpr int kSlots = 4 * kUnits;   // H / T slots: 4u + i (unused slots of units 7, 8 never read)
constexpr int kWB = 10;              // output blocks per range (B = 235 -> 24 ranges, 3 per XCD)

__host__ __device__ constexpr int unit_c0(int u) { return u < 7 ? u + 1 : (u == 7 ? 0 : 8); }
__host__ __device__ constexpr int unit_ncol(int u) { return u < 7 ? 4 : (u == 7 ? 3 : 2); }

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {   // conj(a) b
    return make_double2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ int brev6(int l) { return (int)(__builtin_bitreverse32((unsigned)l) >> 26); }

// The value of lane l ^ S, without LDS: DPP within 16-lane rows (S = 1, 2: quad_perm; 4: two
// row rotations; 8: row_ror 8), v_permlane16/32_swap across rows (gfx950)
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}
template <int S>
__device__ __forceinline__ unsigned xor_u(unsigned v, int l) {
    if constexpr (S == 1) return dpp_u<0xB1>(v);                      // quad_perm [1,0,3,2]
    else if constexpr (S == 2) return dpp_u<0x4E>(v);                 // quad_perm [2,3,0,1]
    else if constexpr (S == 4) {   // row_ror 4 / 12, both for every lane (a DPP read of a lane
        // a branch has switched off returns 0), then a bitwise select
        const unsigned lo = dpp_u<0x124>(v), hi = dpp_u<0x12C>(v);
        const unsigned m = 0u - (unsigned)((l >> 2) & 1);
        return (lo & m) | (hi & ~m);
    }
    else if constexpr (S == 8) return dpp_u<0x128>(v);                // row_ror 8
    else if constexpr (S == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (l & 16) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (l & 32) ? r[0] : r[1];
    }
}
template <int S>
__device__ __forceinline__ double xor_d(double v, int l) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = xor_u<S>((unsigned)b, l), hi = xor_u<S>((unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int S>
__device__ __forceinline__ double2 xor2(double2 v, int l) {
    return make_double2(xor_d<S>(v.x, l), xor_d<S>(v.y, l));
}

// 64-point transforms across a wave's lanes, G independent transforms in lockstep (their
// exchanges and FP64 chains interleave).  tw4k = W4096^k (k < 4096, long double on the host).
struct Fft64 {
    double2 w[6];   // stage q (span s = 32 >> q): W64^((l & (s-1)) 32 / s)
    __device__ __forceinline__ void init(const double2* __restrict__ tw4k, int l) {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const int s = 32 >> q;
            w[q] = tw4k[64 * ((l & (s - 1)) * (32 / s))];
        }
    }
    template <int S, int G>
    __device__ __forceinline__ void fwd_stage(double2 (&v)[G], int l, const double2& wq) const {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double2 o = xor2<S>(v[g], l);
            v[g] = (l & S) ? cmul(csub(o, v[g]), wq) : cadd(v[g], o);
        }
    }
    template <int S, int G>
    __device__ __forceinline__ void inv_stage(double2 (&v)[G], int l, const double2& wq) const {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double2 o = xor2<S>(v[g], l);
            v[g] = (l & S) ? csub(o, cmulc(wq, v[g])) : cadd(v[g], cmulc(wq, o));
        }
    }
    // forward (W64 = e^{-2 pi i / 64}), decimation in frequency: lane n in, lane l out holds X[brev6(l)]
    template <int G>
    __device__ __forceinline__ void fwd(double2 (&v)[G], int l) const {
        fwd_stage<32>(v, l, w[0]);
        fwd_stage<16>(v, l, w[1]);
        fwd_stage<8>(v, l, w[2]);
        fwd_stage<4>(v, l, w[3]);
        fwd_stage<2>(v, l, w[4]);
        fwd_stage<1>(v, l, w[5]);
    }
    // inverse (unnormalised), decimation in time: lane l holds Y[brev6(l)] in, lane n out
    template <int G>
    __device__ __forceinline__ void inv(double2 (&v)[G], int l) const {
        inv_stage<1>(v, l, w[5]);
        inv_stage<2>(v, l, w[4]);
        inv_stage<4>(v, l, w[3]);
        inv_stage<8>(v, l, w[2]);
        inv_stage<16>(v, l, w[1]);
        inv_stage<32>(v, l, w[0]);
    }
};

struct ColArgs {
    const double* hist;   // [K] the K inputs before the call
    const double* x;      // [n]
    long K, off, n_out;   // horizon; the launch's first output sample and count (time shards)
    int Q, B, NR;         // partitions, output blocks, ranges of kWB blocks
    const double2* tw4k;  // [4096] W4096^k
    const double2* Hc;    // [kSlots][Q][64] H_p at bin c + 64 l, / F
    double2* T;           // [B][kSlots][64] inverse columns
};

// Rows are padded to kRow complex so that the transposed accesses of the radix-8 transforms
// spread over the LDS banks
constexpr int kRow = 65;
template <int QP>
struct ColLds {
    double2 z[4][kWB + QP][kRow];   // D of the segments, then Z of the windows, per column
    double2 tn[4][64];              // W4096^(n c), n < 64, per column
    double2 w64[64];                // W64^(r k), [8 r + k]
};

// 8-point DFT in registers, natural order in and out (radix-2 decimation in time); INV: W8 -> conj
template <bool INV>
__device__ __forceinline__ void dft8(double2 (&x)[8]) {
    constexpr double h = 0.70710678118654752440;
    double2 a[8] = {x[0], x[4], x[2], x[6], x[1], x[5], x[3], x[7]};
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        const double2 p = a[i], q = a[i + 1];
        a[i] = cadd(p, q);
        a[i + 1] = csub(p, q);
    }
#pragma unroll
    for (int i = 0; i < 8; i += 4) {
        // span 2: twiddles 1, W4 (= -i forward, +i inverse)
        double2 p = a[i], q = a[i + 2];
        a[i] = cadd(p, q);
        a[i + 2] = csub(p, q);
        p = a[i + 1];
        q = INV ? make_double2(-a[i + 3].y, a[i + 3].x) : make_double2(a[i + 3].y, -a[i + 3].x);
        a[i + 1] = cadd(p, q);
        a[i + 3] = csub(p, q);
    }
    // span 4: twiddles W8^i, i < 4
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double2 q = a[i + 4];
        if (i == 1) q = INV ? make_double2(h * (q.x - q.y), h * (q.x + q.y)) : make_double2(h * (q.x + q.y), h * (q.y - q.x));
        if (i == 2) q = INV ? make_double2(-q.y, q.x) : make_double2(q.y, -q.x);
        if (i == 3) q = INV ? make_double2(-h * (q.x + q.y), h * (q.x - q.y)) : make_double2(h * (q.y - q.x), -h * (q.x + q.y));
        const double2 p = a[i];
        a[i] = cadd(p, q);
        a[i + 4] = csub(p, q);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = a[i];
}

// u = [hist | x | 0 ...] indexed from the launch's first output sample: one segment's source
__device__ __forceinline__ const double* col_segment(const ColArgs& a, long s, long* lim) {
    const long m0 = s * kP + a.off;
    if (m0 < a.K) {   // K and off are multiples of P: the segment lies in the history
        *lim = kP;
        return a.hist + m0;
    }
    *lim = a.off + a.n_out - (m0 - a.K);
    return a.x + (m0 - a.K);
}

#ifdef HZ_DIAG_STAMPS
// (diagnostic builds) per column workgroup, wave 0: start, stage 1 done, stage 3 done, MACs done, end
__device__ long long g_cdiag[1024][5];
#define HZ_COL_STAMP(i)                                                                                   \
    do {                                                                                                  \
        if (t == 0 && blockIdx.x < 1024) g_cdiag[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();       \
    } while (0)
#else
#define HZ_COL_STAMP(i) ((void)0)
#endif

// A 64-point transform of eight rows of one column at once, in place (rows row0 .. row0 + 7, the
// last `valid` of them kept): lane (g, r) = (l >> 3, l & 7) holds the row g + row0's points r + 8 m
// (m < 8, already loaded and twiddled) -> 8-point DFT over m -> x W64^(+-r k1) -> transpose through
// the rows themselves -> 8-point DFT over r; out[k1 + 8 k2] for lane (g, k1), k2 < 8 (natural order)
template <bool INV>
__device__ __forceinline__ void col_fft8x8(double2 (&v)[8], double2 (*rows)[kRow], int row0, int valid, int l,
                                           const double2* __restrict__ w64) {
    const int g = l >> 3, r = l & 7;
    dft8<INV>(v);
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1) {
        const double2 w = w64[8 * r + k1];   // W64^(r k1)
        v[k1] = INV ? cmulc(w, v[k1]) : cmul(v[k1], w);
    }
    const bool live = g < valid;
    if (live) {
#pragma unroll
        for (int k1 = 0; k1 < 8; ++k1) rows[row0 + g][8 * r + k1] = v[k1];
    }
    // (the wave's own LDS writes land before its reads: LDS instructions of a wave run in order)
    if (live) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = rows[row0 + g][8 * q + r];   // lane (g, k1 = r)
    }
    dft8<INV>(v);
}

// kColThreads threads = 8 waves: stage 1 on all eight (more loads in flight), stage 3 and the
// inverse on waves w and w + 4 of column w (alternate groups of eight rows), the MAC on waves 0-3
constexpr int kColThreads = 512;

template <int QP>
__device__ __forceinline__ void col_group(const ColArgs& a, int u, int r, ColLds<QP>& L) {
    const int t = threadIdx.x, l = t & 63, wv = t >> 6;
    HZ_COL_STAMP(0);
    const int c0 = unit_c0(u), ncol = unit_ncol(u);
    const int b0 = r * kWB;
    const int w = wv & 3, half = wv >> 2;   // column, and which of its two waves
    const int g8 = l >> 3, r8 = l & 7;
    // stage-1 twiddles (lane-uniform): W16^(q c0) (rows m = 4q + rr, q < 8) and W64^(rr c0); the
    // later phases' tables into LDS now (visible after stage 1's barrier)
    double2 t16[8], t64[4];
#pragma unroll
    for (int q = 0; q < 8; ++q) t16[q] = a.tw4k[256 * ((q * c0) & 15)];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) t64[rr] = a.tw4k[64 * ((rr * c0) & 63)];
    if (t < 256) L.tn[t >> 6][l] = a.tw4k[l * (c0 + 16 * (t >> 6))];
    else if (t < 320) L.w64[t - 256] = a.tw4k[64 * ((t - 256) >> 3) * ((t - 256) & 7)];
    // ---- stage 1: segments s_l = wv, wv + 8, ... of [0, kWB + QP), the next one's loads in flight
    constexpr int NS = kWB + QP;
    double cur[32], nxt[32];
    auto load = [&](int sl, double (&v)[32]) {
        long lim;
        const double* src = col_segment(a, (long)b0 + sl, &lim);
#pragma unroll
        for (int m = 0; m < 32; ++m) {
            const int i = 64 * m + l;
            v[m] = i < lim ? src[i] : 0.0;
        }
    };
    if (wv < NS) load(wv, nxt);
    for (int sl = wv; sl < NS; sl += 8) {
#pragma unroll
        for (int m = 0; m < 32; ++m) cur[m] = nxt[m];
        if (sl + 8 < NS) load(sl + 8, nxt);
        double2 P[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            double2 acc = make_double2(0.0, 0.0);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                acc.x = fma(cur[4 * q + rr], t16[q].x, acc.x);
                acc.y = fma(cur[4 * q + rr], t16[q].y, acc.y);
            }
            P[rr] = cmul(acc, t64[rr]);
        }
        // D^{c0 + 16 i} = sum_rr W4^(rr i) P_rr, W4 = -i
        const double2 s02 = cadd(P[0], P[2]), d02 = csub(P[0], P[2]);
        const double2 s13 = cadd(P[1], P[3]), d13 = csub(P[1], P[3]);
        L.z[0][sl][l] = cadd(s02, s13);
        L.z[1][sl][l] = make_double2(d02.x + d13.y, d02.y - d13.x);   // d02 - i d13
        L.z[2][sl][l] = csub(s02, s13);
        if (ncol > 3) L.z[3][sl][l] = make_double2(d02.x - d13.y, d02.y + d13.x);   // d02 + i d13
    }
    __syncthreads();
    HZ_COL_STAMP(1);
    const bool colw = w < ncol;   // (units 7, 8: fewer columns than waves)
    double2(*rows)[kRow] = L.z[w];
    // ---- stage 3, in place: window j = segments j, j + 1; eight windows per transform, rounds of
    // two groups (wave w: group 2k, wave w + 4: group 2k + 1).  A group reads its eight rows and the
    // next group's first row and then writes its own eight rows: the round's reads all precede its
    // writes (a barrier between), and the next round's reads touch no row this round writes.
    {
        constexpr int NW = NS - 1, NG = (NW + 7) / 8;
        const double sg = (c0 & 1) ? -1.0 : 1.0;
        for (int k = 0; k < (NG + 1) / 2; ++k) {
            const int j0 = 8 * (2 * k + half);
            const bool act = colw && j0 < NW;
            const int valid = act ? min(8, NW - j0) : 0;
            double2 v[8];
            if (act) {
                const int j = min(j0 + g8, NW - 1);
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const double2 d0 = rows[j][r8 + 8 * m], d1 = rows[j + 1][r8 + 8 * m];
                    v[m] = cmul(make_double2(fma(sg, d1.x, d0.x), fma(sg, d1.y, d0.y)), L.tn[w][r8 + 8 * m]);
                }
            }
            __syncthreads();
            if (act) {
                col_fft8x8<false>(v, rows, j0, valid, l, L.w64);
                if (g8 < valid) {
#pragma unroll
                    for (int k2 = 0; k2 < 8; ++k2) rows[j0 + g8][r8 + 8 * k2] = v[k2];   // bin r + 8 k2
                }
            }
        }
    }
    __syncthreads();
    HZ_COL_STAMP(2);
    // ---- MAC (waves 0-3): Y_b = sum_p H_p Z_{b+Q-1-p} for the range's kWB blocks (lane = bin),
    // window b + t in ring slot (b + t) % kWB at step t = Q - 1 - p; Y into rows 0 .. kWB - 1
    if (colw && half == 0) {
        const double2* hc = a.Hc + ((long)(4 * u + w) * a.Q) * 64 + l;
        double2 Y[kWB], ring[kWB];
#pragma unroll
        for (int b = 0; b < kWB; ++b) {
            Y[b] = make_double2(0.0, 0.0);
            ring[b] = rows[b][l];
        }
#pragma unroll
        for (int ts = 0; ts < QP; ++ts) {
            const double2 h = hc[(long)(QP - 1 - ts) * 64];
#pragma unroll
            for (int b = 0; b < kWB; ++b) {
                const double2 z = ring[(b + ts) % kWB];
                Y[b].x = fma(h.x, z.x, fma(-h.y, z.y, Y[b].x));
                Y[b].y = fma(h.x, z.y, fma(h.y, z.x, Y[b].y));
            }
            if (ts + 1 < QP) ring[ts % kWB] = rows[kWB + ts][l];
        }
#pragma unroll
        for (int b = 0; b < kWB; ++b) rows[b][l] = Y[b];   // (every MAC read of the wave is done)
    }
    __syncthreads();
    HZ_COL_STAMP(3);
    // ---- inverse columns -> T[b][slot][n1], eight blocks per transform, groups alternating
    if (colw) {
        for (int bl0 = 8 * half; bl0 < kWB; bl0 += 16) {
            const int bl = min(bl0 + g8, kWB - 1);
            double2 v[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = rows[bl][r8 + 8 * m];
            const int valid = min(8, kWB - bl0);
            col_fft8x8<true>(v, rows, bl0, valid, l, L.w64);
            const int bg = b0 + bl0 + g8;
            if (g8 < valid && bg < a.B) {
                double2* dst = a.T + ((long)bg * kSlots + 4 * u + w) * 64;
#pragma unroll
                for (int n1b = 0; n1b < 8; ++n1b)   // x W4096^(-n1 c)
                    dst[r8 + 8 * n1b] = cmulc(L.tn[w][r8 + 8 * n1b], v[n1b]);
            }
        }
    }
    HZ_COL_STAMP(4);
}

// bin c + 64 l of the full-spectrum partition spectra from the three-kernel layout (H [Qp][2048]
// complex, Hn [Qp] bin 2048): Hc [kSlots][Q][64]; grid (kSlots, Q), 64 threads
__global__ __launch_bounds__(64) void resp_hcol_kernel(const double2* __restrict__ H, const double* __restrict__ Hn,
                                                      int Q, double2* __restrict__ Hc) {
    const int slot = blockIdx.x, p = blockIdx.y, l = threadIdx.x;
    const int u = slot / 4, i = slot % 4;
    if (i >= unit_ncol(u)) return;
    const int k = unit_c0(u) + 16 * i + 64 * l;
    double2 v;
    if (k < kP) v = H[(long)p * kP + k];
    else if (k == kP) v = make_double2(Hn[p], 0.0);
    else {
        const double2 m = H[(long)p * kP + (2 * kP - k)];
        v = make_double2(m.x, -m.y);
    }
    Hc[((long)slot * Q + p) * 64 + l] = v;
}

// the combine's column table: for c < 64 the slot holding T^c (bit 7 set: conj of that slot's
// T^(64-c)); built on the host
inline void col_map(unsigned char (&m)[64]) {
    for (int c = 0; c < 64; ++c) m[c] = 0xff;
    for (int u = 0; u < kUnits; ++u)
        for (int i = 0; i < unit_ncol(u); ++i) m[unit_c0(u) + 16 * i] = (unsigned char)(4 * u + i);
    for (int c = 1; c < 64; ++c)
        if (m[c] == 0xff) m[c] = (unsigned char)(m[64 - c] | 0x80);
}

struct CombLds {
    double2 ts[kSlots][64];   // the block's inverse columns
    double out[kP];           // its samples, [n2 - 32][n1]
};

// one output block: x[n1 + 64 n2] = sum_c W64^(-n2 c) V^c[n1] for n2 >= 32, two n1 per transform
// (V^c[q] + i V^c[q + 32]: both outputs real); columns 0 and 32 are real (imaginary roundoff
// dropped)
__device__ __forceinline__ void comb_block(const double2* __restrict__ T, const unsigned char* __restrict__ cmap,
                                           const double2* __restrict__ tw4k, long b, CombLds& L,
                                           double* __restrict__ out, long n_out) {
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    const double2* src = T + b * kSlots * 64;
#pragma unroll
    for (int i = 0; i < kSlots * 64 / 256; ++i) (&L.ts[0][0])[t + 256 * i] = src[t + 256 * i];
    const int e = cmap[l];
    const int slot = e & 0x7f;
    const bool cj = (e & 0x80) != 0, re_only = (l & 31) == 0;
    Fft64 f;
    f.init(tw4k, l);
    __syncthreads();
    for (int q = 8 * w; q < 8 * w + 8; ++q) {
        double2 va = L.ts[slot][q], vb = L.ts[slot][q + 32];
        if (cj) {
            va.y = -va.y;
            vb.y = -vb.y;
        }
        if (re_only) va.y = vb.y = 0.0;
        // IDFT(V) = conj(DFT(conj V)), V = va + i vb
        double2 xa[1] = {make_double2(va.x - vb.y, -(va.y + vb.x))};
        f.fwd(xa, l);   // lane l: n2 = brev6(l)
        const double2 xv = xa[0];
        const int n2 = brev6(l);
        if (n2 >= 32) {
            L.out[(n2 - 32) * 64 + q] = xv.x;          // Re: n1 = q
            L.out[(n2 - 32) * 64 + q + 32] = -xv.y;    // Im (conjugated back): n1 = q + 32
        }
    }
    __syncthreads();
    const long t0 = b * kP;
#pragma unroll
    for (int i = 0; i < kP / 256; ++i) {
        const long k = t + 256 * i;
        if (t0 + k < n_out) out[t0 + k] = L.out[k];
    }
}

}  // namespace hz_col
