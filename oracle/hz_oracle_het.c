/*
 * hz_oracle_het.c -- TEST INFRASTRUCTURE ONLY (see hz_oracle.h).
 *
 * Scalar restatement of the heterodyne bank chain of tests/harmbank.cpp:77-101:
 *   out = limiter(dry x + gain mixdown(demodulators(synthesis(),
 *           smoothbank(latchbank(&rmsbank, slidebank(modulators(x, analysis())))))))
 * then analysis/synthesis/slidebank/smoothbank/rmsbank tick, with
 *   Oscbank<T,N>   src/oscbank.h:37-68   (z *= w; z /= (1 + |z|^2) / 2 on active channels)
 *   Modbank<T,N>   src/modbank.h:40-58   (elementwise products)
 *   Slidebank<T,N> src/slidebank.h:60-157 (per channel: new_0 = (1-r) m + r old_0,
 *                  new_q = (1-r) old_{q-1} + r old_q; out = new_{order-1}; the sparse
 *                  product's column order gives ((1-r) a) + (r b))
 *   RMSbank<T,N>   src/rmsbank.h:29-66   (running sum of |s|^2 over `width` samples, sqrt(sum / width))
 *   Latchbank<T,N> src/latchbank.h:65-85 (armed / engaged hysteresis, output s * engaged)
 *   Stickbank<T,N> src/stickbank.h:30-190 (y = (1+rad)^order l - sum_k y[t-1-k] back[k],
 *                  back = coefficients of prod (z - rad) without the leading 1)
 *   Mixer<T,N>     src/mixer.h:30-33     (sum of real parts; summed in channel order here --
 *                  Eigen's reduction order is unspecified, so the sum is pinned to ~1e-15)
 *   limiter        src/wave.h:150        (2/PI atan(p), FUNCTIONAL)
 * Complex products are written out as (ac - bd, ad + bc).  Parity: unpinned by the
 * reference's own files; pinned by tests/test_heterodyne_cpu.py (closed forms, numpy model).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hz_oracle.h"

#define ORC_PI 3.14159265359
#define ORC_SR 48000

struct orc_het {
    int N, order, sorder;
    unsigned width;
    double thresh, ratio, dry, gain, stick_gain; /* stick_gain = pow(1 + rad, order) */
    double* za;    /* [N][2] analysis phasors */
    double* wa;    /* [N][2] analysis frequencies (unit phasors) */
    double* zs;    /* synthesis */
    double* ws;
    unsigned char *act_a, *act_s;
    double* radii; /* [N][2] */
    double* slide; /* [N][order][2] */
    double* ring;  /* [N][width + 1] |s|^2 history */
    double* rsum;  /* [N] */
    unsigned char *armed, *engaged;
    double* back;  /* [sorder] real coefficients */
    double* stick; /* [N][sorder][2] y[t-1-k] */
    int rorigin;   /* RMSbank ring origin (decrements) */
};

static void cmul(double ar, double ai, double br, double bi, double* cr, double* ci) {
    *cr = ar * br - ai * bi;
    *ci = ar * bi + ai * br;
}

orc_het* orc_het_create(int N, int order, const double* radii, double thresh, double ratio, unsigned width,
                        int stick_order, double stick_rad, double dry, double gain) {
    orc_het* h = (orc_het*)calloc(1, sizeof(orc_het));
    h->N = N;
    h->sorder = stick_order > 1 ? stick_order : 1;
    h->width = width;
    h->thresh = thresh;
    h->ratio = ratio;
    h->dry = dry;
    h->gain = gain;
    h->stick_gain = pow(1 + stick_rad, h->sorder);
    h->za = (double*)calloc(2 * (size_t)N, sizeof(double));
    h->wa = (double*)calloc(2 * (size_t)N, sizeof(double));
    h->zs = (double*)calloc(2 * (size_t)N, sizeof(double));
    h->ws = (double*)calloc(2 * (size_t)N, sizeof(double));
    for (int i = 0; i < N; i++) { /* setOnes (oscbank.h:44-45) */
        h->za[2 * i] = h->wa[2 * i] = h->zs[2 * i] = h->ws[2 * i] = 1.0;
    }
    h->act_a = (unsigned char*)calloc(N, 1);
    h->act_s = (unsigned char*)calloc(N, 1);
    h->radii = NULL;
    h->slide = NULL;
    orc_het_setup(h, order, radii);
    h->ring = (double*)calloc((size_t)N * (width + 1), sizeof(double));
    h->rsum = (double*)calloc(N, sizeof(double));
    h->armed = (unsigned char*)calloc(N, 1);
    h->engaged = (unsigned char*)calloc(N, 1);
    /* stickbank.h coefficients(zeros = {rad} x order): polynomial prod (z + ... ) as the reference's
     * recursion: total[i] += first * shifted[i]; total[i+1] += shifted[i] */
    {
        const int d = h->sorder;
        double* c = (double*)calloc(d + 1, sizeof(double));
        c[0] = stick_rad; /* degree 1: {zeros[start], 1} */
        c[1] = 1;
        for (int deg = 2; deg <= d; deg++) { /* prepend another zero: total = first * shifted + (shifted << 1) */
            double* t = (double*)calloc(deg + 1, sizeof(double));
            for (int i = 0; i < deg; i++) {
                t[i] += stick_rad * c[i];
                t[i + 1] += c[i];
            }
            memcpy(c, t, sizeof(double) * (deg + 1));
            free(t);
        }
        h->back = (double*)calloc(d, sizeof(double));
        for (int i = 0; i < d; i++) h->back[i] = c[i];
        free(c);
    }
    h->stick = (double*)calloc(2 * (size_t)N * h->sorder, sizeof(double));
    return h;
}

void orc_het_destroy(orc_het* h) {
    if (!h) return;
    free(h->za);
    free(h->wa);
    free(h->zs);
    free(h->ws);
    free(h->act_a);
    free(h->act_s);
    free(h->radii);
    free(h->slide);
    free(h->ring);
    free(h->rsum);
    free(h->armed);
    free(h->engaged);
    free(h->back);
    free(h->stick);
    free(h);
}

/* Slidebank::setup (slidebank.h:63-100): new radii, zeroed history */
void orc_het_setup(orc_het* h, int order, const double* radii) {
    free(h->radii);
    free(h->slide);
    h->order = order > 1 ? order : 1; /* slidebank.h:65 */
    h->radii = (double*)calloc(2 * (size_t)h->N, sizeof(double));
    memcpy(h->radii, radii, sizeof(double) * 2 * h->N);
    h->slide = (double*)calloc(2 * (size_t)h->N * h->order, sizeof(double));
}

/* Oscbank::freqmod (oscbank.h:49-56); bank 0 analysis, 1 synthesis.  cos and sin are two
 * libm calls as written (called through pointers so gcc cannot merge them into sincos, whose
 * last bit can differ; the engine's host code makes the same two calls). */
static double (*volatile het_cos)(double) = cos;
static double (*volatile het_sin)(double) = sin;

void orc_het_freqmod(orc_het* h, int bank, int index, double hz) {
    if (index < 0 || index >= h->N) return;
    double* w = bank ? h->ws : h->wa;
    w[2 * index] = het_cos(2 * ORC_PI * hz / ORC_SR);
    w[2 * index + 1] = het_sin(2 * ORC_PI * hz / ORC_SR);
}

void orc_het_activate(orc_het* h, int bank, const int* idx, int count, int on) {
    unsigned char* a = bank ? h->act_s : h->act_a;
    for (int k = 0; k < count; k++)
        if (idx[k] >= 0 && idx[k] < h->N) a[idx[k]] = on ? 1 : 0;
}

static void osc_tick(int N, double* z, const double* w, const unsigned char* act) { /* oscbank.h:59-63 */
    for (int i = 0; i < N; i++)
        if (act[i]) {
            double r, m;
            cmul(z[2 * i], z[2 * i + 1], w[2 * i], w[2 * i + 1], &r, &m);
            const double nrm = (1.0 + (r * r + m * m)) / 2;
            z[2 * i] = r / nrm;
            z[2 * i + 1] = m / nrm;
        }
}

double orc_het_sample(orc_het* h, double x) {
    const int N = h->N, O = h->order, S = h->sorder;
    const unsigned W1 = h->width + 1;
    double mix = 0;
    for (int i = 0; i < N; i++) {
        /* modulators(x, analysis()): T * complex */
        const double mr = x * h->za[2 * i], mi = x * h->za[2 * i + 1];
        /* slidebank */
        const double rr = h->radii[2 * i], ri = h->radii[2 * i + 1];
        const double cr = 1.0 - rr, ci = 0.0 - ri;
        double* st = h->slide + (size_t)2 * i * O;
        double prev_r = mr, prev_i = mi; /* stage q input: m (q = 0) or old stage q-1 */
        for (int q = 0; q < O; q++) {
            double ar, ai, br, bi;
            cmul(cr, ci, prev_r, prev_i, &ar, &ai);
            cmul(rr, ri, st[2 * q], st[2 * q + 1], &br, &bi);
            const double nr = ar + br, ni = ai + bi;
            prev_r = st[2 * q]; /* the next stage reads this stage's OLD value */
            prev_i = st[2 * q + 1];
            st[2 * q] = nr;
            st[2 * q + 1] = ni;
        }
        const double sr = st[2 * (O - 1)], si = st[2 * (O - 1) + 1];
        /* rmsbank */
        const double a2 = sr * sr + si * si;
        double* ring = h->ring + (size_t)i * W1;
        const double old = ring[(h->rorigin + h->width) % W1];
        ring[h->rorigin] = a2;
        const double sum = a2 - old + h->rsum[i];
        h->rsum[i] = sum;
        const double rms = sqrt(sum / h->width);
        /* latchbank */
        const double lo = h->thresh * h->ratio, hi = h->thresh * (1 - h->ratio);
        int armed = h->armed[i] || rms < lo;
        const int t1 = h->engaged[i] && rms < lo;
        const int t2 = !h->engaged[i] && rms > hi && armed;
        int engaged = h->engaged[i] && !t1;
        armed = armed && !t1;
        engaged = engaged || t2;
        h->armed[i] = (unsigned char)armed;
        h->engaged[i] = (unsigned char)engaged;
        const double lr = sr * (double)engaged, li = si * (double)engaged;
        /* smoothbank: y = g l - sum_k y[t-1-k] back[k] */
        double* ys = h->stick + (size_t)2 * i * S;
        double accr = 0, acci = 0;
        for (int k = 0; k < S; k++) {
            double pr, pi;
            cmul(ys[2 * k], ys[2 * k + 1], h->back[k], 0.0, &pr, &pi);
            accr += pr;
            acci += pi;
        }
        const double yr = h->stick_gain * lr - accr, yi = h->stick_gain * li - acci;
        for (int k = S - 1; k > 0; k--) {
            ys[2 * k] = ys[2 * (k - 1)];
            ys[2 * k + 1] = ys[2 * (k - 1) + 1];
        }
        ys[0] = yr;
        ys[1] = yi;
        /* demodulators(synthesis(), smooth): synthesis * smooth; mixdown: real parts */
        double dr, di;
        cmul(h->zs[2 * i], h->zs[2 * i + 1], yr, yi, &dr, &di);
        mix += dr;
    }
    const double out = 2.0 / ORC_PI * atan(h->dry * x + h->gain * mix); /* limiter */
    osc_tick(N, h->za, h->wa, h->act_a);
    osc_tick(N, h->zs, h->ws, h->act_s);
    h->rorigin = (h->rorigin - 1 + (int)W1) % (int)W1; /* rmsbank tick (origin--) */
    return out;
}

void orc_het_process(orc_het* h, const double* in, double* out, long n) {
    for (long t = 0; t < n; t++) out[t] = orc_het_sample(h, in[t]);
}

void orc_het_state(orc_het* h, int what, double* dst) {
    const int N = h->N;
    const unsigned W1 = h->width + 1;
    switch (what) {
    case 0: memcpy(dst, h->za, sizeof(double) * 2 * N); break;
    case 1: memcpy(dst, h->zs, sizeof(double) * 2 * N); break;
    case 2: memcpy(dst, h->slide, sizeof(double) * 2 * N * h->order); break;
    case 3: memcpy(dst, h->rsum, sizeof(double) * N); break;
    case 4:
        for (int i = 0; i < N; i++) {
            dst[2 * i] = h->armed[i];
            dst[2 * i + 1] = h->engaged[i];
        }
        break;
    case 5: memcpy(dst, h->stick, sizeof(double) * 2 * N * h->sorder); break;
    case 6: /* RMS history, newest first: |s_{t-1-k}|^2 for k < width */
        for (int i = 0; i < N; i++)
            for (unsigned k = 0; k < h->width; k++)
                dst[(size_t)i * h->width + k] = h->ring[(size_t)i * W1 + (h->rorigin + 1 + k) % W1];
        break;
    default: break;
    }
}
