/*
 * hz_oracle.c -- TEST INFRASTRUCTURE ONLY.  See hz_oracle.h for the parity
 * status.  Compiled with -O2 -ffp-contract=off so rounding is deterministic
 * (no FMA contraction), see oracle/Makefile.
 *
 * Every function cites the reference file:line it restates.
 */
#include "hz_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* src/includes.h:30-32 */
#define ORC_PI 3.14159265359
#define ORC_E 2.718281828459045
#define ORC_SR 48000

/* src/includes.h:38-48 : order = log2(DBL_EPSILON) = -52 */
double orc_relaxation(double k)
{
    if (k == 0) return 0;
    return pow(2.0, log2(DBL_EPSILON) / (fmax(0, k) * ORC_SR));
}

/* src/includes.h:51-59 */
double orc_mtof(double m) { return 440.0 * pow(2, (m - 69) / 12); }
double orc_ftom(double f) { return 69 + log2(f / 440.0) * 12; }

/* Distortion functors used through Filterbank::operator()(T, T(*)(T))
 * (src/filterbank.h:133-139).  Shapes from tests/filterbank.cpp:158-176
 * (softclip, saturate) and src/wave.h:150 (limiter, FUNCTIONAL lookup).
 * abs() is taken as fabs (macOS libc++ semantics). */
static int orc_sgn(double v) { return (0.0 < v) - (v < 0.0); }
double orc_dist(int id, double v, double param)
{
    switch (id) {
    case 0: return v;
    case 1: { /* softclip(sample, width) tests/filterbank.cpp:158-166 */
        double width = param;
        if (fabs(v) < width) return v;
        int sign = orc_sgn(v);
        double gap = v - sign * width;
        return sign * width + (1 - width) * 2.0 / ORC_PI * atan(ORC_PI * gap / (2 * (1 - width)));
    }
    case 2: /* saturate tests/filterbank.cpp:173-176 */
        return 2.0 / ORC_PI * atan(2 * ORC_PI * v / 2.0);
    case 3: /* limiter src/wave.h:150 */
        return 2.0 / ORC_PI * atan(v);
    default: return v;
    }
}

/* ---- Filterbank<double>  src/filterbank.h:16-188 ---------------------- */
struct orc_fb {
    int order, N;
    double sp, sg;          /* smoothing_p, smoothing_g (filterbank.h:36-37,165) */
    double* F;              /* forwards  N x (O+1)  (filterbank.h:49)  F[n*(O+1)+i] */
    double* Bk;             /* backs     N x O      (filterbank.h:50)  Bk[n*O+k]    */
    double* xr;             /* input     2(O+1)     (filterbank.h:51)               */
    double* Y;              /* outputs   2(O+1) x N (filterbank.h:52)  Y[r*N+n]     */
    double *pin, *pout, *gin, *gout;
    double* temp;
    int origin, computed;
};

orc_fb* orc_fb_create(int order, int N, double k_p, double k_g)
{
    orc_fb* fb = (orc_fb*)calloc(1, sizeof(orc_fb));
    int R = 2 * (order + 1);
    fb->order = order;
    fb->N = N;
    fb->sp = orc_relaxation(k_p);
    fb->sg = orc_relaxation(k_g);
    fb->F = (double*)calloc((size_t)N * (order + 1), sizeof(double));
    fb->Bk = (double*)calloc((size_t)N * (order > 0 ? order : 1), sizeof(double));
    fb->xr = (double*)calloc(R, sizeof(double));
    fb->Y = (double*)calloc((size_t)R * N, sizeof(double));
    fb->pin = (double*)calloc(N, sizeof(double));
    fb->pout = (double*)calloc(N, sizeof(double));
    fb->gin = (double*)calloc(N, sizeof(double));
    fb->gout = (double*)calloc(N, sizeof(double));
    fb->temp = (double*)calloc(N, sizeof(double));
    return fb;
}

void orc_fb_destroy(orc_fb* fb)
{
    if (!fb) return;
    free(fb->F); free(fb->Bk); free(fb->xr); free(fb->Y);
    free(fb->pin); free(fb->pout); free(fb->gin); free(fb->gout); free(fb->temp);
    free(fb);
}

/* filterbank.h:73-82 */
void orc_fb_coefficients(orc_fb* fb, int n, const double* fwd, int nf, const double* back, int nb)
{
    int O = fb->order;
    int c = nf < O + 1 ? nf : O + 1;
    for (int i = 0; i < c; i++) fb->F[(size_t)n * (O + 1) + i] = fwd[i];
    c = nb < O ? nb : O;
    for (int i = 0; i < c; i++) fb->Bk[(size_t)n * O + i] = back[i];
}

/* filterbank.h:85-116 */
void orc_fb_boost(orc_fb* fb, int n, double v) { fb->pin[n] = v; }
void orc_fb_boost_all(orc_fb* fb, const double* v, int count)
{
    for (int i = 0; i < (fb->N < count ? fb->N : count); i++) fb->pin[i] = v[i];
}
void orc_fb_mix(orc_fb* fb, int n, double v) { fb->gin[n] = v; }
void orc_fb_mix_all(orc_fb* fb, const double* v, int count)
{
    for (int i = 0; i < (fb->N < count ? fb->N : count); i++) fb->gin[i] = v[i];
}
void orc_fb_open(orc_fb* fb)
{
    for (int i = 0; i < fb->N; i++) fb->gin[i] = 1;
}

/* compute(): filterbank.h:170-187 */
static void orc_fb_compute(orc_fb* fb, double sample)
{
    const int O = fb->order, N = fb->N, o = fb->origin;
    const double sp = fb->sp, sg = fb->sg;
    for (int n = 0; n < N; n++) {                                   /* 172 */
        fb->pout[n] = (1 - sp) * fb->pin[n] + sp * fb->pout[n];
        fb->gout[n] = (1 - sg) * fb->gin[n] + sg * fb->gout[n];     /* 173 */
    }
    fb->xr[o] = sample;                                             /* 175 */
    fb->xr[o + O + 1] = sample;                                     /* 176 */
    for (int n = 0; n < N; n++) {                                   /* 178-179 */
        const double* f = fb->F + (size_t)n * (O + 1);
        double ff = f[0] * fb->xr[o];
        for (int i = 1; i <= O; i++) ff += f[i] * fb->xr[o + i];
        double bsum = 0;
        const double* b = fb->Bk + (size_t)n * O;
        for (int k = 0; k < O; k++) bsum += b[k] * fb->Y[(size_t)(o + 1 + k) * N + n];
        fb->temp[n] = ff * fb->pout[n] - bsum;
    }
    memcpy(fb->Y + (size_t)o * N, fb->temp, sizeof(double) * N);           /* 183 */
    memcpy(fb->Y + (size_t)(o + O + 1) * N, fb->temp, sizeof(double) * N); /* 184 */
    fb->computed = 1;
}

/* operator(): filterbank.h:125-139 */
double orc_fb_sample(orc_fb* fb, double x, int dist_id, double dist_param)
{
    if (!fb->computed) orc_fb_compute(fb, x);
    const double* row = fb->Y + (size_t)fb->origin * fb->N;
    double s = 0;
    if (dist_id == 0)
        for (int n = 0; n < fb->N; n++) s += row[n] * fb->gout[n];
    else
        for (int n = 0; n < fb->N; n++) s += orc_dist(dist_id, row[n] * fb->gout[n], dist_param);
    return s;
}

/* tick(): filterbank.h:142-148 */
void orc_fb_tick(orc_fb* fb)
{
    fb->origin--;
    if (fb->origin < 0) fb->origin += fb->order + 1;
    fb->computed = 0;
}

/* the state in libhuygens_hip's hz_fb_get_state layout, between tick() and the next sample:
 * [x history: x[t-1-k], k < O] [y history: band n's y[t-1-k] at n*O + k] [pre, gain per band] --
 * ring rows origin+1+k of the duplicated rings (filterbank.h:51-52, 175-184) */
void orc_fb_get_state(const orc_fb* fb, double* buf)
{
    const int O = fb->order, N = fb->N, o = fb->origin;
    for (int k = 0; k < O; k++) buf[k] = fb->xr[o + 1 + k];
    for (int n = 0; n < N; n++)
        for (int k = 0; k < O; k++) buf[O + (size_t)n * O + k] = fb->Y[(size_t)(o + 1 + k) * N + n];
    for (int n = 0; n < N; n++) {
        buf[O + (size_t)N * O + 2 * (size_t)n] = fb->pout[n];
        buf[O + (size_t)N * O + 2 * (size_t)n + 1] = fb->gout[n];
    }
}

/* the demo block loop (tests/resynthesis.cpp:35-39) */
void orc_fb_process(orc_fb* fb, const double* in, double* out, long n, int dist_id, double dist_param)
{
    for (long i = 0; i < n; i++) {
        out[i] = orc_fb_sample(fb, in[i], dist_id, dist_param);
        orc_fb_tick(fb);
    }
}

/* ---- Oscbank<double,N>  src/oscbank.h:15-97 ------------------------------
 * Active set: Multichannel<T,N>::where, kept sorted ascending by insert/popout
 * (src/multichannel.h:51-118); tick/mixdown visit it in that order. */
struct orc_osc {
    int N;
    double* zr; double* zi;   /* phases      (oscbank.h:39-46, setOnes) */
    double* wr; double* wi;   /* frequencies (oscbank.h:40-46, setOnes) */
    char* active;             /* multichannel.h:22-24 */
    int* where; int nwhere;   /* sorted active indices */
};

orc_osc* orc_osc_create(int N, double k)
{
    (void)k; /* stiffness = relaxation(k) is stored but never used (oscbank.h:37,96) */
    orc_osc* o = (orc_osc*)calloc(1, sizeof(orc_osc));
    o->N = N;
    o->zr = (double*)malloc(sizeof(double) * N); o->zi = (double*)calloc(N, sizeof(double));
    o->wr = (double*)malloc(sizeof(double) * N); o->wi = (double*)calloc(N, sizeof(double));
    for (int i = 0; i < N; i++) { o->zr[i] = 1.0; o->wr[i] = 1.0; }
    o->active = (char*)calloc(N, 1);
    o->where = (int*)malloc(sizeof(int) * (N > 0 ? N : 1));
    return o;
}

void orc_osc_destroy(orc_osc* o)
{
    if (!o) return;
    free(o->zr); free(o->zi); free(o->wr); free(o->wi); free(o->active); free(o->where); free(o);
}

/* oscbank.h:49-56 */
void orc_osc_freqmod(orc_osc* o, int index, double hz)
{
    if (0 <= index && index < o->N) {
        o->wr[index] = cos(2 * ORC_PI * hz / ORC_SR);
        o->wi[index] = sin(2 * ORC_PI * hz / ORC_SR);
    }
}

/* multichannel.h:87-92 (insert keeps where sorted) */
void orc_osc_activate(orc_osc* o, const int* idx, int count)
{
    for (int c = 0; c < count; c++) {
        int i = idx[c];
        if (0 <= i && i < o->N && !o->active[i]) {
            int pos = o->nwhere;
            while (pos > 0 && o->where[pos - 1] > i) { o->where[pos] = o->where[pos - 1]; pos--; }
            o->where[pos] = i;
            o->nwhere++;
            o->active[i] = 1;
        }
    }
}

/* multichannel.h:95-100 (popout) */
void orc_osc_deactivate(orc_osc* o, const int* idx, int count)
{
    for (int c = 0; c < count; c++) {
        int i = idx[c];
        if (0 <= i && i < o->N && o->active[i]) {
            int pos = 0;
            while (o->where[pos] != i) pos++;
            for (; pos + 1 < o->nwhere; pos++) o->where[pos] = o->where[pos + 1];
            o->nwhere--;
            o->active[i] = 0;
        }
    }
}

void orc_osc_open(orc_osc* o)
{
    for (int i = 0; i < o->N; i++) orc_osc_activate(o, &i, 1);
}

void orc_osc_close(orc_osc* o)
{
    for (int i = 0; i < o->N; i++) orc_osc_deactivate(o, &i, 1);
}

int orc_osc_active_count(orc_osc* o) { return o->nwhere; }

/* oscbank.h:59-63: z *= w; z /= (1 + |z|^2) / 2  (Eigen abs2 = re^2 + im^2) */
void orc_osc_tick(orc_osc* o)
{
    for (int c = 0; c < o->nwhere; c++) {
        int i = o->where[c];
        double ar = o->zr[i], ai = o->zi[i];
        double br = o->wr[i], bi = o->wi[i];
        double zr = ar * br - ai * bi;
        double zi = ar * bi + ai * br;
        double d = (1.0 + (zr * zr + zi * zi)) / 2;
        o->zr[i] = zr / d;
        o->zi[i] = zi / d;
    }
}

/* oscbank.h:81-90 */
void orc_osc_mixdown(orc_osc* o, double* re, double* im)
{
    double r = 0, m = 0;
    for (int c = 0; c < o->nwhere; c++) { r += o->zr[o->where[c]]; m += o->zi[o->where[c]]; }
    *re = r; *im = m;
}

void orc_osc_phases(orc_osc* o, double* z)
{
    for (int i = 0; i < o->N; i++) { z[2 * i] = o->zr[i]; z[2 * i + 1] = o->zi[i]; }
}

void orc_osc_fill(orc_osc* o, double* mix, double* per_band, long n)
{
    for (long t = 0; t < n; t++) {
        orc_osc_mixdown(o, mix + 2 * t, mix + 2 * t + 1);
        if (per_band) orc_osc_phases(o, per_band + 2 * t * o->N);
        orc_osc_tick(o);
    }
}

/* ---- per-sample coefficient streams ----------------
 * Subtractive ALLINONE / ONEPERVOICE (src/subtractive.h:215-228, 300-317) set every band's
 * coefficients in tick(), i.e. between samples.  Row t of the stream holds the coefficients
 * in effect at sample t:
 *   kind 0: stream[t][k][n], k < O+1 forward then k < O back (band-minor rows);
 *   kind 1: stream[t][n] = frequency (Hz), order 2: {g, 0, -g}, {-2 R cos(2 PI f / SR), R^2},
 *           g = resonant(f, R) (subtractive.h:240-249), R = param.
 * resonant(): maximum = 1/(Q-1) - 1/(Q - cos2 - i sin2); 1 / sqrt(|maximum|), with the
 * complex quotient by Smith's algorithm as libgcc's __divdc3 (g++ on Linux) and |.| = hypot. */
static void orc_cdiv(double a, double b, double c, double d, double* x, double* y)
{
    if (fabs(c) < fabs(d)) {
        const double ratio = c / d, denom = (c * ratio) + d;
        *x = ((a * ratio) + b) / denom;
        *y = ((b * ratio) - a) / denom;
    } else {
        const double ratio = d / c, denom = (d * ratio) + c;
        *x = ((b * ratio) + a) / denom;
        *y = (b - (a * ratio)) / denom;
    }
}

double orc_resonant(double frequency, double Q)
{
    const double c2 = cos(4 * ORC_PI * frequency / ORC_SR), s2 = sin(4 * ORC_PI * frequency / ORC_SR);
    /* Q - cosine2 - 1.0i * sine2: (Q - c2, -0) - (0 * s2 - 1 * 0, 0 * 0 + 1 * s2) */
    const double ir = 0.0 * s2 - 1.0 * 0.0, ii = 0.0 * 0.0 + 1.0 * s2;
    const double dr = (Q - c2) - ir, di = -0.0 - ii;
    double qr, qi;
    orc_cdiv(1.0, 0.0, dr, di, &qr, &qi);
    const double mr = 1.0 / (Q - 1) - qr, mi = 0.0 - qi;
    return 1 / sqrt(hypot(mr, mi));
}

void orc_fb_resonant_coefficients(double frequency, double R, double* fwd, double* back)
{
    const double cosine = cos(2 * ORC_PI * frequency / ORC_SR);
    const double gain = orc_resonant(frequency, R);
    fwd[0] = gain;
    fwd[1] = 0;
    fwd[2] = -gain;
    back[0] = -2 * R * cosine;
    back[1] = R * R;
}

void orc_fb_process_tv(orc_fb* fb, const double* in, double* out, long n, int kind, const double* stream,
                       double param, int dist_id, double dist_param)
{
    const int O = fb->order, N = fb->N;
    for (long t = 0; t < n; t++) {
        for (int b = 0; b < N; b++) {
            double f[5], bk[4];
            if (kind == 0) {
                const double* row = stream + (size_t)t * (2 * O + 1) * N;
                for (int k = 0; k <= O; k++) f[k] = row[(size_t)k * N + b];
                for (int k = 0; k < O; k++) bk[k] = row[(size_t)(O + 1 + k) * N + b];
            } else {
                orc_fb_resonant_coefficients(stream[(size_t)t * N + b], param, f, bk);
            }
            orc_fb_coefficients(fb, b, f, O + 1, bk, O);
        }
        out[t] = orc_fb_sample(fb, in[t], dist_id, dist_param);
        orc_fb_tick(fb);
    }
}
