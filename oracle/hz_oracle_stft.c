/*
 * hz_oracle_stft.c -- TEST INFRASTRUCTURE ONLY (see hz_oracle.h).
 * Scalar restatement of Fourier (src/fourier.h:50-194), StaticSTFT (src/staticSTFT.h:10-177)
 * and Cosine (src/fourier.h:197-234).
 *
 * Kept as in the reference: 2*laps slots, slot i starting at writepoint -stride*i; per
 * sample write() then read(); the window evaluated per sample in double with the truncated
 * PI (halfhann for Fourier, hann for StaticSTFT, src/wave.h:148-149); the frame's FFT ->
 * processor -> IFFT when its writepoint reaches N; read() accumulates in long double and
 * divides by the int N*laps/2.
 * FFTW is absent here: its unnormalised FORWARD e^{-2 pi i jk/N} / BACKWARD
 * e^{+} transforms and REDFT10 / REDFT01 are evaluated in long double (radix-2 for powers
 * of two, direct sums otherwise) and rounded to double, i.e. the exact DFT to ~1e-18.
 * FFTW's own double rounding differs from it by ~1e-16 relative; the conventions are pinned
 * against numpy.fft / scipy.fft.dct in tests/golden/make_golden_stft.py.
 * Processors: identity, the StaticSTFT gate (staticSTFT.h:99-128), the spectral.cpp gate
 * (tests/spectral.cpp:32-72), the Hilbert half-band (tests/SFML/hilbert.cpp:37-49), or a
 * caller-supplied function pointer.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hz_oracle.h"

#define ORC_PI 3.14159265359

static double win_eval(int kind, double p) {
    if (kind == 1) return 0.5 * (1 - cos(2 * ORC_PI * p));   /* hann */
    return sqrt(0.5 * (1 - cos(2 * ORC_PI * p)));             /* halfhann */
}

/* unnormalised DFT in long double; sign -1 forward, +1 backward; io interleaved double */
static void dft_ld(const double* x, double* y, int N, int sign) {
    const long double pi = acosl(-1.0L);
    long double* re = (long double*)malloc(sizeof(long double) * N);
    long double* im = (long double*)malloc(sizeof(long double) * N);
    if ((N & (N - 1)) == 0) {
        int lg = 0;
        while ((1 << lg) < N) lg++;
        for (int k = 0; k < N; k++) {
            int r = 0;
            for (int b = 0; b < lg; b++) r |= ((k >> b) & 1) << (lg - 1 - b);
            re[r] = x[2 * k];
            im[r] = x[2 * k + 1];
        }
        for (int half = 1; half < N; half *= 2) {
            for (int pos = 0; pos < half; pos++) {
                const long double a = sign * pi * pos / half;
                const long double wr = cosl(a), wi = sinl(a);
                for (int g = 0; g < N; g += 2 * half) {
                    const int i0 = g + pos, i1 = i0 + half;
                    const long double tr = wr * re[i1] - wi * im[i1];
                    const long double ti = wr * im[i1] + wi * re[i1];
                    re[i1] = re[i0] - tr;
                    im[i1] = im[i0] - ti;
                    re[i0] += tr;
                    im[i0] += ti;
                }
            }
        }
    } else {
        for (int k = 0; k < N; k++) {
            long double sr = 0, si = 0;
            for (int j = 0; j < N; j++) {
                const long double a = sign * 2.0L * pi * (long double)(((long)j * k) % N) / N;
                sr += x[2 * j] * cosl(a) - x[2 * j + 1] * sinl(a);
                si += x[2 * j] * sinl(a) + x[2 * j + 1] * cosl(a);
            }
            re[k] = sr;
            im[k] = si;
        }
    }
    for (int k = 0; k < N; k++) {
        y[2 * k] = (double)re[k];
        y[2 * k + 1] = (double)im[k];
    }
    free(re);
    free(im);
}

void orc_dft(const double* x, double* y, int N, int sign) { dft_ld(x, y, N, sign); }

struct orc_stft {
    int N, laps, stride, S, window, proc;
    double p0, p1;
    orc_stft_cb cb;
    double *in, *mid, *out;   /* [S][N] complex interleaved */
    int *wp, *rp;
    char *reading, *writing;
    long frames;
};

orc_stft* orc_stft_create(int N, int laps, int window, int proc, double p0, double p1) {
    orc_stft* s = (orc_stft*)calloc(1, sizeof(orc_stft));
    s->N = N;
    s->laps = laps;
    s->stride = N / laps;
    s->S = 2 * laps;
    s->window = window;
    s->proc = proc;
    s->p0 = p0;
    s->p1 = p1;
    s->in = (double*)calloc((size_t)2 * N * s->S, sizeof(double));
    s->mid = (double*)calloc((size_t)2 * N * s->S, sizeof(double));
    s->out = (double*)calloc((size_t)2 * N * s->S, sizeof(double));
    s->wp = (int*)calloc(s->S, sizeof(int));
    s->rp = (int*)calloc(s->S, sizeof(int));
    s->reading = (char*)calloc(s->S, 1);
    s->writing = (char*)calloc(s->S, 1);
    for (int i = 0; i < s->S; i++) {
        s->wp[i] = -s->stride * i;
        s->writing[i] = 1;
    }
    return s;
}

void orc_stft_set_callback(orc_stft* s, orc_stft_cb cb) {
    s->cb = cb;
    s->proc = ORC_PROC_CALLBACK;
}

void orc_stft_destroy(orc_stft* s) {
    if (!s) return;
    free(s->in); free(s->mid); free(s->out);
    free(s->wp); free(s->rp); free(s->reading); free(s->writing);
    free(s);
}

static void run_proc(orc_stft* s, const double* in, double* out) {
    const int N = s->N;
    switch (s->proc) {
    case ORC_PROC_STATIC_GATE: {   /* staticSTFT.h:99-128 (in place on the spectrum) */
        double average = 0;
        for (int j = 0; j < N; j++) average += sqrt(in[2 * j] * in[2 * j] + in[2 * j + 1] * in[2 * j + 1]) / N;
        for (int j = 0; j < N; j++) {
            const double b0 = in[2 * j], b1 = in[2 * j + 1];
            if (b0 * b0 + b1 * b1 < s->p0 * average * average) {
                out[2 * j] = b0 * s->p1;
                out[2 * j + 1] = b1 * s->p1;
            } else {
                out[2 * j] = b0;
                out[2 * j + 1] = b1;
            }
        }
        break;
    }
    case ORC_PROC_GATE_KEEP: {     /* tests/spectral.cpp:32-72 */
        long double average = 0;
        for (int i = 0; i < N; i++) {
            out[2 * i] = out[2 * i + 1] = 0;
            average += hypot(in[2 * i], in[2 * i + 1]);
        }
        average /= N;
        for (int i = 0; i < N; i++) {
            const double nrm = in[2 * i] * in[2 * i] + in[2 * i + 1] * in[2 * i + 1];
            if (nrm > s->p0 * average * average) {
                out[2 * i] = in[2 * i];
                out[2 * i + 1] = in[2 * i + 1];
            } else {
                out[2 * i] = out[2 * i + 1] = 0;
            }
        }
        break;
    }
    case ORC_PROC_HILBERT:          /* tests/SFML/hilbert.cpp:37-49 */
        for (int i = 0; i < N; i++) {
            out[2 * i] = i < N / 2 ? in[2 * i] : 0;
            out[2 * i + 1] = i < N / 2 ? in[2 * i + 1] : 0;
        }
        break;
    case ORC_PROC_CALLBACK:
        s->cb(in, out);
        break;
    default:                        /* identity */
        memcpy(out, in, sizeof(double) * 2 * N);
    }
}

/* fourier.h:130-144: the slot operations a caller may also invoke directly */
void orc_stft_forward(orc_stft* s, int i) { dft_ld(s->in + (size_t)2 * s->N * i, s->mid + (size_t)2 * s->N * i, s->N, -1); }
void orc_stft_backward(orc_stft* s, int i) { dft_ld(s->out + (size_t)2 * s->N * i, s->in + (size_t)2 * s->N * i, s->N, +1); }
void orc_stft_process_slot(orc_stft* s, int i) { run_proc(s, s->mid + (size_t)2 * s->N * i, s->out + (size_t)2 * s->N * i); }

void orc_stft_write(orc_stft* s, double re, double im) {   /* fourier.h:102-128 */
    const int N = s->N;
    for (int i = 0; i < s->S; i++) {
        if (!s->writing[i]) continue;
        if (s->wp[i] >= 0) {
            const double w = win_eval(s->window, s->wp[i] / (double)N);
            s->in[2 * ((size_t)s->wp[i] + (size_t)N * i)] = w * re;
            s->in[2 * ((size_t)s->wp[i] + (size_t)N * i) + 1] = w * im;
        }
        s->wp[i]++;
        if (s->wp[i] == N) {
            s->writing[i] = 0;
            s->reading[i] = 1;
            s->rp[i] = 0;
            double* fi = s->in + (size_t)2 * N * i;
            double* fm = s->mid + (size_t)2 * N * i;
            double* fo = s->out + (size_t)2 * N * i;
            dft_ld(fi, fm, N, -1);   /* forward(i) */
            run_proc(s, fm, fo);     /* process(i) */
            dft_ld(fo, fi, N, +1);   /* backward(i) */
            s->frames++;
        }
    }
}

void orc_stft_read(orc_stft* s, double* re, double* im) {   /* fourier.h:147-177 */
    const int N = s->N;
    long double ra = 0, ia = 0;
    for (int i = 0; i < s->S; i++) {
        if (!s->reading[i]) continue;
        const double w = win_eval(s->window, s->rp[i] / (double)N);
        const double* smp = s->in + 2 * ((size_t)s->rp[i] + (size_t)N * i);
        ra += w * smp[0];
        ia += w * smp[1];
        s->rp[i]++;
        if (s->rp[i] == N) {
            s->writing[i] = 1;
            s->reading[i] = 0;
            s->wp[i] = 0;
        }
    }
    ra /= N * s->laps / 2;
    ia /= N * s->laps / 2;
    *re = (double)ra;
    *im = (double)ia;
}

void orc_stft_process_block(orc_stft* s, const double* re, const double* im, double* out_re, double* out_im,
                            long n) {
    for (long t = 0; t < n; t++) {
        double r, i;
        orc_stft_write(s, re[t], im ? im[t] : 0.0);
        orc_stft_read(s, &r, &i);
        out_re[t] = r;
        if (out_im) out_im[t] = i;
    }
}

long orc_stft_frames(orc_stft* s) { return s->frames; }

/* Cosine (fourier.h:197-234): REDFT10 Y_k = 2 sum x_j cos(pi k (2j+1) / 2N);
 * REDFT01 Y_k = x_0 + 2 sum_{j>=1} x_j cos(pi j (2k+1) / 2N); long double direct sums */
void orc_dct(const double* x, double* y, int N, int kind) {
    const long double pi = acosl(-1.0L);
    for (int k = 0; k < N; k++) {
        long double s = 0;
        if (kind == 10) {
            for (int j = 0; j < N; j++) s += 2.0L * x[j] * cosl(pi * (long double)(((long)k * (2 * j + 1)) % (4L * N)) / (2.0L * N));
        } else {
            s = x[0];
            for (int j = 1; j < N; j++) s += 2.0L * x[j] * cosl(pi * (long double)(((long)j * (2 * k + 1)) % (4L * N)) / (2.0L * N));
        }
        y[k] = (double)s;
    }
}
