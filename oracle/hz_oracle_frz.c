/*
 * hz_oracle_frz.c -- TEST INFRASTRUCTURE ONLY (see hz_oracle.h).
 *
 * Scalar restatement of the spectral-freeze family of src/fourier.h: FFrame (236-297),
 * IFrame (300-347), DFrame (350-387) and Freezer<N> (389-562), with its Delay<double>(1, N)
 * dry path (src/delay.h:21-97 over src/buffer.h).  Kept as in the reference:
 *   - write(): frames i = 0..M-1 in order, each writing its windowed spot and, when frame
 *     i reaches spot 0, processing frame (i-1) mod M (FFT + polarize) -- so frame M-1 is
 *     processed before frame M-1's own write of that sample;
 *   - freeze(): DFrames (excluded + 1 .. excluded + M - 2) from the frames' last
 *     polarizations (norms of the second frame, phase differences);
 *   - operator(): while frozen, slots i = 0..M-1 in order read their IFrame
 *     (iqueue[i]) windowed, and the slot at spot 0 draws next = rand() % (M - 2) (+2 past
 *     `excluded`), advances iindex and repopulates IFrame `next` from DFrame `next`
 *     (polar(sqrt(norm), fmod(dphase, 2 PI)), unnormalised BACKWARD FFT); the sum is / N;
 *     otherwise the N-sample Delay, whose input ring is written only while unfrozen.
 * Uninitialised reference state is taken as zero: FFrame norms/phases before a frame's
 * first process(), `frozen` (false) and `excluded`.  FFTs: the long double DFT of
 * hz_oracle_stft.c (orc_dft).  Parity: unpinned by the reference's own files (no fixtures);
 * pinned by tests/test_freezer_cpu.py's closed-form cases.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hz_oracle.h"

#define ORC_PI 3.14159265359

struct orc_frz {
    int N, laps, stride, M, size, readsize;
    double* fdata;    /* [M][2N] FFrame data (complex interleaved) */
    double* fnorm;    /* [M][N] */
    double* fphase;   /* [M][N] */
    double* dnorm;    /* [M][N] DFrame norms */
    double* dphase;   /* [M][N] DFrame phase changes */
    double* idata;    /* [M][2N] IFrame data */
    double* vocoder;  /* [N] */
    double *tmp, *tmp2;
    int* iqueue;
    int iindex, origin, readhead, excluded, frozen;
    /* Delay<double>(1, N): Buffer(N + 1) input and output rings */
    double *din, *dout;
    unsigned dsize, dorigin;
};

static double halfhann(double p) { return sqrt(0.5 * (1 - cos(2 * ORC_PI * p))); } /* wave.h:149 */

orc_frz* orc_frz_create(int N, int laps, double width) {
    orc_frz* z = (orc_frz*)calloc(1, sizeof(orc_frz));
    width = width > 1.0 ? width : 1.0; /* fourier.h:397-398 */
    laps = laps > 2 ? laps : 2;
    z->N = N;
    z->laps = laps;
    z->stride = N / laps;
    z->M = (int)(width * laps) + 1;
    z->size = z->M * z->stride;
    z->readsize = z->size;
    const size_t MN = (size_t)z->M * N;
    z->fdata = (double*)calloc(2 * MN, sizeof(double));
    z->fnorm = (double*)calloc(MN, sizeof(double));
    z->fphase = (double*)calloc(MN, sizeof(double));
    z->dnorm = (double*)calloc(MN, sizeof(double));
    z->dphase = (double*)calloc(MN, sizeof(double));
    z->idata = (double*)calloc(2 * MN, sizeof(double));
    z->vocoder = (double*)calloc(N, sizeof(double));
    z->tmp = (double*)calloc(2 * (size_t)N, sizeof(double));
    z->tmp2 = (double*)calloc(2 * (size_t)N, sizeof(double));
    z->iqueue = (int*)calloc(z->M, sizeof(int));
    z->dsize = (unsigned)N + 1;
    z->din = (double*)calloc(z->dsize, sizeof(double));
    z->dout = (double*)calloc(z->dsize, sizeof(double));
    return z;
}

void orc_frz_destroy(orc_frz* z) {
    if (!z) return;
    free(z->fdata);
    free(z->fnorm);
    free(z->fphase);
    free(z->dnorm);
    free(z->dphase);
    free(z->idata);
    free(z->vocoder);
    free(z->tmp);
    free(z->tmp2);
    free(z->iqueue);
    free(z->din);
    free(z->dout);
    free(z);
}

int orc_frz_geometry(orc_frz* z, int* stride, int* M) {
    if (stride) *stride = z->stride;
    if (M) *M = z->M;
    return z->size;
}

/* FFrame::process + polarize (fourier.h:273-286) */
static void fframe_process(orc_frz* z, int j) {
    const int N = z->N;
    orc_dft(z->fdata + (size_t)j * 2 * N, z->tmp, N, -1);
    for (int i = 0; i < N; i++) {
        const double re = z->tmp[2 * i], im = z->tmp[2 * i + 1];
        z->fnorm[(size_t)j * N + i] = re * re + im * im; /* std::norm */
        z->fphase[(size_t)j * N + i] = atan2(im, re);     /* std::arg */
    }
}

/* Freezer::write (fourier.h:448-466) */
static void frz_write(orc_frz* z, double sample) {
    const int N = z->N;
    for (int i = 0; i < z->M; i++) {
        const int spot = (z->origin - i * z->stride + z->size) % z->size;
        if (spot < N) {
            const double h = halfhann(spot / (double)N);
            z->fdata[(size_t)i * 2 * N + 2 * spot] = h * sample;
            z->fdata[(size_t)i * 2 * N + 2 * spot + 1] = h * 0.0;
        }
        if (spot == 0) fframe_process(z, (z->M + i - 1) % z->M);
    }
    z->origin = (z->origin + 1) % z->size;
}

void orc_frz_freeze(orc_frz* z) { /* fourier.h:468-479 */
    const int N = z->N;
    if (!z->frozen) {
        z->excluded = z->origin / z->stride;
        for (int i = 1; i < z->M - 1; i++) {
            const int d = (z->excluded + i) % z->M, s = (d + 1) % z->M;
            memcpy(z->dnorm + (size_t)d * N, z->fnorm + (size_t)s * N, sizeof(double) * N);
            for (int k = 0; k < N; k++)
                z->dphase[(size_t)d * N + k] = z->fphase[(size_t)s * N + k] - z->fphase[(size_t)d * N + k];
        }
    }
    z->readhead = 0;
    z->frozen = 1;
}

void orc_frz_unfreeze(orc_frz* z) { /* fourier.h:481-485 */
    z->frozen = 0;
    memset(z->vocoder, 0, sizeof(double) * z->N);
}

int orc_frz_frozen(orc_frz* z) { return z->frozen; }

/* Delay<double>(1, N) with forwards {(N, 1)}, backs {(0, 0)} (delay.h:71-89) */
static double delay_sample(orc_frz* z, double x) {
    const unsigned S = z->dsize, o = z->dorigin;
    z->din[o] = x;
    z->dout[o] = 0;
    /* Buffer::operator()(position) with an integer position: disp = 0 (buffer.h:40-47) */
    const double in_n = z->din[(o - (unsigned)z->N + S) % S] * (1 - 0.0) + z->din[(o - (unsigned)(z->N + 1) + S) % S] * 0.0;
    const double out_0 = z->dout[(o - 0u + S) % S] * (1 - 0.0) + z->dout[(o - 1u + S) % S] * 0.0;
    z->dout[o] += 1.0 * in_n - 0.0 * out_0;
    return z->dout[o];
}

double orc_frz_sample(orc_frz* z, double sample) { /* fourier.h:487-536 */
    const int N = z->N;
    frz_write(z, sample);
    double output = 0;
    if (z->frozen) {
        for (int i = 0; i < z->M; i++) {
            const int spot = (z->readhead - i * z->stride + z->readsize) % z->readsize;
            if (spot < N) output += z->idata[(size_t)z->iqueue[i] * 2 * N + 2 * spot] * halfhann(spot / (double)N);
            if (spot == 0) {
                int next = rand() % (z->M - 2);
                if (next >= z->excluded) next += 2;
                z->iindex = (z->iindex + 1) % z->M;
                z->iqueue[z->iindex] = next;
                for (int j = 0; j < N; j++) z->vocoder[j] = fmod(z->dphase[(size_t)next * N + j], 2 * ORC_PI);
                for (int j = 0; j < N; j++) { /* IFrame::populate: std::polar(sqrt(norm), phase) */
                    const double r = sqrt(z->dnorm[(size_t)next * N + j]);
                    z->tmp2[2 * j] = r * cos(z->vocoder[j]);
                    z->tmp2[2 * j + 1] = r * sin(z->vocoder[j]);
                }
                orc_dft(z->tmp2, z->idata + (size_t)next * 2 * N, N, +1);
            }
        }
        z->readhead = (z->readhead + 1) % z->readsize;
        output /= N;
    } else {
        output = delay_sample(z, sample);
    }
    z->dorigin = (z->dorigin + 1) % z->dsize; /* delay->tick() */
    return output;
}

/* n x { events with at == i (1 freeze, 0 unfreeze), in order; out[i] = operator()(in[i]) } */
void orc_frz_process(orc_frz* z, const double* in, double* out, long n, const long* at, const int* kind, int nev) {
    int k = 0;
    for (long i = 0; i < n; i++) {
        for (; k < nev && at[k] == i; k++) {
            if (kind[k]) orc_frz_freeze(z);
            else orc_frz_unfreeze(z);
        }
        out[i] = orc_frz_sample(z, in[i]);
    }
}
