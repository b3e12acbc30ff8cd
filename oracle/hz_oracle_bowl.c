/*
 * hz_oracle_bowl.c -- TEST INFRASTRUCTURE ONLY (see hz_oracle.h).
 * Scalar restatement of Bowl<T> (src/bowl.h:10-74) for T = double and T = float.
 *
 * Bowl<float> mixes precisions exactly as the reference does:
 *   -d[i]*phase/SR and f[i]*phase/SR are float ops (phase is a float counter),
 *   pow(E, float) is evaluated in double, form is a Wave<float> whose lambda takes a
 *   double and returns float (sin(2 PI p) in double, rounded to float), the products are
 *   double and `sample += ...` rounds back to float on every term (bowl.h:54-59).
 * The default form &cycle is a Wave<double> and does not compile for T = float
 * (SURVEY.md 0.12); config C5 supplies cycle_f = Wave<float>(sin(2 PI p)), restated here.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hz_oracle.h"

#define ORC_PI 3.14159265359
#define ORC_E 2.718281828459045
#define ORC_SR 48000

struct orc_bowl {
    int M, is_float;
    double *f, *a, *d;        /* double model */
    float *ff, *af, *df;      /* float model */
    double phase;             /* Bowl<double>::phase */
    float phasef;             /* Bowl<float>::phase */
};

orc_bowl* orc_bowl_create(int overtones, const double* f, const double* a, const double* d, int count,
                          int is_float)
{
    orc_bowl* b = (orc_bowl*)calloc(1, sizeof(orc_bowl));
    b->M = overtones;
    b->is_float = is_float;
    b->f = (double*)calloc(overtones, sizeof(double));
    b->a = (double*)calloc(overtones, sizeof(double));
    b->d = (double*)calloc(overtones, sizeof(double));
    b->ff = (float*)calloc(overtones, sizeof(float));
    b->af = (float*)calloc(overtones, sizeof(float));
    b->df = (float*)calloc(overtones, sizeof(float));
    for (int i = 0; i < overtones && i < count; i++) {  /* resize(overtones, 0), bowl.h:19-22 */
        b->f[i] = f[i]; b->a[i] = a[i]; b->d[i] = d[i];
        b->ff[i] = (float)f[i]; b->af[i] = (float)a[i]; b->df[i] = (float)d[i];
    }
    return b;
}

void orc_bowl_destroy(orc_bowl* b)
{
    if (!b) return;
    free(b->f); free(b->a); free(b->d); free(b->ff); free(b->af); free(b->df); free(b);
}

void orc_bowl_trigger(orc_bowl* b) { b->phase = 0; b->phasef = 0; }   /* bowl.h:25-28 */

/* the state after trigger() and `ticks` samples: the phase counter alone (bowl.h:42-47, 61:
 * phase++ from 0, exact in float below 2^24), so time segments of one signal can be restated
 * independently (tests/test_fullsize_gpu.py) */
void orc_bowl_seek(orc_bowl* b, long ticks) {
    b->phase = 0; b->phasef = 0;
    if (ticks < (1L << 24)) { b->phase = (double)ticks; b->phasef = (float)ticks; return; }
    for (long j = 0; j < ticks; j++) { b->phase++; b->phasef++; }
}

/* bowl.h:35-36 / 55-56, T = double, form = cycle (wave.h:147) */
static double sample_d(orc_bowl* b)
{
    double s = 0;
    for (int i = 0; i < b->M; i++)
        s += b->a[i] * pow(ORC_E, -b->d[i] * b->phase / ORC_SR) * sin(2 * ORC_PI * (b->f[i] * b->phase / ORC_SR));
    return s;
}

/* T = float: see the header comment */
static float cycle_f(double p) { return (float)sin(2 * ORC_PI * p); }
static float sample_f(orc_bowl* b)
{
    float s = 0;
    for (int i = 0; i < b->M; i++) {
        float ex = -b->df[i] * b->phasef / (float)ORC_SR;
        float ph = b->ff[i] * b->phasef / (float)ORC_SR;
        double term = b->af[i] * pow(ORC_E, (double)ex) * cycle_f((double)ph);
        s = (float)((double)s + term);
    }
    return s;
}

/* fill(float* buffer, int bsize)  bowl.h:50-63 */
int orc_bowl_fill(orc_bowl* b, float* buffer, long bsize)
{
    for (long j = 0; j < bsize; j++) {
        if (b->is_float) {
            buffer[j] = sample_f(b);
            b->phasef++;
        } else {
            buffer[j] = (float)sample_d(b);
            b->phase++;
        }
    }
    return 0;
}

/* n x { out[j] = operator()(); tick(); }  (bowl.h:30-48) in T's precision, widened */
void orc_bowl_render(orc_bowl* b, double* out, long n)
{
    for (long j = 0; j < n; j++) {
        if (b->is_float) {
            out[j] = sample_f(b);
            b->phasef++;
        } else {
            out[j] = sample_d(b);
            b->phase++;
        }
    }
}
