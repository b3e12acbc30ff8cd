/*
 * hz_oracle_osc.c -- TEST INFRASTRUCTURE ONLY (see hz_oracle.h).
 * Scalar restatement of Oscillator<T>/Synth<T>, Sinusoids<T> and Additive<T>
 * (+ the Minimizer note API it inherits), op for op.  Physics (Minimizer::physics,
 * src/minimizer.h:61-108) is out of scope and never called, so particle positions stay
 * where request() puts them.  abs() is taken as fabs (macOS libc++).
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hz_oracle.h"

#define ORC_PI 3.14159265359
#define ORC_SR 48000

/* ---- Oscillator<double>  src/oscillator.h:12-71 --------------------------- */
typedef struct {
    double phase, frequency, target_freq, target_phase, stiffness;
} osc_t;

/* oscillator.h:16-24 */
static void osc_init(osc_t* o, double f, double phi, double k)
{
    o->frequency = fabs(f);
    o->target_freq = o->frequency;
    o->phase = fmax(0, phi);
    o->target_phase = o->phase;
    o->stiffness = orc_relaxation(k);
}

/* cycle = sin(2 PI p), src/wave.h:147 (FUNCTIONAL lookup) */
static double cycle(double p) { return sin(2 * ORC_PI * p); }

/* oscillator.h:27-38 */
static void osc_tick(osc_t* o)
{
    o->phase += o->frequency / ORC_SR;
    o->target_phase += o->frequency / ORC_SR;
    o->frequency = o->target_freq * (1 - o->stiffness) + o->frequency * o->stiffness;
    double weight = (1 - o->stiffness) * cycle(2 * fabs(o->target_phase - o->phase) + 0.25);
    o->phase = weight * o->target_phase + (1 - weight) * o->phase;
    o->phase -= (int)o->phase;
    o->target_phase -= (int)o->target_phase;
}

/* ---- Additive<double>  src/additive.h:11-71, src/minimizer.h:23-206 ------- */
struct orc_add {
    int V, O;
    double decay, harmonicity, attack, normalization;
    osc_t* osc;          /* V*O */
    double* amplitudes;  /* V */
    double* active;      /* Minimizer::active (T) */
    double* pitches;
    double* guide;       /* guides[v].position */
    double* position;    /* particles[v*O+j].position */
};

orc_add* orc_add_create(int voices, int overtones, double decay, double harmonicity, double k)
{
    orc_add* a = (orc_add*)calloc(1, sizeof(orc_add));
    a->V = voices; a->O = overtones; a->decay = decay; a->harmonicity = harmonicity;
    a->attack = orc_relaxation(k);                                              /* additive.h:25 */
    a->normalization = decay != 1 ? (1 - pow(decay, overtones)) / (1 - decay) : overtones; /* 27 */
    a->osc = (osc_t*)calloc((size_t)voices * overtones, sizeof(osc_t));
    for (int i = 0; i < voices * overtones; i++) osc_init(&a->osc[i], 0, 0, 0.0001); /* 35 */
    a->amplitudes = (double*)calloc(voices, sizeof(double));
    a->active = (double*)calloc(voices, sizeof(double));
    a->pitches = (double*)calloc(voices, sizeof(double));
    a->guide = (double*)calloc(voices, sizeof(double));
    a->position = (double*)calloc((size_t)voices * overtones, sizeof(double));
    return a;
}

void orc_add_destroy(orc_add* a)
{
    if (!a) return;
    free(a->osc); free(a->amplitudes); free(a->active); free(a->pitches); free(a->guide); free(a->position);
    free(a);
}

/* minimizer.h:111-158 */
int orc_add_request(orc_add* a, double fundamental, double amplitude)
{
    int voice = -1;
    for (int i = 0; i < a->V; i++)
        if (!a->active[i]) { voice = i; break; }
    if (voice < 0) {
        double pitch = orc_ftom(fundamental);
        double distance = 0;
        int nearest = -1;
        for (int i = 0; i < a->V; i++) {
            double offset = pitch - a->guide[i];
            offset *= offset;
            if (nearest < 0 || offset < distance) { nearest = i; distance = offset; }
        }
        voice = nearest;
    }
    double frequency = fundamental;
    a->active[voice] = amplitude;
    a->guide[voice] = orc_ftom(fundamental);
    for (int j = 0; j < a->O; j++) {
        frequency = fundamental * (1 + pow((double)j / (a->O - 1), a->harmonicity) * (a->O - 1));
        a->position[voice * a->O + j] = orc_ftom(frequency);
    }
    return voice;
}

/* minimizer.h:161-172 */
void orc_add_release(orc_add* a, int voice)
{
    if (voice >= 0) { a->active[voice] = 0; return; }
    for (int i = 0; i < a->V; i++) a->active[i] = 0;
}

/* minimizer.h:174-187 */
int orc_add_makenote(orc_add* a, double pitch, double amplitude)
{
    int voice = orc_add_request(a, orc_mtof(pitch), amplitude);
    if (voice >= 0) a->pitches[voice] = pitch;
    return voice;
}

void orc_add_endnote(orc_add* a, double pitch)
{
    for (int j = 0; j < a->V; j++)
        if (a->pitches[j] == pitch) orc_add_release(a, j);
}

/* additive.h:53-62 */
double orc_add_sample(orc_add* a)
{
    double sample = 0;
    for (int i = 0; i < a->V; i++)
        if (a->amplitudes[i])
            for (int j = 0; j < a->O; j++)
                sample += a->amplitudes[i] * pow(a->decay, j) * cycle(a->osc[i * a->O + j].phase) /
                          (a->V * a->normalization);
    return sample;
}

/* additive.h:38-51 */
void orc_add_tick(orc_add* a)
{
    for (int i = 0; i < a->V; i++) a->amplitudes[i] = (1 - a->attack) * a->active[i] + a->attack * a->amplitudes[i];
    for (int i = 0; i < a->V; i++)
        if (a->active[i] || a->amplitudes[i])
            for (int j = 0; j < a->O; j++) {
                a->osc[i * a->O + j].target_freq = orc_mtof(a->position[i * a->O + j]);
                osc_tick(&a->osc[i * a->O + j]);
            }
}

/* tests/additive.cpp:27-37 without physics */
void orc_add_fill(orc_add* a, double* out, long n)
{
    for (long t = 0; t < n; t++) {
        out[t] = orc_add_sample(a);
        orc_add_tick(a);
    }
}

/* ---- Sinusoids<double>  src/sinusoids.h:10-79 ----------------------------- */
struct orc_sin {
    int O;
    double fundamental, target_fundamental, harmonicity, target_harmonicity, decay, target_decay;
    double normalization, stiffness;
    osc_t* synths;
};

orc_sin* orc_sin_create(double fundamental, int overtones, double decay, double harmonicity, double k)
{
    orc_sin* s = (orc_sin*)calloc(1, sizeof(orc_sin));
    s->fundamental = s->target_fundamental = fundamental;
    s->harmonicity = s->target_harmonicity = harmonicity;
    s->O = overtones;
    s->decay = s->target_decay = decay;
    s->synths = (osc_t*)calloc(overtones, sizeof(osc_t));
    for (int i = 0; i < overtones; i++)           /* Synth(form, f) with k = 2.0/SR */
        osc_init(&s->synths[i], fundamental * pow(i + 1, harmonicity), 0, 2.0 / ORC_SR);
    s->normalization = decay != 1 ? (1 - pow(decay, overtones)) / (1 - decay) : overtones;
    s->stiffness = orc_relaxation(k);
    return s;
}

void orc_sin_destroy(orc_sin* s)
{
    if (!s) return;
    free(s->synths);
    free(s);
}

void orc_sin_fundmod(orc_sin* s, double t) { s->target_fundamental = t; }
void orc_sin_decaymod(orc_sin* s, double t) { s->target_decay = t; }
void orc_sin_harmmod(orc_sin* s, double t) { s->target_harmonicity = t; }

/* sinusoids.h:34-41 */
double orc_sin_sample(orc_sin* s)
{
    double sample = 0;
    for (int i = 0; i < s->O; i++) sample += pow(s->decay, i) * cycle(s->synths[i].phase) / s->normalization;
    return sample;
}

/* sinusoids.h:43-57 */
void orc_sin_tick(orc_sin* s)
{
    double k = s->stiffness;
    s->fundamental = s->target_fundamental * (1 - k) + s->fundamental * k;
    s->decay = s->target_decay * (1 - k) + s->decay * k;
    s->harmonicity = s->target_harmonicity * (1 - k) + s->harmonicity * k;
    for (int i = 0; i < s->O; i++) {
        s->synths[i].target_freq = s->fundamental * pow(i + 1, s->harmonicity);
        osc_tick(&s->synths[i]);
    }
    s->normalization = s->decay != 1 ? (1 - pow(s->decay, s->O)) / (1 - s->decay) : s->O;
}

void orc_sin_fill(orc_sin* s, double* out, long n)
{
    for (long t = 0; t < n; t++) {
        out[t] = orc_sin_sample(s);
        orc_sin_tick(s);
    }
}
