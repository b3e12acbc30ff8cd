/*
 * hz_oracle_gran.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Scalar restatement of Granulator<double> (src/granulator.h:12-127) reading a
 * Buffer<double> source (src/buffer.h:9-86) through the FUNCTIONAL hann window
 * (src/wave.h:65-70,148), in the per-sample order of tests/granny.cpp:34-56:
 *   source.write(x); y = granny(); <requests>; source.tick(); granny.tick();
 * Parity: unpinned by the reference's own files (no fixtures or known answers for
 * this class); pinned here by tests/test_granulator_cpu.py's closed-form cases.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "hz_oracle.h"

#define ORC_PI 3.14159265359 /* src/includes.h:30 */
#define ORC_SR 48000         /* src/includes.h:32 */

struct orc_gran {
    unsigned polyphony, activity;
    /* Buffer<double> (src/buffer.h:19-26): size 0 becomes 1 */
    double* data;
    unsigned size, origin;
    unsigned* ticks;
    double *offsets, *sizes, *speeds, *gains, *pans;
    unsigned char* active;
};

orc_gran* orc_gran_create(unsigned polyphony, unsigned buffer_size) {
    orc_gran* g = (orc_gran*)calloc(1, sizeof(orc_gran));
    g->polyphony = polyphony;
    g->size = buffer_size + (buffer_size == 0 ? 1 : 0);
    g->data = (double*)calloc(g->size, sizeof(double));
    g->ticks = (unsigned*)calloc(polyphony ? polyphony : 1, sizeof(unsigned));
    g->offsets = (double*)calloc(polyphony ? polyphony : 1, sizeof(double));
    g->sizes = (double*)calloc(polyphony ? polyphony : 1, sizeof(double));
    g->speeds = (double*)calloc(polyphony ? polyphony : 1, sizeof(double));
    g->gains = (double*)calloc(polyphony ? polyphony : 1, sizeof(double));
    g->pans = (double*)calloc(polyphony ? polyphony : 1, sizeof(double));
    g->active = (unsigned char*)calloc(polyphony ? polyphony : 1, 1);
    return g;
}

void orc_gran_destroy(orc_gran* g) {
    if (!g) return;
    free(g->data);
    free(g->ticks);
    free(g->offsets);
    free(g->sizes);
    free(g->speeds);
    free(g->gains);
    free(g->pans);
    free(g->active);
    free(g);
}

/* granulator.h:51-79; returns the voice, or -1 ((uint)-1 in the reference) */
int orc_gran_request(orc_gran* g, double offset, double size, double speed, double gain, double pan) {
    if (size == 0) return -1;
    const double lo = size * (speed - 1);
    offset = (offset < lo) ? lo : offset; /* std::max(offset, lo) */
    int voice = -1;
    for (int i = 0; i < (int)g->polyphony; i++)
        if (!g->active[i]) {
            voice = i;
            break;
        }
    if (voice >= 0) {
        g->offsets[voice] = ORC_SR * offset;
        g->sizes[voice] = ORC_SR * size;
        g->speeds[voice] = speed;
        g->gains[voice] = gain;
        g->pans[voice] = pan;
        g->active[voice] = 1;
        g->activity++;
        g->ticks[voice] = 0;
    }
    return voice;
}

void orc_gran_write(orc_gran* g, double x) { g->data[g->origin] = x; } /* buffer.h:59-62 */

/* buffer.h:40-47: unsigned origin/size, so origin - center wraps mod 2^32 before % size */
static double buffer_read(const orc_gran* g, double position) {
    const int center = (int)position;
    const int before = center + 1;
    const double disp = position - center;
    return g->data[(g->origin - (unsigned)center + g->size) % g->size] * (1 - disp) +
           g->data[(g->origin - (unsigned)before + g->size) % g->size] * disp;
}

static double hann(double phase) { return 0.5 * (1 - cos(2 * ORC_PI * phase)); } /* wave.h:148 */

/* granulator.h:88-104 */
double orc_gran_sample(orc_gran* g) {
    double out = 0;
    for (unsigned i = 0; i < g->polyphony; i++)
        if (g->active[i]) {
            const double phase = (double)g->ticks[i] / g->sizes[i];
            out += g->gains[i] * buffer_read(g, g->offsets[i] + (1 - g->speeds[i]) * g->ticks[i]) * hann(phase);
            if (g->ticks[i] >= g->sizes[i]) {
                g->active[i] = 0;
                g->activity--;
            }
        }
    return out;
}

/* source.tick() (buffer.h:33-37) then granny.tick() (granulator.h:81-86) */
void orc_gran_tick(orc_gran* g) {
    g->origin++;
    g->origin %= g->size;
    for (unsigned i = 0; i < g->polyphony; i++)
        if (g->active[i]) g->ticks[i]++;
}

unsigned orc_gran_activity(orc_gran* g) { return g->activity; }

void orc_gran_process(orc_gran* g, const double* in, double* out, long n, const long* at, const double* req,
                      int nreq, int* voices) {
    int k = 0;
    for (long i = 0; i < n; i++) {
        orc_gran_write(g, in[i]);
        out[i] = orc_gran_sample(g);
        for (; k < nreq && at[k] == i; k++) {
            const int v = orc_gran_request(g, req[5 * k], req[5 * k + 1], req[5 * k + 2], req[5 * k + 3], req[5 * k + 4]);
            if (voices) voices[k] = v;
        }
        orc_gran_tick(g);
    }
}
