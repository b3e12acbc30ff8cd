/*
 * hz_oracle_dly.c -- TEST INFRASTRUCTURE ONLY (see hz_oracle.h).
 * Scalar restatement of Buffer<T> (src/buffer.h:9-86) and Delay<T> (src/delay.h:10-108),
 * and of the Delaybank<T,N> this build defines on top of them (N independent Delay<T>
 * lines): for T = double and T = float.
 *
 * Kept op-for-op, including the parts that only matter at the edges:
 *   - the interpolated read data[(origin - c + size) % size] * (1 - disp)
 *     + data[(origin - (c+1) + size) % size] * disp, with origin/size uint32 so the
 *     index expression wraps mod 2^32 before `% size` (buffer.h:40-47);
 *   - the tap position is a T (uint -> T -> (int)), so float rounds delays > 2^24;
 *   - taps accumulate into output[origin] in tap order, a feedback read of the current
 *     slot sees the partial sum (delay.h:71-89); zero-time feedback taps become {0,0}
 *     (delay.h:48-51, 64-67).
 * Delaybank mixdown (new): sum of the line outputs in line order, in T, divided by N.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hz_oracle.h"

#define DEFINE_LINE(T, SUF)                                                                  \
    typedef struct {                                                                         \
        T* in;                                                                               \
        T* out;                                                                              \
        uint32_t size, origin;                                                               \
        uint32_t* ft;                                                                        \
        T* fg;                                                                               \
        uint32_t* bt;                                                                        \
        T* bg;                                                                               \
    } line_##SUF;                                                                            \
    static T buf_read_##SUF(const T* data, uint32_t size, uint32_t origin, T position) {     \
        int center = (int)position;                                                          \
        int before = center + 1;                                                             \
        T disp = position - center;                                                          \
        return data[(origin - center + size) % size] * (1 - disp) +                          \
               data[(origin - before + size) % size] * disp;                                 \
    }                                                                                        \
    static T line_step_##SUF(line_##SUF* L, uint32_t S, T x) {                               \
        L->in[L->origin] = x;    /* input.write(sample) */                                   \
        L->out[L->origin] = 0;   /* output.write(0) */                                       \
        for (uint32_t i = 0; i < S; i++) {                                                   \
            T v = L->fg[i] * buf_read_##SUF(L->in, L->size, L->origin, (T)L->ft[i]) -        \
                  L->bg[i] * buf_read_##SUF(L->out, L->size, L->origin, (T)L->bt[i]);        \
            L->out[L->origin] += v; /* output.accum */                                       \
        }                                                                                    \
        T y = buf_read_##SUF(L->out, L->size, L->origin, (T)0);                              \
        L->origin = (L->origin + 1) % L->size; /* tick() on both rings */                    \
        return y;                                                                            \
    }

DEFINE_LINE(double, d)
DEFINE_LINE(float, f)

struct orc_dly {
    int N, is_float;
    uint32_t S, size;
    line_d* ld;
    line_f* lf;
};

orc_dly* orc_dly_create(int lines, unsigned sparsity, unsigned time, int is_float) {
    orc_dly* b = (orc_dly*)calloc(1, sizeof(orc_dly));
    b->N = lines;
    b->is_float = is_float;
    b->S = sparsity;
    b->size = time + 1u;             /* Delay(sparsity, time) : input(time + 1) */
    if (b->size == 0) b->size = 1;   /* Buffer::initialize: disallow size zero */
    if (is_float) {
        b->lf = (line_f*)calloc(lines, sizeof(line_f));
        for (int k = 0; k < lines; k++) {
            line_f* L = &b->lf[k];
            L->size = b->size;
            L->in = (float*)calloc(b->size, sizeof(float));
            L->out = (float*)calloc(b->size, sizeof(float));
            L->ft = (uint32_t*)calloc(sparsity + 1, sizeof(uint32_t));
            L->bt = (uint32_t*)calloc(sparsity + 1, sizeof(uint32_t));
            L->fg = (float*)calloc(sparsity + 1, sizeof(float));
            L->bg = (float*)calloc(sparsity + 1, sizeof(float));
        }
    } else {
        b->ld = (line_d*)calloc(lines, sizeof(line_d));
        for (int k = 0; k < lines; k++) {
            line_d* L = &b->ld[k];
            L->size = b->size;
            L->in = (double*)calloc(b->size, sizeof(double));
            L->out = (double*)calloc(b->size, sizeof(double));
            L->ft = (uint32_t*)calloc(sparsity + 1, sizeof(uint32_t));
            L->bt = (uint32_t*)calloc(sparsity + 1, sizeof(uint32_t));
            L->fg = (double*)calloc(sparsity + 1, sizeof(double));
            L->bg = (double*)calloc(sparsity + 1, sizeof(double));
        }
    }
    return b;
}

void orc_dly_destroy(orc_dly* b) {
    if (!b) return;
    for (int k = 0; k < b->N; k++) {
        if (b->is_float) {
            line_f* L = &b->lf[k];
            free(L->in); free(L->out); free(L->ft); free(L->bt); free(L->fg); free(L->bg);
        } else {
            line_d* L = &b->ld[k];
            free(L->in); free(L->out); free(L->ft); free(L->bt); free(L->fg); free(L->bg);
        }
    }
    free(b->lf);
    free(b->ld);
    free(b);
}

static void set_tap(orc_dly* b, int line, int back, unsigned i, unsigned t, double g) {
    if (back && t == 0) g = 0; /* zero-time feedback -> {0,0} */
    if (b->is_float) {
        line_f* L = &b->lf[line];
        (back ? L->bt : L->ft)[i] = t;
        (back ? L->bg : L->fg)[i] = (float)g;
    } else {
        line_d* L = &b->ld[line];
        (back ? L->bt : L->ft)[i] = t;
        (back ? L->bg : L->fg)[i] = g;
    }
}

/* delay.h:37-56 */
void orc_dly_coefficients(orc_dly* b, int line, const unsigned* ft, const double* fg, int nf,
                          const unsigned* bt, const double* bg, int nb) {
    for (unsigned i = 0; i < b->S; i++) {
        if ((int)i < nf) set_tap(b, line, 0, i, ft[i], fg[i]);
        else set_tap(b, line, 0, i, 0, 0);
        if ((int)i < nb) set_tap(b, line, 1, i, bt[i], bg[i]);
        else set_tap(b, line, 1, i, 0, 0);
    }
}

/* delay.h:59-68 */
void orc_dly_modulate_forward(orc_dly* b, int line, unsigned n, unsigned t, double g) { set_tap(b, line, 0, n, t, g); }
void orc_dly_modulate_back(orc_dly* b, int line, unsigned n, unsigned t, double g) { set_tap(b, line, 1, n, t, g); }

/* one sample per line per step: y_k = line_k(x_k); tick().  in: mono (in_per_line 0) or
 * line-major [N][n]; out: line-major [N][n] (mix 0) or the mixdown [n] (mix 1). */
void orc_dly_process(orc_dly* b, const void* in, void* out, long n, int in_per_line, int mix) {
    const int N = b->N;
    for (long t = 0; t < n; t++) {
        if (b->is_float) {
            const float* x = (const float*)in;
            float* y = (float*)out;
            float s = 0;
            for (int k = 0; k < N; k++) {
                float v = line_step_f(&b->lf[k], b->S, x[in_per_line ? (long)k * n + t : t]);
                if (mix) s += v;
                else y[(long)k * n + t] = v;
            }
            if (mix) y[t] = s / (float)N;
        } else {
            const double* x = (const double*)in;
            double* y = (double*)out;
            double s = 0;
            for (int k = 0; k < N; k++) {
                double v = line_step_d(&b->ld[k], b->S, x[in_per_line ? (long)k * n + t : t]);
                if (mix) s += v;
                else y[(long)k * n + t] = v;
            }
            if (mix) y[t] = s / (double)N;
        }
    }
}

/* tick() without operator() (delay.h:92-97): input.tick(); output.tick() -- the origins move,
 * nothing is written */
void orc_dly_tick(orc_dly* b, unsigned long count) {
    for (unsigned long c = 0; c < count; c++)
        for (int k = 0; k < b->N; k++) {
            if (b->is_float) b->lf[k].origin = (b->lf[k].origin + 1) % b->lf[k].size;
            else b->ld[k].origin = (b->ld[k].origin + 1) % b->ld[k].size;
        }
}

unsigned orc_dly_origin(orc_dly* b) { return b->is_float ? b->lf[0].origin : b->ld[0].origin; }
