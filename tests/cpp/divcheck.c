/* divcheck.c -- host check of the FMA-corrected quotients used by the HIP kernels
 * (test infrastructure, run by tests/test_divcheck_cpu.py).
 *
 *   cdiv_one (huygens_amd/csrc/hz_fb_tv.hip): the two quotients of libgcc's Smith divide
 *       (__divdc3, the complex divide of subtractive.h:240-249's resonant()) for numerator 1,
 *       from ONE correctly rounded reciprocal r = RN(1/den): -1/den = -r exactly, and
 *       ratio/den = RN(q0 + RN(ratio - den q0) r), q0 = RN(ratio r).
 *   div_sr   (hz_fb_tv.hip, hz_bowl.hip): x / 48000 as RN(q0 + RN(x - 48000 q0) / 48000).
 *
 * Each is compared bit for bit with the IEEE quotient over random inputs: the resonant()
 * operand range (c = Q - cos(4 PI f / SR), d = -sin(4 PI f / SR)) and generic random
 * exponents.  Prints "trials mismatches" per case and exits 1 on any mismatch.
 * Build: gcc -O2 -ffp-contract=off divcheck.c -lm (glibc fma() is correctly rounded).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64(void) { /* splitmix64 */
    uint64_t z = (s_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double unif(void) { return (double)(next_u64() >> 11) * 0x1p-53; }
/* random double with a random exponent in [emin, emax] and a random sign */
static double rnd_exp(int emin, int emax) {
    uint64_t m = next_u64() & ((1ull << 52) - 1);
    int e = emin + (int)(next_u64() % (uint64_t)(emax - emin + 1));
    double v = ldexp(1.0 + (double)m * 0x1p-52, e);
    return (next_u64() & 1) ? -v : v;
}
static int same(double a, double b) { return memcmp(&a, &b, sizeof a) == 0 || (a == 0 && b == 0); }

static void cdiv_ref(double c, double d, double *x, double *y) { /* Smith, numerator (1, 0) */
    const double a = 1.0, b = 0.0;
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
static void cdiv_one(double c, double d, double *x, double *y) { /* as in hz_fb_tv.hip */
    const int lt = fabs(c) < fabs(d);
    const double ratio = lt ? c / d : d / c;
    const double den = lt ? (c * ratio) + d : (d * ratio) + c;
    const double r = 1.0 / den;
    const double q0 = ratio * r;
    const double q = fma(fma(-q0, den, ratio), r, q0);
    *x = lt ? q : r;
    *y = lt ? -r : -q;
}
static double div_sr(double x) {
    const double inv = 1.0 / 48000.0;
    const double q = x * inv;
    return fma(fma(-q, 48000.0, x), inv, q);
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 20000000L;
    const double PI = 3.14159265359;
    long bad_res = 0, bad_gen = 0, bad_sr = 0;
    for (long i = 0; i < n; ++i) {
        double x0, y0, x1, y1;
        /* resonant(): Q in [0.5, 1), frequency in [0, SR/2) */
        const double Q = 0.5 + 0.5 * unif() * (1.0 - 0x1p-40);
        const double f = 24000.0 * unif();
        const double c = Q - cos(4 * PI * f / 48000.0), d = -0.0 - sin(4 * PI * f / 48000.0);
        cdiv_ref(c, d, &x0, &y0);
        cdiv_one(c, d, &x1, &y1);
        if (!same(x0, x1) || !same(y0, y1)) {
            if (bad_res < 5) printf("resonant mismatch c=%a d=%a: %a %a vs %a %a\n", c, d, x0, y0, x1, y1);
            ++bad_res;
        }
        /* generic operands, exponents kept away from overflow / subnormal quotients */
        const double cg = rnd_exp(-200, 200), dg = rnd_exp(-200, 200);
        cdiv_ref(cg, dg, &x0, &y0);
        cdiv_one(cg, dg, &x1, &y1);
        if (!same(x0, x1) || !same(y0, y1)) {
            if (bad_gen < 5) printf("generic mismatch c=%a d=%a: %a %a vs %a %a\n", cg, dg, x0, y0, x1, y1);
            ++bad_gen;
        }
        const double xs = fabs(rnd_exp(-900, 900));
        if (!same(div_sr(xs), xs / 48000.0)) {
            if (bad_sr < 5) printf("div_sr mismatch x=%a\n", xs);
            ++bad_sr;
        }
    }
    /* hard cases for the one-step correction: quotient mantissa near 2 (q0 = RN(ratio r) can be
     * ~1.5 ulp off there) and reciprocals with a rounding error near 1/2 ulp */
    long hard = 0, bad_hard = 0;
    for (long i = 0; i < 8 * n; ++i) {
        const double den = 1.0 + unif(), r = 1.0 / den;
        if (fabs(fma(-den, r, 1.0)) < 0x1p-54) continue;
        const double ratio = den * (2.0 - unif() * 0x1p-8) * 0.5;
        const double q0 = ratio * r, q = fma(fma(-q0, den, ratio), r, q0), ref = ratio / den;
        ++hard;
        if (!same(q, ref)) {
            if (bad_hard < 5) printf("hard mismatch ratio=%a den=%a\n", ratio, den);
            ++bad_hard;
        }
    }
    printf("cdiv_one hard %ld %ld\n", hard, bad_hard);
    printf("cdiv_one resonant %ld %ld\n", n, bad_res);
    printf("cdiv_one generic %ld %ld\n", n, bad_gen);
    printf("div_sr generic %ld %ld\n", n, bad_sr);
    return (bad_res || bad_gen || bad_sr || bad_hard) ? 1 : 0;
}
