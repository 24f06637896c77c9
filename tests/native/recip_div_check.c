/* The line sweeps' division a / b from y = RN(1/b) (lssp_amd/csrc/linesweep_dev.h
 * div_rcp): q0 = RN(a y), two corrections q = fma(fma(-b, q, a), y, q).  Checks
 * it against IEEE a / b, bit for bit, on random and adversarial operands within
 * the fast path's range (|a|, |y| in [2^-500, 2^500]); prints the mismatches.
 * Test infrastructure only (tests/test_recip_div.py builds and runs it). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static double fb(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static uint64_t bf(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }
static double mk(int emin, int emax, uint64_t mant)
{
    const int e = emin + (int)(rnd() % (uint64_t)(emax - emin + 1));
    return fb(((uint64_t)(e + 1023) << 52) | (mant & ((1ull << 52) - 1)) | ((rnd() & 1) << 63));
}
static double div_rcp(double a, double b, double y)
{
    const double q0 = a * y;
    const double q1 = fma(fma(-b, q0, a), y, q0);
    return fma(fma(-b, q1, a), y, q1);
}
int main(int argc, char **argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 20000000L;
    long bad = 0;
    for (long i = 0; i < n; i++) {
        double a, b;
        switch (i % 5) {
        case 0: a = mk(-480, 480, rnd()); b = mk(-480, 480, rnd()); break;
        case 1: a = mk(-3, 3, rnd()); b = mk(-3, 3, rnd()); break;
        case 2: /* quotients next to integers */
            b = mk(-20, 20, rnd());
            a = b * (double)(rnd() % 1000000 + 1);
            a = fb(bf(a) + (uint64_t)(rnd() % 5) - 2);
            break;
        case 3: /* divisor significands of (nearly) all ones */
            b = mk(-8, 8, ~(1ull << (rnd() % 64)));
            a = mk(-8, 8, rnd());
            break;
        default: /* dividend significands of nearly all ones */
            a = mk(-8, 8, ~(rnd() & 0xFF));
            b = mk(-8, 8, rnd());
        }
        const double y = 1.0 / b;
        if (bf(div_rcp(a, b, y)) != bf(a / b)) {
            if (bad < 5) printf("mismatch a=%a b=%a\n", a, b);
            bad++;
        }
    }
    printf("%ld %ld\n", n, bad);
    return 0;
}
