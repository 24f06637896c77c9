// div_check.c -- Markstein division (q0 = a y, e = fma(-q0, b, a), q = fma(e, y, q0), y = 1/b)
// against IEEE division, bit for bit (linesweep.hip line2_div).  gcc -O2 -ffp-contract=off -mfma div_check.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double mk(double a, double b) {
  double y = 1.0 / b;
  double q0 = a * y;
  double e = fma(-q0, b, a);
  return fma(e, y, q0);
}
static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
int main(void) {
  long bad = 0, n = 0;
  for (long i = 0; i < 400000000L; i++) {
    uint64_t ma = rnd() & 0xFFFFFFFFFFFFFull, mb = rnd() & 0xFFFFFFFFFFFFFull;
    int mode = i & 7;
    if (mode == 1) mb = 0xFFFFFFFFFFFFFull;           // b significand all ones
    if (mode == 2) mb = 0xFFFFFFFFFFFFFull ^ (rnd() & 0xFF);
    if (mode == 3) ma = 0xFFFFFFFFFFFFFull;
    if (mode == 4) mb = rnd() & 0xFF;                  // b near a power of two
    if (mode == 5) ma = rnd() & 0xFF;
    int ea = 1023 + (int)(rnd() % 801) - 400, eb = 1023 + (int)(rnd() % 801) - 400; if (i & 8) { ea = 1023 + (int)(rnd() % 60) - 30; eb = 1023 + (int)(rnd() % 60) - 30; }
    double a = bits(((uint64_t)ea << 52) | ma), b = bits(((uint64_t)eb << 52) | mb);
    if (rnd() & 1) a = -a;
    if (rnd() & 1) b = -b;
    double q = a / b, m = mk(a, b);
    n++;
    if (memcmp(&q, &m, 8)) { if (bad < 10) printf("a=%a b=%a q=%a m=%a\n", a, b, q, m); bad++; }
  }
  printf("%ld / %ld mismatches\n", bad, n);
  return 0;
}
