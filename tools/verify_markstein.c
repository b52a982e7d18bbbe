/* Exhaustive check that Markstein's reciprocal refinement reproduces IEEE binary64 division
 * (round-to-nearest) for the normalize_to_audio quotient t/R, t = 2*(x - mn), over every
 * integer range R in [1, 65535] and every t in [0, 2R] (the whole 16-bit raster domain), plus
 * random 32-bit-integer and float cases.  Used to justify fra_kernels.hip's division-free
 * normalisation.  gcc -O2 -ffp-contract=off -fopenmp verify_markstein.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
static inline double mk(double t, double b, double y) {
  double q0 = t * y;
  double r = fma(-q0, b, t);
  return fma(r, y, q0);
}
int main(void) {
  long long bad = 0, n = 0;
#pragma omp parallel for reduction(+ : bad, n) schedule(dynamic, 64)
  for (int R = 1; R <= 65535; R++) {
    const double b = (double)R, y = 1.0 / b;
    for (int t = 0; t <= 2 * R; t++) {
      const double tt = (double)t;
      if (mk(tt, b, y) != tt / b) bad++;
      n++;
    }
  }
  printf("16-bit exhaustive: %lld cases, %lld mismatches\n", n, bad);
  uint64_t s = 88172645463325252ull;
  long long bad2 = 0;
  for (long long i = 0; i < 200000000; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    double b, t;
    if (i & 1) { /* 32-bit integer ranges */
      uint64_t R = (s >> 20) & 0xFFFFFFFFull; if (!R) R = 1; b = (double)R;
      t = 2.0 * (double)((s * 0x9E3779B97F4A7C15ull) % (R + 1));
    } else {    /* float data: arbitrary doubles of float precision */
      float fa = (float)((double)(s >> 11) / 9007199254740992.0 * 2.0 - 1.0) * ldexpf(1.0f, (int)(s % 40) - 20);
      float fb = fabsf((float)((double)((s * 31) >> 11) / 9007199254740992.0)) * ldexpf(1.0f, (int)((s >> 7) % 40) - 20);
      if (fb == 0.0f) fb = 1.0f;
      double mn = -(double)fabsf(fa);
      t = 2.0 * ((double)fa - mn); b = (double)fb + (double)fabsf(fa);
    }
    double y = 1.0 / b;
    if (mk(t, b, y) != t / b) bad2++;
  }
  printf("random 32-bit/float: 200000000 cases, %lld mismatches\n", bad2);
  return (bad || bad2) ? 1 : 0;
}
