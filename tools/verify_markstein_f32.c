/* Randomised check that Markstein's correction reproduces IEEE binary64 division (round to nearest) for the
 * normalize_to_audio quotient t/R of FLOAT32 rasters: t = 2*((double)x - (double)mn), R = (double)mx - (double)mn
 * for float32 x, mn, mx with mn <= x <= mx (normalization.py:150-165 op order).  Markstein's theorem covers it
 * (y = RN(1/R), q0 = RN(t*y) within 1 ulp, r = t - q0*R exact by fma, no under/overflow for float32-derived t and R:
 * t/R >= 2^-278), this is the empirical check behind fra_device.h's division-free float32 normalisation (r06).
 * gcc -O2 -ffp-contract=off -fopenmp tools/verify_markstein_f32.c -lm -o /tmp/vmf && /tmp/vmf [millions] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static inline double mk(double t, double b, double y) {
  double q0 = t * y;
  double r = fma(-q0, b, t);
  return fma(r, y, q0);
}
static inline uint64_t xs(uint64_t *s) { *s ^= *s << 13; *s ^= *s >> 7; *s ^= *s << 17; return *s; }
static float f_of(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
/* a finite float from 32 random bits, exponent drawn from the whole range or a narrow one */
static float rnd_float(uint64_t *s, int mode) {
  uint32_t b = (uint32_t)xs(s);
  if (mode == 0) {              /* any finite float */
    uint32_t e = (b >> 23) & 0xFF;
    if (e == 0xFF) b &= ~(1u << 23);
    return f_of(b);
  }
  if (mode == 1) return f_of((b & 0x807FFFFFu) | ((uint32_t)(118 + (xs(s) % 12)) << 23));  /* ~[2^-9, 2^3): reflectance */
  if (mode == 2) return f_of((b & 0x007FFFFFu) | 0x7F7FFFFFu * 0 | ((uint32_t)(1 + xs(s) % 253) << 23)); /* normal, > 0 */
  return f_of(b & 0x807FFFFFu); /* subnormal or zero */
}
int main(int argc, char **argv) {
  const long long M = (argc > 1 ? atoll(argv[1]) : 1000) * 1000000ll;
  long long bad = 0, n = 0;
#pragma omp parallel reduction(+ : bad, n)
  {
    uint64_t s = 88172645463325252ull ^ (uint64_t)(uintptr_t)&s;
#pragma omp for schedule(static)
    for (long long i = 0; i < M; i++) {
      const int mode = (int)(i & 3);
      float a = rnd_float(&s, mode), b = rnd_float(&s, mode == 3 ? 1 : mode), c = rnd_float(&s, mode);
      if (isnan(a) || isnan(b) || isnan(c) || isinf(a) || isinf(b) || isinf(c)) continue;
      /* sort: mn <= x <= mx */
      float mn = fminf(a, fminf(b, c)), mx = fmaxf(a, fmaxf(b, c)), x = a + b + c - mn - mx;
      if (!(mn <= x && x <= mx)) x = (i & 4) ? mn : mx;
      if (i & 8) x = (i & 16) ? mx : mn;        /* the end points too */
      if (i % 97 == 0) mx = nextafterf(mn, INFINITY), x = (i & 32) ? mx : mn;  /* a range of one ulp */
      const double R = (double)mx - (double)mn;
      if (!(R > 0.0) || isinf(R)) continue;
      const double t = 2.0 * ((double)x - (double)mn);
      if (isinf(t)) continue;
      const double y = 1.0 / R;
      n++;
      if (mk(t, R, y) != t / R) bad++;
    }
  }
  printf("float32 quotients: %lld cases, %lld mismatches\n", n, bad);
  return bad ? 1 : 0;
}
