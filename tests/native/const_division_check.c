/* The tracker's division by a constant divisor (tracker.hip div_const: q0 = x r, r = RN(1 / b), then one FMA
 * correction q0 + (x - q0 b) r) against IEEE division, on random normal operands: the reference's difference
 * quotients divide by h = 0.02 (hessian.h:160-171) and the lighting fit by the patch size W^2 (hessian.h:131-133).
 * Compiled with FMA contraction off, like tracker.hip.  Prints mismatches; exit 1 if any.  argv[1]: samples. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }

static double div_const_d(double x, double b, double r) {
  const double q0 = x * r;
  const double q = fma(fma(-q0, b, x), r, q0);
  return isinf(x) ? q0 : q;
}
static float div_const_f(float x, float b, float r) {
  const float q0 = x * r;
  const float q = fmaf(fmaf(-q0, b, x), r, q0);
  return isinf(x) ? q0 : q;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 2000000L;
  long bad = 0;
  const double h = 0.02, rh = 50.0;
  if (1.0 / h != rh) { printf("RN(1 / 0.02) != 50\n"); return 1; }
  for (long i = 0; i < n; ++i) {
    uint64_t u = xr();
    uint64_t bits = (u & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 60 + (u >> 52) % 120) << 52);
    double x;
    memcpy(&x, &bits, 8);
    if (div_const_d(x, h, rh) != x / h) {
      if (bad < 5) printf("double x=%.17g\n", x);
      ++bad;
    }
  }
  for (int W = 1; W <= 16; ++W) {
    const float L = (float)(W * W), rl = 1.0f / L;
    for (long i = 0; i < n / 8; ++i) {
      uint32_t u = (uint32_t)xr();
      uint32_t bits = (u & 0x807FFFFFu) | ((uint32_t)(127 - 40 + (u >> 23) % 80) << 23);
      float x;
      memcpy(&x, &bits, 4);
      if (div_const_f(x, L, rl) != x / L) {
        if (bad < 5) printf("float W=%d x=%.9g\n", W, x);
        ++bad;
      }
    }
  }
  const double inf = INFINITY;
  if (div_const_d(inf, h, rh) != inf / h || div_const_d(-inf, h, rh) != -inf / h || div_const_d(0.0, h, rh) != 0.0) ++bad;
  printf("%ld mismatches\n", bad);
  return bad ? 1 : 0;
}
