/* Exhaustive check of the rotation fast path (wk_device.h sincos_small): for every float
 * x with |x| <= 0.25, (float) of the double Taylor/Horner evaluation equals (float) of the
 * C library's double sin/cos -- the reference's (float)Math.Sin/Cos((double)angle) in
 * XNA's CreateRotationZ, restated by the oracle with glibc.  Odd/even symmetry makes the
 * positive half sufficient (the evaluation negates exactly).
 *   gcc -O2 -fopenmp -ffp-contract=off tests/cpp/sincos_small_check.c -lm && ./a.out */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../ppo-bipedalwalker_amd/csrc/wk_sincos_small.h"

int main(void) {
  const float lim = 0.25f;
  uint32_t hi;
  memcpy(&hi, &lim, 4);
  long bad = 0, n = 0;
#pragma omp parallel for reduction(+ : bad, n) schedule(static, 1 << 16)
  for (long u = 0; u <= (long)hi; u++) {
    uint32_t b = (uint32_t)u;
    float x;
    memcpy(&x, &b, 4);
    double s, c;
    wk_sincos_small((double)x, &s, &c);
    float fs = (float)s, fc = (float)c;
    float rs = (float)sin((double)x), rc = (float)cos((double)x);
    if (memcmp(&fs, &rs, 4) || memcmp(&fc, &rc, 4)) {
      if (bad < 10) printf("mismatch x=%a sin %a/%a cos %a/%a\n", x, fs, rs, fc, rc);
      bad++;
    }
    n++;
  }
  printf("checked %ld floats in [0, 0.25]: %ld mismatches\n", n, bad);
  return bad != 0;
}
