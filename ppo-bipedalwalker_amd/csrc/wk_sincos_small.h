/* wk_sincos_small.h -- sin / cos of a small angle in double, for the rotation's
 * (float)Math.Sin/Cos((double)angle) (XNA CreateRotationZ, Skeleton.Rotate Skeleton.cs:89-97).
 * Taylor series in Horner form with explicit FMAs, valid for |x| <= 0.25 (truncation
 * below 1e-20 relative).  Shared by the device code and the host-side exhaustive check
 * (tests/cpp/sincos_small_check.c), which proves (float) of it equals (float) of the C
 * library's sin / cos for every float in that range. */
#ifndef WK_SINCOS_SMALL_H
#define WK_SINCOS_SMALL_H
#ifdef __HIP__
#define WK_SC_FN __host__ __device__ __forceinline__
#else
#define WK_SC_FN static inline
#include <math.h>
#endif

WK_SC_FN void wk_sincos_small(double x, double* s, double* c) {
  const double x2 = x * x;
  double ps = 1.0 / 6227020800.0;                   /*  1/13! */
  ps = __builtin_fma(ps, x2, -1.0 / 39916800.0);    /* -1/11! */
  ps = __builtin_fma(ps, x2, 1.0 / 362880.0);       /*  1/9!  */
  ps = __builtin_fma(ps, x2, -1.0 / 5040.0);        /* -1/7!  */
  ps = __builtin_fma(ps, x2, 1.0 / 120.0);          /*  1/5!  */
  ps = __builtin_fma(ps, x2, -1.0 / 6.0);           /* -1/3!  */
  *s = __builtin_fma(x * x2, ps, x);
  double pc = -1.0 / 87178291200.0;                 /* -1/14! */
  pc = __builtin_fma(pc, x2, 1.0 / 479001600.0);    /*  1/12! */
  pc = __builtin_fma(pc, x2, -1.0 / 3628800.0);     /* -1/10! */
  pc = __builtin_fma(pc, x2, 1.0 / 40320.0);        /*  1/8!  */
  pc = __builtin_fma(pc, x2, -1.0 / 720.0);         /* -1/6!  */
  pc = __builtin_fma(pc, x2, 1.0 / 24.0);           /*  1/4!  */
  pc = __builtin_fma(pc, x2, -0.5);                 /* -1/2!  */
  *c = __builtin_fma(x2, pc, 1.0);
}
#endif
