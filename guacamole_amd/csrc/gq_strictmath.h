// gq_strictmath.h — java.lang.StrictMath log / exp / log10 on the device (and host).
//
// The somatic caller's decisions (SomaticStandardCaller.scala:196-236) compare sums of
// FP64 logs against thresholds; at germline hets the odds test lands within an ulp of 1
// (GQ_FLAG_KNIFE_EDGE).  Reproducing those decisions needs every transcendental to give the
// same bits as the reference's arithmetic.  The JVM's StrictMath is specified as fdlibm 5.3
// (Sun, 1993); the reference calls scala.math.log / exp / log10 (Likelihood.scala:185-193,
// SomaticStandardCaller.scala:236, ADAM PhredUtils), i.e. java.lang.Math, which may use an
// intrinsic within 1 ulp of these (parity unpinned at that level).  fdlibm is pure IEEE double
// arithmetic — no tables, no fused multiply-add — so it gives identical bits on gfx950 and on
// the host when contraction is off (the pragma below).  oracle/strictmath.h is the checker's
// own copy of the same published algorithms.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GQ_HD __host__ __device__ __forceinline__
#else
#define GQ_HD inline
#endif
// no fused multiply-add inside these bodies (fdlibm's rounding assumes separate mul / add)
#if defined(__clang__)
#define GQ_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define GQ_NO_CONTRACT
#endif

namespace gq {
namespace sm {

GQ_HD int32_t hi_word(double x) { return (int32_t)(__builtin_bit_cast(uint64_t, x) >> 32); }
GQ_HD uint32_t lo_word(double x) { return (uint32_t)__builtin_bit_cast(uint64_t, x); }
GQ_HD double with_hi(double x, int32_t hi) {
  const uint64_t b = (__builtin_bit_cast(uint64_t, x) & 0xFFFFFFFFull) | ((uint64_t)(uint32_t)hi << 32);
  return __builtin_bit_cast(double, b);
}

// fdlibm e_log.c (__ieee754_log)
GQ_HD double log(double x) {
  GQ_NO_CONTRACT
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
               Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  int32_t hx = hi_word(x);
  const uint32_t lx = lo_word(x);
  int32_t k = 0;
  if (hx < 0x00100000) {                                     // x < 2**-1022
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / 0.0;  // log(+-0) = -inf
    if (hx < 0) return (x - x) / 0.0;                          // log(-#) = NaN
    k -= 54;
    x *= two54;  // subnormal: scale up
    hx = hi_word(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i0 = (hx + 0x95f64) & 0x100000;
  x = with_hi(x, hx | (i0 ^ 0x3ff00000));  // normalize x or x/2
  k += (i0 >> 20);
  const double f = x - 1.0;
  if ((0x000fffff & (2 + hx)) < 3) {  // |f| < 2**-20
    if (f == 0.0) {
      if (k == 0) return 0.0;
      const double dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    const double dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  const double dk = (double)k;
  const double z = s * s;
  int32_t i = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  const double R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// fdlibm e_exp.c (__ieee754_exp)
GQ_HD double exp(double x) {
  GQ_NO_CONTRACT
  const double huge = 1.0e+300, twom1000 = 9.33263618503218878990e-302,
               o_threshold = 7.09782712893383973096e+02, u_threshold = -7.45133219101941108420e+02,
               ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00, P1 = 1.66666666666666019037e-01,
               P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
               P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08;
  uint32_t hx = (uint32_t)hi_word(x);
  const int xsb = (int)((hx >> 31) & 1);
  hx &= 0x7fffffff;
  double hi = 0.0, lo = 0.0;
  int32_t k = 0;
  if (hx >= 0x40862E42) {  // |x| >= 709.78...
    if (hx >= 0x7ff00000) {
      if (((hx & 0xfffff) | lo_word(x)) != 0) return x + x;  // NaN
      return xsb == 0 ? x : 0.0;                               // exp(+-inf) = {inf, 0}
    }
    if (x > o_threshold) return huge * huge;           // overflow
    if (x < u_threshold) return twom1000 * twom1000;   // underflow
  }
  if (hx > 0x3fd62e42) {    // |x| > 0.5 ln2
    if (hx < 0x3FF0A2B2) {  // and |x| < 1.5 ln2
      hi = xsb ? x + ln2HI : x - ln2HI;
      lo = xsb ? -ln2LO : ln2LO;
      k = 1 - xsb - xsb;
    } else {
      k = (int32_t)(invln2 * x + (xsb ? -0.5 : 0.5));
      const double t = (double)k;
      hi = x - t * ln2HI;  // t * ln2HI is exact here
      lo = t * ln2LO;
    }
    x = hi - lo;
  } else if (hx < 0x3e300000) {  // |x| < 2**-28
    if (huge + x > 1.0) return 1.0 + x;
  } else {
    k = 0;
  }
  const double t = x * x;
  const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
  double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
  if (k >= -1021) return with_hi(y, (int32_t)((uint32_t)hi_word(y) + ((uint32_t)k << 20)));
  y = with_hi(y, (int32_t)((uint32_t)hi_word(y) + ((uint32_t)(k + 1000) << 20)));
  return y * twom1000;
}

// fdlibm e_log10.c (__ieee754_log10)
GQ_HD double log10(double x) {
  GQ_NO_CONTRACT
  const double two54 = 1.80143985094819840000e+16, ivln10 = 4.34294481903251816668e-01,
               log10_2hi = 3.01029995663611771306e-01, log10_2lo = 3.69423907715893078616e-13;
  int32_t hx = hi_word(x);
  const uint32_t lx = lo_word(x);
  int32_t k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / 0.0;
    if (hx < 0) return (x - x) / 0.0;
    k -= 54;
    x *= two54;
    hx = hi_word(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  const int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
  const double y = (double)(k + i);
  x = with_hi(x, hx);
  const double z = y * log10_2lo + ivln10 * sm::log(x);
  return z + y * log10_2hi;
}

}  // namespace sm
}  // namespace gq
