// strictmath.h — TEST INFRASTRUCTURE (oracle only).  java.lang.StrictMath log / exp / log10,
// i.e. fdlibm 5.3 (e_log.c, e_exp.c, e_log10.c), restated for the CPU oracle.
//
// The reference computes its somatic likelihoods and odds with scala.math.log / exp / log10
// (likelihood/Likelihood.scala:185-193, commands/SomaticStandardCaller.scala:236, ADAM
// PhredUtils).  Those are java.lang.Math; StrictMath mandates exactly these fdlibm results, and
// Math may differ by at most 1 ulp (JVM-dependent, parity unpinned at that level).  The oracle
// uses the fdlibm bits so that knife-edge decisions (odds within an ulp of a threshold) are
// defined; the product restates the same algorithms in guacamole_amd/csrc/gq_strictmath.h
// (tests/test_strictmath.py checks both bitwise against each other and within 1 ulp of libm).
// Compiled with -ffp-contract=off (oracle/Makefile): fdlibm assumes separate multiply and add.
#pragma once
#include <cstdint>
#include <cstring>

namespace strictmath {

inline int32_t HI(double x) {
  uint64_t b;
  std::memcpy(&b, &x, 8);
  return (int32_t)(b >> 32);
}
inline uint32_t LO(double x) {
  uint64_t b;
  std::memcpy(&b, &x, 8);
  return (uint32_t)b;
}
inline void SET_HI(double &x, int32_t hi) {
  uint64_t b;
  std::memcpy(&b, &x, 8);
  b = (b & 0xFFFFFFFFull) | ((uint64_t)(uint32_t)hi << 32);
  std::memcpy(&x, &b, 8);
}

static const double zero = 0.0;

// e_log.c
inline double log(double x) {
  static const double ln2_hi = 6.93147180369123816490e-01, /* 3fe62e42 fee00000 */
      ln2_lo = 1.90821492927058770002e-10,                  /* 3dea39ef 35793c76 */
      two54 = 1.80143985094819840000e+16,                   /* 43500000 00000000 */
      Lg1 = 6.666666666666735130e-01,                       /* 3FE55555 55555593 */
      Lg2 = 3.999999999940941908e-01,                       /* 3FD99999 9997FA04 */
      Lg3 = 2.857142874366239149e-01,                       /* 3FD24924 94229359 */
      Lg4 = 2.222219843214978396e-01,                       /* 3FCC71C5 1D8E78AF */
      Lg5 = 1.818357216161805012e-01,                       /* 3FC74664 96CB03DE */
      Lg6 = 1.531383769920937332e-01,                       /* 3FC39A09 D078C69F */
      Lg7 = 1.479819860511658591e-01;                       /* 3FC2F112 DF3E5244 */
  double hfsq, f, s, z, R, w, t1, t2, dk;
  int32_t k, hx, i, j;
  uint32_t lx;
  hx = HI(x);
  lx = LO(x);
  k = 0;
  if (hx < 0x00100000) { /* x < 2**-1022  */
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / zero; /* log(+-0)=-inf */
    if (hx < 0) return (x - x) / zero;                                /* log(-#) = NaN */
    k -= 54;
    x *= two54; /* subnormal number, scale up x */
    hx = HI(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  i = (hx + 0x95f64) & 0x100000;
  SET_HI(x, hx | (i ^ 0x3ff00000)); /* normalize x or x/2 */
  k += (i >> 20);
  f = x - 1.0;
  if ((0x000fffff & (2 + hx)) < 3) { /* |f| < 2**-20 */
    if (f == zero) {
      if (k == 0) return zero;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  s = f / (2.0 + f);
  dk = (double)k;
  z = s * s;
  i = hx - 0x6147a;
  w = z * z;
  j = 0x6b851 - hx;
  t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  if (i > 0) {
    hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// e_exp.c
inline double exp(double x) {
  static const double one = 1.0, halF[2] = {0.5, -0.5}, huge = 1.0e+300,
                      twom1000 = 9.33263618503218878990e-302,     /* 2**-1000=0x01700000,0 */
      o_threshold = 7.09782712893383973096e+02,                   /* 0x40862E42, 0xFEFA39EF */
      u_threshold = -7.45133219101941108420e+02,                  /* 0xc0874910, 0xD52D3051 */
      ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01},
                      ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10},
                      invln2 = 1.44269504088896338700e+00, /* 0x3ff71547, 0x652b82fe */
      P1 = 1.66666666666666019037e-01,                     /* 0x3FC55555, 0x5555553E */
      P2 = -2.77777777770155933842e-03,                    /* 0xBF66C16C, 0x16BEBD93 */
      P3 = 6.61375632143793436117e-05,                     /* 0x3F11566A, 0xAF25DE2C */
      P4 = -1.65339022054652515390e-06,                    /* 0xBEBBBD41, 0xC5D26BF1 */
      P5 = 4.13813679705723846039e-08;                     /* 0x3E663769, 0x72BEA4D0 */
  double y, hi = 0.0, lo = 0.0, c, t;
  int32_t k = 0, xsb;
  uint32_t hx;
  hx = (uint32_t)HI(x);
  xsb = (int32_t)((hx >> 31) & 1);
  hx &= 0x7fffffff;
  if (hx >= 0x40862E42) { /* if |x|>=709.78... */
    if (hx >= 0x7ff00000) {
      if (((hx & 0xfffff) | LO(x)) != 0) return x + x; /* NaN */
      return (xsb == 0) ? x : 0.0;                     /* exp(+-inf)={inf,0} */
    }
    if (x > o_threshold) return huge * huge;         /* overflow */
    if (x < u_threshold) return twom1000 * twom1000; /* underflow */
  }
  if (hx > 0x3fd62e42) {   /* if  |x| > 0.5 ln2 */
    if (hx < 0x3FF0A2B2) { /* and |x| < 1.5 ln2 */
      hi = x - ln2HI[xsb];
      lo = ln2LO[xsb];
      k = 1 - xsb - xsb;
    } else {
      k = (int32_t)(invln2 * x + halF[xsb]);
      t = k;
      hi = x - t * ln2HI[0]; /* t*ln2HI is exact here */
      lo = t * ln2LO[0];
    }
    x = hi - lo;
  } else if (hx < 0x3e300000) { /* when |x|<2**-28 */
    if (huge + x > one) return one + x;
  } else {
    k = 0;
  }
  t = x * x;
  c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  if (k == 0) return one - ((x * c) / (c - 2.0) - x);
  y = one - ((lo - (x * c) / (2.0 - c)) - hi);
  if (k >= -1021) {
    SET_HI(y, (int32_t)((uint32_t)HI(y) + ((uint32_t)k << 20))); /* add k to y's exponent */
    return y;
  }
  SET_HI(y, (int32_t)((uint32_t)HI(y) + ((uint32_t)(k + 1000) << 20)));
  return y * twom1000;
}

// e_log10.c
inline double log10(double x) {
  static const double two54 = 1.80143985094819840000e+16, /* 0x43500000, 0x00000000 */
      ivln10 = 4.34294481903251816668e-01,                 /* 0x3FDBCB7B, 0x1526E50E */
      log10_2hi = 3.01029995663611771306e-01,              /* 0x3FD34413, 0x509F6000 */
      log10_2lo = 3.69423907715893078616e-13;              /* 0x3D59FEF3, 0x11F12B36 */
  double y, z;
  int32_t i, k, hx;
  uint32_t lx;
  hx = HI(x);
  lx = LO(x);
  k = 0;
  if (hx < 0x00100000) { /* x < 2**-1022  */
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / zero; /* log(+-0)=-inf */
    if (hx < 0) return (x - x) / zero;                                /* log(-#) = NaN */
    k -= 54;
    x *= two54; /* subnormal number, scale up x */
    hx = HI(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
  hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
  y = (double)(k + i);
  SET_HI(x, hx);
  z = y * log10_2lo + ivln10 * strictmath::log(x);
  return z + y * log10_2hi;
}

}  // namespace strictmath
