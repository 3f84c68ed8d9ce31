// Checks the product's StrictMath restatement (guacamole_amd/csrc/gq_strictmath.h, host build)
// against the oracle's (oracle/strictmath.h): bitwise identical, and within 1 ulp of libm.
// Built and run by tests/test_strictmath.py (g++ -ffp-contract=off).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../guacamole_amd/csrc/gq_strictmath.h"
#include "../../oracle/strictmath.h"

static uint64_t bits(double x) {
  uint64_t b;
  std::memcpy(&b, &x, 8);
  return b;
}
static int64_t ulps(double a, double b) {
  if (std::isnan(a) && std::isnan(b)) return 0;
  if (a == b) return 0;
  int64_t ia = (int64_t)bits(a), ib = (int64_t)bits(b);
  if (ia < 0) ia = INT64_MIN - ia;
  if (ib < 0) ib = INT64_MIN - ib;
  return ia > ib ? ia - ib : ib - ia;
}

int main() {
  std::mt19937_64 g(20261016);
  long bad_bits = 0, bad_ulp = 0, n = 0;
  auto check = [&](const char *nm, double x, double p, double o, double lib) {
    ++n;
    if (bits(p) != bits(o) && !(std::isnan(p) && std::isnan(o))) {
      if (bad_bits++ < 5) std::printf("bits %s(%.17g): product %.17g oracle %.17g\n", nm, x, p, o);
    }
    // fdlibm log10 = ivln10 * log(x) + ... is not 1-ulp accurate near x = 1 (a property of the
    // algorithm StrictMath specifies, not of this restatement): allow 4 ulps there
    const int64_t lim = nm[3] == '1' ? 4 : 1;
    if (ulps(o, lib) > lim) {
      if (bad_ulp++ < 5) std::printf("ulp %s(%.17g): oracle %.17g libm %.17g\n", nm, x, o, lib);
    }
  };
  std::uniform_real_distribution<double> u01(0.0, 1.0), uexp(-745.0, 709.0), ulog(-300.0, 300.0);
  for (int i = 0; i < 2000000; ++i) {
    // log: probabilities and sums of two probabilities (the likelihood terms), wide range
    double x = (i & 3) == 0 ? u01(g) * 2.0 : (i & 3) == 1 ? std::pow(10.0, ulog(g)) : (i & 3) == 2 ? 1.0 - u01(g) * 1e-6 : u01(g);
    check("log", x, gq::sm::log(x), strictmath::log(x), std::log(x));
    check("log10", x, gq::sm::log10(x), strictmath::log10(x), std::log10(x));
    double y = (i & 1) ? uexp(g) : (u01(g) - 0.5) * 4.0;
    check("exp", y, gq::sm::exp(y), strictmath::exp(y), std::exp(y));
  }
  // phred-derived inputs exactly as the caller forms them
  for (int q = 0; q < 256; ++q)
    for (int m = 0; m < 256; m += 7) {
      double pc = (1.0 - std::pow(10.0, -q / 10.0)) * (1.0 - std::pow(10.0, -m / 10.0));
      for (double v : {pc + pc, pc + (1.0 - pc), (1.0 - pc) + (1.0 - pc)})
        check("log", v, gq::sm::log(v), strictmath::log(v), std::log(v));
    }
  for (double s : {0.0, -0.0, 1.0, 2.0, 10.0, 1e-310, -1.0, (double)INFINITY, -(double)INFINITY, (double)NAN, 709.7, 709.8, -745.2, -745.1, 1e-20})
    {
      check("log", s, gq::sm::log(s), strictmath::log(s), std::log(s));
      check("exp", s, gq::sm::exp(s), strictmath::exp(s), std::exp(s));
      check("log10", s, gq::sm::log10(s), strictmath::log10(s), std::log10(s));
    }
  std::printf("checked %ld values: %ld bit mismatches, %ld beyond 1 ulp of libm\n", n, bad_bits, bad_ulp);
  return (bad_bits || bad_ulp) ? 1 : 0;
}
