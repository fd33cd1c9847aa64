// gomath.h — Go 1.26 `math` package routines used on izpi's hot path, restated as
// portable IEEE-754 binary64 code that compiles identically for the gfx950 device
// and for the x86-64 host (both built with -ffp-contract=off, no fast-math).
//
// Why: izpi's samplers call math.Sin/Cos (vec3.go:122-137), math.Pow
// (material.go:42, spectral_constant.go:71, pbr.go:124), math.Exp
// (dielectric.go:110,170-172, spectral_constant.go:72), math.Atan2/Asin
// (sphere.go:30-31), math.Tan (camera.go:33, host only). The GPU kernel and the
// CPU oracle must produce bit-identical radiance, so neither may use the vendor
// libm (ocml / glibc differ in the last ulp). The algorithms below are Go's
// pure-Go (generic) implementations, which are themselves Cephes / FreeBSD msun:
//   sin.go (Cephes sin/cos), tan.go, exp.go (FreeBSD e_exp.c), log.go,
//   pow.go, frexp.go, ldexp.go, modf.go, atan.go, atan2.go, asin.go, dim.go.
// Go's amd64/arm64 assembly Exp/Log may differ from the generic code in the last
// ulp; that difference is against Go itself, not against our oracle.
//
// Argument reduction for |x| >= 2^29 (Go's Payne-Hanek trigReduce) is not needed:
// every trig call on the path takes 2*pi*xi with xi in [0,1) or a camera half-fov.
// Such inputs return NaN here and in the oracle (documented, unreachable).
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define IZPI_HD __host__ __device__ __forceinline__
#else
#define IZPI_HD static inline
#endif

namespace gm {

IZPI_HD uint64_t bits(double x) { union { double d; uint64_t u; } v; v.d = x; return v.u; }
IZPI_HD double from_bits(uint64_t u) { union { double d; uint64_t u; } v; v.u = u; return v.d; }
IZPI_HD uint32_t bits32(float x) { union { float f; uint32_t u; } v; v.f = x; return v.u; }
IZPI_HD float from_bits32(uint32_t u) { union { float f; uint32_t u; } v; v.u = u; return v.f; }

IZPI_HD bool is_nan(double x) { return x != x; }
IZPI_HD bool is_inf(double x, int sign) {
  return (sign >= 0 && x > 1.7976931348623157e308) || (sign <= 0 && x < -1.7976931348623157e308);
}
IZPI_HD bool signbit(double x) { return (bits(x) >> 63) != 0; }
IZPI_HD double inf(int sign) { return from_bits(sign >= 0 ? 0x7FF0000000000000ull : 0xFFF0000000000000ull); }
IZPI_HD double nan() { return from_bits(0x7FF8000000000001ull); }
IZPI_HD double abs(double x) { return from_bits(bits(x) & ~(1ull << 63)); }
IZPI_HD double copysign(double f, double s) {
  return from_bits((bits(f) & ~(1ull << 63)) | (bits(s) & (1ull << 63)));
}

// math.Sqrt: compiler intrinsic in Go; IEEE correctly rounded on both targets.
IZPI_HD double sqrt(double x) { return __builtin_sqrt(x); }

// math.Min / math.Max (dim.go): -Inf/+Inf first, then NaN, then signed zeros.
IZPI_HD double min(double x, double y) {
  if (is_inf(x, -1) || is_inf(y, -1)) return inf(-1);
  if (is_nan(x) || is_nan(y)) return nan();
  if (x == 0 && x == y) return signbit(x) ? x : y;
  return x < y ? x : y;
}
IZPI_HD double max(double x, double y) {
  if (is_inf(x, 1) || is_inf(y, 1)) return inf(1);
  if (is_nan(x) || is_nan(y)) return nan();
  if (x == 0 && x == y) return signbit(x) ? y : x;
  return x > y ? x : y;
}

// frexp.go: normalize + exponent extraction; frac in [0.5, 1).
IZPI_HD double frexp(double f, int* e) {
  *e = 0;
  if (f == 0 || is_inf(f, 0) || is_nan(f)) return f;
  int ex = 0;
  if (abs(f) < 2.2250738585072014e-308) { f = f * 4503599627370496.0; ex = -52; }
  uint64_t x = bits(f);
  ex += (int)((x >> 52) & 0x7FF) - 1023 + 1;
  x &= ~(0x7FFull << 52);
  x |= (uint64_t)(-1 + 1023) << 52;
  *e = ex;
  return from_bits(x);
}

// ldexp.go
IZPI_HD double ldexp(double frac, int ex) {
  if (frac == 0) return frac;
  if (is_inf(frac, 0) || is_nan(frac)) return frac;
  int e = 0;
  if (abs(frac) < 2.2250738585072014e-308) { frac = frac * 4503599627370496.0; e = -52; }
  ex += e;
  uint64_t x = bits(frac);
  ex += (int)((x >> 52) & 0x7FF) - 1023;
  if (ex < -1075) return copysign(0, frac);
  if (ex > 1023) return frac < 0 ? inf(-1) : inf(1);
  double m = 1;
  if (ex < -1022) { ex += 53; m = 1.0 / 9007199254740992.0; }
  x &= ~(0x7FFull << 52);
  x |= (uint64_t)(ex + 1023) << 52;
  return m * from_bits(x);
}

// modf.go (generic): integer and fractional parts with the sign of f.
// (Go's `case f < 0: int, frac = Modf(-f); return -int, -frac` is written out without
// recursion: a recursive call on the GPU forces a call stack and the full register file.)
IZPI_HD double modf_ge1(double f, double* frac) {  // f >= 1, +Inf or NaN
  uint64_t x = bits(f);
  uint64_t e = ((x >> 52) & 0x7FF) - 1023;
  if (e < 64 - 12) x &= ~((1ull << (64 - 12 - e)) - 1);
  double ip = from_bits(x);
  *frac = f - ip;
  return ip;
}
IZPI_HD double modf(double f, double* frac) {
  if (f < 1) {
    if (f < 0) {
      const double g = -f;  // > 0
      double fr, ip;
      if (g < 1) { fr = g; ip = 0; } else { ip = modf_ge1(g, &fr); }
      *frac = -fr;
      return -ip;
    }
    if (f == 0) { *frac = f; return f; }
    *frac = f; return 0;
  }
  return modf_ge1(f, frac);
}

IZPI_HD bool is_odd_int(double x) {
  if (abs(x) >= 9007199254740992.0) return false;
  double xf; double xi = modf(x, &xf);
  return xf == 0 && (((int64_t)xi) & 1) == 1;
}

// sin.go (Cephes) — coefficients _sin[], _cos[] and the Pi/4 split PI4A/B/C.
#define GM_PI4A 7.85398125648498535156e-1
#define GM_PI4B 3.77489470793079817668e-8
#define GM_PI4C 2.69515142907905952645e-15
#define GM_4_OVER_PI 1.2732395447351628  /* 0x3FF45F306DC9C883, Go constant 4/Pi */
#define GM_REDUCE_THRESHOLD 536870912.0  /* 1<<29 */

IZPI_HD double sin_poly(double z, double zz) {
  return z + z * zz * ((((((1.58962301576546568060e-10 * zz) + -2.50507477628578072866e-8) * zz + 2.75573136213857245213e-6) * zz + -1.98412698295895385996e-4) * zz + 8.33333333332211858878e-3) * zz + -1.66666666666666307295e-1);
}
IZPI_HD double cos_poly(double zz) {
  return 1.0 - 0.5 * zz + zz * zz * ((((((-1.13585365213876817300e-11 * zz) + 2.08757008419747316778e-9) * zz + -2.75573141792967388112e-7) * zz + 2.48015872888517045348e-5) * zz + -1.38888888888730564116e-3) * zz + 4.16666666666665929218e-2);
}

IZPI_HD double cos(double x) {
  if (is_nan(x) || is_inf(x, 0)) return nan();
  bool sign = false;
  x = abs(x);
  if (x >= GM_REDUCE_THRESHOLD) return nan();  // unreachable on the path (see header)
  uint64_t j = (uint64_t)(x * GM_4_OVER_PI);
  double y = (double)j;
  if (j & 1) { j++; y++; }
  j &= 7;
  double z = ((x - y * GM_PI4A) - y * GM_PI4B) - y * GM_PI4C;
  if (j > 3) { j -= 4; sign = !sign; }
  if (j > 1) sign = !sign;
  double zz = z * z;
  if (j == 1 || j == 2) y = sin_poly(z, zz); else y = cos_poly(zz);
  return sign ? -y : y;
}

IZPI_HD double sin(double x) {
  if (x == 0 || is_nan(x)) return x;
  if (is_inf(x, 0)) return nan();
  bool sign = false;
  if (x < 0) { x = -x; sign = true; }
  if (x >= GM_REDUCE_THRESHOLD) return nan();  // unreachable on the path (see header)
  uint64_t j = (uint64_t)(x * GM_4_OVER_PI);
  double y = (double)j;
  if (j & 1) { j++; y++; }
  j &= 7;
  double z = ((x - y * GM_PI4A) - y * GM_PI4B) - y * GM_PI4C;
  if (j > 3) { sign = !sign; j -= 4; }
  double zz = z * z;
  if (j == 1 || j == 2) y = cos_poly(zz); else y = sin_poly(z, zz);
  return sign ? -y : y;
}

// cos(x) and sin(x) of one x >= 0 below GM_REDUCE_THRESHOLD (random directions' phi = 2 Pi r,
// r in [0, 1)): the two share sin.go's reduction and both polynomials, so one reduction
// and one evaluation of each polynomial give both, bit for bit as cos() and sin() above
// (for x = +0 sin's early return and the polynomial both give +0).
IZPI_HD void sincos_nonneg(double x, double* s, double* c) {
  uint64_t j = (uint64_t)(x * GM_4_OVER_PI);
  double y = (double)j;
  if (j & 1) { j++; y++; }
  j &= 7;
  const double z = ((x - y * GM_PI4A) - y * GM_PI4B) - y * GM_PI4C;
  bool csign = false, ssign = false;
  if (j > 3) { j -= 4; csign = !csign; ssign = !ssign; }
  if (j > 1) csign = !csign;
  const double zz = z * z;
  const double sp = sin_poly(z, zz), cp = cos_poly(zz);
  const bool swap = j == 1 || j == 2;
  const double cy = swap ? sp : cp, sy = swap ? cp : sp;
  *c = csign ? -cy : cy;
  *s = ssign ? -sy : sy;
}

// tan.go (Cephes)
IZPI_HD double tan(double x) {
  if (x == 0 || is_nan(x)) return x;
  if (is_inf(x, 0)) return nan();
  bool sign = false;
  if (x < 0) { x = -x; sign = true; }
  if (x >= GM_REDUCE_THRESHOLD) return nan();
  uint64_t j = (uint64_t)(x * GM_4_OVER_PI);
  double y = (double)j;
  if (j & 1) { j++; y++; }
  double z = ((x - y * GM_PI4A) - y * GM_PI4B) - y * GM_PI4C;
  double zz = z * z;
  if (zz > 1e-14) {
    y = z + z * (zz * (((-1.30936939181383777646e4 * zz) + 1.15351664838587416140e6) * zz + -1.79565251976484877988e7) /
                 ((((zz + 1.36812963470692954678e4) * zz + -1.32089234440210967447e6) * zz + 2.50083801823357915839e7) * zz + -5.38695755929454629881e7));
  } else {
    y = z;
  }
  if (j & 2) y = -1 / y;
  return sign ? -y : y;
}

// exp.go (generic; FreeBSD e_exp.c)
IZPI_HD double exp(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
               Log2e = 1.44269504088896338700e+00, Overflow = 7.09782712893383973096e+02,
               Underflow = -7.45133219101941108420e+02, NearZero = 1.0 / 268435456.0;
  if (is_nan(x) || is_inf(x, 1)) return x;
  if (is_inf(x, -1)) return 0;
  if (x > Overflow) return inf(1);
  if (x < Underflow) return 0;
  if (-NearZero < x && x < NearZero) return 1 + x;
  int k = 0;
  if (x < 0) k = (int)(Log2e * x - 0.5);
  else if (x > 0) k = (int)(Log2e * x + 0.5);
  double hi = x - (double)k * Ln2Hi;
  double lo = (double)k * Ln2Lo;
  // expmulti
  double r = hi - lo;
  double t = r * r;
  double c = r - t * (1.66666666666666657415e-01 + t * (-2.77777777770155933842e-03 + t * (6.61375632143793436117e-05 + t * (-1.65339022054652515390e-06 + t * 4.13813679705723846039e-08))));
  double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
  return ldexp(y, k);
}

// log.go (generic; FreeBSD e_log.c)
IZPI_HD double log(double x) {
  if (is_nan(x) || is_inf(x, 1)) return x;
  if (x < 0) return nan();
  if (x == 0) return inf(-1);
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 0.7071067811865476) { f1 *= 2; ki--; }
  double f = f1 - 1;
  double k = (double)ki;
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (6.666666666666735130e-01 + s4 * (2.857142874366239149e-01 + s4 * (1.818357216161805012e-01 + s4 * 1.479819860511658591e-01)));
  double t2 = s4 * (3.999999999940941908e-01 + s4 * (2.222219843214978396e-01 + s4 * 1.531383769920937332e-01));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + k * 1.90821492927058770002e-10)) - f);
}

// pow.go
// Pow(±0, y) for y != 0 and not NaN (pow.go "case x == 0").
IZPI_HD double pow_zero(double x, double y) {
  if (y < 0) return (signbit(x) && is_odd_int(y)) ? inf(-1) : inf(1);
  return (signbit(x) && is_odd_int(y)) ? x : 0;
}
IZPI_HD double pow(double x, double y) {
  // Pow(x, 2) (the spectral Gaussian textures' exponent, spectral_constant.go:102): pow.go's
  // loop computes frexp's mantissa m squared, rounded once, times 2^(2e) by exact steps,
  // which is the correctly rounded x * x whenever x * x is a normal number, 0 or inf.
  // Only 0 < |x| < 2^-511 (a subnormal or zero square: the loop rounds twice) takes the loop.
  if (y == 2.0) {
    const double ax = abs(x);
    if (ax >= 0x1p-511 || ax == 0) return x * x;  // (NaN: Go returns its own NaN bits, below)
  }
  // Pow(x, 5) (PBR's Schlick term, pbr.go:102): the loop takes frexp's mantissa m and makes
  // a1 = m, x1 = rn(m*m), x1 = rn(x1*x1), a1 = rn(a1*x1) with exact doublings in between,
  // then ldexp: the same roundings as x * ((x*x) * (x*x)) whenever x^2, x^4 and x^5 are
  // normal numbers (2^-204 <= |x| <= 2^204), and the same signed zero for x = +-0
  if (y == 5.0) {
    const double ax = abs(x);
    if ((ax >= 0x1p-204 && ax <= 0x1p+204) || ax == 0) {
      const double x2 = x * x, x4 = x2 * x2;
      return x * x4;
    }
  }
  if (y == 0 || x == 1) return 1;
  if (y == 1) return x;
  if (is_nan(x) || is_nan(y)) return nan();
  if (x == 0) {
    return pow_zero(x, y);
  } else if (is_inf(y, 0)) {
    if (x == -1) return 1;
    if ((abs(x) < 1) == is_inf(y, 1)) return 0;
    return inf(1);
  } else if (is_inf(x, 0)) {
    // Go: `return Pow(1/x, -y)`, i.e. Pow(-0, -y) (written out: no recursion on the GPU,
    // where a recursive call forces a call stack and the full register file)
    if (is_inf(x, -1)) return pow_zero(1 / x, -y);
    if (y < 0) return 0;
    if (y > 0) return inf(1);
  } else if (y == 0.5) {
    return sqrt(x);
  } else if (y == -0.5) {
    return 1 / sqrt(x);
  }
  double yf;
  double yi = modf(abs(y), &yf);
  if (yf != 0 && x < 0) return nan();
  if (yi >= 9223372036854775808.0) {
    if (x == -1) return 1;
    if ((abs(x) < 1) == (y > 0)) return 0;
    return inf(1);
  }
  double a1 = 1.0;
  int ae = 0;
  if (yf != 0) {
    if (yf > 0.5) { yf--; yi++; }
    a1 = exp(yf * log(x));
  }
  int xe;
  double x1 = frexp(x, &xe);
  for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
    if (xe < -(1 << 12) || (1 << 12) < xe) { ae += xe; break; }
    if ((i & 1) == 1) { a1 *= x1; ae += xe; }
    x1 *= x1;
    xe <<= 1;
    if (x1 < .5) { x1 += x1; xe--; }
  }
  if (y < 0) { a1 = 1 / a1; ae = -ae; }
  return ldexp(a1, ae);
}

// atan.go (Cephes xatan/satan)
IZPI_HD double xatan(double x) {
  double z = x * x;
  z = z * ((((-8.750608600031904122785e-01 * z + -1.615753718733365076637e+01) * z + -7.500855792314704667340e+01) * z + -1.228866684490136173410e+02) * z + -6.485021904942025371773e+01) /
      (((((z + 2.485846490142306297962e+01) * z + 1.650270098316988542046e+02) * z + 4.328810604912902668951e+02) * z + 4.853903996359136964868e+02) * z + 1.945506571482613964425e+02);
  z = x * z + x;
  return z;
}
IZPI_HD double satan(double x) {
  const double Morebits = 6.123233995736765886130e-17, Tan3pio8 = 2.41421356237309504880;
  if (x <= 0.66) return xatan(x);
  if (x > Tan3pio8) return 1.5707963267948966 - xatan(1 / x) + Morebits;
  return 0.7853981633974483 + xatan((x - 1) / (x + 1)) + 0.5 * Morebits;
}
IZPI_HD double atan(double x) {
  if (x == 0) return x;
  if (x > 0) return satan(x);
  return -satan(-x);
}
// atan2.go
IZPI_HD double atan2(double y, double x) {
  const double Pi = 3.141592653589793;
  if (is_nan(y) || is_nan(x)) return nan();
  if (y == 0) {
    if (x >= 0 && !signbit(x)) return copysign(0, y);
    return copysign(Pi, y);
  }
  if (x == 0) return copysign(Pi / 2, y);
  if (is_inf(x, 0)) {
    if (is_inf(x, 1)) return is_inf(y, 0) ? copysign(Pi / 4, y) : copysign(0, y);
    return is_inf(y, 0) ? copysign(2.356194490192345, y) : copysign(Pi, y);
  }
  if (is_inf(y, 0)) return copysign(Pi / 2, y);
  double q = atan(y / x);
  if (x < 0) return q <= 0 ? q + Pi : q - Pi;
  return q;
}
// asin.go
IZPI_HD double asin(double x) {
  if (x == 0) return x;
  bool sign = false;
  if (x < 0) { x = -x; sign = true; }
  if (x > 1) return nan();
  double temp = sqrt(1 - x * x);
  if (x > 0.7) temp = 1.5707963267948966 - satan(temp / x);
  else temp = satan(x / temp);
  return sign ? -temp : temp;
}

// math.Nextafter32 (nextafter.go)
IZPI_HD float nextafter32(float x, float y) {
  if (x != x || y != y) return from_bits32(0x7FC00000u);
  if (x == y) return x;
  if (x == 0) return from_bits32(1u | (bits32(y) & 0x80000000u));
  if ((y > x) == (x > 0)) return from_bits32(bits32(x) + 1);
  return from_bits32(bits32(x) - 1);
}

}  // namespace gm
