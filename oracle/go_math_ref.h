/* go_math_ref.h — TEST INFRASTRUCTURE (oracle). Independent CPU restatement of
 * the Go 1.26 `math` routines izpi's hot path calls. Only tests/, smoke() and
 * bench.py's cpu_baseline may load anything under oracle/.
 *
 * Sources restated (Go stdlib, pure-Go/generic versions; go.mod:3 pins Go 1.26):
 *   math/sin.go   cos, sin (Cephes, _sin/_cos tables, PI4A/B/C)
 *   math/tan.go   tan (Cephes _tanP/_tanQ)
 *   math/exp.go   exp + expmulti (FreeBSD e_exp.c)
 *   math/log.go   log (FreeBSD e_log.c)
 *   math/pow.go   pow (Modf/Frexp/Ldexp squaring loop)
 *   math/atan.go, atan2.go, asin.go (Cephes xatan/satan)
 *   math/frexp.go, ldexp.go, modf.go, dim.go (Min/Max), nextafter.go
 * Constants were checked against their IEEE hex encodings in Go's source comments
 * (see tests/test_gomath.py). Payne-Hanek reduction (|x| >= 2^29) is not restated:
 * such inputs return NaN, never reached by izpi's call sites.
 * Compiled with -ffp-contract=off: every a*b+c below is two roundings, as in
 * Go on amd64 (GOAMD64=v1 emits no FMA).
 */
#ifndef IZPI_ORACLE_GO_MATH_REF_H
#define IZPI_ORACLE_GO_MATH_REF_H
#include <stdint.h>
#include <string.h>
#include <math.h>

static inline uint64_t go_f64bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double go_f64frombits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }
static inline uint32_t go_f32bits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static inline float go_f32frombits(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }

static const double GO_PI = 3.14159265358979323846264338327950288419716939937510582097494459;
static const double GO_MAXFLOAT64 = 1.79769313486231570814527423731704356798070e+308;
static const float GO_MAXFLOAT32 = 3.40282346638528859811704183484516925440e+38f;

static inline int go_isnan(double x) { return x != x; }
static inline int go_isinf(double x, int sign) {
  return sign >= 0 && x > GO_MAXFLOAT64 ? 1 : (sign <= 0 && x < -GO_MAXFLOAT64 ? 1 : 0);
}
static inline int go_signbit(double x) { return (int)(go_f64bits(x) >> 63); }
static inline double go_inf(int sign) { return sign >= 0 ? go_f64frombits(0x7FF0000000000000ULL) : go_f64frombits(0xFFF0000000000000ULL); }
static inline double go_nan(void) { return go_f64frombits(0x7FF8000000000001ULL); }
static inline double go_abs(double x) { return go_f64frombits(go_f64bits(x) & ~(1ULL << 63)); }
static inline double go_copysign(double f, double sign) {
  const uint64_t s = 1ULL << 63;
  return go_f64frombits((go_f64bits(f) & ~s) | (go_f64bits(sign) & s));
}
/* math.Sqrt: a compiler intrinsic (SQRTSD), correctly rounded. */
static inline double go_sqrt(double x) { return sqrt(x); }

static inline double go_min(double x, double y) {
  if (go_isinf(x, -1) || go_isinf(y, -1)) return go_inf(-1);
  if (go_isnan(x) || go_isnan(y)) return go_nan();
  if (x == 0 && x == y) { if (go_signbit(x)) return x; return y; }
  if (x < y) return x;
  return y;
}
static inline double go_max(double x, double y) {
  if (go_isinf(x, 1) || go_isinf(y, 1)) return go_inf(1);
  if (go_isnan(x) || go_isnan(y)) return go_nan();
  if (x == 0 && x == y) { if (go_signbit(x)) return y; return x; }
  if (x > y) return x;
  return y;
}

static inline double go_normalize(double x, int* e) {
  const double SmallestNormal = 2.2250738585072014e-308;
  if (go_abs(x) < SmallestNormal) { *e = -52; return x * (double)(1ULL << 52); }
  *e = 0;
  return x;
}

static inline double go_frexp(double f, int* exp) {
  if (f == 0) { *exp = 0; return f; }
  if (go_isinf(f, 0) || go_isnan(f)) { *exp = 0; return f; }
  int e;
  f = go_normalize(f, &e);
  uint64_t x = go_f64bits(f);
  e += (int)((x >> 52) & 0x7FF) - 1023 + 1;
  x &= ~((uint64_t)0x7FF << 52);
  x |= (uint64_t)(-1 + 1023) << 52;
  *exp = e;
  return go_f64frombits(x);
}

static inline double go_ldexp(double frac, int exp) {
  if (frac == 0) return frac;
  if (go_isinf(frac, 0) || go_isnan(frac)) return frac;
  int e;
  frac = go_normalize(frac, &e);
  exp += e;
  uint64_t x = go_f64bits(frac);
  exp += (int)((x >> 52) & 0x7FF) - 1023;
  if (exp < -1075) return go_copysign(0, frac);
  if (exp > 1023) return frac < 0 ? go_inf(-1) : go_inf(1);
  double m = 1;
  if (exp < -1022) { exp += 53; m = 1.0 / (double)(1ULL << 53); }
  x &= ~((uint64_t)0x7FF << 52);
  x |= (uint64_t)(exp + 1023) << 52;
  return m * go_f64frombits(x);
}

static inline double go_modf(double f, double* frac) {
  if (f < 1) {
    if (f < 0) {
      double fr;
      double in = go_modf(-f, &fr);
      *frac = -fr;
      return -in;
    }
    if (f == 0) { *frac = f; return f; }
    *frac = f;
    return 0;
  }
  uint64_t x = go_f64bits(f);
  unsigned e = (unsigned)((x >> 52) & 0x7FF) - 1023u;
  if (e < 64 - 12) x &= ~((1ULL << (64 - 12 - e)) - 1);
  double in = go_f64frombits(x);
  *frac = f - in;
  return in;
}

static inline int go_isoddint(double x) {
  if (go_abs(x) >= (double)(1ULL << 53)) return 0;
  double xf;
  double xi = go_modf(x, &xf);
  return xf == 0 && (((int64_t)xi) & 1) == 1;
}

/* sin.go */
static const double go_sin_c[6] = {
    1.58962301576546568060e-10, -2.50507477628578072866e-8, 2.75573136213857245213e-6,
    -1.98412698295895385996e-4, 8.33333333332211858878e-3, -1.66666666666666307295e-1};
static const double go_cos_c[6] = {
    -1.13585365213876817300e-11, 2.08757008419747316778e-9, -2.75573141792967388112e-7,
    2.48015872888517045348e-5, -1.38888888888730564116e-3, 4.16666666666665929218e-2};
static const double GO_PI4A = 7.85398125648498535156e-1;
static const double GO_PI4B = 3.77489470793079817668e-8;
static const double GO_PI4C = 2.69515142907905952645e-15;
static const double GO_FOUR_OVER_PI = 1.27323954473516268615107010698011489627567716592365; /* 4/Pi */
static const double GO_REDUCE_THRESHOLD = (double)(1 << 29);

static inline double go_cos(double x) {
  if (go_isnan(x) || go_isinf(x, 0)) return go_nan();
  int sign = 0;
  x = go_abs(x);
  if (x >= GO_REDUCE_THRESHOLD) return go_nan();
  uint64_t j = (uint64_t)(x * GO_FOUR_OVER_PI);
  double y = (double)j;
  if ((j & 1) == 1) { j++; y++; }
  j &= 7;
  double z = ((x - y * GO_PI4A) - y * GO_PI4B) - y * GO_PI4C;
  if (j > 3) { j -= 4; sign = !sign; }
  if (j > 1) sign = !sign;
  double zz = z * z;
  if (j == 1 || j == 2) {
    y = z + z * zz * ((((((go_sin_c[0] * zz) + go_sin_c[1]) * zz + go_sin_c[2]) * zz + go_sin_c[3]) * zz + go_sin_c[4]) * zz + go_sin_c[5]);
  } else {
    y = 1.0 - 0.5 * zz + zz * zz * ((((((go_cos_c[0] * zz) + go_cos_c[1]) * zz + go_cos_c[2]) * zz + go_cos_c[3]) * zz + go_cos_c[4]) * zz + go_cos_c[5]);
  }
  if (sign) y = -y;
  return y;
}

static inline double go_sin(double x) {
  if (x == 0 || go_isnan(x)) return x;
  if (go_isinf(x, 0)) return go_nan();
  int sign = 0;
  if (x < 0) { x = -x; sign = 1; }
  if (x >= GO_REDUCE_THRESHOLD) return go_nan();
  uint64_t j = (uint64_t)(x * GO_FOUR_OVER_PI);
  double y = (double)j;
  if ((j & 1) == 1) { j++; y++; }
  j &= 7;
  double z = ((x - y * GO_PI4A) - y * GO_PI4B) - y * GO_PI4C;
  if (j > 3) { sign = !sign; j -= 4; }
  double zz = z * z;
  if (j == 1 || j == 2) {
    y = 1.0 - 0.5 * zz + zz * zz * ((((((go_cos_c[0] * zz) + go_cos_c[1]) * zz + go_cos_c[2]) * zz + go_cos_c[3]) * zz + go_cos_c[4]) * zz + go_cos_c[5]);
  } else {
    y = z + z * zz * ((((((go_sin_c[0] * zz) + go_sin_c[1]) * zz + go_sin_c[2]) * zz + go_sin_c[3]) * zz + go_sin_c[4]) * zz + go_sin_c[5]);
  }
  if (sign) y = -y;
  return y;
}

/* tan.go */
static const double go_tanP[3] = {-1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7};
static const double go_tanQ[5] = {1.0, 1.36812963470692954678e4, -1.32089234440210967447e6, 2.50083801823357915839e7, -5.38695755929454629881e7};
static inline double go_tan(double x) {
  if (x == 0 || go_isnan(x)) return x;
  if (go_isinf(x, 0)) return go_nan();
  int sign = 0;
  if (x < 0) { x = -x; sign = 1; }
  if (x >= GO_REDUCE_THRESHOLD) return go_nan();
  uint64_t j = (uint64_t)(x * GO_FOUR_OVER_PI);
  double y = (double)j;
  if ((j & 1) == 1) { j++; y++; }
  double z = ((x - y * GO_PI4A) - y * GO_PI4B) - y * GO_PI4C;
  double zz = z * z;
  if (zz > 1e-14) {
    y = z + z * (zz * (((go_tanP[0] * zz) + go_tanP[1]) * zz + go_tanP[2]) / ((((zz + go_tanQ[1]) * zz + go_tanQ[2]) * zz + go_tanQ[3]) * zz + go_tanQ[4]));
  } else {
    y = z;
  }
  if ((j & 2) == 2) y = -1 / y;
  if (sign) y = -y;
  return y;
}

/* exp.go */
static inline double go_expmulti(double hi, double lo, int k) {
  const double P1 = 1.66666666666666657415e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  double r = hi - lo;
  double t = r * r;
  double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  double y = 1 - ((lo - (r * c) / (2 - c)) - hi);
  return go_ldexp(y, k);
}
static inline double go_exp(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
               Log2e = 1.44269504088896338700e+00, Overflow = 7.09782712893383973096e+02,
               Underflow = -7.45133219101941108420e+02, NearZero = 1.0 / (double)(1 << 28);
  if (go_isnan(x) || go_isinf(x, 1)) return x;
  if (go_isinf(x, -1)) return 0;
  if (x > Overflow) return go_inf(1);
  if (x < Underflow) return 0;
  if (-NearZero < x && x < NearZero) return 1 + x;
  int k = 0;
  if (x < 0) k = (int)(Log2e * x - 0.5);
  else if (x > 0) k = (int)(Log2e * x + 0.5);
  double hi = x - (double)k * Ln2Hi;
  double lo = (double)k * Ln2Lo;
  return go_expmulti(hi, lo, k);
}

/* log.go */
static inline double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
               L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  const double Sqrt2over2 = 0.70710678118654752440084436210484903928483593768847 ;
  if (go_isnan(x) || go_isinf(x, 1)) return x;
  if (x < 0) return go_nan();
  if (x == 0) return go_inf(-1);
  int ki;
  double f1 = go_frexp(x, &ki);
  if (f1 < Sqrt2over2) { f1 *= 2; ki--; }
  double f = f1 - 1;
  double k = (double)ki;
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

/* pow.go */
static inline double go_pow(double x, double y) {
  if (y == 0 || x == 1) return 1;
  if (y == 1) return x;
  if (go_isnan(x) || go_isnan(y)) return go_nan();
  if (x == 0) {
    if (y < 0) { if (go_signbit(x) && go_isoddint(y)) return go_inf(-1); return go_inf(1); }
    if (y > 0) { if (go_signbit(x) && go_isoddint(y)) return x; return 0; }
  } else if (go_isinf(y, 0)) {
    if (x == -1) return 1;
    if ((go_abs(x) < 1) == go_isinf(y, 1)) return 0;
    return go_inf(1);
  } else if (go_isinf(x, 0)) {
    if (go_isinf(x, -1)) return go_pow(1 / x, -y);
    if (y < 0) return 0;
    if (y > 0) return go_inf(1);
  } else if (y == 0.5) {
    return go_sqrt(x);
  } else if (y == -0.5) {
    return 1 / go_sqrt(x);
  }
  double yf;
  double yi = go_modf(go_abs(y), &yf);
  if (yf != 0 && x < 0) return go_nan();
  if (yi >= 9223372036854775808.0) {
    if (x == -1) return 1;
    if ((go_abs(x) < 1) == (y > 0)) return 0;
    return go_inf(1);
  }
  double a1 = 1.0;
  int ae = 0;
  if (yf != 0) {
    if (yf > 0.5) { yf--; yi++; }
    a1 = go_exp(yf * go_log(x));
  }
  int xe;
  double x1 = go_frexp(x, &xe);
  for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
    if (xe < -(1 << 12) || (1 << 12) < xe) { ae += xe; break; }
    if ((i & 1) == 1) { a1 *= x1; ae += xe; }
    x1 *= x1;
    xe <<= 1;
    if (x1 < .5) { x1 += x1; xe--; }
  }
  if (y < 0) { a1 = 1 / a1; ae = -ae; }
  return go_ldexp(a1, ae);
}

/* atan.go */
static inline double go_xatan(double x) {
  const double P0 = -8.750608600031904122785e-01, P1 = -1.615753718733365076637e+01,
               P2 = -7.500855792314704667340e+01, P3 = -1.228866684490136173410e+02,
               P4 = -6.485021904942025371773e+01, Q0 = +2.485846490142306297962e+01,
               Q1 = +1.650270098316988542046e+02, Q2 = +4.328810604912902668951e+02,
               Q3 = +4.853903996359136964868e+02, Q4 = +1.945506571482613964425e+02;
  double z = x * x;
  z = z * ((((P0 * z + P1) * z + P2) * z + P3) * z + P4) / (((((z + Q0) * z + Q1) * z + Q2) * z + Q3) * z + Q4);
  z = x * z + x;
  return z;
}
static inline double go_satan(double x) {
  const double Morebits = 6.123233995736765886130e-17, Tan3pio8 = 2.41421356237309504880;
  if (x <= 0.66) return go_xatan(x);
  if (x > Tan3pio8) return GO_PI / 2 - go_xatan(1 / x) + Morebits;
  return GO_PI / 4 + go_xatan((x - 1) / (x + 1)) + 0.5 * Morebits;
}
static inline double go_atan(double x) {
  if (x == 0) return x;
  if (x > 0) return go_satan(x);
  return -go_satan(-x);
}
static inline double go_atan2(double y, double x) {
  if (go_isnan(y) || go_isnan(x)) return go_nan();
  if (y == 0) {
    if (x >= 0 && !go_signbit(x)) return go_copysign(0, y);
    return go_copysign(GO_PI, y);
  }
  if (x == 0) return go_copysign(GO_PI / 2, y);
  if (go_isinf(x, 0)) {
    if (go_isinf(x, 1)) { if (go_isinf(y, 0)) return go_copysign(GO_PI / 4, y); return go_copysign(0, y); }
    if (go_isinf(y, 0)) return go_copysign(2.35619449019234492884698253745962716314787704953132936573120844, y);
    return go_copysign(GO_PI, y);
  }
  if (go_isinf(y, 0)) return go_copysign(GO_PI / 2, y);
  double q = go_atan(y / x);
  if (x < 0) { if (q <= 0) return q + GO_PI; return q - GO_PI; }
  return q;
}
/* asin.go */
static inline double go_asin(double x) {
  if (x == 0) return x;
  int sign = 0;
  if (x < 0) { x = -x; sign = 1; }
  if (x > 1) return go_nan();
  double temp = go_sqrt(1 - x * x);
  if (x > 0.7) temp = GO_PI / 2 - go_satan(temp / x);
  else temp = go_satan(x / temp);
  if (sign) temp = -temp;
  return temp;
}

/* nextafter.go: Nextafter32 */
static inline float go_nextafter32(float x, float y) {
  if (x != x || y != y) return go_f32frombits(0x7FC00000u);
  if (x == y) return x;
  if (x == 0) return go_f32frombits(1u | (go_f32bits(y) & 0x80000000u));
  if ((y > x) == (x > 0)) return go_f32frombits(go_f32bits(x) + 1);
  return go_f32frombits(go_f32bits(x) - 1);
}

#endif
