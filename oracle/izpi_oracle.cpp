/* izpi_oracle.cpp — TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * A deterministic CPU restatement of izpi's path-tracing hot path, written in the
 * reference's own shape (interfaces -> virtual classes, recursive samplers, the
 * pointer-tree BVH build) so that it can be read against the Go line by line.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and only as the checker / CPU baseline: the product never routes through it.
 *
 * Reference files restated (all under /root/reference/internal):
 *   fastrandom/fastrandom.go:13-47     LCG
 *   vec3/vec3.go:18-264                vector ops, RandomCosineDirection, RandomToSphere, DeNAN
 *   onb/onb.go:38-67                   BuildFromW, Local
 *   ray/ray.go, hitrecord/hitrecord.go
 *   aabb/aabb.go:26-54                 SurroundingBox, BoxLess*
 *   camera/camera.go:28-89             New, GetRay, GetRayWithLambda, randomInUnitDisc
 *   hitable/bvh4.go:49-164, 478-855    BVH4.Hit, conservative f32, NewBVH4, flatten, collectChildren
 *   hitable/bvh4_simd_generic.go:10-52 RayAABB4 (scalar twin; == amd64 SIMD on non-NaN input)
 *   hitable/triangle.go:61-134,193-326 NewTriangleWithUV, Hit, PDFValue, Random
 *   hitable/sphere.go:29-145           getSphereUV, Hit, BoundingBox, center, PDFValue, Random
 *   hitable/hitable_slice.go:30-110    Hit, PDFValue, Random
 *   material/material.go:10-43         randomInUnitSphere, reflect, refract, schlick
 *   material/lambertian.go, diffuselight.go, dielectric.go, metal.go, pbr.go, isotropic.go
 *   pdf/cosine.go, hitable.go, mixture.go
 *   texture/constant.go, image.go:73-101, spectral_constant.go:65-106, spectral_image.go:64-259
 *   spectral/spectral.go:151-253, firefly_rejection.go:12-113, rgb_image.go:28-67
 *   sampler/colour.go:33-65, sampler/spectral.go:47-80
 *   render/rgb.go:12-57, render/spectral.go:71-106, common/tiles.go, grid/grid.go
 *   transport/transport.go:53-92, 551-680  (lights = IsEmitter hitables; World = Slice{BVH4})
 *   sort.Slice (Go stdlib pdqsort_func, zsortfunc.go) — used by the BVH build
 * Also (not the reference): oracle_lbvh4, a sequential restatement of the GPU BVH4
 * builder of izpi_amd/csrc/bvh_build.hip written from its
 * algorithm description — top-down binary radix splits instead of Karras' parallel
 * construction, a sequential breadth-first collapse (collectChildren's rule, but the
 * inner child with the largest surface area is expanded first) — and oracle_set_bvh, which makes
 * the oracle traverse an externally built tree.
 *
 * Documented deviations from the reference:
 *   * RNG streams are per pixel-sample (splitmix64 of seed and (sample,pixel)), both
 *     for the worker LCG and the camera LCG, instead of per goroutine / one shared
 *     racy camera LCG (renderer.go:128, camera.go:46). Draw ORDER inside a sample is
 *     the reference's.
 *   * The BVH split-axis LCG is seeded with izpi_scene_input.bvh_seed instead of
 *     math/rand (bvh4.go:520).
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>
#include <string>
#include <algorithm>
#include <array>

#include "../include/izpi_host.h"
#include "go_math_ref.h"
#include "cie_tables_ref.h"

namespace orc {

// ------------------------------------------------------------------ counters
struct Counters {
  uint64_t rays = 0, node_visits = 0, tri_tests = 0, sph_tests = 0, light_tri = 0, light_sph = 0, samples = 0;
};
static thread_local Counters g_cnt;
static thread_local uint32_t g_last_prim = 0xFFFFFFFFu;  // side channel: winner of the last BVH4.Hit

// ------------------------------------------------------------------ vec3.go
struct Vec3 { double X = 0, Y = 0, Z = 0; };
static inline Vec3 V(double x, double y, double z) { Vec3 v; v.X = x; v.Y = y; v.Z = z; return v; }
static inline double Length(Vec3 v) { return go_sqrt((v.X * v.X) + (v.Y * v.Y) + (v.Z * v.Z)); }
static inline double SquaredLength(Vec3 v) { return (v.X * v.X) + (v.Y * v.Y) + (v.Z * v.Z); }
static inline Vec3 MakeUnitVector(Vec3 v) { double l = Length(v); v.X = v.X / l; v.Y = v.Y / l; v.Z = v.Z / l; return v; }
static inline Vec3 Add(Vec3 a, Vec3 b) { a.X += b.X; a.Y += b.Y; a.Z += b.Z; return a; }
static inline Vec3 Add(Vec3 a, Vec3 b, Vec3 c) { return Add(Add(a, b), c); }
static inline Vec3 Sub(Vec3 a, Vec3 b) { a.X -= b.X; a.Y -= b.Y; a.Z -= b.Z; return a; }
static inline Vec3 Sub(Vec3 a, Vec3 b, Vec3 c) { return Sub(Sub(a, b), c); }
static inline Vec3 Sub(Vec3 a, Vec3 b, Vec3 c, Vec3 d) { return Sub(Sub(Sub(a, b), c), d); }
static inline Vec3 Mul(Vec3 a, Vec3 b) { return V(a.X * b.X, a.Y * b.Y, a.Z * b.Z); }
static inline Vec3 ScalarMul(Vec3 a, double t) { return V(a.X * t, a.Y * t, a.Z * t); }
static inline Vec3 ScalarDiv(Vec3 a, double t) { return V(a.X / t, a.Y / t, a.Z / t); }
static inline double Dot(Vec3 a, Vec3 b) { return (a.X * b.X) + (a.Y * b.Y) + (a.Z * b.Z); }
static inline Vec3 Cross(Vec3 a, Vec3 b) {
  return V((a.Y * b.Z) - (a.Z * b.Y), -((a.X * b.Z) - (a.Z * b.X)), (a.X * b.Y) - (a.Y * b.X));
}
static inline Vec3 UnitVector(Vec3 v) { return ScalarDiv(v, Length(v)); }
static inline Vec3 Lerp(Vec3 v0, Vec3 v1, double t) {
  return V((1 - t) * v0.X + t * v1.X, (1 - t) * v0.Y + t * v1.Y, (1 - t) * v0.Z + t * v1.Z);
}
static inline Vec3 Min3(Vec3 a, Vec3 b, Vec3 c) {
  double x = GO_MAXFLOAT64, y = GO_MAXFLOAT64, z = GO_MAXFLOAT64;
  if (a.X < x) x = a.X; if (b.X < x) x = b.X; if (c.X < x) x = c.X;
  if (a.Y < y) y = a.Y; if (b.Y < y) y = b.Y; if (c.Y < y) y = c.Y;
  if (a.Z < z) z = a.Z; if (b.Z < z) z = b.Z; if (c.Z < z) z = c.Z;
  return V(x, y, z);
}
static inline Vec3 Max3(Vec3 a, Vec3 b, Vec3 c) {
  double x = -GO_MAXFLOAT64, y = -GO_MAXFLOAT64, z = -GO_MAXFLOAT64;
  if (a.X > x) x = a.X; if (b.X > x) x = b.X; if (c.X > x) x = c.X;
  if (a.Y > y) y = a.Y; if (b.Y > y) y = b.Y; if (c.Y > y) y = c.Y;
  if (a.Z > z) z = a.Z; if (b.Z > z) z = b.Z; if (c.Z > z) z = c.Z;
  return V(x, y, z);
}
static inline int bad(double x) { return go_isnan(x) || go_isinf(x, -1) || go_isinf(x, 1); }
static inline Vec3 DeNAN(Vec3 v) { return V(bad(v.X) ? 0 : v.X, bad(v.Y) ? 0 : v.Y, bad(v.Z) ? 0 : v.Z); }
static inline Vec3 Load(const double* p) { return V(p[0], p[1], p[2]); }

// Go's int(float64) on amd64 (CVTTSD2SQ): NaN / out of range -> INT64_MIN.
static inline int64_t go_int(double x) {
  if (x != x || x >= 9223372036854775808.0 || x < -9223372036854775808.0) return INT64_MIN;
  return (int64_t)x;
}

// ------------------------------------------------------------ fastrandom.go
struct LCG {
  uint64_t state, m, a, c;
  double Float64() {
    state = (a * state + c) % m;
    return (double)state / (double)m;
  }
};
static inline LCG NewLCG(uint64_t seed) { return LCG{seed, 4294967296ULL, 1664525ULL, 1013904223ULL}; }

static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
// Per pixel-sample streams.
static const uint64_t CAMERA_STREAM_SALT = 0xD6E8FEB86659FD93ULL;
static inline uint64_t sample_key(uint32_t pixel, uint32_t s) { return ((uint64_t)s << 32) | (uint64_t)pixel; }

// --------------------------------------------------------- ray / hitrecord
struct Ray { Vec3 o, d; double lambda = 0, time = 0; };
static inline Ray NewRay(Vec3 o, Vec3 d, double time) { Ray r; r.o = o; r.d = d; r.time = time; return r; }
static inline Ray NewRayL(Vec3 o, Vec3 d, double time, double lambda) { Ray r = NewRay(o, d, time); r.lambda = lambda; return r; }
static inline Vec3 PointAtParameter(const Ray& r, double t) { return Add(r.o, ScalarMul(r.d, t)); }

struct HitRecord { double u = 0, v = 0, t = 0; Vec3 p, normal; };
static inline HitRecord NewHR(double t, double u, double v, Vec3 p, Vec3 n) { HitRecord h; h.t = t; h.u = u; h.v = v; h.p = p; h.normal = n; return h; }

// ---------------------------------------------------------------- aabb.go
struct AABB { Vec3 min, max; };
static inline AABB SurroundingBox(const AABB& a, const AABB& b) {
  AABB r;
  r.min = V(go_min(a.min.X, b.min.X), go_min(a.min.Y, b.min.Y), go_min(a.min.Z, b.min.Z));
  r.max = V(go_max(a.max.X, b.max.X), go_max(a.max.Y, b.max.Y), go_max(a.max.Z, b.max.Z));
  return r;
}

// ----------------------------------------------------------------- onb.go
struct Onb {
  Vec3 axis[3];
  void BuildFromW(Vec3 n) {
    axis[2] = UnitVector(n);
    Vec3 a = go_abs(axis[2].X) > 0.9 ? V(0, 1, 0) : V(1, 0, 0);
    axis[1] = UnitVector(Cross(axis[2], a));
    axis[0] = Cross(axis[2], axis[1]);
  }
  Vec3 Local(Vec3 a) const { return Add(ScalarMul(axis[0], a.X), ScalarMul(axis[1], a.Y), ScalarMul(axis[2], a.Z)); }
};

static inline Vec3 RandomCosineDirection(LCG& rnd) {
  double r1 = rnd.Float64();
  double r2 = rnd.Float64();
  double z = go_sqrt(1 - r2);
  double phi = 2 * GO_PI * r1;
  double x = go_cos(phi) * 2 * go_sqrt(r2);
  double y = go_sin(phi) * 2 * go_sqrt(r2);
  return V(x, y, z);
}
static inline Vec3 RandomToSphere(double radius, double distanceSquared, LCG& rnd) {
  double r1 = rnd.Float64();
  double r2 = rnd.Float64();
  double z = 1 + r2 * (go_sqrt(1 - radius * radius / distanceSquared) - 1);
  double phi = 2 * GO_PI * r1;
  double x = go_cos(phi) * go_sqrt(1 - z * z);
  double y = go_sin(phi) * go_sqrt(1 - z * z);
  return V(x, y, z);
}

// ---------------------------------------------------------- spectral.go
struct SPD {
  std::vector<double> wl, val;
  double Value(double w) const {  // spectral.go:151-181
    if (wl.empty()) return 0.0;
    if (w <= wl[0]) return val[0];
    if (w >= wl.back()) return val.back();
    for (size_t i = 0; i + 1 < wl.size(); i++) {
      double w1 = wl[i], w2 = wl[i + 1];
      if (w >= w1 && w <= w2) {
        double t = (w - w1) / (w2 - w1);
        return val[i] + t * (val[i + 1] - val[i]);
      }
    }
    return 0.0;
  }
};

static void SampleWavelength(double random, double* lambda, double* pdf) {  // spectral.go:184-224
  double target = random * ORACLE_CIE_Y_INTEGRAL;
  double current = 0.0;
  *pdf = 0;
  for (int i = 0; i < ORACLE_CIE_N; i++) {
    double y = oracle_cie_y[i];
    if (current + y >= target) {
      if (i > 0) {
        double prev = current;
        double t = (target - prev) / y;
        *lambda = oracle_cie_wavelengths[i - 1] + t * (oracle_cie_wavelengths[i] - oracle_cie_wavelengths[i - 1]);
        double interpolatedY = oracle_cie_y[i - 1] + t * (oracle_cie_y[i] - oracle_cie_y[i - 1]);
        *pdf = interpolatedY / ORACLE_CIE_Y_INTEGRAL;
        return;
      }
      *lambda = oracle_cie_wavelengths[i];
      *pdf = y / ORACLE_CIE_Y_INTEGRAL;
      return;
    }
    current += y;
  }
  *lambda = 750;  // WavelengthMax
  *pdf = oracle_cie_y[ORACLE_CIE_N - 1] / ORACLE_CIE_Y_INTEGRAL;
}

static void GetCIEValues(double w, double* x, double* y, double* z) {  // spectral.go:227-253
  if (w <= oracle_cie_wavelengths[0]) { *x = oracle_cie_x[0]; *y = oracle_cie_y[0]; *z = oracle_cie_z[0]; return; }
  if (w >= oracle_cie_wavelengths[ORACLE_CIE_N - 1]) {
    int l = ORACLE_CIE_N - 1; *x = oracle_cie_x[l]; *y = oracle_cie_y[l]; *z = oracle_cie_z[l]; return;
  }
  int index = 0;
  for (int i = 0; i < ORACLE_CIE_N; i++) if (oracle_cie_wavelengths[i] >= w) { index = i; break; }
  double w1 = oracle_cie_wavelengths[index - 1], w2 = oracle_cie_wavelengths[index];
  double t = (w - w1) / (w2 - w1);
  *x = oracle_cie_x[index - 1] + t * (oracle_cie_x[index] - oracle_cie_x[index - 1]);
  *y = oracle_cie_y[index - 1] + t * (oracle_cie_y[index] - oracle_cie_y[index - 1]);
  *z = oracle_cie_z[index - 1] + t * (oracle_cie_z[index] - oracle_cie_z[index - 1]);
}

// ------------------------------------------------------------- textures
struct Texture { virtual ~Texture() {} virtual Vec3 Value(double u, double v, Vec3 p) const = 0; };
struct SpectralTexture { virtual ~SpectralTexture() {} virtual double Value(double u, double v, double lambda, Vec3 p) const = 0; };

struct ConstantTex : Texture {  // constant.go:20
  Vec3 color;
  Vec3 Value(double, double, Vec3) const override { return color; }
};
struct ImageTex : Texture {  // image.go:73-101 (Float64NRGBA branch)
  int sizeX, sizeY;
  const double* pix;  // row-major, 4 per texel
  Vec3 Value(double u, double v, Vec3) const override {
    int64_t i = go_int(u * (double)sizeX);
    int64_t j = go_int((1 - v) * ((double)sizeY - 0.001));
    if (i < 0) i = 0;
    if (j < 0) j = 0;
    if (i > (int64_t)(sizeX - 1)) i = sizeX - 1;
    if (j > (int64_t)(sizeY - 1)) j = sizeY - 1;
    const double* px = pix + ((size_t)j * sizeX + (size_t)i) * 4;
    return V(px[0], px[1], px[2]);
  }
};
struct SpectralConstantTex : SpectralTexture {  // spectral_constant.go:65-106
  bool tabulated = false;
  double peak = 0, center = 0, width = 0;
  SPD spd;
  double Value(double, double, double lambda, Vec3) const override {
    if (tabulated) {
      if (spd.wl.empty()) return 0.0;
      if (lambda < spd.wl[0]) return spd.val[0];
      if (lambda > spd.wl.back()) return spd.val.back();
      for (size_t i = 0; i + 1 < spd.wl.size(); i++) {
        double w1 = spd.wl[i], w2 = spd.wl[i + 1];
        if (lambda >= w1 && lambda <= w2) {
          double t = (lambda - w1) / (w2 - w1);
          return spd.val[i] + t * (spd.val[i + 1] - spd.val[i]);
        }
      }
      return 0.0;
    }
    double exponent = -go_pow((lambda - center) / width, 2);
    return peak * go_exp(exponent);
  }
};

// spectral_image.go:64-259 (NewSpectralImageFromImage of a Float64NRGBA image): the
// spectral value of every texel at every 5-nm bucket is tabulated up front, as the
// reference does; Value reads the texel ImageTxt.Value would and the first bucket >= lambda.
struct SpectralImageTex : SpectralTexture {
  int sizeX = 0, sizeY = 0;
  std::vector<double> wavelengths;          // 380, 385, ..., 750
  std::vector<std::vector<double>> data;    // [bucket][pixel]
  static double rgbToSpectralValue(double r, double g, double b, double wavelength) {  // :130-190
    double spectralValue = 0;
    if (wavelength >= 580.0 && wavelength <= 750.0) {
      double center = 650.0, distance = go_abs(wavelength - center), width = 60.0;
      double falloff = go_exp(-(distance * distance) / (2.0 * width * width));
      spectralValue += r * falloff;
    }
    if (wavelength >= 480.0 && wavelength <= 620.0) {
      double center = 550.0, distance = go_abs(wavelength - center), width = 60.0;
      double falloff = go_exp(-(distance * distance) / (2.0 * width * width));
      spectralValue += g * falloff;
    }
    if (wavelength >= 380.0 && wavelength <= 520.0) {
      double center = 450.0, distance = go_abs(wavelength - center), width = 60.0;
      double falloff = go_exp(-(distance * distance) / (2.0 * width * width));
      spectralValue += b * falloff;
    }
    if (go_abs(r - g) < 0.15 && go_abs(g - b) < 0.15 && go_abs(r - b) < 0.15) {
      double maxRGB = go_max(r, go_max(g, b));
      spectralValue = go_max(spectralValue, maxRGB);
    }
    double maxRGB = go_max(r, go_max(g, b));
    if (maxRGB > 0.7 && spectralValue < maxRGB * 0.8) spectralValue = go_max(spectralValue, maxRGB * 0.8);
    return go_max(0.0, go_min(1.0, spectralValue));
  }
  void Build(int w, int h, const double* pix) {  // NewSpectralImageFromImage + transformRGBToSpectral
    sizeX = w; sizeY = h;
    for (int k = 0; k < 75; k++) wavelengths.push_back(380.0 + 5.0 * k);
    data.assign(wavelengths.size(), std::vector<double>((size_t)w * h));
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        const double* px = pix + ((size_t)y * w + x) * 4;
        for (size_t i = 0; i < wavelengths.size(); i++) data[i][(size_t)y * w + x] = rgbToSpectralValue(px[0], px[1], px[2], wavelengths[i]);
      }
  }
  int findWavelengthIndex(double lambda) const {
    if (lambda < wavelengths[0]) return 0;
    if (lambda > wavelengths.back()) return (int)wavelengths.size() - 1;
    for (size_t i = 0; i < wavelengths.size(); i++)
      if (lambda <= wavelengths[i]) return (int)i;
    return (int)wavelengths.size() - 1;
  }
  double Value(double u, double v, double lambda, Vec3) const override {
    int64_t i = go_int(u * (double)sizeX);
    int64_t j = go_int((1 - v) * ((double)sizeY - 0.001));
    if (i < 0) i = 0;
    if (j < 0) j = 0;
    if (i > (int64_t)(sizeX - 1)) i = sizeX - 1;
    if (j > (int64_t)(sizeY - 1)) j = sizeY - 1;
    const int64_t pixelIndex = j * sizeX + i;
    const int wi = findWavelengthIndex(lambda);
    if (wi < 0 || wi >= (int)data.size()) return 0.0;
    if (pixelIndex < 0 || pixelIndex >= (int64_t)data[(size_t)wi].size()) return 0.0;
    return data[(size_t)wi][(size_t)pixelIndex];
  }
};

// ---------------------------------------------------------------- pdfs
struct HitableBase;
struct CosinePDF {  // pdf/cosine.go
  Onb uvw;
  void Init(Vec3 w) { uvw.BuildFromW(w); }
  double Value(Vec3 dir) const {
    double cosine = Dot(UnitVector(dir), uvw.axis[2]);
    if (cosine > 0) return cosine / GO_PI;
    return 0;
  }
  Vec3 Generate(LCG& rnd) const { return uvw.Local(RandomCosineDirection(rnd)); }
};

struct ScatterRecord {  // scatterrecord.go
  Ray specularRay;
  bool isSpecular = false;
  Vec3 albedo;
  bool hasPDF = false;
  CosinePDF pdf;
};
struct SpectralScatterRecord {  // spectralscatterrecord.go
  Ray specularRay;
  bool isSpecular = false;
  double albedo = 0, lambda = 0;
  bool hasPDF = false;
  CosinePDF pdf;
};

// ------------------------------------------------------------- materials
struct SceneGeometry;
struct Material {
  virtual ~Material() {}
  virtual bool Scatter(const Ray& r, const HitRecord& hr, LCG& rnd, ScatterRecord& srec) const = 0;
  virtual bool SpectralScatter(const Ray& r, const HitRecord& hr, LCG& rnd, SpectralScatterRecord& srec) const = 0;
  virtual const Texture* NormalMap() const { return nullptr; }
  virtual double ScatteringPDF(const Ray&, const HitRecord&, const Ray&) const { return 0; }
  virtual bool IsEmitter() const { return false; }
  virtual Vec3 Emitted(const Ray&, const HitRecord&, double, double, Vec3) const { return Vec3(); }
  virtual double EmittedSpectral(const Ray&, const HitRecord&, double, double, double, Vec3) const { return 0.0; }
};

static Vec3 randomInUnitSphere(LCG& rnd) {  // material.go:10-18
  for (;;) {
    double x = rnd.Float64(), y = rnd.Float64(), z = rnd.Float64();
    Vec3 p = Sub(ScalarMul(V(x, y, z), 2.0), V(1.0, 1.0, 1.0));
    if (SquaredLength(p) < 1.0) return p;
  }
}
static Vec3 reflect(Vec3 v, Vec3 n) { return Sub(v, ScalarMul(n, 2 * Dot(v, n))); }
static bool refract(Vec3 v, Vec3 n, double niOverNt, Vec3* out) {
  Vec3 uv = UnitVector(v);
  double dt = Dot(uv, n);
  double discriminant = 1.0 - niOverNt * niOverNt * (1 - dt * dt);
  if (discriminant > 0) {
    *out = Sub(ScalarMul(Sub(uv, ScalarMul(n, dt)), niOverNt), ScalarMul(n, go_sqrt(discriminant)));
    return true;
  }
  *out = Vec3();
  return false;
}
static double schlick(double cosine, double refIdx) {
  double r0 = (1.0 - refIdx) / (1.0 + refIdx);
  r0 = r0 * r0;
  return r0 + (1.0 - r0) * go_pow((1.0 - cosine), 5);
}

struct Lambertian : Material {  // lambertian.go
  const Texture* albedo = nullptr;
  const SpectralTexture* spectralAlbedo = nullptr;
  void scatterCommon(const HitRecord& hr, LCG& rnd, CosinePDF& pdf) const {
    Onb uvw;
    uvw.BuildFromW(hr.normal);
    Vec3 direction = uvw.Local(RandomCosineDirection(rnd));
    (void)UnitVector(direction);  // scattered ray: built and discarded by the sampler
    pdf.Init(hr.normal);
  }
  bool Scatter(const Ray& r, const HitRecord& hr, LCG& rnd, ScatterRecord& srec) const override {
    (void)r;
    scatterCommon(hr, rnd, srec.pdf);
    srec.hasPDF = true;
    srec.albedo = albedo->Value(hr.u, hr.v, hr.p);
    srec.isSpecular = false;
    return true;
  }
  bool SpectralScatter(const Ray& r, const HitRecord& hr, LCG& rnd, SpectralScatterRecord& srec) const override {
    scatterCommon(hr, rnd, srec.pdf);
    srec.hasPDF = true;
    srec.lambda = r.lambda;
    srec.albedo = spectralAlbedo->Value(hr.u, hr.v, r.lambda, hr.p);
    srec.isSpecular = false;
    return true;
  }
  double ScatteringPDF(const Ray&, const HitRecord& hr, const Ray& scattered) const override {
    double cosine = Dot(hr.normal, UnitVector(scattered.d));
    if (cosine < 0) cosine = 0;
    return cosine / GO_PI;
  }
};

struct Isotropic : Material {  // isotropic.go
  const Texture* albedo = nullptr;
  bool Scatter(const Ray& r, const HitRecord& hr, LCG& rnd, ScatterRecord& srec) const override {
    (void)r;
    (void)randomInUnitSphere(rnd);  // the scattered ray: built and discarded by the sampler
    srec.albedo = albedo->Value(hr.u, hr.v, hr.p);
    srec.pdf.Init(hr.normal);
    srec.hasPDF = true;
    srec.isSpecular = false;
    return true;
  }
  bool SpectralScatter(const Ray& r, const HitRecord& hr, LCG& rnd, SpectralScatterRecord& srec) const override {
    (void)randomInUnitSphere(rnd);
    srec.lambda = r.lambda;
    srec.albedo = albedo->Value(hr.u, hr.v, hr.p).X;  // "red component as approximation"
    srec.pdf.Init(hr.normal);
    srec.hasPDF = true;
    srec.isSpecular = false;
    return true;
  }
  // ScatteringPDF: 0 (Material's default)
};

struct DiffuseLight : Material {  // diffuselight.go
  const Texture* emit = nullptr;
  const SpectralTexture* spectralEmit = nullptr;
  bool Scatter(const Ray&, const HitRecord&, LCG&, ScatterRecord&) const override { return false; }
  bool SpectralScatter(const Ray&, const HitRecord&, LCG&, SpectralScatterRecord&) const override { return false; }
  Vec3 Emitted(const Ray& rIn, const HitRecord& rec, double u, double v, Vec3 p) const override {
    if (Dot(rec.normal, rIn.d) < 0.0) return emit->Value(u, v, p);
    return Vec3();
  }
  double EmittedSpectral(const Ray& rIn, const HitRecord& rec, double u, double v, double lambda, Vec3 p) const override {
    if (Dot(rec.normal, rIn.d) < 0.0) return spectralEmit->Value(u, v, lambda, p);
    return 0.0;
  }
  bool IsEmitter() const override { return true; }
};

struct SceneGeometry { virtual ~SceneGeometry() {} virtual bool Hit(const Ray& r, double tMin, double tMax, HitRecord& rec, const Material*& mat) const = 0; };

struct Dielectric : Material {  // dielectric.go
  double refIdx = 0;
  const SpectralTexture* spectralRefIdx = nullptr;
  bool computeBeerLambert = false;
  Vec3 absorptionCoeff;
  const SpectralTexture* spectralAbsorptionCoeff = nullptr;
  const SceneGeometry* world = nullptr;

  bool scatterCommon(const Ray& r, const HitRecord& hr, LCG& rnd, double ri, Ray& scattered, bool& isReflected) const {
    double niOverNt, cosine, reflectProb;
    Vec3 outwardNormal, refracted;
    Vec3 reflected = reflect(r.d, hr.normal);
    if (Dot(r.d, hr.normal) > 0) {
      outwardNormal = ScalarMul(hr.normal, -1.0);
      niOverNt = ri;
      cosine = ri * Dot(r.d, hr.normal) / Length(r.d);
    } else {
      outwardNormal = hr.normal;
      niOverNt = 1.0 / ri;
      cosine = -Dot(r.d, hr.normal) / Length(r.d);
    }
    if (refract(r.d, outwardNormal, niOverNt, &refracted)) reflectProb = schlick(cosine, ri);
    else reflectProb = 1.0;
    if (rnd.Float64() < reflectProb) { scattered = NewRayL(hr.p, reflected, r.time, r.lambda); isReflected = true; }
    else { scattered = NewRayL(hr.p, refracted, r.time, r.lambda); isReflected = false; }
    return true;
  }
  double calculatePathLength(const Ray& r, const HitRecord& hr, const Ray& scattered) const {
    double epsilon = 0.001;
    Vec3 startPoint = Add(hr.p, ScalarMul(scattered.d, epsilon));
    Ray traceRay = NewRayL(startPoint, scattered.d, r.time, r.lambda);
    HitRecord exitHit; const Material* m;
    if (world->Hit(traceRay, 0.0, 1000.0, exitHit, m)) {
      double pathLength = Length(Sub(exitHit.p, hr.p));
      if (pathLength < 0.1) pathLength = 0.1;
      if (pathLength > 100.0) pathLength = 100.0;
      return pathLength;
    }
    return 10.0;
  }
  bool Scatter(const Ray& r, const HitRecord& hr, LCG& rnd, ScatterRecord& srec) const override {
    Ray scattered; bool isReflected;
    scatterCommon(r, hr, rnd, refIdx, scattered, isReflected);
    Vec3 att;
    bool absNonZero = !(absorptionCoeff.X == 0 && absorptionCoeff.Y == 0 && absorptionCoeff.Z == 0);
    if (computeBeerLambert && absNonZero && !isReflected) {
      double pathLength = calculatePathLength(r, hr, scattered);
      att = V(go_exp(-absorptionCoeff.X * pathLength), go_exp(-absorptionCoeff.Y * pathLength), go_exp(-absorptionCoeff.Z * pathLength));
    } else {
      att = V(1.0, 1.0, 1.0);
    }
    srec.specularRay = scattered; srec.isSpecular = true; srec.albedo = att; srec.hasPDF = false;
    return true;
  }
  bool SpectralScatter(const Ray& r, const HitRecord& hr, LCG& rnd, SpectralScatterRecord& srec) const override {
    double lambda = r.lambda;
    double ri = spectralRefIdx->Value(hr.u, hr.v, lambda, hr.p);
    Ray scattered; bool isReflected;
    scatterCommon(r, hr, rnd, ri, scattered, isReflected);
    double albedo;
    if (!isReflected) {
      double pathLength = calculatePathLength(r, hr, scattered);
      if (spectralAbsorptionCoeff) albedo = go_exp(-spectralAbsorptionCoeff->Value(hr.u, hr.v, lambda, hr.p) * pathLength);
      else albedo = 1.0;
    } else {
      albedo = 1.0;
    }
    srec.specularRay = scattered; srec.isSpecular = true; srec.albedo = albedo; srec.lambda = lambda; srec.hasPDF = false;
    return true;
  }
  bool IsEmitter() const override { return true; }  // dielectric.go:215-217
};

struct Metal : Material {  // metal.go
  Vec3 albedo; double fuzz = 0;
  bool Scatter(const Ray& r, const HitRecord& hr, LCG& rnd, ScatterRecord& srec) const override {
    Vec3 reflected = reflect(UnitVector(r.d), hr.normal);
    srec.specularRay = NewRay(hr.p, Add(reflected, ScalarMul(randomInUnitSphere(rnd), fuzz)), r.time);
    srec.isSpecular = true; srec.albedo = albedo; srec.hasPDF = false;
    return true;
  }
  bool SpectralScatter(const Ray&, const HitRecord&, LCG&, SpectralScatterRecord&) const override { return false; }
};

struct PBR : Material {  // pbr.go
  const Texture* albedo = nullptr;
  const SpectralTexture* spectralAlbedo = nullptr;
  const Texture* normalMap = nullptr;
  const Texture* roughness = nullptr;
  const Texture* metalness = nullptr;
  const Texture* NormalMap() const override { return normalMap; }

  // Shared body of Scatter / SpectralScatter (pbr.go:59-155 and 158-263 are identical up to the albedo).
  bool common(const Ray& r, const HitRecord& hr, LCG& rnd, Ray& scattered, bool& isSpecular, CosinePDF& pdf) const {
    Vec3 normal;
    if (normalMap) {
      Vec3 normalAtUV = normalMap->Value(hr.u, hr.v, hr.p);
      Vec3 tangentNormal = V(2.0 * normalAtUV.X - 1.0, 2.0 * normalAtUV.Y - 1.0, normalAtUV.Z);
      Vec3 n = hr.normal;
      Vec3 t = Cross(n, V(0, 1, 0));
      if (Dot(t, t) < 0.001) t = Cross(n, V(1, 0, 0));
      t = MakeUnitVector(t);
      Vec3 b = MakeUnitVector(Cross(n, t));
      normal = MakeUnitVector(V(t.X * tangentNormal.X + b.X * tangentNormal.Y + n.X * tangentNormal.Z,
                                t.Y * tangentNormal.X + b.Y * tangentNormal.Y + n.Y * tangentNormal.Z,
                                t.Z * tangentNormal.X + b.Z * tangentNormal.Y + n.Z * tangentNormal.Z));
    } else {
      normal = hr.normal;
    }
    Vec3 rough = roughness ? roughness->Value(hr.u, hr.v, hr.p) : V(0.5, 0.5, 0.5);
    Vec3 metal = metalness ? metalness->Value(hr.u, hr.v, hr.p) : V(0.0, 0.0, 0.0);
    double roughnessValue = (rough.X + rough.Y + rough.Z) / 3.0;
    double metalnessValue = (metal.X + metal.Y + metal.Z) / 3.0;
    Onb uvw;
    uvw.BuildFromW(normal);
    Vec3 reflected = reflect(UnitVector(r.d), normal);
    double cosTheta = go_abs(Dot(UnitVector(r.d), normal));
    double fresnel = 0.04 + (1.0 - 0.04) * go_pow(1.0 - cosTheta, 5.0);
    fresnel = fresnel + (metalnessValue * 0.5);
    double specularProbability = fresnel * (1.0 - roughnessValue);
    Vec3 finalDir;
    if (rnd.Float64() < specularProbability) {
      double roughnessFactor = go_max(0.01, roughnessValue * 0.3);
      Vec3 randomDir = randomInUnitSphere(rnd);
      finalDir = UnitVector(Add(reflected, ScalarMul(randomDir, roughnessFactor)));
      isSpecular = true;
    } else {
      finalDir = UnitVector(uvw.Local(RandomCosineDirection(rnd)));
      isSpecular = false;
    }
    scattered = NewRayL(hr.p, finalDir, r.time, r.lambda);
    pdf.Init(normal);
    return true;
  }
  bool Scatter(const Ray& r, const HitRecord& hr, LCG& rnd, ScatterRecord& srec) const override {
    Vec3 alb = albedo->Value(hr.u, hr.v, hr.p);
    Ray sc; bool spec;
    common(r, hr, rnd, sc, spec, srec.pdf);
    srec.specularRay = NewRay(sc.o, sc.d, sc.time);
    srec.isSpecular = spec; srec.albedo = alb; srec.hasPDF = true;
    return true;
  }
  bool SpectralScatter(const Ray& r, const HitRecord& hr, LCG& rnd, SpectralScatterRecord& srec) const override {
    double alb;
    if (spectralAlbedo) alb = spectralAlbedo->Value(hr.u, hr.v, r.lambda, hr.p);
    else { Vec3 c = albedo->Value(hr.u, hr.v, hr.p); alb = 0.299 * c.X + 0.587 * c.Y + 0.114 * c.Z; }
    Ray sc; bool spec;
    common(r, hr, rnd, sc, spec, srec.pdf);
    srec.specularRay = sc;
    srec.isSpecular = spec;
    srec.albedo = spec ? alb * 1.5 : alb;
    srec.lambda = r.lambda; srec.hasPDF = true;
    return true;
  }
  double ScatteringPDF(const Ray&, const HitRecord& hr, const Ray& scattered) const override {
    double cosine = Dot(hr.normal, UnitVector(scattered.d));
    if (cosine < 0) cosine = 0;
    return cosine / GO_PI;
  }
};

// -------------------------------------------------------------- hitables
struct Hitable {
  virtual ~Hitable() {}
  virtual bool Hit(const Ray& r, double tMin, double tMax, HitRecord& rec, const Material*& mat) const = 0;
  virtual AABB BoundingBox() const = 0;
  virtual double PDFValue(Vec3 o, Vec3 v) const = 0;
  virtual Vec3 Random(Vec3 o, LCG& rnd) const = 0;
  virtual bool IsEmitter() const = 0;
  uint32_t ref = 0;  // IZPI_PRIM_REF in transport order
};

struct Mat3 { double A11, A12, A13, A21, A22, A23, A31, A32, A33; };  // mat3.go:6-16
// mat3.go:19-31: the tangent, bitangent and normal as the matrix's columns
Mat3 NewTBN(Vec3 t, Vec3 b, Vec3 n) { return Mat3{t.X, b.X, n.X, t.Y, b.Y, n.Y, t.Z, b.Z, n.Z}; }
// mat3.go:34-40 (no FMA: Go on amd64 rounds each product and sum)
Vec3 MatrixVectorMul(const Mat3& a, Vec3 v) {
  return V(a.A11 * v.X + a.A12 * v.Y + a.A13 * v.Z, a.A21 * v.X + a.A22 * v.Y + a.A23 * v.Z,
           a.A31 * v.X + a.A32 * v.Y + a.A33 * v.Z);
}

struct Triangle : Hitable {  // triangle.go
  Vec3 vertex0, vertex1, vertex2, edge1, edge2, normal, tangent, bitangent;
  double area = 0, u0 = 0, u1 = 0, u2 = 0, v0 = 0, v1 = 0, v2 = 0;
  const Material* material = nullptr;
  AABB bb;

  static Triangle* NewWithUV(Vec3 a, Vec3 b, Vec3 c, double u0, double v0, double u1, double v1, double u2, double v2, const Material* m) {
    Vec3 e1 = Sub(b, a), e2 = Sub(c, a);
    Vec3 normal = MakeUnitVector(Cross(e1, e2));
    Triangle* t = new Triangle();
    double deltaU1 = u1 - u0, deltaU2 = u2 - u0, deltaV1 = v1 - v0, deltaV2 = v2 - v0;
    Vec3 n = Cross(e1, e2);
    t->area = Length(n) / 2.0;
    double f = 1.0 / (deltaU1 * deltaV2 - deltaU2 * deltaV1);
    t->tangent = MakeUnitVector(V(f * (deltaV2 * e1.X - deltaV1 * e2.X), f * (deltaV2 * e1.Y - deltaV1 * e2.Y), f * (deltaV2 * e1.Z - deltaV1 * e2.Z)));
    t->bitangent = MakeUnitVector(V(f * (-deltaU2 * e1.X + deltaU1 * e2.X), f * (-deltaU2 * e1.Y + deltaU1 * e2.Y), f * (-deltaU2 * e1.Z + deltaU1 * e2.Z)));
    Vec3 mn = Min3(a, b, c), mx = Max3(a, b, c);
    Vec3 size = Sub(mx, mn);
    double maxDim = go_max(size.X, go_max(size.Y, size.Z));
    double eps = go_max(maxDim * 1e-4, 1e-6);
    Vec3 delta = V(eps, eps, eps);
    t->bb.min = Sub(mn, delta);
    t->bb.max = Add(mx, delta);
    t->vertex0 = a; t->vertex1 = b; t->vertex2 = c; t->edge1 = e1; t->edge2 = e2; t->normal = normal;
    t->u0 = u0; t->u1 = u1; t->u2 = u2; t->v0 = v0; t->v1 = v1; t->v2 = v2; t->material = m;
    return t;
  }
  // Möller–Trumbore acceptance (triangle.go:193-221); returns t,u,v.
  bool intersect(const Ray& r, double tMin, double tMax, double& t, double& u, double& v) const {
    const double epsilon = 1e-8;
    Vec3 h = Cross(r.d, edge2);
    double a = Dot(edge1, h);
    if (go_abs(a) < epsilon) return false;
    double f = 1.0 / a;
    Vec3 s = Sub(r.o, vertex0);
    u = f * Dot(s, h);
    if (u < -epsilon || u > 1.0 + epsilon) return false;
    Vec3 q = Cross(s, edge1);
    v = f * Dot(r.d, q);
    if (v < -epsilon || u + v > 1.0 + epsilon) return false;
    t = f * Dot(edge2, q);
    if (t < tMin || t > tMax) return false;
    return true;
  }
  bool Hit(const Ray& r, double tMin, double tMax, HitRecord& rec, const Material*& mat) const override {
    const double epsilon = 1e-8;
    double t, u, v;
    if (!intersect(r, tMin, tMax, t, u, v)) return false;
    double w = 1.0 - u - v;
    double sum = u + v + w;
    if (go_abs(sum - 1.0) > epsilon) { u /= sum; v /= sum; w /= sum; }
    double uu = w * u0 + u * u1 + v * u2;
    double vv = w * v0 + u * v1 + v * v2;
    Vec3 nrm = normal;
    const Texture* nm = material->NormalMap();
    mat = material;
    if (!nm) { rec = NewHR(t, uu, vv, PointAtParameter(r, t), nrm); return true; }
    Vec3 nts = nm->Value(uu, vv, Vec3());
    nts.X = 2 * nts.X - 1.0; nts.Y = 2 * nts.Y - 1.0; nts.Z = 2 * nts.Z - 1.0;
    Vec3 nn = MatrixVectorMul(NewTBN(tangent, bitangent, nrm), nts);  // triangle.go:260-261
    rec = NewHR(t, uu, vv, PointAtParameter(r, t), MakeUnitVector(nn));
    return true;
  }
  AABB BoundingBox() const override { return bb; }
  double PDFValue(Vec3 o, Vec3 v) const override {
    g_cnt.light_tri++;
    Ray r = NewRay(o, v, 0);
    HitRecord rec; const Material* m;
    if (Hit(r, 0.001, GO_MAXFLOAT64, rec, m)) {
      double distanceSquared = rec.t * rec.t * SquaredLength(v);
      double cosine = go_abs(Dot(v, ScalarDiv(rec.normal, Length(v))));
      return distanceSquared / (cosine * area);
    }
    return 0;
  }
  Vec3 Random(Vec3 o, LCG& rnd) const override {
    double t1 = rnd.Float64();
    Vec3 p01 = Lerp(vertex0, vertex1, t1);
    double t2 = rnd.Float64();
    Vec3 p02 = Lerp(vertex0, vertex2, t2);
    double t3 = rnd.Float64();
    Vec3 p = Lerp(p01, p02, t3);
    return Sub(p, o);
  }
  bool IsEmitter() const override { return material->IsEmitter(); }
};

static void getSphereUV(Vec3 p, double* u, double* v) {  // sphere.go:29-35
  double phi = go_atan2(p.Z, p.X);
  double theta = go_asin(p.Y);
  *u = 1.0 - (phi + GO_PI) / (2.0 * GO_PI);
  *v = (theta + GO_PI / 2.0) / GO_PI;
}

struct Sphere : Hitable {  // sphere.go
  Vec3 center0, center1; double time0 = 0, time1 = 1, radius = 0;
  const Material* material = nullptr;
  Vec3 center(double time) const {
    return Add(center0, ScalarMul(Sub(center1, center0), ((time - time0) / (time1 - time0))));
  }
  bool Hit(const Ray& r, double tMin, double tMax, HitRecord& rec, const Material*& mat) const override {
    Vec3 oc = Sub(r.o, center(r.time));
    double a = Dot(r.d, r.d);
    double b = Dot(oc, r.d);
    double c = Dot(oc, oc) - (radius * radius);
    double discriminant = (b * b) - (a * c);
    if (discriminant > 0) {
      double temp = (-b - go_sqrt(b * b - a * c)) / a;
      if (temp < tMax && temp > tMin) {
        Vec3 on = ScalarDiv(Sub(PointAtParameter(r, temp), center(r.time)), radius);
        if (Dot(r.d, on) >= 0) on = ScalarMul(on, -1);
        double u, v; getSphereUV(on, &u, &v);
        rec = NewHR(temp, u, v, PointAtParameter(r, temp), on);
        mat = material;
        return true;
      }
      temp = (-b + go_sqrt(b * b - a * c)) / a;
      if (temp < tMax && temp > tMin) {
        Vec3 on = ScalarDiv(Sub(PointAtParameter(r, temp), center(r.time)), radius);
        if (Dot(r.d, on) >= 0) on = ScalarMul(on, -1);
        double u, v; getSphereUV(on, &u, &v);
        rec = NewHR(temp, u, v, PointAtParameter(r, temp), ScalarDiv(Sub(PointAtParameter(r, temp), center(r.time)), radius));
        mat = material;
        return true;
      }
    }
    return false;
  }
  AABB BoundingBox() const override {
    AABB b0, b1;
    b0.min = Sub(center0, V(radius, radius, radius)); b0.max = Add(center0, V(radius, radius, radius));
    b1.min = Sub(center1, V(radius, radius, radius)); b1.max = Add(center1, V(radius, radius, radius));
    return SurroundingBox(b0, b1);
  }
  double PDFValue(Vec3 o, Vec3 v) const override {
    g_cnt.light_sph++;
    HitRecord rec; const Material* m;
    if (Hit(NewRay(o, v, 0), 0.001, GO_MAXFLOAT64, rec, m)) {
      double cosThetaMax = go_sqrt(1 - radius * radius / SquaredLength(Sub(center0, o)));
      double solidAngle = 2 * GO_PI * (1 - cosThetaMax);
      return 1 / solidAngle;
    }
    return 0.0;
  }
  Vec3 Random(Vec3 o, LCG& rnd) const override {
    Vec3 direction = Sub(center0, o);
    double distanceSquared = SquaredLength(direction);
    Onb uvw; uvw.BuildFromW(direction);
    return uvw.Local(RandomToSphere(radius, distanceSquared, rnd));
  }
  bool IsEmitter() const override { return material->IsEmitter(); }
};

// ------------------------------------------------------------------ BVH4
// bvh4_simd_generic.go:10-52
static inline float min32(float a, float b) { return a < b ? a : b; }
static inline float max32(float a, float b) { return a > b ? a : b; }
static uint8_t RayAABB4(float ox, float oy, float oz, float ix, float iy, float iz, const float* minX, const float* minY,
                        const float* minZ, const float* maxX, const float* maxY, const float* maxZ, float tMax) {
  uint8_t mask = 0;
  for (int i = 0; i < 4; i++) {
    float t0x = (minX[i] - ox) * ix, t1x = (maxX[i] - ox) * ix;
    if (t0x > t1x) { float t = t0x; t0x = t1x; t1x = t; }
    float t0y = (minY[i] - oy) * iy, t1y = (maxY[i] - oy) * iy;
    if (t0y > t1y) { float t = t0y; t0y = t1y; t1y = t; }
    float t0z = (minZ[i] - oz) * iz, t1z = (maxZ[i] - oz) * iz;
    if (t0z > t1z) { float t = t0z; t0z = t1z; t1z = t; }
    float tNear = max32(max32(t0x, t0y), t0z);
    float tFar = min32(min32(t1x, t1y), t1z);
    if (tNear <= tFar && tFar >= 0 && tNear <= tMax) mask |= (uint8_t)(1 << i);
  }
  return mask;
}

static float conservativeFloat32Min(double val) {  // bvh4.go:494-502
  float f32 = (float)val;
  if ((double)f32 > val) return go_nextafter32(f32, -INFINITY);
  return f32;
}
static float conservativeFloat32Max(double val) {  // bvh4.go:506-514
  float f32 = (float)val;
  if ((double)f32 < val) return go_nextafter32(f32, INFINITY);
  return f32;
}

struct BVH4 : Hitable {
  std::vector<izpi_bvh4_node> Nodes;
  std::vector<const Hitable*> Primitives;
  bool Hit(const Ray& r, double tMin, double tMax, HitRecord& best, const Material*& bestMat) const override {
    if (Nodes.empty()) return false;
    bool hitFound = false;
    Vec3 inv = V(1.0 / r.d.X, 1.0 / r.d.Y, 1.0 / r.d.Z);
    float rInvX = (float)inv.X, rInvY = (float)inv.Y, rInvZ = (float)inv.Z;
    float rOrgX = (float)r.o.X, rOrgY = (float)r.o.Y, rOrgZ = (float)r.o.Z;
    int32_t stack[64];
    int32_t stackPtr = 0;
    int32_t cur = 0;
    for (;;) {
      if (cur == -1) break;
      if (cur >= (int32_t)Nodes.size()) break;
      const izpi_bvh4_node& node = Nodes[(size_t)cur];
      g_cnt.node_visits++;
      uint8_t mask = RayAABB4(rOrgX, rOrgY, rOrgZ, rInvX, rInvY, rInvZ, node.min_x, node.min_y, node.min_z, node.max_x,
                              node.max_y, node.max_z, (float)tMax);
      int32_t next = -1;
      for (int i = 0; i < 4; i++) {
        if (((mask >> i) & 1) == 0) continue;
        int32_t childIndex = node.child[i];
        int32_t primitiveCount = node.prim_count[i];
        if (childIndex == -1) continue;
        if (primitiveCount > 0) {
          for (int32_t p = 0; p < primitiveCount; p++) {
            const Hitable* prim = Primitives[(size_t)(childIndex + p)];
            if (IZPI_PRIM_KIND(prim->ref) == IZPI_PRIM_TRIANGLE) g_cnt.tri_tests++; else g_cnt.sph_tests++;
            HitRecord rec; const Material* m;
            if (prim->Hit(r, tMin, tMax, rec, m)) {
              tMax = rec.t; best = rec; bestMat = m; hitFound = true; g_last_prim = prim->ref;
            }
          }
        } else {
          if (next == -1) next = childIndex;
          else {
            if (stackPtr >= 64) { fprintf(stderr, "oracle: BVH4 stack overflow (Go would panic)\n"); abort(); }
            stack[stackPtr++] = childIndex;
          }
        }
      }
      if (next != -1) cur = next;
      else if (stackPtr > 0) cur = stack[--stackPtr];
      else cur = -1;
    }
    return hitFound;
  }
  AABB BoundingBox() const override { AABB b; return b; }
  double PDFValue(Vec3, Vec3) const override { return 0.0; }
  Vec3 Random(Vec3, LCG&) const override { return V(1, 0, 0); }
  bool IsEmitter() const override { return false; }
};

// --- Go sort.Slice = pdqsort_func (sort/zsortfunc.go), restated over index pairs.
struct SortData {
  std::vector<const Hitable*>* h;
  std::vector<int>* idx;
  std::vector<double>* key;  // box.min[axis] cached per element (BoxLess* compares it with <)
  bool Less(int i, int j) const { return (*key)[(size_t)i] < (*key)[(size_t)j]; }
  void Swap(int i, int j) {
    std::swap((*h)[(size_t)i], (*h)[(size_t)j]);
    std::swap((*idx)[(size_t)i], (*idx)[(size_t)j]);
    std::swap((*key)[(size_t)i], (*key)[(size_t)j]);
  }
};
static void insertionSort(SortData& d, int a, int b) {
  for (int i = a + 1; i < b; i++)
    for (int j = i; j > a && d.Less(j, j - 1); j--) d.Swap(j, j - 1);
}
static void siftDown(SortData& d, int lo, int hi, int first) {
  int root = lo;
  for (;;) {
    int child = 2 * root + 1;
    if (child >= hi) return;
    if (child + 1 < hi && d.Less(first + child, first + child + 1)) child++;
    if (!d.Less(first + root, first + child)) return;
    d.Swap(first + root, first + child);
    root = child;
  }
}
static void heapSort(SortData& d, int a, int b) {
  int first = a, lo = 0, hi = b - a;
  for (int i = (hi - 1) / 2; i >= 0; i--) siftDown(d, i, hi, first);
  for (int i = hi - 1; i >= 0; i--) { d.Swap(first, first + i); siftDown(d, lo, i, first); }
}
static int bitsLen(uint64_t x) { int n = 0; while (x) { n++; x >>= 1; } return n; }
static void breakPatterns(SortData& d, int a, int b) {
  int length = b - a;
  if (length >= 8) {
    uint64_t random = (uint64_t)length;
    uint64_t modulus = 1ULL << bitsLen((uint64_t)length);
    int idx = a + (length / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
      random ^= random << 13; random ^= random >> 7; random ^= random << 17;
      int other = (int)((unsigned)random & (unsigned)(modulus - 1));
      if (other >= length) other -= length;
      d.Swap(idx - 1 + i, a + other);
    }
  }
}
static void order2(SortData& d, int a, int b, int* swaps, int* x, int* y) {
  if (d.Less(b, a)) { (*swaps)++; *x = b; *y = a; return; }
  *x = a; *y = b;
}
static int median(SortData& d, int a, int b, int c, int* swaps) {
  order2(d, a, b, swaps, &a, &b);
  order2(d, b, c, swaps, &b, &c);
  order2(d, a, b, swaps, &a, &b);
  return b;
}
static int medianAdjacent(SortData& d, int a, int* swaps) { return median(d, a - 1, a, a + 1, swaps); }
enum { unknownHint = 0, increasingHint = 1, decreasingHint = 2 };
static int choosePivot(SortData& d, int a, int b, int* hint) {
  const int shortestNinther = 50, maxSwaps = 4 * 3;
  int l = b - a;
  int swaps = 0;
  int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
  if (l >= 8) {
    if (l >= shortestNinther) {
      i = medianAdjacent(d, i, &swaps);
      j = medianAdjacent(d, j, &swaps);
      k = medianAdjacent(d, k, &swaps);
    }
    j = median(d, i, j, k, &swaps);
  }
  if (swaps == 0) *hint = increasingHint;
  else if (swaps == maxSwaps) *hint = decreasingHint;
  else *hint = unknownHint;
  return j;
}
static void reverseRange(SortData& d, int a, int b) {
  int i = a, j = b - 1;
  while (i < j) { d.Swap(i, j); i++; j--; }
}
static bool partialInsertionSort(SortData& d, int a, int b) {
  const int maxSteps = 5, shortestShifting = 50;
  int i = a + 1;
  for (int j = 0; j < maxSteps; j++) {
    while (i < b && !d.Less(i, i - 1)) i++;
    if (i == b) return true;
    if (b - a < shortestShifting) return false;
    d.Swap(i, i - 1);
    if (i - a >= 2) {
      for (int k = i - 1; k >= 1; k--) { if (!d.Less(k, k - 1)) break; d.Swap(k, k - 1); }
    }
    if (b - i >= 2) {
      for (int k = i + 1; k < b; k++) { if (!d.Less(k, k - 1)) break; d.Swap(k, k - 1); }
    }
  }
  return false;
}
static int partitionEqual(SortData& d, int a, int b, int pivot) {
  d.Swap(a, pivot);
  int i = a + 1, j = b - 1;
  for (;;) {
    while (i <= j && !d.Less(a, i)) i++;
    while (i <= j && d.Less(a, j)) j--;
    if (i > j) break;
    d.Swap(i, j); i++; j--;
  }
  return i;
}
static int partition(SortData& d, int a, int b, int pivot, bool* already) {
  d.Swap(a, pivot);
  int i = a + 1, j = b - 1;
  while (i <= j && d.Less(i, a)) i++;
  while (i <= j && !d.Less(j, a)) j--;
  if (i > j) { d.Swap(j, a); *already = true; return j; }
  d.Swap(i, j); i++; j--;
  for (;;) {
    while (i <= j && d.Less(i, a)) i++;
    while (i <= j && !d.Less(j, a)) j--;
    if (i > j) break;
    d.Swap(i, j); i++; j--;
  }
  d.Swap(j, a);
  *already = false;
  return j;
}
static void pdqsort(SortData& d, int a, int b, int limit) {
  const int maxInsertion = 12;
  bool wasBalanced = true, wasPartitioned = true;
  for (;;) {
    int length = b - a;
    if (length <= maxInsertion) { insertionSort(d, a, b); return; }
    if (limit == 0) { heapSort(d, a, b); return; }
    if (!wasBalanced) { breakPatterns(d, a, b); limit--; }
    int hint;
    int pivot = choosePivot(d, a, b, &hint);
    if (hint == decreasingHint) {
      reverseRange(d, a, b);
      pivot = (b - 1) - (pivot - a);
      hint = increasingHint;
    }
    if (wasBalanced && wasPartitioned && hint == increasingHint) {
      if (partialInsertionSort(d, a, b)) return;
    }
    if (a > 0 && !d.Less(a - 1, pivot)) {
      int mid = partitionEqual(d, a, b, pivot);
      a = mid;
      continue;
    }
    bool already;
    int mid = partition(d, a, b, pivot, &already);
    wasPartitioned = already;
    int leftLen = mid - a, rightLen = b - mid;
    int balanceThreshold = length / 8;
    if (leftLen < rightLen) {
      wasBalanced = leftLen >= balanceThreshold;
      pdqsort(d, a, mid, limit);
      a = mid + 1;
    } else {
      wasBalanced = rightLen >= balanceThreshold;
      pdqsort(d, mid + 1, b, limit);
      b = mid;
    }
  }
}

struct BuildNode {
  bool hasBox = false;
  AABB box;
  std::vector<BuildNode*> children;
  std::vector<int> primitiveIndices;
};

static BuildNode* buildBinaryBVH(std::vector<const Hitable*> hitables, std::vector<int> indices, LCG& rnd) {
  if (hitables.empty()) return nullptr;
  BuildNode* node = new BuildNode();
  if (hitables.size() == 1) {
    node->primitiveIndices = indices;
    node->box = hitables[0]->BoundingBox();
    node->hasBox = true;
    return node;
  }
  AABB overall = hitables[0]->BoundingBox();
  for (size_t i = 1; i < hitables.size(); i++) overall = SurroundingBox(overall, hitables[i]->BoundingBox());
  node->box = overall; node->hasBox = true;
  int axis = (int)(3 * rnd.Float64());
  std::vector<double> key(hitables.size());
  for (size_t i = 0; i < hitables.size(); i++) {
    AABB b = hitables[i]->BoundingBox();
    key[i] = axis == 0 ? b.min.X : (axis == 1 ? b.min.Y : b.min.Z);
  }
  SortData sd{&hitables, &indices, &key};
  int n = (int)hitables.size();
  pdqsort(sd, 0, n, bitsLen((uint64_t)n));
  if (hitables.size() <= 4) { node->primitiveIndices = indices; return node; }
  size_t mid = hitables.size() / 2;
  BuildNode* l = buildBinaryBVH(std::vector<const Hitable*>(hitables.begin(), hitables.begin() + (long)mid),
                                std::vector<int>(indices.begin(), indices.begin() + (long)mid), rnd);
  BuildNode* r = buildBinaryBVH(std::vector<const Hitable*>(hitables.begin() + (long)mid, hitables.end()),
                                std::vector<int>(indices.begin() + (long)mid, indices.end()), rnd);
  node->children = {l, r};
  return node;
}

static std::vector<BuildNode*> collectChildren(BuildNode* node, size_t maxChildren) {
  if (node == nullptr || !node->primitiveIndices.empty()) return {node};
  if (node->children.empty()) return {node};
  std::vector<BuildNode*> result;
  for (BuildNode* c : node->children) if (c) result.push_back(c);
  bool expanded = true;
  while (expanded && result.size() < maxChildren) {
    expanded = false;
    for (size_t i = 0; i < result.size(); i++) {
      BuildNode* cur = result[i];
      if (!cur->primitiveIndices.empty()) continue;
      if (cur->children.empty()) continue;
      size_t after = result.size() - 1 + cur->children.size();
      if (after <= maxChildren) {
        result.erase(result.begin() + (long)i);
        for (BuildNode* c : cur->children) result.push_back(c);
        expanded = true;
        break;
      }
    }
  }
  if (result.size() > maxChildren) result.resize(maxChildren);
  return result;
}

static int32_t flattenBVH4(BuildNode* node, BVH4& bvh, std::vector<int>& prims) {
  if (!node) return -1;
  int32_t nodeIndex = (int32_t)bvh.Nodes.size();
  izpi_bvh4_node n;
  for (int i = 0; i < 4; i++) {
    n.child[i] = -1; n.prim_count[i] = 0;
    n.min_x[i] = n.min_y[i] = n.min_z[i] = n.max_x[i] = n.max_y[i] = n.max_z[i] = GO_MAXFLOAT32;
  }
  if (!node->primitiveIndices.empty()) {
    int32_t primStart = (int32_t)prims.size();
    prims.insert(prims.end(), node->primitiveIndices.begin(), node->primitiveIndices.end());
    n.child[0] = primStart;
    n.prim_count[0] = (int32_t)node->primitiveIndices.size();
    if (node->hasBox) {
      n.min_x[0] = conservativeFloat32Min(node->box.min.X); n.min_y[0] = conservativeFloat32Min(node->box.min.Y);
      n.min_z[0] = conservativeFloat32Min(node->box.min.Z); n.max_x[0] = conservativeFloat32Max(node->box.max.X);
      n.max_y[0] = conservativeFloat32Max(node->box.max.Y); n.max_z[0] = conservativeFloat32Max(node->box.max.Z);
    }
    bvh.Nodes.push_back(n);
    return nodeIndex;
  }
  std::vector<BuildNode*> children = collectChildren(node, 4);
  bvh.Nodes.push_back(n);
  for (size_t i = 0; i < children.size() && i < 4; i++) {
    BuildNode* child = children[i];
    int32_t ci = flattenBVH4(child, bvh, prims);
    izpi_bvh4_node& p = bvh.Nodes[(size_t)nodeIndex];
    p.child[i] = ci;
    if (child->hasBox) {
      p.min_x[i] = conservativeFloat32Min(child->box.min.X); p.min_y[i] = conservativeFloat32Min(child->box.min.Y);
      p.min_z[i] = conservativeFloat32Min(child->box.min.Z); p.max_x[i] = conservativeFloat32Max(child->box.max.X);
      p.max_y[i] = conservativeFloat32Max(child->box.max.Y); p.max_z[i] = conservativeFloat32Max(child->box.max.Z);
    }
  }
  return nodeIndex;
}
static void freeTree(BuildNode* n) { if (!n) return; for (BuildNode* c : n->children) freeTree(c); delete n; }

struct HitableSlice : Hitable, SceneGeometry {  // hitable_slice.go
  std::vector<const Hitable*> hitables;
  bool Hit(const Ray& r, double tMin, double tMax, HitRecord& rec, const Material*& mat) const override {
    bool hitAnything = false;
    double closest = tMax;
    for (const Hitable* h : hitables) {
      HitRecord tr; const Material* tm;
      if (h->Hit(r, tMin, closest, tr, tm)) { rec = tr; mat = tm; hitAnything = true; closest = rec.t; }
    }
    return hitAnything;
  }
  AABB BoundingBox() const override { AABB b; return b; }
  double PDFValue(Vec3 o, Vec3 v) const override {
    double weight = 1.0 / (double)hitables.size();
    double sum = 0;
    for (const Hitable* h : hitables) sum += weight * h->PDFValue(o, v);
    return sum;
  }
  Vec3 Random(Vec3 o, LCG& rnd) const override {
    int64_t index = go_int(rnd.Float64() * (double)hitables.size());
    return hitables[(size_t)index]->Random(o, rnd);
  }
  bool IsEmitter() const override { return false; }
};

// -------------------------------------------------------------- camera.go
struct Camera {
  double lensRadius, time0, time1, exposure;
  Vec3 u, v, origin, lowerLeftCorner, horizontal, vertical;
  static Camera New(Vec3 lookFrom, Vec3 lookAt, Vec3 vup, double vfov, double aspect, double aperture, double focusDist,
                    double t0, double t1, double exposure) {
    Camera c;
    c.lensRadius = aperture / 2.0;
    double theta = vfov * GO_PI / 180;
    double halfHeight = go_tan(theta / 2.0);
    double halfWidth = aspect * halfHeight;
    Vec3 w = UnitVector(Sub(lookFrom, lookAt));
    c.u = UnitVector(Cross(vup, w));
    c.v = Cross(w, c.u);
    c.lowerLeftCorner = Sub(lookFrom, ScalarMul(c.u, halfWidth * focusDist), ScalarMul(c.v, halfHeight * focusDist), ScalarMul(w, focusDist));
    c.horizontal = ScalarMul(c.u, 2.0 * halfWidth * focusDist);
    c.vertical = ScalarMul(c.v, 2.0 * halfHeight * focusDist);
    c.origin = lookFrom;
    c.time0 = t0; c.time1 = t1; c.exposure = exposure;
    return c;
  }
  Vec3 randomInUnitDisc(LCG& rnd) const {
    for (;;) {
      double x = rnd.Float64(), y = rnd.Float64();
      Vec3 p = Sub(ScalarMul(V(x, y, 0), 2.0), V(1.0, 1.0, 0));
      if (Dot(p, p) < 1.0) return p;
    }
  }
  Ray GetRay(double s, double t, LCG& camRnd, double lambda) const {
    Vec3 rd = ScalarMul(randomInUnitDisc(camRnd), lensRadius);
    Vec3 offset = Add(ScalarMul(u, rd.X), ScalarMul(v, rd.Y));
    double time = time0 + camRnd.Float64() * (time1 - time0);
    return NewRayL(Add(origin, offset),
                   Sub(Add(lowerLeftCorner, ScalarMul(horizontal, s), ScalarMul(vertical, t)), origin, offset), time, lambda);
  }
};

// ------------------------------------------------------------- samplers
struct World {
  HitableSlice world;     // Slice{BVH4}
  HitableSlice lights;    // Scene.Lights
  BVH4 bvh;
  Camera camera;
  std::vector<std::unique_ptr<Hitable>> owned;
  std::vector<std::unique_ptr<Material>> mats;
  std::vector<std::unique_ptr<Texture>> texs;
  std::vector<std::unique_ptr<SpectralTexture>> stexs;
  std::vector<double> texels;
  std::vector<const Hitable*> byRef;  // transport order
  uint32_t numTris = 0, numSpheres = 0;
};

struct ColourSampler {  // sampler/colour.go
  int maxDepth; Vec3 background;
  Vec3 Sample(const Ray& r, const World& W, int depth, LCG& rnd) const {
    if (depth >= maxDepth) return V(0, 0, 1.0);
    g_cnt.rays++;
    HitRecord rec; const Material* mat;
    if (W.world.Hit(r, 0.001, GO_MAXFLOAT64, rec, mat)) {
      ScatterRecord srec;
      bool ok = mat->Scatter(r, rec, rnd, srec);
      Vec3 emitted = mat->Emitted(r, rec, rec.u, rec.v, rec.p);
      if (depth < maxDepth && ok) {
        if (srec.isSpecular) {
          return Mul(srec.albedo, Sample(srec.specularRay, W, depth + 1, rnd));
        }
        // Mixture(Hitable(lights, P), srec.PDF())
        Vec3 dir;
        if (rnd.Float64() < 0.5) dir = W.lights.Random(rec.p, rnd);
        else dir = srec.pdf.Generate(rnd);
        Ray scattered = NewRay(rec.p, dir, r.time);
        double pdfVal = 0.5 * W.lights.PDFValue(rec.p, scattered.d) + 0.5 * srec.pdf.Value(scattered.d);
        Vec3 v1 = ScalarMul(Sample(scattered, W, depth + 1, rnd), mat->ScatteringPDF(r, rec, scattered));
        Vec3 v2 = Mul(srec.albedo, v1);
        Vec3 v3 = ScalarDiv(v2, pdfVal);
        return Add(emitted, v3);
      }
      return emitted;
    }
    return background;
  }
  // The same estimator with the throughput carried forward (IZPI_ACC_FORWARD; a restatement
  // of the GPU's forward mode, not of izpi): identical rays, draws and counters; the radiance
  // is T * (terminal radiance) with T = (T * att) * (s / p) per non-specular bounce and T *= att
  // per specular one. Every scattering material emits 0 (non_emitter.go:12-14,
  // dielectric.go:219-221), so colour.go:57's `emitted +` adds nothing before the end.
  Vec3 SampleForward(Ray r, const World& W, LCG& rnd) const {
    Vec3 T = V(1.0, 1.0, 1.0);
    for (int depth = 0;; depth++) {
      if (depth >= maxDepth) return Mul(T, V(0, 0, 1.0));
      g_cnt.rays++;
      HitRecord rec; const Material* mat;
      if (!W.world.Hit(r, 0.001, GO_MAXFLOAT64, rec, mat)) return Mul(T, background);
      ScatterRecord srec;
      bool ok = mat->Scatter(r, rec, rnd, srec);
      Vec3 emitted = mat->Emitted(r, rec, rec.u, rec.v, rec.p);
      if (!ok) return Mul(T, emitted);
      if (srec.isSpecular) {
        T = Mul(T, srec.albedo);
        r = srec.specularRay;
        continue;
      }
      Vec3 dir;
      if (rnd.Float64() < 0.5) dir = W.lights.Random(rec.p, rnd);
      else dir = srec.pdf.Generate(rnd);
      Ray scattered = NewRay(rec.p, dir, r.time);
      double pdfVal = 0.5 * W.lights.PDFValue(rec.p, scattered.d) + 0.5 * srec.pdf.Value(scattered.d);
      const double w = mat->ScatteringPDF(r, rec, scattered) / pdfVal;
      T = ScalarMul(Mul(T, srec.albedo), w);
      r = scattered;
    }
  }
};

struct SpectralSampler {  // sampler/spectral.go
  int maxDepth; SPD background;
  double SampleSpectral(const Ray& r, const World& W, int depth, LCG& rnd) const {
    if (depth >= maxDepth) return background.Value(r.lambda);
    g_cnt.rays++;
    HitRecord rec; const Material* mat;
    if (W.world.Hit(r, 0.001, GO_MAXFLOAT64, rec, mat)) {
      SpectralScatterRecord srec;
      bool ok = mat->SpectralScatter(r, rec, rnd, srec);
      double emitted = mat->EmittedSpectral(r, rec, rec.u, rec.v, r.lambda, rec.p);
      if (depth < maxDepth && ok) {
        if (srec.isSpecular) return srec.albedo * SampleSpectral(srec.specularRay, W, depth + 1, rnd);
        Vec3 dir;
        if (rnd.Float64() < 0.5) dir = W.lights.Random(rec.p, rnd);
        else dir = srec.pdf.Generate(rnd);
        Ray scattered = NewRayL(rec.p, dir, r.time, r.lambda);
        double pdfVal = 0.5 * W.lights.PDFValue(rec.p, scattered.d) + 0.5 * srec.pdf.Value(scattered.d);
        double v1 = SampleSpectral(scattered, W, depth + 1, rnd) * mat->ScatteringPDF(r, rec, scattered);
        double v2 = srec.albedo * v1;
        double v3 = v2 / pdfVal;
        return emitted + v3;
      }
      return emitted;
    }
    return background.Value(r.lambda);
  }
  // Forward form of SampleSpectral (see ColourSampler::SampleForward).
  double SampleSpectralForward(Ray r, const World& W, LCG& rnd) const {
    double T = 1.0;
    for (int depth = 0;; depth++) {
      if (depth >= maxDepth) return T * background.Value(r.lambda);
      g_cnt.rays++;
      HitRecord rec; const Material* mat;
      if (!W.world.Hit(r, 0.001, GO_MAXFLOAT64, rec, mat)) return T * background.Value(r.lambda);
      SpectralScatterRecord srec;
      bool ok = mat->SpectralScatter(r, rec, rnd, srec);
      double emitted = mat->EmittedSpectral(r, rec, rec.u, rec.v, r.lambda, rec.p);
      if (!ok) return T * emitted;
      if (srec.isSpecular) {
        T = T * srec.albedo;
        r = srec.specularRay;
        continue;
      }
      Vec3 dir;
      if (rnd.Float64() < 0.5) dir = W.lights.Random(rec.p, rnd);
      else dir = srec.pdf.Generate(rnd);
      Ray scattered = NewRayL(rec.p, dir, r.time, r.lambda);
      double pdfVal = 0.5 * W.lights.PDFValue(rec.p, scattered.d) + 0.5 * srec.pdf.Value(scattered.d);
      const double w = mat->ScatteringPDF(r, rec, scattered) / pdfVal;
      T = (T * srec.albedo) * w;
      r = scattered;
    }
  }
};

}  // namespace orc

using namespace orc;

// ================================================================= C API
struct oracle_scene {
  World w;
  std::string err;
};


extern "C" {

oracle_scene* oracle_build(const izpi_scene_input* in) {
  oracle_scene* s = new oracle_scene();
  World& W = s->w;
  // textures
  std::vector<const Texture*> rgb(in->num_textures, nullptr);
  std::vector<const SpectralTexture*> spec(in->num_textures, nullptr);
  W.texels.assign(in->texels, in->texels + in->num_texels);
  for (uint32_t i = 0; i < in->num_textures; i++) {
    const izpi_texture& t = in->textures[i];
    if (t.kind == IZPI_TEX_CONSTANT) {
      ConstantTex* c = new ConstantTex(); c->color = Load(t.value); W.texs.emplace_back(c); rgb[i] = c;
    } else if (t.kind == IZPI_TEX_IMAGE) {
      ImageTex* c = new ImageTex(); c->sizeX = (int)t.width; c->sizeY = (int)t.height; c->pix = W.texels.data() + t.texel_offset;
      W.texs.emplace_back(c); rgb[i] = c;
    } else if (t.kind == IZPI_TEX_SPECTRAL_GAUSSIAN) {
      SpectralConstantTex* c = new SpectralConstantTex(); c->peak = t.peak; c->center = t.center; c->width = t.width_nm;
      W.stexs.emplace_back(c); spec[i] = c;
    } else if (t.kind == IZPI_TEX_SPECTRAL_TABULATED) {
      SpectralConstantTex* c = new SpectralConstantTex(); c->tabulated = true;
      c->spd.wl.assign(in->spd_wavelengths + t.spd_offset, in->spd_wavelengths + t.spd_offset + t.spd_count);
      c->spd.val.assign(in->spd_values + t.spd_offset, in->spd_values + t.spd_offset + t.spd_count);
      W.stexs.emplace_back(c); spec[i] = c;
    } else if (t.kind == IZPI_TEX_SPECTRAL_IMAGE) {
      SpectralImageTex* c = new SpectralImageTex();
      c->Build((int)t.width, (int)t.height, W.texels.data() + t.texel_offset);
      W.stexs.emplace_back(c); spec[i] = c;
    }
  }
  auto R = [&](int32_t id) -> const Texture* { return id < 0 ? nullptr : rgb[(size_t)id]; };
  auto S = [&](int32_t id) -> const SpectralTexture* { return id < 0 ? nullptr : spec[(size_t)id]; };
  std::vector<Dielectric*> dielectrics;
  std::vector<const Material*> mats(in->num_materials, nullptr);
  for (uint32_t i = 0; i < in->num_materials; i++) {
    const izpi_material& m = in->materials[i];
    Material* out = nullptr;
    switch (m.kind) {
      case IZPI_MAT_LAMBERT: { Lambertian* l = new Lambertian(); l->albedo = R(m.albedo_tex); l->spectralAlbedo = S(m.spectral_tex); out = l; break; }
      case IZPI_MAT_DIFFUSE_LIGHT: { DiffuseLight* l = new DiffuseLight(); l->emit = R(m.albedo_tex); l->spectralEmit = S(m.spectral_tex); out = l; break; }
      case IZPI_MAT_DIELECTRIC: {
        Dielectric* d = new Dielectric(); d->refIdx = m.ref_idx; d->spectralRefIdx = S(m.spectral_tex);
        d->computeBeerLambert = (m.flags & IZPI_MATF_BEER_LAMBERT) != 0; d->absorptionCoeff = Load(m.rgb);
        d->spectralAbsorptionCoeff = S(m.absorb_tex); dielectrics.push_back(d); out = d; break;
      }
      case IZPI_MAT_METAL: { Metal* mm = new Metal(); mm->albedo = Load(m.rgb); mm->fuzz = m.fuzz; out = mm; break; }
      case IZPI_MAT_ISOTROPIC: { Isotropic* is = new Isotropic(); is->albedo = R(m.albedo_tex); out = is; break; }
      case IZPI_MAT_PBR: {
        PBR* p = new PBR(); p->albedo = R(m.albedo_tex); p->spectralAlbedo = S(m.spectral_tex); p->normalMap = R(m.normal_tex);
        p->roughness = R(m.roughness_tex); p->metalness = R(m.metalness_tex); out = p; break;
      }
      default: s->err = "unknown material kind"; return s;
    }
    W.mats.emplace_back(out); mats[i] = out;
  }
  // objects: triangles then spheres (transport.go:551-567)
  std::vector<const Hitable*> hitables;
  for (uint32_t i = 0; i < in->num_tris; i++) {
    const izpi_tri_in& t = in->tris[i];
    Triangle* tr = Triangle::NewWithUV(Load(t.v0), Load(t.v1), Load(t.v2), t.uv[0], t.uv[1], t.uv[2], t.uv[3], t.uv[4], t.uv[5], mats[t.material]);
    tr->ref = IZPI_PRIM_REF(IZPI_PRIM_TRIANGLE, i);
    W.owned.emplace_back(tr); hitables.push_back(tr);
  }
  for (uint32_t i = 0; i < in->num_spheres; i++) {
    const izpi_sphere_in& sp = in->spheres[i];
    Sphere* so = new Sphere(); so->center0 = Load(sp.center); so->center1 = Load(sp.center); so->time0 = 0; so->time1 = 1;
    so->radius = sp.radius; so->material = mats[sp.material]; so->ref = IZPI_PRIM_REF(IZPI_PRIM_SPHERE, i);
    W.owned.emplace_back(so); hitables.push_back(so);
  }
  W.numTris = in->num_tris; W.numSpheres = in->num_spheres;
  W.byRef = hitables;
  for (const Hitable* h : hitables) if (h->IsEmitter()) W.lights.hitables.push_back(h);
  // NewBVH4 (bvh4.go:517-593) with the split-axis LCG seeded from bvh_seed
  if (!hitables.empty()) {
    LCG axisRnd = NewLCG(in->bvh_seed);
    std::vector<int> indices(hitables.size());
    for (size_t i = 0; i < indices.size(); i++) indices[i] = (int)i;
    BuildNode* root = buildBinaryBVH(hitables, indices, axisRnd);
    std::vector<int> primIdx;
    flattenBVH4(root, W.bvh, primIdx);
    freeTree(root);
    for (int idx : primIdx) W.bvh.Primitives.push_back(hitables[(size_t)idx]);
  }
  W.world.hitables.push_back(&W.bvh);
  for (Dielectric* d : dielectrics) d->world = &W.world;
  const izpi_camera_in& c = in->camera;
  double aspect = in->aspect_override != 0.0 ? in->aspect_override : c.aspect;
  W.camera = Camera::New(Load(c.look_from), Load(c.look_at), Load(c.vup), c.vfov, aspect, c.aperture, c.focus_dist, c.time0, c.time1, c.exposure);
  return s;
}

/* Attach an external BVH4 (e.g. the GPU builder's): nodes + leaf order of the
 * transport-order primitives (triangles, then spheres). */
/* IZPI_SCENE_QUANTIZED_BVH restated (a transform of the tree's boxes, not izpi code): every
 * inner node's valid slot boxes are replaced by their 8-bit quantisation against the node's
 * per-axis minimum and a power-of-two scale (the smallest 2^e >= 2^-126 for which every
 * bound, rounded outwards to the grid and decoded as org + float(q) * 2^e in f32, contains
 * the exact bound), and a leaf node's slot-0 box by its parent slot's decoded box. Returns
 * 0, with `out` = `in`, when a valid bound is not finite or no exponent fits. */
static float orc_qdec(float org, int q, float sc) { float p = (float)q * sc; return org + p; }
int oracle_quantize_bvh4(const izpi_bvh4_node* in, uint32_t n, izpi_bvh4_node* out) {
  std::vector<izpi_bvh4_node> w(in, in + n);
  for (uint32_t k = 0; k < n; k++) {
    izpi_bvh4_node& nd = w[k];
    if (nd.prim_count[0] > 0) continue;  // leaf node: its box comes from its parent
    float* lo[3] = {nd.min_x, nd.min_y, nd.min_z};
    float* hi[3] = {nd.max_x, nd.max_y, nd.max_z};
    for (int a = 0; a < 3; a++) {
      bool first = true;
      float org = 0.0f, top = 0.0f;
      for (int i = 0; i < 4; i++) {
        if (nd.child[i] == -1) continue;
        if (!std::isfinite(lo[a][i]) || !std::isfinite(hi[a][i])) { std::copy(in, in + n, out); return 0; }
        if (first || lo[a][i] < org) org = lo[a][i];
        if (first || hi[a][i] > top) top = hi[a][i];
        first = false;
      }
      const double span = (double)top - (double)org;
      int e = span > 0 ? (int)std::ceil(std::log2(span / 255.0)) : -126;
      if (e < -126) e = -126;
      int qa[4] = {0, 0, 0, 0}, qb[4] = {0, 0, 0, 0};
      for (;;) {
        if (e > 127) { std::copy(in, in + n, out); return 0; }
        const float sc = std::ldexp(1.0f, e);
        bool fits = true;
        for (int i = 0; i < 4; i++) {
          if (nd.child[i] == -1) continue;
          int a0 = (int)std::max(0.0, std::min(255.0, std::floor(((double)lo[a][i] - (double)org) / (double)sc)));
          while (a0 > 0 && orc_qdec(org, a0, sc) > lo[a][i]) a0--;
          int b0 = (int)std::max((double)a0, std::min(256.0, std::ceil(((double)hi[a][i] - (double)org) / (double)sc)));
          while (b0 <= 255 && orc_qdec(org, b0, sc) < hi[a][i]) b0++;
          if (b0 > 255) fits = false;
          qa[i] = a0; qb[i] = b0;
        }
        if (fits) break;
        e++;
      }
      const float sc = std::ldexp(1.0f, e);
      for (int i = 0; i < 4; i++) {
        if (nd.child[i] == -1) continue;
        lo[a][i] = orc_qdec(org, qa[i], sc);
        hi[a][i] = orc_qdec(org, qb[i], sc);
      }
    }
  }
  for (uint32_t k = 0; k < n; k++) {  // leaf nodes take their parent slot's decoded box (A10 re-test)
    const izpi_bvh4_node& nd = w[k];
    if (nd.prim_count[0] > 0) continue;
    for (int i = 0; i < 4; i++) {
      const int32_t c = nd.child[i];
      if (c < 0 || w[(size_t)c].prim_count[0] == 0) continue;
      izpi_bvh4_node& L = w[(size_t)c];
      L.min_x[0] = nd.min_x[i]; L.min_y[0] = nd.min_y[i]; L.min_z[0] = nd.min_z[i];
      L.max_x[0] = nd.max_x[i]; L.max_y[0] = nd.max_y[i]; L.max_z[0] = nd.max_z[i];
    }
  }
  std::copy(w.begin(), w.end(), out);
  return 1;
}

void oracle_set_bvh(oracle_scene* s, const izpi_bvh4_node* nodes, uint32_t num_nodes, const uint32_t* order) {
  World& W = s->w;
  W.bvh.Nodes.assign(nodes, nodes + num_nodes);
  W.bvh.Primitives.clear();
  for (size_t k = 0; k < W.byRef.size(); k++) W.bvh.Primitives.push_back(W.byRef[order[k]]);
}

/* Primitive boxes in transport order ([n][6]): Triangle.bb / Sphere.BoundingBox. */
void oracle_prim_boxes(oracle_scene* s, double* out) {
  const World& W = s->w;
  for (size_t i = 0; i < W.byRef.size(); i++) {
    const AABB b = W.byRef[i]->BoundingBox();
    out[6 * i] = b.min.X; out[6 * i + 1] = b.min.Y; out[6 * i + 2] = b.min.Z;
    out[6 * i + 3] = b.max.X; out[6 * i + 4] = b.max.Y; out[6 * i + 5] = b.max.Z;
  }
}

/* Sequential restatement of the GPU LBVH4 builder (see the file header). Returns the
 * node count; nodes needs 2n entries, order n. */
uint32_t oracle_lbvh4(const double* boxes, uint32_t n, uint32_t leaf_max, uint32_t method, izpi_bvh4_node* nodes,
                      uint32_t* order) {
  if (n == 0) return 0;
  const bool sah = (method & 0x100u) != 0;  // IZPI_BVH_SAH
  method &= ~0x100u;
  // Morton codes of the centroids, 21 bits per axis
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (uint32_t i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) {
      const double c = (boxes[6 * i + k] + boxes[6 * i + 3 + k]) * 0.5;
      lo[k] = fmin(lo[k], c); hi[k] = fmax(hi[k], c);
    }
  std::vector<std::pair<uint64_t, uint32_t>> key(n);
  for (uint32_t i = 0; i < n; i++) {
    uint64_t code = 0;
    for (int k = 0; k < 3; k++) {
      const double c = (boxes[6 * i + k] + boxes[6 * i + 3 + k]) * 0.5;
      const double ext = hi[k] - lo[k];
      double t = ext > 0 ? (c - lo[k]) / ext : 0.0;
      t = fmin(fmax(t * 2097152.0, 0.0), 2097151.0);
      const uint64_t q = (uint64_t)t;
      for (int b = 0; b < 21; b++) code |= ((q >> b) & 1ull) << (3 * b + (2 - k));
    }
    key[i] = {code, i};
  }
  std::sort(key.begin(), key.end());  // equal codes keep input order (stable radix sort)
  for (uint32_t i = 0; i < n; i++) order[i] = key[i].second;
  struct BN { int lo, hi, l, r; double box[6]; };
  std::vector<BN> bn;
  if (method == 1) {
    // PLOC: clusters in Morton order; nearest neighbour by merged half-area within +-8;
    // mutual pairs merge at the lower position; repeat.
    const int R = 8, N2 = 2 * (int)n - 1;
    std::vector<int> pl(N2, -1), pr(N2, -1), psz(N2, 1), off(N2, 0);
    std::vector<std::array<double, 6>> pb(N2);
    for (uint32_t i = 0; i < n; i++)
      for (int k = 0; k < 6; k++) pb[i][k] = boxes[6 * (size_t)key[i].second + k];
    auto uni = [&](int a, int b) {
      std::array<double, 6> r2;
      for (int k = 0; k < 3; k++) { r2[k] = fmin(pb[a][k], pb[b][k]); r2[k + 3] = fmax(pb[a][k + 3], pb[b][k + 3]); }
      return r2;
    };
    auto ha = [](const std::array<double, 6>& x) {
      const double dx = x[3] - x[0], dy = x[4] - x[1], dz = x[5] - x[2];
      return dx * dy + dy * dz + dz * dx;
    };
    std::vector<int> cl(n);
    for (uint32_t i = 0; i < n; i++) cl[i] = (int)i;
    int nxt = (int)n;
    while (cl.size() > 1) {
      const int m = (int)cl.size();
      std::vector<int> nn(m);
      for (int i = 0; i < m; i++) {
        double best = INFINITY;
        int bj = -1, bkey = 0;
        for (int j = std::max(0, i - R); j <= std::min(m - 1, i + R); j++) {
          if (j == i) continue;
          const double a = ha(uni(cl[i], cl[j]));
          // equal areas: nearer position first, then i+1 for even i and i-1 for odd i
          const int dist = j > i ? j - i : i - j;
          const bool pref = (j > i) == (i % 2 == 0);
          const int k2 = 2 * dist + (pref ? 0 : 1);
          if (a < best || (a == best && k2 < bkey)) { best = a; bj = j; bkey = k2; }
        }
        nn[i] = bj;
      }
      std::vector<int> nc;
      for (int i = 0; i < m; i++) {
        const int j = nn[i];
        const bool mutual = j >= 0 && nn[j] == i;
        if (mutual && i > j) continue;  // merged into its partner's position
        if (mutual) {
          const int c = nxt++;
          pl[c] = cl[i]; pr[c] = cl[j]; pb[c] = uni(cl[i], cl[j]); psz[c] = psz[cl[i]] + psz[cl[j]];
          nc.push_back(c);
        } else {
          nc.push_back(cl[i]);
        }
      }
      cl.swap(nc);
    }
    const int root = cl[0];
    std::vector<int> stk{root};
    while (!stk.empty()) {  // DFS positions: subtrees become contiguous ranges
      const int x = stk.back(); stk.pop_back();
      if (pl[x] < 0) continue;
      off[pl[x]] = off[x]; off[pr[x]] = off[x] + psz[pl[x]];
      stk.push_back(pr[x]); stk.push_back(pl[x]);
    }
    auto map = [&](int x) { return x < (int)n ? (int)n - 1 + off[x] : N2 - 1 - x; };
    bn.assign(N2, BN{0, 0, -1, -1, {0}});
    std::vector<uint32_t> ord(n);
    for (int x = 0; x < N2 && (x < (int)n || x < nxt); x++) {
      BN& b = bn[map(x)];
      b.lo = off[x]; b.hi = off[x] + psz[x] - 1;
      b.l = pl[x] < 0 ? -1 : map(pl[x]); b.r = pr[x] < 0 ? -1 : map(pr[x]);
      for (int k = 0; k < 6; k++) b.box[k] = pb[x][k];
      if (x < (int)n) ord[off[x]] = key[x].second;
    }
    for (uint32_t i = 0; i < n; i++) order[i] = ord[i];
  } else {
  // binary radix tree over the augmented keys (code, position), built top-down
  auto clz64 = [](uint64_t x) { return x ? __builtin_clzll(x) : 64; };
  std::vector<int> stack;
  bn.push_back(BN{0, (int)n - 1, -1, -1, {0}});
  stack.push_back(0);
  while (!stack.empty()) {
    const int id = stack.back(); stack.pop_back();
    const int a = bn[id].lo, b = bn[id].hi;
    if (a == b) continue;
    int split;  // last position of the left half
    if (key[a].first != key[b].first) {
      const int bit = 63 - clz64(key[a].first ^ key[b].first);
      int p = a;  // last position whose code has `bit` clear
      while (p + 1 <= b && !((key[p + 1].first >> bit) & 1)) p++;
      split = p;
    } else {
      const int bit = 31 - __builtin_clz((unsigned)(a ^ b));
      split = ((b >> bit) << bit) - 1;
    }
    const int l = (int)bn.size(); bn.push_back(BN{a, split, -1, -1, {0}});
    const int r = (int)bn.size(); bn.push_back(BN{split + 1, b, -1, -1, {0}});
    bn[id].l = l; bn[id].r = r;
    stack.push_back(l); stack.push_back(r);
  }
  for (size_t id = bn.size(); id-- > 0;) {  // children were created after their parent
    BN& x = bn[id];
    if (x.l < 0) {
      for (int k = 0; k < 6; k++) x.box[k] = boxes[6 * (size_t)order[x.lo] + k];
    } else {
      for (int k = 0; k < 3; k++) {
        x.box[k] = fmin(bn[x.l].box[k], bn[x.r].box[k]);
        x.box[k + 3] = fmax(bn[x.l].box[k + 3], bn[x.r].box[k + 3]);
      }
    }
  }
  }  // method
  auto size = [&](int id) { return bn[id].hi - bn[id].lo + 1; };
  // IZPI_BVH_SAH (PLOC trees): the collapse of least surface-area cost. For each binary
  // node and i = 1..4, D[i] = the least cost of covering its subtree with at most i child
  // slots; a slot is a leaf (<= leaf_max primitives: Cl + Ct per primitive) or a 4-wide
  // node (Cn plus the best split of its two children over 4 slots), all weighted by the
  // box's half area. Children have larger indices than their parents in PLOC's numbering,
  // so one backward sweep sees them first. Same costs, operation order and tie rules as the
  // device builder's k_sah_leaves / k_sah_level (bvh_build.hip).
  const double Cn = 1.0, Cl = 0.5, Ct = 1.0;
  std::vector<std::array<double, 5>> D;
  std::vector<uint32_t> dec;
  if (sah && method == 1) {
    D.assign(bn.size(), {0, 0, 0, 0, 0});
    dec.assign(bn.size(), 0);
    for (size_t id = bn.size(); id-- > 0;) {
      const BN& x = bn[id];
      const double* b = x.box;
      const double dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
      const double area = dx * dy + dy * dz + dz * dx;
      if (x.l < 0) {
        const double c = area * (Cl + Ct);
        D[id] = {0, c, c, c, c};
        dec[id] = 1;
        continue;
      }
      const auto& L = D[x.l];
      const auto& R = D[x.r];
      double best4 = L[1] + R[3];
      uint32_t k4 = 1;
      for (uint32_t j = 2; j <= 3; j++)
        if (L[j] + R[4 - j] < best4) { best4 = L[j] + R[4 - j]; k4 = j; }
      std::array<double, 5> d{};
      d[1] = area * Cn + best4;
      uint32_t bits = k4 << 1;
      const int sz = x.hi - x.lo + 1;
      if (sz <= (int)leaf_max) {
        const double lc = area * (Cl + Ct * (double)sz);
        if (lc <= d[1]) { d[1] = lc; bits |= 1u; }
      }
      for (uint32_t i = 2; i <= 4; i++) {
        d[i] = d[i - 1];
        uint32_t ki = 0;
        for (uint32_t j = 1; j < i; j++)
          if (L[j] + R[i - j] < d[i]) { d[i] = L[j] + R[i - j]; ki = j; }
        bits |= ki << (1 + 2 * (i - 1));
      }
      D[id] = d;
      dec[id] = bits;
    }
  }
  auto is_leaf = [&](int id) { return dec.empty() ? size(id) <= (int)leaf_max : (dec[id] & 1u) != 0; };
  // the wide node's slots from the recorded splits, left to right
  auto sah_slots = [&](int b, int* res) {
    int c = 0;
    std::vector<std::pair<int, int>> work{{bn[b].r, 4 - (int)((dec[b] >> 1) & 3u)}, {bn[b].l, (int)((dec[b] >> 1) & 3u)}};
    while (!work.empty()) {
      auto [m, i] = work.back();
      work.pop_back();
      while (i > 1 && bn[m].l >= 0 && ((dec[m] >> (1 + 2 * (i - 1))) & 3u) == 0) i--;
      if (i <= 1 || bn[m].l < 0) { res[c++] = m; continue; }
      const int ki = (int)((dec[m] >> (1 + 2 * (i - 1))) & 3u);
      work.push_back({bn[m].r, i - ki});
      work.push_back({bn[m].l, ki});
    }
    return c;
  };
  auto empty = [](izpi_bvh4_node& nd) {
    for (int s2 = 0; s2 < 4; s2++) {
      nd.child[s2] = -1; nd.prim_count[s2] = 0;
      nd.min_x[s2] = nd.min_y[s2] = nd.min_z[s2] = nd.max_x[s2] = nd.max_y[s2] = nd.max_z[s2] = 3.40282346638528859811704183484516925440e+38f;
    }
  };
  auto slot = [&](izpi_bvh4_node& nd, int s2, int id) {
    const double* b = bn[id].box;
    nd.min_x[s2] = conservativeFloat32Min(b[0]); nd.min_y[s2] = conservativeFloat32Min(b[1]); nd.min_z[s2] = conservativeFloat32Min(b[2]);
    nd.max_x[s2] = conservativeFloat32Max(b[3]); nd.max_y[s2] = conservativeFloat32Max(b[4]); nd.max_z[s2] = conservativeFloat32Max(b[5]);
  };
  if (size(0) <= (int)leaf_max) {  // the whole scene is one leaf (the device builder's n <= leaf_max)
    empty(nodes[0]);
    nodes[0].child[0] = 0; nodes[0].prim_count[0] = (int32_t)n;
    slot(nodes[0], 0, 0);
    return 1;
  }
  // breadth-first collapse: node indices in allocation order
  std::vector<std::pair<int, uint32_t>> frontier{{0, 0u}}, next;
  uint32_t total = 1;
  while (!frontier.empty()) {
    next.clear();
    for (auto& fe : frontier) {
      int res[4], c = 0;
      if (!dec.empty()) c = sah_slots(fe.first, res);
      else { res[c++] = bn[fe.first].l; res[c++] = bn[fe.first].r; }
      bool expanded = dec.empty();
      while (expanded && c < 4) {  // collectChildren (bvh4.go:796-855), largest surface area first
        expanded = false;
        int pick = -1;
        double best = -1.0;
        for (int i = 0; i < c; i++) {
          if (is_leaf(res[i])) continue;
          const double* b = bn[res[i]].box;
          const double dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
          const double area = dx * dy + dy * dz + dz * dx;
          if (area > best) { best = area; pick = i; }
        }
        if (pick >= 0) {
          const int cur = res[pick];
          for (int k = pick; k + 1 < c; k++) res[k] = res[k + 1];
          c--;
          res[c++] = bn[cur].l; res[c++] = bn[cur].r;
          expanded = true;
        }
      }
      izpi_bvh4_node nd; empty(nd);
      for (int s2 = 0; s2 < c; s2++) {
        const uint32_t idx = total++;
        nd.child[s2] = (int32_t)idx;
        slot(nd, s2, res[s2]);
        if (is_leaf(res[s2])) {
          izpi_bvh4_node lf; empty(lf);
          lf.child[0] = bn[res[s2]].lo; lf.prim_count[0] = size(res[s2]);
          slot(lf, 0, res[s2]);
          nodes[idx] = lf;
        } else {
          next.push_back({res[s2], idx});
        }
      }
      nodes[fe.second] = nd;
    }
    frontier.swap(next);
  }
  return total;
}

const char* oracle_error(oracle_scene* s) { return s->err.empty() ? nullptr : s->err.c_str(); }
void oracle_free(oracle_scene* s) { delete s; }

uint32_t oracle_num_nodes(oracle_scene* s) { return (uint32_t)s->w.bvh.Nodes.size(); }
void oracle_copy_nodes(oracle_scene* s, izpi_bvh4_node* out) {
  memcpy(out, s->w.bvh.Nodes.data(), s->w.bvh.Nodes.size() * sizeof(izpi_bvh4_node));
}
void oracle_copy_prim_refs(oracle_scene* s, uint32_t* out) {
  for (size_t i = 0; i < s->w.bvh.Primitives.size(); i++) out[i] = s->w.bvh.Primitives[i]->ref;
}
uint32_t oracle_num_lights(oracle_scene* s) { return (uint32_t)s->w.lights.hitables.size(); }
void oracle_copy_light_refs(oracle_scene* s, uint32_t* out) {
  for (size_t i = 0; i < s->w.lights.hitables.size(); i++) out[i] = s->w.lights.hitables[i]->ref;
}
/* Triangle fields for fixture comparison: per triangle 25 doubles:
 * e1[3] e2[3] normal[3] tangent[3] bitangent[3] area bbmin[3] bbmax[3] */
void oracle_copy_triangle(oracle_scene* s, uint32_t i, double* out) {
  const Triangle* t = static_cast<const Triangle*>(s->w.byRef[i]);
  const Vec3 v[] = {t->edge1, t->edge2, t->normal, t->tangent, t->bitangent};
  for (int k = 0; k < 5; k++) { out[3 * k] = v[k].X; out[3 * k + 1] = v[k].Y; out[3 * k + 2] = v[k].Z; }
  out[15] = t->area;
  out[16] = t->bb.min.X; out[17] = t->bb.min.Y; out[18] = t->bb.min.Z;
  out[19] = t->bb.max.X; out[20] = t->bb.max.Y; out[21] = t->bb.max.Z;
}
void oracle_copy_camera(oracle_scene* s, izpi_camera* out) {
  const Camera& c = s->w.camera;
  const Vec3 v[] = {c.origin, c.lowerLeftCorner, c.horizontal, c.vertical, c.u, c.v};
  double* dst[] = {out->origin, out->lower_left, out->horizontal, out->vertical, out->u, out->v};
  for (int k = 0; k < 6; k++) { dst[k][0] = v[k].X; dst[k][1] = v[k].Y; dst[k][2] = v[k].Z; }
  out->lens_radius = c.lensRadius; out->time0 = c.time0; out->time1 = c.time1; out->exposure = c.exposure;
}

uint8_t oracle_ray_aabb4(const float* box24, const float* ray7) {
  return RayAABB4(ray7[0], ray7[1], ray7[2], ray7[3], ray7[4], ray7[5], box24, box24 + 4, box24 + 8, box24 + 12,
                  box24 + 16, box24 + 20, ray7[6]);
}
float oracle_conservative_f32(double v, int is_max) { return is_max ? conservativeFloat32Max(v) : conservativeFloat32Min(v); }

/* Standalone Triangle.Hit for the triangle_test.go KATs: tri = v0[3] v1[3] v2[3];
 * ray = o[3] d[3] tmin tmax; out = t u v p[3] n[3]; returns hit. */
int oracle_triangle_hit(const double* tri, const double* ray, double* out) {
  Lambertian dummy;
  Triangle* t = Triangle::NewWithUV(Load(tri), Load(tri + 3), Load(tri + 6), 0, 0, 0, 0, 0, 0, &dummy);
  HitRecord rec; const Material* m;
  bool hit = t->Hit(NewRay(Load(ray), Load(ray + 3), 0), ray[6], ray[7], rec, m);
  if (hit) {
    out[0] = rec.t; out[1] = rec.u; out[2] = rec.v;
    out[3] = rec.p.X; out[4] = rec.p.Y; out[5] = rec.p.Z; out[6] = rec.normal.X; out[7] = rec.normal.Y; out[8] = rec.normal.Z;
  }
  delete t;
  return hit ? 1 : 0;
}

/* mat3_test.go:10-54: MatrixVectorMul(NewTBN(t, b, n), v); in = t[3] b[3] n[3] v[3]. */
void oracle_tbn_mul(const double* in, double* out3) {
  const Vec3 r = MatrixVectorMul(NewTBN(Load(in), Load(in + 3), Load(in + 6)), Load(in + 9));
  out3[0] = r.X; out3[1] = r.Y; out3[2] = r.Z;
}

/* dielectric_test.go:47-84: Dielectric.calculatePathLength against a world whose Hit
 * always returns the exit point `exit3` (mockSceneGeometry); in = hit point p[3], normal
 * n[3], ray o[3] d[3], scattered direction s[3]. */
double oracle_path_length(const double* in, const double* exit3) {
  struct Mock : SceneGeometry {
    Vec3 exit;
    bool Hit(const Ray&, double, double, HitRecord& rec, const Material*& mat) const override {
      rec = NewHR(2.0, 0.0, 0.0, exit, V(0, 0, 1));
      mat = nullptr;
      return true;
    }
  } world;
  world.exit = Load(exit3);
  Dielectric d;
  d.refIdx = 1.5;
  d.world = &world;
  const HitRecord hr = NewHR(1.0, 0.0, 0.0, Load(in), Load(in + 3));
  const Ray r = NewRay(Load(in + 6), Load(in + 9), 0.0), scattered = NewRay(Load(in + 6), Load(in + 12), 0.0);
  return d.calculatePathLength(r, hr, scattered);
}

double oracle_gomath(int op, double x, double y) {
  switch (op) {
    case 0: return go_sin(x);
    case 1: return go_cos(x);
    case 2: return go_tan(x);
    case 3: return go_exp(x);
    case 4: return go_log(x);
    case 5: return go_pow(x, y);
    case 6: return go_atan2(x, y);
    case 7: return go_asin(x);
    case 8: return go_sqrt(x);
    case 9: return x / y;
    case 10: return go_atan(x);
  }
  return go_nan();
}

/* LCG KAT: n draws from seed. */
void oracle_lcg(uint64_t seed, uint32_t n, double* out, uint64_t* states) {
  LCG l = NewLCG(seed);
  for (uint32_t i = 0; i < n; i++) { out[i] = l.Float64(); if (states) states[i] = l.state; }
}

void oracle_trace(oracle_scene* s, const double* rays, uint32_t n, izpi_hit* out) {
  for (uint32_t i = 0; i < n; i++) {
    const double* r = rays + (size_t)i * 8;
    HitRecord rec; const Material* m;
    izpi_hit& h = out[i];
    memset(&h, 0, sizeof(h));
    h.prim_ref = 0xFFFFFFFFu;
    // BVH4.Hit through the world slice; report which primitive won via a side channel
    Ray ray = NewRay(Load(r), Load(r + 3), 0);
    g_last_prim = 0xFFFFFFFFu;
    if (s->w.world.Hit(ray, r[6], r[7], rec, m)) {
      h.hit = 1; h.prim_ref = g_last_prim; h.t = rec.t; h.u = rec.u; h.v = rec.v;
      h.p[0] = rec.p.X; h.p[1] = rec.p.Y; h.p[2] = rec.p.Z;
      h.normal[0] = rec.normal.X; h.normal[1] = rec.normal.Y; h.normal[2] = rec.normal.Z;
    }
  }
}

typedef struct oracle_stats {
  uint64_t rays, node_visits, tri_tests, sph_tests, light_tri_tests, light_sph_tests, samples;
  double seconds;
  uint32_t threads, pad;
} oracle_stats;

uint32_t oracle_tiles(uint32_t W, uint32_t H, uint32_t* tiles, uint32_t max_tiles);

/* Render the requested tiles into `canvas` (W*H*4 doubles, NOT cleared here). For the
 * spectral sampler the canvas receives CIE XYZ (post-processing is separate). */
int oracle_render(oracle_scene* s, const izpi_render_req* req, double* canvas, oracle_stats* st, int nthreads) {
  const World& W = s->w;
  std::vector<uint32_t> tiles;
  if (req->num_tiles) tiles.assign(req->tiles, req->tiles + 4 * (size_t)req->num_tiles);
  else {
    tiles.resize(4 * (size_t)(req->width * req->height));
    uint32_t n = oracle_tiles(req->width, req->height, tiles.data(), req->width * req->height);
    tiles.resize(4 * (size_t)n);
  }
  size_t ntiles = tiles.size() / 4;
  const int nx = (int)req->width, ny = (int)req->height;
  ColourSampler cs{(int)req->max_depth, V(req->background[0], req->background[1], req->background[2])};
  SpectralSampler ss;
  ss.maxDepth = (int)req->max_depth;
  if (req->num_bg_spd) {
    ss.background.wl.assign(req->bg_spd_wavelengths, req->bg_spd_wavelengths + req->num_bg_spd);
    ss.background.val.assign(req->bg_spd_values, req->bg_spd_values + req->num_bg_spd);
  } else {
    ss.background.wl.assign(oracle_cie_wavelengths, oracle_cie_wavelengths + ORACLE_CIE_N);
    ss.background.val.assign(ORACLE_CIE_N, 0.0);  // colours.SpectralBlack
  }
  const bool spectral = req->sampler == IZPI_SAMPLER_SPECTRAL;
  const bool forward = req->abi_version >= 3 && req->accumulation == IZPI_ACC_FORWARD;
  std::atomic<size_t> next(0);
  std::vector<Counters> per((size_t)(nthreads > 0 ? nthreads : 1));
  auto worker = [&](int tid) {
    g_cnt = Counters();
    for (;;) {
      size_t ti = next.fetch_add(1);
      if (ti >= ntiles) break;
      const uint32_t* t = &tiles[ti * 4];
      for (int y = (int)t[1]; y <= (int)t[3]; y++) {
        for (int x = (int)t[0]; x <= (int)t[2]; x++) {
          uint32_t pix = (uint32_t)(y * nx + x);
          double out[3];
          if (!spectral) {  // render/rgb.go:31-41
            Vec3 col;
            for (uint32_t smp = 0; smp < req->spp; smp++) {
              uint64_t key = sample_key(pix, smp);
              LCG rnd = NewLCG(splitmix64(req->seed ^ key));
              LCG cam = NewLCG(splitmix64(req->seed ^ key ^ CAMERA_STREAM_SALT));
              g_cnt.samples++;
              double u = ((double)x + rnd.Float64()) / (double)nx;
              double v = ((double)y + rnd.Float64()) / (double)ny;
              Ray r = W.camera.GetRay(u, v, cam, 0);
              col = Add(col, DeNAN(forward ? cs.SampleForward(r, W, rnd) : cs.Sample(r, W, 0, rnd)));
            }
            col = ScalarDiv(col, (double)req->spp);
            out[0] = col.X; out[1] = col.Y; out[2] = col.Z;
          } else {  // render/spectral.go:71-106
            double sumX = 0, sumY = 0, sumZ = 0;
            for (uint32_t smp = 0; smp < req->spp; smp++) {
              uint64_t key = sample_key(pix, smp);
              LCG rnd = NewLCG(splitmix64(req->seed ^ key));
              LCG cam = NewLCG(splitmix64(req->seed ^ key ^ CAMERA_STREAM_SALT));
              g_cnt.samples++;
              double lambda, pdf;
              SampleWavelength(rnd.Float64(), &lambda, &pdf);
              if (pdf == 0) continue;
              double u = ((double)x + rnd.Float64()) / (double)nx;
              double v = ((double)y + rnd.Float64()) / (double)ny;
              Ray r = W.camera.GetRay(u, v, cam, lambda);
              double radiance = forward ? ss.SampleSpectralForward(r, W, rnd) : ss.SampleSpectral(r, W, 0, rnd);
              double cx, cy, cz;
              GetCIEValues(lambda, &cx, &cy, &cz);
              sumX += (radiance * cx) / pdf;
              sumY += (radiance * cy) / pdf;
              sumZ += (radiance * cz) / pdf;
            }
            double inv = 1.0 / (double)req->spp;
            out[0] = sumX * inv; out[1] = sumY * inv; out[2] = sumZ * inv;
          }
          int row = ny - y;  // canvas.Set(x, ny-y, ...) — row ny is out of bounds (A9)
          if (row >= 0 && row < ny) {
            double* px = canvas + ((size_t)row * (size_t)nx + (size_t)x) * 4;
            px[0] = out[0]; px[1] = out[1]; px[2] = out[2]; px[3] = 1.0;
          }
        }
      }
    }
    per[(size_t)tid] = g_cnt;
  };
  auto t0 = std::chrono::steady_clock::now();
  int nt = nthreads > 0 ? nthreads : 1;
  std::vector<std::thread> th;
  for (int i = 0; i < nt; i++) th.emplace_back(worker, i);
  for (auto& t : th) t.join();
  auto t1 = std::chrono::steady_clock::now();
  if (st) {
    memset(st, 0, sizeof(*st));
    for (auto& c : per) {
      st->rays += c.rays; st->node_visits += c.node_visits; st->tri_tests += c.tri_tests; st->sph_tests += c.sph_tests;
      st->light_tri_tests += c.light_tri; st->light_sph_tests += c.light_sph; st->samples += c.samples;
    }
    st->seconds = std::chrono::duration<double>(t1 - t0).count();
    st->threads = (uint32_t)nt;
  }
  return 0;
}

/* spectral.FireflyRejection (firefly_rejection.go:12-113), in place on W*H*4. */
void oracle_firefly(double* pix, int width, int height) {
  if (width == 0 || height == 0) return;
  std::vector<double> yv((size_t)width * height);
  for (int y = 0; y < height; y++)
    for (int x = 0; x < width; x++) yv[(size_t)y * width + x] = pix[((size_t)y * width + x) * 4 + 1];
  for (int y = 0; y < height; y++) {
    for (int x = 0; x < width; x++) {
      size_t pi = ((size_t)y * width + x) * 4;
      double cur = yv[(size_t)y * width + x];
      if (cur <= 0) continue;
      double nb[8]; int nn = 0;
      for (int dy = -1; dy <= 1; dy++)
        for (int dx = -1; dx <= 1; dx++) {
          if (dx == 0 && dy == 0) continue;
          int nx = x + dx, ny = y + dy;
          if (nx >= 0 && nx < width && ny >= 0 && ny < height) {
            double v = yv[(size_t)ny * width + nx];
            if (v > 0) nb[nn++] = v;
          }
        }
      if (nn < 3) continue;
      double sum = 0.0;
      for (int i = 0; i < nn; i++) sum += nb[i];
      double mean = sum / (double)nn;
      double vs = 0.0;
      for (int i = 0; i < nn; i++) { double d = nb[i] - mean; vs += d * d; }
      double stddev = go_sqrt(vs / (double)nn);
      double threshold = mean + 2.5 * stddev;
      if (cur > threshold && threshold > 0) {
        double ratio = threshold / cur;
        pix[pi] *= ratio; pix[pi + 1] *= ratio; pix[pi + 2] *= ratio;
      }
    }
  }
}

/* spectral.XYZToRGB (rgb_image.go:28-67) with the ACEScg matrix (rgb_image.go:13-17). */
void oracle_xyz_to_rgb(const double* in, double* out, int width, int height, double exposure) {
  static const double M[3][3] = {{1.6410234, -0.3248033, -0.2364247}, {-0.6636629, 1.6153316, 0.0167563}, {0.0117219, -0.0082845, 0.9883949}};
  for (size_t i = 0; i < (size_t)width * height; i++) {
    double x = in[i * 4] * exposure, y = in[i * 4 + 1] * exposure, z = in[i * 4 + 2] * exposure;
    out[i * 4] = M[0][0] * x + M[0][1] * y + M[0][2] * z;
    out[i * 4 + 1] = M[1][0] * x + M[1][1] * y + M[1][2] * z;
    out[i * 4 + 2] = M[2][0] * x + M[2][1] * y + M[2][2] * z;
    out[i * 4 + 3] = in[i * 4 + 3];
  }
}

/* postprocess.Pipeline (pipeline.go:20-31) over the whole canvas, written the way the
 * reference loops (gamma.go:30-38, clamp.go:33-41): every filter walks every pixel, then
 * the next filter runs. kind 1 = Gamma (math.Sqrt of R, G, B), 2 = Clamp(max). */
void oracle_postprocess(double* pix, int width, int height, const uint32_t* kinds, const double* params, int n) {
  for (int f = 0; f < n; f++)
    for (int y = 0; y < height; y++)
      for (int x = 0; x < width; x++) {
        double* p = pix + ((size_t)y * width + x) * 4;
        for (int c = 0; c < 3; c++) {
          if (kinds[f] == 1) p[c] = std::sqrt(p[c]);
          else if (p[c] >= params[f] || p[c] != p[c]) p[c] = params[f];  /* clamp(): `if v < max {return v}; return max` */
        }
      }
}

/* common.Tiles (tiles.go:6-24) + grid.WalkGrid spiral (grid.go:48-125). */
uint32_t oracle_tiles(uint32_t W, uint32_t H, uint32_t* tiles, uint32_t max_tiles) {
  static const int steps[] = {32, 25, 24, 20, 16, 12, 10, 8, 5, 4};
  int sx = 0, sy = 0;
  for (int s : steps) if ((int)W % s == 0) { sx = s; break; }
  for (int s : steps) if ((int)H % s == 0) { sy = s; break; }
  if (sx == 0 || sy == 0) return 0;
  int gx = (int)W / sx, gy = (int)H / sy;
  int total = gx * gy;
  std::vector<uint8_t> seen;
  // visited set over an expanded window (the spiral may step outside the grid)
  int pad = gx + gy + 4;
  int ww = gx + 2 * pad, wh = gy + 2 * pad;
  seen.assign((size_t)ww * wh, 0);
  auto mark = [&](int x, int y) { seen[(size_t)(y + pad) * ww + (x + pad)] = 1; };
  auto has = [&](int x, int y) { return seen[(size_t)(y + pad) * ww + (x + pad)] != 0; };
  std::vector<std::pair<int, int>> path;
  int cx = gx / 2, cy = gy / 2;
  path.push_back({cx, cy}); mark(cx, cy);
  int walked = 1, dirIdx = 0;
  const int dirs[4] = {0 /*UP*/, 1 /*RIGHT*/, 2 /*DOWN*/, 3 /*LEFT*/};
  while (walked != total) {
    int d = dirs[((dirIdx % 4) + 4) % 4];
    int nx = cx, ny = cy;
    if (d == 0) ny--; else if (d == 2) ny++; else if (d == 3) nx--; else nx++;
    if (has(nx, ny)) { dirIdx--; continue; }
    cx = nx; cy = ny; mark(cx, cy);
    if (cx >= 0 && cx < gx && cy >= 0 && cy < gy) { walked++; path.push_back({cx, cy}); }
    dirIdx++;
  }
  uint32_t n = 0;
  for (auto& p : path) {
    if (n >= max_tiles) break;
    tiles[4 * n] = (uint32_t)(p.first * sx); tiles[4 * n + 1] = (uint32_t)(p.second * sy);
    tiles[4 * n + 2] = (uint32_t)(p.first * sx + sx - 1); tiles[4 * n + 3] = (uint32_t)(p.second * sy + sy - 1);
    n++;
  }
  return n;
}

void oracle_sample_wavelength(double r, double* lambda, double* pdf) { SampleWavelength(r, lambda, pdf); }
void oracle_cie_values(double w, double* out3) { GetCIEValues(w, out3, out3 + 1, out3 + 2); }
// SpectralConstant.Value of a tabulated SPD (spectral_constant.go:88-106): the linear scan
double oracle_spd_tabulated_value(const double* wl, const double* val, uint32_t n, double lambda) {
  SpectralConstantTex t;
  t.tabulated = true;
  t.spd.wl.assign(wl, wl + n);
  t.spd.val.assign(val, val + n);
  return t.Value(0, 0, lambda, Vec3());
}
double oracle_spectral_value(int gaussian, double a, double b, double c, double lambda) {
  SpectralConstantTex t; t.peak = a; t.center = b; t.width = c; (void)gaussian;
  return t.Value(0, 0, lambda, Vec3());
}

}  // extern "C"
