// izpi_dev.h — device-side data layouts and per-lane primitives of the gfx950
// path-tracing inner loop. Included only by izpi_gpu.hip.
//
// HBM layout (DESIGN.md §Data layout):
//   GInner  128 B  inner BVH4 nodes: SoA f32 bounds of 4 children + encoded child refs.
//                  (== hitable.BVH4Node, bvh4.go:23-39, with PrimitiveCount — always 0 in
//                  inner nodes — replaced by nothing; leaf children become leaf refs).
//   GLeaf   32 B   one per reference leaf node, indexed by its first primitive: its slot-0
//                  bounds + primitive range.
//                  A reference leaf node carries only slot 0 (bvh4.go:736-760), so the
//                  re-test on visit (quirk A10) needs 32 B instead of a 128 B node load.
//   GPrim   80 B   primitives in BVH leaf order: triangle v0,e1,e2 (the 72 B Hit reads,
//                  triangle.go:198-218) or sphere c0,c1,r,t0,t1; + kind/index.
//   shading data (normals, UVs, materials) stays in transport order and is read once per
//   closest hit, after traversal (deferred hit record).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/izpi_gpu.h"
#include "gomath.h"

#define IZPI_DEV __device__ __forceinline__

namespace izd {

// child ref encoding inside GInner / the traversal stack
//   r >= 0 : inner node index;   r == -1 : empty slot;   r <= -2 : leaf (below)
//   leaf refs carry the leaf's primitive range: r = -(1 + (start << 3 | count)), count 1..4
//   (bvh4.go:638-642 makes leaves of <= 4 primitives)
__host__ __device__ inline bool ref_is_leaf(int32_t r) { return r <= -2; }
__host__ __device__ inline int32_t leaf_start(int32_t r) { return (-r - 1) >> 3; }
__host__ __device__ inline int32_t leaf_count(int32_t r) { return (-r - 1) & 7; }
__host__ __device__ inline int32_t make_leaf_ref(int32_t start, int32_t count) { return -(1 + ((start << 3) | count)); }

struct alignas(16) GInner {
  float mnx[4], mny[4], mnz[4], mxx[4], mxy[4], mxz[4];
  int32_t child[4];
  int32_t pad[4];
};
// An inner node with its child boxes quantised (IZPI_SCENE_QUANTIZED_BVH), 64 B: two per
// 128-B line, four 16-B loads per visit instead of seven. Bound b of child i on axis a is
// org[a] + q * 2^(e[a] - 127), q = byte i of the bound's word: the product is exact (q < 256,
// a normal power of two), so a fused multiply-add decodes it bit for bit as the upload's
// `org + (float)q * s` does (qdecode). Child refs as in GInner.
struct alignas(64) GInnerQ {
  float org[3];
  uint32_t ex;        // biased exponents: x bits 0-7, y 8-15, z 16-23
  uint32_t q[6];      // mnx, mny, mnz, mxx, mxy, mxz: byte i = child i
  int32_t child[4];
  uint32_t pad[2];
};
static_assert(sizeof(GInnerQ) == 64, "GInnerQ is 64 B");
// The upload's decoding of one quantised bound (host), which the kernels' fmaf reproduces.
__host__ __device__ inline float qdecode(float org, uint32_t q, float s) {
  const float p = (float)q * s;  // exact
  return org + p;
}
struct alignas(16) GLeaf {
  float mn[3], mx[3];
  int32_t start, count;
};
struct alignas(16) GPrim {
  double a[9];      // tri: v0[3] e1[3] e2[3];  sphere: c0[3] c1[3] radius t0 t1
  uint32_t kind;    // IZPI_PRIM_*
  uint32_t index;   // transport-order index (shading data, lights)
};
// Shading record of a primitive, in BVH leaf order next to GPrim: everything the
// deferred hit record needs, in 32 B (half a 64-B line: one sector per closest hit). The
// material's constant RGB albedo / emit value, when it has one, is in DevScene::mat_const.
struct alignas(32) GShade {
  double n[3];      // triangle: unit(e1 x e2) (triangle.go:100); sphere: unused
  uint32_t ref;     // IZPI_PRIM_REF(kind, transport index)
  uint32_t mk;      // material index << 8 | material kind << 2 | cflags
                    // (cflags bit0: mat_const holds the albedo; bit1: a texture of the material reads the hit (u,v))
};
__host__ __device__ inline uint32_t gs_mat(const GShade& g) { return g.mk >> 8; }
__host__ __device__ inline uint32_t gs_kind(const GShade& g) { return (g.mk >> 2) & 63u; }
__host__ __device__ inline uint32_t gs_cflags(const GShade& g) { return g.mk & 3u; }
// Texture-space data of a triangle, in BVH leaf order next to GShade (a hit's primitive
// indexes it directly, so it loads in parallel with GShade instead of after it): the
// vertex UVs (triangle.go:61-134) and the tangent / bitangent of the normal map's TBN
// (triangle.go:250-264). Uploaded only for scenes with image textures or normal maps.
struct alignas(16) GTriTex {
  double uv[6];     // u0, v0, u1, v1, u2, v2
  double tg[3], bt[3];
};
// Light record (Scene.Lights entry, transport order): everything PDFValue/Random read.
struct alignas(16) GLight {
  double v0[3], v1[3], v2[3], e1[3], e2[3], n[3];  // triangle
  double area;
  double c0[3], c1[3], radius, t0, t1;             // sphere
  double cz[3];                                    // sphere: center(0), the PDFValue ray's time
  uint32_t kind, index;
};

// An image texture's texels in their device storage form (izpi_gpu_upload_scene repacks
// each IMAGE texture): RGBA = 4 doubles per texel as uploaded, GRAY = 1 double per texel
// for a texture whose every texel has R, G and B bit-identical (a roughness or metalness
// map): the lookup returns the same three values from an 8-B read instead of a 32-B one.
enum { TEXF_RGBA = 0, TEXF_GRAY = 1, TEXF_OTHER = 2, TEXF_NONE = 3 };
// One texture slot of a material (DevScene::mat_tex), resolved at upload so that a hit
// reads its material's textures with one dependent load less (material -> texels instead
// of material -> texture record -> texels): off = first texel (doubles into
// DevScene::texels), w, hf = height | format << 30. TEXF_OTHER: a non-image texture, off =
// its index into DevScene::textures; TEXF_NONE: no texture (-1).
struct alignas(16) TexSlot {
  uint64_t off;
  uint32_t w, hf;
};
// Slots 0..3: albedo, normal map, roughness, metalness (the PBR set, pbr.go:20-56).
struct alignas(64) MatTex {
  TexSlot s[4];
};

// The scene as the kernels read it (izpi_gpu_upload_scene). The small tables k_shade / k_tail
// stage per block in LDS are laid out by izpi_gpu.hip's lds_off (compile-time offsets; a
// render sizes the arena to the prefix it stages, lds_bytes).
struct DevScene {
  const GInner* inner;
  const GInnerQ* innerq;        // the same nodes quantised (DevScene::quantized), else null
  const GLeaf* leaves;
  const GPrim* prims;
  const GShade* shade;          // [num_prims], leaf order
  const GTriTex* tritex;        // [num_prims], leaf order: triangle UVs and tangent frame (textured scenes only, else null)
  const GLight* lights;
  const izpi_material* materials;
  const izpi_texture* textures;
  const double4* mat_const;     // per material: its constant RGB albedo / emit texture value (GShade cflags bit0)
  const MatTex* mat_tex;        // per material: its RGB texture slots
  const double* texels;
  const double* spd_wl;
  const double* spd_val;
  int32_t root;                 // encoded ref of BVH4.Nodes[0]; -1 when empty
  uint32_t num_lights;
  uint32_t nan_free_bounds;     // no NaN in any inner-node bound: slab4_fast allowed
  uint32_t leaf_shortcut;       // every leaf's slot-0 box equals its parent slot's box
  uint32_t tri_only;            // no spheres: leaf tests may be spread over the wave
  uint32_t no_pathlen;          // no dielectric material: every traced ray is a sampler ray (RAY_MAIN)
  uint32_t num_inner;           // GInner records
  uint32_t num_prims;           // GPrim records (and GLeaf slots, indexed by first primitive)
  izpi_camera cam;
  uint32_t lds_bytes;           // per render (render_body): k_shade / k_tail's dynamic LDS arena (lds_off)
  uint32_t time_free;           // no sphere moves: traversal needs no ray times (upload)
  uint32_t quantized;           // IZPI_SCENE_QUANTIZED_BVH: `inner` holds the decoded boxes of `innerq`
#ifdef IZPI_SHADOW
  // measurement builds only (byte breakdown): copies of the traversal arrays that
  // k_trace2 reads beside the real ones, so a class's bytes past L2 show as extra FETCH_SIZE
  const GInner* sh_inner;
  const GLeaf* sh_leaves;
  const GPrim* sh_prims;
#endif
};

struct RenderParams {
  uint32_t width, height, spp, max_depth;
  uint32_t chunk_spp;       // samples per pixel in this launch
  uint32_t s0;              // first sample index of this launch
  uint32_t num_pixels;      // pixels in the request
  uint32_t tile_w, tile_h;  // all tiles equal-sized
  uint32_t total_units;     // num_pixels * chunk_spp
  uint32_t lanes;           // gridDim.x * blockDim.x
  uint32_t num_bg_spd;
  const uint32_t* tiles;    // [n][4]
  const double* bg_wl;
  const double* bg_val;
  double background[3];
  uint64_t seed;
  double* out;              // [total_units][3] per-sample result
  double* recs;             // [max_depth][6][lanes] unwinding records
  uint32_t* head;           // work queue head
  unsigned long long* counters;  // 6 counters
  uint32_t* error;          // device-side guard flag
};

// ---------------------------------------------------------------- RNG
// fastrandom.LCG (fastrandom.go:41-47): state = (a*state + c) mod 2^32 — with a
// 64-bit seed the first step already reduces mod 2^32, so a uint32 state is exact.
struct Lcg {
  uint32_t s;
  IZPI_DEV double next() {
    s = 1664525u * s + 1013904223u;
    return (double)s / 4294967296.0;
  }
};
IZPI_DEV uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
#define IZPI_CAMERA_STREAM_SALT 0xD6E8FEB86659FD93ull

// Go int(float64) on amd64 (CVTTSD2SQ): NaN / out of range -> INT64_MIN.
IZPI_DEV int64_t go_int(double x) {
  if (x != x || x >= 9223372036854775808.0 || x < -9223372036854775808.0) return INT64_MIN;
  return (int64_t)x;
}

// ------------------------------------------------------------- vec3
struct V3 { double x, y, z; };
IZPI_DEV V3 mk(double x, double y, double z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
IZPI_DEV V3 ld3(const double* p) { return mk(p[0], p[1], p[2]); }
IZPI_DEV V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
IZPI_DEV V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
IZPI_DEV V3 mul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
IZPI_DEV V3 smul(V3 a, double t) { return mk(a.x * t, a.y * t, a.z * t); }
// a / t per component, correctly rounded as `/`. gfx950's f64 division is v_div_scale (x2),
// v_rcp, a Newton refinement of the reciprocal that depends on the divisor only, then
// mul, fma, v_div_fmas, v_div_fixup per dividend. When no operand needs v_div_scale's
// rescaling (divisor and dividends within 2^+-300, dividends also +-0: v_div_fixup
// alone settles a zero dividend), that is the same sequence with the scales the
// identity, so one refined reciprocal serves the three dividends: 18 instructions
// instead of 36, bit for bit the three divisions (test_sdiv_shared_reciprocal_bitwise).
IZPI_DEV bool sdiv_plain(double x) {  // exponent within 2^+-300
  return ((uint32_t)(__double2hiint(x) >> 20) & 0x7FFu) - (1023u - 300u) <= 600u;
}
IZPI_DEV V3 sdiv(V3 a, double t) {
  // (bitwise: one test, no branches)
  const int px = (int)sdiv_plain(a.x) | (int)(a.x == 0.0), py = (int)sdiv_plain(a.y) | (int)(a.y == 0.0),
            pz = (int)sdiv_plain(a.z) | (int)(a.z == 0.0);
  const bool plain = ((int)sdiv_plain(t) & px & py & pz) != 0;
  if (plain) {
    double r = __builtin_amdgcn_rcp(t);
    double e = __builtin_fma(-t, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-t, r, 1.0);
    r = __builtin_fma(r, e, r);
    auto q1 = [&](double n) {
      const double q = n * r;
      const double res = __builtin_fma(-t, q, n);
      return __builtin_amdgcn_div_fixup(__builtin_amdgcn_div_fmas(res, r, q, false), t, n);
    };
    return mk(q1(a.x), q1(a.y), q1(a.z));
  }
  return mk(a.x / t, a.y / t, a.z / t);
}
IZPI_DEV double dot(V3 a, V3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
IZPI_DEV V3 cross(V3 a, V3 b) { return mk((a.y * b.z) - (a.z * b.y), -((a.x * b.z) - (a.z * b.x)), (a.x * b.y) - (a.y * b.x)); }
IZPI_DEV double sqlen(V3 a) { return (a.x * a.x) + (a.y * a.y) + (a.z * a.z); }
IZPI_DEV double length(V3 a) { return gm::sqrt(sqlen(a)); }
IZPI_DEV V3 unit(V3 a) { return sdiv(a, length(a)); }
IZPI_DEV V3 lerp(V3 a, V3 b, double t) {
  return mk((1 - t) * a.x + t * b.x, (1 - t) * a.y + t * b.y, (1 - t) * a.z + t * b.z);
}
IZPI_DEV bool bad(double x) { return x != x || gm::is_inf(x, 0); }
IZPI_DEV V3 denan(V3 v) { return mk(bad(v.x) ? 0.0 : v.x, bad(v.y) ? 0.0 : v.y, bad(v.z) ? 0.0 : v.z); }

// onb.go:38-67
struct Onb {
  V3 u, v, w;
  IZPI_DEV void build(V3 n) {
    w = unit(n);
    V3 a = gm::abs(w.x) > 0.9 ? mk(0, 1, 0) : mk(1, 0, 0);
    v = unit(cross(w, a));
    u = cross(w, v);
  }
  IZPI_DEV V3 local(V3 a) const { return add(add(smul(u, a.x), smul(v, a.y)), smul(w, a.z)); }
};

// vec3.go:119-138
IZPI_DEV V3 random_cosine_direction(Lcg& r) {
  double r1 = r.next();
  double r2 = r.next();
  double z = gm::sqrt(1 - r2);
  double phi = 6.283185307179586 * r1;   // 2*math.Pi folded by the Go compiler
  double sp, cp;
  gm::sincos_nonneg(phi, &sp, &cp);      // = gm::sin(phi), gm::cos(phi): phi in [0, 2 Pi)
  double x = cp * 2 * gm::sqrt(r2);
  double y = sp * 2 * gm::sqrt(r2);
  return mk(x, y, z);
}
IZPI_DEV V3 random_to_sphere(double radius, double dist2, Lcg& r) {
  double r1 = r.next();
  double r2 = r.next();
  double z = 1 + r2 * (gm::sqrt(1 - radius * radius / dist2) - 1);
  double phi = 6.283185307179586 * r1;
  double sp, cp;
  gm::sincos_nonneg(phi, &sp, &cp);
  double x = cp * gm::sqrt(1 - z * z);
  double y = sp * gm::sqrt(1 - z * z);
  return mk(x, y, z);
}
// material.go:10-18
IZPI_DEV V3 random_in_unit_sphere(Lcg& r) {
  for (;;) {
    double x = r.next(), y = r.next(), z = r.next();
    V3 p = sub(smul(mk(x, y, z), 2.0), mk(1.0, 1.0, 1.0));
    if (sqlen(p) < 1.0) return p;
  }
}

// --------------------------------------------------- RayAABB4 (bvh4_simd_generic.go)
// Comparisons written as the scalar twin's select form: never fminf/fmaxf (A14).
IZPI_DEV float max32(float a, float b) { return a > b ? a : b; }
IZPI_DEV float min32(float a, float b) { return a < b ? a : b; }
IZPI_DEV bool slab(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, float ox, float oy, float oz,
                   float ix, float iy, float iz, float tmax) {
  float t0x = (mnx - ox) * ix, t1x = (mxx - ox) * ix;
  if (t0x > t1x) { float t = t0x; t0x = t1x; t1x = t; }
  float t0y = (mny - oy) * iy, t1y = (mxy - oy) * iy;
  if (t0y > t1y) { float t = t0y; t0y = t1y; t1y = t; }
  float t0z = (mnz - oz) * iz, t1z = (mxz - oz) * iz;
  if (t0z > t1z) { float t = t0z; t0z = t1z; t1z = t; }
  float tn = max32(max32(t0x, t0y), t0z);
  float tf = min32(min32(t1x, t1y), t1z);
  return tn <= tf && tf >= 0 && tn <= tmax;
}

// RayAABB4 over the 4 slots of an inner node, NaN-free fast form. When the ray's f32
// origin is finite and its f32 inverse direction is finite and non-zero on every axis,
// and the node bounds hold no NaN (checked once at upload), no t value can be NaN, so
// the scalar twin's swap / max32 / min32 reduce to IEEE min/max (they can differ only in
// the sign of a zero, which no comparison below sees): the mask is bit-identical.
// The subtract and multiply run as packed f32 pairs (children 0-1 and 2-3), min3/max3
// fold the three axes.
typedef float f32x2 __attribute__((ext_vector_type(2)));
IZPI_DEV uint32_t slab4_fast(float4 mnx, float4 mny, float4 mnz, float4 mxx, float4 mxy, float4 mxz, float ox, float oy,
                             float oz, float ix, float iy, float iz, float tmax) {
  const f32x2 o_x = {ox, ox}, o_y = {oy, oy}, o_z = {oz, oz};
  const f32x2 i_x = {ix, ix}, i_y = {iy, iy}, i_z = {iz, iz};
  const f32x2 a0x = (f32x2{mnx.x, mnx.y} - o_x) * i_x, a1x = (f32x2{mnx.z, mnx.w} - o_x) * i_x;
  const f32x2 b0x = (f32x2{mxx.x, mxx.y} - o_x) * i_x, b1x = (f32x2{mxx.z, mxx.w} - o_x) * i_x;
  const f32x2 a0y = (f32x2{mny.x, mny.y} - o_y) * i_y, a1y = (f32x2{mny.z, mny.w} - o_y) * i_y;
  const f32x2 b0y = (f32x2{mxy.x, mxy.y} - o_y) * i_y, b1y = (f32x2{mxy.z, mxy.w} - o_y) * i_y;
  const f32x2 a0z = (f32x2{mnz.x, mnz.y} - o_z) * i_z, a1z = (f32x2{mnz.z, mnz.w} - o_z) * i_z;
  const f32x2 b0z = (f32x2{mxz.x, mxz.y} - o_z) * i_z, b1z = (f32x2{mxz.z, mxz.w} - o_z) * i_z;
  const float t0x[4] = {a0x.x, a0x.y, a1x.x, a1x.y}, t1x[4] = {b0x.x, b0x.y, b1x.x, b1x.y};
  const float t0y[4] = {a0y.x, a0y.y, a1y.x, a1y.y}, t1y[4] = {b0y.x, b0y.y, b1y.x, b1y.y};
  const float t0z[4] = {a0z.x, a0z.y, a1z.x, a1z.y}, t1z[4] = {b0z.x, b0z.y, b1z.x, b1z.y};
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x[i], t1x[i]), __builtin_fminf(t0y[i], t1y[i])),
                                     __builtin_fminf(t0z[i], t1z[i]));
    const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x[i], t1x[i]), __builtin_fmaxf(t0y[i], t1y[i])),
                                     __builtin_fmaxf(t0z[i], t1z[i]));
    m |= (tn <= tf && tf >= 0.0f && tn <= tmax) ? (1u << i) : 0u;
  }
  return m;
}
IZPI_DEV bool ray_fast_ok(float ox, float oy, float oz, float ix, float iy, float iz) {
  const float inf = __builtin_huge_valf();
  return __builtin_fabsf(ox) < inf && __builtin_fabsf(oy) < inf && __builtin_fabsf(oz) < inf &&
         __builtin_fabsf(ix) < inf && __builtin_fabsf(iy) < inf && __builtin_fabsf(iz) < inf &&
         ix != 0.0f && iy != 0.0f && iz != 0.0f;
}

// ----------------------------------------------------- primitive tests
// Möller–Trumbore acceptance of Triangle.Hit (triangle.go:193-221).
IZPI_DEV bool tri_intersect(const double* a, V3 o, V3 d, double tmin, double tmax, double& t, double& u, double& v) {
  const double eps = 1e-8;
  V3 v0 = mk(a[0], a[1], a[2]), e1 = mk(a[3], a[4], a[5]), e2 = mk(a[6], a[7], a[8]);
  V3 h = cross(d, e2);
  double aa = dot(e1, h);
  if (gm::abs(aa) < eps) return false;
  double f = 1.0 / aa;
  V3 s = sub(o, v0);
  u = f * dot(s, h);
  if (u < -eps || u > 1.0 + eps) return false;
  V3 q = cross(s, e1);
  v = f * dot(d, q);
  if (v < -eps || u + v > 1.0 + eps) return false;
  t = f * dot(e2, q);
  if (t < tmin || t > tmax) return false;
  return true;
}
// The same test without the final `t > tMax` rejection: that last comparison is the
// only one that depends on tMax, so tests of one leaf can run in parallel and be
// accepted afterwards in primitive order against the running tMax (bit-identical).
IZPI_DEV bool tri_intersect_no_tmax(const double* a, V3 o, V3 d, double tmin, double& t, double& u, double& v) {
  const double eps = 1e-8;
  V3 v0 = mk(a[0], a[1], a[2]), e1 = mk(a[3], a[4], a[5]), e2 = mk(a[6], a[7], a[8]);
  V3 h = cross(d, e2);
  double aa = dot(e1, h);
  if (gm::abs(aa) < eps) return false;
  double f = 1.0 / aa;
  V3 s = sub(o, v0);
  u = f * dot(s, h);
  if (u < -eps || u > 1.0 + eps) return false;
  V3 q = cross(s, e1);
  v = f * dot(d, q);
  if (v < -eps || u + v > 1.0 + eps) return false;
  t = f * dot(e2, q);
  if (t < tmin) return false;
  return true;
}
// Sphere.center (sphere.go:495-497)
IZPI_DEV V3 sph_center(const double* a, double time) {
  V3 c0 = mk(a[0], a[1], a[2]), c1 = mk(a[3], a[4], a[5]);
  return add(c0, smul(sub(c1, c0), ((time - a[7]) / (a[8] - a[7]))));
}
// Sphere.Hit acceptance (sphere.go:63-95): root 0 or 1; strict bounds.
IZPI_DEV bool sph_intersect_at(V3 center, double radius, V3 o, V3 d, double tmin, double tmax, double& t, int& root) {
  V3 oc = sub(o, center);
  double aa = dot(d, d);
  double b = dot(oc, d);
  double c = dot(oc, oc) - (radius * radius);
  double disc = (b * b) - (aa * c);
  if (disc > 0) {
    double temp = (-b - gm::sqrt(b * b - aa * c)) / aa;
    if (temp < tmax && temp > tmin) { t = temp; root = 0; return true; }
    temp = (-b + gm::sqrt(b * b - aa * c)) / aa;
    if (temp < tmax && temp > tmin) { t = temp; root = 1; return true; }
  }
  return false;
}
// The two candidate roots of sph_intersect_at, computed without tMax/tMin (the acceptance
// `temp < tMax && temp > tMin`, root 0 first, is applied by the caller).
IZPI_DEV bool sph_roots(V3 center, double radius, V3 o, V3 d, double& t0, double& t1) {
  V3 oc = sub(o, center);
  double aa = dot(d, d);
  double b = dot(oc, d);
  double c = dot(oc, oc) - (radius * radius);
  double disc = (b * b) - (aa * c);
  if (!(disc > 0)) return false;
  t0 = (-b - gm::sqrt(b * b - aa * c)) / aa;
  t1 = (-b + gm::sqrt(b * b - aa * c)) / aa;
  return true;
}
IZPI_DEV bool sph_intersect(const double* a, V3 o, V3 d, double time, double tmin, double tmax, double& t, int& root) {
  return sph_intersect_at(sph_center(a, time), a[6], o, d, tmin, tmax, t, root);
}

}  // namespace izd
