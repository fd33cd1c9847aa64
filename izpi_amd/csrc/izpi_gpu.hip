// izpi_gpu.hip — MI355X (gfx950) path-tracing inner loop for izpi + its C ABI.
//
// Hot path restated as device code (reference files under /root/reference/internal):
//   render/rgb.go:27-41, render/spectral.go:71-106   per-sample loop   -> k_render + k_accumulate
//   camera/camera.go:61-89                           GetRay            -> camera_ray()
//   sampler/colour.go:33-65, sampler/spectral.go:47-80  recursive sampler -> iterative bounce loop
//                                                    with an explicit unwinding record per bounce
//   hitable/bvh4.go:49-164                           BVH4.Hit          -> traverse()
//   hitable/bvh4_simd_generic.go:10-52               RayAABB4          -> izd::slab()
//   hitable/triangle.go:193-280,317-326, sphere.go:63-145  prims, PDFValue, Random
//   material/*.go, pdf/*.go, texture/*.go, spectral/spectral.go:151-253
//
// Execution scheme: one persistent launch per chunk of samples.
// Work unit = one pixel-sample path (its own LCG streams). Each wave keeps 64 paths
// in flight; when a lane's path terminates it writes its radiance and the wave
// refills idle lanes from a global atomic queue (__ballot + mbcnt compaction), so
// SIMD lanes stay busy across samples of different lengths. Traversal stacks live in
// LDS ([entry][lane] layout, conflict-free at equal depth). A second, HBM-bound
// kernel sums the per-sample radiance of each pixel in sample order (bit-exact with
// render/rgb.go:36's sequential col += ...) and writes the canvas.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <thread>

#include "../../include/izpi_host.h"
#include "../../include/izpi_gpu_debug.h"
#include "izpi_dev.h"
#include "cie_tables.h"

using namespace izd;

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);                    \
      return IZPI_ERR_HIP;                                                             \
    }                                                                                  \
  } while (0)

__constant__ double c_cie_wl[IZPI_CIE_N] = IZPI_CIE_WAVELENGTHS_INIT;
__constant__ double c_cie_x[IZPI_CIE_N] = IZPI_CIE_X_INIT;
__constant__ double c_cie_y[IZPI_CIE_N] = IZPI_CIE_Y_INIT;
__constant__ double c_cie_z[IZPI_CIE_N] = IZPI_CIE_Z_INIT;
// Running sums of CIE y in SampleWavelength's own order (current += y from 0): entry i is
// the loop's `current + y` at step i, so a bisection over it stops where the scan stops.
struct CieCum { double v[IZPI_CIE_N]; };
constexpr CieCum cie_y_running_sums() {
  CieCum c{};
  constexpr double y[IZPI_CIE_N] = IZPI_CIE_Y_INIT;
  double cur = 0.0;
  for (int i = 0; i < IZPI_CIE_N; i++) { c.v[i] = cur + y[i]; cur += y[i]; }
  return c;
}
__constant__ CieCum c_cie_ycum = cie_y_running_sums();

namespace izpi_bvh {  // bvh_build.hip
int build(hipStream_t st, const double* h_boxes, uint32_t n, uint32_t leaf_max, uint32_t method,
          std::vector<izpi_bvh4_node>& nodes, std::vector<uint32_t>& order, float* ms, std::string& err);
}

#define IZPI_PASS_BATCH 8  // wavefront passes launched per host poll
// k_shade's block. Its reservation phase takes one unit-head and one queue atomic per
// block-iteration; 384-thread blocks (6 waves, 2 per CU) take a third fewer but measured
// C3 shade 114 -> 161 ms (the barriers of block_reserve2 wait for 6 waves), so 256 stays.
constexpr uint32_t SHADE_THREADS = 256, SHADE_WAVES = SHADE_THREADS / 64;
// k_shade's queue of deferred unwinding jobs per block (fin_flush): FINQ_WORDS 8-B words
// per job; flushed once FINQ_FLUSH are queued, an iteration adds at most SHADE_THREADS.
// C5 at 32 spp: shading 327.7 ms at a flush of 128, 323.1 at 256, 319.9 at 512, 318.3 at 1024
constexpr uint32_t FINQ_WORDS = 5, FINQ_FLUSH = 1024, FINQ_CAP = FINQ_FLUSH + SHADE_THREADS;
constexpr int MISC_STRIDE = 64;  // words between the fields of izpi_ctx::d_misc (misc())

enum { CNT_RAYS = 0, CNT_NODES, CNT_TRI, CNT_SPH, CNT_LTRI, CNT_LSPH, CNT_NSTEP, CNT_PSTEP, CNT_SHORT,
       CNT_CLK_REFILL, CNT_CLK_NODE, CNT_CLK_PRIM, CNT_CLK_ADV, CNT_TAIL_NODES, CNT_TAIL_TRI, CNT_TAIL_SPH,
       CNT_SCLK_ITEM, CNT_SCLK_REFILL, CNT_SCLK_PUSH, CNT_PARK, CNT_SCLK_MAT, CNT_SCLK_FIN, CNT_SCLK_MIX, CNT_SCLK_LPDF,
       CNT_SCLK_ENTRY, CNT_SCLK_TEX, CNT_SCLK_RB1, CNT_SCLK_RATOM, CNT_SCLK_RB2,
       CNT_N };  // SCLK_*: -DIZPI_SHADE_CLOCKS builds only  // CLK_*: -DIZPI_TRACE_CLOCKS builds only

// Frame counters without atomics: a render's kernels add their per-wave counts to the
// wave's own row of `cpart` ([rows][CNT_N], rows = 4 x the largest grid, zeroed per frame)
// with a plain load and store by lane 0 (the waves of a launch own distinct rows; launches
// run one after another), and k_cpart_reduce folds the rows into the counters at the end of
// the frame. Per-wave atomics on the one line of counters made every launch end in a burst
// of ~36k serialised atomics when all waves finish together: a ~0.4 ms floor per k_trace2
// pass, 4 ms of a 45-ms eighth-of-C3 share. Without `cpart` (component entries) the
// counts go to the counters by atomics as before.
IZPI_DEV void count_add(unsigned long long* cpart, unsigned long long* counters, int k, unsigned long long v) {
  if (v == 0) return;
  if (cpart) cpart[(size_t)__builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * CNT_N + k] += v;
  else atomicAdd(counters + k, v);
}

// Loads and stores of the wavefront's streamed state (rays, kind words, path state, hit
// records, unwinding records, per-sample results). (Non-temporal accesses, so that the
// stream would not displace the BVH's lines, measured no better: DESIGN 3.6.)
template <class T>
IZPI_DEV T sld(const T* p) { return *p; }
template <class T>
IZPI_DEV void sst(T* p, const T& v) { *p = v; }

// A load from a pointer known to point into LDS (the per-block staged tables): typed in
// the LDS address space, so it is a ds_read even where the same data is read from global
// memory on the other side of a branch (an untyped pointer there becomes a flat load).
template <class T>
IZPI_DEV T lds_ld(const T* p) {
  if constexpr (sizeof(T) % 8 == 0 && alignof(T) >= 8) {  // records: word by word (no copy from an LDS lvalue)
    T r;
    uint64_t* d = reinterpret_cast<uint64_t*>(&r);
    const __attribute__((address_space(3))) uint64_t* q = (const __attribute__((address_space(3))) uint64_t*)p;
#pragma unroll
    for (uint32_t i = 0; i < sizeof(T) / 8; i++) d[i] = q[i];
    return r;
  } else {
    return *(const __attribute__((address_space(3))) T*)p;
  }
}

// Loader of the table lookups below: L = the table is a staged LDS copy.
template <bool L, class T>
IZPI_DEV T tld(const T* p) {
  if constexpr (L) return lds_ld(p);
  else return *p;
}
// The scene's small tables staged in LDS by every k_shade / k_tail block (shade_stage),
// when they fit (ShadeParams::staged): materials, textures, tabulated SPDs, the background
// SPD and the CIE tables. Shading then reads them with LDS reads instead of dependent
// global loads (the compiler cannot use scalar loads for scene arrays it cannot prove
// unwritten): the light records alone took C3's shading from 128 to 114 ms.
constexpr uint32_t MAT_LDS = 64, TEX_LDS = 64, SPD_LDS = 384, BG_LDS = 128, MT_LDS = 64, LT_LDS = 64, PR_LDS = 64;
// The staged tables live at fixed offsets of the block's dynamic LDS arena, ordered so that
// what a render stages is a prefix of it: the Colour tables, then the Spectral ones, then
// the primitives. render_body sizes the arena to that prefix (lds_arena_bytes), so a render
// that stages little leaves k_tail (whose traversal stacks are LDS too) more blocks per CU.
// The offsets are compile-time: per-render offsets cost k_shade registers (the Spectral
// instances spilled 8 more VGPRs, C5's shading +2.5%; profiles/r5a/ab_arena_c5.jsonl).
namespace lds_off {
constexpr uint32_t al(uint64_t b) { return (uint32_t)((b + 31) & ~31ull); }
constexpr uint32_t MC = 0;                                        // double4 [MT_LDS]: constant colours
constexpr uint32_t MT = MC + al(MT_LDS * sizeof(double4));        // MatTex [MT_LDS]
constexpr uint32_t LT = MT + al(MT_LDS * sizeof(MatTex));         // double [LT_LDS][16]: light records
constexpr uint32_t LT2 = LT + al(LT_LDS * 16 * sizeof(double));   // double [LT_LDS][6]
constexpr uint32_t MAT = LT2 + al(LT_LDS * 6 * sizeof(double));   // izpi_material [MAT_LDS]
constexpr uint32_t TEX = MAT + al(MAT_LDS * sizeof(izpi_material));
constexpr uint32_t COLOUR_END = TEX + al(TEX_LDS * sizeof(izpi_texture));
constexpr uint32_t SPD = COLOUR_END;                              // tabulated SPDs: wavelengths
constexpr uint32_t SPDV = SPD + al(SPD_LDS * sizeof(double));     // values
constexpr uint32_t CIE = SPDV + al(SPD_LDS * sizeof(double));     // 5 x IZPI_CIE_N: wl, x, y, z, running y
constexpr uint32_t BG = CIE + al(5 * IZPI_CIE_N * sizeof(double));  // the background SPD: wavelengths
constexpr uint32_t BGV = BG + al(BG_LDS * sizeof(double));        // values
constexpr uint32_t SPECTRAL_END = BGV + al(BG_LDS * sizeof(double));
constexpr uint32_t GS = SPECTRAL_END;                             // GShade [PR_LDS]
constexpr uint32_t TT = GS + al(PR_LDS * sizeof(GShade));         // GTriTex [PR_LDS]
constexpr uint32_t GP = TT + al(PR_LDS * sizeof(GTriTex));        // GPrim [PR_LDS]
constexpr uint32_t END = GP + al(PR_LDS * sizeof(GPrim));
}  // namespace lds_off
IZPI_DEV char* lds_arena() {
  extern __shared__ __attribute__((aligned(16))) char izpi_lds_arena[];
  return izpi_lds_arena;
}
IZPI_DEV izpi_material* mat_lds() { return (izpi_material*)(lds_arena() + lds_off::MAT); }
IZPI_DEV izpi_texture* tex_lds() { return (izpi_texture*)(lds_arena() + lds_off::TEX); }
IZPI_DEV double* spd_lds() { return (double*)(lds_arena() + lds_off::SPD); }
IZPI_DEV double* spdv_lds() { return (double*)(lds_arena() + lds_off::SPDV); }
IZPI_DEV double* cie_lds() { return (double*)(lds_arena() + lds_off::CIE); }
IZPI_DEV double* bg_lds() { return (double*)(lds_arena() + lds_off::BG); }
IZPI_DEV double* bgv_lds() { return (double*)(lds_arena() + lds_off::BGV); }
IZPI_DEV izpi_material mat_rec(const DevScene& sc, bool st, uint32_t m) {
  if (st) return lds_ld(mat_lds() + m);
  return sc.materials[m];
}
IZPI_DEV izpi_texture tex_rec(const DevScene& sc, bool st, int32_t id) {
  if (st) return lds_ld(tex_lds() + id);
  return sc.textures[id];
}

// ======================================================= textures / spectra
// ImageTxt.Value (image.go:73-101): the nearest texel of a w x h image at (u, v), from
// its device storage form (TEXF_RGBA or TEXF_GRAY, see TexSlot).
IZPI_DEV V3 image_rgb(const double* texels, uint64_t off, uint32_t w, uint32_t h, uint32_t fmt, double u, double v) {
  int64_t i = go_int(u * (double)w);
  int64_t j = go_int((1 - v) * ((double)h - 0.001));
  if (i < 0) i = 0;
  if (j < 0) j = 0;
  if (i > (int64_t)w - 1) i = (int64_t)w - 1;
  if (j > (int64_t)h - 1) j = (int64_t)h - 1;
  uint64_t k = (uint64_t)j * w + (uint64_t)i;
  if (fmt == TEXF_GRAY) {
    const double g = texels[off + k];
    return mk(g, g, g);
  }
  const double* px = texels + off + k * 4;
  const double2 rg = *reinterpret_cast<const double2*>(px);  // 32-B aligned texel: one 16-B load + one 8-B load
  return mk(rg.x, rg.y, px[2]);
}
// The texel index image_rgb computes, and the lookup at a given index: a PBR hit's
// image textures usually share their size, so one index serves its four lookups.
IZPI_DEV uint64_t image_index(uint32_t w, uint32_t h, double u, double v) {
  int64_t i = go_int(u * (double)w);
  int64_t j = go_int((1 - v) * ((double)h - 0.001));
  if (i < 0) i = 0;
  if (j < 0) j = 0;
  if (i > (int64_t)w - 1) i = (int64_t)w - 1;
  if (j > (int64_t)h - 1) j = (int64_t)h - 1;
  return (uint64_t)j * w + (uint64_t)i;
}
IZPI_DEV V3 image_at(const double* texels, uint64_t off, uint32_t fmt, uint64_t k) {
  if (fmt == TEXF_GRAY) {
    const double g = texels[off + k];
    return mk(g, g, g);
  }
  const double* px = texels + off + k * 4;
  const double2 rg = *reinterpret_cast<const double2*>(px);
  return mk(rg.x, rg.y, px[2]);
}
// texture.Constant / texture.ImageTxt (constant.go:20, image.go:73-101); the device copy
// of an IMAGE texture has pad0 = its storage format
IZPI_DEV V3 tex_rgb(const DevScene& sc, int32_t id, double u, double v, bool st = false) {
  const izpi_texture t = tex_rec(sc, st, id);
  if (t.kind == IZPI_TEX_IMAGE) return image_rgb(sc.texels, t.texel_offset, t.width, t.height, t.pad0, u, v);
  return mk(t.value[0], t.value[1], t.value[2]);
}
// A material's texture slot (MatTex): images straight from their texels, other textures
// through their record
IZPI_DEV V3 slot_rgb(const DevScene& sc, const TexSlot& s, double u, double v, bool st = false) {
  const uint32_t fmt = s.hf >> 30;
  if (fmt <= TEXF_GRAY) return image_rgb(sc.texels, s.off, s.w, s.hf & 0x3FFFFFFFu, fmt, u, v);
  return tex_rgb(sc, (int32_t)s.off, u, v, st);
}
IZPI_DEV bool slot_set(const TexSlot& s) { return (s.hf >> 30) != TEXF_NONE; }
// slot_rgb with the texel index k0 of a w0 x h0 image at the same (u, v) (image_index):
// reused when this slot's image has that size, else computed.
IZPI_DEV V3 slot_rgb_k(const DevScene& sc, const TexSlot& s, double u, double v, bool st, uint32_t w0, uint32_t h0, uint64_t k0) {
  const uint32_t fmt = s.hf >> 30, h = s.hf & 0x3FFFFFFFu;
  if (fmt <= TEXF_GRAY) {
    uint64_t k = k0;
    if (s.w != w0 || h != h0) k = image_index(s.w, h, u, v);
    return image_at(sc.texels, s.off, fmt, k);
  }
  return slot_rgb(sc, s, u, v, st);
}
// The materials' texture slots staged in LDS next to their constants (mc_stage): a PBR
// hit reads its slots with an LDS read instead of a dependent L2 load.
IZPI_DEV MatTex* mt_lds() { return (MatTex*)(lds_arena() + lds_off::MT); }
// Slot k of material m: from LDS when staged (`staged`), else from DevScene::mat_tex.
IZPI_DEV TexSlot mat_slot(const DevScene& sc, bool staged, uint32_t m, int k) {
  if (staged) return lds_ld(&mt_lds()[m].s[k]);
  return sc.mat_tex[m].s[k];
}
// First interval [wl[i], wl[i+1]] of a NON-DECREASING table that holds w, for
// n >= 2 and wl[0] <= w <= wl[n-1]: i = (first j >= 1 with wl[j] >= w) - 1, which is the interval
// the reference's linear scan stops at (spectral.go:151-181, spectral_constant.go:88-106):
// every earlier interval ends below w. ~log2(n) dependent loads instead of up to n.
template <bool L = false>
IZPI_DEV uint32_t sorted_interval(const double* wl, uint32_t n, double w) {
  uint32_t lo = 1, hi = n - 1;  // wl[n-1] >= w, so the answer is in [1, n-1]
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (tld<L>(wl + mid) >= w) hi = mid; else lo = mid + 1;
  }
  return lo - 1;
}

// SpectralImage.rgbToSpectralValue (spectral_image.go:130-190): the spectral value of an
// RGB texel at a bucket wavelength.
IZPI_DEV double spectral_image_value(double r, double g, double b, double wl) {
  double sv = 0;
  if (wl >= 580.0 && wl <= 750.0) {  // red: Gaussian falloff around 650 nm, width 60
    const double dist = gm::abs(wl - 650.0);
    sv += r * gm::exp(-(dist * dist) / (2.0 * 60.0 * 60.0));
  }
  if (wl >= 480.0 && wl <= 620.0) {  // green: around 550 nm
    const double dist = gm::abs(wl - 550.0);
    sv += g * gm::exp(-(dist * dist) / (2.0 * 60.0 * 60.0));
  }
  if (wl >= 380.0 && wl <= 520.0) {  // blue: around 450 nm
    const double dist = gm::abs(wl - 450.0);
    sv += b * gm::exp(-(dist * dist) / (2.0 * 60.0 * 60.0));
  }
  if (gm::abs(r - g) < 0.15 && gm::abs(g - b) < 0.15 && gm::abs(r - b) < 0.15) sv = gm::max(sv, gm::max(r, gm::max(g, b)));
  const double mx = gm::max(r, gm::max(g, b));
  if (mx > 0.7 && sv < mx * 0.8) sv = gm::max(sv, mx * 0.8);
  return gm::max(0.0, gm::min(1.0, sv));
}
// SpectralImage.Value (spectral_image.go:193-259): the texel ImageTxt.Value reads, at the
// first 5-nm bucket (380..750 nm) >= lambda. The reference tabulates rgbToSpectralValue
// per texel and bucket up front; the same function is evaluated here per lookup.
IZPI_DEV double tex_spectral_image(const DevScene& sc, const izpi_texture& t, double u, double v, double lambda) {
  int64_t i = go_int(u * (double)t.width);
  int64_t j = go_int((1 - v) * ((double)t.height - 0.001));
  if (i < 0) i = 0;
  if (j < 0) j = 0;
  if (i > (int64_t)t.width - 1) i = (int64_t)t.width - 1;
  if (j > (int64_t)t.height - 1) j = (int64_t)t.height - 1;
  int k = 74;  // findWavelengthIndex: below 380 -> 0, above 750 (or NaN) -> 74
  if (lambda < 380.0) k = 0;
  else if (!(lambda > 750.0))
    for (k = 0; k < 74; k++)
      if (lambda <= 380.0 + 5.0 * (double)k) break;
  const double* px = sc.texels + t.texel_offset + ((uint64_t)j * t.width + (uint64_t)i) * 4;
  return spectral_image_value(px[0], px[1], px[2], 380.0 + 5.0 * (double)k);
}

// texture.SpectralConstant.Value (spectral_constant.go:65-106); SpectralImage reads (u, v)
// The tabulated SPD lookup of SpectralConstant.Value (spectral_constant.go:88-106) on the
// table at wl / vl (L: staged in LDS)
template <bool L>
IZPI_DEV double tab_value(const double* wl, const double* vl, const izpi_texture& t, double lambda) {
  const uint32_t n = t.spd_count;
  if (n == 0) return 0.0;
  if (lambda < tld<L>(wl)) return tld<L>(vl);
  if (lambda > tld<L>(wl + n - 1)) return tld<L>(vl + n - 1);
  if (t.pad0 == 2 && lambda == lambda) {
    // near-uniform wavelengths (set at upload): the interval's index is guessed from
    // lambda, its two wavelengths and values load together, and a short walk fixes a
    // wrong guess, so the result is the scan's interval exactly
    uint32_t g = 1u + (uint32_t)((lambda - t.value[0]) * t.value[1]);
    g = g > n - 1 ? n - 1 : g;
    double w1 = tld<L>(wl + g - 1), w2 = tld<L>(wl + g), v1 = tld<L>(vl + g - 1), v2 = tld<L>(vl + g);
    if (!((g == 1 || w1 < lambda) && w2 >= lambda)) {
      while (g > 1 && tld<L>(wl + g - 1) >= lambda) g--;
      while (tld<L>(wl + g) < lambda) g++;
      w1 = tld<L>(wl + g - 1); w2 = tld<L>(wl + g); v1 = tld<L>(vl + g - 1); v2 = tld<L>(vl + g);
    }
    const double tt = (lambda - w1) / (w2 - w1);
    return v1 + tt * (v2 - v1);
  }
  if (t.pad0 && lambda == lambda) {  // pad0: wavelengths non-decreasing (set at upload)
    const uint32_t i = sorted_interval<L>(wl, n, lambda);
    const double w1 = tld<L>(wl + i), w2 = tld<L>(wl + i + 1);
    const double tt = (lambda - w1) / (w2 - w1);
    return tld<L>(vl + i) + tt * (tld<L>(vl + i + 1) - tld<L>(vl + i));
  }
  for (uint32_t i = 0; i + 1 < n; i++) {
    double w1 = tld<L>(wl + i), w2 = tld<L>(wl + i + 1);
    if (lambda >= w1 && lambda <= w2) {
      double tt = (lambda - w1) / (w2 - w1);
      return tld<L>(vl + i) + tt * (tld<L>(vl + i + 1) - tld<L>(vl + i));
    }
  }
  return 0.0;
}
IZPI_DEV double tex_spectral(const DevScene& sc, int32_t id, double lambda, double u = 0.0, double v = 0.0, bool st = false) {
  const izpi_texture t = tex_rec(sc, st, id);
  if (t.kind == IZPI_TEX_SPECTRAL_IMAGE) return tex_spectral_image(sc, t, u, v, lambda);
  if (t.kind == IZPI_TEX_SPECTRAL_TABULATED) {
    if (st) return tab_value<true>(spd_lds() + t.spd_offset, spdv_lds() + t.spd_offset, t, lambda);
    return tab_value<false>(sc.spd_wl + t.spd_offset, sc.spd_val + t.spd_offset, t, lambda);
  }
  double exponent = -gm::pow((lambda - t.center) / t.width_nm, 2);
  return t.peak * gm::exp(exponent);
}
// SpectralPowerDistribution.Value (spectral.go:151-181)
template <bool L = false>
IZPI_DEV double spd_value(const double* wl, const double* vl, uint32_t n, double w, bool sorted = false) {
  if (n == 0) return 0.0;
  if (w <= tld<L>(wl)) return tld<L>(vl);
  if (w >= tld<L>(wl + n - 1)) return tld<L>(vl + n - 1);
  if (sorted && w == w) {  // (NaN falls through to the scan, which matches no interval)
    const uint32_t i = sorted_interval<L>(wl, n, w);
    const double w1 = tld<L>(wl + i), w2 = tld<L>(wl + i + 1);
    const double t = (w - w1) / (w2 - w1);
    return tld<L>(vl + i) + t * (tld<L>(vl + i + 1) - tld<L>(vl + i));
  }
  for (uint32_t i = 0; i + 1 < n; i++) {
    double w1 = tld<L>(wl + i), w2 = tld<L>(wl + i + 1);
    if (w >= w1 && w <= w2) {
      double t = (w - w1) / (w2 - w1);
      return tld<L>(vl + i) + t * (tld<L>(vl + i + 1) - tld<L>(vl + i));
    }
  }
  return 0.0;
}
// spectral.SampleWavelength (spectral.go:184-224): the scan stops at the first i whose
// running sum reaches the target (y >= 0, so the sums never decrease): bisected.
// The CIE tables: __constant__ memory, or the block's LDS copy (L; shade_stage)
template <bool L>
struct Cie {
  IZPI_DEV static const double* wl() { return L ? cie_lds() : c_cie_wl; }
  IZPI_DEV static const double* x() { return L ? cie_lds() + IZPI_CIE_N : c_cie_x; }
  IZPI_DEV static const double* y() { return L ? cie_lds() + 2 * IZPI_CIE_N : c_cie_y; }
  IZPI_DEV static const double* z() { return L ? cie_lds() + 3 * IZPI_CIE_N : c_cie_z; }
  IZPI_DEV static const double* ycum() { return L ? cie_lds() + 4 * IZPI_CIE_N : c_cie_ycum.v; }
};
template <bool L = false>
IZPI_DEV void sample_wavelength(double random, double& lambda, double& pdf) {
  using C = Cie<L>;
  const double target = random * IZPI_CIE_Y_INTEGRAL;
  const double* cum = C::ycum();
  if (!(tld<L>(cum + IZPI_CIE_N - 1) >= target)) {  // the scan ran off the end
    lambda = 750;
    pdf = tld<L>(C::y() + IZPI_CIE_N - 1) / IZPI_CIE_Y_INTEGRAL;
    return;
  }
  uint32_t lo = 0, hi = IZPI_CIE_N - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (tld<L>(cum + mid) >= target) hi = mid; else lo = mid + 1;
  }
  const uint32_t i = lo;
  const double y = tld<L>(C::y() + i);
  if (i > 0) {
    const double prev = tld<L>(cum + i - 1);
    const double t = (target - prev) / y;
    lambda = tld<L>(C::wl() + i - 1) + t * (tld<L>(C::wl() + i) - tld<L>(C::wl() + i - 1));
    const double iy = tld<L>(C::y() + i - 1) + t * (tld<L>(C::y() + i) - tld<L>(C::y() + i - 1));
    pdf = iy / IZPI_CIE_Y_INTEGRAL;
    return;
  }
  lambda = tld<L>(C::wl() + i);
  pdf = y / IZPI_CIE_Y_INTEGRAL;
}
// spectral.GetCIEValues (spectral.go:227-253); the index scan over the ascending CIE
// wavelengths is bisected (sorted_interval returns index - 1)
template <bool L = false>
IZPI_DEV void cie_values(double w, double& x, double& y, double& z) {
  using C = Cie<L>;
  const double *W = C::wl(), *X = C::x(), *Y = C::y(), *Z = C::z();
  if (w <= tld<L>(W)) { x = tld<L>(X); y = tld<L>(Y); z = tld<L>(Z); return; }
  if (w >= tld<L>(W + IZPI_CIE_N - 1)) {
    x = tld<L>(X + IZPI_CIE_N - 1); y = tld<L>(Y + IZPI_CIE_N - 1); z = tld<L>(Z + IZPI_CIE_N - 1);
    return;
  }
  int index = 0;
  if (w == w) index = (int)sorted_interval<L>(W, IZPI_CIE_N, w) + 1;
  double w1 = tld<L>(W + index - 1), w2 = tld<L>(W + index);
  double t = (w - w1) / (w2 - w1);
  x = tld<L>(X + index - 1) + t * (tld<L>(X + index) - tld<L>(X + index - 1));
  y = tld<L>(Y + index - 1) + t * (tld<L>(Y + index) - tld<L>(Y + index - 1));
  z = tld<L>(Z + index - 1) + t * (tld<L>(Z + index) - tld<L>(Z + index - 1));
}

// ============================================================ wavefront state
// The paths in flight live in queue order: entry i of a pass's queue IS path i's state
// (ray, hit, path), held in record arrays indexed by queue position and double-buffered
// between passes (WaveBuf in / out). k_trace2 reads the rays of a chunk of consecutive
// entries and writes their hits in place; k_shade reads entry i and writes a continuing
// path to the position its block reserved on the output side, so every wave reads and
// writes contiguous runs: no slot indirection, no scattered partial-line stores. Only a
// path's unwinding records stay put, in its record slot (rslot), written once per bounce
// and read back when the path finishes.
struct RayRec {               // register form
  double o[3], d[3];
  double time;
  uint32_t kind;              // kind word (below)
};
struct alignas(16) RayOD { double o[3], d[3]; };  // 48 B
// kind word: bits 0-1 RAY_MAIN / RAY_PATHLEN, bit 2 RAY_PARKED, bit 3 RAY_DEAD, bits 4-31
// the dielectric material of a path-length ray (<< KIND_MAT_SHIFT).
// RAY_MAIN rays count as Sampler calls and run tMin 0.001 .. MaxFloat64 (colour.go:39);
// RAY_PATHLEN rays are calculatePathLength's World.Hit, tMin 0 .. 1000 (dielectric.go:135).
// RAY_PARKED: the entry's shading pass waits for an overflow record block (pool_alloc);
// k_trace2 skips it and the next k_shade shades the same traced ray again (the pass reads
// only stored state, so the retry computes exactly what the first attempt would have).
// RAY_DEAD: an entry reserved for a new path that has no ray (its sample completed at once:
// spectral pdf 0, maxDepth 0; or the units ran out); every kernel skips it. Its ray origin
// x also holds DEAD_BITS, a signalling-NaN pattern no arithmetic produces, so k_trace2
// tells it apart without reading kind words.
constexpr uint64_t DEAD_BITS = 0x7FF4DEADDEADDEADull;
enum { RAY_MAIN = 0, RAY_PATHLEN = 1, RAY_PARKED = 4, RAY_DEAD = 8, KIND_MAT_SHIFT = 4 };
IZPI_DEV uint32_t kind_of(uint32_t k) { return k & 3u; }
// Closest hit of an entry's ray: ONE aligned 32-B record (t, primitive, barycentrics).
// k_shade reads the first 16 B on every pass and (u, v) only for UV-textured and sphere hits.
struct HitOut {               // register form
  double t, u, v;             // triangle barycentrics, or u = sphere root
  int32_t prim;               // leaf-order primitive, -1 = miss
  uint32_t pad;
};
// A traced ray's closest hit, in two per-entry arrays (WaveBuf::hit, ::huv): (t, primitive)
// as a double2 whose second double carries the primitive in its low word (-1: none), and
// (u, v) (a sphere: u = the root taken, A16) only for scenes whose shading reads them.
IZPI_DEV double2 hit_pack(double t, int32_t prim) { return make_double2(t, __hiloint2double(0, prim)); }
IZPI_DEV int32_t hit_prim(double2 h) { return (int32_t)__double2loint(h.y); }
struct PathSt {               // register form
  double lambda, lpdf;        // wavelength and its pdf (spectral)
  double pend[3];             // dielectric hit point while its path-length ray is traced
  double thr[3];              // IZPI_ACC_FORWARD: the path's throughput (Spectral: thr[0])
  uint32_t rng, depth, unit, rslot, blk;
  uint32_t zf;                // ZF_*: what unwinding its records does to a zero radiance (finish)
};
// What the unwinding of a path's records (finish) makes of a terminal radiance of +0, kept
// up to date as the records are written (rec_zero_track), so that finish can skip the
// record reads for such paths (open-box escapes, max depth into a black background):
//   ZF_UNSAFE: some level may turn a zero into a non-zero or a NaN (an infinite or NaN
//              attenuation or scattering pdf, or a pdf of 0 or NaN);
//   ZF_RESET:  a non-specular level was written: 0.0 + (att * (L * s)) / p maps +-0 to +0,
//              so the levels written after it (applied before it) cannot change the sign;
//   ZF_SIGN:   bit c = the sign of component c after unwinding a +0: the XOR of the
//              attenuation signs of the specular levels below the first non-specular one.
// Stored in the high half of PathHot::depth.
enum : uint32_t { ZF_UNSAFE = 1, ZF_RESET = 2, ZF_SIGN_SHIFT = 2 };
// rslot: the path's record slot; blk: 1 + the overflow record block holding its
// unwinding records at depths >= ShadeParams::rec_dense (0 = none yet), see pool_alloc.
struct alignas(16) PathHot { uint32_t rng, depth, unit, rslot; };
struct alignas(16) PathCold { double lambda, lpdf; double pend[3]; double pad; };

// One side of the double-buffered state, indexed by queue position.
struct WaveBuf {
  RayOD* ray;
  uint32_t* kind;     // kind word
  double* time;       // ray time (scenes with spheres), else null
  PathHot* path;
  uint32_t* blk;      // overflow block + 1
  PathCold* cold;     // spectral / dielectric scenes, else null
  double2* hit;       // (t, primitive): hit_pack; entry i at hit[i * hs]
  double2* huv;       // (u, v) of the hit, entry i at huv[i * hs]; null when nothing reads it (WaveParams::hit_uv == 0)
  uint32_t hs;        // 1: hit alone (16-B stride); 2: hit and (u, v) interleaved (huv = hit + 1), one 32-B record per entry
  const double2* tminmax;  // izpi_gpu_trace only: per-entry (tMin, tMax) instead of the kind's
  double* thr;        // IZPI_ACC_FORWARD: the throughput, component c of entry i at thr[c * tplane + i]; else null
  uint32_t tplane;
};
struct WaveParams {
  WaveBuf in, out;
  const uint32_t* in_count;   // entries in `in` this pass
  uint32_t* out_count;        // entries k_shade appends to `out`
  uint32_t* trace_next;       // dynamic-fetch cursor of k_trace2
  unsigned long long* pool_ctr;  // overflow-record ring counters (k_trace2 publishes frees), or null
  uint32_t slots;
  uint32_t read_kind;         // path-length rays or explicit tMin / tMax can occur (k_trace2 reads kind words)
  const uint32_t* in_park;    // nonzero: the pass that wrote `in` parked entries (k_trace2 reads kind words), or null
  uint32_t* out_park;         // set by k_shade when it parks an entry of `out` (zeroed by k_trace2)
  uint32_t hit_uv;            // k_shade may read a hit's (u, v): spheres (the root) or (u,v)-reading textures;
                              // then the hit records are interleaved (WaveBuf::hs == 2)
  unsigned long long* cpart;  // per-wave counter rows (count_add), or null
};
IZPI_DEV double ray_tmin(const WaveBuf& b, uint32_t i, uint32_t kind) {
  return b.tminmax ? b.tminmax[i].x : (kind_of(kind) == RAY_PATHLEN ? 0.0 : 0.001);
}
IZPI_DEV double ray_tmax(const WaveBuf& b, uint32_t i, uint32_t kind) {
  return b.tminmax ? b.tminmax[i].y : (kind_of(kind) == RAY_PATHLEN ? 1000.0 : 1.7976931348623157e308);
}

// Overflow record blocks (see pool_alloc) come in POOL_SHARDS independent rings, each
// with its own counters on its own 128-B line: [0] allocation head, [1] free tail,
// [2] published free tail (one counter word serialises its atomics, ~88/us chip-wide).
constexpr uint32_t POOL_SHARDS = 256, POOL_CTR_STRIDE = 16;
// Make the frees of the last shading pass available to allocations (thread t of the
// calling block handles rings t, t + blockDim, ...); failed allocations overshot the
// head, so clamp it first.
IZPI_DEV void pool_publish(unsigned long long* ctr) {
  for (uint32_t r = threadIdx.x; r < POOL_SHARDS; r += blockDim.x) {
    unsigned long long* c = ctr + (size_t)r * POOL_CTR_STRIDE;
    const unsigned long long head = c[0], pub = c[2];
    c[0] = head < pub ? head : pub;
    c[2] = c[1];
  }
}

// ============================================================ traversal
// BVH4.Hit (bvh4.go:49-164) for one ray in one lane: k_tail's traversal (the wavefront
// passes use k_trace2 below). Same visit order and counters. The stack's first
// TAIL_LDS_STACK entries are in LDS (stk, stride 256), deeper ones (STACK > TAIL_LDS_STACK,
// rare) in the lane's global spill column (gsp, stride gstride).
constexpr int TAIL_LDS_STACK = 32;
template <int STACK>
IZPI_DEV void trace_one(const DevScene& sc, const WaveBuf& b, uint32_t qi, int32_t* stk, int32_t* gsp, uint32_t gstride,
                        uint32_t& c_rays, uint32_t& c_nodes, uint32_t& c_tri, uint32_t& c_sph, uint32_t* err) {
  const RayOD& r = b.ray[qi];
  const uint32_t kind = b.kind[qi];
  const V3 o = mk(r.o[0], r.o[1], r.o[2]), d = mk(r.d[0], r.d[1], r.d[2]);
  const double tmin = ray_tmin(b, qi, kind), time = b.time ? b.time[qi] : 0.0;
  double tmax = ray_tmax(b, qi, kind);
  if (kind_of(kind) == RAY_MAIN) c_rays++;
  const float ix = (float)(1.0 / d.x), iy = (float)(1.0 / d.y), iz = (float)(1.0 / d.z);
  const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
  int32_t cur = sc.root;
  int sp = 0;
  double bu = 0, bv = 0;
  int32_t bprim = -1;
  while (cur != -1) {
    c_nodes++;
    const float tm = (float)tmax;
    int32_t next = -1;
    if (ref_is_leaf(cur)) {
      const float4* lp = reinterpret_cast<const float4*>(sc.leaves + leaf_start(cur));
      const float4 a = lp[0], b = lp[1];
      if (slab(a.x, a.y, a.z, a.w, b.x, b.y, ox, oy, oz, ix, iy, iz, tm)) {
        const int32_t start = leaf_start(cur), end = start + leaf_count(cur);
        for (int32_t k = start; k < end; k++) {  // bvh4.go:123-134
          const double2* pp = reinterpret_cast<const double2*>(sc.prims + k);
          const double2 p0 = pp[0], p1 = pp[1], p2 = pp[2], p3 = pp[3], p4 = pp[4];
          const double pa[9] = {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y, p4.x};
          if ((uint32_t)__double2loint(p4.y) == IZPI_PRIM_TRIANGLE) {
            c_tri++;
            double t, u, v;
            if (tri_intersect(pa, o, d, tmin, tmax, t, u, v)) { tmax = t; bu = u; bv = v; bprim = k; }
          } else {
            c_sph++;
            double t; int root;
            if (sph_intersect(pa, o, d, time, tmin, tmax, t, root)) { tmax = t; bu = (double)root; bv = 0; bprim = k; }
          }
        }
      }
    } else {
      const float4* np = reinterpret_cast<const float4*>(sc.inner + cur);
      const float4 mnx = np[0], mny = np[1], mnz = np[2], mxx = np[3], mxy = np[4], mxz = np[5];
      const int4 ch = *reinterpret_cast<const int4*>(np + 6);
      const float amnx[4] = {mnx.x, mnx.y, mnx.z, mnx.w}, amny[4] = {mny.x, mny.y, mny.z, mny.w},
                  amnz[4] = {mnz.x, mnz.y, mnz.z, mnz.w}, amxx[4] = {mxx.x, mxx.y, mxx.z, mxx.w},
                  amxy[4] = {mxy.x, mxy.y, mxy.z, mxy.w}, amxz[4] = {mxz.x, mxz.y, mxz.z, mxz.w};
      const int32_t ach[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {  // bvh4.go:119-146
        if (ach[i] == -1) continue;
        if (!slab(amnx[i], amny[i], amnz[i], amxx[i], amxy[i], amxz[i], ox, oy, oz, ix, iy, iz, tm)) continue;
        if (next == -1) {
          next = ach[i];
        } else if (sp < STACK) {
          if (STACK <= TAIL_LDS_STACK || sp < TAIL_LDS_STACK) stk[sp * 256] = ach[i];
          else gsp[(size_t)(sp - TAIL_LDS_STACK) * gstride] = ach[i];
          sp++;
        } else {
          atomicOr(err, 1u);  // unreachable: STACK >= host-computed bound
        }
      }
    }
    if (next != -1) {
      cur = next;
    } else if (sp > 0) {
      sp--;
      cur = (STACK <= TAIL_LDS_STACK || sp < TAIL_LDS_STACK) ? stk[sp * 256] : gsp[(size_t)(sp - TAIL_LDS_STACK) * gstride];
    } else {
      cur = -1;
    }
  }
  b.hit[(size_t)qi * b.hs] = hit_pack(bprim >= 0 ? tmax : 0.0, bprim);
  if (b.huv) b.huv[(size_t)qi * b.hs] = make_double2(bu, bv);
}

// BVH4.Hit, step-scheduled variant. Each lane is in one of two modes: NODE (visit
// the node `cur`: the 4-slot box test of an inner node, or the slot-0 re-test of a
// leaf, A10) or PRIM (test primitive pk of the leaf being scanned, one per step).
// Every loop iteration the wave runs ONE kind of step — the one most of its busy lanes
// want (weighted by the relative cost of a node step and an f64 primitive test) — so
// f32 node code and f64 triangle code no longer serialise inside one iteration. Each
// ray still performs exactly the reference's sequence of node visits and primitive
// tests (bvh4.go:76-160), only interleaved differently with other rays, so results and
// counters are unchanged.
// The traversal stack is a ring of S entries per lane in LDS; when a push finds the
// ring full, the oldest entry is spilled to a per-thread global area (entry e at
// spill[e * stride + gtid], <= 64 entries as bvh4.go:71) and read back on pop. Counters
// are kept per wave in SGPRs (popcounts of ballots).
// TRI: the scene holds no spheres (DevScene::tri_only), so the sphere code is compiled out.
// LB: the whole BVH (inner nodes, leaf records, primitives) is small enough to sit in this
// block's LDS (bvh_lds_fits: at most BVH_LDS_BYTES): every node and primitive load is an
// LDS read instead of an L1/L2 round trip (C2, C4, C5: 10-22 primitives).
// RL: triangle-only scene whose hits need no (u, v) (wp.hit_uv == 0, C3): the lane's f64 ray
// is kept in LDS from its refill on, so a primitive test reads its owner's ray with three
// ds_read_b128 instead of re-reading the 48-B record from global memory, where it has
// usually left the XCD's L2 by then; the (u, v) arrays it does not need make room for it
// (31.8 KB of LDS per block: still 5 blocks per CU).
constexpr uint32_t BVH_LDS_BYTES = 4096;
template <int S, int WPE, bool DIST, bool TRI, bool LB, bool RL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) k_trace2(const DevScene sc, const WaveParams wp, unsigned long long* counters,
                                                uint32_t* err, int32_t* spill, uint32_t spill_stride, uint32_t prim_w,
                                                uint32_t tchunk, uint32_t refill_min) {
  static_assert((S & (S - 1)) == 0, "ring size must be a power of two");
  static_assert(!LB || DIST, "the LDS-resident BVH instance runs the distributed leaf tests");
  static_assert(!RL || (DIST && (TRI || LB)), "the LDS-resident ray instances: triangle-only global BVH, or the BVH in LDS");
  // (u, v) of the accepted hit: kept in lds_uv until the ray finishes (UVL), stored to the
  // hit record at acceptance (UVS: the BVH-in-LDS ray instance, whose steps issue no global
  // loads for the store to hold up), or not kept (C3's instance: nothing reads it)
  constexpr bool UVL = !RL, UVS = RL && LB, DUV = !RL || LB;
  typedef float v4f __attribute__((ext_vector_type(4)));   // clang vectors: copyable out of an LDS lvalue
  typedef double v2d __attribute__((ext_vector_type(2)));
  typedef const __attribute__((address_space(3))) v4f LF4;
  typedef const __attribute__((address_space(3))) v2d LD2;
  __shared__ float4 bvh_lds[LB ? BVH_LDS_BYTES / 16 : 1];
  // LDS layout: inner nodes (8 float4 each), leaf records by first primitive (2), primitives (5)
  LF4* const l_inner = (LF4*)bvh_lds;
  LF4* const l_leaves = l_inner + (size_t)8 * (LB ? sc.num_inner : 0);
  LD2* const l_prims = (LD2*)(l_leaves + (size_t)2 * (LB ? sc.num_prims : 0));
  if constexpr (LB) {
    const uint32_t ni = 8 * sc.num_inner, nl = 2 * sc.num_prims, np5 = 5 * sc.num_prims;
    for (uint32_t t = threadIdx.x; t < ni + nl + np5; t += 256)
      bvh_lds[t] = t < ni ? reinterpret_cast<const float4*>(sc.inner)[t]
                          : (t < ni + nl ? reinterpret_cast<const float4*>(sc.leaves)[t - ni]
                                         : reinterpret_cast<const float4*>(sc.prims)[t - ni - nl]);
    __syncthreads();
  }
  __shared__ int32_t lds_stack[S * 256];
  // DIST: one wave-wide batch of leaf tests: (primitive << 6 | owner lane), then the
  // test's result flags in the same word; distances and barycentrics
  // (+4: an owner reads its four entries unconditionally, past the wave's last batch entry)
  __shared__ uint32_t dist_owner[DIST ? 260 : 1];
  __shared__ double dist_t[DIST ? 260 : 1], dist_u[DIST && DUV ? 260 : 1], dist_v[DIST && DUV ? 260 : 1];
  // (u, v) of the lane's accepted hit so far: the hit record is stored once, when the ray finishes
  // (a global store per accepted hit would hold up the wave's next load wait, since
  // vmcnt counts stores and loads in one queue)
  __shared__ double2 lds_uv[UVL ? 256 : 1];
  // RL: the lane's ray (o, d) as three double2, written at its refill
  __shared__ double2 ray_lds[RL ? 3 * 256 : 1];
  const uint32_t wbase = threadIdx.x & ~63u;
  int32_t* stk = lds_stack + threadIdx.x;
  int32_t* gsp = spill + blockIdx.x * 256 + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n = *wp.in_count;
  if (wp.pool_ctr && blockIdx.x == 0) pool_publish(wp.pool_ctr);
  // the next k_shade appends to out_count from 0 (its old value, an earlier pass's input
  // count, is read by no one any more): no memset launch per pass
  if (wp.out_count && blockIdx.x == 0 && threadIdx.x == 0) *wp.out_count = 0;
  if (wp.out_park && blockIdx.x == 0 && threadIdx.x == 0) *wp.out_park = 0;
  // kind words other than RAY_MAIN exist only with dielectrics (path-length rays), explicit
  // tMin / tMax, or after a shading pass that parked entries on an empty overflow pool (dead
  // entries are recognised by their ray)
  const bool read_kind = wp.read_kind != 0 || (wp.in_park && *wp.in_park != 0);
  // Small queues (the wavefront's tail passes): chunks shrink so the rays spread over
  // more waves, and waves past the last chunk exit at once instead of each paying a
  // dequeue atomic on the one counter word (~88/us chip-wide).
  const uint32_t nwaves = gridDim.x * 4u;
  const uint32_t chunk = min(tchunk, max(16u, (n + nwaves - 1u) / nwaves));
  // each wave's first chunk is its own, without an atomic; the rest is dequeued in chunks
  // (larger static first ranges measured slower: DESIGN 3.6)
  const uint32_t first = chunk;
  if ((uint64_t)(blockIdx.x * 4u + (threadIdx.x >> 6)) * first >= n) return;
  uint64_t c_rays = 0, c_nodes = 0, c_tri = 0, c_sph = 0;  // wave-uniform (SGPR)
  uint64_t c_nstep = 0, c_pstep = 0, c_short = 0;
  bool busy = false, in_prim = false;
  bool exhausted = false;
  uint32_t qi = 0;        // the lane's queue entry (its ray, hit and path state index)
  uint32_t lkind = RAY_MAIN;
  double tmax = 0;
  float ix = 0, iy = 0, iz = 0, ox = 0, oy = 0, oz = 0;
  int32_t cur = -1, pk = 0, pend = 0;
  int sp = 0, low = 0;
  int clean_from = 0;     // stack entries at positions >= clean_from were pushed after the last accepted hit
  int32_t bprim = -1;
  bool fast = false;      // slab4_fast is exact for this ray
#ifdef IZPI_SHADOW
  // measurement: spilled stack entries stored / loaded (wave counts), and a sink for the
  // shadow loads (bit 1: inner nodes, 2: leaf records, 4: primitives)
  uint64_t c_spill_st = 0, c_spill_ld = 0;
  uint32_t sh_acc = 0;
#endif
  // wave-private range [c_pos, c_end) of the input queue; the first one is the wave's own
  uint32_t c_pos = __builtin_amdgcn_readfirstlane((blockIdx.x * 4u + (threadIdx.x >> 6)) * first);  // (uniform: SGPR)
  uint32_t c_end = c_pos + first < n ? c_pos + first : n;
#ifdef IZPI_TRACE_CLOCKS
  uint64_t k_refill = 0, k_node = 0, k_prim = 0, k_adv = 0, k0 = 0, k1 = 0;
#define IZPI_CLK(v) (v) = __builtin_readcyclecounter()
#else
#define IZPI_CLK(v) (void)0
#endif
  for (;;) {
    IZPI_CLK(k0);
    const uint64_t idle = __ballot(!busy);
    if (idle != 0) {
      const uint32_t nidle = (uint32_t)__popcll(idle);
      if (!exhausted && (nidle >= refill_min || idle == ~0ull) && c_pos >= c_end) {
        // the wave's private range of the queue is used up: take the next `chunk`
        // entries with one atomic (a single head word saturates near 88 dequeues/us).
        // Every wave's first chunk is its own (chunk w, set before the loop), without an
        // atomic: a pass of at most nwaves chunks (the tail passes) dequeues without any.
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(wp.trace_next, chunk);
        b = __builtin_amdgcn_readfirstlane(b) + nwaves * first;
        if (b >= n) exhausted = true;
        c_pos = b;
        c_end = b + chunk < n ? b + chunk : n;
      }
      if (!exhausted && (nidle >= refill_min || idle == ~0ull) && c_pos < c_end) {
        const uint32_t take = nidle < c_end - c_pos ? nidle : c_end - c_pos;
        const uint32_t base = c_pos;
        c_pos += take;
        bool main_ray = false;
        const uint32_t rank = (uint32_t)__popcll(idle & ((1ull << lane) - 1));
        const uint32_t my = base + rank;
        if (!busy && rank < take) {
          const uint32_t k = read_kind ? sld(wp.in.kind + my) : (uint32_t)RAY_MAIN;
          // a parked entry is not traced: its hit record (copied by k_shade) stays for the retry
          // (RL: the ray is read once, here, so it is a streamed load; otherwise primitive
          // steps read it again)
          RayOD r;
          if constexpr (RL) {
            r = sld(wp.in.ray + my);
            const double2* rp = reinterpret_cast<const double2*>(&r);
            const double2 r0 = rp[0], r1 = rp[1], r2 = rp[2];
            ray_lds[3 * threadIdx.x] = r0; ray_lds[3 * threadIdx.x + 1] = r1; ray_lds[3 * threadIdx.x + 2] = r2;
          } else {
            r = wp.in.ray[my];
          }
          if (!(k & (RAY_PARKED | RAY_DEAD)) && (uint64_t)__double_as_longlong(r.o[0]) != DEAD_BITS) {
            qi = my;
            lkind = k;
            tmax = ray_tmax(wp.in, my, k);
            main_ray = kind_of(k) == RAY_MAIN;
            ix = (float)(1.0 / r.d[0]); iy = (float)(1.0 / r.d[1]); iz = (float)(1.0 / r.d[2]);
            ox = (float)r.o[0]; oy = (float)r.o[1]; oz = (float)r.o[2];
            fast = sc.nan_free_bounds && ray_fast_ok(ox, oy, oz, ix, iy, iz);
            cur = sc.root;
            sp = 0; low = 0; clean_from = 0;
            in_prim = false;
            bprim = -1;
            busy = cur != -1;
            if (!busy) {
              if ((UVL || UVS) && wp.hit_uv) {  // (t, prim) and (u, v) interleaved: hs == 2
                double2* rec = wp.in.hit + ((size_t)my << 1);
                sst(rec, hit_pack(0.0, -1)); sst(rec + 1, make_double2(0.0, 0.0));
              } else {
                sst(wp.in.hit + my, hit_pack(0.0, -1));
              }
            }
          }
        }
        c_rays += (uint64_t)__popcll(__ballot(main_ray));
        // drain the new rays' loads here: left pending they make the compiler wait for
        // vmcnt(0) at the loop head, i.e. for every hit-record store, on every iteration
        __builtin_amdgcn_s_waitcnt(0x0F70);
      } else if (exhausted && idle == ~0ull) {
        break;
      }
    }
    const uint64_t m_prim = __ballot(busy && in_prim);
    const uint64_t m_node = __ballot(busy && !in_prim);
    if ((m_prim | m_node) == 0) continue;
    const uint32_t n_prim = (uint32_t)__popcll(m_prim), n_node = (uint32_t)__popcll(m_node);
    bool advance = false;   // lane finished its current node / leaf: take next or pop
    bool leaf_next = false; // the step went straight into a leaf whose re-test is known to pass
    int32_t next = -1;
#ifdef IZPI_TRACE_CLOCKS
    IZPI_CLK(k1); k_refill += k1 - k0; k0 = k1;
    const bool clk_prim = n_prim * prim_w >= n_node * 16u;
#endif
    if (n_prim * prim_w >= n_node * 16u) {
      if constexpr (DIST) {
        // ---- distributed primitive step: every pending test of the PRIM lanes' leaves
        // (up to 64) runs on its own lane, then each owner accepts its leaf's results in
        // primitive order against its running tMax (bvh4.go:123-134, triangle.go:219)
        const uint32_t cnt = (busy && in_prim) ? (uint32_t)(pend - pk) : 0u;  // 1..4
        const uint64_t lt = (1ull << lane) - 1;
        const uint32_t base = (uint32_t)__popcll(__ballot(cnt & 1u) & lt) + 2u * (uint32_t)__popcll(__ballot(cnt & 2u) & lt) +
                              4u * (uint32_t)__popcll(__ballot(cnt & 4u) & lt);
        const bool served = cnt > 0 && base + cnt <= 64;
        const uint64_t ms = __ballot(served);
        const int last = 63 - __clzll((long long)ms);
        const uint32_t total = (uint32_t)__shfl((int)(base + cnt), last);
        {  // a leaf has 1..4 primitives (bvh4.go:638): four predicated writes, no loop
          const uint32_t e = ((uint32_t)pk << 6) | lane;
          uint32_t* dq = dist_owner + wbase + base;
          if (served) dq[0] = e;
          if (served && cnt > 1) dq[1] = e + 64u;
          if (served && cnt > 2) dq[2] = e + 128u;
          if (served && cnt > 3) dq[3] = e + 192u;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t ent = lane < total ? dist_owner[wbase + lane] : lane;
        const uint32_t ow = ent & 63u;
        const uint32_t oqi = (uint32_t)__shfl((int)qi, (int)ow);
        const uint32_t okind = (uint32_t)__shfl((int)lkind, (int)ow);
        if (lane < total) {
          const int32_t pi = (int32_t)(ent >> 6);
          double2 r0, r1, r2;
          if constexpr (RL) {
            const uint32_t ro = 3 * (wbase + ow);
            r0 = ray_lds[ro]; r1 = ray_lds[ro + 1]; r2 = ray_lds[ro + 2];
          } else {
            const double2* rp = reinterpret_cast<const double2*>(wp.in.ray + oqi);
            r0 = rp[0]; r1 = rp[1]; r2 = rp[2];
          }
          const double otmin = ray_tmin(wp.in, oqi, okind);
          double2 p0, p1, p2, p3, p4;
          if constexpr (LB) {
            LD2* pp = l_prims + (size_t)5 * pi;
            const v2d a0 = pp[0], a1 = pp[1], a2 = pp[2], a3 = pp[3], a4 = pp[4];
            p0 = make_double2(a0.x, a0.y); p1 = make_double2(a1.x, a1.y); p2 = make_double2(a2.x, a2.y);
            p3 = make_double2(a3.x, a3.y); p4 = make_double2(a4.x, a4.y);
          } else {
            const double2* pp = reinterpret_cast<const double2*>(sc.prims + pi);
            p0 = pp[0]; p1 = pp[1]; p2 = pp[2]; p3 = pp[3]; p4 = pp[4];
#ifdef IZPI_SHADOW
            if (IZPI_SHADOW & 4) {
              const uint4* sq = reinterpret_cast<const uint4*>(sc.sh_prims + pi);
              const uint4 s0 = sq[0], s1 = sq[1], s2 = sq[2], s3 = sq[3], s4 = sq[4];
              sh_acc ^= s0.x ^ s1.y ^ s2.z ^ s3.w ^ s4.x;
            }
#endif
          }
          const double pa[9] = {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y, p4.x};
          double t = 0, u = 0, v = 0;
          const V3 o = mk(r0.x, r0.y, r1.x), d = mk(r1.y, r2.x, r2.y);
          uint32_t flags;
          if (TRI || (uint32_t)__double2loint(p4.y) == IZPI_PRIM_TRIANGLE) {
            flags = tri_intersect_no_tmax(pa, o, d, otmin, t, u, v) ? 1u : 0u;
          } else {
            // sphere: both roots now, their tMin tests as flags; tMax is applied in order
            // by the owner (sphere.go:72-92: root 0 if tMin < t0 < tMax, else root 1)
            // (a scene whose spheres do not move: center(time) == center(time0), no load)
            // (the BVH-in-LDS ray instance runs only on such scenes: make_tracer)
            const double time = (RL && LB) || sc.time_free ? pa[7] : (wp.in.time ? wp.in.time[oqi] : 0.0);
            flags = 2u;
            if (sph_roots(sph_center(pa, time), pa[6], o, d, t, u))
              flags |= 1u | (t > otmin ? 4u : 0u) | (u > otmin ? 8u : 0u);
          }
          dist_t[wbase + lane] = t;
          if constexpr (DUV) { dist_u[wbase + lane] = u; dist_v[wbase + lane] = v; }
          dist_owner[wbase + lane] = flags;
        }
        const uint32_t n_sph_tests = TRI ? 0u : (uint32_t)__popcll(__ballot(lane < total && (dist_owner[wbase + lane] & 2u)));
        __builtin_amdgcn_wave_barrier();
        if (served && (TRI || n_sph_tests == 0)) {
          // triangles only: the leaf's flags and distances come in one LDS round trip, the
          // ordered accept runs in registers, and only the accepted (u, v) is read back
          const uint32_t j0 = wbase + base;
          uint32_t f[4];
          double tt[4];
#pragma unroll
          for (uint32_t i = 0; i < 4; i++) { f[i] = dist_owner[j0 + i]; tt[i] = dist_t[j0 + i]; }
          int32_t acc = -1;
#pragma unroll
          for (uint32_t i = 0; i < 4; i++)  // reject only `t > tMax` (triangle.go:219), in primitive order
            if (i < cnt && (f[i] & 1u) && !(tt[i] > tmax)) { tmax = tt[i]; acc = (int32_t)i; }
          if (acc >= 0) {
            if constexpr (UVL) lds_uv[threadIdx.x] = make_double2(dist_u[j0 + acc], dist_v[j0 + acc]);
            if constexpr (UVS)
              if (wp.hit_uv) sst(wp.in.hit + ((size_t)qi << 1) + 1, make_double2(dist_u[j0 + acc], dist_v[j0 + acc]));
            bprim = pk + acc;
            clean_from = sp;
          }
          pk = pend;
          in_prim = false;
          advance = true;
        } else if (!TRI && served) {
          int32_t acc = -1;
          double acc_u = 0, acc_v = 0;
          for (uint32_t i = 0; i < cnt; i++) {
            const uint32_t j = wbase + base + i;
            const uint32_t f = dist_owner[j];
            if (!(f & 1u)) continue;
            if (!(f & 2u)) {  // triangle: reject only `t > tMax` (triangle.go:219)
              const double t = dist_t[j];
              if (!(t > tmax)) { tmax = t; acc = (int32_t)j; acc_u = dist_u[j]; acc_v = dist_v[j]; bprim = pk + (int32_t)i; }
            } else {  // sphere: strict bounds, root 0 first
              const double ta = dist_t[j], tb = dist_u[j];
              if (ta < tmax && (f & 4u)) { tmax = ta; acc = (int32_t)j; acc_u = 0.0; acc_v = 0.0; bprim = pk + (int32_t)i; }
              else if (tb < tmax && (f & 8u)) { tmax = tb; acc = (int32_t)j; acc_u = 1.0; acc_v = 0.0; bprim = pk + (int32_t)i; }
            }
          }
          if (acc >= 0) {
            if constexpr (UVS) {
              if (wp.hit_uv) sst(wp.in.hit + ((size_t)qi << 1) + 1, make_double2(acc_u, acc_v));
            } else {
              lds_uv[threadIdx.x] = make_double2(acc_u, acc_v);
            }
            clean_from = sp;
          }
          pk = pend;
          in_prim = false;
          advance = true;
        }
        __builtin_amdgcn_wave_barrier();
        c_tri += total - n_sph_tests;
        c_sph += n_sph_tests;
        c_pstep++;
      } else {
      // ---- primitive step: one Hit() per PRIM lane (bvh4.go:123-134)
      bool is_tri = false;
      if (busy && in_prim) {
        // the f64 ray is re-read here (L2) instead of living in 14 VGPRs across node steps
        // (measured: keeping it in LDS instead makes k_shade's later read of the same
        // record miss and costs more than it saves)
        const double2* rp = reinterpret_cast<const double2*>(wp.in.ray + qi);
        const double2 r0 = rp[0], r1 = rp[1], r2 = rp[2];
        const V3 o = mk(r0.x, r0.y, r1.x), d = mk(r1.y, r2.x, r2.y);
        const double tmin = ray_tmin(wp.in, qi, lkind);
        const double2* pp = reinterpret_cast<const double2*>(sc.prims + pk);
        const double2 p0 = pp[0], p1 = pp[1], p2 = pp[2], p3 = pp[3], p4 = pp[4];
        const double pa[9] = {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y, p4.x};
        is_tri = TRI || (uint32_t)__double2loint(p4.y) == IZPI_PRIM_TRIANGLE;
        if (is_tri) {
          double t, u, v;
          if (tri_intersect(pa, o, d, tmin, tmax, t, u, v)) {  // barycentrics wait in LDS (lds_uv)
            tmax = t; bprim = pk; lds_uv[threadIdx.x] = make_double2(u, v); clean_from = sp;
          }
        } else if (!TRI) {
          const double time = wp.in.time ? wp.in.time[qi] : 0.0;  // only spheres read the ray time
          double t; int root;
          if (sph_intersect(pa, o, d, time, tmin, tmax, t, root)) {
            tmax = t; bprim = pk; lds_uv[threadIdx.x] = make_double2((double)root, 0.0); clean_from = sp;
          }
        }
        pk++;
        if (pk == pend) { in_prim = false; advance = true; }
      }
      const uint32_t n_tri = (uint32_t)__popcll(__ballot(is_tri));
      c_tri += n_tri;
      c_sph += n_prim - n_tri;
      c_pstep++;
      }
    } else {
      c_nodes += n_node;
      c_nstep++;
      // ---- node step: visit `cur` (bvh4.go:87-146)
      const bool wave_fast = __ballot(busy && !in_prim && !fast) == 0;
      if (__ballot(busy && !in_prim && sp + 3 - low > S) != 0) {
        // ring too full for this step's three writes: spill the oldest entries (rare)
        if (busy && !in_prim) {
          while (sp + 3 - low > S) {
            gsp[(size_t)low * spill_stride] = stk[(low & (S - 1)) * 256];
            low++;
#ifdef IZPI_SHADOW
            c_spill_st++;
#endif
          }
        }
      }
      if (busy && !in_prim) {
        const float tm = (float)tmax;
        // An inner node (4-slot box test) and a leaf's slot-0 re-test (A10) run as ONE
        // code path: a leaf lane's 32-B GLeaf box lands in slot 0 (selects below), its
        // slots 1-3 are invalid. Mixed waves (nearly every node step) then issue one set
        // of loads and wait once, instead of running the two branches one after the other.
        const bool is_leaf = ref_is_leaf(cur);
        float4 q0, q1, mnz_, mxx_, mxy_, mxz_;
        int4 ch_;
        if constexpr (LB) {
          LF4* lp = is_leaf ? l_leaves + (size_t)2 * leaf_start(cur) : l_inner + (size_t)8 * cur;
          LF4* np = is_leaf ? l_inner : lp;
          const v4f a0 = lp[0], a1 = lp[1], a2 = np[2], a3 = np[3], a4 = np[4], a5 = np[5], c = np[6];
          q0 = make_float4(a0.x, a0.y, a0.z, a0.w); q1 = make_float4(a1.x, a1.y, a1.z, a1.w);
          mnz_ = make_float4(a2.x, a2.y, a2.z, a2.w); mxx_ = make_float4(a3.x, a3.y, a3.z, a3.w);
          mxy_ = make_float4(a4.x, a4.y, a4.z, a4.w); mxz_ = make_float4(a5.x, a5.y, a5.z, a5.w);
          ch_ = make_int4(__float_as_int(c.x), __float_as_int(c.y), __float_as_int(c.z), __float_as_int(c.w));
        } else {
          const float4* lp = reinterpret_cast<const float4*>(is_leaf ? (const void*)(sc.leaves + leaf_start(cur))
                                                                     : (const void*)(sc.inner + cur));
          // leaf lanes read their last five loads from the root node (a cached valid address;
          // the values are not used)
          const float4* np = is_leaf ? reinterpret_cast<const float4*>(sc.inner) : lp;
          q0 = lp[0]; q1 = lp[1];
          mnz_ = np[2]; mxx_ = np[3]; mxy_ = np[4]; mxz_ = np[5];
          ch_ = *reinterpret_cast<const int4*>(np + 6);
#ifdef IZPI_SHADOW
          if ((IZPI_SHADOW & 1) && !is_leaf) {
            const uint4* sq = reinterpret_cast<const uint4*>(sc.sh_inner + cur);
            const uint4 s0 = sq[0], s1 = sq[1], s2 = sq[2], s3 = sq[3], s4 = sq[4], s5 = sq[5], s6 = sq[6];
            sh_acc ^= s0.x ^ s1.y ^ s2.z ^ s3.w ^ s4.x ^ s5.y ^ s6.z;
          }
          if ((IZPI_SHADOW & 2) && is_leaf) {
            const uint4* sq = reinterpret_cast<const uint4*>(sc.sh_leaves + leaf_start(cur));
            const uint4 s0 = sq[0], s1 = sq[1];
            sh_acc ^= s0.x ^ s1.y;
          }
#endif
        }
        // GLeaf = (mn.x, mn.y, mn.z, mx.x), (mx.y, mx.z, start, count)
        const float4 mnx = q0;
        const float4 mny = make_float4(is_leaf ? q0.y : q1.x, q1.y, q1.z, q1.w);
        const float4 mnz = make_float4(is_leaf ? q0.z : mnz_.x, mnz_.y, mnz_.z, mnz_.w);
        const float4 mxx = make_float4(is_leaf ? q0.w : mxx_.x, mxx_.y, mxx_.z, mxx_.w);
        const float4 mxy = make_float4(is_leaf ? q1.x : mxy_.x, mxy_.y, mxy_.z, mxy_.w);
        const float4 mxz = make_float4(is_leaf ? q1.y : mxz_.x, mxz_.y, mxz_.z, mxz_.w);
        const int4 ch = make_int4(is_leaf ? cur : ch_.x, ch_.y, ch_.z, ch_.w);
        uint32_t hm;
        if (wave_fast) {
          hm = slab4_fast(mnx, mny, mnz, mxx, mxy, mxz, ox, oy, oz, ix, iy, iz, tm);
        } else {
          const float amnx[4] = {mnx.x, mnx.y, mnx.z, mnx.w}, amny[4] = {mny.x, mny.y, mny.z, mny.w},
                      amnz[4] = {mnz.x, mnz.y, mnz.z, mnz.w}, amxx[4] = {mxx.x, mxx.y, mxx.z, mxx.w},
                      amxy[4] = {mxy.x, mxy.y, mxy.z, mxy.w}, amxz[4] = {mxz.x, mxz.y, mxz.z, mxz.w};
          hm = 0;
#pragma unroll
          for (int i = 0; i < 4; i++)
            if (slab(amnx[i], amny[i], amnz[i], amxx[i], amxy[i], amxz[i], ox, oy, oz, ix, iy, iz, tm)) hm |= 1u << i;
        }
        // slots 0..3 with ChildIndex != -1 whose box is hit (bvh4.go:119-146): the first
        // is visited next, the others are pushed in slot order (popped LIFO). Selects
        // instead of branches: each divergent branch costs exec-mask and lane-mask
        // bookkeeping on the scalar unit, which is as busy as the vector unit here.
        const uint32_t valid = is_leaf ? 1u
                                       : ((ch.x != -1 ? 1u : 0u) | (ch.y != -1 ? 2u : 0u) | (ch.z != -1 ? 4u : 0u) |
                                          (ch.w != -1 ? 8u : 0u));
        const uint32_t m = hm & valid;
        const int32_t c01 = (m & 1u) ? ch.x : ch.y, c23 = (m & 4u) ? ch.z : ch.w;
        next = m == 0 ? -1 : ((m & 3u) ? c01 : c23);
        // A passed leaf re-test starts on the leaf's primitives. A leaf visited straight
        // after its parent re-tests the same f32 box with the same tMax (A10): the result
        // is known to be a hit, so its node load is skipped too (the visit is still counted).
        const bool enter = ref_is_leaf(next) && (is_leaf || sc.leaf_shortcut);
        leaf_next = enter && !is_leaf;
        in_prim = enter;
        pk = enter ? leaf_start(next) : pk;
        pend = enter ? leaf_start(next) + leaf_count(next) : pend;
        next = enter ? -1 : next;
        // the other hit children, compacted in slot order, are written unconditionally to
        // ring positions sp..sp+2 (the ring keeps 3 free entries above sp); sp moves by
        // their count
        const uint32_t rest = m & (m - 1u);  // bits 1..3 only
        const int np_ = __builtin_popcount(rest);
        const int32_t e0 = (rest & 2u) ? ch.y : ((rest & 4u) ? ch.z : ch.w);
        const int32_t e1 = ((rest & 6u) == 6u) ? ch.z : ch.w;
        stk[(sp & (S - 1)) * 256] = e0;
        stk[((sp + 1) & (S - 1)) * 256] = e1;
        stk[((sp + 2) & (S - 1)) * 256] = ch.w;
        if (sp + np_ > 64) atomicOr(err, 1u);  // unreachable: the host rejects BVHs deeper than 64 entries
        sp += np_;
        advance = !enter;
      }
    }
#ifdef IZPI_TRACE_CLOCKS
    IZPI_CLK(k1); if (clk_prim) k_prim += k1 - k0; else k_node += k1 - k0; k0 = k1;
#endif
    // ---- advance: next child, else pop (bvh4.go:150-160), else the ray is done
    {
      const bool do_pop = advance && next == -1 && sp > 0;
      const bool do_fin = advance && next == -1 && sp == 0;
      // the LDS read is unconditional (and volatile, so that the compiler keeps it a ds_read:
      // a select of the LDS and spill addresses becomes a flat load, whose wait also
      // drains every store)
      const int spn = sp - 1;
      int32_t top = *(volatile __attribute__((address_space(3))) int32_t*)&lds_stack[threadIdx.x + (spn & (S - 1)) * 256];
      if (__ballot(do_pop && spn < low) != 0) {
        if (do_pop && spn < low) {
          top = gsp[(size_t)spn * spill_stride];
          low = spn;
#ifdef IZPI_SHADOW
          c_spill_ld++;
#endif
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) here, not for every pop
      }
      cur = (advance && next != -1) ? next : (do_pop ? top : cur);
      sp = do_pop ? spn : sp;
      // An entry pushed after the last accepted hit meets the same tMax it was pushed
      // with, so a leaf's re-test against its (identical) box passes: skip the load.
      const bool lf = do_pop && ref_is_leaf(top) && spn >= clean_from && sc.leaf_shortcut;
      in_prim = in_prim || lf;
      leaf_next = leaf_next || lf;
      pk = lf ? leaf_start(top) : pk;
      pend = lf ? leaf_start(top) + leaf_count(top) : pend;
      clean_from = (do_pop && spn < clean_from) ? spn : clean_from;
      if (do_fin) {
        const double2 uv = (UVL && bprim >= 0) ? lds_uv[threadIdx.x] : make_double2(0.0, 0.0);
        if ((UVL || UVS) && wp.hit_uv) {  // (t, prim) and (u, v) in one 32-B record (hs == 2)
          double2* rec = wp.in.hit + ((size_t)qi << 1);
          sst(rec, hit_pack(bprim >= 0 ? tmax : 0.0, bprim));
          if (!UVS || bprim < 0) sst(rec + 1, uv);  // (UVS: an accepted hit's (u, v) is there already)
        } else {  // nothing reads (u, v): 16 B per entry (hs == 1)
          sst(wp.in.hit + qi, hit_pack(bprim >= 0 ? tmax : 0.0, bprim));
        }
        busy = false;
      }
    }
    const uint64_t n_short = (uint64_t)__popcll(__ballot(leaf_next));  // leaf visits taken by a shortcut
    c_nodes += n_short;
    c_short += n_short;
#ifdef IZPI_TRACE_CLOCKS
    IZPI_CLK(k1); k_adv += k1 - k0;
#endif
  }
#ifdef IZPI_TRACE_CLOCKS
  if (lane == 0) {
    atomicAdd(counters + CNT_CLK_REFILL, (unsigned long long)k_refill);
    atomicAdd(counters + CNT_CLK_NODE, (unsigned long long)k_node);
    atomicAdd(counters + CNT_CLK_PRIM, (unsigned long long)k_prim);
    atomicAdd(counters + CNT_CLK_ADV, (unsigned long long)k_adv);
  }
#endif
#ifdef IZPI_SHADOW
  {
    if (c_spill_st) atomicAdd(counters + CNT_CLK_REFILL, (unsigned long long)c_spill_st);
    if (c_spill_ld) atomicAdd(counters + CNT_CLK_NODE, (unsigned long long)c_spill_ld);
    if (sh_acc == 0x9E3779B9u) atomicOr(err, 0u);
  }
#endif
  if (lane == 0) {
    count_add(wp.cpart, counters, CNT_RAYS, c_rays);
    count_add(wp.cpart, counters, CNT_NODES, c_nodes);
    count_add(wp.cpart, counters, CNT_TRI, c_tri);
    count_add(wp.cpart, counters, CNT_SPH, c_sph);
    count_add(wp.cpart, counters, CNT_NSTEP, c_nstep);
    count_add(wp.cpart, counters, CNT_PSTEP, c_pstep);
    count_add(wp.cpart, counters, CNT_SHORT, c_short);
  }
}

// Small scenes' per-primitive shading data staged in LDS by every k_shade / k_tail block
// (shade_stage, ShadeParams::prims_staged: at most PR_LDS primitives, as in C1, C2, C4, C5):
// the closest hit's GShade, its triangle UVs and tangent frame and a sphere's record are
// then LDS reads instead of a chain of dependent global loads (entry -> GShade -> UVs ->
// texels -> tangent frame).
IZPI_DEV GShade* gs_lds() { return (GShade*)(lds_arena() + lds_off::GS); }
IZPI_DEV GTriTex* tt_lds() { return (GTriTex*)(lds_arena() + lds_off::TT); }
IZPI_DEV GPrim* gp_lds() { return (GPrim*)(lds_arena() + lds_off::GP); }
IZPI_DEV GShade gshade_of(const DevScene& sc, bool pst, int32_t prim) {
  if (pst) return lds_ld(gs_lds() + prim);
  return sc.shade[prim];
}
// Full hit record of the closest primitive (triangle.go:223-264, sphere.go:71-92).
struct HitRec {
  double t, u, v;
  V3 p, n;
  uint32_t mat;
  bool nraw_ok;  // nraw holds the normal map's texel at (u, v), already read for a PBR triangle
  V3 nraw;
};
// `uvp` is the hit record, whose (u, v): read only for UV-textured triangles and for spheres.
// A normal map's texel nts at the hit of triangle `prim` (leaf order) applied to the
// geometric normal n through the triangle's tangent frame (triangle.go:250-264).
IZPI_DEV V3 nmap_tbn(const DevScene& sc, int32_t prim, V3 n, V3 nts, bool pst = false) {
  nts.x = 2 * nts.x - 1.0; nts.y = 2 * nts.y - 1.0; nts.z = 2 * nts.z - 1.0;
  V3 tg, bt;
  if (pst) {
    const __attribute__((address_space(3))) double* q = (const __attribute__((address_space(3))) double*)(tt_lds() + prim);
    constexpr uint32_t TG = offsetof(GTriTex, tg) / 8, BT = offsetof(GTriTex, bt) / 8;
    tg = mk(q[TG], q[TG + 1], q[TG + 2]);
    bt = mk(q[BT], q[BT + 1], q[BT + 2]);
  } else {
    const GTriTex& tt = sc.tritex[prim];
    tg = ld3(tt.tg); bt = ld3(tt.bt);
  }
  V3 nn = mk(tg.x * nts.x + bt.x * nts.y + n.x * nts.z, tg.y * nts.x + bt.y * nts.y + n.y * nts.z,
             tg.z * nts.x + bt.z * nts.y + n.z * nts.z);
  return sdiv(nn, length(nn));
}
// defer_nmap: a PBR triangle's normal map is left to the caller (h.n stays geometric), which
// looks the texel up together with the material's other three (one round of texel loads).
IZPI_DEV void hit_record(const DevScene& sc, const HitOut& c, const double2* uvp, const GShade& gs, V3 o, V3 d, double time,
                         bool want_uv, HitRec& h, bool mt_staged = false, bool defer_nmap = false, bool pst = false) {
  h.t = c.t;
  h.p = add(o, smul(d, c.t));
  h.mat = gs_mat(gs);
  h.nraw_ok = false;
  if (IZPI_PRIM_KIND(gs.ref) == IZPI_PRIM_TRIANGLE) {
    V3 n = mk(gs.n[0], gs.n[1], gs.n[2]);
    h.u = 0; h.v = 0;
    if (want_uv && sc.tritex) {  // (u,v) are read only by image textures
      const double eps = 1e-8;
      // (the host keeps huv for every scene that can get here: need_uv = !tri_only || any_uv;
      // a null record reads as (0, 0) rather than faulting)
      const double2 huv = uvp ? *uvp : make_double2(0.0, 0.0);
      double u = huv.x, v = huv.y;
      double w = 1.0 - u - v;
      double sum = u + v + w;
      if (gm::abs(sum - 1.0) > eps) { u /= sum; v /= sum; w /= sum; }
      double uv[6];  // u0,v0,u1,v1,u2,v2
      if (pst) {
        const __attribute__((address_space(3))) double* q = (const __attribute__((address_space(3))) double*)(tt_lds() + c.prim);
        for (int k = 0; k < 6; k++) uv[k] = q[k];
      } else {
        for (int k = 0; k < 6; k++) uv[k] = sc.tritex[c.prim].uv[k];
      }
      h.u = w * uv[0] + u * uv[2] + v * uv[4];
      h.v = w * uv[1] + u * uv[3] + v * uv[5];
    }
    if (gs_kind(gs) == IZPI_MAT_PBR && !defer_nmap) {
      const TexSlot ns = mat_slot(sc, mt_staged, h.mat, 1);
      if (slot_set(ns)) {  // Material.NormalMap() != nil (triangle.go:250-264), constant maps too
        const V3 nts = slot_rgb(sc, ns, h.u, h.v, mt_staged);
        h.nraw = nts;  // PBR.Scatter reads the same texel again (pbr.go:65-91)
        h.nraw_ok = true;
        n = nmap_tbn(sc, c.prim, n, nts, pst);
      }
    }
    h.n = n;
  } else {
    double pa[9];
    if (pst) {
      const __attribute__((address_space(3))) double* q = (const __attribute__((address_space(3))) double*)(gp_lds() + c.prim);
      for (int k = 0; k < 9; k++) pa[k] = q[k];
    } else {
      const GPrim& pr = sc.prims[c.prim];
      for (int k = 0; k < 9; k++) pa[k] = pr.a[k];
    }
    V3 ctr = sph_center(pa, time);
    V3 on = sdiv(sub(h.p, ctr), pa[6]);
    V3 flipped = dot(d, on) >= 0 ? smul(on, -1) : on;
    h.n = (uvp ? uvp->x : 0.0) == 0.0 ? flipped : on;  // second root keeps the unflipped normal (A16)
    if (want_uv) {
      double phi = gm::atan2(flipped.z, flipped.x);
      double theta = gm::asin(flipped.y);
      h.u = 1.0 - (phi + 3.141592653589793) / (2.0 * 3.141592653589793);
      h.v = (theta + 3.141592653589793 / 2.0) / 3.141592653589793;
    } else {
      h.u = 0; h.v = 0;  // no texture of this material reads (u,v)
    }
  }
}

// ================================================================ lights
// HitableSlice.PDFValue over Scene.Lights (hitable_slice.go:98-105) with
// Triangle.PDFValue (triangle.go:271-280) / Sphere.PDFValue (sphere.go:129-137).
// What PDFValue reads of light i, 16 doubles: a triangle's v0, e1, e2, n, area; a
// sphere's center(0), radius, c0; [15] = kind. Staged in LDS by k_shade / k_tail (lt_lds,
// at most LT_LDS lights): the light loop then reads LDS broadcasts instead of one
// dependent global load per light (the compiler cannot use scalar loads for the GLight
// records, which it cannot prove unwritten).
IZPI_DEV double* lt_lds() { return (double*)(lds_arena() + lds_off::LT); }
IZPI_DEV void light_pack(const GLight& L, uint32_t k, double* out) {  // k = 0..15
  double v = 0;
  if (L.kind == IZPI_PRIM_TRIANGLE) {
    v = k < 3 ? L.v0[k] : k < 6 ? L.e1[k - 3] : k < 9 ? L.e2[k - 6] : k < 12 ? L.n[k - 9] : k == 12 ? L.area : 0.0;
  } else {
    v = k < 3 ? L.cz[k] : k == 3 ? L.radius : k < 7 ? L.c0[k - 4] : 0.0;
  }
  if (k == 15) v = (double)L.kind;
  out[k] = v;
}
// HitableSlice.PDFValue over Scene.Lights (hitable_slice.go:98-105) from the packed
// records (LDS when staged, else packed the same way on the fly from the GLight records).
IZPI_DEV double lights_pdf(const DevScene& sc, bool staged, V3 o, V3 v, uint32_t& c_lt, uint32_t& c_ls) {
  const double weight = 1.0 / (double)sc.num_lights;
  double sum = 0;
  for (uint32_t i = 0; i < sc.num_lights; i++) {
    double r[16];
    if (staged) {
#pragma unroll
      for (int k = 0; k < 16; k++) r[k] = lds_ld(lt_lds() + i * 16 + k);
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) light_pack(sc.lights[i], k, r);
    }
    double pdf = 0;
    if (r[15] == (double)IZPI_PRIM_TRIANGLE) {
      c_lt++;
      double t, u, w;
      if (tri_intersect(r, o, v, 0.001, 1.7976931348623157e308, t, u, w)) {  // r[0..8] = v0, e1, e2
        double dist2 = t * t * sqlen(v);
        double cosine = gm::abs(dot(v, sdiv(mk(r[9], r[10], r[11]), length(v))));
        pdf = dist2 / (cosine * r[12]);
      }
    } else {
      c_ls++;
      double t; int root;
      const double radius = r[3];
      if (sph_intersect_at(mk(r[0], r[1], r[2]), radius, o, v, 0.001, 1.7976931348623157e308, t, root)) {
        double cosThetaMax = gm::sqrt(1 - radius * radius / sqlen(sub(mk(r[4], r[5], r[6]), o)));
        double solidAngle = 6.283185307179586 * (1 - cosThetaMax);
        pdf = 1 / solidAngle;
      }
    }
    sum += weight * pdf;
  }
  return sum;
}
// What Triangle.Random reads beyond the PDFValue record: v1 and v2 (6 doubles per light,
// staged next to lt_lds), so a light sample is an LDS read instead of a dependent load.
IZPI_DEV double* lt2_lds() { return (double*)(lds_arena() + lds_off::LT2); }
// HitableSlice.Random (hitable_slice.go:107-110) + Triangle/Sphere.Random
IZPI_DEV V3 lights_random(const DevScene& sc, bool staged, V3 o, Lcg& rng) {
  int64_t index = go_int(rng.next() * (double)sc.num_lights);
  if (staged) {
    const double* r = lt_lds() + index * 16;
    if (lds_ld(r + 15) == (double)IZPI_PRIM_TRIANGLE) {
      const double* q = lt2_lds() + index * 6;
      const V3 v0 = mk(lds_ld(r), lds_ld(r + 1), lds_ld(r + 2));
      const V3 v1 = mk(lds_ld(q), lds_ld(q + 1), lds_ld(q + 2)), v2 = mk(lds_ld(q + 3), lds_ld(q + 4), lds_ld(q + 5));
      double t1 = rng.next();
      V3 p01 = lerp(v0, v1, t1);
      double t2 = rng.next();
      V3 p02 = lerp(v0, v2, t2);
      double t3 = rng.next();
      return sub(lerp(p01, p02, t3), o);
    }
    V3 dir = sub(mk(lds_ld(r + 4), lds_ld(r + 5), lds_ld(r + 6)), o);  // c0
    double dist2 = sqlen(dir);
    Onb uvw;
    uvw.build(dir);
    return uvw.local(random_to_sphere(lds_ld(r + 3), dist2, rng));
  }
  const GLight& L = sc.lights[index];
  if (L.kind == IZPI_PRIM_TRIANGLE) {
    double t1 = rng.next();
    V3 p01 = lerp(ld3(L.v0), ld3(L.v1), t1);
    double t2 = rng.next();
    V3 p02 = lerp(ld3(L.v0), ld3(L.v2), t2);
    double t3 = rng.next();
    return sub(lerp(p01, p02, t3), o);
  }
  V3 dir = sub(ld3(L.c0), o);
  double dist2 = sqlen(dir);
  Onb uvw;
  uvw.build(dir);
  return uvw.local(random_to_sphere(L.radius, dist2, rng));
}

// ============================================================== materials
IZPI_DEV V3 reflect(V3 v, V3 n) { return sub(v, smul(n, 2 * dot(v, n))); }
IZPI_DEV bool refract(V3 v, V3 n, double ni, V3& out) {
  V3 uv = unit(v);
  double dt = dot(uv, n);
  double disc = 1.0 - ni * ni * (1 - dt * dt);
  if (disc > 0) {
    out = sub(smul(sub(uv, smul(n, dt)), ni), smul(n, gm::sqrt(disc)));
    return true;
  }
  return false;
}
IZPI_DEV double schlick(double cosine, double ri) {
  double r0 = (1.0 - ri) / (1.0 + ri);
  r0 = r0 * r0;
  return r0 + (1.0 - r0) * gm::pow((1.0 - cosine), 5);
}
// Dielectric.scatterCommon (dielectric.go:66-102): returns the scattered direction.
IZPI_DEV V3 dielectric_scatter(V3 d, V3 n, double ri, Lcg& rng, bool& reflected_out) {
  V3 reflected = reflect(d, n);
  V3 outward;
  double ni, cosine, prob;
  if (dot(d, n) > 0) {
    outward = smul(n, -1.0);
    ni = ri;
    cosine = ri * dot(d, n) / length(d);
  } else {
    outward = n;
    ni = 1.0 / ri;
    cosine = -dot(d, n) / length(d);
  }
  V3 refracted = mk(0, 0, 0);
  if (refract(d, outward, ni, refracted)) prob = schlick(cosine, ri);
  else prob = 1.0;
  if (rng.next() < prob) { reflected_out = true; return reflected; }
  reflected_out = false;
  return refracted;
}

// ============================================================ shading
struct ShadeParams {
  uint32_t width, height, max_depth;
  uint32_t chunk_spp, s0, tile_w, tile_h, total_units;
  uint32_t num_bg_spd, slots;
  uint32_t rec_dense;          // unwinding records per slot in the dense array (depths 0..rec_dense-1)
  uint32_t rec_pool;           // records per overflow block (depths rec_dense..max_depth-1); 0 = no pool
  uint32_t pool_shift;         // log2(overflow blocks per ring); ring r holds blocks [r << shift, (r + 1) << shift)
  uint32_t unit_base;          // k_start: slot i of this lane starts unit unit_base + i
  uint32_t bg_sorted;          // background SPD wavelengths non-decreasing (binary-search lookups)
  const uint32_t* tiles;
  const double* bg_wl;
  const double* bg_val;
  double background[3];
  uint64_t seed;
  double* out;                 // [total_units][3] per-sample result
  double* recs;                // [slots][rec_dense][D] unwinding records
  unsigned long long* finq;    // [k_shade block][FINQ_WORDS][FINQ_CAP] deferred unwinding jobs (fin_flush)
  double* pool;                // [blocks][rec_pool][D] overflow unwinding records
  const double4* mat_const;    // DevScene::mat_const (MATSET_CONST records)
  uint32_t num_mc, num_tex, num_spd;  // materials, textures, SPD table entries of the scene
  uint32_t staged;             // the scene's small tables are staged in LDS per block (shade_stage): 1 the Colour ones, 2 + the Spectral ones
  uint32_t prims_staged;       // so are its primitives' GShade / GTriTex / GPrim records (at most PR_LDS)
  uint32_t* pool_ring;         // [blocks] free block ids: POOL_SHARDS rings of 1 << pool_shift entries
  unsigned long long* pool_ctr;  // [POOL_SHARDS][POOL_CTR_STRIDE] ring counters (pool_publish)
  uint32_t* head;              // next work unit
  unsigned long long* counters;
  unsigned long long* cpart;   // per-wave counter rows (count_add), or null
  uint32_t* error;
};

// Unwinding records, one per bounce, laid out [slot][depth] so that a finishing path
// reads its records as one contiguous run (40 B per level for Colour: att xyz, s, p;
// 24 B for Spectral: att, s, p; a specular level marks s, see REC_SPEC_BITS). A
// [depth][field][slot] layout made every field
// of every level a separate scattered 64-B sector read (measured: 44% of C5 shading).
// Only the first rec_dense levels are stored per slot. Few paths go deeper (C3: ~3% of
// the paths in flight at depth >= 8), so the deeper levels live in overflow blocks of
// rec_pool levels, taken by a path when it reaches depth rec_dense and returned when it
// finishes: the state of 40M slots at maxDepth 50 takes ~20 GB instead of ~100 GB.
// MATSET selects the compiled material code: MATSET_BASIC covers Lambertian +
// DiffuseLight only (the Cornell/dragon configs) and keeps the kernel's register
// footprint small; MATSET_CONST is MATSET_BASIC for scenes whose albedos are all
// constant RGB textures (Colour sampler): a bounce's attenuation is then its material's
// constant, so its unwinding record holds the material instead of the colour (24 B
// instead of 40 B); MATSET_SURF adds Metal and PBR, MATSET_FULL Dielectric and Isotropic
// too. The host picks the variant from the scene's materials (results are identical).
// A MATSET is a set of feature bits: only the material branches it holds are compiled in.
// The host runs the smallest instance holding the scene's material kinds: MATSET_SURF for
// Metal/PBR scenes (C4: shading -2% against MATSET_FULL). A Lambert/light/dielectric
// instance measured 3% SLOWER than MATSET_FULL on C5 (its register allocation came out
// worse), so dielectric scenes run MATSET_FULL.
enum { MS_DIEL = 1, MS_METAL = 2, MS_PBR = 4, MS_ISO = 8, MS_CONST = 16 };
enum {
  MATSET_BASIC = 0,
  MATSET_SURF = MS_METAL | MS_PBR,
  MATSET_FULL = MS_DIEL | MS_METAL | MS_PBR | MS_ISO,
  MATSET_CONST = MS_CONST
};
constexpr bool ms_has(int matset, int feature) { return (matset & feature) != 0; }
// specular bounces (records without a pdf) can occur
constexpr bool ms_spec(int matset) { return (matset & (MS_DIEL | MS_METAL | MS_PBR)) != 0; }
// Record: Colour (flag, att xyz, s, p); Colour + MATSET_CONST (material, s, p); Spectral
// (flag, att, s, p). p is always last.
constexpr uint32_t SMP_D = 3;  // doubles per per-sample result (padding them to 32 B measured no better: DESIGN 3.2)
template <int SAMPLER, int MATSET>
struct RecLayout {
  static constexpr bool COMPACT = SAMPLER == IZPI_SAMPLER_COLOUR && MATSET == MATSET_CONST;
  static constexpr bool THREE = COMPACT || SAMPLER != IZPI_SAMPLER_COLOUR;             // (material or att, s, p)
  static constexpr uint32_t D = THREE ? 3 : 5;                          // doubles per record
  static constexpr uint32_t P = THREE ? 2 : 4;                                         // index of p
  static constexpr uint32_t S = THREE ? 1 : 3;                                         // index of s
};
// Records are (att, s, p): att xyz for Colour, att for Spectral. A specular bounce has no
// s or p and stores s = REC_SPEC_BITS, a signalling-NaN pattern: ScatteringPDF's
// arithmetic only ever makes quiet NaNs, so no non-specular record carries it.
constexpr uint64_t REC_SPEC_BITS = 0x7FF4C0DEC0DEC0DEull;
template <int SAMPLER, int MATSET>
IZPI_DEV double* rec_ptr(const ShadeParams& sp, uint32_t rslot, uint32_t blk, uint32_t depth) {
  constexpr uint32_t D = RecLayout<SAMPLER, MATSET>::D;
  if (depth < sp.rec_dense) return sp.recs + ((size_t)rslot * sp.rec_dense + depth) * D;
  return sp.pool + ((size_t)(blk - 1) * sp.rec_pool + (depth - sp.rec_dense)) * D;
}
// A bounce's record without p (written once the light pdf is known).
template <int SAMPLER, int MATSET>
IZPI_DEV void rec_store(const ShadeParams& sp, uint32_t rslot, uint32_t blk, uint32_t depth, bool spec, V3 att, double s,
                        uint32_t mat) {
  double* rp = rec_ptr<SAMPLER, MATSET>(sp, rslot, blk, depth);
  if constexpr (RecLayout<SAMPLER, MATSET>::COMPACT) {  // never specular
    if constexpr (RecLayout<SAMPLER, MATSET>::D == 4) {  // 32-B records: (material, s) in one 16-B store
      sst(reinterpret_cast<double2*>(rp), make_double2((double)mat, s));
    } else {
      sst(rp, (double)mat);
      sst(rp + 1, s);
    }
    return;
  }
  const double sv = spec ? __longlong_as_double((long long)REC_SPEC_BITS) : s;
  sst(rp, att.x);
  if (SAMPLER == IZPI_SAMPLER_COLOUR) { sst(rp + 1, att.y); sst(rp + 2, att.z); }
  sst(rp + RecLayout<SAMPLER, MATSET>::S, sv);
}
IZPI_DEV bool rec_is_spec(double s) { return (uint64_t)__double_as_longlong(s) == REC_SPEC_BITS; }
// Update P.zf (ZF_*) for the record of the level being written: attenuation att (colour
// xyz, spectral x), and for a non-specular level its scattering pdf s and pdf p.
template <int SAMPLER>
IZPI_DEV void rec_zero_track(uint32_t& zf, bool spec, V3 att, double s, double p) {
  const bool colour = SAMPLER == IZPI_SAMPLER_COLOUR;
  bool ok = isfinite(att.x) && (!colour || (isfinite(att.y) && isfinite(att.z)));
  if (!spec) ok = ok && isfinite(s) && p != 0.0 && !isnan(p);
  if (!ok) zf |= ZF_UNSAFE;
  if (zf & ZF_RESET) return;
  if (spec) {
    zf ^= (signbit(att.x) ? 1u : 0u) << ZF_SIGN_SHIFT;
    if (colour) zf ^= ((signbit(att.y) ? 2u : 0u) | (signbit(att.z) ? 4u : 0u)) << ZF_SIGN_SHIFT;
  } else {
    zf |= ZF_RESET;
  }
}

// The materials' constant RGB values (DevScene::mat_const) and texture slots (mt_lds)
// staged in LDS by k_shade and k_tail when there are at most MC_LDS materials: the compact
// records' unwinding (finish) and constant-albedo hits read them with an LDS read instead
// of a dependent L2 load.
constexpr uint32_t MC_LDS = MT_LDS;
IZPI_DEV double4* mc_lds() { return (double4*)(lds_arena() + lds_off::MC); }
// Copy the scene's small tables into this block's LDS (ShadeParams::staged): the
// materials' constant colours and texture slots, the lights' PDFValue records, the
// material and texture records, the tabulated SPDs, the background SPD, the CIE tables.
IZPI_DEV void shade_stage(const DevScene& sc, const ShadeParams& sp) {
  if (sp.staged) {
    const uint32_t t0 = threadIdx.x, nt = blockDim.x;
    for (uint32_t t = t0; t < sp.num_mc; t += nt) mc_lds()[t] = sp.mat_const[t];
    for (uint32_t t = t0; t < 4 * sp.num_mc; t += nt) mt_lds()[t >> 2].s[t & 3] = sc.mat_tex[t >> 2].s[t & 3];
    for (uint32_t t = t0; t < 16 * sc.num_lights; t += nt) light_pack(sc.lights[t >> 4], t & 15, lt_lds() + (t & ~15u));
    for (uint32_t t = t0; t < 6 * sc.num_lights; t += nt) {
      const GLight& L = sc.lights[t / 6];
      const uint32_t k = t % 6;
      lt2_lds()[t] = L.kind == IZPI_PRIM_TRIANGLE ? (k < 3 ? L.v1[k] : L.v2[k - 3]) : 0.0;
    }
    constexpr uint32_t MW = sizeof(izpi_material) / 8, TW = sizeof(izpi_texture) / 8;
    for (uint32_t t = t0; t < MW * sp.num_mc; t += nt)
      reinterpret_cast<uint64_t*>(mat_lds())[t] = reinterpret_cast<const uint64_t*>(sc.materials)[t];
    for (uint32_t t = t0; t < TW * sp.num_tex; t += nt)
      reinterpret_cast<uint64_t*>(tex_lds())[t] = reinterpret_cast<const uint64_t*>(sc.textures)[t];
    if (sp.staged == 2) {  // the Spectral tables (the arena holds them: lds_arena_bytes)
      for (uint32_t t = t0; t < sp.num_spd; t += nt) { spd_lds()[t] = sc.spd_wl[t]; spdv_lds()[t] = sc.spd_val[t]; }
      for (uint32_t t = t0; t < sp.num_bg_spd; t += nt) { bg_lds()[t] = sp.bg_wl[t]; bgv_lds()[t] = sp.bg_val[t]; }
      for (uint32_t t = t0; t < IZPI_CIE_N; t += nt) {
        double* c = cie_lds();
        c[t] = c_cie_wl[t]; c[IZPI_CIE_N + t] = c_cie_x[t]; c[2 * IZPI_CIE_N + t] = c_cie_y[t];
        c[3 * IZPI_CIE_N + t] = c_cie_z[t]; c[4 * IZPI_CIE_N + t] = c_cie_ycum.v[t];
      }
    }
  }
  if (sp.prims_staged) {
    const uint32_t t0 = threadIdx.x, nt = blockDim.x, np = sc.num_prims;
    constexpr uint32_t SW = sizeof(GShade) / 8, TW = sizeof(GTriTex) / 8, PW = sizeof(GPrim) / 8;
    for (uint32_t t = t0; t < SW * np; t += nt)
      reinterpret_cast<uint64_t*>(gs_lds())[t] = reinterpret_cast<const uint64_t*>(sc.shade)[t];
    if (sc.tritex)
      for (uint32_t t = t0; t < TW * np; t += nt)
        reinterpret_cast<uint64_t*>(tt_lds())[t] = reinterpret_cast<const uint64_t*>(sc.tritex)[t];
    for (uint32_t t = t0; t < PW * np; t += nt)
      reinterpret_cast<uint64_t*>(gp_lds())[t] = reinterpret_cast<const uint64_t*>(sc.prims)[t];
  }
  __syncthreads();
}
IZPI_DEV double4 mat_const_of(const ShadeParams& sp, uint32_t m) {
  if (sp.staged) return lds_ld(&mc_lds()[m]);
  return sp.mat_const[m];
}

// Result slot of work unit `unit` (= pixel * chunk_spp + sample). Unit-major: paths of
// neighbouring units finish close in time and fill whole lines (a sample-major layout
// made k_accumulate coalesced but cost k_shade 16% in scattered partial-line stores).
IZPI_DEV double* sample_out(const ShadeParams& sp, uint32_t unit) { return sp.out + (size_t)unit * SMP_D; }

// Write the finished path's radiance after unwinding the recursion of
// colour.go:44-57 / sampler/spectral.go:60-72 from depth-1 down to 0.
template <int SAMPLER, int MATSET>
IZPI_DEV void finish(const ShadeParams& sp, const PathSt& P, V3 L) {
  constexpr bool NO_SPEC = !ms_spec(MATSET);
  if (SAMPLER == IZPI_SAMPLER_COLOUR && NO_SPEC && gm::bits(L.x) == 0 && gm::bits(L.y) == 0 && gm::bits(L.z) == 0) {
    // +0 radiance through only non-specular records: every level computes
    // 0.0 + (att*(0*s))/p, which is +0 or NaN, and DeNAN maps NaN to +0 (rgb.go:36),
    // so the result is +0 without reading the records
    double* out = sample_out(sp, P.unit);
    sst(out, 0.0); sst(out + 1, 0.0); sst(out + 2, 0.0);
    return;
  }
  // A terminal radiance of +0 through levels that all keep a zero a zero (P.zf): the
  // unwinding ends in a signed zero per component that zf already holds, so the records
  // need not be read (C5 / C4: paths escaping the box or ending at max depth into a black
  // background; the levels' arithmetic on +-0 is exact: see ZF_*)
  const bool zero_term = gm::bits(L.x) == 0 && (SAMPLER != IZPI_SAMPLER_COLOUR || (gm::bits(L.y) == 0 && gm::bits(L.z) == 0));
  const bool skip = zero_term && !(P.zf & ZF_UNSAFE);
  if (skip) {
    const uint32_t sg = P.zf >> ZF_SIGN_SHIFT;
    L = mk((sg & 1u) ? -0.0 : 0.0, (sg & 2u) ? -0.0 : 0.0, (sg & 4u) ? -0.0 : 0.0);
  }
  // The records are read four levels at a time (one batch of independent loads, then
  // the levels applied in order), so a path of depth d waits ~d/4 memory round trips.
  constexpr uint32_t D = RecLayout<SAMPLER, MATSET>::D;
  // levels per batch of record loads: 8 for the Spectral sampler's 24-B records (C5 shade
  // -2.2% against 4), 4 for Colour (8 made C3's compact records +13%: more live registers)
  constexpr int RB = SAMPLER == IZPI_SAMPLER_SPECTRAL ? 8 : 4;
  for (int dd = skip ? -1 : (int)P.depth - 1; dd >= 0; dd -= RB) {
    double rv[RB][D];
    if constexpr (RecLayout<SAMPLER, MATSET>::COMPACT) {
      // (material, s, p): the attenuation is the material's constant albedo
      double cv[RB][3];
#pragma unroll
      for (int j = 0; j < RB; j++) {
        if (dd - j >= 0) {
          const double* r = rec_ptr<SAMPLER, MATSET>(sp, P.rslot, P.blk, (uint32_t)(dd - j));
          if constexpr (D == 4) {  // 32-B records: two 16-B loads
            const double2 a = sld(reinterpret_cast<const double2*>(r)), b = sld(reinterpret_cast<const double2*>(r) + 1);
            rv[j][0] = a.x; rv[j][1] = a.y; rv[j][2] = b.x;
          } else {
            rv[j][0] = sld(r); rv[j][1] = sld(r + 1); rv[j][2] = sld(r + 2);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < RB; j++) {
        if (dd - j >= 0) {
          const double4 c = mat_const_of(sp, (uint32_t)rv[j][0]);
          cv[j][0] = c.x; cv[j][1] = c.y; cv[j][2] = c.z;
        }
      }
#pragma unroll
      for (int j = 0; j < RB; j++) {
        if (dd - j < 0) break;
        const V3 att = mk(cv[j][0], cv[j][1], cv[j][2]);
        V3 v1 = smul(L, rv[j][1]);                         // ScalarMul(Sample(...), ScatteringPDF)
        V3 v2 = mul(att, v1);
        V3 v3 = sdiv(v2, rv[j][2]);
        L = mk(0.0 + v3.x, 0.0 + v3.y, 0.0 + v3.z);        // Add(emitted == 0, v3)
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < RB; j++) {
      if (dd - j >= 0) {
        const double* rp = rec_ptr<SAMPLER, MATSET>(sp, P.rslot, P.blk, (uint32_t)(dd - j));
        if constexpr (D % 2 == 0) {
          const double2* r2 = reinterpret_cast<const double2*>(rp);
#pragma unroll
          for (uint32_t q = 0; q < D / 2; q++) { const double2 v = sld(r2 + q); rv[j][2 * q] = v.x; rv[j][2 * q + 1] = v.y; }
        } else {
#pragma unroll
          for (uint32_t q = 0; q < D; q++) rv[j][q] = sld(rp + q);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RB; j++) {
      if (dd - j < 0) break;
      const double* r = rv[j];
      if (SAMPLER == IZPI_SAMPLER_COLOUR) {
        V3 att = mk(r[0], r[1], r[2]);
        if (rec_is_spec(r[RecLayout<SAMPLER, MATSET>::S])) {
          L = mul(att, L);                                   // vec3.Mul(att, Sample(...))
        } else {
          const double s = r[RecLayout<SAMPLER, MATSET>::S], p = r[RecLayout<SAMPLER, MATSET>::P];
          V3 v1 = smul(L, s);                                // ScalarMul(Sample(...), ScatteringPDF)
          V3 v2 = mul(att, v1);
          V3 v3 = sdiv(v2, p);
          L = mk(0.0 + v3.x, 0.0 + v3.y, 0.0 + v3.z);        // Add(emitted == 0, v3)
        }
      } else {
        const double att = r[0];
        if (rec_is_spec(r[1])) {
          L.x = att * L.x;
        } else {
          const double s = r[1], p = r[2];
          double v1 = L.x * s;
          double v2 = att * v1;
          double v3 = v2 / p;
          L.x = 0.0 + v3;
        }
      }
    }
  }
  double* out = sample_out(sp, P.unit);
  if (SAMPLER == IZPI_SAMPLER_COLOUR) {
    V3 c = denan(L);  // rgb.go:36 DeNAN per sample
    sst(out, c.x); sst(out + 1, c.y); sst(out + 2, c.z);
  } else {
    double cx, cy, cz;  // render/spectral.go:162-166
    if (sp.staged) cie_values<true>(P.lambda, cx, cy, cz);
    else cie_values<false>(P.lambda, cx, cy, cz);
    const V3 o = sdiv(mk(L.x * cx, L.x * cy, L.x * cz), P.lpdf);  // three divisions by lpdf
    sst(out, o.x); sst(out + 1, o.y); sst(out + 2, o.z);
  }
}

// Whether finish(P, L) reads the path's records: not when it is at depth 0 or when its
// terminal radiance is a +0 that the levels keep a zero (finish's two shortcuts).
template <int SAMPLER, int MATSET>
IZPI_DEV bool finish_reads(const PathSt& P, V3 L) {
  const bool colour = SAMPLER == IZPI_SAMPLER_COLOUR;
  const bool zero_term = gm::bits(L.x) == 0 && (!colour || (gm::bits(L.y) == 0 && gm::bits(L.z) == 0));
  if (zero_term && ((colour && !ms_spec(MATSET)) || !(P.zf & ZF_UNSAFE))) return false;
  return P.depth > 0;
}

// IZPI_ACC_FORWARD: the finished path's sample is its throughput times the terminal
// radiance L (Colour: DeNAN per sample, rgb.go:36; Spectral: the XYZ weights of
// render/spectral.go:92-96), with no records to read.
template <int SAMPLER>
IZPI_DEV void finish_fwd(const ShadeParams& sp, const PathSt& P, V3 L) {
  double* out = sample_out(sp, P.unit);
  if (SAMPLER == IZPI_SAMPLER_COLOUR) {
    const V3 c = denan(mk(P.thr[0] * L.x, P.thr[1] * L.y, P.thr[2] * L.z));
    sst(out, c.x); sst(out + 1, c.y); sst(out + 2, c.z);
  } else {
    const double r = P.thr[0] * L.x;
    double cx, cy, cz;
    if (sp.staged) cie_values<true>(P.lambda, cx, cy, cz);
    else cie_values<false>(P.lambda, cx, cy, cz);
    const V3 o = sdiv(mk(r * cx, r * cy, r * cz), P.lpdf);
    sst(out, o.x); sst(out + 1, o.y); sst(out + 2, o.z);
  }
}

// The background SPD at lambda (sampler/spectral.go:48-51,79), staged or not
IZPI_DEV double bg_value(const ShadeParams& sp, double lambda) {
  if (sp.staged) return spd_value<true>(bg_lds(), bgv_lds(), sp.num_bg_spd, lambda, sp.bg_sorted != 0);
  return spd_value<false>(sp.bg_wl, sp.bg_val, sp.num_bg_spd, lambda, sp.bg_sorted != 0);
}
IZPI_DEV V3 terminal_max_depth(const ShadeParams& sp, const PathSt& P, bool colour) {
  // colour.go:34-36 returns blue; sampler/spectral.go:48-51 the background SPD.
  return colour ? mk(0, 0, 1.0) : mk(bg_value(sp, P.lambda), 0, 0);
}

// Start the path of work unit `unit`: per-sample LCG streams, wavelength (spectral),
// jitter, Camera.GetRay (camera.go:61-89). P.rslot (the record slot) is the caller's.
// Returns false when the sample is already complete (spectral pdf == 0 or maxDepth ==
// 0); its result is written.
template <int SAMPLER>
IZPI_DEV bool start_path(const DevScene& sc, const ShadeParams& sp, uint32_t unit, PathSt& P, RayRec& R) {
  const uint32_t pix_local = unit / sp.chunk_spp;
  const uint32_t s = sp.s0 + unit % sp.chunk_spp;
  const uint32_t tile_px = sp.tile_w * sp.tile_h;
  const uint32_t tile = pix_local / tile_px, in_tile = pix_local % tile_px;
  const uint32_t x = sp.tiles[4 * tile] + in_tile % sp.tile_w;
  const uint32_t y = sp.tiles[4 * tile + 1] + in_tile / sp.tile_w;
  const uint64_t key = ((uint64_t)s << 32) | (uint64_t)(y * sp.width + x);
  Lcg rng;
  rng.s = (uint32_t)splitmix64(sp.seed ^ key);
  Lcg cam;
  cam.s = (uint32_t)splitmix64(sp.seed ^ key ^ IZPI_CAMERA_STREAM_SALT);
  P.unit = unit;
  P.depth = 0;
  P.zf = 0;
  P.blk = 0;
  P.lambda = 0;
  P.lpdf = 1;
  P.thr[0] = 1.0; P.thr[1] = 1.0; P.thr[2] = 1.0;
  if (SAMPLER == IZPI_SAMPLER_SPECTRAL) {
    const double r = rng.next();
    if (sp.staged) sample_wavelength<true>(r, P.lambda, P.lpdf);
    else sample_wavelength<false>(r, P.lambda, P.lpdf);
    if (P.lpdf == 0) {  // render/spectral.go:78-80: skipped, still counted in 1/spp
      double* out = sample_out(sp, unit);
      sst(out, 0.0); sst(out + 1, 0.0); sst(out + 2, 0.0);
      return false;
    }
  }
  const double u = ((double)x + rng.next()) / (double)sp.width;
  const double v = ((double)y + rng.next()) / (double)sp.height;
  double px, py;
  for (;;) {  // randomInUnitDisc
    double rx = cam.next(), ry = cam.next();
    px = rx * 2.0 - 1.0;
    py = ry * 2.0 - 1.0;
    double pz = 0.0 * 2.0 - 0.0;
    if ((px * px) + (py * py) + (pz * pz) < 1.0) break;
  }
  const izpi_camera& c = sc.cam;
  const double rdx = px * c.lens_radius, rdy = py * c.lens_radius;
  V3 offset = add(smul(ld3(c.u), rdx), smul(ld3(c.v), rdy));
  const double time = c.time0 + cam.next() * (c.time1 - c.time0);
  V3 origin = ld3(c.origin);
  V3 ro = add(origin, offset);
  V3 rd = sub(sub(add(add(ld3(c.lower_left), smul(ld3(c.horizontal), u)), smul(ld3(c.vertical), v)), origin), offset);
  P.rng = rng.s;
  if (sp.max_depth == 0) {
    finish<SAMPLER, MATSET_FULL>(sp, P, terminal_max_depth(sp, P, SAMPLER == IZPI_SAMPLER_COLOUR));  // depth 0: reads no record
    return false;
  }
  R.o[0] = ro.x; R.o[1] = ro.y; R.o[2] = ro.z;
  R.d[0] = rd.x; R.d[1] = rd.y; R.d[2] = rd.z;
  R.time = time;
  R.kind = RAY_MAIN;
  return true;
}

// A path's state into entry `pos` of buffer `b` (coalesced: the writing wave's entries
// are consecutive). The cold record carries the wavelength (spectral) and, for a
// path-length ray, the dielectric hit point.
template <int SAMPLER, bool FWD>
IZPI_DEV void store_entry(const WaveBuf& b, uint32_t pos, const PathSt& P, const RayRec& R) {
  if constexpr (FWD) {  // one plane per component: every store a coalesced 8 B per lane
    sst(b.thr + pos, P.thr[0]);
    if (SAMPLER == IZPI_SAMPLER_COLOUR) { sst(b.thr + b.tplane + pos, P.thr[1]); sst(b.thr + 2 * (size_t)b.tplane + pos, P.thr[2]); }
  }
  double2* r = reinterpret_cast<double2*>(b.ray + pos);
  sst(r, make_double2(R.o[0], R.o[1]));
  sst(r + 1, make_double2(R.o[2], R.d[0]));
  sst(r + 2, make_double2(R.d[1], R.d[2]));
  sst(b.kind + pos, R.kind);
  if (b.time) sst(b.time + pos, R.time);
  sst(b.path + pos, PathHot{P.rng, P.depth | P.zf << 16, P.unit, P.rslot});
  if (b.blk) sst(b.blk + pos, P.blk);
  if (b.cold) {
    double2* c = reinterpret_cast<double2*>(b.cold + pos);
    if (SAMPLER == IZPI_SAMPLER_SPECTRAL) sst(c, make_double2(P.lambda, P.lpdf));
    if (kind_of(R.kind) == RAY_PATHLEN) { sst(c + 1, make_double2(P.pend[0], P.pend[1])); sst(c + 2, make_double2(P.pend[2], 0.0)); }
  }
}
// A parked entry moves to the output unchanged (its hit record too), flagged RAY_PARKED.
IZPI_DEV void dead_entry(const WaveBuf& out, uint32_t pos) {
  sst(out.kind + pos, (uint32_t)RAY_DEAD);
  sst(&out.ray[pos].o[0], __longlong_as_double((long long)DEAD_BITS));
}
IZPI_DEV void copy_entry(const WaveBuf& in, uint32_t i, const WaveBuf& out, uint32_t pos) {
  out.ray[pos] = in.ray[i];
  out.kind[pos] = in.kind[i] | RAY_PARKED;
  if (in.time) out.time[pos] = in.time[i];
  out.path[pos] = in.path[i];
  if (in.blk) out.blk[pos] = in.blk[i];
  if (in.cold) out.cold[pos] = in.cold[i];
  out.hit[(size_t)pos * out.hs] = in.hit[(size_t)i * in.hs];
  if (in.huv) out.huv[(size_t)pos * out.hs] = in.huv[(size_t)i * in.hs];
  // (no throughput: only a render with overflow record blocks parks, and IZPI_ACC_FORWARD has none)
}
// The path state of entry i (the ray and hit are read by shade_item).
// What a shading pass reads of entry i besides its path state: the traced ray, the first
// 16 B of its hit record (t, primitive) and the ray time.
struct EntryIn {
  RayOD ray;
  double2 hit;
  double time;
};
IZPI_DEV void load_entry(const WaveBuf& b, uint32_t i, EntryIn& E) {
  E.ray = sld(b.ray + i);
  E.hit = sld(b.hit + (size_t)i * b.hs);
  E.time = b.time ? sld(b.time + i) : 0.0;
}
template <int SAMPLER, bool FWD>
IZPI_DEV void load_path(const WaveBuf& b, uint32_t i, PathSt& P) {
  if constexpr (FWD) {
    P.thr[0] = sld(b.thr + i);
    if (SAMPLER == IZPI_SAMPLER_COLOUR) { P.thr[1] = sld(b.thr + b.tplane + i); P.thr[2] = sld(b.thr + 2 * (size_t)b.tplane + i); }
  }
  const PathHot ph = sld(b.path + i);
  P.rng = ph.rng; P.depth = ph.depth & 0xFFFFu; P.zf = ph.depth >> 16; P.unit = ph.unit; P.rslot = ph.rslot;
  P.blk = b.blk ? sld(b.blk + i) : 0u;
  P.lambda = 0; P.lpdf = 1;
  if (SAMPLER == IZPI_SAMPLER_SPECTRAL) { const double2 c = sld(reinterpret_cast<const double2*>(b.cold + i)); P.lambda = c.x; P.lpdf = c.y; }
}

// Take units for the lanes that ask (one atomic per wave); returns UINT32_MAX when drained.
IZPI_DEV uint32_t grab_unit(const ShadeParams& sp, bool want) {
  const uint64_t m = __ballot(want);
  if (m == 0) return 0xFFFFFFFFu;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(sp.head, (uint32_t)__popcll(m));
  base = __shfl(base, (int)leader);
  const uint32_t my = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
  return (want && my < sp.total_units) ? my : 0xFFFFFFFFu;
}

// First fill of the queue (first pass of a chunk): record slot j takes unit j (the host
// starts the unit head at min(slots, units), so no atomic is needed: one counter word
// serialises ~88 atomics/us), then further units from the head while its path needs no
// tracing; the path goes to entry j of `out`.
template <int SAMPLER, bool FWD>
__global__ void __launch_bounds__(256) k_start(const DevScene sc, const ShadeParams sp_in, const WaveParams wp) {
  ShadeParams sp = sp_in;
  sp.staged = 0;  // k_start stages no tables: its path starts read them from global memory
  sp.prims_staged = 0;
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  bool want = j < sp.slots;
  bool push = false;
  bool first = true;
  PathSt P;
  RayRec R;
  P.rslot = j;
  // a wave keeps grabbing while any of its lanes still lacks a traceable path
  for (;;) {
    uint32_t unit;
    if (first) {
      unit = (want && j < sp.total_units) ? j : 0xFFFFFFFFu;
      first = false;
    } else {
      unit = grab_unit(sp, want);
    }
    if (__ballot(want) == 0) break;
    if (want) {
      if (unit == 0xFFFFFFFFu) {
        want = false;
      } else if (start_path<SAMPLER>(sc, sp, unit, P, R)) {
        want = false;
        push = true;
      }
    }
  }
  // Entry j of the first queue belongs to record slot j (no queue atomic: one per block on
  // one counter word made this kernel 1.9 ms per C3 frame); a slot whose samples all
  // completed without a ray (spectral pdf 0, the units ran out) leaves a dead entry, which
  // the first shading pass drops.
  const uint32_t fill = min(sp.slots, sp.total_units);
  if (j < fill) {
    if (push) store_entry<SAMPLER, FWD>(wp.out, j, P, R);
    else dead_entry(wp.out, j);
  }
  if (j == 0) *wp.out_count = fill;
}

#ifdef IZPI_SHADE_CLOCKS
// Timing builds only: wave cycles per section of shade_item, accumulated in LDS by the
// first active lane of the wave that runs the section (so divergent sections count the
// wave's time once), added to the CNT_SCLK_* counters at the end of the kernel.
enum { SCLK_MAT = 0, SCLK_FIN, SCLK_MIX, SCLK_LPDF, SCLK_ENTRY, SCLK_TEX, SCLK_RB1, SCLK_RATOM, SCLK_RB2, SCLK_N };
IZPI_DEV unsigned long long* sclk_lds() {
  __shared__ unsigned long long c[16][SCLK_N];
  return &c[(threadIdx.x >> 6) & 15][0];
}
IZPI_DEV void sclk_add(int sec, uint64_t dt) {
  const uint64_t act = __ballot(1);
  if ((threadIdx.x & 63) == (uint32_t)(__ffsll((long long)act) - 1)) sclk_lds()[sec] += dt;
}
IZPI_DEV void sclk_flush(unsigned long long* counters) {
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < SCLK_N; k++) atomicAdd(counters + CNT_SCLK_MAT + k, sclk_lds()[k]);
}
IZPI_DEV void sclk_zero() {
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < SCLK_N; k++) sclk_lds()[k] = 0;
  __syncthreads();
}
#define SCLK_T(v) const uint64_t v = __builtin_readcyclecounter()
#define SCLK_ADD(sec, t0) sclk_add(sec, __builtin_readcyclecounter() - (t0))
// wait for every outstanding vector memory access (vmcnt(0); expcnt, lgkmcnt left alone):
// separates a section's memory wait from the work after it
#define SCLK_VMWAIT() __builtin_amdgcn_s_waitcnt(0x0F70)
#else
#define SCLK_VMWAIT() (void)0
#define SCLK_T(v) (void)0
#define SCLK_ADD(sec, t0) (void)0
#endif

// One block-wide reservation phase for a shading iteration (ONE pair of barriers, two
// atomics by one thread): `unit_want` lanes get consecutive work units from the unit
// head (the units past total_units are not granted); lanes with `put` and granted
// `unit_want` lanes get consecutive output entries, `put` lanes first. q_rank: the
// lane's rank among the block's `queue` lanes (deferred unwinding jobs), q_total: their number. A granted lane
// whose new path cannot trace (start_path false) leaves a RAY_DEAD entry behind.
// QSEP: `queue` lanes are a subset of the `unit_want` lanes with a ballot of their own;
// otherwise they are the `unit_want` lanes.
template <bool QSEP>
IZPI_DEV void block_reserve2(const ShadeParams& sp, uint32_t* out_count, bool put, bool unit_want, uint32_t& unit,
                             uint32_t& pos, uint32_t& parity, bool& exhausted, bool queue, uint32_t& q_rank, uint32_t& q_total) {
  __shared__ uint32_t s_p[2][SHADE_WAVES], s_u[2][SHADE_WAVES], s_q[2][SHADE_WAVES];
  __shared__ uint32_t s_pbase[2], s_ubase[2], s_granted[2], s_nput[2], s_nent[2];
  const uint32_t b = parity;
  parity ^= 1u;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1;
  const uint64_t mp = __ballot(put), mu = __ballot(unit_want), mq = QSEP ? __ballot(queue) : 0ull;
  if (lane == 0) { s_p[b][w] = (uint32_t)__popcll(mp); s_u[b][w] = (uint32_t)__popcll(mu); if (QSEP) s_q[b][w] = (uint32_t)__popcll(mq); }
  SCLK_T(rb0);
  __syncthreads();
  SCLK_ADD(SCLK_RB1, rb0);
  SCLK_T(rb1);
  // both atomics in flight together: entries are reserved for every unit_want lane
  // until this block has seen the unit head run out (`exhausted`, thread 0's register);
  // a lane reserved an entry but denied a unit leaves a dead entry (at most one
  // iteration per block, in the frame's last passes)
  uint32_t np = 0, nu = 0, u0 = 0, pb = 0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (uint32_t k = 0; k < SHADE_WAVES; k++) { np += s_p[b][k]; nu += s_u[b][k]; }
    if (exhausted) nu = 0;
    u0 = nu ? atomicAdd(sp.head, nu) : sp.total_units;
    pb = np + nu ? atomicAdd(out_count, np + nu) : 0u;
  }
  if (threadIdx.x == 0) {
    const uint32_t ne = np + nu;
    // (an iteration without finished paths asks for nothing and learns nothing: it must
    // not mark the block exhausted, or the block's later finished paths lose their slots)
    if (nu && u0 + nu >= sp.total_units) exhausted = true;
    s_pbase[b] = pb;
    s_ubase[b] = u0;
    s_granted[b] = u0 >= sp.total_units ? 0u : min(nu, sp.total_units - u0);
    s_nput[b] = np;
    s_nent[b] = ne;
    SCLK_VMWAIT();
    SCLK_ADD(SCLK_RATOM, rb1);
  }
  __syncthreads();
  SCLK_ADD(SCLK_RB2, rb1);
  uint32_t ur = (uint32_t)__popcll(mu & lt), pr = (uint32_t)__popcll(mp & lt);
  for (uint32_t i = 0; i < w; i++) { ur += s_u[b][i]; pr += s_p[b][i]; }
  if constexpr (QSEP) {
    q_rank = (uint32_t)__popcll(mq & lt);
    q_total = 0;
#pragma unroll
    for (uint32_t k = 0; k < SHADE_WAVES; k++) {
      q_rank += k < w ? s_q[b][k] : 0u;
      q_total += s_q[b][k];
    }
  } else {
    q_rank = ur;
    q_total = 0;
#pragma unroll
    for (uint32_t k = 0; k < SHADE_WAVES; k++) q_total += s_u[b][k];
  }
  const bool has_entry = unit_want && s_nput[b] + ur < s_nent[b];
  const bool granted = unit_want && ur < s_granted[b];
  unit = granted ? s_ubase[b] + ur : 0xFFFFFFFFu;
  pos = put ? s_pbase[b] + pr : (has_entry ? s_pbase[b] + s_nput[b] + ur : 0xFFFFFFFFu);
}

// A lane whose path finished got `unit` and entry `pos` (block_reserve2): start the
// unit's path in the finished path's record slot and store it; when its sample completes
// without a ray, take further units one at a time (rare), and leave a dead entry when
// none traces.
template <int SAMPLER, bool FWD>
IZPI_DEV void refill_one(const DevScene& sc, const ShadeParams& sp, const WaveBuf& out, uint32_t unit, uint32_t pos,
                         PathSt& P) {
  RayRec R;
  for (;;) {
    if (start_path<SAMPLER>(sc, sp, unit, P, R)) {
      store_entry<SAMPLER, FWD>(out, pos, P, R);
      return;
    }
    unit = atomicAdd(sp.head, 1u);
    if (unit >= sp.total_units) {
      dead_entry(out, pos);
      return;
    }
  }
}



// calculatePathLength's length of a found exit point (dielectric.go:141-150): |exit - p|
// clamped to [0.1, 100]
IZPI_DEV double path_length(V3 hp, V3 exit_p) {
  double len = length(sub(exit_p, hp));
  if (len < 0.1) len = 0.1;
  if (len > 100.0) len = 100.0;
  return len;
}

// One shading pass of `slot` (its ray was traced): Colour.Sample / SampleSpectral
// one bounce deep (colour.go:33-65, sampler/spectral.go:47-80). Sets `push` when the path
// has a ray to trace next and `done` when its sample finished.
// Entry i of `in`: P is its path state (load_path), with blk set to the path's overflow
// block when it needs one (P.depth >= rec_dense); `kind` its kind word. On return, P and
// R hold the continuing path and its next ray (`push`), or `done` is set and `fblk` is
// the block to free. DEFER: a finished path is not unwound here (`queued`; Colour: only
// one whose unwinding reads records, finish_reads); R.o holds its terminal radiance
// (Spectral: R.o[0]) for the caller's queue (fin_queue), and the caller frees its block
// after the unwinding. (Spectral queues every finished path: the test cost the Spectral
// instances up to 24 more spilled VGPRs, C5 shade 320 -> 352 ms.)
template <int SAMPLER, int MATSET, bool DEFER, bool FWD>
IZPI_DEV void shade_item(const DevScene& sc, const ShadeParams& sp, const WaveBuf& in, uint32_t i, uint32_t kind,
                         const EntryIn& E, PathSt& P, RayRec& R, bool& push, bool& done, uint32_t& fblk, uint32_t& c_lt,
                         uint32_t& c_ls, bool& queued) {
  const bool COLOUR = SAMPLER == IZPI_SAMPLER_COLOUR;
  const bool st = sp.staged != 0;  // the scene's small tables are in this block's LDS
  SCLK_T(sc0);
  SCLK_VMWAIT();
  SCLK_ADD(SCLK_ENTRY, sc0);
  for (int k = 0; k < 3; k++) { R.o[k] = E.ray.o[k]; R.d[k] = E.ray.d[k]; }
  R.kind = kind;
  R.time = E.time;  // NewRay(hr.P, dir, r.Time()): the next ray keeps the time
  HitOut H;
  H.t = E.hit.x; H.prim = (int32_t)__double2loint(E.hit.y); H.pad = 0; H.u = 0; H.v = 0;  // (u, v) read on demand
  Lcg rng;
  rng.s = P.rng;
  const V3 ro = mk(R.o[0], R.o[1], R.o[2]), rd = mk(R.d[0], R.d[1], R.d[2]);
  V3 L = mk(0, 0, 0);
  bool terminal = false;
  bool spec = false, have_pdf = false, zero_spdf = false;
  V3 att = mk(0, 0, 0), next_o = mk(0, 0, 0), next_d = mk(0, 0, 0);
  V3 hit_n = mk(0, 0, 0);
  uint32_t rec_mat = 0;
  Onb cos_onb;
  if (ms_has(MATSET, MS_DIEL) && kind_of(R.kind) == RAY_PATHLEN) {
    // calculatePathLength result (dielectric.go:135-152) -> finish the glass bounce
    const PathCold& pc = in.cold[i];
    const V3 hp = mk(pc.pend[0], pc.pend[1], pc.pend[2]);
    const double len = H.prim >= 0 ? path_length(hp, add(ro, smul(rd, H.t))) : 10.0;  // no exit: dielectric.go:152
    const uint32_t mat_id = R.kind >> KIND_MAT_SHIFT;  // dielectric material stashed by the glass bounce
    const izpi_material gm_ = mat_rec(sc, st, mat_id);
    if (COLOUR) att = mk(gm::exp(-gm_.rgb[0] * len), gm::exp(-gm_.rgb[1] * len), gm::exp(-gm_.rgb[2] * len));
    else att.x = gm_.absorb_tex >= 0 ? gm::exp(-tex_spectral(sc, gm_.absorb_tex, P.lambda, 0.0, 0.0, st) * len) : 1.0;
    spec = true;
    next_o = hp;
    next_d = rd;
  } else if (H.prim < 0) {
    L = COLOUR ? mk(sp.background[0], sp.background[1], sp.background[2])
               : mk(bg_value(sp, P.lambda), 0, 0);
    terminal = true;
  } else {
    const bool pst = sp.prims_staged != 0;
    const GShade gs = gshade_of(sc, pst, H.prim);
    HitRec h;
    hit_record(sc, H, in.huv ? in.huv + (size_t)i * in.hs : nullptr, gs, ro, rd, R.time, (gs_cflags(gs) & 2u) != 0, h, st, ms_has(MATSET, MS_PBR), pst);
    hit_n = h.n;
    rec_mat = h.mat;
    next_o = h.p;
    // the shade record carries the material kind and, for a constant RGB texture, its
    // value: the common Lambert/light hit reads no material or texture record
    const izpi_material m = mat_rec(sc, st, h.mat);
    const bool cconst = COLOUR && (gs_cflags(gs) & 1u) != 0;
    V3 cval = mk(0, 0, 0);
    if (cconst) { const double4 c4 = mat_const_of(sp, h.mat); cval = mk(c4.x, c4.y, c4.z); }
    switch (gs_kind(gs)) {
      case IZPI_MAT_DIFFUSE_LIGHT: {  // no scatter: return emitted (diffuselight.go:49-63)
        if (dot(h.n, rd) < 0.0) {
          if (cconst) L = cval;
          else if (COLOUR) L = tex_rgb(sc, m.albedo_tex, h.u, h.v, st);
          else L.x = tex_spectral(sc, m.spectral_tex, P.lambda, h.u, h.v, st);
        }
        terminal = true;
        break;
      }
      case IZPI_MAT_LAMBERT: {  // lambertian.go:44-70: 2 draws for a ray the sampler discards (A6)
        rng.next();
        rng.next();
        cos_onb.build(h.n);
        if (cconst) att = cval;
        else if (COLOUR) att = tex_rgb(sc, m.albedo_tex, h.u, h.v, st);
        else att.x = tex_spectral(sc, m.spectral_tex, P.lambda, h.u, h.v, st);
        have_pdf = true;
        break;
      }
      case IZPI_MAT_ISOTROPIC: {  // isotropic.go:32-60: a randomInUnitSphere ray the sampler discards,
        // Cosine(N) as the material pdf of the mixture, ScatteringPDF 0; Spectral: the albedo's red
        if constexpr (!ms_has(MATSET, MS_ISO)) { atomicOr(sp.error, 2u); terminal = true; break; }
        (void)random_in_unit_sphere(rng);
        cos_onb.build(h.n);
        const V3 a = tex_rgb(sc, m.albedo_tex, h.u, h.v, st);
        if (COLOUR) att = a; else att.x = a.x;
        have_pdf = true;
        zero_spdf = true;
        break;
      }
      case IZPI_MAT_DIELECTRIC: {  // dielectric.go:156-207
        if constexpr (!ms_has(MATSET, MS_DIEL)) { atomicOr(sp.error, 2u); terminal = true; break; }
        const double ri = COLOUR ? m.ref_idx : tex_spectral(sc, m.spectral_tex, P.lambda, 0.0, 0.0, st);
        bool reflected;
        next_d = dielectric_scatter(rd, h.n, ri, rng, reflected);
        const bool beer_rgb = COLOUR && (m.flags & IZPI_MATF_BEER_LAMBERT) && !(m.rgb[0] == 0 && m.rgb[1] == 0 && m.rgb[2] == 0);
        if (!reflected && (!COLOUR || beer_rgb)) {
          // the extra World.Hit of calculatePathLength: trace it, finish next pass
          P.pend[0] = h.p.x; P.pend[1] = h.p.y; P.pend[2] = h.p.z;
          P.rng = rng.s;
          const V3 po = add(h.p, smul(next_d, 0.001));
          R.o[0] = po.x; R.o[1] = po.y; R.o[2] = po.z;
          R.d[0] = next_d.x; R.d[1] = next_d.y; R.d[2] = next_d.z;
          R.kind = RAY_PATHLEN | (h.mat << KIND_MAT_SHIFT);
          push = true;
          break;
        }
        att = mk(1.0, 1.0, 1.0);
        spec = true;
        break;
      }
      case IZPI_MAT_METAL: {  // metal.go:34-41 (RGB only: SpectralScatter is nonSpectral)
        if constexpr (!ms_has(MATSET, MS_METAL)) { atomicOr(sp.error, 2u); terminal = true; break; }
        if (!COLOUR) { terminal = true; break; }
        V3 reflected = reflect(unit(rd), h.n);
        next_d = add(reflected, smul(random_in_unit_sphere(rng), m.fuzz));
        att = mk(m.rgb[0], m.rgb[1], m.rgb[2]);
        spec = true;
        break;
      }
      case IZPI_MAT_PBR: {  // pbr.go:59-155 / 158-263
        if constexpr (!ms_has(MATSET, MS_PBR)) { atomicOr(sp.error, 2u); terminal = true; break; }
        // the four texture slots (LDS, or one 64-B record); every lookup below is issued
        // before the first of them is used
        SCLK_T(sct);
        const TexSlot s_alb = mat_slot(sc, st, h.mat, 0), s_nrm = mat_slot(sc, st, h.mat, 1),
                      s_rgh = mat_slot(sc, st, h.mat, 2), s_met = mat_slot(sc, st, h.mat, 3);
        // one texel index for the images of the normal map's size (C4: all four)
        const uint32_t w0 = s_nrm.w, h0 = s_nrm.hf & 0x3FFFFFFFu;
        const uint64_t k0 = (s_nrm.hf >> 30) <= TEXF_GRAY ? image_index(w0, h0, h.u, h.v) : 0;
        double alb_s = 0;
        if (COLOUR) att = slot_rgb_k(sc, s_alb, h.u, h.v, st, w0, h0, k0);
        else if (m.spectral_tex >= 0) alb_s = tex_spectral(sc, m.spectral_tex, P.lambda, h.u, h.v, st);
        else { V3 c = slot_rgb_k(sc, s_alb, h.u, h.v, st, w0, h0, k0); alb_s = 0.299 * c.x + 0.587 * c.y + 0.114 * c.z; }
        V3 rough = slot_set(s_rgh) ? slot_rgb_k(sc, s_rgh, h.u, h.v, st, w0, h0, k0) : mk(0.5, 0.5, 0.5);
        V3 metal = slot_set(s_met) ? slot_rgb_k(sc, s_met, h.u, h.v, st, w0, h0, k0) : mk(0.0, 0.0, 0.0);
        const bool has_nmap = slot_set(s_nrm);
        const V3 nuv = has_nmap ? slot_rgb_k(sc, s_nrm, h.u, h.v, st, w0, h0, k0) : mk(0, 0, 0);  // one texel for both uses
        SCLK_VMWAIT();
        SCLK_ADD(SCLK_TEX, sct);
        if (has_nmap && IZPI_PRIM_KIND(gs.ref) == IZPI_PRIM_TRIANGLE) {
          h.n = nmap_tbn(sc, H.prim, h.n, nuv, pst);  // the hit record's normal (triangle.go:250-264)
          hit_n = h.n;
        }
        V3 normal = h.n;
        if (has_nmap) {
          V3 tn = mk(2.0 * nuv.x - 1.0, 2.0 * nuv.y - 1.0, nuv.z);
          V3 nn0 = h.n;
          V3 t = cross(nn0, mk(0, 1, 0));
          if (dot(t, t) < 0.001) t = cross(nn0, mk(1, 0, 0));
          t = sdiv(t, length(t));
          V3 b = cross(nn0, t);
          b = sdiv(b, length(b));
          V3 nn = mk(t.x * tn.x + b.x * tn.y + nn0.x * tn.z, t.y * tn.x + b.y * tn.y + nn0.y * tn.z,
                     t.z * tn.x + b.z * tn.y + nn0.z * tn.z);
          normal = sdiv(nn, length(nn));
        }
        double rv = (rough.x + rough.y + rough.z) / 3.0;
        double mv = (metal.x + metal.y + metal.z) / 3.0;
        cos_onb.build(normal);  // the scatter's ONB and the sampler's Cosine(normal) pdf: one build (onb.go:38-67)
        const Onb& uvw = cos_onb;
        const V3 urd = unit(rd);  // (one evaluation for both uses)
        V3 reflected = reflect(urd, normal);
        double cosTheta = gm::abs(dot(urd, normal));
        double fresnel = 0.04 + (1.0 - 0.04) * gm::pow(1.0 - cosTheta, 5.0);
        fresnel = fresnel + (mv * 0.5);
        double sprob = fresnel * (1.0 - rv);
        if (rng.next() < sprob) {
          double rf = gm::max(0.01, rv * 0.3);
          V3 rdir = random_in_unit_sphere(rng);
          next_d = unit(add(reflected, smul(rdir, rf)));
          spec = true;
        } else {
          next_d = unit(uvw.local(random_cosine_direction(rng)));
          spec = false;
          have_pdf = true;  // the sampler ignores this ray and samples the mixture pdf
        }
        if (!COLOUR) att.x = spec ? alb_s * 1.5 : alb_s;
        break;
      }
      default: {
        atomicOr(sp.error, 2u);
        terminal = true;
      }
    }
  }
  SCLK_ADD(SCLK_MAT, sc0);
  if (!push) {
    if (terminal) {
      SCLK_T(sc1);
      if constexpr (FWD) finish_fwd<SAMPLER>(sp, P, L);
      else if constexpr (DEFER && !COLOUR) { R.o[0] = L.x; R.o[1] = L.y; R.o[2] = L.z; }
      else if (DEFER && finish_reads<SAMPLER, MATSET>(P, L)) { R.o[0] = L.x; R.o[1] = L.y; R.o[2] = L.z; queued = true; }
      else finish<SAMPLER, MATSET>(sp, P, L);
      SCLK_ADD(SCLK_FIN, sc1);
      done = true;
      fblk = P.blk;
    } else {
      SCLK_T(sc2);
      if (have_pdf) {
        // Mixture(Hitable(lights, P), Cosine(N)) (colour.go:48-51, mixture.go:17-33)
        V3 dir;
        if (rng.next() < 0.5) dir = lights_random(sc, st, next_o, rng);
        else dir = cos_onb.local(random_cosine_direction(rng));
        // (evaluated in an order that frees the ONB, normal and attenuation before
        // the light-pdf loop; every value is computed exactly as in the reference)
        const V3 ud = unit(dir);
        const double cosv = dot(ud, cos_onb.w);
        const double cos_pdf = cosv > 0 ? cosv / 3.141592653589793 : 0;
        double sc_cos = dot(hit_n, ud);  // ScatteringPDF with the hit normal
        if (sc_cos < 0) sc_cos = 0;
        const double spdf = zero_spdf ? 0.0 : sc_cos / 3.141592653589793;  // Isotropic.ScatteringPDF is 0
        if constexpr (FWD) {  // T * att now (frees T and att during the light-pdf loop), * (s / p) after it
          P.thr[0] = P.thr[0] * att.x;
          if (COLOUR) { P.thr[1] = P.thr[1] * att.y; P.thr[2] = P.thr[2] * att.z; }
        } else {
          rec_store<SAMPLER, MATSET>(sp, P.rslot, P.blk, P.depth, false, att, spdf, rec_mat);
        }
        SCLK_T(sc3);
        const double pdf_val = 0.5 * lights_pdf(sc, st, next_o, dir, c_lt, c_ls) + 0.5 * cos_pdf;
        SCLK_ADD(SCLK_LPDF, sc3);
        if constexpr (FWD) {
          const double w = spdf / pdf_val;
          P.thr[0] = P.thr[0] * w;
          if (COLOUR) { P.thr[1] = P.thr[1] * w; P.thr[2] = P.thr[2] * w; }
        } else {
          sst(rec_ptr<SAMPLER, MATSET>(sp, P.rslot, P.blk, P.depth) + RecLayout<SAMPLER, MATSET>::P, pdf_val);
          if constexpr (ms_spec(MATSET) || SAMPLER == IZPI_SAMPLER_SPECTRAL) rec_zero_track<SAMPLER>(P.zf, false, att, spdf, pdf_val);
        }
        next_d = dir;
      } else if constexpr (FWD) {
        P.thr[0] = P.thr[0] * att.x;
        if (COLOUR) { P.thr[1] = P.thr[1] * att.y; P.thr[2] = P.thr[2] * att.z; }
      } else {
        rec_store<SAMPLER, MATSET>(sp, P.rslot, P.blk, P.depth, true, att, 0, rec_mat);
        rec_zero_track<SAMPLER>(P.zf, true, att, 0.0, 0.0);
      }
      SCLK_ADD(SCLK_MIX, sc2);
      P.depth++;
      P.rng = rng.s;
      if (P.depth >= sp.max_depth) {
        const V3 Lt = terminal_max_depth(sp, P, COLOUR);
        if constexpr (FWD) finish_fwd<SAMPLER>(sp, P, Lt);
        else if constexpr (DEFER && !COLOUR) { R.o[0] = Lt.x; R.o[1] = Lt.y; R.o[2] = Lt.z; }
        else if (DEFER && finish_reads<SAMPLER, MATSET>(P, Lt)) { R.o[0] = Lt.x; R.o[1] = Lt.y; R.o[2] = Lt.z; queued = true; }
        else finish<SAMPLER, MATSET>(sp, P, Lt);
        done = true;
        fblk = P.blk;
      } else {
        R.o[0] = next_o.x; R.o[1] = next_o.y; R.o[2] = next_o.z;
        R.d[0] = next_d.x; R.d[1] = next_d.y; R.d[2] = next_d.z;
        R.kind = RAY_MAIN;
        push = true;
      }
    }
  }
}

// ---- overflow record blocks
// POOL_SHARDS rings of free block ids. A ring holds its own blocks only: block b belongs
// to ring b >> pool_shift, and a freed block goes back to its ring, so no ring ever holds
// more than its 1 << pool_shift entries. Each ring is a FIFO between an allocation head
// and a free tail (64-bit counters, index = counter & (ring size - 1)). Allocations take
// from the head but only below the PUBLISHED tail, which k_trace2 advances once per pass
// (kernel boundaries order the frees' ring writes before the next pass's reads). A wave
// allocates from its own ring; an allocation that finds no published block there parks
// its slot for one pass (PARK_BIT). Paths that hold a block never wait, so parked slots
// always get one back.
IZPI_DEV unsigned long long* pool_ring_ctr(const ShadeParams& sp, uint32_t r) {
  return sp.pool_ctr + (size_t)r * POOL_CTR_STRIDE;
}
// Wave-aggregated allocation for the lanes with `need`: returns 1 + block, or 0 (`need`
// lanes with 0 are parked).
IZPI_DEV uint32_t pool_alloc(const ShadeParams& sp, bool need) {
  const uint64_t m = __ballot(need);
  if (m == 0) return 0;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t ring = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (POOL_SHARDS - 1);
  unsigned long long* c = pool_ring_ctr(sp, ring);
  const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1;
  unsigned long long base = 0, pub = 0;
  if (lane == leader) {
    base = atomicAdd(c, (unsigned long long)__popcll(m));
    pub = __atomic_load_n(c + 2, __ATOMIC_RELAXED);
  }
  base = __shfl(base, (int)leader);
  pub = __shfl(pub, (int)leader);
  const unsigned long long idx = base + (unsigned long long)__popcll(m & ((1ull << lane) - 1));
  const uint32_t size_mask = (1u << sp.pool_shift) - 1u;
  return (need && idx < pub) ? sp.pool_ring[((size_t)ring << sp.pool_shift) + (idx & size_mask)] + 1u : 0u;
}
// Return a lane's block (1 + block, 0 = none) to its ring.
IZPI_DEV void pool_free_one(const ShadeParams& sp, uint32_t fblk) {
  const uint32_t b = fblk - 1u, ring = b >> sp.pool_shift, size_mask = (1u << sp.pool_shift) - 1u;
  const unsigned long long pos = atomicAdd(pool_ring_ctr(sp, ring) + 1, 1ull);
  sp.pool_ring[((size_t)ring << sp.pool_shift) + (pos & size_mask)] = b;
}
// Single-lane allocation that tries every ring (k_tail: cannot park), or 0.
IZPI_DEV uint32_t pool_alloc_any(const ShadeParams& sp, uint32_t first) {
  const uint32_t size_mask = (1u << sp.pool_shift) - 1u;
  for (uint32_t k = 0; k < POOL_SHARDS; k++) {
    const uint32_t ring = (first + k) & (POOL_SHARDS - 1);
    unsigned long long* c = pool_ring_ctr(sp, ring);
    if (__atomic_load_n(c, __ATOMIC_RELAXED) >= __atomic_load_n(c + 2, __ATOMIC_RELAXED)) continue;  // exhausted
    const unsigned long long idx = atomicAdd(c, 1ull);
    if (idx < __atomic_load_n(c + 2, __ATOMIC_RELAXED)) return sp.pool_ring[((size_t)ring << sp.pool_shift) + (idx & size_mask)] + 1u;
  }
  return 0u;
}

// Deferred unwinding. A path that ends in a shading pass is unwound (finish) from its
// records, depth - 1 down to 0; done in the finishing lane itself, a wave waits for its
// deepest finishing lane while its other lanes idle (C5: finish took 48% of k_shade's
// wave cycles with a few lanes of a wave finishing per iteration). Instead the finishing
// lane queues a job in its block's queue, and the block unwinds the queued jobs with every
// lane busy once FINQ_FLUSH are queued (and at the end of the launch). The records stay
// put until then: the slot's next path writes its first record in the NEXT pass, after
// its first ray is traced, and the finished path's overflow block is freed by fin_flush.
// A job: unit | rslot << 32, blk | (depth | zf << 16) << 32, then the terminal radiance
// (Colour) or L.x, lambda, lpdf (Spectral), word-major (word k of job j at k * FINQ_CAP + j).
template <int SAMPLER>
IZPI_DEV void fin_queue(unsigned long long* q, uint32_t j, const PathSt& P, const RayRec& R) {
  const bool colour = SAMPLER == IZPI_SAMPLER_COLOUR;
  q[j] = P.unit | (unsigned long long)P.rslot << 32;
  q[FINQ_CAP + j] = P.blk | (unsigned long long)(P.depth | P.zf << 16) << 32;
  q[2 * FINQ_CAP + j] = (unsigned long long)__double_as_longlong(R.o[0]);
  q[3 * FINQ_CAP + j] = (unsigned long long)__double_as_longlong(colour ? R.o[1] : P.lambda);
  q[4 * FINQ_CAP + j] = (unsigned long long)__double_as_longlong(colour ? R.o[2] : P.lpdf);
}
template <int SAMPLER, int MATSET>
IZPI_DEV void fin_flush(const ShadeParams& sp, const unsigned long long* q, uint32_t n) {
  const bool colour = SAMPLER == IZPI_SAMPLER_COLOUR;
  for (uint32_t j = threadIdx.x; j < n; j += SHADE_THREADS) {
    PathSt P;
    const unsigned long long w0 = q[j], w1 = q[FINQ_CAP + j];
    P.unit = (uint32_t)w0; P.rslot = (uint32_t)(w0 >> 32);
    P.blk = (uint32_t)w1; P.depth = (uint32_t)(w1 >> 32) & 0xFFFFu; P.zf = (uint32_t)(w1 >> 48);
    const double a = __longlong_as_double((long long)q[2 * FINQ_CAP + j]);
    const double b = __longlong_as_double((long long)q[3 * FINQ_CAP + j]);
    const double c = __longlong_as_double((long long)q[4 * FINQ_CAP + j]);
    P.lambda = colour ? 0.0 : b; P.lpdf = colour ? 0.0 : c;
    finish<SAMPLER, MATSET>(sp, P, colour ? mk(a, b, c) : mk(a, 0.0, 0.0));
    if (sp.rec_pool && P.blk) pool_free_one(sp, P.blk);
  }
}
// Which k_shade instances defer: 1 = the Spectral ones and the Colour ones with specular
// materials (C5 at 32 spp: shading 377 -> 320 ms; C4, queueing only the unwindings that
// read records: 464.7 -> 453.7 ms), not C1-C3's Lambert-only instances (C3 +3.4% even
// with only the record-reading unwindings queued: they are short, and the queue costs
// stores), 2 = all, 0 = none. Handing each wave's lanes jobs of similar depth (a counting
// sort of a flush's jobs by depth) measured slower: C5 338 ms, C4 +1.4%.

// One shading pass over the slots traced in the previous k_trace.
// k_shade's register budget: 3 waves per SIMD (168 VGPRs). MATSET_BASIC colour at 4 waves spilled
// 47 VGPRs and measured 1% slower; the spectral / MATSET_FULL instances ran C5 7% faster at 3
// waves than at 2 despite ~100 B/lane of spill.
constexpr int SHADE_WPE = 3;
template <int SAMPLER, int MATSET, bool FWD>
__global__ void __launch_bounds__(SHADE_THREADS) __attribute__((amdgpu_waves_per_eu(SHADE_WPE)))
k_shade(const DevScene sc, const ShadeParams sp, const WaveParams wp) {
  shade_stage(sc, sp);
  uint32_t parity = 0;  // block_reserve2 LDS buffer set
  const uint32_t n = *wp.in_count;
  // this pass's k_trace2 is done with its dequeue cursor: reset it for the next pass's
  if (blockIdx.x == 0 && threadIdx.x == 0) *wp.trace_next = 0;
  bool exhausted = false;  // (thread 0) this block has seen the unit head run out
  uint32_t c_lt = 0, c_ls = 0, c_park = 0;
  const uint32_t stride = gridDim.x * SHADE_THREADS;
  constexpr bool DEFER = !FWD && (SAMPLER == IZPI_SAMPLER_SPECTRAL || ms_spec(MATSET));
  constexpr bool COLOUR_DEFER = DEFER && SAMPLER == IZPI_SAMPLER_COLOUR;  // a subset of the finished paths is queued
  unsigned long long* fq = sp.finq + (size_t)blockIdx.x * FINQ_WORDS * FINQ_CAP;
  uint32_t fq_n = 0;  // jobs in this block's queue (the same in every thread)
#ifdef IZPI_SHADE_CLOCKS
  uint64_t k_item = 0, k_ref = 0, k_push = 0;
  sclk_zero();
#endif
  // Block-uniform trip count: the unit and queue reservations are block-wide.
  for (uint32_t base = blockIdx.x * SHADE_THREADS; base < n; base += stride) {
    const uint32_t i = base + threadIdx.x;
    const bool valid = i < n;
    bool push = false;      // the path has a ray to trace next (P, R)
    bool done = false;      // its sample finished: start a new unit in its record slot
    bool parked = false;
    uint32_t fblk = 0;
#ifdef IZPI_SHADE_CLOCKS
    uint64_t t0 = __builtin_readcyclecounter();
#endif
    PathSt P;
    RayRec R;
    P.rslot = 0; P.blk = 0; P.depth = 0; P.zf = 0;
    uint32_t kind = RAY_DEAD;
    EntryIn E;
    if (valid) {
      // the kind word, path state, ray and hit record in one round of loads (a dead entry's
      // path and hit are read too, and ignored): waiting for the kind word first, then the
      // path, then the ray put three memory round trips in front of every item
      kind = sld(wp.in.kind + i) & ~(uint32_t)RAY_PARKED;  // a parked entry retries its pass
      load_path<SAMPLER, FWD>(wp.in, i, P);
      load_entry(wp.in, i, E);
    }
    const bool live = valid && !(kind & RAY_DEAD);
    if (sp.rec_pool) {  // a path at depth >= rec_dense writes its records to an overflow block
      const bool need = live && P.depth >= sp.rec_dense && P.blk == 0;
      const uint32_t b = pool_alloc(sp, need);
      P.blk = need ? b : P.blk;
      parked = need && b == 0;
      c_park += parked ? 1u : 0u;
    }
    bool queued = false;    // (DEFER) its unwinding waits in the block's queue
    if (live && !parked) shade_item<SAMPLER, MATSET, DEFER, FWD>(sc, sp, wp.in, i, kind, E, P, R, push, done, fblk, c_lt, c_ls, queued);
    if (SAMPLER == IZPI_SAMPLER_SPECTRAL) queued = DEFER && done;  // (every finished path)
    // a queued path's overflow block is freed after its unwinding (fin_flush)
    if ((COLOUR_DEFER ? !queued : !DEFER) && sp.rec_pool && fblk) pool_free_one(sp, fblk);
#ifdef IZPI_SHADE_CLOCKS
    uint64_t t1 = __builtin_readcyclecounter();
    k_item += t1 - t0;
    t0 = t1;
#endif
    // one reservation phase: output entries for continuing and parked paths, new units
    // (and their entries) for finished ones
    uint32_t unit, pos, frank, ftotal;
    block_reserve2<COLOUR_DEFER>(sp, wp.out_count, push || parked, done, unit, pos, parity, exhausted, queued, frank, ftotal);
    if (queued) fin_queue<SAMPLER>(fq, fq_n + frank, P, R);  // (before refill_one reuses P)
    fq_n += ftotal;
    if (push) store_entry<SAMPLER, FWD>(wp.out, pos, P, R);
    if (parked) copy_entry(wp.in, i, wp.out, pos);
#ifdef IZPI_SHADE_CLOCKS
    t1 = __builtin_readcyclecounter();
    k_push += t1 - t0;
    t0 = t1;
#endif
    if (unit != 0xFFFFFFFFu) refill_one<SAMPLER, FWD>(sc, sp, wp.out, unit, pos, P);
    else if (done && pos != 0xFFFFFFFFu) dead_entry(wp.out, pos);  // entry reserved, the units ran out
#ifdef IZPI_SHADE_CLOCKS
    t1 = __builtin_readcyclecounter();
    k_ref += t1 - t0;
#endif
    if (DEFER && fq_n >= FINQ_FLUSH) {  // (block-uniform; the next iteration's jobs wait for its reservation's barriers)
      __syncthreads();
      fin_flush<SAMPLER, MATSET>(sp, fq, fq_n);
      fq_n = 0;
    }
  }
  if (DEFER && fq_n) {
    __syncthreads();
    fin_flush<SAMPLER, MATSET>(sp, fq, fq_n);
  }
  const uint32_t lane = threadIdx.x & 63;
#ifdef IZPI_SHADE_CLOCKS
  if (lane == 0) {
    atomicAdd(sp.counters + CNT_SCLK_ITEM, (unsigned long long)k_item);
    atomicAdd(sp.counters + CNT_SCLK_REFILL, (unsigned long long)k_ref);
    atomicAdd(sp.counters + CNT_SCLK_PUSH, (unsigned long long)k_push);
  }
  sclk_flush(sp.counters);
#endif
  if (c_park && wp.out_park) *wp.out_park = 1u;  // the next k_trace2 must read kind words
  unsigned long long vals[3] = {c_lt, c_ls, c_park};
  const int idx[3] = {CNT_LTRI, CNT_LSPH, CNT_PARK};
  for (int k = 0; k < 3; k++) {
    unsigned long long s = vals[k];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
    if (lane == 0) count_add(sp.cpart, sp.counters, idx[k], s);
  }
}

// The wavefront's tail. Once every work unit has started and few paths remain, the
// pass-synchronous loop pays, per pass, the latency of that pass's longest traversal.
// k_tail instead runs each remaining path to its end in one lane: trace, shade, trace...
// (no refill: the unit head is exhausted), so the passes of different paths overlap.
// Same per-ray code paths, results and counters as k_trace + k_shade.
template <int SAMPLER, int MATSET, int STACK, bool FWD>
__global__ void __launch_bounds__(256) k_tail(const DevScene sc, const ShadeParams sp, const WaveParams wp, int32_t* spill) {
  shade_stage(sc, sp);
  __shared__ int32_t lds_stack[std::min(STACK, TAIL_LDS_STACK) * 256];
  int32_t* stk = lds_stack + threadIdx.x;
  const uint32_t gstride = gridDim.x * 256;
  int32_t* gsp = spill + blockIdx.x * 256 + threadIdx.x;
  const uint32_t n = *wp.in_count;
  uint32_t c_rays = 0, c_nodes = 0, c_tri = 0, c_sph = 0, c_lt = 0, c_ls = 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    // entry i runs to its end in this lane; its next ray goes back to entry i
    if (wp.in.kind[i] & RAY_DEAD) continue;
    bool traced = (wp.in.kind[i] & RAY_PARKED) != 0;  // a parked entry's ray is already traced
    for (;;) {
      if (!traced) trace_one<STACK>(sc, wp.in, i, stk, gsp, gstride, c_rays, c_nodes, c_tri, c_sph, sp.error);
      traced = false;
      PathSt P;
      RayRec R;
      load_path<SAMPLER, FWD>(wp.in, i, P);
      const uint32_t kind = wp.in.kind[i] & ~(uint32_t)RAY_PARKED;
      if (sp.rec_pool && P.depth >= sp.rec_dense && P.blk == 0) {
        // The host launches k_tail with at most pool blocks paths, all of the free
        // blocks published, so this cannot fail (guarded anyway: no spin on a bug).
        P.blk = pool_alloc_any(sp, blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
        if (P.blk == 0) { atomicOr(sp.error, 4u); break; }
      }
      bool push = false, done = false;
      uint32_t fblk = 0;
      EntryIn E;
      load_entry(wp.in, i, E);
      bool queued = false;  // (k_tail unwinds in place)
      shade_item<SAMPLER, MATSET, false, FWD>(sc, sp, wp.in, i, kind, E, P, R, push, done, fblk, c_lt, c_ls, queued);
      if (fblk) pool_free_one(sp, fblk);
      if (!push) break;
      store_entry<SAMPLER, FWD>(wp.in, i, P, R);
    }
  }
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long vals[9] = {c_rays, c_nodes, c_tri, c_sph, c_lt, c_ls, c_nodes, c_tri, c_sph};
  const int idx[9] = {CNT_RAYS, CNT_NODES, CNT_TRI, CNT_SPH, CNT_LTRI, CNT_LSPH, CNT_TAIL_NODES, CNT_TAIL_TRI, CNT_TAIL_SPH};
#pragma unroll
  for (int k = 0; k < 9; k++) {
    unsigned long long v = vals[k];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if (lane == 0) count_add(sp.cpart, sp.counters, idx[k], v);
  }
}

constexpr uint32_t CPART_BLOCKS_PER_CU = 16;  // counter rows per CU / 4: above any resident 256-thread grid
// End of frame: counters[k] += the sum of column k of the per-wave rows (count_add).
__global__ void __launch_bounds__(256) k_cpart_reduce(const unsigned long long* cpart, uint32_t rows,
                                                      unsigned long long* counters) {
  __shared__ unsigned long long red[256];
  unsigned long long v = 0;
  for (uint32_t r = threadIdx.x; r < rows; r += 256) v += cpart[(size_t)r * CNT_N + blockIdx.x];
  red[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) counters[blockIdx.x] += red[0];
}

// Publish the frees of the last shading pass (k_trace2 does it at its start; k_tail and
// the host's pool checks need it on their own).
__global__ void k_pool_publish(unsigned long long* ctr) { pool_publish(ctr); }
// Every ring holds all of its blocks at the start of a render.
__global__ void k_pool_init(uint32_t* ring, uint32_t n, uint32_t per_ring, unsigned long long* ctr) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) ring[i] = i;
  if (i < POOL_SHARDS) {
    unsigned long long* c = ctr + (size_t)i * POOL_CTR_STRIDE;
    c[0] = 0; c[1] = per_ring; c[2] = per_ring;
  }
}

// Per-pixel sequential sum of the chunk's samples (render/rgb.go:36 col += ...,
// render/spectral.go:164-166 sum += ...), in sample order; finalize on the last chunk.
struct AccumParams {
  uint32_t num_pixels, chunk_spp, spp, width, height, tile_w, tile_h, sampler, last, out_layout;
  const uint32_t* tiles;
  const double* samples;  // [num_pixels][chunk_spp][3]
  double* running;        // [num_pixels][3]
  double* out;
};
__global__ void __launch_bounds__(256) k_accumulate(const AccumParams ap) {
  const uint32_t p = blockIdx.x * 256 + threadIdx.x;
  if (p >= ap.num_pixels) return;
  double c0 = ap.running[3 * (size_t)p], c1 = ap.running[3 * (size_t)p + 1], c2 = ap.running[3 * (size_t)p + 2];
  const double* s = ap.samples + (size_t)p * ap.chunk_spp * SMP_D;
  uint32_t k = 0;
  if constexpr (SMP_D == 4) {  // padded results: (x, y), (z, pad) per sample
    const double2* s2 = reinterpret_cast<const double2*>(s);
    for (; k < ap.chunk_spp; k++) {
      const double2 a = s2[2 * k], b = s2[2 * k + 1];
      c0 = c0 + a.x; c1 = c1 + a.y; c2 = c2 + b.x;
    }
  }
  if (SMP_D == 3 && (ap.chunk_spp & 3u) == 0 && blockIdx.x * 256 + 256 <= ap.num_pixels) {
    // Staged through LDS, 4 samples (96 B) of each of the wave's 64 pixels at a time: the
    // wave's lanes load the 64 runs as consecutive 16-B pieces (a load instruction covers
    // ~11 neighbouring runs instead of one piece of 64 runs 12 KB apart), then each lane
    // adds its own pixel's 4 samples from LDS in sample order (rgb.go:36).
    __shared__ double2 st[4][64 * 6];
    double2* w = st[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t p0 = p - lane;  // the wave's first pixel
    const size_t run = (size_t)ap.chunk_spp * 3 / 2;  // double2 per pixel
    const double2* s2 = reinterpret_cast<const double2*>(ap.samples) + (size_t)p0 * run;
    for (; k < ap.chunk_spp; k += 4) {
      double2 v[6];
#pragma unroll
      for (int i = 0; i < 6; i++) {
        const uint32_t q = lane + 64 * i, j = q / 6, c = q % 6;
        v[i] = sld(s2 + (size_t)j * run + (k >> 1) * 3 + c);
      }
#pragma unroll
      for (int i = 0; i < 6; i++) w[lane + 64 * i] = v[i];
      __builtin_amdgcn_wave_barrier();
      const double2 a = w[6 * lane], b = w[6 * lane + 1], c = w[6 * lane + 2];
      const double2 d = w[6 * lane + 3], e = w[6 * lane + 4], f = w[6 * lane + 5];
      __builtin_amdgcn_wave_barrier();
      c0 = c0 + a.x; c1 = c1 + a.y; c2 = c2 + b.x;  // sample k
      c0 = c0 + b.y; c1 = c1 + c.x; c2 = c2 + c.y;  // sample k + 1
      c0 = c0 + d.x; c1 = c1 + d.y; c2 = c2 + e.x;  // sample k + 2
      c0 = c0 + e.y; c1 = c1 + f.x; c2 = c2 + f.y;  // sample k + 3
    }
  }
  if ((ap.chunk_spp & 1u) == 0 && k == 0) {
    // two samples (48 B, 16-B aligned for an even chunk_spp) per three 16-B loads: the
    // lanes' runs lie chunk_spp * 24 B apart, so every load instruction touches 64 lines
    // and the instruction count, not the bytes, bounds this loop
    const double2* s2 = reinterpret_cast<const double2*>(s);
    for (; k + 1 < ap.chunk_spp; k += 2) {  // sample order, as rgb.go:36
      const double2 a = s2[3 * (k >> 1)], b = s2[3 * (k >> 1) + 1], c = s2[3 * (k >> 1) + 2];
      c0 = c0 + a.x; c1 = c1 + a.y; c2 = c2 + b.x;  // sample k
      c0 = c0 + b.y; c1 = c1 + c.x; c2 = c2 + c.y;  // sample k + 1
    }
  }
  for (; k < ap.chunk_spp; k++) {  // sample order, as rgb.go:36
    c0 = c0 + s[3 * k];
    c1 = c1 + s[3 * k + 1];
    c2 = c2 + s[3 * k + 2];
  }
  if (!ap.last) {
    ap.running[3 * (size_t)p] = c0; ap.running[3 * (size_t)p + 1] = c1; ap.running[3 * (size_t)p + 2] = c2;
    return;
  }
  double r0, r1, r2;
  if (ap.sampler == IZPI_SAMPLER_COLOUR) {  // vec3.ScalarDiv(col, numSamples)
    r0 = c0 / (double)ap.spp; r1 = c1 / (double)ap.spp; r2 = c2 / (double)ap.spp;
  } else {  // sum * (1/numSamples)
    const double inv = 1.0 / (double)ap.spp;
    r0 = c0 * inv; r1 = c1 * inv; r2 = c2 * inv;
  }
  const uint32_t tile_px = ap.tile_w * ap.tile_h;
  if (ap.out_layout == IZPI_OUT_PACKED) {
    double* o = ap.out + (size_t)p * 4;
    o[0] = r0; o[1] = r1; o[2] = r2; o[3] = 1.0;
    return;
  }
  const uint32_t tile = p / tile_px, in_tile = p % tile_px;
  const uint32_t x = ap.tiles[4 * tile] + in_tile % ap.tile_w;
  const uint32_t y = ap.tiles[4 * tile + 1] + in_tile / ap.tile_w;
  const uint32_t row = ap.height - y;  // canvas.Set(x, ny-y): row ny is dropped (A9)
  if (row < ap.height) {
    double* o = ap.out + ((size_t)row * ap.width + x) * 4;
    o[0] = r0; o[1] = r1; o[2] = r2; o[3] = 1.0;
  }
}

// FireflyRejection (firefly_rejection.go:12-113) fused with XYZToRGB (rgb_image.go:28-67).
// FireflyRejection reads only the ORIGINAL Y plane (it copies it first, :33-39) and
// scales the pixel's own X, Y, Z, so pixels are independent: one thread per pixel, the
// 18x18 Y halo of a 16x16 tile staged in LDS. The scaled XYZ then goes through the
// exposure multiply and the ACEScg matrix in XYZToRGB's operation order.
__global__ void __launch_bounds__(256) k_spectral_post(const double* in, double* out, uint32_t W, uint32_t H,
                                                       double exposure) {
  __shared__ double ys[18][18];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int x0 = blockIdx.x * 16, y0 = blockIdx.y * 16;
  for (int i = threadIdx.x; i < 18 * 18; i += 256) {
    const int hx = x0 + (i % 18) - 1, hy = y0 + (i / 18) - 1;
    ys[i / 18][i % 18] = (hx >= 0 && hx < (int)W && hy >= 0 && hy < (int)H) ? in[((size_t)hy * W + hx) * 4 + 1] : 0.0;
  }
  __syncthreads();
  const int x = x0 + tx, y = y0 + ty;
  if (x >= (int)W || y >= (int)H) return;
  const size_t pi = ((size_t)y * W + x) * 4;
  const double2 xy = *reinterpret_cast<const double2*>(in + pi), za = *reinterpret_cast<const double2*>(in + pi + 2);
  double X = xy.x, Y = xy.y, Z = za.x;
  const double cur = ys[ty + 1][tx + 1];
  if (cur > 0) {  // `currentY <= 0` skips (NaN does not)
    double nb[8];
    int nn = 0;
    for (int dy = -1; dy <= 1; dy++)
      for (int dx = -1; dx <= 1; dx++) {
        if (dx == 0 && dy == 0) continue;
        const int nx = x + dx, ny = y + dy;
        if (nx >= 0 && nx < (int)W && ny >= 0 && ny < (int)H) {
          const double v = ys[ty + 1 + dy][tx + 1 + dx];
          if (v > 0) nb[nn++] = v;
        }
      }
    if (nn >= 3) {
      double sum = 0.0;
      for (int i = 0; i < nn; i++) sum += nb[i];
      const double mean = sum / (double)nn;
      double vs = 0.0;
      for (int i = 0; i < nn; i++) { const double d = nb[i] - mean; vs += d * d; }
      const double stddev = gm::sqrt(vs / (double)nn);
      const double threshold = mean + 2.5 * stddev;
      if (cur > threshold && threshold > 0) {
        const double ratio = threshold / cur;
        X *= ratio; Y *= ratio; Z *= ratio;
      }
    }
  }
  X *= exposure; Y *= exposure; Z *= exposure;
  double2 rg, ba;
  rg.x = 1.6410234 * X + -0.3248033 * Y + -0.2364247 * Z;
  rg.y = -0.6636629 * X + 1.6153316 * Y + 0.0167563 * Z;
  ba.x = 0.0117219 * X + -0.0082845 * Y + 0.9883949 * Z;
  ba.y = za.y;  // alpha unchanged
  *reinterpret_cast<double2*>(out + pi) = rg;
  *reinterpret_cast<double2*>(out + pi + 2) = ba;
}

// postprocess.Pipeline (pipeline.go:20-31) of Gamma (gamma.go:24-41: R,G,B = math.Sqrt)
// and Clamp (clamp.go:27-51: v < max ? v : max, so NaN -> max) filters, applied in list
// order to each pixel; alpha unchanged. The reference walks x <= Max.X, y <= Max.Y: the
// extra row/column reads zero and its Set is dropped, so only in-bounds pixels change.
// HBM-streaming, 32 B in + 32 B out per pixel.
struct PostFilters {
  uint32_t n;
  uint32_t kind[IZPI_MAX_FILTERS];
  double param[IZPI_MAX_FILTERS];
};

__global__ void __launch_bounds__(256) k_postprocess(double* canvas, uint64_t num_pixels, const PostFilters pf) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= num_pixels) return;
  double2* p = reinterpret_cast<double2*>(canvas + i * 4);
  double2 rg = p[0], ba = p[1];
  double c[3] = {rg.x, rg.y, ba.x};
  for (uint32_t f = 0; f < pf.n; f++) {
    if (pf.kind[f] == IZPI_FILTER_GAMMA) {
      for (int k = 0; k < 3; k++) c[k] = gm::sqrt(c[k]);
    } else {
      const double mx = pf.param[f];
      for (int k = 0; k < 3; k++) c[k] = c[k] < mx ? c[k] : mx;
    }
  }
  p[0] = make_double2(c[0], c[1]);
  p[1] = make_double2(c[2], ba.y);
}

// Packed pixel p (IZPI_OUT_PACKED: tile after tile, the rows of each tile) -> its canvas
// column x and row H - y (rgb.go:41); false for sample row y = 0, which has no canvas row.
// k_unpack and izpi_host_assemble_shares share this rule.
__host__ __device__ inline bool packed_target(const uint32_t* tiles, uint32_t p, uint32_t tile_w, uint32_t tile_h,
                                              uint32_t height, uint32_t* x, uint32_t* row) {
  const uint32_t tile_px = tile_w * tile_h;
  const uint32_t tile = p / tile_px, in_tile = p % tile_px;
  *x = tiles[4 * tile] + in_tile % tile_w;
  *row = height - (tiles[4 * tile + 1] + in_tile / tile_w);
  return *row < height;
}
__global__ void k_unpack(const uint32_t* tiles, uint32_t num_pixels, uint32_t tile_w, uint32_t tile_h, uint32_t width,
                         uint32_t height, const double* packed, double* canvas) {
  const uint32_t p = blockIdx.x * 256 + threadIdx.x;
  if (p >= num_pixels) return;
  uint32_t x, row;
  if (packed_target(tiles, p, tile_w, tile_h, height, &x, &row)) {
    const double* s = packed + (size_t)p * 4;
    double* o = canvas + ((size_t)row * width + x) * 4;
    o[0] = s[0]; o[1] = s[1]; o[2] = s[2]; o[3] = s[3];
  }
}

// ------------------------------------------------------- component kernels
// izpi_gpu_trace: rays [n][8] -> queue entries with explicit (tMin, tMax)
__global__ void k_trace_setup(const double* rays, uint32_t n, RayOD* ray, uint32_t* kind, double2* tminmax, uint32_t* qn) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) *qn = n;
  if (i >= n) return;
  const double* r = rays + (size_t)i * 8;
  RayOD h;
  for (int k = 0; k < 3; k++) { h.o[k] = r[k]; h.d[k] = r[3 + k]; }
  ray[i] = h;
  kind[i] = RAY_PATHLEN;  // not a Sampler call
  tminmax[i] = make_double2(r[6], r[7]);
}
__global__ void k_trace_records(const DevScene sc, const RayOD* rr, const double2* hit, uint32_t n, izpi_hit* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  izpi_hit h;
  memset(&h, 0, sizeof(h));
  h.prim_ref = 0xFFFFFFFFu;
  HitOut c;
  const double2* rec = hit + 2 * (size_t)i;  // (t, prim), (u, v)
  c.t = rec[0].x; c.prim = hit_prim(rec[0]); c.u = rec[1].x; c.v = rec[1].y; c.pad = 0;
  if (c.prim >= 0) {
    const RayOD R = rr[i];
    HitRec hr;
    const GShade gs = sc.shade[c.prim];
    hit_record(sc, c, rec + 1, gs, mk(R.o[0], R.o[1], R.o[2]), mk(R.d[0], R.d[1], R.d[2]), 0.0, true, hr);
    const GPrim& p = sc.prims[c.prim];
    h.hit = 1; h.t = hr.t; h.u = hr.u; h.v = hr.v;
    h.p[0] = hr.p.x; h.p[1] = hr.p.y; h.p[2] = hr.p.z;
    h.normal[0] = hr.n.x; h.normal[1] = hr.n.y; h.normal[2] = hr.n.z;
    h.prim_ref = IZPI_PRIM_REF(p.kind, p.index);
  }
  out[i] = h;
}

__global__ void k_aabb4(const float* boxes, const float* rays, uint32_t n, uint8_t* masks) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float* b = boxes + (size_t)i * 24;
  const float* r = rays + (size_t)i * 7;
  uint8_t m = 0;
  for (int k = 0; k < 4; k++)
    if (slab(b[k], b[4 + k], b[8 + k], b[12 + k], b[16 + k], b[20 + k], r[0], r[1], r[2], r[3], r[4], r[5], r[6])) m |= (uint8_t)(1 << k);
  masks[i] = m;
}

__global__ void k_gomath(const DevScene sc, int op, const double* x, const double* y, uint32_t n, double* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (op == 14) {  // path_length(hit point x[i], exit point y[i]): 3 doubles each
    out[i] = path_length(mk(x[3 * i], x[3 * i + 1], x[3 * i + 2]), mk(y[3 * i], y[3 * i + 1], y[3 * i + 2]));
    return;
  }
  double a = x[i], b = y ? y[i] : 0.0, r;
  switch (op) {
    case 0: r = gm::sin(a); break;
    case 1: r = gm::cos(a); break;
    case 2: r = gm::tan(a); break;
    case 3: r = gm::exp(a); break;
    case 4: r = gm::log(a); break;
    case 5: r = gm::pow(a, b); break;
    case 6: r = gm::atan2(a, b); break;
    case 7: r = gm::asin(a); break;
    case 8: r = gm::sqrt(a); break;
    case 9: r = a / b; break;
    case 10: r = gm::atan(a); break;
    case 11: case 12: { double sv, cv; gm::sincos_nonneg(a, &sv, &cv); r = op == 11 ? sv : cv; break; }
    case 13: r = sdiv(mk(a, 0.0, 0.0), b).x; break;  // sdiv's shared reciprocal (= a / b)
    case 32: case 33: { double l, pdf; sample_wavelength(a, l, pdf); r = op == 32 ? l : pdf; break; }
    case 34: case 35: case 36: { double cx, cy, cz; cie_values(a, cx, cy, cz); r = op == 34 ? cx : op == 35 ? cy : cz; break; }
    case 37: r = tex_spectral(sc, (int32_t)b, a); break;
    default: r = gm::nan();
  }
  out[i] = r;
}

// ================================================================ host side
// Scratch device buffers of one ABI call, freed when it returns (on every path).
struct DevBufs {
  std::vector<void*> p;
  template <typename T>
  hipError_t alloc(T** out, size_t count) {
    *out = nullptr;
    const hipError_t e = hipMalloc((void**)out, count * sizeof(T));
    if (e == hipSuccess) p.push_back(*out);
    return e;
  }
  ~DevBufs() {
    for (void* q : p) (void)hipFree(q);
  }
};

struct izpi_ctx {
  int device = 0;
  std::string err;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  int num_cus = 0;
  // scene
  bool have_scene = false;
  uint32_t num_textures = 0;     // of the uploaded scene (izpi_gpu_gomath texture lookups)
  uint32_t num_materials = 0;    // of the uploaded scene
  uint32_t num_spd = 0;          // tabulated SPD entries of the uploaded scene
  // The workspace sizing of the last render and what it was decided for (render_impl): a
  // request of the same shape reuses it, so frames of one renderer never re-size (sizing
  // from the free HBM of each frame made C4 reallocate its 148 GB every frame, 2 s each).
  struct Sizing {
    uint64_t key[8];
    uint32_t chunk, slots, pool_blocks, pool_div;
  } sizing{};
  bool sizing_valid = false;
  DevScene sc{};
  uint32_t stack_needed = 0;
  uint32_t num_prims = 0;
  std::vector<void*> scene_allocs;
  size_t scene_bytes = 0;
  // render workspace (grown on demand)
  double* d_samples = nullptr; size_t samples_cap = 0;
  double* d_recs = nullptr; size_t recs_cap = 0;
  double* d_pool = nullptr; size_t pool_cap = 0;       // overflow unwinding records
  uint32_t* d_ring = nullptr; size_t ring_cap = 0;     // free ring of overflow blocks
  unsigned long long* d_pool_ctr = nullptr;            // ring counters, [POOL_SHARDS][POOL_CTR_STRIDE]
  double* d_running = nullptr; size_t running_cap = 0;
  double* d_out = nullptr; size_t out_cap = 0;
  uint32_t* d_tiles = nullptr; size_t tiles_cap = 0;
  uint32_t* d_utiles = nullptr; size_t utiles_cap = 0;  // tile lists of k_unpack (multi-GPU root)
  double* d_bg = nullptr; size_t bg_cap = 0;
  uint32_t* d_misc = nullptr;              // words k * MISC_STRIDE (misc()): 0 unit head, 1 error, 2 trace cursor, 3..4 queue counts, 6..7 park flags
  unsigned long long* d_counters = nullptr;
  unsigned long long* d_cpart = nullptr; size_t cpart_cap = 0;  // per-wave counter rows of a render (count_add)
  unsigned long long* d_finq = nullptr; size_t finq_cap = 0;  // k_shade blocks' deferred unwinding jobs (fin_flush)
  char* d_state = nullptr; size_t state_cap = 0;      // the two WaveBufs (carve_state)
  int32_t* d_spill = nullptr; size_t spill_cap = 0;  // traversal-stack spill area of k_trace2
  double* d_post = nullptr; size_t post_cap = 0;      // spectral post-processing output
  double* d_share = nullptr; size_t share_cap = 0;    // multi-GPU: this device's packed tiles
  double* d_gather = nullptr; size_t gather_cap = 0;  // multi-GPU root: every device's packed tiles
  uint32_t* h_count = nullptr;                        // pinned readback of d_misc (unit head, queue lengths; same stride) + scratch
  hipEvent_t ev3 = nullptr;
  hipEvent_t evb[3 * IZPI_PASS_BATCH] = {};
  // RCCL communicator of a multi-process render (izpi_gpu_comm_init), or null
  ncclComm_t comm = nullptr;
  // izpi_gpu_debug_fault 3: the pinned word a stalled stream waits on (null when none)
  volatile uint32_t* stall_word = nullptr;
  uint32_t* stall_host = nullptr;  // its allocation (coherent pinned host memory)
  uint32_t comm_rank = 0, comm_size = 1;
  int32_t* d_status = nullptr;   // agreement word of izpi_gpu_render_rank ([0] in, [1] max over ranks)
  int fault_inject = 0;          // izpi_gpu_debug_fault: 1 fail before rendering, 2 fail the render
  izpi_render_stats last{};
  bool mat_ok_rgb = false, mat_ok_spectral = false;
  bool basic_materials = false;  // only Lambertian + DiffuseLight: use the MATSET_BASIC shader
  uint32_t matset = 0;           // MS_* bits of the scene's material kinds
  bool const_albedo = false;     // ... and every albedo / emit texture a constant RGB: MATSET_CONST (Colour)
  bool any_uv = false;           // a material reads the hit's (u, v) (image textures)
  uint32_t pool_grow = 0;        // overflow pool doublings earned by frames that parked (render_impl)
  uint32_t dev_share = 1;        // contexts of this process on this device (izpi_gpu_multi_open): they split its HBM
  // Progress of the running render (izpi_gpu_progress, read from other threads): samples
  // whose paths have finished, as of the host's last queue poll, and the request's samples.
  std::atomic<uint64_t> prog_done{0}, prog_total{0};
};

namespace {

// The words of d_misc lie MISC_STRIDE words (256 B) apart: the unit head and the queue
// counts take one returning atomic each per shading block-iteration (~11M per C3 frame),
// and atomics on one line are served one at a time (a single word saturates near 88 per
// microsecond, MI355X_MICROARCH.md "dequeue").
uint32_t* misc(izpi_ctx* ctx, int k) { return ctx->d_misc + (size_t)k * MISC_STRIDE; }

template <typename T>
int dev_upload(izpi_ctx* ctx, const T* host, size_t count, T** out) {
  *out = nullptr;
  if (count == 0) return IZPI_OK;
  HIP_TRY(hipMalloc((void**)out, count * sizeof(T)));
  ctx->scene_allocs.push_back(*out);
  ctx->scene_bytes += count * sizeof(T);
  if (host) HIP_TRY(hipMemcpy(*out, host, count * sizeof(T), hipMemcpyHostToDevice));
  return IZPI_OK;
}
#define UP(ptr, n, dst)                                   \
  do {                                                    \
    int rc_ = dev_upload(ctx, ptr, (size_t)(n), dst);     \
    if (rc_) return rc_;                                  \
  } while (0)

int grow(izpi_ctx* ctx, void** p, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return IZPI_OK;
  if (*p) HIP_TRY(hipFree(*p));
  *p = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(p, bytes));
  *cap = bytes;
  return IZPI_OK;
}

// Device bytes of the render workspace (the buffers `grow` manages).
uint64_t workspace_bytes(const izpi_ctx* ctx) {
  return (uint64_t)ctx->samples_cap + ctx->recs_cap + ctx->pool_cap + ctx->ring_cap + ctx->running_cap + ctx->out_cap +
         ctx->tiles_cap + ctx->utiles_cap + ctx->bg_cap + ctx->state_cap + ctx->spill_cap + ctx->post_cap + ctx->share_cap +
         ctx->gather_cap + ctx->cpart_cap + ctx->finq_cap;
}

// Device bytes of the buffers render_impl sizes per frame and may release to re-size
// (not the output, share, gather and post-processing buffers, which it never frees).
uint64_t render_buffer_bytes(const izpi_ctx* ctx) {
  return (uint64_t)ctx->samples_cap + ctx->recs_cap + ctx->pool_cap + ctx->ring_cap + ctx->running_cap + ctx->state_cap +
         ctx->spill_cap;
}

struct RenderBuf {
  void** p;
  size_t* cap;
  size_t bytes;
};

// Make every buffer of `b` at least its `bytes`: if any must grow, free them all first,
// then allocate each at exactly its size.
int grow_render_buffers(izpi_ctx* ctx, RenderBuf* b, size_t n, bool* fresh) {
  for (size_t i = 0; i < n; i++)  // a buffer this render does not use (the records of IZPI_ACC_FORWARD)
    if (b[i].bytes == 0 && *b[i].p) {
      HIP_TRY(hipStreamSynchronize(ctx->stream));
      HIP_TRY(hipFree(*b[i].p));
      *b[i].p = nullptr;
      *b[i].cap = 0;
    }
  bool must = false;
  for (size_t i = 0; i < n; i++) must = must || *b[i].cap < b[i].bytes;
  *fresh = must;
  if (!must) return IZPI_OK;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  for (size_t i = 0; i < n; i++) {
    if (*b[i].p) HIP_TRY(hipFree(*b[i].p));
    *b[i].p = nullptr;
    *b[i].cap = 0;
  }
  for (size_t i = 0; i < n; i++) {
    if (b[i].bytes == 0) continue;
    const hipError_t e = hipMalloc(b[i].p, b[i].bytes);
    if (e != hipSuccess) {
      *b[i].p = nullptr;
      ctx->err = "render workspace: hipMalloc of " + std::to_string(b[i].bytes) + " bytes: " + hipGetErrorString(e);
      return IZPI_ERR_HIP;
    }
    *b[i].cap = b[i].bytes;
  }
  return IZPI_OK;
}

// The two sides of the wavefront state, `slots` entries each, in one allocation:
// returns the bytes (base == nullptr) or fills b[0], b[1].
size_t carve_state(char* base, uint32_t slots, bool time, bool blk, bool cold, bool uv, uint32_t thr_planes, WaveBuf* b) {
  size_t off = 0;
  auto take = [&](size_t bytes) -> char* {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return p;
  };
  for (int k = 0; k < 2; k++) {
    WaveBuf w{};
    w.ray = (RayOD*)take((size_t)slots * sizeof(RayOD));
    w.kind = (uint32_t*)take((size_t)slots * sizeof(uint32_t));
    w.time = time ? (double*)take((size_t)slots * sizeof(double)) : nullptr;
    w.path = (PathHot*)take((size_t)slots * sizeof(PathHot));
    w.blk = blk ? (uint32_t*)take((size_t)slots * sizeof(uint32_t)) : nullptr;
    w.cold = cold ? (PathCold*)take((size_t)slots * sizeof(PathCold)) : nullptr;
    // with (u, v): one 32-B record per entry, (t, prim) then (u, v), so a finished ray's
    // two stores land in one line (two separate arrays made C4 / C5 trace 6-7% slower)
    w.hs = uv ? 2u : 1u;
    w.hit = (double2*)take((size_t)slots * w.hs * sizeof(double2));
    w.huv = uv && w.hit ? w.hit + 1 : nullptr;
    w.tminmax = nullptr;
    w.thr = thr_planes ? (double*)take((size_t)slots * thr_planes * sizeof(double)) : nullptr;
    w.tplane = slots;
    if (b) b[k] = w;
  }
  return off;
}

void free_scene(izpi_ctx* ctx) {
  for (void* p : ctx->scene_allocs) (void)hipFree(p);
  ctx->scene_allocs.clear();
  ctx->scene_bytes = 0;
  ctx->have_scene = false;
}

template <typename K>
int resident_blocks(izpi_ctx* ctx, K kernel, int* blocks, int threads = 256, size_t dyn_lds = 0) {
  int per_cu = 0;
  if (dyn_lds) HIP_TRY(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn_lds));
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, dyn_lds));
  if (per_cu < 1) per_cu = 1;
  *blocks = per_cu * ctx->num_cus;
  return IZPI_OK;
}

// Traversal kernel selection: k_trace2 with a 16-entry LDS stack ring and global spill,
// 5 waves/SIMD. Instances: DIST (leaf tests spread over the wave; off only when primitive
// indices do not fit the 26-bit LDS packing, or IZPI_TUNE_NO_DIST) x TRI (sphere code
// compiled out for triangle-only scenes; IZPI_TUNE_GENERAL_TRACE forces the general one).
// izpi_render_tuning: prim_weight (default 32) weighs primitive steps against node steps
// (x/16); trace_chunk queue entries per dequeue; refill_min idle lanes per refill. All
// settings give identical results and counters.
constexpr int TRACE_RING = 16, TRACE_WPE = 5;
struct Tracer {
  bool p2 = true;    // DIST
  bool tri = false;  // TRI
  bool lds_bvh = false;  // LB
  bool ray_lds = false;  // RL
  // queue entries per dequeue and idle lanes per refill, measured on C3: chunk 128 / refill
  // 16 -> 211 ms of k_trace2 per frame, 512 / 24 -> 201, 1024 -> 207, 2048 -> 216, 64 -> 303
  uint32_t prim_w = 32, tchunk = 512, refill_min = 24;
  int blocks = 0;
  size_t spill_bytes = 0;  // the per-thread traversal-stack spill area this launch needs
};

// The request's tuning. ABI 1's izpi_render_tuning ended at tail_paths (an ABI-1 request,
// abi_version 0, has its tuning pointer at the same place): its fields are read and the
// later ones keep their defaults.
const izpi_render_tuning kDefaultTuning{};
inline izpi_render_tuning tuning_of(const izpi_render_req* req) {
  izpi_render_tuning t{};
  if (!req || !req->tuning) return t;
  if (req->abi_version >= 2) return *req->tuning;
  memcpy(&t, req->tuning, offsetof(izpi_render_tuning, tail_paths) + sizeof(t.tail_paths));
  return t;
}

#define IZPI_T2_LIST(X)                                                                                      \
  X(true, false, false, false) X(true, true, false, false) X(false, false, false, false) X(false, true, false, false) \
  X(true, false, true, false) X(true, true, true, false) X(true, true, false, true) X(true, false, true, true)  \
  X(true, true, true, true)
// The BVH-in-LDS ray instances run an 8-entry stack ring: their trees (at most 4 KB) are
// too shallow to fill it, and the 8 KB it frees hold the rays (still 5 blocks per CU).
constexpr int ring_of(bool lb, bool rl) { return lb && rl ? 8 : TRACE_RING; }

// Pick the k_trace2 instance and its grid (no allocation: the caller grows d_spill to
// t->spill_bytes).
// need_uv: the caller reads the hits' (u, v) (WaveParams::hit_uv).
int make_tracer(izpi_ctx* ctx, const izpi_render_tuning& tu, bool need_uv, Tracer* t) {
  *t = Tracer();
  if (tu.flags & IZPI_TUNE_NO_DIST) t->p2 = false;
  // DIST packs (primitive << 6 | lane) into one LDS word
  if (ctx->num_prims >= (1u << 26)) t->p2 = false;
  t->tri = ctx->sc.tri_only != 0 && !(tu.flags & IZPI_TUNE_GENERAL_TRACE);
  t->lds_bvh = t->p2 && !(tu.flags & IZPI_TUNE_NO_LDS_BVH) &&
               (uint64_t)ctx->sc.num_inner * sizeof(GInner) + (uint64_t)ctx->sc.num_prims * (sizeof(GLeaf) + sizeof(GPrim)) <= BVH_LDS_BYTES;
  if (t->lds_bvh) {
    // With the tree in LDS a step costs little next to a refill's ray loads: refill later
    // and weight primitive steps less (profiles/r3i/tune_sweep2.log, trace per frame
    // against 24 / 32: C5 -10.5%, C4 -6.3%, C2 -5.2%; C3's global-memory instance keeps them)
    t->refill_min = 40;
    t->prim_w = 24;
  }
  t->ray_lds = t->p2 && ((t->tri && !t->lds_bvh && !need_uv) || (t->lds_bvh && (t->tri || ctx->sc.time_free))) &&
               !(tu.flags & IZPI_TUNE_NO_RAY_LDS);
  if (tu.prim_weight) t->prim_w = tu.prim_weight;
  if (tu.trace_chunk) t->tchunk = tu.trace_chunk;
  if (tu.refill_min) t->refill_min = std::min<uint32_t>(64, tu.refill_min);
  int rc = IZPI_ERR_INVALID;
#define IZPI_T2_OCC(P, T, L, R)                                               \
  if (t->p2 == P && t->tri == T && t->lds_bvh == L && t->ray_lds == R) \
    rc = resident_blocks(ctx, k_trace2<ring_of(L, R), TRACE_WPE, P, T, L, R>, &t->blocks);
  IZPI_T2_LIST(IZPI_T2_OCC)
#undef IZPI_T2_OCC
  if (rc) return rc;
  t->spill_bytes = (size_t)t->blocks * 256 * 64 * sizeof(int32_t);
  return IZPI_OK;
}

void launch_trace(izpi_ctx* ctx, const DevScene& sc, const Tracer& t, const WaveParams& wp, hipStream_t st, int32_t* spill) {
  const dim3 g(t.blocks), b(256);
  const uint32_t stride = (uint32_t)t.blocks * 256;
#define IZPI_T2_LAUNCH(P, T, L, R)                                                                             \
  if (t.p2 == P && t.tri == T && t.lds_bvh == L && t.ray_lds == R) {                                           \
    hipLaunchKernelGGL((k_trace2<ring_of(L, R), TRACE_WPE, P, T, L, R>), g, b, 0, st, sc, wp, ctx->d_counters,  \
                       misc(ctx, 1), spill, stride, t.prim_w, t.tchunk, t.refill_min);                        \
    return;                                                                                                    \
  }
  IZPI_T2_LIST(IZPI_T2_LAUNCH)
#undef IZPI_T2_LAUNCH
}

uint32_t validate_tiles(const izpi_render_req* req, const uint32_t* tiles, uint32_t n, uint32_t* tw, uint32_t* th) {
  if (n == 0) return 0;
  *tw = tiles[2] - tiles[0] + 1;
  *th = tiles[3] - tiles[1] + 1;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t* t = tiles + 4 * i;
    if (t[2] < t[0] || t[3] < t[1] || t[2] >= req->width || t[3] >= req->height) return 0;
    if (t[2] - t[0] + 1 != *tw || t[3] - t[1] + 1 != *th) return 0;
  }
  return n;
}

// One chunk loop of the wavefront scheme: k_start fills the slots, then k_trace2 /
// k_shade alternate until no slot has a ray left (the last few paths run to their end
// in k_tail); k_accumulate folds the chunk's per-sample radiance into the pixels in
// sample order.
template <int SAMPLER, int MATSET, bool FWD>
int run_chunks(izpi_ctx* ctx, const izpi_render_req* req, const DevScene& sc, const Tracer& tr, ShadeParams& sp,
               WaveParams& wp, AccumParams& ap, uint32_t num_pixels, uint32_t chunk, uint32_t pool_blocks,
               float* trace_ms, float* shade_ms, float* tail_ms, uint32_t* launches) {
  hipStream_t st = ctx->stream;
  const izpi_render_tuning& tu = tuning_of(req);
  int shade_res = 0;
  const size_t dyn = sc.lds_bytes;  // the staged tables' LDS arena (render_body)
  int rc = resident_blocks(ctx, k_shade<SAMPLER, MATSET, FWD>, &shade_res, (int)SHADE_THREADS, dyn);
  if (rc) return rc;
  // tail kernel: used once every unit has started and at most `tail_max` paths remain
  const bool tail_deep = ctx->stack_needed > 32;
  int tail_res = 0;
  if ((rc = tail_deep ? resident_blocks(ctx, k_tail<SAMPLER, MATSET, 64, FWD>, &tail_res, 256, dyn)
                      : resident_blocks(ctx, k_tail<SAMPLER, MATSET, 32, FWD>, &tail_res, 256, dyn))) return rc;
  if ((uint32_t)std::max({tr.blocks * 4, shade_res * (int)SHADE_WAVES, tail_res * 4}) > ctx->num_cus * CPART_BLOCKS_PER_CU * 4 ||
      (uint32_t)shade_res > ctx->num_cus * CPART_BLOCKS_PER_CU) {
    ctx->err = "grid larger than the counter rows or the unwinding queues";
    return IZPI_ERR_INVALID;
  }
  if (tail_deep && (size_t)tail_res * 256 * (64 - TAIL_LDS_STACK) * sizeof(int32_t) > ctx->spill_cap) {
    ctx->err = "k_tail's stack spill does not fit k_trace2's spill area";
    return IZPI_ERR_INVALID;
  }
  uint64_t tail_max = (uint64_t)tail_res * 256;
  if (tu.tail_paths) tail_max = tu.tail_paths;
  if (tu.flags & IZPI_TUNE_NO_TAIL) tail_max = 0;
  // k_tail's allocations cannot park: every tail path must find a published block
  if (sp.rec_pool) tail_max = std::min<uint64_t>(tail_max, pool_blocks);
  const WaveBuf q[2] = {wp.in, wp.out};  // the two sides of the state; entry counts in d_misc[3..4]
  uint32_t* qn[2] = {misc(ctx, 3), misc(ctx, 4)};
  if (sp.rec_pool)
    hipLaunchKernelGGL(k_pool_init, dim3((pool_blocks + 255) / 256), dim3(256), 0, st, sp.pool_ring, pool_blocks,
                       pool_blocks / POOL_SHARDS, sp.pool_ctr);
  HIP_TRY(hipGetLastError());
  for (uint32_t s0 = 0; s0 < req->spp; s0 += chunk) {
    const uint32_t cs = std::min(chunk, req->spp - s0);
    sp.chunk_spp = cs; sp.s0 = s0; sp.total_units = num_pixels * cs;
    const uint32_t fill = std::min<uint32_t>(sp.slots, sp.total_units);
    HIP_TRY(hipMemsetD32Async(misc(ctx, 0), (int)fill, 1, st));  // unit head: k_start gives slot i unit i
    HIP_TRY(hipMemsetAsync(misc(ctx, 2), 0, 3 * MISC_STRIDE * sizeof(uint32_t), st));  // dequeue cursor, queue counts
    HIP_TRY(hipMemsetAsync(misc(ctx, 6), 0, 2 * MISC_STRIDE * sizeof(uint32_t), st));  // park flags of the two sides
    wp.out = q[0]; wp.out_count = qn[0];
    hipLaunchKernelGGL((k_start<SAMPLER, FWD>), dim3((fill + 255) / 256), dim3(256), 0, st, sc, sp, wp);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(ctx->h_count, qn[0], sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    uint32_t n = ctx->h_count[0];
    int cur = 0;
    // Launch passes in batches without a host round-trip per pass: both kernels read
    // their queue length from device memory and exit at once when it is zero, so the
    // host only polls the queue length once per batch (overshoot costs a few empty
    // launches of ~5 us).
    // Once every unit has started, the queue only shrinks: poll after every pass, so that
    // k_tail takes over as soon as few enough paths remain instead of up to 8 passes later
    // (each of those last passes costs ~0.3-1 ms of mostly idle machine).
    int B = IZPI_PASS_BATCH;
    const bool pass_log = (tu.flags & IZPI_TUNE_PASS_LOG) != 0;  // diagnostics: per-pass times on stderr
    while (n > 0) {
      for (int b = 0; b < B; b++) {
        wp.in = q[cur]; wp.in_count = qn[cur];
        wp.out = q[1 - cur]; wp.out_count = qn[1 - cur];
        wp.in_park = misc(ctx, 6 + cur); wp.out_park = misc(ctx, 6 + (1 - cur));
        // (k_trace2 zeroes out_count and out_park, k_shade the dequeue cursor for the next pass)
        HIP_TRY(hipEventRecord(ctx->evb[3 * b], st));
        launch_trace(ctx, sc, tr, wp, st, ctx->d_spill);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ctx->evb[3 * b + 1], st));
        hipLaunchKernelGGL((k_shade<SAMPLER, MATSET, FWD>), dim3(shade_res), dim3(SHADE_THREADS), dyn, st, sc, sp, wp);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ctx->evb[3 * b + 2], st));
        cur = 1 - cur;
      }
      HIP_TRY(hipMemcpyAsync(ctx->h_count, ctx->d_misc, 8 * MISC_STRIDE * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      for (int b = 0; b < B; b++) {
        float t_ms = 0, s_ms = 0;
        HIP_TRY(hipEventElapsedTime(&t_ms, ctx->evb[3 * b], ctx->evb[3 * b + 1]));
        HIP_TRY(hipEventElapsedTime(&s_ms, ctx->evb[3 * b + 1], ctx->evb[3 * b + 2]));
        *trace_ms += t_ms;
        *shade_ms += s_ms;
        if (pass_log) fprintf(stderr, "IZPI_PASS %u trace %.3f shade %.3f\n", *launches, t_ms, s_ms);
        (*launches)++;
      }
      const uint32_t head = ctx->h_count[0];
      n = ctx->h_count[(3 + cur) * MISC_STRIDE];
      {  // units handed out minus the entries still queued: samples finished (a lower bound)
        const uint64_t started = std::min<uint64_t>(head, sp.total_units);
        ctx->prog_done.store((uint64_t)s0 * num_pixels + (started > n ? started - n : 0), std::memory_order_relaxed);
      }
      if (pass_log) fprintf(stderr, "IZPI_BATCH queue %u head %u\n", n, head);
      if (head >= sp.total_units) B = 1;
      // every unit has started: finish the remaining paths in one k_tail launch
      if (n > 0 && n <= tail_max && head >= sp.total_units) {
        wp.in = q[cur]; wp.in_count = qn[cur];
        HIP_TRY(hipEventRecord(ctx->ev2, st));
        if (sp.rec_pool) hipLaunchKernelGGL(k_pool_publish, dim3(1), dim3(256), 0, st, sp.pool_ctr);
        // (the deep instance spills stack entries past 32 into k_trace2's spill area, which
        // holds 64 entries for each of k_trace2's threads, more than k_tail has)
        if (tail_deep) hipLaunchKernelGGL((k_tail<SAMPLER, MATSET, 64, FWD>), dim3(tail_res), dim3(256), dyn, st, sc, sp, wp, ctx->d_spill);
        else hipLaunchKernelGGL((k_tail<SAMPLER, MATSET, 32, FWD>), dim3(tail_res), dim3(256), dyn, st, sc, sp, wp, ctx->d_spill);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ctx->ev3, st));
        HIP_TRY(hipEventSynchronize(ctx->ev3));
        float t_ms = 0;
        HIP_TRY(hipEventElapsedTime(&t_ms, ctx->ev2, ctx->ev3));
        *tail_ms += t_ms;
        n = 0;
      }
    }
    ap.chunk_spp = cs;
    ap.last = (s0 + cs >= req->spp) ? 1u : 0u;
    ctx->prog_done.store((uint64_t)(s0 + cs) * num_pixels, std::memory_order_relaxed);
    hipLaunchKernelGGL(k_accumulate, dim3((num_pixels + 255) / 256), dim3(256), 0, st, ap);
    HIP_TRY(hipGetLastError());
  }
  return IZPI_OK;
}

// The request's tiles: its own list, or the whole frame in common.Tiles steps and
// grid.WalkGrid's spiral order (tiles.go:6-24, renderer.go:172-188).
int request_tiles(izpi_ctx* ctx, const izpi_render_req* req, std::vector<uint32_t>& tiles) {
  if (req->num_tiles) {
    if (!req->tiles) { ctx->err = "num_tiles without tiles"; return IZPI_ERR_INVALID; }
    tiles.assign(req->tiles, req->tiles + 4 * (size_t)req->num_tiles);
    return IZPI_OK;
  }
  tiles.resize(4 * ((size_t)req->width * req->height / 16 + 16));
  const uint32_t nt = izpi_host_tiles(req->width, req->height, tiles.data(), (uint32_t)(tiles.size() / 4));
  if (nt == 0) { ctx->err = "image size not divisible by any common.Tiles step"; return IZPI_ERR_INVALID; }
  tiles.resize(4 * (size_t)nt);
  return IZPI_OK;
}

// Render's post-processing of a whole-frame canvas on the context's stream: the Spectral
// sampler's FireflyRejection + XYZToRGB (renderer.go:215-219), then the leader's "png"
// pipeline, Gamma and Clamp(1.0) (leader.go:179-182).
int apply_post(izpi_ctx* ctx, const izpi_render_req* req, double* canvas_dev) {
  hipStream_t st = ctx->stream;
  int rc;
  if (req->post & IZPI_POST_SPECTRAL) {
    if ((rc = grow(ctx, (void**)&ctx->d_post, &ctx->post_cap, (size_t)req->width * req->height * 4 * sizeof(double)))) return rc;
    dim3 g((req->width + 15) / 16, (req->height + 15) / 16);
    hipLaunchKernelGGL(k_spectral_post, g, dim3(256), 0, st, canvas_dev, ctx->d_post, req->width, req->height, req->exposure);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(canvas_dev, ctx->d_post, (size_t)req->width * req->height * 4 * sizeof(double),
                           hipMemcpyDeviceToDevice, st));
  }
  if (req->post & IZPI_POST_GAMMA_CLAMP) {
    PostFilters pf;
    memset(&pf, 0, sizeof pf);
    pf.n = 2; pf.kind[0] = IZPI_FILTER_GAMMA; pf.kind[1] = IZPI_FILTER_CLAMP; pf.param[1] = 1.0;
    const uint64_t np = (uint64_t)req->width * req->height;
    hipLaunchKernelGGL(k_postprocess, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, canvas_dev, np, pf);
    HIP_TRY(hipGetLastError());
  }
  return IZPI_OK;
}

int render_body(izpi_ctx* ctx, const izpi_render_req* req, double* out_dev);
// One render on one context. The progress counters (izpi_gpu_progress) start at 0/0 before
// any check and read done == total on every return, failed calls included.
int render_impl(izpi_ctx* ctx, const izpi_render_req* req, double* out_dev) {
  ctx->prog_done.store(0, std::memory_order_relaxed);
  ctx->prog_total.store(0, std::memory_order_relaxed);
  const int rc = render_body(ctx, req, out_dev);
  ctx->prog_done.store(ctx->prog_total.load(std::memory_order_relaxed), std::memory_order_relaxed);
  return rc;
}

int render_body(izpi_ctx* ctx, const izpi_render_req* req, double* out_dev) {
  if (ctx->fault_inject == 2) { ctx->err = "injected render fault (izpi_gpu_debug_fault)"; return IZPI_ERR_DEVICE; }
  if (!ctx->have_scene) { ctx->err = "render before izpi_gpu_upload_scene"; return IZPI_ERR_NO_SCENE; }
  if (!req || req->width == 0 || req->height == 0 || req->spp == 0) { ctx->err = "invalid render request"; return IZPI_ERR_INVALID; }
  if (req->abi_version > IZPI_ABI_VERSION) { ctx->err = "render request from a newer ABI"; return IZPI_ERR_INVALID; }
  if (req->sampler != IZPI_SAMPLER_COLOUR && req->sampler != IZPI_SAMPLER_SPECTRAL) { ctx->err = "unsupported sampler"; return IZPI_ERR_UNSUPPORTED; }
  // (a request of ABI 1 or 2 ends at `tuning`: accumulation is not read)
  const uint32_t acc = req->abi_version >= 3 ? req->accumulation : (uint32_t)IZPI_ACC_RECURSIVE;
  if (acc != IZPI_ACC_RECURSIVE && acc != IZPI_ACC_FORWARD) { ctx->err = "unknown accumulation mode"; return IZPI_ERR_INVALID; }
  const bool fwd = acc == IZPI_ACC_FORWARD;
  if (req->post != IZPI_POST_NONE &&
      ((req->post & ~(uint32_t)(IZPI_POST_SPECTRAL | IZPI_POST_GAMMA_CLAMP)) || req->out_layout != IZPI_OUT_CANVAS ||
       req->num_tiles != 0)) {
    ctx->err = "post-processing needs a whole-frame IZPI_OUT_CANVAS request";
    return IZPI_ERR_INVALID;
  }
  if (req->sampler == IZPI_SAMPLER_COLOUR ? !ctx->mat_ok_rgb : !ctx->mat_ok_spectral) {
    ctx->err = "a material lacks the textures this sampler reads";
    return IZPI_ERR_INVALID;
  }
  if (ctx->sc.num_lights == 0) { ctx->err = "scene has no lights (HitableSlice.PDFValue divides by zero)"; return IZPI_ERR_INVALID; }
  std::vector<uint32_t> tiles;
  int rc = request_tiles(ctx, req, tiles);
  if (rc) return rc;
  uint32_t tw = 0, th = 0;
  const uint32_t ntiles = validate_tiles(req, tiles.data(), (uint32_t)(tiles.size() / 4), &tw, &th);
  if (ntiles == 0) { ctx->err = "tiles must be non-empty, in bounds and equal-sized"; return IZPI_ERR_INVALID; }
  const uint64_t num_pixels64 = (uint64_t)ntiles * tw * th;
  if (num_pixels64 > (1ull << 30)) { ctx->err = "too many pixels in one request"; return IZPI_ERR_INVALID; }
  const uint32_t num_pixels = (uint32_t)num_pixels64;
  ctx->prog_total.store(num_pixels64 * req->spp, std::memory_order_relaxed);
  if (ctx->stack_needed > 64) { ctx->err = "BVH deeper than the 64-entry traversal stack (bvh4.go:71)"; return IZPI_ERR_UNSUPPORTED; }
  const izpi_render_tuning& tu = tuning_of(req);
  // this render's view of the scene: the traversal shortcuts the tuning switches off
  DevScene sc = ctx->sc;
  if (tu.flags & IZPI_TUNE_NO_LEAF_SHORTCUT) sc.leaf_shortcut = 0;
  if (tu.flags & IZPI_TUNE_SCALAR_SLAB) sc.nan_free_bounds = 0;
  Tracer tr;
  int trc = make_tracer(ctx, tu, !ctx->sc.tri_only || ctx->any_uv, &tr);
  if (trc) return trc;
  // Sizing against the HBM this context may use: what is free plus the render buffers it
  // holds and would release (a later frame reuses them, so every frame of a renderer sizes
  // alike), shared evenly by the contexts of one process on this device.
  const uint64_t size_key[8] = {num_pixels, req->spp, req->sampler, req->max_depth, ctx->pool_grow,
                                ((uint64_t)tu.slots << 32) | tu.chunk_units, ((uint64_t)tu.rec_dense << 32) | tu.pool_div, acc};
  const bool reuse = ctx->sizing_valid && memcmp(size_key, ctx->sizing.key, sizeof(size_key)) == 0;
  size_t free_b = 0, total_b = 0;
  if (!reuse && hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
  const uint64_t avail = free_b ? ((uint64_t)free_b + render_buffer_bytes(ctx)) / std::max(1u, ctx->dev_share) : 0;
  // The render workspace stays within 15/32 of the HBM (~135 GB of 288, under the ~137 GB
  // C3 takes at its slot cap): per-sample results within 1/8, the wavefront state in the
  // rest. At 17/32 C4 took 153 GB, and a fresh process allocating it right after processes
  // of ~131-137 GB waited 0.4-3.9 s for the driver to clear VRAM (first frame up to 6.6x
  // steady); at 113 GB it allocated in 2 ms and its steady frame was 0.7% slower.
  // Per-sample results wait in HBM ([units][3] doubles) until k_accumulate folds them in
  // sample order. One chunk per request when it fits in 1/8 of the HBM (C3: 12.9 GB of
  // 288 GB), so the wavefront drains once per frame instead of once per chunk (C4 at 1024
  // spp: 2 chunks, C5 at 4096 spp: 12; a chunk's drain costs a few ms).
  uint64_t max_units = std::max<uint64_t>(64ull << 20, (avail / 8) / (3 * sizeof(double)));
  if (tu.chunk_units) max_units = tu.chunk_units;
  // the chunks of a request are balanced: as many as the limit needs, equal in size (C4 at
  // 1024 spp: 2 chunks of 512 instead of 774 + 250, 13 GB less to allocate, same drains)
  uint32_t chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(req->spp, max_units / num_pixels));
  const uint32_t nchunks = (req->spp + chunk - 1) / chunk;
  chunk = (req->spp + nchunks - 1) / nchunks;
  if (reuse) chunk = ctx->sizing.chunk;
  // Unwinding records: the first rec_dense levels per slot, deeper levels in overflow
  // blocks (ShadeParams::rec_pool). Colour records are 40 B (24 B compact), spectral 24 B.
  const bool spectral = req->sampler == IZPI_SAMPLER_SPECTRAL;
  const bool compact = !fwd && !spectral && ctx->basic_materials && ctx->const_albedo;
  const uint32_t D = spectral  ? RecLayout<IZPI_SAMPLER_SPECTRAL, MATSET_FULL>::D
                     : compact ? RecLayout<IZPI_SAMPLER_COLOUR, MATSET_CONST>::D
                               : RecLayout<IZPI_SAMPLER_COLOUR, MATSET_FULL>::D;
  const uint32_t max_depth = std::max(1u, req->max_depth);
  // Spectral glass paths run deep (C5: 12 rays per sample): with 16 dense levels the first
  // frame parked 15% of its shading items on an empty overflow pool; 32 levels park none
  // (C5 256 spp first frame 8854 -> 8130 ms; 92 GB of workspace, less than a pool twice the
  // size would take).
  uint32_t rec_dense = spectral ? 32u : 8u;
  if (tu.rec_dense) rec_dense = tu.rec_dense;
  rec_dense = std::min(rec_dense, max_depth);
  if (fwd) rec_dense = max_depth;  // (no records at all: see need[] and the pool below)
  const uint32_t rec_pool = max_depth - rec_dense;
  // IZPI_ACC_FORWARD: the throughput per entry instead of the records (3 planes Colour, 1 Spectral)
  const uint32_t thr_planes = fwd ? (spectral ? 1u : 3u) : 0u;
  const uint64_t rec_bytes_slot = fwd ? 0 : (uint64_t)rec_dense * D * sizeof(double);
  // PathCold (wavelength, dielectric point) is read only by the spectral sampler and glass
  const bool need_cold = spectral || !ctx->sc.no_pathlen;
  // a hit's (u, v) array: read by (u, v)-reading textures and, for spheres, the root (A16)
  const bool need_uv = !ctx->sc.tri_only || ctx->any_uv;
  // Paths in flight per wavefront pass. Larger = fewer k_trace/k_shade launches and
  // a smaller share of launch tails.
  // C3 per frame (round 2, tiered records): 40M slots 349 ms, 100M 334, 160M 326, 250M 320
  // (fewer passes and pass tails; the first frame, fresh allocations included, is faster
  // too: 371 ms at 40M, 349 ms at 250M); C5 at 64 spp 120M slots: -6%; C4 100M: -3%.
  // The state stays within half of the HBM (below).
  uint64_t slot_cap = 256ull << 20;
  if (tu.slots) slot_cap = std::max<uint64_t>(1024, tu.slots);
  const uint64_t per_slot = 2 * (sizeof(RayOD) + sizeof(uint32_t) + (ctx->sc.tri_only ? 0 : sizeof(double)) + sizeof(PathHot) +
                                 sizeof(uint32_t) + (need_cold ? sizeof(PathCold) : 0) + sizeof(double2) * (need_uv ? 2 : 1) +
                                 thr_planes * sizeof(double)) +
                            rec_bytes_slot;
  // Overflow blocks per slot. Lambert/light scenes: 1 per 16 slots (C3: ~3% of the paths
  // in flight are deeper than 8). Scenes with glass or the spectral sampler run deep
  // chains through glass: 1 per 4 slots (C5 at 1 per 16 parked 29% of its
  // shading items, 574 -> 502 ms per 16-spp frame with no parks at 1 per 4). A frame that
  // still parks more than 1/64 of its rays doubles the pool for the renderer's next frame.
  // Metal / PBR scenes without glass stay at 1 per 16: C4's paths (1.85 rays per sample)
  // park none, and 1 per 4 allocated 56 GB of pool there (a second of a first frame on
  // boxes whose driver clears memory as it maps it).
  uint32_t pool_div = (spectral || !ctx->sc.no_pathlen) ? 4u : 16u;
  pool_div = std::max(1u, pool_div >> std::min(ctx->pool_grow, 4u));
  if (tu.pool_div) pool_div = tu.pool_div;
  if (reuse) pool_div = ctx->sizing.pool_div;
  const uint64_t per_block = (uint64_t)rec_pool * D * sizeof(double) + sizeof(uint32_t);
  // The wavefront state in the rest of the workspace budget. The overflow pool rounds up
  // to a power of two per ring, up to twice slots / pool_div blocks: counted at that worst
  // case (C4 at 256M slots otherwise took 271 GB of the 288). C3 keeps its 256M slots
  // (135 GB); C5 at 128 spp ran 1.4% faster at 64M slots than at 118M (less state, better
  // cache and TLB reach in k_shade), so the smaller budget costs the deep-path scenes nothing.
  const uint64_t samples_bytes = (uint64_t)num_pixels * chunk * SMP_D * sizeof(double);
  const uint64_t budget = avail / 32 * 15;
  if (avail > 0)
    slot_cap = std::min<uint64_t>(slot_cap, std::max<uint64_t>(1024, (budget > samples_bytes ? budget - samples_bytes : 0) /
                                                                          (per_slot + 2 * per_block / pool_div + 1)));
  const uint32_t slots = reuse ? ctx->sizing.slots : (uint32_t)std::min<uint64_t>((uint64_t)num_pixels * chunk, slot_cap);
  uint32_t pool_blocks = 0;
  if (rec_pool) {  // POOL_SHARDS rings of a power of two each, at least 16 blocks per ring
    pool_blocks = POOL_SHARDS * 16;
    while (pool_blocks < slots / pool_div && pool_blocks < (1u << 30)) pool_blocks <<= 1;
  }
  memcpy(ctx->sizing.key, size_key, sizeof(size_key));
  ctx->sizing.chunk = chunk; ctx->sizing.slots = slots; ctx->sizing.pool_blocks = pool_blocks; ctx->sizing.pool_div = pool_div;
  ctx->sizing_valid = true;
  const bool need_time = !ctx->sc.tri_only;  // only sphere tests read the ray time
  // The render buffers this frame needs. When one of them must grow, all are released
  // before any is allocated, so a frame never holds an old buffer next to a new one (the
  // sizing above counted every one of them as available).
  const auto t_alloc0 = std::chrono::steady_clock::now();
  RenderBuf need[] = {
      {(void**)&ctx->d_samples, &ctx->samples_cap, (size_t)num_pixels * chunk * SMP_D * sizeof(double)},
      {(void**)&ctx->d_recs, &ctx->recs_cap, (size_t)rec_bytes_slot * slots},
      {(void**)&ctx->d_pool, &ctx->pool_cap, rec_pool ? (size_t)pool_blocks * rec_pool * D * sizeof(double) : 0},
      {(void**)&ctx->d_ring, &ctx->ring_cap, rec_pool ? (size_t)pool_blocks * sizeof(uint32_t) : 0},
      {(void**)&ctx->d_running, &ctx->running_cap, (size_t)num_pixels * 3 * sizeof(double)},
      {(void**)&ctx->d_state, &ctx->state_cap, carve_state(nullptr, slots, need_time, rec_pool != 0, need_cold, need_uv, thr_planes, nullptr)},
      {(void**)&ctx->d_spill, &ctx->spill_cap, tr.spill_bytes},
  };
  bool fresh = false;
  if ((rc = grow_render_buffers(ctx, need, sizeof(need) / sizeof(need[0]), &fresh))) {
    ctx->sizing_valid = false;
    return rc;
  }
  if ((rc = grow(ctx, (void**)&ctx->d_tiles, &ctx->tiles_cap, tiles.size() * sizeof(uint32_t)))) return rc;
  const size_t nbg = req->num_bg_spd;
  if (nbg && (!req->bg_spd_wavelengths || !req->bg_spd_values)) { ctx->err = "num_bg_spd without the SPD arrays"; return IZPI_ERR_INVALID; }
  if ((rc = grow(ctx, (void**)&ctx->d_bg, &ctx->bg_cap, (2 * nbg + 1) * sizeof(double)))) return rc;
  // counter rows: one per wave of the largest grid (run_chunks checks the grids against it)
  const uint32_t cpart_rows = ctx->num_cus * CPART_BLOCKS_PER_CU * 4u;
  if ((rc = grow(ctx, (void**)&ctx->d_cpart, &ctx->cpart_cap, (size_t)cpart_rows * CNT_N * sizeof(unsigned long long)))) return rc;
  // deferred unwinding jobs: one queue per k_shade block (run_chunks checks its grid against it)
  if (!fwd && (rc = grow(ctx, (void**)&ctx->d_finq, &ctx->finq_cap, (size_t)ctx->num_cus * CPART_BLOCKS_PER_CU * FINQ_WORDS * FINQ_CAP * sizeof(unsigned long long)))) return rc;
  const double alloc_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_alloc0).count();
  WaveBuf bufs[2];
  carve_state(ctx->d_state, slots, need_time, rec_pool != 0, need_cold, need_uv, thr_planes, bufs);
  hipStream_t st = ctx->stream;
  HIP_TRY(hipMemcpyAsync(ctx->d_tiles, tiles.data(), tiles.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  if (nbg) {
    HIP_TRY(hipMemcpyAsync(ctx->d_bg, req->bg_spd_wavelengths, nbg * sizeof(double), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->d_bg + nbg, req->bg_spd_values, nbg * sizeof(double), hipMemcpyHostToDevice, st));
  }
  HIP_TRY(hipMemsetAsync(ctx->d_running, 0, (size_t)num_pixels * 3 * sizeof(double), st));
  HIP_TRY(hipMemsetAsync(ctx->d_counters, 0, CNT_N * sizeof(unsigned long long), st));
  HIP_TRY(hipMemsetAsync(ctx->d_cpart, 0, (size_t)cpart_rows * CNT_N * sizeof(unsigned long long), st));
  HIP_TRY(hipMemsetAsync(ctx->d_misc, 0, 8 * MISC_STRIDE * sizeof(uint32_t), st));

  ShadeParams sp{};
  sp.width = req->width; sp.height = req->height; sp.max_depth = req->max_depth;
  sp.tile_w = tw; sp.tile_h = th; sp.num_bg_spd = (uint32_t)nbg; sp.slots = slots;
  sp.bg_sorted = nbg >= 2;
  for (size_t i = 1; i < nbg; i++)
    if (!(req->bg_spd_wavelengths[i - 1] <= req->bg_spd_wavelengths[i])) sp.bg_sorted = 0;
  sp.tiles = ctx->d_tiles; sp.bg_wl = ctx->d_bg; sp.bg_val = ctx->d_bg + nbg;
  sp.background[0] = req->background[0]; sp.background[1] = req->background[1]; sp.background[2] = req->background[2];
  sp.rec_dense = rec_dense; sp.rec_pool = rec_pool;
  sp.pool_shift = 0;
  while (pool_blocks && (POOL_SHARDS << sp.pool_shift) < pool_blocks) sp.pool_shift++;
  sp.seed = req->seed; sp.out = ctx->d_samples; sp.recs = fwd ? nullptr : ctx->d_recs; sp.mat_const = sc.mat_const; sp.head = misc(ctx, 0);
  sp.num_mc = ctx->num_materials; sp.num_tex = ctx->num_textures; sp.num_spd = ctx->num_spd;
  sp.staged = ctx->num_materials <= MC_LDS && ctx->num_materials <= MAT_LDS && sc.num_lights <= LT_LDS &&
              ctx->num_textures <= TEX_LDS && ctx->num_spd <= SPD_LDS && nbg <= BG_LDS;
  sp.prims_staged = sc.num_prims <= PR_LDS && !(tuning_of(req).flags & IZPI_TUNE_NO_PRIM_LDS);
  if (sp.staged && (req->sampler == IZPI_SAMPLER_SPECTRAL || ctx->num_spd)) sp.staged = 2;  // + the Spectral tables
  // k_shade / k_tail's LDS arena: the prefix of lds_off's layout that this render stages
  sc.lds_bytes = sp.prims_staged ? lds_off::END : sp.staged == 2 ? lds_off::SPECTRAL_END : sp.staged ? lds_off::COLOUR_END : 0;
  sp.pool = rec_pool ? ctx->d_pool : nullptr; sp.pool_ring = rec_pool ? ctx->d_ring : nullptr;
  sp.pool_ctr = rec_pool ? ctx->d_pool_ctr : nullptr;
  sp.counters = ctx->d_counters; sp.cpart = ctx->d_cpart; sp.error = misc(ctx, 1);
  sp.finq = ctx->d_finq;
  WaveParams wp{};
  wp.in = bufs[0]; wp.out = bufs[1]; wp.trace_next = misc(ctx, 2); wp.slots = slots;
  // kind words other than plain main rays: path-length rays, parked entries
  wp.read_kind = !ctx->sc.no_pathlen ? 1u : 0u;  // parked entries: wp.in_park, per pass
  wp.hit_uv = need_uv ? 1u : 0u;
  wp.pool_ctr = sp.pool_ctr;
  wp.cpart = ctx->d_cpart;
  AccumParams ap{};
  ap.num_pixels = num_pixels; ap.spp = req->spp; ap.width = req->width; ap.height = req->height;
  ap.tile_w = tw; ap.tile_h = th; ap.sampler = req->sampler; ap.out_layout = req->out_layout;
  ap.tiles = ctx->d_tiles; ap.samples = ctx->d_samples; ap.running = ctx->d_running; ap.out = out_dev;

  float trace_ms = 0, shade_ms = 0, tail_ms = 0;
  uint32_t launches = 0;
  HIP_TRY(hipEventRecord(ctx->ev0, st));
#define IZPI_RUN(S, M) (fwd ? run_chunks<S, M == MATSET_CONST ? MATSET_BASIC : M, true>(ctx, req, sc, tr, sp, wp, ap, num_pixels, chunk, pool_blocks, &trace_ms, &shade_ms, &tail_ms, &launches) \
                          : run_chunks<S, M, false>(ctx, req, sc, tr, sp, wp, ap, num_pixels, chunk, pool_blocks, &trace_ms, &shade_ms, &tail_ms, &launches))
  // the smallest compiled material set holding the scene's material kinds
  const uint32_t ms = ctx->matset;
  const int set = ms == 0 ? MATSET_BASIC : (ms & ~(uint32_t)MATSET_SURF) == 0 ? MATSET_SURF : MATSET_FULL;
  if (req->sampler == IZPI_SAMPLER_COLOUR)
    rc = compact               ? IZPI_RUN(IZPI_SAMPLER_COLOUR, MATSET_CONST)
         : set == MATSET_BASIC ? IZPI_RUN(IZPI_SAMPLER_COLOUR, MATSET_BASIC)
         : set == MATSET_SURF  ? IZPI_RUN(IZPI_SAMPLER_COLOUR, MATSET_SURF)
                               : IZPI_RUN(IZPI_SAMPLER_COLOUR, MATSET_FULL);
  else
    rc = set == MATSET_BASIC  ? IZPI_RUN(IZPI_SAMPLER_SPECTRAL, MATSET_BASIC)
         : set == MATSET_SURF ? IZPI_RUN(IZPI_SAMPLER_SPECTRAL, MATSET_SURF)
                              : IZPI_RUN(IZPI_SAMPLER_SPECTRAL, MATSET_FULL);
#undef IZPI_RUN
  if (rc) return rc;
  hipLaunchKernelGGL(k_cpart_reduce, dim3(CNT_N), dim3(256), 0, st, ctx->d_cpart, cpart_rows, ctx->d_counters);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev1, st));
  if ((rc = apply_post(ctx, req, out_dev))) return rc;
  HIP_TRY(hipEventSynchronize(ctx->ev1));
  float total_ms = 0;
  HIP_TRY(hipEventElapsedTime(&total_ms, ctx->ev0, ctx->ev1));
  unsigned long long cnt[CNT_N];
  uint32_t misc_w[MISC_STRIDE + 1];
  HIP_TRY(hipMemcpy(cnt, ctx->d_counters, sizeof(cnt), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(misc_w, misc(ctx, 0), sizeof(misc_w), hipMemcpyDeviceToHost));
  izpi_render_stats& s = ctx->last;
  memset(&s, 0, sizeof(s));
  s.rays = cnt[CNT_RAYS]; s.node_visits = cnt[CNT_NODES]; s.tri_tests = cnt[CNT_TRI]; s.sph_tests = cnt[CNT_SPH];
  s.light_tri_tests = cnt[CNT_LTRI]; s.light_sph_tests = cnt[CNT_LSPH];
  s.samples = (uint64_t)num_pixels * req->spp;
  s.kernel_ms = trace_ms; s.shade_ms = shade_ms; s.total_ms = total_ms; s.launches = launches; s.tail_ms = tail_ms;
  s.node_steps = cnt[CNT_NSTEP]; s.prim_steps = cnt[CNT_PSTEP]; s.leaf_shortcuts = cnt[CNT_SHORT];
  s.tail_node_visits = cnt[CNT_TAIL_NODES]; s.tail_tri_tests = cnt[CNT_TAIL_TRI]; s.tail_sph_tests = cnt[CNT_TAIL_SPH];
  s.parks = cnt[CNT_PARK];
  s.workspace_bytes = workspace_bytes(ctx);
  s.scene_bytes = ctx->scene_bytes;
  s.slots = slots; s.rec_dense = fwd ? 0 : rec_dense; s.pool_blocks = pool_blocks; s.chunk_spp = chunk;
  s.alloc_ms = alloc_ms;
  if (rec_pool && s.parks * 64 > s.rays && pool_blocks < slots) ctx->pool_grow++;
#ifdef IZPI_SHADE_CLOCKS
  fprintf(stderr, "IZPI_SHADE_CLOCKS item %llu refill %llu push %llu mat %llu finish %llu mix %llu lpdf %llu entry %llu tex %llu "
          "res_barrier1 %llu res_atomics %llu res_barrier2 %llu (wave cycles; res_atomics: thread 0 only)\n",
          cnt[CNT_SCLK_ITEM], cnt[CNT_SCLK_REFILL], cnt[CNT_SCLK_PUSH], cnt[CNT_SCLK_MAT], cnt[CNT_SCLK_FIN],
          cnt[CNT_SCLK_MIX], cnt[CNT_SCLK_LPDF], cnt[CNT_SCLK_ENTRY], cnt[CNT_SCLK_TEX], cnt[CNT_SCLK_RB1],
          cnt[CNT_SCLK_RATOM], cnt[CNT_SCLK_RB2]);
#endif
#ifdef IZPI_SHADOW
  fprintf(stderr, "IZPI_SHADOW spill_stores %llu spill_loads %llu (entries)\n", cnt[CNT_CLK_REFILL], cnt[CNT_CLK_NODE]);
#endif
#ifdef IZPI_TRACE_CLOCKS
  fprintf(stderr, "IZPI_TRACE_CLOCKS refill %llu node %llu prim %llu advance %llu (wave cycles)\n", cnt[CNT_CLK_REFILL],
          cnt[CNT_CLK_NODE], cnt[CNT_CLK_PRIM], cnt[CNT_CLK_ADV]);
#endif
  const uint32_t guard = misc_w[MISC_STRIDE];  // the error word
  if (guard) {
    ctx->err = guard & 1u   ? "device guard: traversal stack overflow"
               : guard & 2u ? "device guard: unknown material kind"
                              : "device guard: no overflow record block in k_tail";
    return IZPI_ERR_DEVICE;
  }
  return IZPI_OK;
}

// ------------------------------------------------------------------ multi-GPU
// The frame is split into G shares: tile t (in common.Tiles' spiral order) goes to share
// t % G, so the costly centre tiles spread over all devices. Share r is rendered packed
// (IZPI_OUT_PACKED) into d_share, padded to the largest share's size so that one gather
// moves equal blocks; the root scatters share r's tiles from block r into the canvas.
struct Shares {
  std::vector<uint32_t> all;  // the frame's tiles, [n][4]
  uint32_t n = 1;             // shares
  size_t block = 0;           // doubles per (padded) share
  std::vector<uint32_t> mine(uint32_t r) const {
    std::vector<uint32_t> t(all.size());
    t.resize(4 * (size_t)izpi_host_share_tiles(all.data(), (uint32_t)(all.size() / 4), r, n, t.data()));
    return t;
  }
};

size_t share_block(size_t ntiles, uint32_t tw, uint32_t th, uint32_t n) { return ((ntiles + n - 1) / n) * (size_t)tw * th * 4; }

int make_shares(izpi_ctx* ctx, const izpi_render_req* req, uint32_t n, Shares& sh) {
  if (!req || req->width == 0 || req->height == 0) { ctx->err = "invalid render request"; return IZPI_ERR_INVALID; }
  if (req->out_layout != IZPI_OUT_CANVAS) { ctx->err = "multi-GPU renders produce a canvas (IZPI_OUT_CANVAS)"; return IZPI_ERR_INVALID; }
  int rc = request_tiles(ctx, req, sh.all);
  if (rc) return rc;
  uint32_t tw = 0, th = 0;
  if (!validate_tiles(req, sh.all.data(), (uint32_t)(sh.all.size() / 4), &tw, &th)) {
    ctx->err = "tiles must be non-empty, in bounds and equal-sized";
    return IZPI_ERR_INVALID;
  }
  sh.n = n;
  const size_t ntiles = sh.all.size() / 4;
  sh.block = share_block(ntiles, tw, th, n);
  return IZPI_OK;
}

// Render share r of the frame into ctx->d_share (stats in ctx->last).
int render_share(izpi_ctx* ctx, const izpi_render_req* req, const Shares& sh, uint32_t r) {
  int rc = grow(ctx, (void**)&ctx->d_share, &ctx->share_cap, sh.block * sizeof(double));
  if (rc) return rc;
  const std::vector<uint32_t> mine = sh.mine(r);
  memset(&ctx->last, 0, sizeof(ctx->last));
  if (mine.empty()) return IZPI_OK;  // more shares than tiles: an empty block joins the gather
  izpi_render_req q = *req;
  q.num_tiles = (uint32_t)(mine.size() / 4);
  q.tiles = mine.data();
  q.out_layout = IZPI_OUT_PACKED;
  q.post = IZPI_POST_NONE;
  return render_impl(ctx, &q, ctx->d_share);
}

// Root: scatter every share's packed tiles from d_gather into the canvas (row H - y,
// rgb.go:41), then Render's post-processing of the assembled frame.
int assemble(izpi_ctx* ctx, const izpi_render_req* req, const Shares& sh, double* canvas_dev) {
  izpi_ctx* root = ctx;  // (HIP_TRY reports into ctx)
  hipStream_t st = root->stream;
  for (uint32_t r = 0; r < sh.n; r++) {
    const std::vector<uint32_t> t = sh.mine(r);
    if (t.empty()) continue;
    const uint32_t nt = (uint32_t)(t.size() / 4), tw = t[2] - t[0] + 1, th = t[3] - t[1] + 1;
    int rc = grow(root, (void**)&root->d_utiles, &root->utiles_cap, sh.all.size() * sizeof(uint32_t));
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(root->d_utiles, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    const uint32_t np = nt * tw * th;
    hipLaunchKernelGGL(k_unpack, dim3((np + 255) / 256), dim3(256), 0, st, root->d_utiles, np, tw, th, req->width,
                       req->height, root->d_gather + (size_t)r * sh.block, canvas_dev);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));  // d_utiles is reused by the next share
  }
  int rc = apply_post(root, req, canvas_dev);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(st));
  return IZPI_OK;
}

}  // namespace

// One context per device of a single-process multi-GPU render (izpi_gpu_multi_*).
struct izpi_multi {
  std::vector<izpi_ctx*> ctx;
  std::string err;
};

extern "C" {

int izpi_gpu_open(int device, izpi_ctx** out) {
  if (!out) return IZPI_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0 || device < 0 || device >= n) return IZPI_ERR_HIP;
  if (hipSetDevice(device) != hipSuccess) return IZPI_ERR_HIP;
  izpi_ctx* ctx = new izpi_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  bool ok = hipGetDeviceProperties(&prop, device) == hipSuccess;
  ctx->num_cus = ok ? prop.multiProcessorCount : 0;
  ok = ok && hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) == hipSuccess &&
       hipEventCreate(&ctx->ev0) == hipSuccess && hipEventCreate(&ctx->ev1) == hipSuccess &&
       hipEventCreate(&ctx->ev2) == hipSuccess && hipEventCreate(&ctx->ev3) == hipSuccess &&
       hipHostMalloc((void**)&ctx->h_count, 9 * MISC_STRIDE * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess &&
       hipMalloc((void**)&ctx->d_misc, 8 * MISC_STRIDE * sizeof(uint32_t)) == hipSuccess &&
       hipMalloc((void**)&ctx->d_pool_ctr, POOL_SHARDS * POOL_CTR_STRIDE * sizeof(unsigned long long)) == hipSuccess &&
       hipMalloc((void**)&ctx->d_counters, CNT_N * sizeof(unsigned long long)) == hipSuccess;
  for (int i = 0; ok && i < 3 * IZPI_PASS_BATCH; i++) ok = hipEventCreate(&ctx->evb[i]) == hipSuccess;
  if (!ok) {
    izpi_gpu_close(ctx);
    return IZPI_ERR_HIP;
  }
  *out = ctx;
  return IZPI_OK;
}

int izpi_gpu_close(izpi_ctx* ctx) {
  if (!ctx) return IZPI_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  free_scene(ctx);
  void* bufs[] = {ctx->d_samples, ctx->d_recs, ctx->d_pool, ctx->d_ring, ctx->d_pool_ctr, ctx->d_running, ctx->d_out,
                  ctx->d_tiles, ctx->d_utiles, ctx->d_bg, ctx->d_misc, ctx->d_counters, ctx->d_state,
                  ctx->d_spill, ctx->d_post, ctx->d_share,
                  ctx->d_gather, ctx->d_status, ctx->d_cpart, ctx->d_finq};
  for (void* p : bufs) if (p) (void)hipFree(p);
  if (ctx->h_count) (void)hipHostFree(ctx->h_count);
  if (ctx->stall_host) (void)hipHostFree(ctx->stall_host);
  for (int i = 0; i < 3 * IZPI_PASS_BATCH; i++) if (ctx->evb[i]) (void)hipEventDestroy(ctx->evb[i]);
  hipEvent_t evs[] = {ctx->ev0, ctx->ev1, ctx->ev2, ctx->ev3};
  for (hipEvent_t ev : evs) if (ev) (void)hipEventDestroy(ev);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return IZPI_OK;
}

const char* izpi_gpu_last_error(izpi_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int izpi_gpu_upload_scene(izpi_ctx* ctx, const izpi_scene_desc* d) {
  if (!ctx || !d) return IZPI_ERR_INVALID;
  // the scene descriptor is laid out alike in ABI 1 and 2
  if (d->abi_version < 1 || d->abi_version > IZPI_ABI_VERSION) { ctx->err = "ABI version mismatch"; return IZPI_ERR_INVALID; }
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  free_scene(ctx);
  const uint32_t nt = d->num_tris, ns = d->num_spheres;
  // ---- BVH4: split reference nodes into inner nodes and leaf records
  std::vector<int32_t> ref(d->num_nodes);
  uint32_t n_inner = 0;
  for (uint32_t k = 0; k < d->num_nodes; k++) {
    const izpi_bvh4_node& n = d->nodes[k];
    if (n.prim_count[0] > 0) {
      for (int i = 1; i < 4; i++)
        if (n.child[i] != -1) { ctx->err = "leaf node with more than one slot"; return IZPI_ERR_INVALID; }
      const int32_t st = n.child[0], cnt = n.prim_count[0];
      if (st < 0 || (uint64_t)st + (uint64_t)cnt > d->num_prims) { ctx->err = "leaf primitive range out of bounds"; return IZPI_ERR_INVALID; }
      if (cnt > 7 || st >= (1 << 27)) { ctx->err = "leaf too large for the leaf-ref encoding"; return IZPI_ERR_UNSUPPORTED; }
      ref[k] = make_leaf_ref(st, cnt);
    } else {
      for (int i = 0; i < 4; i++)
        if (n.prim_count[i] != 0) { ctx->err = "inner node with a primitive slot"; return IZPI_ERR_INVALID; }
      ref[k] = (int32_t)n_inner++;
    }
  }
  std::vector<GInner> inner(std::max<uint32_t>(1, n_inner));  // >= 1: k_trace2's leaf lanes read a dummy inner node
  std::vector<GLeaf> leaves(std::max<uint32_t>(1, d->num_prims));  // indexed by first primitive
  uint32_t leaf_shortcut = 1;
  for (uint32_t k = 0; k < d->num_nodes; k++) {
    const izpi_bvh4_node& n = d->nodes[k];
    if (ref[k] <= -2) {
      GLeaf& L = leaves[(size_t)leaf_start(ref[k])];
      L.mn[0] = n.min_x[0]; L.mn[1] = n.min_y[0]; L.mn[2] = n.min_z[0];
      L.mx[0] = n.max_x[0]; L.mx[1] = n.max_y[0]; L.mx[2] = n.max_z[0];
      L.start = n.child[0]; L.count = n.prim_count[0];
    } else {
      GInner& g = inner[(size_t)ref[k]];
      memcpy(g.mnx, n.min_x, 16); memcpy(g.mny, n.min_y, 16); memcpy(g.mnz, n.min_z, 16);
      memcpy(g.mxx, n.max_x, 16); memcpy(g.mxy, n.max_y, 16); memcpy(g.mxz, n.max_z, 16);
      for (int i = 0; i < 4; i++) {
        int32_t c = n.child[i];
        if (c != -1 && (c < 0 || (uint32_t)c >= d->num_nodes)) { ctx->err = "child index out of bounds"; return IZPI_ERR_INVALID; }
        g.child[i] = c == -1 ? -1 : ref[(size_t)c];
        g.pad[i] = 0;
        if (c >= 0 && ref[(size_t)c] <= -2) {
          // a leaf's re-test (A10) may be skipped only if its slot-0 box is bit-identical
          // to this slot's box (flattenBVH4 converts the same node.box twice, bvh4.go:745-781)
          const izpi_bvh4_node& lnode = d->nodes[(size_t)c];
          const float pb[6] = {n.min_x[i], n.min_y[i], n.min_z[i], n.max_x[i], n.max_y[i], n.max_z[i]};
          const float lb[6] = {lnode.min_x[0], lnode.min_y[0], lnode.min_z[0], lnode.max_x[0], lnode.max_y[0], lnode.max_z[0]};
          if (memcmp(pb, lb, sizeof(pb)) != 0) leaf_shortcut = 0;
        }
      }
    }
  }
  // ---- primitives in leaf order
  std::vector<GPrim> prims(d->num_prims);
  std::vector<GShade> shade(d->num_prims);
  for (uint32_t k = 0; k < d->num_prims; k++) {
    const uint32_t r = d->prim_ref[k], kind = IZPI_PRIM_KIND(r), idx = IZPI_PRIM_INDEX(r);
    GPrim& g = prims[k];
    g.kind = kind; g.index = idx;
    GShade& gs = shade[k];
    memset(&gs, 0, sizeof(gs));
    gs.ref = r;
    if (kind == IZPI_PRIM_TRIANGLE) {
      if (idx >= nt) { ctx->err = "triangle ref out of range"; return IZPI_ERR_INVALID; }
      memcpy(gs.n, d->tri_normal + 3 * (size_t)idx, 24);
      gs.mk = d->tri_mat[idx];
      memcpy(g.a, d->tri_v0 + 3 * (size_t)idx, 24); memcpy(g.a + 3, d->tri_e1 + 3 * (size_t)idx, 24);
      memcpy(g.a + 6, d->tri_e2 + 3 * (size_t)idx, 24);
    } else {
      if (idx >= ns) { ctx->err = "sphere ref out of range"; return IZPI_ERR_INVALID; }
      gs.mk = d->sph_mat[idx];
      memcpy(g.a, d->sph_center0 + 3 * (size_t)idx, 24); memcpy(g.a + 3, d->sph_center1 + 3 * (size_t)idx, 24);
      g.a[6] = d->sph_radius[idx]; g.a[7] = d->sph_time[2 * (size_t)idx]; g.a[8] = d->sph_time[2 * (size_t)idx + 1];
    }
  }
  // ---- lights
  std::vector<GLight> lights(d->num_lights);
  for (uint32_t i = 0; i < d->num_lights; i++) {
    GLight& L = lights[i];
    memset(&L, 0, sizeof(L));
    const uint32_t r = d->light_ref[i], kind = IZPI_PRIM_KIND(r), idx = IZPI_PRIM_INDEX(r);
    L.kind = kind; L.index = idx;
    if (kind == IZPI_PRIM_TRIANGLE) {
      if (idx >= nt) { ctx->err = "light triangle out of range"; return IZPI_ERR_INVALID; }
      const izpi_material& m = d->materials[d->tri_mat[idx]];
      if (m.kind == IZPI_MAT_PBR && m.normal_tex >= 0) { ctx->err = "normal-mapped light"; return IZPI_ERR_UNSUPPORTED; }
      memcpy(L.v0, d->tri_v0 + 3 * (size_t)idx, 24); memcpy(L.v1, d->tri_v1 + 3 * (size_t)idx, 24);
      memcpy(L.v2, d->tri_v2 + 3 * (size_t)idx, 24); memcpy(L.e1, d->tri_e1 + 3 * (size_t)idx, 24);
      memcpy(L.e2, d->tri_e2 + 3 * (size_t)idx, 24); memcpy(L.n, d->tri_normal + 3 * (size_t)idx, 24);
      L.area = d->tri_area[idx];
    } else {
      if (idx >= ns) { ctx->err = "light sphere out of range"; return IZPI_ERR_INVALID; }
      memcpy(L.c0, d->sph_center0 + 3 * (size_t)idx, 24); memcpy(L.c1, d->sph_center1 + 3 * (size_t)idx, 24);
      L.radius = d->sph_radius[idx]; L.t0 = d->sph_time[2 * (size_t)idx]; L.t1 = d->sph_time[2 * (size_t)idx + 1];
      // Sphere.center(0) (sphere.go:125-127) with the device's operation order:
      // c0 + (c1 - c0) * ((0 - t0) / (t1 - t0)), computed once here
      const double k = (0.0 - L.t0) / (L.t1 - L.t0);
      for (int q = 0; q < 3; q++) L.cz[q] = L.c0[q] + (L.c1[q] - L.c0[q]) * k;
    }
  }
  // ---- material flags: bit0 a texture of the material reads (u,v); bit1 usable by
  // the Colour sampler; bit2 usable by the Spectral sampler (the reference would
  // dereference a nil texture otherwise).
  std::vector<uint32_t> mflags(d->num_materials, 0);
  ctx->mat_ok_rgb = ctx->mat_ok_spectral = true;
  ctx->basic_materials = true;
  ctx->matset = 0;
  ctx->pool_grow = 0;
  for (uint32_t i = 0; i < d->num_materials; i++) {
    const izpi_material& m = d->materials[i];
    const int32_t ids[] = {m.albedo_tex, m.spectral_tex, m.normal_tex, m.roughness_tex, m.metalness_tex, m.absorb_tex};
    for (int32_t t : ids) {
      if (t < -1 || t >= (int32_t)d->num_textures) { ctx->err = "texture index out of range"; return IZPI_ERR_INVALID; }
      if (t >= 0 && (d->textures[t].kind == IZPI_TEX_IMAGE || d->textures[t].kind == IZPI_TEX_SPECTRAL_IMAGE)) mflags[i] |= 1u;
    }
    // a SpectralImage is made for PBR albedos (transport.go:486-497) and reads the hit's
    // (u, v): Lambert / DiffuseLight / PBR spectral textures only
    for (int32_t t : {m.normal_tex, m.roughness_tex, m.metalness_tex, m.absorb_tex, m.albedo_tex})
      if (t >= 0 && d->textures[t].kind == IZPI_TEX_SPECTRAL_IMAGE) { ctx->err = "SpectralImage outside a spectral albedo"; return IZPI_ERR_INVALID; }
    if (m.spectral_tex >= 0 && d->textures[m.spectral_tex].kind == IZPI_TEX_SPECTRAL_IMAGE && m.kind != IZPI_MAT_LAMBERT &&
        m.kind != IZPI_MAT_DIFFUSE_LIGHT && m.kind != IZPI_MAT_PBR) {
      ctx->err = "SpectralImage outside a spectral albedo";
      return IZPI_ERR_INVALID;
    }
    auto is_rgb = [&](int32_t t) { return t >= 0 && (d->textures[t].kind == IZPI_TEX_CONSTANT || d->textures[t].kind == IZPI_TEX_IMAGE); };
    auto is_spec = [&](int32_t t) {
      return t >= 0 && (d->textures[t].kind == IZPI_TEX_SPECTRAL_GAUSSIAN || d->textures[t].kind == IZPI_TEX_SPECTRAL_TABULATED ||
                        d->textures[t].kind == IZPI_TEX_SPECTRAL_IMAGE);
    };
    auto opt_rgb = [&](int32_t t) { return t == -1 || is_rgb(t); };
    bool rgb = false, spec = false;
    switch (m.kind) {
      case IZPI_MAT_LAMBERT: case IZPI_MAT_DIFFUSE_LIGHT: rgb = is_rgb(m.albedo_tex); spec = is_spec(m.spectral_tex); break;
      case IZPI_MAT_DIELECTRIC: rgb = true; spec = is_spec(m.spectral_tex) && (m.absorb_tex == -1 || is_spec(m.absorb_tex)); break;
      case IZPI_MAT_METAL: rgb = spec = true; break;
      case IZPI_MAT_ISOTROPIC: rgb = spec = is_rgb(m.albedo_tex); break;  // SpectralScatter reads the RGB albedo's X
      case IZPI_MAT_PBR: {
        bool aux = opt_rgb(m.normal_tex) && opt_rgb(m.roughness_tex) && opt_rgb(m.metalness_tex);
        rgb = aux && is_rgb(m.albedo_tex);
        spec = aux && (is_spec(m.spectral_tex) || is_rgb(m.albedo_tex));
        break;
      }
      default: ctx->err = "unknown material kind"; return IZPI_ERR_INVALID;
    }
    if (m.kind != IZPI_MAT_LAMBERT && m.kind != IZPI_MAT_DIFFUSE_LIGHT) ctx->basic_materials = false;
    ctx->matset |= m.kind == IZPI_MAT_DIELECTRIC ? MS_DIEL : m.kind == IZPI_MAT_METAL ? MS_METAL
                 : m.kind == IZPI_MAT_PBR ? MS_PBR : m.kind == IZPI_MAT_ISOTROPIC ? MS_ISO : 0u;
    if (rgb) mflags[i] |= 2u; else ctx->mat_ok_rgb = false;
    if (spec) mflags[i] |= 4u; else ctx->mat_ok_spectral = false;
  }
  // ---- material essentials in the per-primitive shade records
  // (gs.mk holds the bare material index until here)
  if (d->num_materials >= (1u << 24)) { ctx->err = "too many materials"; return IZPI_ERR_INVALID; }
  std::vector<double4> mconst(std::max<uint32_t>(1, d->num_materials), make_double4(0, 0, 0, 0));
  std::vector<uint32_t> mcflags(d->num_materials, 0);
  for (uint32_t i = 0; i < d->num_materials; i++) {
    const izpi_material& m = d->materials[i];
    mcflags[i] = (mflags[i] & 1u) ? 2u : 0u;
    if ((m.kind == IZPI_MAT_LAMBERT || m.kind == IZPI_MAT_DIFFUSE_LIGHT) && m.albedo_tex >= 0 &&
        d->textures[m.albedo_tex].kind == IZPI_TEX_CONSTANT) {
      const double* v = d->textures[m.albedo_tex].value;
      mconst[i] = make_double4(v[0], v[1], v[2], 0.0);
      mcflags[i] |= 1u;
    }
  }
  ctx->const_albedo = true;
  ctx->any_uv = false;
  for (uint32_t i = 0; i < d->num_materials; i++)
    if (mflags[i] & 1u) ctx->any_uv = true;
  for (uint32_t i = 0; i < d->num_materials; i++)
    if ((d->materials[i].kind == IZPI_MAT_LAMBERT || d->materials[i].kind == IZPI_MAT_DIFFUSE_LIGHT) && !(mcflags[i] & 1u))
      ctx->const_albedo = false;
  for (GShade& gs : shade) {
    const uint32_t mat = gs.mk;
    if (mat >= d->num_materials) { ctx->err = "material index out of range"; return IZPI_ERR_INVALID; }
    if (d->materials[mat].kind >= 64u) { ctx->err = "unknown material kind"; return IZPI_ERR_INVALID; }
    gs.mk = mat << 8 | d->materials[mat].kind << 2 | mcflags[mat];
  }
  // ---- upload
  DevScene& sc = ctx->sc;
  memset(&sc, 0, sizeof(sc));
  GInner* di; GLeaf* dl; GPrim* dp; GShade* dsh; GLight* dlt; GTriTex* dtt = nullptr;
  double *dtex, *dswl, *dsv;
  izpi_material* dm; izpi_texture* dtx;
  UP(inner.data(), inner.size(), &di);
  UP(leaves.data(), leaves.size(), &dl);
  UP(prims.data(), prims.size(), &dp);
  UP(shade.data(), shade.size(), &dsh);
  for (uint32_t i = 0; i < d->num_materials; i++)
    if (d->materials[i].kind == IZPI_MAT_PBR && d->materials[i].normal_tex >= 0 && nt && (!d->tri_tangent || !d->tri_bitangent)) {
      ctx->err = "a PBR normal map needs the triangles' tangents and bitangents";
      return IZPI_ERR_INVALID;
    }
  // triangle UVs and tangent frames in leaf order (shading reads them for image textures
  // and normal maps; izpi_gpu_trace's hit records carry the UVs)
  if (d->num_prims && (d->tri_uv || d->tri_tangent || d->tri_bitangent)) {
    std::vector<GTriTex> tt(d->num_prims);
    for (uint32_t k = 0; k < d->num_prims; k++) {
      memset(&tt[k], 0, sizeof(GTriTex));
      const uint32_t r = d->prim_ref[k];
      if (IZPI_PRIM_KIND(r) != IZPI_PRIM_TRIANGLE) continue;
      const size_t ti = IZPI_PRIM_INDEX(r);
      if (d->tri_uv) memcpy(tt[k].uv, d->tri_uv + 6 * ti, 48);
      if (d->tri_tangent) memcpy(tt[k].tg, d->tri_tangent + 3 * ti, 24);
      if (d->tri_bitangent) memcpy(tt[k].bt, d->tri_bitangent + 3 * ti, 24);
    }
    UP(tt.data(), tt.size(), &dtt);
  }
  UP(lights.data(), lights.size(), &dlt);
  UP(d->materials, d->num_materials, &dm);
  double4* dmc;
  UP(mconst.data(), mconst.size(), &dmc);
  for (uint32_t i = 0; i < d->num_textures; i++) {
    const izpi_texture& t = d->textures[i];
    if (t.kind != IZPI_TEX_IMAGE && t.kind != IZPI_TEX_SPECTRAL_IMAGE) continue;
    if (t.width == 0 || t.height == 0 || t.texel_offset + 4ull * t.width * t.height > d->num_texels || !d->texels) {
      ctx->err = "image texture outside the texel array";
      return IZPI_ERR_INVALID;
    }
  }
  // device copy of the textures: pad0 = 1 marks a tabulated SPD with non-decreasing
  // wavelengths, which tex_spectral searches by bisection; pad0 = 2 one whose wavelengths
  // are also near-uniform (entry j within half a step of wl[0] + j * step), whose interval
  // tex_spectral guesses from lambda with value[0] = wl[0] and value[1] = 1 / step
  std::vector<izpi_texture> texs(d->textures, d->textures + d->num_textures);
  for (izpi_texture& t : texs) {
    t.pad0 = 0;
    if (t.kind != IZPI_TEX_SPECTRAL_TABULATED || t.spd_count < 2) continue;  // n = 1: the scan returns 0.0
    if ((uint64_t)t.spd_offset + t.spd_count > d->num_spd) { ctx->err = "SPD range out of bounds"; return IZPI_ERR_INVALID; }
    const double* wl = d->spd_wavelengths + t.spd_offset;
    const uint32_t n = t.spd_count;
    bool sorted = true;
    for (uint32_t i = 1; i < n; i++)
      if (!(wl[i - 1] <= wl[i])) sorted = false;
    t.pad0 = sorted ? 1u : 0u;
    const double span = wl[n - 1] - wl[0];
    if (!sorted || !(span > 0) || !std::isfinite(span)) continue;
    const double scale = (double)(n - 1) / span;
    bool uniform = std::isfinite(scale);
    for (uint32_t i = 0; i < n && uniform; i++)
      if (!(std::fabs((wl[i] - wl[0]) * scale - (double)i) <= 0.5)) uniform = false;
    if (uniform) { t.pad0 = 2; t.value[0] = wl[0]; t.value[1] = scale; }
  }
  // texels in their device storage form (TexSlot): every image texture gets its own run,
  // RGBA runs 32-B aligned; a texture whose R, G and B are bit-identical in every texel is
  // stored as one double per texel
  std::vector<double> texels;
  std::vector<uint32_t> tex_fmt(d->num_textures, TEXF_OTHER);
  for (uint32_t i = 0; i < d->num_textures; i++) {
    izpi_texture& t = texs[i];
    if (t.kind != IZPI_TEX_IMAGE && t.kind != IZPI_TEX_SPECTRAL_IMAGE) continue;
    const double* src = d->texels + t.texel_offset;
    const uint64_t np = (uint64_t)t.width * t.height;
    bool gray = t.kind == IZPI_TEX_IMAGE;
    for (uint64_t k = 0; k < np && gray; k++)
      gray = memcmp(src + 4 * k, src + 4 * k + 1, 8) == 0 && memcmp(src + 4 * k, src + 4 * k + 2, 8) == 0;
    texels.resize((texels.size() + 3) & ~(size_t)3);
    t.texel_offset = texels.size();
    if (gray) {
      for (uint64_t k = 0; k < np; k++) texels.push_back(src[4 * k]);
    } else {
      texels.insert(texels.end(), src, src + 4 * np);
    }
    if (t.kind == IZPI_TEX_IMAGE) t.pad0 = tex_fmt[i] = gray ? TEXF_GRAY : TEXF_RGBA;
  }
  // the materials' texture slots (albedo, normal, roughness, metalness)
  std::vector<MatTex> mtex(std::max<uint32_t>(1, d->num_materials));
  for (uint32_t i = 0; i < d->num_materials; i++) {
    const izpi_material& m = d->materials[i];
    const int32_t ids[4] = {m.albedo_tex, m.normal_tex, m.roughness_tex, m.metalness_tex};
    for (int k = 0; k < 4; k++) {
      TexSlot& sl = mtex[i].s[k];
      const int32_t id = ids[k];
      if (id < 0) { sl.off = 0; sl.w = 0; sl.hf = (uint32_t)TEXF_NONE << 30; continue; }
      const izpi_texture& t = texs[id];
      if (tex_fmt[id] <= TEXF_GRAY && t.height < (1u << 30)) {
        sl.off = t.texel_offset; sl.w = t.width; sl.hf = t.height | tex_fmt[id] << 30;
      } else {
        sl.off = (uint64_t)id; sl.w = 0; sl.hf = (uint32_t)TEXF_OTHER << 30;
      }
    }
  }
  MatTex* dmt;
  UP(mtex.data(), mtex.size(), &dmt);
  UP(texs.data(), d->num_textures, &dtx);
  if (texels.empty()) texels.push_back(0.0);
  UP(texels.data(), texels.size(), &dtex);
  UP(d->spd_wavelengths, d->num_spd, &dswl);
  UP(d->spd_values, d->num_spd, &dsv);
  sc.num_inner = n_inner; sc.num_prims = d->num_prims;
#ifdef IZPI_SHADOW
  {
    GInner* si; GLeaf* sl; GPrim* sp;
    UP(inner.data(), inner.size(), &si);
    UP(leaves.data(), leaves.size(), &sl);
    UP(prims.data(), prims.size(), &sp);
    sc.sh_inner = si; sc.sh_leaves = sl; sc.sh_prims = sp;
  }
#endif
  sc.inner = di; sc.leaves = dl; sc.prims = dp; sc.shade = dsh; sc.tritex = dtt; sc.lights = dlt; sc.materials = dm;
  sc.mat_const = dmc; sc.mat_tex = dmt; sc.textures = dtx; sc.texels = dtex; sc.spd_wl = dswl; sc.spd_val = dsv;
  sc.root = d->num_nodes ? ref[0] : -1;
  sc.num_lights = d->num_lights;
  sc.tri_only = d->num_spheres == 0 ? 1u : 0u;
  {  // time_free: no sphere moves, so Sphere.center(time) == center(time0) for every ray time
     // (c1 == c0 finite: (c1 - c0) * x = +0 for the x >= 0 every camera time gives)
    bool tf = true;
    const double tmin_cam = std::min(d->camera.time0, d->camera.time1);
    if (!std::isfinite(d->camera.time0) || !std::isfinite(d->camera.time1)) tf = false;
    for (uint32_t i = 0; tf && i < d->num_spheres; i++) {
      const double* c0 = d->sph_center0 + 3 * (size_t)i;
      const double* c1 = d->sph_center1 + 3 * (size_t)i;
      const double t0 = d->sph_time[2 * (size_t)i], t1 = d->sph_time[2 * (size_t)i + 1];
      for (int k = 0; k < 3; k++)
        if (!std::isfinite(c0[k]) || memcmp(c0 + k, c1 + k, sizeof(double)) != 0) tf = false;
      if (!std::isfinite(t0) || !std::isfinite(t1) || !(t1 > t0) || !(tmin_cam >= t0)) tf = false;
    }
    sc.time_free = tf ? 1u : 0u;
  }
  sc.no_pathlen = 1;
  for (uint32_t i = 0; i < d->num_materials; i++)
    if (d->materials[i].kind == IZPI_MAT_DIELECTRIC) sc.no_pathlen = 0;
  sc.leaf_shortcut = leaf_shortcut;
  sc.nan_free_bounds = 1;
  for (const GInner& g : inner) {
    const float* f = g.mnx;  // the 24 bounds are contiguous
    for (int i = 0; i < 24; i++) if (f[i] != f[i]) sc.nan_free_bounds = 0;
  }
  for (const GLeaf& L : leaves)  // leaf re-tests run through the same 4-slot test
    for (int i = 0; i < 3; i++) if (L.mn[i] != L.mn[i] || L.mx[i] != L.mx[i]) sc.nan_free_bounds = 0;
  sc.cam = d->camera;
  // traversal stack bound (see host_scene.cpp stack_bound)
  {
    std::vector<uint32_t> best(d->num_nodes, 0);
    for (size_t k = d->num_nodes; k-- > 0;) {
      const izpi_bvh4_node& n = d->nodes[k];
      if (n.prim_count[0] > 0) continue;
      uint32_t valid = 0, deepest = 0;
      for (int i = 0; i < 4; i++) {
        if (n.child[i] < 0) continue;
        valid++;
        if ((uint32_t)n.child[i] <= k) { ctx->err = "BVH4 nodes not in pre-order"; return IZPI_ERR_INVALID; }
        deepest = std::max(deepest, best[(size_t)n.child[i]]);
      }
      best[k] = (valid ? valid - 1 : 0) + deepest;
    }
    ctx->stack_needed = d->num_nodes ? best[0] : 0;
    ctx->num_prims = d->num_prims;
  }
  ctx->have_scene = true;
  ctx->sizing_valid = false;  // per-slot sizes depend on the scene
  ctx->num_textures = d->num_textures;
  ctx->num_materials = d->num_materials;
  ctx->num_spd = d->num_spd;
  return IZPI_OK;
}

uint64_t izpi_gpu_output_bytes(const izpi_render_req* req) {
  if (!req) return 0;
  if (req->out_layout == IZPI_OUT_PACKED && req->num_tiles) {
    uint64_t px = 0;
    for (uint32_t i = 0; i < req->num_tiles; i++) {
      const uint32_t* t = req->tiles + 4 * i;
      px += (uint64_t)(t[2] - t[0] + 1) * (t[3] - t[1] + 1);
    }
    return px * 4 * sizeof(double);
  }
  return (uint64_t)req->width * req->height * 4 * sizeof(double);
}

int izpi_gpu_render_device(izpi_ctx* ctx, const izpi_render_req* req, double* out_dev, izpi_render_stats* stats) {
  if (!ctx) return IZPI_ERR_INVALID;
  if (!out_dev) { ctx->err = "null output"; return IZPI_ERR_INVALID; }
  HIP_TRY(hipSetDevice(ctx->device));
  int rc = render_impl(ctx, req, out_dev);
  if (stats) *stats = ctx->last;
  return rc;
}

int izpi_gpu_render(izpi_ctx* ctx, const izpi_render_req* req, double* out_host, izpi_render_stats* stats) {
  if (!ctx) return IZPI_ERR_INVALID;
  if (!out_host || !req) { ctx->err = "null argument"; return IZPI_ERR_INVALID; }
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t bytes = izpi_gpu_output_bytes(req);
  int rc = grow(ctx, (void**)&ctx->d_out, &ctx->out_cap, bytes);
  if (rc) return rc;
  // start from the caller's buffer so untouched pixels keep their values
  HIP_TRY(hipMemcpyAsync(ctx->d_out, out_host, bytes, hipMemcpyHostToDevice, ctx->stream));
  rc = render_impl(ctx, req, ctx->d_out);
  if (stats) *stats = ctx->last;
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_host, ctx->d_out, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return IZPI_OK;
}

int izpi_gpu_spectral_post(izpi_ctx* ctx, const double* xyz_dev, double* rgba_dev, uint32_t width, uint32_t height,
                           double exposure) {
  if (!ctx) return IZPI_ERR_INVALID;
  if (!xyz_dev || !rgba_dev || xyz_dev == rgba_dev || width == 0 || height == 0) {
    ctx->err = "spectral_post: bad arguments (buffers must be distinct device canvases)";
    return IZPI_ERR_INVALID;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  dim3 g((width + 15) / 16, (height + 15) / 16);
  hipLaunchKernelGGL(k_spectral_post, g, dim3(256), 0, ctx->stream, xyz_dev, rgba_dev, width, height, exposure);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return IZPI_OK;
}

int izpi_gpu_build_bvh4(izpi_ctx* ctx, const double* boxes, uint32_t n, uint32_t leaf_max, uint32_t method,
                        izpi_bvh4_node* nodes, uint32_t max_nodes, uint32_t* num_nodes, uint32_t* order, double* build_ms) {
  if (!ctx) return IZPI_ERR_INVALID;
  if (num_nodes) *num_nodes = 0;
  if ((n && (!boxes || !nodes || !order)) || !num_nodes || (uint64_t)max_nodes < 2ull * n) {
    ctx->err = "build_bvh4: bad arguments (nodes needs 2n entries)";
    return IZPI_ERR_INVALID;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  std::vector<izpi_bvh4_node> out;
  std::vector<uint32_t> ord;
  float ms = 0;
  const int rc = izpi_bvh::build(ctx->stream, boxes, n, leaf_max, method, out, ord, &ms, ctx->err);
  if (rc) return rc;
  if (!out.empty()) memcpy(nodes, out.data(), out.size() * sizeof(izpi_bvh4_node));
  if (!ord.empty()) memcpy(order, ord.data(), ord.size() * sizeof(uint32_t));
  *num_nodes = (uint32_t)out.size();
  if (build_ms) *build_ms = ms;
  return IZPI_OK;
}

int izpi_gpu_postprocess(izpi_ctx* ctx, double* canvas_dev, uint32_t width, uint32_t height, const uint32_t* filters,
                         const double* params, uint32_t num_filters) {
  if (!ctx) return IZPI_ERR_INVALID;
  if (!canvas_dev || num_filters > IZPI_MAX_FILTERS || (num_filters && (!filters || !params))) {
    ctx->err = "postprocess: bad arguments";
    return IZPI_ERR_INVALID;
  }
  PostFilters pf;
  memset(&pf, 0, sizeof pf);
  pf.n = num_filters;
  for (uint32_t i = 0; i < num_filters; i++) {
    if (filters[i] != IZPI_FILTER_GAMMA && filters[i] != IZPI_FILTER_CLAMP) {
      ctx->err = "postprocess: unknown filter (colour grading needs a .cube LUT reader, not on this path)";
      return IZPI_ERR_UNSUPPORTED;
    }
    pf.kind[i] = filters[i];
    pf.param[i] = params[i];
  }
  const uint64_t np = (uint64_t)width * height;
  if (np == 0 || num_filters == 0) return IZPI_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_postprocess, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, ctx->stream, canvas_dev, np, pf);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return IZPI_OK;
}

int izpi_gpu_unpack_tiles(izpi_ctx* ctx, const izpi_render_req* req, const double* packed_dev, double* canvas_dev) {
  if (!ctx || !req || !packed_dev || !canvas_dev || !req->num_tiles) return IZPI_ERR_INVALID;
  HIP_TRY(hipSetDevice(ctx->device));
  uint32_t tw, th;
  if (!validate_tiles(req, req->tiles, req->num_tiles, &tw, &th)) { ctx->err = "bad tiles"; return IZPI_ERR_INVALID; }
  int rc = grow(ctx, (void**)&ctx->d_tiles, &ctx->tiles_cap, 4 * (size_t)req->num_tiles * sizeof(uint32_t));
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(ctx->d_tiles, req->tiles, 4 * (size_t)req->num_tiles * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
  const uint32_t np = req->num_tiles * tw * th;
  hipLaunchKernelGGL(k_unpack, dim3((np + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_tiles, np, tw, th, req->width,
                     req->height, packed_dev, canvas_dev);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return IZPI_OK;
}

int izpi_gpu_trace(izpi_ctx* ctx, const double* rays, uint32_t n, izpi_hit* out) {
  if (!ctx || !rays || !out) return IZPI_ERR_INVALID;
  if (!ctx->have_scene) { ctx->err = "no scene"; return IZPI_ERR_NO_SCENE; }
  if (n == 0) return IZPI_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  DevBufs tmp;  // freed on every return
  double* dr; izpi_hit* dh; RayOD* rr; uint32_t* kk; double2* tm; double2* hh;
  HIP_TRY(tmp.alloc(&dr, (size_t)n * 8));
  HIP_TRY(tmp.alloc(&dh, n));
  HIP_TRY(tmp.alloc(&rr, n));
  HIP_TRY(tmp.alloc(&kk, n));
  HIP_TRY(tmp.alloc(&tm, n));
  HIP_TRY(tmp.alloc(&hh, 2 * (size_t)n));  // (t, prim) and (u, v) interleaved
  HIP_TRY(hipMemcpy(dr, rays, (size_t)n * 8 * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemsetAsync(ctx->d_misc, 0, 8 * MISC_STRIDE * sizeof(uint32_t), ctx->stream));
  HIP_TRY(hipMemsetAsync(ctx->d_counters, 0, CNT_N * sizeof(unsigned long long), ctx->stream));
  hipLaunchKernelGGL(k_trace_setup, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, dr, n, rr, kk, tm, misc(ctx, 3));
  WaveParams wp{};
  wp.in.ray = rr; wp.in.kind = kk; wp.in.tminmax = tm; wp.in.hit = hh; wp.in.huv = hh + 1; wp.in.hs = 2;
  wp.in_count = misc(ctx, 3); wp.trace_next = misc(ctx, 2); wp.slots = n; wp.read_kind = 1; wp.hit_uv = 1;
  Tracer tr;
  int rc = make_tracer(ctx, kDefaultTuning, true, &tr);
  if (rc) return rc;
  if ((rc = grow(ctx, (void**)&ctx->d_spill, &ctx->spill_cap, tr.spill_bytes))) return rc;
  launch_trace(ctx, ctx->sc, tr, wp, ctx->stream, ctx->d_spill);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_trace_records, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, ctx->sc, rr, hh, n, dh);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipMemcpy(out, dh, (size_t)n * sizeof(izpi_hit), hipMemcpyDeviceToHost));
  return IZPI_OK;
}

int izpi_gpu_ray_aabb4(izpi_ctx* ctx, const float* boxes, const float* rays, uint32_t n, uint8_t* masks) {
  if (!ctx || !boxes || !rays || !masks) return IZPI_ERR_INVALID;
  if (n == 0) return IZPI_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  DevBufs tmp;  // freed on every return
  float *db, *dr; uint8_t* dm;
  HIP_TRY(tmp.alloc(&db, (size_t)n * 24));
  HIP_TRY(tmp.alloc(&dr, (size_t)n * 7));
  HIP_TRY(tmp.alloc(&dm, n));
  HIP_TRY(hipMemcpy(db, boxes, (size_t)n * 24 * sizeof(float), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dr, rays, (size_t)n * 7 * sizeof(float), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_aabb4, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, db, dr, n, dm);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipMemcpy(masks, dm, n, hipMemcpyDeviceToHost));
  return IZPI_OK;
}

int izpi_gpu_gomath(izpi_ctx* ctx, int op, const double* x, const double* y, uint32_t n, double* out) {
  if (!ctx || !x || !out) return IZPI_ERR_INVALID;
  if (n == 0) return IZPI_OK;
  if (op == 37) {  // texture lookups: a scene, and texture numbers in range
    if (!ctx->have_scene) { ctx->err = "texture lookup before izpi_gpu_upload_scene"; return IZPI_ERR_NO_SCENE; }
    if (!y) { ctx->err = "texture lookup without texture numbers"; return IZPI_ERR_INVALID; }
    for (uint32_t i = 0; i < n; i++)
      if (!(y[i] >= 0 && y[i] < (double)ctx->num_textures)) { ctx->err = "texture number out of range"; return IZPI_ERR_INVALID; }
  }
  if (op == 14 && !y) { ctx->err = "path length without exit points"; return IZPI_ERR_INVALID; }
  const size_t nin = op == 14 ? 3 * (size_t)n : n;  // op 14 reads 3-vectors
  HIP_TRY(hipSetDevice(ctx->device));
  DevBufs tmp;  // freed on every return
  double *dx, *dy = nullptr, *dout;
  HIP_TRY(tmp.alloc(&dx, nin));
  HIP_TRY(tmp.alloc(&dout, n));
  HIP_TRY(hipMemcpy(dx, x, nin * sizeof(double), hipMemcpyHostToDevice));
  if (y) {
    HIP_TRY(tmp.alloc(&dy, nin));
    HIP_TRY(hipMemcpy(dy, y, nin * sizeof(double), hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(k_gomath, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, ctx->sc, op, dx, dy, n, dout);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipMemcpy(out, dout, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
  return IZPI_OK;
}

// ------------------------------------------------- multi-GPU, one process
int izpi_gpu_multi_open(const int* devices, uint32_t num_devices, izpi_multi** out) {
  if (!out) return IZPI_ERR_INVALID;
  *out = nullptr;
  if (!devices || num_devices == 0) return IZPI_ERR_INVALID;
  izpi_multi* m = new izpi_multi();
  for (uint32_t i = 0; i < num_devices; i++) {
    izpi_ctx* c = nullptr;
    const int rc = izpi_gpu_open(devices[i], &c);
    if (rc) {
      izpi_gpu_multi_close(m);
      return rc;
    }
    m->ctx.push_back(c);
  }
  // contexts on one device split its HBM when they size their workspaces
  for (izpi_ctx* c : m->ctx) {
    c->dev_share = 0;
    for (izpi_ctx* o : m->ctx) c->dev_share += o->device == c->device ? 1u : 0u;
  }
  // device 0 receives every share: let it read/write peers directly over xGMI
  for (uint32_t i = 1; i < num_devices; i++) {
    if (devices[i] == devices[0]) continue;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, devices[i], devices[0]) == hipSuccess && can) {
      (void)hipSetDevice(devices[i]);
      (void)hipDeviceEnablePeerAccess(devices[0], 0);  // "already enabled" is fine
      (void)hipGetLastError();
    }
  }
  *out = m;
  return IZPI_OK;
}

int izpi_gpu_multi_close(izpi_multi* m) {
  if (!m) return IZPI_OK;
  for (izpi_ctx* c : m->ctx) izpi_gpu_close(c);
  delete m;
  return IZPI_OK;
}

const char* izpi_gpu_multi_last_error(izpi_multi* m) { return m ? m->err.c_str() : "null context"; }

uint32_t izpi_gpu_multi_size(izpi_multi* m) { return m ? (uint32_t)m->ctx.size() : 0u; }

izpi_ctx* izpi_gpu_multi_context(izpi_multi* m, uint32_t i) { return (m && i < m->ctx.size()) ? m->ctx[i] : nullptr; }

int izpi_gpu_multi_upload_scene(izpi_multi* m, const izpi_scene_desc* scene) {
  if (!m) return IZPI_ERR_INVALID;
  for (size_t i = 0; i < m->ctx.size(); i++) {  // the scene is replicated per GPU
    const int rc = izpi_gpu_upload_scene(m->ctx[i], scene);
    if (rc) {
      m->err = "device " + std::to_string(i) + ": " + m->ctx[i]->err;
      return rc;
    }
  }
  return IZPI_OK;
}

int izpi_gpu_multi_render(izpi_multi* m, const izpi_render_req* req, double* out_host, izpi_render_stats* stats) {
  if (!m || m->ctx.empty()) return IZPI_ERR_INVALID;
  const uint32_t G = (uint32_t)m->ctx.size();
  izpi_ctx* root = m->ctx[0];
  Shares sh;
  int rc = make_shares(root, req, G, sh);
  if (rc) { m->err = root->err; return rc; }
  if (req->post != IZPI_POST_NONE && req->num_tiles != 0) {
    m->err = "post-processing needs a whole-frame request";
    return IZPI_ERR_INVALID;
  }
  const size_t canvas_bytes = (size_t)req->width * req->height * 4 * sizeof(double);
  if (hipSetDevice(root->device) != hipSuccess) { m->err = "hipSetDevice"; return IZPI_ERR_HIP; }
  if ((rc = grow(root, (void**)&root->d_gather, &root->gather_cap, (size_t)G * sh.block * sizeof(double))) ||
      (rc = grow(root, (void**)&root->d_out, &root->out_cap, canvas_bytes))) {
    m->err = root->err;
    return rc;
  }
  // the caller's canvas is the starting point (pixels of no tile keep their values)
  if (out_host) {
    if (hipMemcpy(root->d_out, out_host, canvas_bytes, hipMemcpyHostToDevice) != hipSuccess) { m->err = "hipMemcpy"; return IZPI_ERR_HIP; }
  } else if (hipMemset(root->d_out, 0, canvas_bytes) != hipSuccess) {
    m->err = "hipMemset";
    return IZPI_ERR_HIP;
  }
  // one host thread per device: render its share, then copy it into block i of the
  // root's gather buffer (peer copy over xGMI; a plain device copy for the root)
  std::vector<int> rcs(G, IZPI_OK);
  std::vector<std::thread> th;
  for (uint32_t i = 0; i < G; i++) {
    th.emplace_back([&, i]() {
      izpi_ctx* c = m->ctx[i];
      if (hipSetDevice(c->device) != hipSuccess) { rcs[i] = IZPI_ERR_HIP; c->err = "hipSetDevice"; return; }
      int r = render_share(c, req, sh, i);
      if (!r) {
        hipError_t e = hipMemcpyPeerAsync(root->d_gather + (size_t)i * sh.block, root->device, c->d_share, c->device,
                                          sh.block * sizeof(double), c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) { c->err = std::string("gather copy: ") + hipGetErrorString(e); r = IZPI_ERR_HIP; }
      }
      rcs[i] = r;
    });
  }
  for (std::thread& t : th) t.join();
  for (uint32_t i = 0; i < G; i++) {
    if (stats) stats[i] = m->ctx[i]->last;
    if (rcs[i]) {
      m->err = "device " + std::to_string(i) + ": " + m->ctx[i]->err;
      return rcs[i];
    }
  }
  if (hipSetDevice(root->device) != hipSuccess) { m->err = "hipSetDevice"; return IZPI_ERR_HIP; }
  if ((rc = assemble(root, req, sh, root->d_out))) { m->err = root->err; return rc; }
  if (out_host && hipMemcpy(out_host, root->d_out, canvas_bytes, hipMemcpyDeviceToHost) != hipSuccess) {
    m->err = "hipMemcpy";
    return IZPI_ERR_HIP;
  }
  return IZPI_OK;
}

// ------------------------------------------ multi-GPU, one process per GPU
int izpi_gpu_comm_id(uint8_t* id) {
  if (!id) return IZPI_ERR_INVALID;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return IZPI_ERR_HIP;
  memcpy(id, u.internal, IZPI_COMM_ID_BYTES);
  return IZPI_OK;
}

int izpi_gpu_comm_init(izpi_ctx* ctx, uint32_t nranks, uint32_t rank, const uint8_t* id) {
  if (!ctx) return IZPI_ERR_INVALID;
  if (!id || nranks == 0 || rank >= nranks) { ctx->err = "comm_init: bad arguments"; return IZPI_ERR_INVALID; }
  HIP_TRY(hipSetDevice(ctx->device));
  if (ctx->comm) { (void)ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
  // the status word of izpi_gpu_render_rank's agreement steps, allocated here so that a
  // render never fails to reach them for want of it
  if (!ctx->d_status) HIP_TRY(hipMalloc((void**)&ctx->d_status, 2 * sizeof(int32_t)));
  ncclUniqueId u;
  memcpy(u.internal, id, IZPI_COMM_ID_BYTES);
  const ncclResult_t r = ncclCommInitRank(&ctx->comm, (int)nranks, u, (int)rank);
  if (r != ncclSuccess) {
    ctx->comm = nullptr;
    ctx->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    return IZPI_ERR_HIP;
  }
  ctx->comm_rank = rank;
  ctx->comm_size = nranks;
  return IZPI_OK;
}

}  // extern "C"

namespace {
// Agreement step of a multi-rank render: every rank contributes (status << 16 | rank) and
// all receive the maximum, i.e. the worst status and the highest rank that had it
// (ncclAllReduce(max), rccl.h). Returns non-zero only if the collective itself failed.
// Device-side stall of the fault-injection hook (izpi_gpu_debug_fault 3): one thread spins
// until the host sets *release (a coherent pinned word), as a stream stuck in a collective
// on a dead peer does; bounded (about 7 s of clock) so that the grid always drains.
__global__ void k_stall(const volatile uint32_t* release) {
  const uint64_t t0 = __builtin_readcyclecounter();
  while (__atomic_load_n(release, __ATOMIC_RELAXED) == 0u && __builtin_readcyclecounter() - t0 < (1ull << 34))
    __builtin_amdgcn_s_sleep(100);
}

// Wait for this context's stream (a collective step) as a rank that may outlive its peers:
// poll the stream and the communicator's asynchronous error; an RCCL error, a HIP error of
// this rank's stream or a wait past the deadline aborts the communicator and returns
// IZPI_ERR_PEER (render/remote.go:40-55 logs a failed remote tile and carries on; here the
// call returns instead of hanging). After a local HIP error this rank cannot join the
// remaining collectives, and peers blocked in them would never return: aborting the
// communicator ends their waits too (they see the async error), and the communicator is
// gone on this rank (izpi_gpu_comm_init makes a new one).
int wait_peers(izpi_ctx* ctx, uint32_t timeout_ms, const char* step) {
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t naps = 0;
  for (;;) {
    hipError_t q = hipStreamQuery(ctx->stream);
    if (ctx->fault_inject == 4 && q != hipErrorNotReady) q = hipErrorLaunchFailure;  // test hook: a failed stream
    if (q == hipSuccess) return IZPI_OK;
    ncclResult_t ae = ncclSuccess;
    const ncclResult_t qr = q == hipErrorNotReady ? ncclCommGetAsyncError(ctx->comm, &ae) : ncclSuccess;
    const bool failed = qr != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (q != hipErrorNotReady || failed || (timeout_ms && ms > timeout_ms)) {
      ctx->err = std::string(step) +
                 (q != hipErrorNotReady ? ": this rank's stream failed: " + std::string(hipGetErrorString(q))
                  : failed ? ": RCCL reported " + std::string(ncclGetErrorString(qr != ncclSuccess ? qr : ae))
                           : ": no answer from the other ranks within " + std::to_string(timeout_ms) + " ms") +
                 "; communicator aborted";
      // test hook: let the stall drain first (ncclCommAbort waits for the operations it
      // aborts, which sit behind it on the stream)
      if (ctx->stall_word) { *ctx->stall_word = 1u; ctx->stall_word = nullptr; }
      (void)ncclCommAbort(ctx->comm);
      ctx->comm = nullptr;
      (void)hipStreamSynchronize(ctx->stream);
      return IZPI_ERR_PEER;
    }
    // sub-millisecond polls at first (a collective normally completes in microseconds),
    // then 1 ms naps for a gather that waits on the slowest rank's render
    std::this_thread::sleep_for(std::chrono::microseconds(naps++ < 200 ? 20 : 1000));
  }
}

// Agree on the worst status over all ranks. The collective is issued whatever failed
// locally before it (a failed staging copy only makes this rank's word stale), so that no
// rank is left waiting in it; a local HIP error is reported after the collective.
int agree_status(izpi_ctx* ctx, int local, uint32_t timeout_ms, int* worst_status, uint32_t* worst_rank) {
  const int32_t word = (int32_t)((uint32_t)std::min(local, 0x7FFF) << 16 | (ctx->comm_rank & 0xFFFFu));
  int32_t* h = (int32_t*)ctx->h_count + 8 * MISC_STRIDE;  // pinned scratch
  h[0] = word;
  h[1] = word;  // this rank's own word, should the collective's copy-back fail
  const hipError_t e1 = hipMemcpyAsync(ctx->d_status, h, sizeof(word), hipMemcpyHostToDevice, ctx->stream);
  const ncclResult_t r = ncclAllReduce(ctx->d_status, ctx->d_status + 1, 1, ncclInt32, ncclMax, ctx->comm, ctx->stream);
  if (r != ncclSuccess) {
    ctx->err = std::string("ncclAllReduce: ") + ncclGetErrorString(r) + "; communicator aborted";
    (void)ncclCommAbort(ctx->comm);
    ctx->comm = nullptr;
    return IZPI_ERR_PEER;
  }
  const hipError_t e2 = hipMemcpyAsync(h + 1, ctx->d_status + 1, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream);
  const int rc = wait_peers(ctx, timeout_ms, "status agreement");
  if (rc) return rc;
  if (e1 != hipSuccess || e2 != hipSuccess) {
    ctx->err = std::string("status agreement: ") + hipGetErrorString(e1 != hipSuccess ? e1 : e2);
    return IZPI_ERR_HIP;
  }
  const int32_t out = h[1];
  *worst_status = (int)((uint32_t)out >> 16);
  *worst_rank = (uint32_t)out & 0xFFFFu;
  return IZPI_OK;
}

// A rank whose own step succeeded returns IZPI_ERR_PEER when another rank's failed.
int peer_failure(izpi_ctx* ctx, int worst, uint32_t worst_rank, const char* when) {
  ctx->err = "rank " + std::to_string(worst_rank) + " failed " + when + " (status " + std::to_string(worst) + ")";
  return IZPI_ERR_PEER;
}
}  // namespace

extern "C" {

// Every rank runs the same sequence of collectives whatever fails locally, so no rank is
// left waiting in one (render/remote.go:40-55 logs a failed remote tile; here every rank
// learns the worst status):
//   1. local checks and buffers (share block; gather buffer on rank 0), then agree: if any
//      rank failed, all return before rendering;
//   2. render the share (a failed share posts a zeroed block), ncclGather to rank 0, agree
//      again: if any rank failed, all return it and rank 0 does not assemble;
//   3. rank 0 assembles and post-processes (a failure there is rank 0's alone).
int izpi_gpu_render_rank(izpi_ctx* ctx, const izpi_render_req* req, double* out_dev, izpi_render_stats* stats) {
  if (!ctx) return IZPI_ERR_INVALID;
  // without a communicator no collective can run: every rank in this state returns here
  if (!ctx->comm || !ctx->d_status) { ctx->err = "render_rank before izpi_gpu_comm_init"; return IZPI_ERR_INVALID; }
  memset(&ctx->last, 0, sizeof(ctx->last));
  ctx->prog_done.store(0, std::memory_order_relaxed);  // (no stale count while the ranks agree)
  ctx->prog_total.store(0, std::memory_order_relaxed);
  if (stats) *stats = ctx->last;
  const uint32_t timeout_ms = tuning_of(req).peer_timeout_ms;
  // ---- 1 (local failures, HIP ones included, are recorded and agreed on, not returned early)
  Shares sh;
  int prc = IZPI_OK;
  const hipError_t de = hipSetDevice(ctx->device);
  if (de != hipSuccess) { ctx->err = std::string("hipSetDevice: ") + hipGetErrorString(de); prc = IZPI_ERR_HIP; }
  else if (ctx->comm_rank == 0 && !out_dev) { ctx->err = "rank 0 needs an output canvas"; prc = IZPI_ERR_INVALID; }
  else if (req && req->post != IZPI_POST_NONE && req->num_tiles != 0) { ctx->err = "post-processing needs a whole-frame request"; prc = IZPI_ERR_INVALID; }
  if (!prc) prc = make_shares(ctx, req, ctx->comm_size, sh);
  if (!prc) prc = grow(ctx, (void**)&ctx->d_share, &ctx->share_cap, sh.block * sizeof(double));
  if (!prc && ctx->comm_rank == 0) prc = grow(ctx, (void**)&ctx->d_gather, &ctx->gather_cap, (size_t)ctx->comm_size * sh.block * sizeof(double));
  if (prc == IZPI_OK && ctx->fault_inject == 1) { ctx->err = "injected fault before rendering"; prc = IZPI_ERR_DEVICE; }
  const std::string local_err = ctx->err;
  int worst = 0;
  uint32_t wr = 0;
  int rc = agree_status(ctx, prc, timeout_ms, &worst, &wr);
  if (rc) return rc;
  if (prc) { ctx->err = local_err; return prc; }
  if (worst) return peer_failure(ctx, worst, wr, "before rendering");
  // ---- 2 (a failed share posts a zeroed block: the gather runs on every rank)
  int rrc = render_share(ctx, req, sh, ctx->comm_rank);
  if (stats) *stats = ctx->last;
  if (rrc) (void)hipMemsetAsync(ctx->d_share, 0, sh.block * sizeof(double), ctx->stream);
  if (ctx->fault_inject == 3) {  // test hook: this rank's stream stalls as on a dead peer
    // the release word is fine-grained (coherent) host memory: the spinning kernel sees
    // the host's store while it runs
    if (!ctx->stall_host && hipHostMalloc((void**)&ctx->stall_host, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
      ctx->stall_host = nullptr;
    if (ctx->stall_host) {
      ctx->stall_word = ctx->stall_host;
      *ctx->stall_word = 0u;
      hipLaunchKernelGGL(k_stall, dim3(1), dim3(1), 0, ctx->stream, (const volatile uint32_t*)ctx->stall_word);
    }
  }
  // ncclGather (rccl.h:745): block r of the root's buffer = rank r's packed share
  const ncclResult_t r = ncclGather(ctx->d_share, ctx->comm_rank == 0 ? ctx->d_gather : nullptr, sh.block, ncclFloat64, 0,
                                    ctx->comm, ctx->stream);
  if (r != ncclSuccess) {  // the peers may already wait in the gather: abort rather than leave them there
    ctx->err = std::string("ncclGather: ") + ncclGetErrorString(r) + "; communicator aborted";
    if (ctx->stall_word) { *ctx->stall_word = 1u; ctx->stall_word = nullptr; }
    (void)ncclCommAbort(ctx->comm);
    ctx->comm = nullptr;
    (void)hipStreamSynchronize(ctx->stream);
    return IZPI_ERR_PEER;
  }
  if ((rc = wait_peers(ctx, timeout_ms, "share gather"))) return rc;
  const std::string share_err = ctx->err;
  if ((rc = agree_status(ctx, rrc, timeout_ms, &worst, &wr))) return rc;
  if (rrc) { ctx->err = share_err; return rrc; }
  if (worst) return peer_failure(ctx, worst, wr, "while rendering its share");
  // ---- 3
  if (ctx->comm_rank == 0 && (rc = assemble(ctx, req, sh, out_dev))) return rc;
  return IZPI_OK;
}

uint64_t izpi_host_share_block(uint32_t num_tiles, uint32_t tile_w, uint32_t tile_h, uint32_t num_shares) {
  return num_shares ? share_block(num_tiles, tile_w, tile_h, num_shares) : 0;
}

int izpi_host_assemble_shares(uint32_t width, uint32_t height, const uint32_t* tiles, uint32_t num_tiles,
                              uint32_t num_shares, const double* gathered, double* canvas) {
  if (!tiles || !gathered || !canvas || num_tiles == 0 || num_shares == 0 || width == 0 || height == 0) return IZPI_ERR_INVALID;
  izpi_render_req req{};
  req.width = width; req.height = height;
  uint32_t tw = 0, th = 0;
  if (!validate_tiles(&req, tiles, num_tiles, &tw, &th)) return IZPI_ERR_INVALID;
  const size_t block = share_block(num_tiles, tw, th, num_shares);
  std::vector<uint32_t> mine(4 * (size_t)num_tiles);
  for (uint32_t r = 0; r < num_shares; r++) {
    const uint32_t nt = izpi_host_share_tiles(tiles, num_tiles, r, num_shares, mine.data());
    const double* packed = gathered + (size_t)r * block;
    for (uint32_t p = 0; p < nt * tw * th; p++) {
      uint32_t x, row;
      if (packed_target(mine.data(), p, tw, th, height, &x, &row))
        memcpy(canvas + ((size_t)row * width + x) * 4, packed + (size_t)p * 4, 4 * sizeof(double));
    }
  }
  return IZPI_OK;
}

int izpi_gpu_progress(izpi_ctx* ctx, uint64_t* samples_done, uint64_t* samples_total) {
  if (!ctx || !samples_done || !samples_total) return IZPI_ERR_INVALID;
  // total first: a render starting between the two loads shows 0 of its own total at worst
  *samples_total = ctx->prog_total.load(std::memory_order_relaxed);
  *samples_done = std::min(ctx->prog_done.load(std::memory_order_relaxed), *samples_total);
  return IZPI_OK;
}

int izpi_gpu_multi_progress(izpi_multi* m, uint64_t* samples_done, uint64_t* samples_total) {
  if (!m || !samples_done || !samples_total) return IZPI_ERR_INVALID;
  *samples_done = 0; *samples_total = 0;
  for (izpi_ctx* c : m->ctx) {
    uint64_t d = 0, t = 0;
    izpi_gpu_progress(c, &d, &t);
    *samples_done += d; *samples_total += t;
  }
  return IZPI_OK;
}

int izpi_gpu_debug_realloc(izpi_ctx* ctx, uint32_t mask) {
  if (!ctx) return IZPI_ERR_INVALID;
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  struct { void** p; size_t cap; } bufs[] = {{(void**)&ctx->d_samples, ctx->samples_cap}, {(void**)&ctx->d_recs, ctx->recs_cap},
                                             {(void**)&ctx->d_pool, ctx->pool_cap}, {(void**)&ctx->d_ring, ctx->ring_cap},
                                             {(void**)&ctx->d_running, ctx->running_cap}, {(void**)&ctx->d_state, ctx->state_cap},
                                             {(void**)&ctx->d_spill, ctx->spill_cap}};
  for (uint32_t k = 0; k < sizeof(bufs) / sizeof(bufs[0]); k++) {
    if (!(mask >> k & 1u) || !*bufs[k].p || !bufs[k].cap) continue;
    void* fresh = nullptr;  // allocated while the old buffer is still held: other pages
    HIP_TRY(hipMalloc(&fresh, bufs[k].cap));
    HIP_TRY(hipFree(*bufs[k].p));
    *bufs[k].p = fresh;
  }
  return IZPI_OK;
}

int izpi_gpu_debug_fault(izpi_ctx* ctx, int where) {
  if (!ctx || where < 0 || where > 4) return IZPI_ERR_INVALID;
  ctx->fault_inject = where;
  return IZPI_OK;
}

}  // extern "C"
