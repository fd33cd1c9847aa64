// izpi_kern.h — internal header of libizpi_gpu.so, shared by its three HIP translation units:
//   trace.hip     k_trace2 (BVH4.Hit) and its instance selection;
//   shade.hip     k_start / k_shade / k_tail / k_accumulate and the wavefront pass loop;
//   izpi_gpu.hip  the C ABI, the context, scene upload, workspace sizing, multi-GPU.
// Device helpers (textures, spectra, the wavefront state, hit records, lights, materials,
// the shading records) and the host context live here. Not part of the ABI.
#pragma once
//
// Hot path restated as device code (reference files under /root/reference/internal):
//   render/rgb.go:27-41, render/spectral.go:71-106   per-sample loop   -> k_start / k_shade + k_accumulate
//   camera/camera.go:61-89                           GetRay            -> start_path()
//   sampler/colour.go:33-65, sampler/spectral.go:47-80  recursive sampler -> one bounce per k_shade pass,
//                                                    unwound from records or carried forward (IZPI_ACC_*)
//   hitable/bvh4.go:49-164                           BVH4.Hit          -> k_trace2 / trace_one()
//   hitable/bvh4_simd_generic.go:10-52               RayAABB4          -> izd::slab()
//   hitable/triangle.go:193-280,317-326, sphere.go:63-145  prims, PDFValue, Random
//   material/*.go, pdf/*.go, texture/*.go, spectral/spectral.go:151-253
//
// Execution scheme: a wavefront of paths in flight in queue order;
// k_trace2 and k_shade alternate over it until no entry holds a ray, k_tail runs the last
// paths to their ends, k_accumulate sums each pixel's samples in sample order.
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

static __constant__ double c_cie_wl[IZPI_CIE_N] = IZPI_CIE_WAVELENGTHS_INIT;
static __constant__ double c_cie_x[IZPI_CIE_N] = IZPI_CIE_X_INIT;
static __constant__ double c_cie_y[IZPI_CIE_N] = IZPI_CIE_Y_INIT;
static __constant__ double c_cie_z[IZPI_CIE_N] = IZPI_CIE_Z_INIT;
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
static __constant__ CieCum c_cie_ycum = cie_y_running_sums();

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
  // IZPI_ACC_FORWARD: `in`'s camera entries, [cam[0], cam[0] + cam[2]) holding units
  // cam[1] + (i - cam[0]) (k_refill_plan's plan); their path state is not stored
  // (camera_path), or null
  const uint32_t* cam;
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
// render/spectral.go:92-96), with no records to read. Spectral: the sample is stored raw,
// (radiance, lambda, pdf), and k_accumulate applies the XYZ weights (raw_spectral): the CIE
// lookup inlined at the item's two exits cost the Spectral forward instances 26 spilled VGPRs.
template <int SAMPLER>
IZPI_DEV void finish_fwd(const ShadeParams& sp, const PathSt& P, V3 L) {
  double* out = sample_out(sp, P.unit);
  if (SAMPLER == IZPI_SAMPLER_COLOUR) {
    const V3 c = denan(mk(P.thr[0] * L.x, P.thr[1] * L.y, P.thr[2] * L.z));
    sst(out, c.x); sst(out + 1, c.y); sst(out + 2, c.z);
  } else {
    sst(out, P.thr[0] * L.x); sst(out + 1, P.lambda); sst(out + 2, P.lpdf);
  }
}
// A raw Spectral sample (radiance r, lambda, pdf) as render/spectral.go:92-96 weighs it:
// (r * x(lambda)) / pdf, ... (finish's own order: sdiv is bit for bit a division).
IZPI_DEV void spectral_weigh(double r, double lambda, double pdf, double& x, double& y, double& z) {
  double cx, cy, cz;
  cie_values<false>(lambda, cx, cy, cz);
  x = (r * cx) / pdf; y = (r * cy) / pdf; z = (r * cz) / pdf;
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
template <int SAMPLER, bool FWD>
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
      // (a raw forward sample (0, 380, 1) weighs to +0: 0 * x / 1)
      sst(out, 0.0); sst(out + 1, FWD ? 380.0 : 0.0); sst(out + 2, FWD ? 1.0 : 0.0);
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
    if constexpr (FWD) finish_fwd<SAMPLER>(sp, P, terminal_max_depth(sp, P, SAMPLER == IZPI_SAMPLER_COLOUR));  // (T = 1)
    else finish<SAMPLER, MATSET_FULL>(sp, P, terminal_max_depth(sp, P, SAMPLER == IZPI_SAMPLER_COLOUR));  // depth 0: reads no record
    return false;
  }
  R.o[0] = ro.x; R.o[1] = ro.y; R.o[2] = ro.z;
  R.d[0] = rd.x; R.d[1] = rd.y; R.d[2] = rd.z;
  R.time = time;
  R.kind = RAY_MAIN;
  return true;
}

// IZPI_ACC_FORWARD's camera entries: k_refill stores only the camera ray of a new path
// (ray, kind word, ray time), 40 B less per entry than store_entry (path state and
// throughput; 56 B for the Spectral sampler's wavelength); its path state is exactly what
// start_path set, so camera_path computes it again from the unit where the entry is
// shaded: the sample's stream after its wavelength and jitter draws (render/spectral.go:
// 74-84, rgb.go:21-31, camera.go:61-89 draws from its own stream), depth 0, T = 1.
template <int SAMPLER>
IZPI_DEV void camera_path(const ShadeParams& sp, uint32_t unit, PathSt& P) {
  const uint32_t pix_local = unit / sp.chunk_spp;
  const uint32_t s = sp.s0 + unit % sp.chunk_spp;
  const uint32_t tile_px = sp.tile_w * sp.tile_h;
  const uint32_t tile = pix_local / tile_px, in_tile = pix_local % tile_px;
  const uint32_t x = sp.tiles[4 * tile] + in_tile % sp.tile_w;
  const uint32_t y = sp.tiles[4 * tile + 1] + in_tile / sp.tile_w;
  const uint64_t key = ((uint64_t)s << 32) | (uint64_t)(y * sp.width + x);
  Lcg rng;
  rng.s = (uint32_t)splitmix64(sp.seed ^ key);
  P.unit = unit; P.depth = 0; P.zf = 0; P.blk = 0; P.rslot = 0;
  P.lambda = 0; P.lpdf = 1;
  P.thr[0] = 1.0; P.thr[1] = 1.0; P.thr[2] = 1.0;
  if (SAMPLER == IZPI_SAMPLER_SPECTRAL) {
    const double r = rng.next();
    if (sp.staged) sample_wavelength<true>(r, P.lambda, P.lpdf);
    else sample_wavelength<false>(r, P.lambda, P.lpdf);
  }
  (void)rng.next();  // the jitter of u
  (void)rng.next();  // and of v
  P.rng = rng.s;
}
IZPI_DEV void store_camera_entry(const WaveBuf& b, uint32_t pos, const RayRec& R) {
  double2* r = reinterpret_cast<double2*>(b.ray + pos);
  sst(r, make_double2(R.o[0], R.o[1]));
  sst(r + 1, make_double2(R.o[2], R.d[0]));
  sst(r + 2, make_double2(R.d[1], R.d[2]));
  sst(b.kind + pos, R.kind);
  if (b.time) sst(b.time + pos, R.time);
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


// calculatePathLength's length of a found exit point (dielectric.go:141-150): |exit - p|
// clamped to [0.1, 100]
IZPI_DEV double path_length(V3 hp, V3 exit_p) {
  double len = length(sub(exit_p, hp));
  if (len < 0.1) len = 0.1;
  if (len > 100.0) len = 100.0;
  return len;
}

// ================================================================ host side (shared)
constexpr uint32_t CPART_BLOCKS_PER_CU = 16;  // counter rows per CU / 4: above any resident 256-thread grid
// Per-pixel sequential sum of the chunk's samples (render/rgb.go:36 col += ...,
// render/spectral.go:164-166 sum += ...), in sample order; finalize on the last chunk.
struct AccumParams {
  uint32_t num_pixels, chunk_spp, spp, width, height, tile_w, tile_h, sampler, last, out_layout;
  uint32_t raw_spectral;  // the samples are (radiance, lambda, pdf): weigh each (spectral_weigh) before summing
  const uint32_t* tiles;
  const double* samples;  // [num_pixels][chunk_spp][3]
  double* running;        // [num_pixels][3]
  double* out;
};
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
  bool prepare_only = false;     // izpi_gpu_prepare: render_body sizes and allocates, then returns
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

// The words of d_misc lie MISC_STRIDE words (256 B) apart: the unit head and the queue
// counts take one returning atomic each per shading block-iteration (~11M per C3 frame),
// and atomics on one line are served one at a time (a single word saturates near 88 per
// microsecond, MI355X_MICROARCH.md "dequeue").
inline uint32_t* misc(izpi_ctx* ctx, int k) { return ctx->d_misc + (size_t)k * MISC_STRIDE; }

template <typename K>
inline int resident_blocks(izpi_ctx* ctx, K kernel, int* blocks, int threads = 256, size_t dyn_lds = 0) {
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
  bool qnodes = false;   // Q
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

// trace.hip: pick the k_trace2 instance and its grid (no allocation: the caller grows d_spill
// to t->spill_bytes; need_uv: the caller reads the hits' (u, v), WaveParams::hit_uv), and
// launch it for one pass.
int make_tracer(izpi_ctx* ctx, const izpi_render_tuning& tu, bool need_uv, Tracer* t);
void launch_trace(izpi_ctx* ctx, const DevScene& sc, const Tracer& t, const WaveParams& wp, hipStream_t st, int32_t* spill);
// shade_*.hip (shade.h): every chunk of the request through the wavefront passes with the
// shading instance of (SAMPLER, FWD) and the scene's material set; one explicit instance per
// translation unit. Device times of the passes are added to *trace_ms / *shade_ms / *tail_ms.
template <int SAMPLER, bool FWD>
int run_sampler(izpi_ctx* ctx, const izpi_render_req* req, const DevScene& sc, const Tracer& tr, ShadeParams& sp,
                WaveParams& wp, AccumParams& ap, uint32_t num_pixels, uint32_t chunk, uint32_t pool_blocks, bool compact,
                float* trace_ms, float* shade_ms, float* tail_ms, uint32_t* launches);
// shade_*.hip: load the code of the shading kernels run_sampler<SAMPLER, FWD> would launch
// for the uploaded scene (izpi_gpu_upload_scene, ahead of the first frame).
template <int SAMPLER, bool FWD>
int prepare_sampler(izpi_ctx* ctx, bool compact);
// Diagnostics (IZPI_TUNE_PASS_LOG): host milliseconds on a process-wide steady clock.
inline double diag_clock_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
