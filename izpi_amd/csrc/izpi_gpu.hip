// izpi_gpu.hip — the C ABI of the MI355X path-tracing inner loop for izpi (include/izpi_gpu.h):
// contexts, scene upload, workspace sizing, the render call, multi-GPU (threads and RCCL ranks),
// post-processing and the component entries. The kernels of the hot path are in trace.hip and
// shade.hip (izpi_kern.h).
#include "izpi_kern.h"

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

namespace {


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

// Quantise inner node g's child boxes (IZPI_SCENE_QUANTIZED_BVH) into q and replace g's
// valid slot boxes by the decoded ones. Per axis: the origin is the minimum over the valid
// children's mins, the scale 2^e the smallest for which every child's bounds, rounded
// outwards to the grid, fit a byte; each rounded bound is then checked in the kernels' own
// f32 decode (qdecode) and moved one step outwards while it would not contain the exact
// bound. False when a valid bound is not finite or no exponent fits (the scene then keeps
// its exact boxes).
bool quantize_node(GInner& g, GInnerQ& q) {
  memset(&q, 0, sizeof(q));
  float* mn[3] = {g.mnx, g.mny, g.mnz};
  float* mx[3] = {g.mxx, g.mxy, g.mxz};
  for (int i = 0; i < 4; i++) q.child[i] = g.child[i];
  for (int a = 0; a < 3; a++) {
    float lo = 0.0f, hi = 0.0f;
    bool any = false;
    for (int i = 0; i < 4; i++) {
      if (g.child[i] == -1) continue;
      if (!std::isfinite(mn[a][i]) || !std::isfinite(mx[a][i])) return false;
      lo = any ? std::min(lo, mn[a][i]) : mn[a][i];
      hi = any ? std::max(hi, mx[a][i]) : mx[a][i];
      any = true;
    }
    const double ext = (double)hi - (double)lo;
    int e = -126;
    if (ext > 0) e = std::max(-126, (int)std::ceil(std::log2(ext / 255.0)));
    uint32_t qlo[4] = {0, 0, 0, 0}, qhi[4] = {0, 0, 0, 0};
    for (;; e++) {
      if (e > 127) return false;
      const float sc = std::ldexp(1.0f, e);
      bool ok = true;
      for (int i = 0; i < 4 && ok; i++) {
        if (g.child[i] == -1) continue;
        double fl = std::floor(((double)mn[a][i] - (double)lo) / (double)sc);
        int ql = (int)std::min(255.0, std::max(0.0, fl));
        while (ql > 0 && qdecode(lo, (uint32_t)ql, sc) > mn[a][i]) ql--;  // qdecode(lo, 0) == lo <= every min
        double fh = std::ceil(((double)mx[a][i] - (double)lo) / (double)sc);
        int qh = (int)std::max((double)ql, std::min(256.0, fh));
        while (qh <= 255 && qdecode(lo, (uint32_t)qh, sc) < mx[a][i]) qh++;
        if (qh > 255) ok = false;
        qlo[i] = (uint32_t)ql; qhi[i] = (uint32_t)qh;
      }
      if (ok) break;
    }
    const float sc = std::ldexp(1.0f, e);
    q.org[a] = lo;
    q.ex |= (uint32_t)(e + 127) << (8 * a);
    for (int i = 0; i < 4; i++) {
      q.q[a] |= qlo[i] << (8 * i);
      q.q[3 + a] |= qhi[i] << (8 * i);
      if (g.child[i] == -1) continue;
      mn[a][i] = qdecode(lo, qlo[i], sc);
      mx[a][i] = qdecode(lo, qhi[i], sc);
    }
  }
  return true;
}

void free_scene(izpi_ctx* ctx) {
  for (void* p : ctx->scene_allocs) (void)hipFree(p);
  ctx->scene_allocs.clear();
  ctx->scene_bytes = 0;
  ctx->have_scene = false;
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
  const auto t_body0 = std::chrono::steady_clock::now();
  auto host_ms = [&t_body0]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_body0).count(); };
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
  const double t_tiles = host_ms();
  int trc = make_tracer(ctx, tu, !ctx->sc.tri_only || ctx->any_uv, &tr);
  if (trc) return trc;
  const double t_tracer = host_ms();
  // Sizing against the HBM this context may use: what is free plus the render buffers it
  // holds and would release (a later frame reuses them, so every frame of a renderer sizes
  // alike), shared evenly by the contexts of one process on this device.
  const uint64_t size_key[8] = {num_pixels, req->spp, req->sampler, req->max_depth, ctx->pool_grow,
                                ((uint64_t)tu.slots << 32) | tu.chunk_units, ((uint64_t)tu.rec_dense << 32) | tu.pool_div, acc};
  const bool reuse = ctx->sizing_valid && memcmp(size_key, ctx->sizing.key, sizeof(size_key)) == 0;
  size_t free_b = 0, total_b = 0;
  if (!reuse && hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
  const double t_meminfo = host_ms();
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
  const double t_sized = host_ms();
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
  if (ctx->prepare_only) {
    // izpi_gpu_prepare: the device's first work on the fresh workspace (its first submission
    // after a large allocation waited ~7 ms, and the kernels' first touch of its pages)
    // happens here, in the renderer's setup, not in its first frame
    hipStream_t ps = ctx->stream;
    HIP_TRY(hipMemsetAsync(ctx->d_state, 0, ctx->state_cap, ps));
    HIP_TRY(hipMemsetAsync(ctx->d_samples, 0, ctx->samples_cap, ps));
    if (ctx->d_recs) HIP_TRY(hipMemsetAsync(ctx->d_recs, 0, ctx->recs_cap, ps));
    HIP_TRY(hipStreamSynchronize(ps));
    ctx->last = izpi_render_stats{};
    ctx->last.workspace_bytes = workspace_bytes(ctx);
    ctx->last.slots = slots; ctx->last.chunk_spp = chunk; ctx->last.alloc_ms = alloc_ms;
    return IZPI_OK;
  }
  if (tu.flags & IZPI_TUNE_PASS_LOG) HIP_TRY(hipEventRecord(ctx->evb[0], ctx->stream));
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
  const double t_launch = host_ms();
  HIP_TRY(hipEventRecord(ctx->ev0, st));
  if (tu.flags & IZPI_TUNE_PASS_LOG) {  // diagnostics: the GPU time of the setup copies before ev0
    HIP_TRY(hipEventSynchronize(ctx->ev0));
    float prep = 0;
    HIP_TRY(hipEventElapsedTime(&prep, ctx->evb[0], ctx->ev0));
    fprintf(stderr, "IZPI_T ev0_synced %.3f prep_gpu_ms %.3f body_start %.3f\n", diag_clock_ms(), prep,
            diag_clock_ms() - host_ms());
  }
#define IZPI_RUN(S, F) run_sampler<S, F>(ctx, req, sc, tr, sp, wp, ap, num_pixels, chunk, pool_blocks, compact, &trace_ms, &shade_ms, \
                                        &tail_ms, &launches)
  if (req->sampler == IZPI_SAMPLER_COLOUR) rc = fwd ? IZPI_RUN(IZPI_SAMPLER_COLOUR, true) : IZPI_RUN(IZPI_SAMPLER_COLOUR, false);
  else rc = fwd ? IZPI_RUN(IZPI_SAMPLER_SPECTRAL, true) : IZPI_RUN(IZPI_SAMPLER_SPECTRAL, false);
#undef IZPI_RUN
  if (rc) return rc;
  hipLaunchKernelGGL(k_cpart_reduce, dim3(CNT_N), dim3(256), 0, st, ctx->d_cpart, cpart_rows, ctx->d_counters);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev1, st));
  if ((rc = apply_post(ctx, req, out_dev))) return rc;
  const double t_issued = host_ms();
  HIP_TRY(hipEventSynchronize(ctx->ev1));
  if (tu.flags & IZPI_TUNE_PASS_LOG)  // diagnostics: where the call's host time goes
    fprintf(stderr, "IZPI_HOST tiles %.3f tracer %.3f meminfo %.3f sized %.3f allocated %.3f launched %.3f issued %.3f done %.3f ms\n",
            t_tiles, t_tracer, t_meminfo, t_sized, t_sized + alloc_ms, t_launch, t_issued, host_ms());
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
// The frame is split into G shares: tile t (in common.Tiles' spiral order, each cut into
// quarters: make_shares) goes to share t % G, so the costly centre tiles spread over all
// devices. Share r is rendered packed
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
  // Several shares: deal quarter tiles (each even-sized tile of at least 16 x 16 pixels cut
  // 2 x 2, in the tile's order), twice as many units to average the tiles' costs over: C3's
  // eighth-shares' slowest against mean 1.016 / 1.021 over two runs against 1.035 / 1.017
  // dealing whole tiles (0.816 / 0.811 of linear against 0.801 / 0.813; `profiles/r6ag/`,
  // `r6ah/`). The image does not depend on the partition (per-sample streams).
  if (n > 1 && tw % 2 == 0 && th % 2 == 0 && tw >= 16 && th >= 16) {
    std::vector<uint32_t> sub;
    sub.reserve(sh.all.size() * 4);
    const uint32_t hw = tw / 2, hh = th / 2;
    for (size_t t = 0; t + 3 < sh.all.size(); t += 4)
      for (uint32_t j = 0; j < 2; j++)
        for (uint32_t i = 0; i < 2; i++) {
          const uint32_t x0 = sh.all[t] + i * hw, y0 = sh.all[t + 1] + j * hh;
          sub.insert(sub.end(), {x0, y0, x0 + hw - 1, y0 + hh - 1});
        }
    sh.all.swap(sub);
    tw = hw;
    th = hh;
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
  // ---- quantised child boxes (IZPI_SCENE_QUANTIZED_BVH, ABI 3): `inner` and the leaf
  // records take the decoded boxes, which every traversal instance then tests (the 64-B
  // nodes and the 128-B ones describe the same tree); a leaf's re-test box is its decoded
  // parent slot, so its shortcut holds
  std::vector<GInnerQ> innerq;
  bool quantized = false;
  if (d->abi_version >= 3 && (d->flags & IZPI_SCENE_QUANTIZED_BVH) && n_inner > 0) {
    std::vector<GInner> dec(inner);
    innerq.resize(n_inner);
    quantized = true;
    for (uint32_t k = 0; k < n_inner && quantized; k++) quantized = quantize_node(dec[k], innerq[k]);
    if (quantized) {
      inner.swap(dec);
      for (uint32_t k = 0; k < n_inner; k++) {
        const GInner& g = inner[k];
        for (int i = 0; i < 4; i++) {
          if (!ref_is_leaf(g.child[i])) continue;
          GLeaf& L = leaves[(size_t)leaf_start(g.child[i])];
          L.mn[0] = g.mnx[i]; L.mn[1] = g.mny[i]; L.mn[2] = g.mnz[i];
          L.mx[0] = g.mxx[i]; L.mx[1] = g.mxy[i]; L.mx[2] = g.mxz[i];
        }
      }
      leaf_shortcut = 1;
    } else {
      innerq.clear();
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
  GInnerQ* dq = nullptr;
  if (quantized) UP(innerq.data(), innerq.size(), &dq);
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
  sc.inner = di; sc.innerq = dq; sc.quantized = quantized ? 1u : 0u; sc.leaves = dl; sc.prims = dp; sc.shade = dsh; sc.tritex = dtt; sc.lights = dlt; sc.materials = dm;
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
  // Load the code of the kernels this scene's renders run now, as part of the scene setup
  // (izpi's Render timer starts after it, renderer.go:170): a first occupancy query loads a
  // kernel's code object, 14 ms of a fresh renderer's first frame otherwise.
  {
    Tracer tr;
    int rc = make_tracer(ctx, kDefaultTuning, !ctx->sc.tri_only || ctx->any_uv, &tr);
    const bool compact = ctx->basic_materials && ctx->const_albedo;
    if (!rc && ctx->mat_ok_rgb) rc = prepare_sampler<IZPI_SAMPLER_COLOUR, true>(ctx, compact);
    if (!rc && ctx->mat_ok_rgb) rc = prepare_sampler<IZPI_SAMPLER_COLOUR, false>(ctx, compact);
    if (!rc && ctx->mat_ok_spectral) rc = prepare_sampler<IZPI_SAMPLER_SPECTRAL, true>(ctx, false);
    if (!rc && ctx->mat_ok_spectral) rc = prepare_sampler<IZPI_SAMPLER_SPECTRAL, false>(ctx, false);
    if (rc) return rc;
  }
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

int izpi_gpu_prepare(izpi_ctx* ctx, const izpi_render_req* req) {
  if (!ctx) return IZPI_ERR_INVALID;
  HIP_TRY(hipSetDevice(ctx->device));
  izpi_render_req q = *req;
  std::vector<uint32_t> mine;
  if (ctx->comm && ctx->comm_size > 1) {  // izpi_gpu_render_rank's share of the frame on this rank
    Shares sh;
    int rc = make_shares(ctx, req, ctx->comm_size, sh);
    if (rc) return rc;
    if ((rc = grow(ctx, (void**)&ctx->d_share, &ctx->share_cap, sh.block * sizeof(double)))) return rc;
    if (ctx->comm_rank == 0 &&
        (rc = grow(ctx, (void**)&ctx->d_gather, &ctx->gather_cap, (size_t)ctx->comm_size * sh.block * sizeof(double))))
      return rc;
    mine = sh.mine(ctx->comm_rank);
    if (mine.empty()) return IZPI_OK;
    q.num_tiles = (uint32_t)(mine.size() / 4);
    q.tiles = mine.data();
    q.out_layout = IZPI_OUT_PACKED;
    q.post = IZPI_POST_NONE;
  }
  ctx->prepare_only = true;
  const int rc = render_impl(ctx, &q, nullptr);
  ctx->prepare_only = false;
  return rc;
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
int izpi_gpu_multi_prepare(izpi_multi* m, const izpi_render_req* req) {
  if (!m) return IZPI_ERR_INVALID;
  izpi_ctx* c0 = m->ctx[0];
  Shares sh;
  int rc = make_shares(c0, req, (uint32_t)m->ctx.size(), sh);
  if (rc) { m->err = c0->err; return rc; }
  const uint32_t G = (uint32_t)m->ctx.size();
  if (hipSetDevice(c0->device) != hipSuccess) { m->err = "hipSetDevice"; return IZPI_ERR_HIP; }
  if ((rc = grow(c0, (void**)&c0->d_gather, &c0->gather_cap, (size_t)G * sh.block * sizeof(double))) ||
      (rc = grow(c0, (void**)&c0->d_out, &c0->out_cap, (size_t)req->width * req->height * 4 * sizeof(double)))) {
    m->err = c0->err;
    return rc;
  }
  // the devices' workspaces, one host thread each (as izpi_gpu_multi_render renders them)
  std::vector<int> rcs(G, IZPI_OK);
  std::vector<std::thread> th;
  for (uint32_t i = 0; i < G; i++) {
    th.emplace_back([&, i]() {
      izpi_ctx* c = m->ctx[i];
      if (hipSetDevice(c->device) != hipSuccess) { c->err = "hipSetDevice"; rcs[i] = IZPI_ERR_HIP; return; }
      int r = grow(c, (void**)&c->d_share, &c->share_cap, sh.block * sizeof(double));
      const std::vector<uint32_t> mine = sh.mine(i);
      if (r || mine.empty()) { rcs[i] = r; return; }
      izpi_render_req q = *req;
      q.num_tiles = (uint32_t)(mine.size() / 4);
      q.tiles = mine.data();
      q.out_layout = IZPI_OUT_PACKED;
      q.post = IZPI_POST_NONE;
      c->prepare_only = true;
      rcs[i] = render_impl(c, &q, nullptr);
      c->prepare_only = false;
    });
  }
  for (std::thread& t : th) t.join();
  for (uint32_t i = 0; i < G; i++)
    if (rcs[i]) { m->err = "device " + std::to_string(i) + ": " + m->ctx[i]->err; return rcs[i]; }
  return IZPI_OK;
}

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

