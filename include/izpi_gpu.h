/* izpi_gpu.h — C ABI of the MI355X path-tracing inner loop for izpi.
 *
 * Drop-in boundary: a Go `GPURenderer` implementing
 * render.Renderer (internal/render/renderer.go:26-28) flattens the scene once and
 * calls izpi_gpu_render per frame (or per tile batch), replacing
 *   render.New(...).Render(ctx)      leader/leader.go:136-158, renderer.go:73-222
 * and, per tile, the per-pixel loops
 *   renderRectRGB                     render/rgb.go:12-57
 *   renderRectSpectral / RenderPixelSpectral  render/spectral.go:14-106
 * The per-sample Sampler interface (sampler.go:30-33) is deliberately NOT the
 * boundary: cgo costs ~35 ns per call (hitable/bvh4_simd_arm64.go:14).
 *
 * Ownership: host arrays passed to izpi_gpu_upload_scene are read during the call
 * only; the library owns all device buffers inside the opaque context. Output
 * buffers are caller-allocated. Calls on one context are serialised by the caller;
 * one context per GPU. No C++ exception or abort() crosses this ABI: every entry
 * point returns an IZPI_* status and izpi_gpu_last_error() explains failures.
 */
#ifndef IZPI_GPU_H
#define IZPI_GPU_H
#include <stddef.h>
#include <stdint.h>
#include "izpi_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct izpi_ctx izpi_ctx;

/* Flattened scene, as the Go host holds it after transport.ToScene
 * (transport/transport.go:53-92) and hitable.NewBVH4 (hitable/bvh4.go:517-593).
 * Every per-triangle array is [num_tris][3] doubles unless noted. */
typedef struct izpi_scene_desc {
  uint32_t abi_version;      /* IZPI_ABI_VERSION */
  uint32_t num_nodes;        /* len(BVH4.Nodes) */
  uint32_t num_prims;        /* len(BVH4.Primitives) */
  uint32_t num_tris, num_spheres, num_lights, num_materials, num_textures;
  uint32_t num_spd;          /* entries in spd_wavelengths / spd_values */
  uint32_t flags;            /* IZPI_SCENE_* (ABI 3; was padding, 0 in ABI 1 and 2 descriptors) */
  uint64_t num_texels;       /* doubles in texels[] */
  const izpi_bvh4_node* nodes;  /* BVH4.Nodes, root = 0 (bvh4.go:42-47) */
  const uint32_t* prim_ref;     /* BVH4.Primitives (leaf order, bvh4.go:585-590) as IZPI_PRIM_REF */
  /* hitable.Triangle fields (triangle.go:20-52) */
  const double* tri_v0;
  const double* tri_v1;
  const double* tri_v2;
  const double* tri_e1;        /* edge1 = v1 - v0 */
  const double* tri_e2;        /* edge2 = v2 - v0 */
  const double* tri_normal;    /* unit(edge1 x edge2) */
  const double* tri_tangent;   /* normal-mapping frame */
  const double* tri_bitangent;
  const double* tri_uv;        /* [num_tris][6]: u0,v0,u1,v1,u2,v2 */
  const double* tri_area;      /* [num_tris] */
  const uint32_t* tri_mat;     /* [num_tris] material index */
  /* hitable.Sphere fields (sphere.go:20-27) */
  const double* sph_center0;   /* [num_spheres][3] */
  const double* sph_center1;   /* [num_spheres][3] */
  const double* sph_time;      /* [num_spheres][2]: time0, time1 */
  const double* sph_radius;    /* [num_spheres] */
  const uint32_t* sph_mat;     /* [num_spheres] */
  /* Scene.Lights = every hitable whose material IsEmitter() (transport.go:67-72) */
  const uint32_t* light_ref;   /* [num_lights] IZPI_PRIM_REF, transport order */
  const izpi_material* materials;
  const izpi_texture* textures;
  const double* texels;        /* image textures, float64 NRGBA */
  const double* spd_wavelengths;
  const double* spd_values;
  izpi_camera camera;
} izpi_scene_desc;

/* izpi_scene_desc.flags */
enum {
  /* Store the inner nodes' child boxes quantised to 8 bits per bound against a per-node f32
   * origin and power-of-two scale (64-B nodes instead of 128 B). Every decoded box contains
   * the node's own f32 box (rounded outwards; checked at upload in the kernels' own f32
   * arithmetic), so the traversal visits every node the exact boxes do, and maybe more: the
   * closest hit can differ only where two primitives are hit at the same t (A11) or a box
   * is culled at tMax by float rounding. The traversal is that of the BVH whose slot boxes
   * are the decoded ones (the oracle restates it, oracle_quantize_bvh4).
   * Ignored (the scene traverses its exact boxes) when a bound is not finite. */
  IZPI_SCENE_QUANTIZED_BVH = 1
};

enum { IZPI_SAMPLER_COLOUR = 2, IZPI_SAMPLER_SPECTRAL = 5 }; /* sampler.go:13-20 */
enum {
  IZPI_OUT_CANVAS = 0, /* W*H*4 float64 NRGBA canvas; pixel (x,y) lands in row H-y (rgb.go:41) */
  IZPI_OUT_PACKED = 1  /* tiles packed in request order, each (x1-x0+1)*(y1-y0+1)*4,
                          row-major by sample row y then x; the row-H-y rule is applied
                          by izpi_gpu_unpack_tiles */
};

/* Launch tuning of one render call. Every setting gives a bit-identical canvas and
 * identical counters; they trade memory and scheduling only. Zero fields take the
 * defaults, and a NULL izpi_render_req.tuning means all defaults. The library reads
 * no environment variables: an inherited variable cannot change a production render. */
typedef struct izpi_render_tuning {
  uint32_t slots;        /* cap on paths in flight; 0 = 256M, within 15/32 of the HBM this context may use */
  uint32_t chunk_units;  /* per-sample results held at once (pixels x spp of a chunk); 0 = 1/8 of that HBM */
  uint32_t rec_dense;    /* unwinding levels per record slot; 0 = 8 (Colour), 32 (Spectral) */
  uint32_t pool_div;     /* record slots per overflow block; 0 = 16 (Colour scenes without glass), 4 (others) */
  uint32_t trace_chunk;  /* queue entries per k_trace2 dequeue; 0 = 512 */
  uint32_t refill_min;   /* idle lanes before a k_trace2 refill (1..64); 0 = 24 (40 with the BVH in LDS) */
  uint32_t prim_weight;  /* k_trace2 primitive-step weight against node steps, x/16; 0 = 32 (24 with the BVH in LDS) */
  uint32_t flags;        /* IZPI_TUNE_* */
  uint64_t tail_paths;   /* k_tail takes over at <= this many paths; 0 = the resident lanes */
  /* izpi_gpu_render_rank: longest wait for the other ranks in one collective step, in ms
   * (the gather waits for the slowest rank's render: set it above a frame's time); past it,
   * or when RCCL reports an asynchronous error, the communicator is aborted and the call
   * returns IZPI_ERR_PEER. 0 = wait without a deadline (the async-error poll still runs). */
  uint32_t peer_timeout_ms;
  uint32_t pad_tuning;
} izpi_render_tuning;
enum {
  IZPI_TUNE_NO_DIST = 1,          /* k_trace2 runs each leaf's tests in its own lane */
  IZPI_TUNE_GENERAL_TRACE = 2,    /* the sphere-capable k_trace2 instance on triangle-only scenes */
  IZPI_TUNE_NO_LEAF_SHORTCUT = 4, /* re-test every leaf box (A10) instead of inferring it */
  IZPI_TUNE_SCALAR_SLAB = 8,      /* the scalar twin of RayAABB4 for every ray */
  IZPI_TUNE_NO_TAIL = 16,         /* no k_tail: wavefront passes to the end */
  IZPI_TUNE_PASS_LOG = 32,        /* diagnostics: per-pass device times on stderr */
  IZPI_TUNE_NO_LDS_BVH = 64,      /* small scenes: traverse from global memory, not the per-block LDS copy */
  IZPI_TUNE_NO_RAY_LDS = 128,     /* triangle-only scenes without (u, v) reads: primitive tests re-read the ray from global memory */
  IZPI_TUNE_NO_PRIM_LDS = 256,    /* small scenes: shading reads the primitives' records from global memory, not the per-block LDS copy */
  IZPI_TUNE_NO_PLACE_PICK = 512,  /* ignored since ABI 3 (the record arrays' page pick of ABI 2 is gone) */
  IZPI_TUNE_NO_QNODES = 1024      /* a quantised scene (IZPI_SCENE_QUANTIZED_BVH): k_trace2 reads the decoded 128-B nodes
                                     instead of the 64-B quantised ones (the same boxes) */
};

typedef struct izpi_render_req {
  uint32_t width, height;     /* canvas size = Renderer sizeX, sizeY */
  uint32_t spp;               /* numSamples */
  uint32_t max_depth;         /* maxDepth (main.go:25 default 50) */
  uint32_t sampler;           /* IZPI_SAMPLER_* */
  uint32_t out_layout;        /* IZPI_OUT_* */
  uint32_t num_tiles;         /* 0 = whole frame in common.Tiles steps */
  uint32_t num_bg_spd;        /* entries of the spectral background SPD (0 = black) */
  const uint32_t* tiles;      /* [num_tiles][4] = x0,y0,x1,y1 inclusive (workUnit, renderer.go:56-70) */
  const double* bg_spd_wavelengths; /* spectral background (Spectral.background) */
  const double* bg_spd_values;
  double background[3];       /* Colour background (leader.go:140: black) */
  uint64_t seed;              /* master seed of the per-sample LCG streams */
  uint32_t post;              /* IZPI_POST_*: post-processing of a whole-frame IZPI_OUT_CANVAS render */
  uint32_t abi_version;       /* IZPI_ABI_VERSION (3); 0 = a request laid out by ABI 1 (this field was padding):
                                 its tuning, when set, is read as ABI 1's izpi_render_tuning, which ended at
                                 tail_paths; the later fields keep their defaults. A request of ABI 1 or 2
                                 ends at `tuning`: it renders IZPI_ACC_RECURSIVE */
  double exposure;            /* XYZToRGB exposure (Scene.Exposure = camera exposure) */
  const izpi_render_tuning* tuning; /* NULL = defaults */
  uint32_t accumulation;      /* IZPI_ACC_* (ABI 3) */
  uint32_t pad_req;
} izpi_render_req;

/* How a path's radiance is summed (izpi_render_req.accumulation). Both trace the same
 * rays with the same random draws, so every counter is the same.
 *  IZPI_ACC_RECURSIVE: the recursion of Colour.Sample / SampleSpectral (colour.go:44-57,
 *    sampler/spectral.go:60-72) unwound from the deepest bounce, in its operation order:
 *    bit-identical to the CPU restatement. The default.
 *  IZPI_ACC_FORWARD: the path's throughput is carried forward, T = (T * att) * (s / p) per
 *    non-specular bounce and T *= att per specular one, and the sample is T * (terminal
 *    radiance). Only the rounding differs (a few ulp per bounce; pixel RMSE < 1e-6, the
 *    north star's contract); NaN and Inf land where the recursion puts them (DESIGN.md
 *    section 3.2). No per-bounce records: a smaller, faster workspace. */
enum { IZPI_ACC_RECURSIVE = 0, IZPI_ACC_FORWARD = 1 };

/* Post-processing applied by Render for the Spectral sampler (renderer.go:215-219):
 * spectral.FireflyRejection (firefly_rejection.go:12-113) then spectral.XYZToRGB
 * (rgb_image.go:28-67, ACEScg matrix :13-17) with req->exposure. */
enum { IZPI_POST_NONE = 0, IZPI_POST_SPECTRAL = 1,
       /* bit 2: the leader's "png" output pipeline, Gamma then Clamp(1.0) (leader.go:179-182),
        * after the spectral post when both are set */
       IZPI_POST_GAMMA_CLAMP = 2 };

/* postprocess.Filter kinds for izpi_gpu_postprocess (postprocess/api.go:10-14) */
enum { IZPI_FILTER_GAMMA = 1, /* gamma.go:24-41, R,G,B = math.Sqrt; param unused */
       IZPI_FILTER_CLAMP = 2  /* clamp.go:27-51, v < max ? v : max; param = max */ };
#define IZPI_MAX_FILTERS 8

/* Per-render counters. The traversal is bit-identical to the CPU restatement, so
 * these equal the oracle's counts exactly (used for algorithmic bytes, §8(d)). */
typedef struct izpi_render_stats {
  uint64_t rays;          /* Sampler calls past the depth check == numRays (colour.go:38) */
  uint64_t node_visits;   /* BVH4 node loads (bvh4.go:91), incl. dielectric path-length traversals */
  uint64_t tri_tests;     /* Triangle.Hit calls inside traversal (bvh4.go:127) */
  uint64_t sph_tests;     /* Sphere.Hit calls inside traversal */
  uint64_t light_tri_tests; /* Triangle.PDFValue intersection tests (hitable_slice.go:98-105) */
  uint64_t light_sph_tests; /* Sphere.PDFValue intersection tests */
  uint64_t samples;       /* pixel samples evaluated */
  double kernel_ms;       /* device time of the traversal kernel (k_trace), HIP events on the library stream */
  double shade_ms;        /* device time of the shading kernel (k_shade) */
  double total_ms;        /* device time of the whole render call (kernels + accumulation) */
  uint32_t launches;      /* k_trace launches (wavefront iterations) in the call */
  uint32_t pad;
  /* traversal-kernel work breakdown (diagnostics, not reference quantities): wave-level
   * loop iterations that ran a node step / a primitive step, and leaf visits taken by a
   * shortcut (no node load). */
  uint64_t node_steps, prim_steps, leaf_shortcuts;
  /* device time of k_tail, which traces AND shades the last paths once every work unit
   * has started (not included in kernel_ms / shade_ms) */
  double tail_ms;
  /* the part of node_visits / tri_tests / sph_tests done inside k_tail */
  uint64_t tail_node_visits, tail_tri_tests, tail_sph_tests;
  /* shading passes deferred one pass for want of an overflow record block (diagnostic) */
  uint64_t parks;
  /* device memory of the context after the call: render workspace and uploaded scene */
  uint64_t workspace_bytes, scene_bytes;
  /* wavefront configuration of the call: paths in flight, unwinding records per path kept
   * in the dense array, overflow record blocks, samples per pixel per chunk */
  uint32_t slots, rec_dense, pool_blocks, chunk_spp;
  /* host wall time of the call's workspace allocations (a fresh context's first frame pays
   * for its HBM here; 0 when every buffer was already large enough) */
  double alloc_ms;
} izpi_render_stats;

/* Hit record returned by izpi_gpu_trace: BVH4.Hit (bvh4.go:49-164) followed by
 * the closest primitive's record (triangle.go:193-265 / sphere.go:63-95). */
typedef struct izpi_hit {
  double t, u, v;
  double p[3];
  double normal[3];
  uint32_t prim_ref;  /* IZPI_PRIM_REF of the closest primitive, 0xFFFFFFFF on miss */
  uint32_t hit;       /* 0/1 */
} izpi_hit;

/* Open a context on HIP device `device` (>=0). */
int izpi_gpu_open(int device, izpi_ctx** out);
int izpi_gpu_close(izpi_ctx* ctx);
const char* izpi_gpu_last_error(izpi_ctx* ctx);

/* Copy a flattened scene to the device (repacking to the GPU layouts of DESIGN.md). */
int izpi_gpu_upload_scene(izpi_ctx* ctx, const izpi_scene_desc* scene);

/* Render into a caller-owned HOST buffer: W*H*4 doubles for IZPI_OUT_CANVAS.
 * Pixels outside the requested tiles are left untouched (the caller zero-fills,
 * like floatimage.NewFloat64NRGBA). This is the Renderer.Render drop-in. */
int izpi_gpu_render(izpi_ctx* ctx, const izpi_render_req* req, double* out_host, izpi_render_stats* stats);

/* Size and allocate the render workspace of requests shaped like `req` (and run the device's
 * first work on it), so that the first frame renders only: the setup render.New does when it
 * allocates the canvas (renderer.go:73-104), ahead of the Render izpi times
 * (renderer.go:170,213). With a communicator (izpi_gpu_comm_init, nranks > 1) this rank's share
 * of izpi_gpu_render_rank is prepared. Optional: a render sizes its own workspace otherwise. */
int izpi_gpu_prepare(izpi_ctx* ctx, const izpi_render_req* req);

/* Same, but `out_dev` is a DEVICE pointer (e.g. a framebuffer owned by the caller
 * on this context's device). Used by multi-GPU runs that gather over RCCL. */
int izpi_gpu_render_device(izpi_ctx* ctx, const izpi_render_req* req, double* out_dev, izpi_render_stats* stats);

/* Scatter packed tiles (IZPI_OUT_PACKED, device memory) into a W*H*4 canvas
 * (device memory) applying the row = H - y rule of rgb.go:41 / spectral.go:36. */
int izpi_gpu_unpack_tiles(izpi_ctx* ctx, const izpi_render_req* req, const double* packed_dev, double* canvas_dev);

/* FireflyRejection + XYZToRGB of a W*H*4 float64 CIE-XYZ canvas (device memory) into
 * `rgba_dev` (device memory, may not alias `xyz_dev`): the multi-GPU path runs it on
 * rank 0 after the gather. */
int izpi_gpu_spectral_post(izpi_ctx* ctx, const double* xyz_dev, double* rgba_dev, uint32_t width, uint32_t height,
                           double exposure);

/* postprocess.Pipeline.Apply (pipeline.go:20-31) on a W*H*4 float64 canvas in device
 * memory, in place: filters[i] (IZPI_FILTER_*) with params[i], in list order. */
int izpi_gpu_postprocess(izpi_ctx* ctx, double* canvas_dev, uint32_t width, uint32_t height, const uint32_t* filters,
                         const double* params, uint32_t num_filters);

/* GPU BVH4 builder: Morton codes and a radix sort, then a binary
 * tree (method: IZPI_BVH_PLOC clustering or IZPI_BVH_LBVH radix tree), collapsed to
 * 4-wide nodes with collectChildren's rule (or, with IZPI_BVH_SAH, the collapse of least
 * surface-area cost) and <= leaf_max (1..4) primitives per leaf, written in the reference's BVH4Node
 * format (conservative f32 bounds, separate leaf nodes), breadth-first with the root at
 * 0. boxes: [n][6] f64 host array (izpi_host_scene_prim_boxes). nodes: host array of at
 * least 2n entries; order[k] (n entries) = input index of leaf position k. The topology
 * differs from hitable.NewBVH4's, so images match the reference tree's except for
 * equal-t tie-breaks and f32 culling at tMax. */
enum { IZPI_BVH_LBVH = 0, /* Karras radix tree over the Morton order */
       IZPI_BVH_PLOC = 1, /* locally-ordered clustering (Meister & Bittner 2018) over the Morton order */
       /* flag (PLOC only): collapse to 4-wide nodes by the surface-area cost model's
        * dynamic programme instead of collectChildren's rule; leaves still hold <= leaf_max */
       IZPI_BVH_SAH = 0x100 };
int izpi_gpu_build_bvh4(izpi_ctx* ctx, const double* boxes, uint32_t n, uint32_t leaf_max, uint32_t method,
                        izpi_bvh4_node* nodes, uint32_t max_nodes, uint32_t* num_nodes, uint32_t* order, double* build_ms);

/* ---- Multi-GPU (SURVEY.md §8(b),(e)) ---------------------------------------------
 * Render fans out over the GPUs of the node in ONE call, as RendererImpl.Render fans
 * out over its workers (render/renderer.go:123-147): one host thread and stream per
 * device instead of one goroutine per core. The frame's tiles (common.Tiles in
 * grid.WalkGrid's spiral order, or req->tiles) are dealt tile % G == i; device i renders
 * its share packed; the shares are gathered to device 0 (peer copies over xGMI), which
 * scatters them into the W*H*4 canvas (row H - y, rgb.go:41) and applies req->post.
 * Per pixel-sample RNG streams make the canvas bit-identical for every G. A device may
 * appear twice in `devices` (two contexts on one GPU). */
typedef struct izpi_multi izpi_multi;
int izpi_gpu_multi_open(const int* devices, uint32_t num_devices, izpi_multi** out);
int izpi_gpu_multi_close(izpi_multi* m);
const char* izpi_gpu_multi_last_error(izpi_multi* m);
uint32_t izpi_gpu_multi_size(izpi_multi* m);
/* context of device i (e.g. for izpi_gpu_build_bvh4), owned by `m` */
izpi_ctx* izpi_gpu_multi_context(izpi_multi* m, uint32_t i);
/* the scene is replicated on every device */
int izpi_gpu_multi_upload_scene(izpi_multi* m, const izpi_scene_desc* scene);
/* izpi_gpu_prepare for every device's share of `req` */
int izpi_gpu_multi_prepare(izpi_multi* m, const izpi_render_req* req);
/* out_host: the caller's W*H*4 canvas (read first: pixels of no tile keep their values),
 * or NULL to leave the canvas in device 0's memory (timing). stats: [num_devices] or NULL. */
int izpi_gpu_multi_render(izpi_multi* m, const izpi_render_req* req, double* out_host, izpi_render_stats* stats);

/* One process per GPU (torchrun / MPI style launchers): the library's own RCCL
 * communicator. Rank 0 makes the id with izpi_gpu_comm_id and the launcher broadcasts
 * it; every rank calls izpi_gpu_comm_init on its context. */
#define IZPI_COMM_ID_BYTES 128 /* == NCCL_UNIQUE_ID_BYTES */
int izpi_gpu_comm_id(uint8_t* id /* [IZPI_COMM_ID_BYTES] */);
int izpi_gpu_comm_init(izpi_ctx* ctx, uint32_t nranks, uint32_t rank, const uint8_t* id /* [IZPI_COMM_ID_BYTES] */);
/* Collective: every rank passes the same whole-frame request. Rank r renders the tiles
 * t % nranks == r, ncclGather moves the packed shares to rank 0, which writes the canvas
 * into out_dev (device memory on its GPU; ignored on other ranks) and applies req->post.
 * stats: this rank's share. Every rank runs the same collectives whatever fails locally
 * (its own HIP errors included), and two ncclAllReduce(max) agreement steps (after the
 * buffers, after the gather) give every rank the worst status: a rank's own failure returns
 * its status, a failure of another rank IZPI_ERR_PEER (last_error names the rank).
 * A rank that dies or hangs instead of failing: each collective step is waited on by
 * polling the stream and ncclCommGetAsyncError; an asynchronous RCCL error, or a wait past
 * tuning->peer_timeout_ms, aborts the communicator (ncclCommAbort) and returns
 * IZPI_ERR_PEER. The context then has no communicator: izpi_gpu_comm_init makes a new one. */
int izpi_gpu_render_rank(izpi_ctx* ctx, const izpi_render_req* req, double* out_dev, izpi_render_stats* stats);

/* Progress of the render running on ctx (izpi_gpu_render, _render_device, _render_rank),
 * callable from another thread while it runs (RendererImpl.Render's per-tile progress
 * bar, renderer.go:119-121, rgb.go:54-56): samples (pixels x spp) whose paths have
 * finished, as of the library's last queue poll (every <= 8 wavefront passes, a lower
 * bound), and the request's samples. After the call returns, done == total (both 0 when
 * the request failed its checks), whether or not it succeeded. The multi
 * form sums the contexts of `m` (their shares of one frame). */
int izpi_gpu_progress(izpi_ctx* ctx, uint64_t* samples_done, uint64_t* samples_total);
int izpi_gpu_multi_progress(izpi_multi* m, uint64_t* samples_done, uint64_t* samples_total);

/* Bytes of device output izpi_gpu_render_device writes for `req`. */
uint64_t izpi_gpu_output_bytes(const izpi_render_req* req);

/* Component entry points (parity tests of the path's pieces). All arrays host. */
/* Closest hit through World (HitableSlice{BVH4}); rays are [n][8]: o[3], d[3], tmin, tmax. */
int izpi_gpu_trace(izpi_ctx* ctx, const double* rays, uint32_t n, izpi_hit* out);
/* RayAABB4 masks (bvh4_simd_generic.go:10-52): boxes [n][24] f32 (SoA as BVH4Node),
 * rays [n][7] f32: org[3], invdir[3], tmax. */
int izpi_gpu_ray_aabb4(izpi_ctx* ctx, const float* boxes, const float* rays, uint32_t n, uint8_t* masks);
/* Go-math on device, op codes in izpi_amd/csrc/gomath.h order: 0 sin 1 cos 2 tan 3 exp
 * 4 log 5 pow(x,y) 6 atan2(x,y) 7 asin 8 sqrt 9 div(x,y) 10 atan, 11/12 sin/cos from one
 * shared reduction (x >= 0), 13 the shared-reciprocal vector division (= x / y); 14
 * calculatePathLength's clamped |exit - p| (dielectric.go:141-150) with x the hit points
 * and y the exit points as [n][3]; spectral helpers:
 * 32/33 SampleWavelength(x) lambda/pdf (spectral.go:184-224), 34/35/36 GetCIEValues(x)
 * x/y/z (spectral.go:227-253); 37 SpectralConstant.Value(x) of the uploaded scene's texture
 * number y (spectral_constant.go:65-106, needs a scene). */
int izpi_gpu_gomath(izpi_ctx* ctx, int op, const double* x, const double* y, uint32_t n, double* out);

#ifdef __cplusplus
}
#endif
#endif
