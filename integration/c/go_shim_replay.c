/* go_shim_replay.c — the C call sequence of integration/go/render/gpu/renderer_gpu.go,
 * step for step, so that it runs (and is tested) where no Go toolchain exists.
 *
 *   gpu.New (renderer_gpu.go:101-226), Renderer.Render (:229-245), Renderer.RenderTiles
 *   (:251-283):
 *   1. proto.Marshal(scene) -> izpi_scene_parse_binary   (here: a .izpi file = those bytes)
 *   2. izpi_scene_set_image per loaded image texture      (here: none / a flat test texture)
 *   3. izpi_scene_to_input(aspect = W/H, bvh seed 12345) -> izpi_host_build_scene_ex(SKIP_BVH)
 *   4. izpi_gpu_open / izpi_gpu_multi_open (Options.Devices), izpi_host_scene_prim_boxes,
 *      izpi_gpu_build_bvh4(leaf izpi_host_bvh_leaf_max, PLOC) -> izpi_host_scene_set_bvh
 *   5. izpi_gpu_upload_scene / izpi_gpu_multi_upload_scene, the whole-frame request:
 *      sampler from the scene's colour representation, IZPI_POST_SPECTRAL for the
 *      spectral sampler, IZPI_POST_GAMMA_CLAMP with --png-pipeline, exposure = camera's;
 *      with --bg-spd the spectral background of Options.SpectralBackground (75 zeros, as
 *      leader mode's colours.SpectralBlack) in malloc'ed memory, as the shim's C.malloc;
 *      then izpi_gpu_prepare / izpi_gpu_multi_prepare (render.New's workspace allocation)
 *   6. Render: izpi_gpu_render / izpi_gpu_multi_render into a zeroed W*H*4 float64 canvas;
 *      with --tiles N instead RenderTiles over the frame's first N tiles (common.Tiles,
 *      spiral order): one izpi_gpu_render with IZPI_OUT_PACKED, tile list in malloc'ed
 *      memory, the packed tiles written out
 *
 *   With --ref-bvh the scene keeps the host's NewBVH4 tree (Options.BVH != BVHGPU): no
 *   SKIP_BVH flag and no GPU build. The request carries
 *   IZPI_ACC_FORWARD (Options.Accumulation's default), IZPI_ACC_RECURSIVE with --recursive.
 *   The replay is written in the subset tests/go_shim_sequence.py reads (calls of the
 *   library in plain statements and if conditions, no call inside a ?: arm), which checks
 *   that its call sequence is the shim's in every branch.
 *
 *   usage: go_shim_replay scene.izpi W H SPP out.f64 [--png-pipeline] [--devices 0,0,...]
 *                         [--bg-spd] [--tiles N] [--ref-bvh] [--recursive]
 * Exit status 0 on success; the canvas is written as raw little-endian float64.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "izpi_gpu.h"
#include "izpi_host.h"

static int fail(const char* what, const char* msg) {
  fprintf(stderr, "%s: %s\n", what, msg ? msg : "");
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 6) return fail("usage", "go_shim_replay scene.izpi W H SPP out.f64 [--png-pipeline] [--devices a,b,..]");
  const uint32_t W = (uint32_t)atoi(argv[2]), H = (uint32_t)atoi(argv[3]), spp = (uint32_t)atoi(argv[4]);
  int png = 0, devices[16], ndev = 0, bg_spd = 0, ntiles = 0, ref_bvh = 0, recursive = 0;
  for (int i = 6; i < argc; i++) {
    if (!strcmp(argv[i], "--png-pipeline")) png = 1;
    else if (!strcmp(argv[i], "--bg-spd")) bg_spd = 1;
    else if (!strcmp(argv[i], "--ref-bvh")) ref_bvh = 1;
    else if (!strcmp(argv[i], "--recursive")) recursive = 1;
    else if (!strcmp(argv[i], "--tiles") && i + 1 < argc) ntiles = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--devices") && i + 1 < argc) {
      for (char* t = strtok(argv[++i], ","); t && ndev < 16; t = strtok(NULL, ",")) devices[ndev++] = atoi(t);
    }
  }
  /* 1. the marshalled transport.Scene */
  FILE* f = fopen(argv[1], "rb");
  if (!f) return fail("open", argv[1]);
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* buf = (uint8_t*)malloc(n > 0 ? (size_t)n : 1);
  if (fread(buf, 1, (size_t)n, f) != (size_t)n) return fail("read", argv[1]);
  fclose(f);
  izpi_proto_scene* ps = NULL;
  if (izpi_scene_parse_binary(buf, (uint64_t)n, &ps)) return fail("izpi_scene_parse_binary", izpi_host_last_error());
  free(buf);
  izpi_proto_info info;
  if (izpi_scene_info(ps, &info)) return fail("izpi_scene_info", izpi_host_last_error());
  /* 2. image textures: a flat mid-grey 2x2 float64 NRGBA texture per referenced file */
  for (uint32_t i = 0; i < info.num_image_textures; i++) {
    const double texels[16] = {0.5, 0.5, 0.5, 1, 0.5, 0.5, 0.5, 1, 0.5, 0.5, 0.5, 1, 0.5, 0.5, 0.5, 1};
    if (izpi_scene_set_image(ps, izpi_scene_image_file(ps, i), 2, 2, texels))
      return fail("izpi_scene_set_image", izpi_host_last_error());
  }
  /* 3. transport.ToScene up to the BVH, leader-mode aspect override */
  const izpi_scene_input* in = NULL;
  if (izpi_scene_to_input(ps, (double)W / (double)H, 12345, &in)) return fail("izpi_scene_to_input", izpi_host_last_error());
  izpi_host_scene* host = NULL;
  const uint32_t flags = ref_bvh ? 0u : (uint32_t)IZPI_HOST_SKIP_BVH;
  if (izpi_host_build_scene_ex(in, flags, &host)) return fail("izpi_host_build_scene_ex", izpi_host_last_error());
  /* 4. device(s), GPU BVH4 */
  izpi_ctx* ctx = NULL;
  izpi_multi* m = NULL;
  if (ndev > 1) {
    if (izpi_gpu_multi_open(devices, (uint32_t)ndev, &m)) return fail("izpi_gpu_multi_open", "");
    ctx = izpi_gpu_multi_context(m, 0);
  } else if (izpi_gpu_open(ndev ? devices[0] : 0, &ctx)) {
    return fail("izpi_gpu_open", "");
  }
  const izpi_scene_desc* desc;
  if (!ref_bvh) {  /* Options.BVH == BVHGPU */
    desc = izpi_host_scene_desc(host);
    const uint32_t np = desc->num_tris + desc->num_spheres;
    if (np > 0) {
      double* boxes = (double*)malloc(sizeof(double) * 6 * np);
      izpi_bvh4_node* nodes = (izpi_bvh4_node*)malloc(sizeof(izpi_bvh4_node) * 2 * np);
      uint32_t* order = (uint32_t*)malloc(sizeof(uint32_t) * np);
      uint32_t num_nodes = 0;
      double ms = 0;
      if (izpi_host_scene_prim_boxes(host, boxes)) return fail("izpi_host_scene_prim_boxes", izpi_host_last_error());
      if (izpi_gpu_build_bvh4(ctx, boxes, np, izpi_host_bvh_leaf_max(desc), IZPI_BVH_PLOC | IZPI_BVH_SAH, nodes, 2 * np, &num_nodes, order, &ms))
        return fail("izpi_gpu_build_bvh4", izpi_gpu_last_error(ctx));
      if (izpi_host_scene_set_bvh(host, nodes, num_nodes, order)) return fail("izpi_host_scene_set_bvh", izpi_host_last_error());
      free(boxes); free(nodes); free(order);
    }
  }
  /* 5. upload and the request */
  if (m) {
    if (izpi_gpu_multi_upload_scene(m, izpi_host_scene_desc(host))) return fail("upload", izpi_gpu_multi_last_error(m));
  } else if (izpi_gpu_upload_scene(ctx, izpi_host_scene_desc(host))) {
    return fail("upload", izpi_gpu_last_error(ctx));
  }
  desc = izpi_host_scene_desc(host);
  izpi_render_req req;
  memset(&req, 0, sizeof req);
  req.abi_version = IZPI_ABI_VERSION;
  req.width = W; req.height = H; req.spp = spp; req.max_depth = 50;
  req.out_layout = IZPI_OUT_CANVAS;
  req.seed = 12345;
  req.exposure = desc->camera.exposure;
  req.accumulation = IZPI_ACC_FORWARD;
  if (recursive) req.accumulation = IZPI_ACC_RECURSIVE;
  uint32_t post = IZPI_POST_NONE;
  req.sampler = IZPI_SAMPLER_COLOUR;
  double* bg = NULL;
  if (info.colour_representation == IZPI_COLOUR_SPECTRAL) {  /* leader.go:77-81 */
    req.sampler = IZPI_SAMPLER_SPECTRAL;
    post |= IZPI_POST_SPECTRAL;
    if (bg_spd) {  /* colours.SpectralBlack: 75 zeros at 380, 385, ... 750 nm */
      bg = (double*)malloc(2 * 75 * sizeof(double));
      for (int i = 0; i < 75; i++) { bg[i] = 380 + 5 * (double)i; bg[75 + i] = 0.0; }
      req.num_bg_spd = 75;
      req.bg_spd_wavelengths = bg;
      req.bg_spd_values = bg + 75;
    }
  }
  if (png) post |= IZPI_POST_GAMMA_CLAMP;
  req.post = post;
  /* render.New's share: the request's workspace prepared before the first frame */
  if (m) {
    if (izpi_gpu_multi_prepare(m, &req)) return fail("prepare", izpi_gpu_multi_last_error(m));
  } else if (izpi_gpu_prepare(ctx, &req)) {
    return fail("prepare", izpi_gpu_last_error(ctx));
  }
  /* 6. Render, or RenderTiles */
  size_t nout = (size_t)W * H * 4;
  double* pix = NULL;
  izpi_render_stats st;
  if (ntiles > 0) {
    uint32_t* all = (uint32_t*)malloc(4 * sizeof(uint32_t) * ((size_t)W * H / 16 + 16));
    const uint32_t nt = izpi_host_tiles(W, H, all, (uint32_t)((size_t)W * H / 16 + 16));
    if (nt == 0 || (uint32_t)ntiles > nt) return fail("tiles", "bad --tiles");
    izpi_render_req tr = req;
    tr.num_tiles = (uint32_t)ntiles;
    tr.tiles = all;
    tr.out_layout = IZPI_OUT_PACKED;
    tr.post = IZPI_POST_NONE;
    nout = (size_t)(izpi_gpu_output_bytes(&tr) / sizeof(double));
    pix = (double*)calloc(nout, sizeof(double));
    if (izpi_gpu_render(ctx, &tr, pix, &st)) return fail("render tiles", izpi_gpu_last_error(ctx));
    free(all);
  } else {
    pix = (double*)calloc(nout, sizeof(double));
    if (m) {
      if (izpi_gpu_multi_render(m, &req, pix, NULL)) return fail("render", izpi_gpu_multi_last_error(m));
    } else if (izpi_gpu_render(ctx, &req, pix, &st)) {
      return fail("render", izpi_gpu_last_error(ctx));
    }
  }
  FILE* o = fopen(argv[5], "wb");
  if (!o || fwrite(pix, sizeof(double), nout, o) != nout) return fail("write", argv[5]);
  fclose(o);
  free(pix);
  free(bg);
  /* Renderer.Close */
  if (m) izpi_gpu_multi_close(m);
  else izpi_gpu_close(ctx);
  izpi_host_scene_free(host);
  izpi_scene_free(ps);
  printf("{\"sampler\": \"%s\", \"devices\": %d, \"post\": %u, \"bg_spd\": %u, \"tiles\": %d, \"ref_bvh\": %d, \"recursive\": %d}\n",
         req.sampler == IZPI_SAMPLER_SPECTRAL ? "spectral" : "colour", ndev > 1 ? ndev : 1, post, req.num_bg_spd, ntiles, ref_bvh,
         recursive);
  return 0;
}
