// izpi_render.cpp — a C++ host for the MI355X path: what `izpi --role standalone`
// (cmd/izpi/main.go, leader/leader.go:37-230) does for one frame, through the C ABI
// only (include/izpi_gpu.h, include/izpi_host.h). No Python, no Go.
//
//   izpi-render --scene cornell.pbtxt [--obj mesh.obj --obj-material White] [--x 1024 --y 1024]
//               [--samples 512] [--depth 50] [--bvh gpu|reference] [--quantized] [--png-pipeline]
//               [--accumulation forward|recursive] [--out image.pfm] [--raw canvas.f64]
//               [--device 0 | --gpus N] [--seed 12345]
//
// Defaults are the Go shim's: the GPU-built tree and the forward accumulation
// (IZPI_ACC_FORWARD; --accumulation recursive is bit-identical to the CPU oracle).
// --quantized uploads the tree with 64-B quantised nodes (IZPI_SCENE_QUANTIZED_BVH).
//
// The scene file is read as leader.go:54-75 does (.pbtxt text, .izpi binary); a SPECTRAL
// scene renders with the spectral sampler and Render's post-processing (leader.go:77-81,
// renderer.go:215-219). --obj streams a Wavefront mesh into the scene with the
// transforms of scenes/spectral.go:644-646. The canvas is written as a PFM (float32 RGB,
// bottom row first) and/or the raw W*H*4 float64 canvas.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "../../include/izpi_gpu.h"
#include "../../include/izpi_host.h"

namespace {

bool read_file(const std::string& path, std::vector<char>& out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + n);
  fclose(f);
  return true;
}

[[noreturn]] void die(const std::string& m) {
  fprintf(stderr, "izpi-render: %s\n", m.c_str());
  exit(1);
}

std::string dir_of(const std::string& p) {
  const size_t k = p.find_last_of('/');
  return k == std::string::npos ? "." : p.substr(0, k);
}

// -(60 * math.Pi / 180) as Go evaluates the constant expression: pi/3 rounded once
constexpr double kMinus60Deg = -0x1.0c152382d7366p+0;  // == -ingest.go_radians(60) (test_ingest.py)

}  // namespace

int main(int argc, char** argv) {
  std::string scene_path, obj_path, obj_material = "White", out_pfm, out_raw, bvh = "gpu", acc = "forward";
  bool quantized = false;
  uint32_t W = 1024, H = 1024, spp = 16, depth = 50, device = 0, gpus = 1;
  uint64_t seed = 12345;
  bool png = false;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string { if (i + 1 >= argc) die("missing value for " + a); return argv[++i]; };
    if (a == "--scene") scene_path = val();
    else if (a == "--obj") obj_path = val();
    else if (a == "--obj-material") obj_material = val();
    else if (a == "--x") W = (uint32_t)atoi(val().c_str());
    else if (a == "--y") H = (uint32_t)atoi(val().c_str());
    else if (a == "--samples") spp = (uint32_t)atoi(val().c_str());
    else if (a == "--depth") depth = (uint32_t)atoi(val().c_str());
    else if (a == "--bvh") bvh = val();
    else if (a == "--quantized") quantized = true;
    else if (a == "--accumulation") acc = val();
    else if (a == "--png-pipeline") png = true;
    else if (a == "--out") out_pfm = val();
    else if (a == "--raw") out_raw = val();
    else if (a == "--device") device = (uint32_t)atoi(val().c_str());
    else if (a == "--gpus") gpus = (uint32_t)atoi(val().c_str());
    else if (a == "--seed") seed = strtoull(val().c_str(), nullptr, 10);
    else die("unknown option " + a);
  }
  if (scene_path.empty()) die("--scene is required");
  if (bvh != "gpu" && bvh != "reference") die("--bvh must be gpu or reference");
  if (acc != "forward" && acc != "recursive") die("--accumulation must be forward or recursive");
  // ---- scene file (leader.go:54-75)
  std::vector<char> text;
  if (!read_file(scene_path, text)) die("cannot read " + scene_path);
  izpi_proto_scene* ps = nullptr;
  const std::string ext = scene_path.size() > 5 ? scene_path.substr(scene_path.size() - 5) : "";
  int rc;
  if (ext == "pbtxt") rc = izpi_scene_parse_text(text.data(), text.size(), &ps);
  else if (ext == ".izpi") rc = izpi_scene_parse_binary(text.data(), text.size(), &ps);
  else die("Unknown scene file extension: " + scene_path);
  if (rc) die(izpi_host_last_error());
  izpi_proto_info info;
  izpi_scene_info(ps, &info);
  if (info.num_image_textures) die("image textures need a host-side decoder (not part of this tool)");
  // ---- optional streamed mesh (scenes/spectral.go:639-657)
  if (!obj_path.empty()) {
    std::vector<char> obj;
    if (!read_file(obj_path, obj)) die("cannot read " + obj_path);
    izpi_obj* mesh = nullptr;
    if (izpi_obj_parse(obj.data(), obj.size(), dir_of(obj_path).c_str(), 0, &mesh)) die(izpi_host_last_error());
    izpi_obj_scale(mesh, 90.0, 90.0, 90.0);
    izpi_obj_rotate(mesh, 0.0, kMinus60Deg, 0.0);
    izpi_obj_translate(mesh, 50.0, 25.1, 60.0);
    izpi_obj_info oi;
    izpi_obj_info_get(mesh, &oi);
    for (uint32_t g = 0; g < oi.num_groups; g++) {
      uint64_t n = 0;
      if (izpi_obj_group_to_triangles(mesh, g, 1, nullptr, 0, &n)) die(izpi_host_last_error());
      std::vector<izpi_tri_in> tris(n);
      if (n && izpi_obj_group_to_triangles(mesh, g, 1, tris.data(), n, &n)) die(izpi_host_last_error());
      if (n && izpi_scene_add_triangles(ps, tris.data(), n, obj_material.c_str())) die(izpi_host_last_error());
    }
    izpi_obj_free(mesh);
  }
  const bool spectral = info.colour_representation == IZPI_COLOUR_SPECTRAL;
  // ---- transport.ToScene, BVH, upload
  auto t0 = std::chrono::steady_clock::now();
  const izpi_scene_input* in = nullptr;
  if (izpi_scene_to_input(ps, (double)W / H, 12345, &in)) die(izpi_host_last_error());
  izpi_host_scene* host = nullptr;
  if (izpi_host_build_scene_ex(in, bvh == "gpu" ? IZPI_HOST_SKIP_BVH : 0u, &host)) die(izpi_host_last_error());
  // --gpus N: one Render fans out over GPUs 0..N-1 (izpi_gpu_multi_*, renderer.go:123-147)
  izpi_ctx* ctx = nullptr;
  izpi_multi* multi = nullptr;
  if (gpus > 1) {
    std::vector<int> devs(gpus);
    for (uint32_t i = 0; i < gpus; i++) devs[i] = (int)i;
    if (izpi_gpu_multi_open(devs.data(), gpus, &multi)) die("izpi_gpu_multi_open failed (fewer GPUs?)");
    ctx = izpi_gpu_multi_context(multi, 0);
  } else if (izpi_gpu_open((int)device, &ctx)) {
    die("izpi_gpu_open failed (no HIP device?)");
  }
  const izpi_scene_desc* desc = izpi_host_scene_desc(host);
  if (bvh == "gpu") {
    const uint32_t n = desc->num_tris + desc->num_spheres;
    std::vector<double> boxes(6 * (size_t)n);
    std::vector<izpi_bvh4_node> nodes(2 * (size_t)n + 1);
    std::vector<uint32_t> order(n + 1);
    uint32_t num_nodes = 0;
    double ms = 0;
    if (n) {
      izpi_host_scene_prim_boxes(host, boxes.data());
      if (izpi_gpu_build_bvh4(ctx, boxes.data(), n, izpi_host_bvh_leaf_max(desc), IZPI_BVH_PLOC | IZPI_BVH_SAH, nodes.data(), (uint32_t)nodes.size(), &num_nodes,
                              order.data(), &ms))
        die(izpi_gpu_last_error(ctx));
      if (izpi_host_scene_set_bvh(host, nodes.data(), num_nodes, order.data())) die(izpi_host_last_error());
      if (quantized && izpi_host_scene_set_flags(host, IZPI_SCENE_QUANTIZED_BVH)) die(izpi_host_last_error());
    }
    fprintf(stderr, "izpi-render: GPU BVH4 of %u primitives, %u nodes, %.1f ms\n", n, num_nodes, ms);
  }
  if (multi ? izpi_gpu_multi_upload_scene(multi, izpi_host_scene_desc(host)) : izpi_gpu_upload_scene(ctx, izpi_host_scene_desc(host)))
    die(multi ? izpi_gpu_multi_last_error(multi) : izpi_gpu_last_error(ctx));
  const double setup_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  // ---- Render (renderer.go:108-222)
  izpi_render_req req;
  memset(&req, 0, sizeof req);
  req.abi_version = IZPI_ABI_VERSION;
  req.width = W; req.height = H; req.spp = spp; req.max_depth = depth;
  req.sampler = spectral ? IZPI_SAMPLER_SPECTRAL : IZPI_SAMPLER_COLOUR;
  req.out_layout = IZPI_OUT_CANVAS;
  req.seed = seed;
  req.exposure = izpi_host_scene_desc(host)->camera.exposure;
  req.post = (spectral ? IZPI_POST_SPECTRAL : IZPI_POST_NONE) | (png ? IZPI_POST_GAMMA_CLAMP : 0u);
  req.accumulation = acc == "forward" ? IZPI_ACC_FORWARD : IZPI_ACC_RECURSIVE;
  std::vector<double> canvas((size_t)W * H * 4);
  std::vector<izpi_render_stats> stv(gpus > 1 ? gpus : 1);
  auto t1 = std::chrono::steady_clock::now();
  if (multi) {
    if (izpi_gpu_multi_render(multi, &req, canvas.data(), stv.data())) die(izpi_gpu_multi_last_error(multi));
  } else if (izpi_gpu_render(ctx, &req, canvas.data(), stv.data())) {
    die(izpi_gpu_last_error(ctx));
  }
  izpi_render_stats st = stv[0];
  for (size_t i = 1; i < stv.size(); i++) { st.rays += stv[i].rays; st.node_visits += stv[i].node_visits; }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
  printf("{\"scene\": \"%s\", \"width\": %u, \"height\": %u, \"spp\": %u, \"bvh\": \"%s\", \"quantized\": %d, \"accumulation\": \"%s\", \"sampler\": \"%s\", \"gpus\": %u, "
         "\"setup_s\": %.3f, \"render_s\": %.4f, \"msamples_per_s\": %.2f, \"rays\": %llu, \"node_visits\": %llu}\n",
         scene_path.c_str(), W, H, spp, bvh.c_str(), bvh == "gpu" && quantized ? 1 : 0, acc.c_str(), spectral ? "spectral" : "colour", gpus > 1 ? gpus : 1u, setup_s, secs,
         (double)W * H * spp / secs / 1e6, (unsigned long long)st.rays, (unsigned long long)st.node_visits);
  // ---- outputs
  if (!out_raw.empty()) {
    FILE* f = fopen(out_raw.c_str(), "wb");
    if (!f || fwrite(canvas.data(), sizeof(double), canvas.size(), f) != canvas.size()) die("cannot write " + out_raw);
    fclose(f);
  }
  if (!out_pfm.empty()) {  // PFM: "PF", W H, -1 (little endian), rows bottom to top
    FILE* f = fopen(out_pfm.c_str(), "wb");
    if (!f) die("cannot write " + out_pfm);
    fprintf(f, "PF\n%u %u\n-1.0\n", W, H);
    std::vector<float> row(3 * (size_t)W);
    for (uint32_t y = H; y-- > 0;) {
      for (uint32_t x = 0; x < W; x++)
        for (int c = 0; c < 3; c++) row[3 * x + c] = (float)canvas[((size_t)y * W + x) * 4 + c];
      fwrite(row.data(), sizeof(float), row.size(), f);
    }
    fclose(f);
  }
  if (multi) izpi_gpu_multi_close(multi);
  else izpi_gpu_close(ctx);
  izpi_host_scene_free(host);
  izpi_scene_free(ps);
  return 0;
}
