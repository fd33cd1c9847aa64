/* izpi_host.h — host-side scene producer (C++), standing in for the Go host's
 * transport.ToScene (transport/transport.go:53-92, 551-680) + camera.New
 * (camera/camera.go:28-58) + hitable.NewBVH4 (hitable/bvh4.go:517-855).
 *
 * Input is the protobuf-level scene (transport.proto): vertices, UVs, materials,
 * textures, spheres, camera. Output is the flattened izpi_scene_desc consumed by
 * izpi_gpu_upload_scene. In the production Go integration this step stays in Go
 * (the Go side already owns BVH4.Nodes); here it lets the C++/Python harness
 * build the same arrays without a Go toolchain.
 */
#ifndef IZPI_HOST_H
#define IZPI_HOST_H
#include <stdint.h>
#include "izpi_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* transport.proto Triangle: vertices/uv are proto floats widened to float64. */
typedef struct izpi_tri_in {
  double v0[3], v1[3], v2[3];
  double uv[6];          /* u0,v0,u1,v1,u2,v2 */
  uint32_t material;
  uint32_t pad;
} izpi_tri_in;

/* transport.proto Sphere: NewSphere(c, c, 0, 1, r, mat) (transport.go:679) */
typedef struct izpi_sphere_in {
  double center[3];
  double radius;
  uint32_t material;
  uint32_t pad;
} izpi_sphere_in;

/* transport.proto Camera */
typedef struct izpi_camera_in {
  double look_from[3], look_at[3], vup[3];
  double vfov, aspect, aperture, focus_dist, time0, time1, exposure;
} izpi_camera_in;

typedef struct izpi_scene_input {
  uint32_t num_tris, num_spheres, num_materials, num_textures;
  uint32_t num_spd;
  uint32_t pad0;
  uint64_t num_texels;
  const izpi_tri_in* tris;       /* embedded + streamed triangles, transport order */
  const izpi_sphere_in* spheres;
  const izpi_material* materials;
  const izpi_texture* textures;
  const double* texels;
  const double* spd_wavelengths;
  const double* spd_values;
  izpi_camera_in camera;
  double aspect_override;        /* leader: W/H (transport.go aspectOverride), 0 = camera.aspect */
  uint64_t bvh_seed;             /* seed of the BVH split-axis LCG (bvh4.go:520) */
} izpi_scene_input;

typedef struct izpi_host_scene izpi_host_scene;

/* Build; on failure returns non-zero and *out = NULL. */
int izpi_host_build_scene(const izpi_scene_input* in, izpi_host_scene** out);
/* flags: IZPI_HOST_SKIP_BVH leaves the BVH out (num_nodes = 0, primitives in transport
 * order) for another builder, e.g. izpi_gpu_build_bvh4, to attach with
 * izpi_host_scene_set_bvh. */
#define IZPI_HOST_SKIP_BVH 1u
int izpi_host_build_scene_ex(const izpi_scene_input* in, uint32_t flags, izpi_host_scene** out);
/* The f64 primitive boxes the BVH is built over ([num_tris + num_spheres][6]: min xyz,
 * max xyz; triangles first, transport order): Triangle.BoundingBox with its relative
 * epsilon (triangle.go:100-113), Sphere.BoundingBox (sphere.go). */
int izpi_host_scene_prim_boxes(const izpi_host_scene* s, double* boxes);
/* Attach a BVH4 built elsewhere: nodes in BVH4Node format with children after their
 * parents, order[k] = primitive (triangles then spheres) at leaf position k. */
int izpi_host_scene_set_bvh(izpi_host_scene* s, const izpi_bvh4_node* nodes, uint32_t num_nodes, const uint32_t* order);
/* Set the descriptor's IZPI_SCENE_* flags (izpi_scene_desc.flags), e.g. IZPI_SCENE_QUANTIZED_BVH
 * for a GPU-built tree. */
int izpi_host_scene_set_flags(izpi_host_scene* s, uint32_t flags);
const izpi_scene_desc* izpi_host_scene_desc(const izpi_host_scene* s);
/* Max stack depth the traversal of this BVH can reach (host-computed bound). */
uint32_t izpi_host_scene_stack_bound(const izpi_host_scene* s);
double izpi_host_scene_build_ms(const izpi_host_scene* s);
void izpi_host_scene_free(izpi_host_scene* s);
const char* izpi_host_last_error(void);

/* Tile grid of common.Tiles (common/tiles.go:6-24) + grid.WalkGrid spiral order
 * (grid/grid.go:27-130): writes up to max_tiles entries of x0,y0,x1,y1; returns count. */
uint32_t izpi_host_tiles(uint32_t width, uint32_t height, uint32_t* tiles, uint32_t max_tiles);

/* Multi-GPU share of a tile list (the rule izpi_gpu_multi_render / izpi_gpu_render_rank
 * use): copies tiles t with t % num_shares == share, in order, into `out`; returns how
 * many. The largest share has ceil(num_tiles / num_shares) tiles. */
uint32_t izpi_host_share_tiles(const uint32_t* tiles, uint32_t num_tiles, uint32_t share, uint32_t num_shares,
                               uint32_t* out);

/* Primitives per leaf for izpi_gpu_build_bvh4 on this scene: 3, or 2 when spheres are at
 * least a quarter of the primitives (a sphere test costs more than a node visit; C5 at
 * 32 spp: -2.9% per frame with 2). The Python host, the C replay and the Go shim all use it. */
uint32_t izpi_host_bvh_leaf_max(const izpi_scene_desc* desc);

/* Doubles per padded share block of a packed multi-GPU gather: ceil(num_tiles /
 * num_shares) * tile_w * tile_h * 4 (every share's block has this size). */
uint64_t izpi_host_share_block(uint32_t num_tiles, uint32_t tile_w, uint32_t tile_h, uint32_t num_shares);

/* What the root of izpi_gpu_multi_render / izpi_gpu_render_rank does after the gather,
 * on the host: block r of `gathered` (izpi_host_share_block doubles each) holds share r's
 * tiles packed (IZPI_OUT_PACKED); every pixel is scattered to canvas row height - y
 * (render/rgb.go:41; sample row y = 0 has no canvas row). The same index rule as the
 * device's k_unpack. Replaces the framebuffer assembly of renderer.go:172-211 (workers
 * write their tiles into the shared canvas). Tiles must be equal-sized and in bounds. */
int izpi_host_assemble_shares(uint32_t width, uint32_t height, const uint32_t* tiles, uint32_t num_tiles,
                              uint32_t num_shares, const double* gathered, double* canvas);

/* The Go-math routines of izpi_amd/csrc/gomath.h evaluated on the host (same op
 * codes as izpi_gpu_gomath); used by the parity tests. */
double izpi_host_gomath(int op, double x, double y);

/* sizeof() of the boundary structs: 0 izpi_bvh4_node 1 izpi_texture 2 izpi_material
 * 3 izpi_camera 4 izpi_scene_desc 5 izpi_render_req 6 izpi_render_stats 7 izpi_hit
 * 8 izpi_tri_in 9 izpi_sphere_in 10 izpi_camera_in 11 izpi_scene_input 12 izpi_proto_info
 * 13 izpi_obj_info 14 izpi_obj_group 15 izpi_obj_material (0 = unknown). */
uint32_t izpi_abi_struct_size(int which);

/* ======================================================================
 * Scene ingestion — for hosts without Go.
 * In the Go integration these steps stay in Go (prototext/proto + transport).
 * ====================================================================== */

/* transport.Scene, parsed from the text (.pbtxt, prototext.Unmarshal, leader.go:64-71)
 * or binary (.izpi, proto.Unmarshal, leader.go:56-63) encoding of transport.proto.
 * Text format follows prototext: unknown fields, a repeated singular field and two
 * members of one oneof are errors. Binary: unknown fields are skipped. */
typedef struct izpi_proto_scene izpi_proto_scene;

enum { IZPI_COLOUR_RGB = 1, IZPI_COLOUR_SPECTRAL = 2 }; /* transport.proto ColourRepresentation */

typedef struct izpi_proto_info {
  uint32_t colour_representation; /* IZPI_COLOUR_*, 0 = unspecified */
  uint32_t stream_triangles;
  uint64_t total_triangles;
  uint32_t num_triangles;          /* Scene.objects.triangles (embedded) */
  uint32_t num_streamed_triangles; /* added with izpi_scene_add_triangles */
  uint32_t num_spheres, num_materials, num_image_textures, num_displacement_maps;
  uint32_t num_background;         /* spectral_background entries */
  uint32_t pad;
  const char* name;
  const char* version;
  const char* warnings;            /* e.g. unknown light source -> CIE A (transport.go:474-478) */
} izpi_proto_info;

int izpi_scene_parse_text(const char* text, uint64_t len, izpi_proto_scene** out);
int izpi_scene_parse_binary(const void* buf, uint64_t len, izpi_proto_scene** out);
/* The parsed scene as transport.Scene wire bytes, as proto.Marshal writes them (fields in
 * number order, repeated scalars packed, proto3 zero scalars omitted): the .izpi form of
 * a .pbtxt. Writes min(cap, size) bytes to buf (may be NULL with cap 0) and the size to
 * *len. Streamed triangles (izpi_scene_add_triangles) are not part of the message. */
int izpi_scene_serialize(const izpi_proto_scene* s, void* buf, uint64_t cap, uint64_t* len);
int izpi_scene_info(const izpi_proto_scene* s, izpi_proto_info* out);
/* Filenames of Scene.image_textures, which the host decodes (leader.go:84-98)... */
const char* izpi_scene_image_file(const izpi_proto_scene* s, uint32_t i);
/* ...and hands over as float64 NRGBA texels, row 0 = top (texture.ImageTxt). */
int izpi_scene_set_image(izpi_proto_scene* s, const char* filename, uint32_t width, uint32_t height, const double* rgba);
/* Streamed triangles (transport.go:574-583, e.g. from izpi_obj_group_to_triangles);
 * `material` of each izpi_tri_in is ignored, the name is resolved at conversion. */
int izpi_scene_add_triangles(izpi_proto_scene* s, const izpi_tri_in* tris, uint64_t n, const char* material_name);
/* Scene.spectral_background; returns its length, copies up to max entries. */
uint32_t izpi_scene_background(const izpi_proto_scene* s, double* wavelengths, double* values, uint32_t max);
/* transport.ToScene (transport.go:53-92) up to the BVH build: materials (registered by
 * Material.name), textures, light-source library, camera, embedded then streamed
 * triangles, spheres. *out stays valid until the next call or izpi_scene_free; pass
 * it to izpi_host_build_scene. */
int izpi_scene_to_input(izpi_proto_scene* s, double aspect_override, uint64_t bvh_seed, const izpi_scene_input** out);
/* name of material i of the last izpi_scene_to_input */
const char* izpi_scene_material_name(const izpi_proto_scene* s, uint32_t i);
void izpi_scene_free(izpi_proto_scene* s);

/* lightsources.GetLightSource (lightsources.go:472-475): copies the 75 values at the CIE
 * wavelengths (blackbody entries computed as spectral.NewBlackbodySPD); returns 75, or
 * 0 if the name is unknown. izpi_light_source_name(i) enumerates the library. */
uint32_t izpi_light_source(const char* name, double* values);
const char* izpi_light_source_name(uint32_t i);

/* Wavefront OBJ (wavefront.go:107-625). */
typedef struct izpi_obj izpi_obj;
#define IZPI_OBJ_IGNORE_NORMALS 1u   /* ParseOption IGNORE_NORMALS */
#define IZPI_OBJ_IGNORE_MATERIALS 2u /* IGNORE_MATERIALS: mtllib lines are skipped */
#define IZPI_OBJ_IGNORE_TEXTURES 4u  /* IGNORE_TEXTURES */
#define IZPI_OBJ_FACE_POLYGON 1u     /* ObjFaceType OBJ_FACE_TYPE_POLYGON */

typedef struct izpi_obj_info {
  uint32_t has_normals, has_uv, ignore_materials, ignore_normals, ignore_textures;
  uint32_t num_groups, num_materials, pad;
  uint64_t num_vertices, num_normals, num_uvs;
  double centre[3];
  const char* object_name;
} izpi_obj_info;

typedef struct izpi_obj_group {
  const char* name;
  const char* material;
  uint32_t face_type;
  uint32_t is_null;                /* the trailing nil group of a file without faces */
  uint64_t num_faces;
  uint64_t num_face_vertices;
} izpi_obj_group;

typedef struct izpi_obj_material { /* wavefront.Material; Kd/Ka/Ks up to 3 values */
  const char* name;
  double kd[3], ka[3], ks[3];
  uint32_t num_kd, num_ka, num_ks, pad;
  double ns, ni, d;
  int64_t sharpness, illum;
} izpi_obj_material;

/* NewObjFromReader: mtllib files are read from container_dir (wavefront.go:193-204). */
int izpi_obj_parse(const char* text, uint64_t len, const char* container_dir, uint32_t options, izpi_obj** out);
int izpi_obj_info_get(const izpi_obj* o, izpi_obj_info* out);
int izpi_obj_copy_vertices(const izpi_obj* o, double* v, double* vn, double* vt);
int izpi_obj_group_get(const izpi_obj* o, uint32_t g, izpi_obj_group* out);
/* per face its vertex count; per face vertex (VIdx, VtIdx, VnIdx) as in the file (1-based) */
int izpi_obj_copy_faces(const izpi_obj* o, uint32_t g, uint32_t* face_sizes, int64_t* indices);
/* materials in name order */
int izpi_obj_material_get(const izpi_obj* o, uint32_t i, izpi_obj_material* out);
void izpi_obj_translate(izpi_obj* o, double x, double y, double z);
void izpi_obj_scale(izpi_obj* o, double x, double y, double z);
void izpi_obj_rotate(izpi_obj* o, double alpha, double beta, double gamma);
/* GroupToTransportTrianglesWithMaterial (wavefront.go:240-312); out = NULL: count only */
int izpi_obj_group_to_triangles(const izpi_obj* o, uint32_t g, uint32_t without_uvs, izpi_tri_in* out, uint64_t max,
                                uint64_t* n);
void izpi_obj_free(izpi_obj* o);

#ifdef __cplusplus
}
#endif
#endif
