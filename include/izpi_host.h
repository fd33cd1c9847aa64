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
const izpi_scene_desc* izpi_host_scene_desc(const izpi_host_scene* s);
/* Max stack depth the traversal of this BVH can reach (host-computed bound). */
uint32_t izpi_host_scene_stack_bound(const izpi_host_scene* s);
double izpi_host_scene_build_ms(const izpi_host_scene* s);
void izpi_host_scene_free(izpi_host_scene* s);
const char* izpi_host_last_error(void);

/* Tile grid of common.Tiles (common/tiles.go:6-24) + grid.WalkGrid spiral order
 * (grid/grid.go:27-130): writes up to max_tiles entries of x0,y0,x1,y1; returns count. */
uint32_t izpi_host_tiles(uint32_t width, uint32_t height, uint32_t* tiles, uint32_t max_tiles);

/* The Go-math routines of izpi_amd/csrc/gomath.h evaluated on the host (same op
 * codes as izpi_gpu_gomath); used by the parity tests. */
double izpi_host_gomath(int op, double x, double y);

/* sizeof() of the boundary structs: 0 izpi_bvh4_node 1 izpi_texture 2 izpi_material
 * 3 izpi_camera 4 izpi_scene_desc 5 izpi_render_req 6 izpi_render_stats 7 izpi_hit
 * 8 izpi_tri_in 9 izpi_sphere_in 10 izpi_camera_in 11 izpi_scene_input (0 = unknown). */
uint32_t izpi_abi_struct_size(int which);

#ifdef __cplusplus
}
#endif
#endif
