/* izpi_types.h — plain-C data types crossing the izpi GPU boundary.
 *
 * Everything here is POD with fixed-width fields and no pointers to host objects,
 * so a Go caller can pass its own slices through cgo (a Go []BVH4Node is
 * byte-identical to izpi_bvh4_node[]).
 *
 * Enum values follow the reference's own numbering:
 *   material kinds  = transport.proto MaterialType (DIELECTRIC=1 … PBR=6)
 *   texture kinds   = transport.proto TextureType, with the SpectralConstant oneof
 *                     split into GAUSSIAN/TABULATED (texture/spectral_constant.go:65-106)
 *   sampler kinds   = sampler.go:13-20 (ColourSampler=2, SpectralSampler=5)
 */
#ifndef IZPI_TYPES_H
#define IZPI_TYPES_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IZPI_ABI_VERSION 3u

/* ---- status codes (0 = OK) ------------------------------------------------ */
enum {
  IZPI_OK = 0,
  IZPI_ERR_INVALID = 1,     /* bad argument / malformed scene */
  IZPI_ERR_HIP = 2,         /* HIP runtime failure */
  IZPI_ERR_NO_SCENE = 3,    /* render before upload */
  IZPI_ERR_UNSUPPORTED = 4, /* feature outside this build (e.g. Payne-Hanek trig) */
  IZPI_ERR_DEVICE = 5,      /* device-side guard tripped (stack overflow, …) */
  IZPI_ERR_PEER = 6         /* multi-GPU: this device/rank succeeded but another one failed */
};

/* ---- BVH4 node: byte-identical to hitable.BVH4Node (bvh4.go:23-39), 128 B ---- */
typedef struct izpi_bvh4_node {
  float min_x[4], min_y[4], min_z[4];
  float max_x[4], max_y[4], max_z[4];
  int32_t child[4];      /* ChildIndex: node index (inner) or primitive start (leaf), -1 = empty */
  int32_t prim_count[4]; /* PrimitiveCount: >0 leaf, 0 inner */
} izpi_bvh4_node;

/* primitive / light reference: kind in bit 31, index below (transport order) */
#define IZPI_PRIM_TRIANGLE 0u
#define IZPI_PRIM_SPHERE 1u
#define IZPI_PRIM_REF(kind, idx) (((uint32_t)(kind) << 31) | (uint32_t)(idx))
#define IZPI_PRIM_KIND(ref) ((uint32_t)(ref) >> 31)
#define IZPI_PRIM_INDEX(ref) ((uint32_t)(ref) & 0x7FFFFFFFu)

/* ---- textures (texture package) ---------------------------------------------- */
enum {
  IZPI_TEX_CONSTANT = 1,           /* texture.Constant (constant.go:20) */
  IZPI_TEX_IMAGE = 3,              /* texture.ImageTxt, float64 NRGBA (image.go:73-101) */
  IZPI_TEX_SPECTRAL_GAUSSIAN = 5,  /* SpectralConstant, Gaussian (spectral_constant.go:72) */
  IZPI_TEX_SPECTRAL_TABULATED = 7, /* SpectralConstant from SPD (spectral_constant.go:77-106) */
  IZPI_TEX_SPECTRAL_IMAGE = 9      /* texture.SpectralImage of an IMAGE texture's texels (spectral_image.go:64-259;
                                      transport.go:486-497): width/height/texel_offset as IMAGE */
};

typedef struct izpi_texture {
  uint32_t kind;
  uint32_t width, height;   /* IMAGE: texel grid, row-major, row 0 = image top */
  uint32_t spd_offset;      /* TABULATED: first entry in spd_wavelengths/spd_values */
  uint32_t spd_count;       /* TABULATED: number of entries */
  uint32_t pad0;
  uint64_t texel_offset;    /* IMAGE: offset in doubles into texels[] (4 per texel: R,G,B,A) */
  double value[3];          /* CONSTANT: rgb */
  double peak, center, width_nm; /* GAUSSIAN: peakValue, centerWavelength, width */
} izpi_texture;

/* ---- materials (material package) -------------------------------------------- */
enum {
  IZPI_MAT_DIELECTRIC = 1,    /* dielectric.go */
  IZPI_MAT_DIFFUSE_LIGHT = 2, /* diffuselight.go */
  IZPI_MAT_ISOTROPIC = 3,     /* isotropic.go (RGB albedo; transport.go:269-289) */
  IZPI_MAT_LAMBERT = 4,       /* lambertian.go */
  IZPI_MAT_METAL = 5,         /* metal.go */
  IZPI_MAT_PBR = 6            /* pbr.go */
};

#define IZPI_MATF_BEER_LAMBERT 1u /* Dielectric.computeBeerLambertAttenuation */

typedef struct izpi_material {
  uint32_t kind;
  int32_t albedo_tex;     /* LAMBERT/PBR/ISOTROPIC albedo, DIFFUSE_LIGHT emit (RGB texture), -1 none */
  int32_t spectral_tex;   /* LAMBERT spectral albedo, DIFFUSE_LIGHT spectral emit,
                             DIELECTRIC spectral refractive index, PBR spectral albedo
                             (LAMBERT / DIFFUSE_LIGHT / PBR may use a SPECTRAL_IMAGE) */
  int32_t normal_tex;     /* PBR normal map (also read by Triangle.Hit, triangle.go:250) */
  int32_t roughness_tex;  /* PBR */
  int32_t metalness_tex;  /* PBR */
  int32_t absorb_tex;     /* DIELECTRIC spectral absorption coefficient */
  uint32_t flags;         /* IZPI_MATF_* */
  double ref_idx;         /* DIELECTRIC scalar refractive index */
  double fuzz;            /* METAL */
  double rgb[3];          /* METAL albedo; DIELECTRIC RGB absorption coefficient */
  double pad1;
} izpi_material;

/* ---- camera as computed by camera.New (camera.go:13-58) ------------------- */
typedef struct izpi_camera {
  double origin[3], lower_left[3], horizontal[3], vertical[3], u[3], v[3];
  double lens_radius, time0, time1, exposure;
} izpi_camera;

#ifdef __cplusplus
}
#endif
#endif
