"""ctypes view of the C ABI in include/izpi_gpu.h and include/izpi_host.h.

The structures below mirror the headers field for field; tests/test_abi.py checks
their sizes against the compiled library's expectations. Loading fails loudly when
the native library is missing: there is no Python fallback for the hot path.
"""
import ctypes as C
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LIB_PATH = ROOT / "izpi_amd" / "_lib" / "libizpi_gpu.so"

c_double_p = C.POINTER(C.c_double)
c_uint32_p = C.POINTER(C.c_uint32)
c_float_p = C.POINTER(C.c_float)

# ---- include/izpi_types.h
COMM_ID_BYTES = 128
IZPI_OK, IZPI_ERR_INVALID, IZPI_ERR_HIP, IZPI_ERR_NO_SCENE, IZPI_ERR_UNSUPPORTED, IZPI_ERR_DEVICE, IZPI_ERR_PEER = range(7)
IZPI_ABI_VERSION = 3
ACC_RECURSIVE, ACC_FORWARD = 0, 1
SCENE_QUANTIZED_BVH = 1
PRIM_TRIANGLE, PRIM_SPHERE = 0, 1
TEX_CONSTANT, TEX_IMAGE, TEX_SPECTRAL_GAUSSIAN, TEX_SPECTRAL_TABULATED, TEX_SPECTRAL_IMAGE = 1, 3, 5, 7, 9
MAT_DIELECTRIC, MAT_DIFFUSE_LIGHT, MAT_ISOTROPIC, MAT_LAMBERT, MAT_METAL, MAT_PBR = 1, 2, 3, 4, 5, 6
MATF_BEER_LAMBERT = 1
SAMPLER_COLOUR, SAMPLER_SPECTRAL = 2, 5
OUT_CANVAS, OUT_PACKED = 0, 1
POST_NONE, POST_SPECTRAL, POST_GAMMA_CLAMP = 0, 1, 2
FILTER_GAMMA, FILTER_CLAMP = 1, 2
MAX_FILTERS = 8
HOST_SKIP_BVH = 1
BVH_LBVH, BVH_PLOC = 0, 1
BVH_SAH = 0x100  # flag: collapse by the surface-area cost model (PLOC only)
BVH_PLOC_SAH = BVH_PLOC | BVH_SAH


def prim_ref(kind, idx):
    return (kind << 31) | idx


class BVH4Node(C.Structure):
    _fields_ = [("min_x", C.c_float * 4), ("min_y", C.c_float * 4), ("min_z", C.c_float * 4),
                ("max_x", C.c_float * 4), ("max_y", C.c_float * 4), ("max_z", C.c_float * 4),
                ("child", C.c_int32 * 4), ("prim_count", C.c_int32 * 4)]


class Texture(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("spd_offset", C.c_uint32), ("spd_count", C.c_uint32), ("pad0", C.c_uint32),
                ("texel_offset", C.c_uint64), ("value", C.c_double * 3),
                ("peak", C.c_double), ("center", C.c_double), ("width_nm", C.c_double)]


class Material(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("albedo_tex", C.c_int32), ("spectral_tex", C.c_int32),
                ("normal_tex", C.c_int32), ("roughness_tex", C.c_int32), ("metalness_tex", C.c_int32),
                ("absorb_tex", C.c_int32), ("flags", C.c_uint32), ("ref_idx", C.c_double),
                ("fuzz", C.c_double), ("rgb", C.c_double * 3), ("pad1", C.c_double)]


class Camera(C.Structure):
    _fields_ = [("origin", C.c_double * 3), ("lower_left", C.c_double * 3), ("horizontal", C.c_double * 3),
                ("vertical", C.c_double * 3), ("u", C.c_double * 3), ("v", C.c_double * 3),
                ("lens_radius", C.c_double), ("time0", C.c_double), ("time1", C.c_double), ("exposure", C.c_double)]


# ---- include/izpi_gpu.h
class SceneDesc(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("num_nodes", C.c_uint32), ("num_prims", C.c_uint32),
                ("num_tris", C.c_uint32), ("num_spheres", C.c_uint32), ("num_lights", C.c_uint32),
                ("num_materials", C.c_uint32), ("num_textures", C.c_uint32), ("num_spd", C.c_uint32),
                ("flags", C.c_uint32), ("num_texels", C.c_uint64),
                ("nodes", C.POINTER(BVH4Node)), ("prim_ref", c_uint32_p),
                ("tri_v0", c_double_p), ("tri_v1", c_double_p), ("tri_v2", c_double_p),
                ("tri_e1", c_double_p), ("tri_e2", c_double_p), ("tri_normal", c_double_p),
                ("tri_tangent", c_double_p), ("tri_bitangent", c_double_p), ("tri_uv", c_double_p),
                ("tri_area", c_double_p), ("tri_mat", c_uint32_p),
                ("sph_center0", c_double_p), ("sph_center1", c_double_p), ("sph_time", c_double_p),
                ("sph_radius", c_double_p), ("sph_mat", c_uint32_p),
                ("light_ref", c_uint32_p), ("materials", C.POINTER(Material)), ("textures", C.POINTER(Texture)),
                ("texels", c_double_p), ("spd_wavelengths", c_double_p), ("spd_values", c_double_p),
                ("camera", Camera)]


class RenderTuning(C.Structure):
    _fields_ = [("slots", C.c_uint32), ("chunk_units", C.c_uint32), ("rec_dense", C.c_uint32),
                ("pool_div", C.c_uint32), ("trace_chunk", C.c_uint32), ("refill_min", C.c_uint32),
                ("prim_weight", C.c_uint32), ("flags", C.c_uint32), ("tail_paths", C.c_uint64),
                ("peer_timeout_ms", C.c_uint32), ("pad_tuning", C.c_uint32)]


TUNE_NO_DIST, TUNE_GENERAL_TRACE, TUNE_NO_LEAF_SHORTCUT, TUNE_SCALAR_SLAB, TUNE_NO_TAIL, TUNE_PASS_LOG = 1, 2, 4, 8, 16, 32
TUNE_NO_LDS_BVH = 64
TUNE_NO_RAY_LDS = 128
TUNE_NO_PRIM_LDS = 256
TUNE_NO_QNODES = 1024


def tuning(**kw):
    """izpi_render_tuning from keyword fields; `flags` may also be given as a list of TUNE_* bits."""
    t = RenderTuning()
    for k, v in kw.items():
        if k == "flags" and not isinstance(v, int):
            v = sum(v)
        setattr(t, k, v)
    return t


class RenderReq(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32), ("max_depth", C.c_uint32),
                ("sampler", C.c_uint32), ("out_layout", C.c_uint32), ("num_tiles", C.c_uint32),
                ("num_bg_spd", C.c_uint32), ("tiles", c_uint32_p), ("bg_spd_wavelengths", c_double_p),
                ("bg_spd_values", c_double_p), ("background", C.c_double * 3), ("seed", C.c_uint64),
                ("post", C.c_uint32), ("abi_version", C.c_uint32), ("exposure", C.c_double),
                ("tuning", C.POINTER(RenderTuning)), ("accumulation", C.c_uint32), ("pad_req", C.c_uint32)]


class RenderStats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_visits", C.c_uint64), ("tri_tests", C.c_uint64),
                ("sph_tests", C.c_uint64), ("light_tri_tests", C.c_uint64), ("light_sph_tests", C.c_uint64),
                ("samples", C.c_uint64), ("kernel_ms", C.c_double), ("shade_ms", C.c_double),
                ("total_ms", C.c_double), ("launches", C.c_uint32), ("pad", C.c_uint32),
                ("node_steps", C.c_uint64), ("prim_steps", C.c_uint64), ("leaf_shortcuts", C.c_uint64),
                ("tail_ms", C.c_double), ("tail_node_visits", C.c_uint64), ("tail_tri_tests", C.c_uint64),
                ("tail_sph_tests", C.c_uint64), ("parks", C.c_uint64), ("workspace_bytes", C.c_uint64),
                ("scene_bytes", C.c_uint64), ("slots", C.c_uint32), ("rec_dense", C.c_uint32),
                ("pool_blocks", C.c_uint32), ("chunk_spp", C.c_uint32), ("alloc_ms", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


class Hit(C.Structure):
    _fields_ = [("t", C.c_double), ("u", C.c_double), ("v", C.c_double), ("p", C.c_double * 3),
                ("normal", C.c_double * 3), ("prim_ref", C.c_uint32), ("hit", C.c_uint32)]


# ---- include/izpi_host.h
class TriIn(C.Structure):
    _fields_ = [("v0", C.c_double * 3), ("v1", C.c_double * 3), ("v2", C.c_double * 3),
                ("uv", C.c_double * 6), ("material", C.c_uint32), ("pad", C.c_uint32)]


class SphereIn(C.Structure):
    _fields_ = [("center", C.c_double * 3), ("radius", C.c_double), ("material", C.c_uint32), ("pad", C.c_uint32)]


class CameraIn(C.Structure):
    _fields_ = [("look_from", C.c_double * 3), ("look_at", C.c_double * 3), ("vup", C.c_double * 3),
                ("vfov", C.c_double), ("aspect", C.c_double), ("aperture", C.c_double), ("focus_dist", C.c_double),
                ("time0", C.c_double), ("time1", C.c_double), ("exposure", C.c_double)]


class SceneInput(C.Structure):
    _fields_ = [("num_tris", C.c_uint32), ("num_spheres", C.c_uint32), ("num_materials", C.c_uint32),
                ("num_textures", C.c_uint32), ("num_spd", C.c_uint32), ("pad0", C.c_uint32),
                ("num_texels", C.c_uint64), ("tris", C.c_void_p), ("spheres", C.c_void_p),
                ("materials", C.POINTER(Material)), ("textures", C.POINTER(Texture)), ("texels", c_double_p),
                ("spd_wavelengths", c_double_p), ("spd_values", c_double_p), ("camera", CameraIn),
                ("aspect_override", C.c_double), ("bvh_seed", C.c_uint64)]


COLOUR_RGB, COLOUR_SPECTRAL = 1, 2
OBJ_IGNORE_NORMALS, OBJ_IGNORE_MATERIALS, OBJ_IGNORE_TEXTURES = 1, 2, 4
OBJ_FACE_POLYGON = 1


class ProtoInfo(C.Structure):
    _fields_ = [("colour_representation", C.c_uint32), ("stream_triangles", C.c_uint32),
                ("total_triangles", C.c_uint64), ("num_triangles", C.c_uint32), ("num_streamed_triangles", C.c_uint32),
                ("num_spheres", C.c_uint32), ("num_materials", C.c_uint32), ("num_image_textures", C.c_uint32),
                ("num_displacement_maps", C.c_uint32), ("num_background", C.c_uint32), ("pad", C.c_uint32),
                ("name", C.c_char_p), ("version", C.c_char_p), ("warnings", C.c_char_p)]


class ObjInfo(C.Structure):
    _fields_ = [("has_normals", C.c_uint32), ("has_uv", C.c_uint32), ("ignore_materials", C.c_uint32),
                ("ignore_normals", C.c_uint32), ("ignore_textures", C.c_uint32), ("num_groups", C.c_uint32),
                ("num_materials", C.c_uint32), ("pad", C.c_uint32), ("num_vertices", C.c_uint64),
                ("num_normals", C.c_uint64), ("num_uvs", C.c_uint64), ("centre", C.c_double * 3),
                ("object_name", C.c_char_p)]


class ObjGroup(C.Structure):
    _fields_ = [("name", C.c_char_p), ("material", C.c_char_p), ("face_type", C.c_uint32), ("is_null", C.c_uint32),
                ("num_faces", C.c_uint64), ("num_face_vertices", C.c_uint64)]


class ObjMaterial(C.Structure):
    _fields_ = [("name", C.c_char_p), ("kd", C.c_double * 3), ("ka", C.c_double * 3), ("ks", C.c_double * 3),
                ("num_kd", C.c_uint32), ("num_ka", C.c_uint32), ("num_ks", C.c_uint32), ("pad", C.c_uint32),
                ("ns", C.c_double), ("ni", C.c_double), ("d", C.c_double), ("sharpness", C.c_int64),
                ("illum", C.c_int64)]


ABI_STRUCTS = [BVH4Node, Texture, Material, Camera, SceneDesc, RenderReq, RenderStats, Hit, TriIn, SphereIn, CameraIn,
               SceneInput, ProtoInfo, ObjInfo, ObjGroup, ObjMaterial, RenderTuning]

# Symbols include/izpi_gpu.h and include/izpi_host.h declare (checked by tests).
EXPORTS = [
    "izpi_gpu_open", "izpi_gpu_close", "izpi_gpu_prepare", "izpi_gpu_multi_prepare", "izpi_gpu_last_error", "izpi_gpu_upload_scene", "izpi_gpu_render",
    "izpi_gpu_render_device", "izpi_gpu_unpack_tiles", "izpi_gpu_output_bytes", "izpi_gpu_trace",
    "izpi_gpu_ray_aabb4", "izpi_gpu_gomath", "izpi_gpu_spectral_post", "izpi_gpu_postprocess",
    "izpi_gpu_build_bvh4", "izpi_gpu_multi_open", "izpi_gpu_multi_close", "izpi_gpu_multi_last_error",
    "izpi_gpu_multi_size", "izpi_gpu_multi_context", "izpi_gpu_multi_upload_scene", "izpi_gpu_multi_render",
    "izpi_gpu_comm_id", "izpi_gpu_comm_init", "izpi_gpu_render_rank", "izpi_gpu_debug_fault", "izpi_gpu_debug_realloc", "izpi_gpu_progress", "izpi_gpu_multi_progress", "izpi_host_build_scene_ex", "izpi_host_scene_prim_boxes", "izpi_host_scene_set_bvh", "izpi_host_scene_set_flags",
    "izpi_host_build_scene", "izpi_host_scene_desc", "izpi_host_scene_stack_bound", "izpi_host_scene_build_ms",
    "izpi_host_scene_free", "izpi_host_last_error", "izpi_host_tiles", "izpi_host_share_tiles", "izpi_host_share_block", "izpi_host_assemble_shares", "izpi_host_bvh_leaf_max", "izpi_host_gomath", "izpi_abi_struct_size",
    "izpi_scene_parse_text", "izpi_scene_parse_binary", "izpi_scene_serialize", "izpi_scene_info", "izpi_scene_image_file",
    "izpi_scene_set_image", "izpi_scene_add_triangles", "izpi_scene_background", "izpi_scene_to_input",
    "izpi_scene_material_name", "izpi_scene_free", "izpi_light_source", "izpi_light_source_name",
    "izpi_obj_parse", "izpi_obj_info_get", "izpi_obj_copy_vertices", "izpi_obj_group_get", "izpi_obj_copy_faces",
    "izpi_obj_material_get", "izpi_obj_translate", "izpi_obj_scale", "izpi_obj_rotate",
    "izpi_obj_group_to_triangles", "izpi_obj_free",
]

_lib = None


def lib():
    """Load libizpi_gpu.so (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError("izpi native library missing: %s (run `python -m izpi_amd.build`)" % LIB_PATH)
    try:  # bind to the HIP runtime torch already ships (same SONAME), not a second copy
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(str(LIB_PATH))
    L.izpi_gpu_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.izpi_gpu_close.argtypes = [C.c_void_p]
    L.izpi_gpu_last_error.argtypes = [C.c_void_p]
    L.izpi_gpu_last_error.restype = C.c_char_p
    L.izpi_gpu_upload_scene.argtypes = [C.c_void_p, C.POINTER(SceneDesc)]
    L.izpi_gpu_render.argtypes = [C.c_void_p, C.POINTER(RenderReq), c_double_p, C.POINTER(RenderStats)]
    L.izpi_gpu_prepare.argtypes = [C.c_void_p, C.POINTER(RenderReq)]
    L.izpi_gpu_multi_prepare.argtypes = [C.c_void_p, C.POINTER(RenderReq)]
    L.izpi_gpu_render_device.argtypes = [C.c_void_p, C.POINTER(RenderReq), C.c_void_p, C.POINTER(RenderStats)]
    L.izpi_gpu_unpack_tiles.argtypes = [C.c_void_p, C.POINTER(RenderReq), C.c_void_p, C.c_void_p]
    L.izpi_gpu_output_bytes.argtypes = [C.POINTER(RenderReq)]
    L.izpi_gpu_output_bytes.restype = C.c_uint64
    L.izpi_gpu_trace.argtypes = [C.c_void_p, c_double_p, C.c_uint32, C.POINTER(Hit)]
    L.izpi_gpu_ray_aabb4.argtypes = [C.c_void_p, c_float_p, c_float_p, C.c_uint32, C.POINTER(C.c_uint8)]
    L.izpi_gpu_gomath.argtypes = [C.c_void_p, C.c_int, c_double_p, c_double_p, C.c_uint32, c_double_p]
    L.izpi_gpu_spectral_post.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_double]
    L.izpi_gpu_postprocess.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, c_uint32_p, c_double_p,
                                       C.c_uint32]
    L.izpi_gpu_build_bvh4.argtypes = [C.c_void_p, c_double_p, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(BVH4Node),
                                      C.c_uint32, c_uint32_p, c_uint32_p, c_double_p]
    L.izpi_gpu_multi_open.argtypes = [C.POINTER(C.c_int), C.c_uint32, C.POINTER(C.c_void_p)]
    L.izpi_gpu_multi_close.argtypes = [C.c_void_p]
    L.izpi_gpu_multi_last_error.argtypes = [C.c_void_p]
    L.izpi_gpu_multi_last_error.restype = C.c_char_p
    L.izpi_gpu_multi_size.argtypes = [C.c_void_p]
    L.izpi_gpu_multi_size.restype = C.c_uint32
    L.izpi_gpu_multi_context.argtypes = [C.c_void_p, C.c_uint32]
    L.izpi_gpu_multi_context.restype = C.c_void_p
    L.izpi_gpu_multi_upload_scene.argtypes = [C.c_void_p, C.POINTER(SceneDesc)]
    L.izpi_gpu_multi_render.argtypes = [C.c_void_p, C.POINTER(RenderReq), C.c_void_p, C.POINTER(RenderStats)]
    L.izpi_gpu_comm_id.argtypes = [C.POINTER(C.c_uint8)]
    L.izpi_gpu_comm_init.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8)]
    L.izpi_gpu_render_rank.argtypes = [C.c_void_p, C.POINTER(RenderReq), C.c_void_p, C.POINTER(RenderStats)]
    L.izpi_gpu_debug_fault.argtypes = [C.c_void_p, C.c_int]
    L.izpi_gpu_debug_realloc.argtypes = [C.c_void_p, C.c_uint32]
    L.izpi_gpu_progress.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.izpi_gpu_multi_progress.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.izpi_host_build_scene_ex.argtypes = [C.POINTER(SceneInput), C.c_uint32, C.POINTER(C.c_void_p)]
    L.izpi_host_scene_prim_boxes.argtypes = [C.c_void_p, c_double_p]
    L.izpi_host_scene_set_bvh.argtypes = [C.c_void_p, C.POINTER(BVH4Node), C.c_uint32, c_uint32_p]
    L.izpi_host_scene_set_flags.argtypes = [C.c_void_p, C.c_uint32]
    L.izpi_host_build_scene.argtypes = [C.POINTER(SceneInput), C.POINTER(C.c_void_p)]
    L.izpi_host_scene_desc.argtypes = [C.c_void_p]
    L.izpi_host_scene_desc.restype = C.POINTER(SceneDesc)
    L.izpi_host_scene_stack_bound.argtypes = [C.c_void_p]
    L.izpi_host_scene_stack_bound.restype = C.c_uint32
    L.izpi_host_scene_build_ms.argtypes = [C.c_void_p]
    L.izpi_host_scene_build_ms.restype = C.c_double
    L.izpi_host_scene_free.argtypes = [C.c_void_p]
    L.izpi_host_last_error.restype = C.c_char_p
    L.izpi_host_tiles.argtypes = [C.c_uint32, C.c_uint32, c_uint32_p, C.c_uint32]
    L.izpi_host_tiles.restype = C.c_uint32
    L.izpi_host_share_tiles.argtypes = [c_uint32_p, C.c_uint32, C.c_uint32, C.c_uint32, c_uint32_p]
    L.izpi_host_share_tiles.restype = C.c_uint32
    L.izpi_host_bvh_leaf_max.argtypes = [C.POINTER(SceneDesc)]
    L.izpi_host_bvh_leaf_max.restype = C.c_uint32
    L.izpi_host_share_block.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    L.izpi_host_share_block.restype = C.c_uint64
    L.izpi_host_assemble_shares.argtypes = [C.c_uint32, C.c_uint32, c_uint32_p, C.c_uint32, C.c_uint32, c_double_p,
                                            c_double_p]
    L.izpi_host_gomath.argtypes = [C.c_int, C.c_double, C.c_double]
    L.izpi_host_gomath.restype = C.c_double
    L.izpi_abi_struct_size.argtypes = [C.c_int]
    L.izpi_abi_struct_size.restype = C.c_uint32
    # scene ingestion (izpi_host.h)
    vp, vpp = C.c_void_p, C.POINTER(C.c_void_p)
    L.izpi_scene_parse_text.argtypes = [C.c_char_p, C.c_uint64, vpp]
    L.izpi_scene_parse_binary.argtypes = [C.c_char_p, C.c_uint64, vpp]
    L.izpi_scene_info.argtypes = [vp, C.POINTER(ProtoInfo)]
    L.izpi_scene_serialize.argtypes = [vp, vp, C.c_uint64, C.POINTER(C.c_uint64)]
    L.izpi_scene_image_file.argtypes = [vp, C.c_uint32]
    L.izpi_scene_image_file.restype = C.c_char_p
    L.izpi_scene_set_image.argtypes = [vp, C.c_char_p, C.c_uint32, C.c_uint32, c_double_p]
    L.izpi_scene_add_triangles.argtypes = [vp, vp, C.c_uint64, C.c_char_p]
    L.izpi_scene_background.argtypes = [vp, c_double_p, c_double_p, C.c_uint32]
    L.izpi_scene_background.restype = C.c_uint32
    L.izpi_scene_to_input.argtypes = [vp, C.c_double, C.c_uint64, C.POINTER(C.POINTER(SceneInput))]
    L.izpi_scene_material_name.argtypes = [vp, C.c_uint32]
    L.izpi_scene_material_name.restype = C.c_char_p
    L.izpi_scene_free.argtypes = [vp]
    L.izpi_scene_free.restype = None
    L.izpi_light_source.argtypes = [C.c_char_p, c_double_p]
    L.izpi_light_source.restype = C.c_uint32
    L.izpi_light_source_name.argtypes = [C.c_uint32]
    L.izpi_light_source_name.restype = C.c_char_p
    L.izpi_obj_parse.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint32, vpp]
    L.izpi_obj_info_get.argtypes = [vp, C.POINTER(ObjInfo)]
    L.izpi_obj_copy_vertices.argtypes = [vp, c_double_p, c_double_p, c_double_p]
    L.izpi_obj_group_get.argtypes = [vp, C.c_uint32, C.POINTER(ObjGroup)]
    L.izpi_obj_copy_faces.argtypes = [vp, C.c_uint32, c_uint32_p, C.POINTER(C.c_int64)]
    L.izpi_obj_material_get.argtypes = [vp, C.c_uint32, C.POINTER(ObjMaterial)]
    for f in ("izpi_obj_translate", "izpi_obj_scale", "izpi_obj_rotate"):
        getattr(L, f).argtypes = [vp, C.c_double, C.c_double, C.c_double]
        getattr(L, f).restype = None
    L.izpi_obj_group_to_triangles.argtypes = [vp, C.c_uint32, C.c_uint32, vp, C.c_uint64, C.POINTER(C.c_uint64)]
    L.izpi_obj_free.argtypes = [vp]
    L.izpi_obj_free.restype = None
    _lib = L
    return L
