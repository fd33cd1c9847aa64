"""TEST INFRASTRUCTURE — ctypes binding of the CPU oracle (oracle/izpi_oracle.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product (izpi_amd) never does. The oracle is a deterministic CPU
restatement of izpi's hot path (see the header of izpi_oracle.cpp for the
reference file:line list it follows).
"""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liboracle.so"

_lib = None


class OracleStats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_visits", C.c_uint64), ("tri_tests", C.c_uint64),
                ("sph_tests", C.c_uint64), ("light_tri_tests", C.c_uint64), ("light_sph_tests", C.c_uint64),
                ("samples", C.c_uint64), ("seconds", C.c_double), ("threads", C.c_uint32), ("pad", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


def build(force=False):
    """make -C oracle (test infrastructure build)."""
    subprocess.run(["make", "-C", str(HERE)] + (["-B"] if force else []), check=True, stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    build()
    from izpi_amd import _native as N  # struct layouts of the boundary headers only
    L = C.CDLL(str(LIB_PATH))
    L.oracle_build.argtypes = [C.POINTER(N.SceneInput)]
    L.oracle_build.restype = C.c_void_p
    L.oracle_error.argtypes = [C.c_void_p]
    L.oracle_error.restype = C.c_char_p
    L.oracle_free.argtypes = [C.c_void_p]
    L.oracle_num_nodes.argtypes = [C.c_void_p]
    L.oracle_num_nodes.restype = C.c_uint32
    L.oracle_copy_nodes.argtypes = [C.c_void_p, C.c_void_p]
    L.oracle_copy_prim_refs.argtypes = [C.c_void_p, C.c_void_p]
    L.oracle_num_lights.argtypes = [C.c_void_p]
    L.oracle_num_lights.restype = C.c_uint32
    L.oracle_copy_light_refs.argtypes = [C.c_void_p, C.c_void_p]
    L.oracle_copy_triangle.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_double)]
    L.oracle_copy_camera.argtypes = [C.c_void_p, C.POINTER(N.Camera)]
    L.oracle_ray_aabb4.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float)]
    L.oracle_ray_aabb4.restype = C.c_uint8
    L.oracle_conservative_f32.argtypes = [C.c_double, C.c_int]
    L.oracle_conservative_f32.restype = C.c_float
    L.oracle_triangle_hit.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.oracle_gomath.argtypes = [C.c_int, C.c_double, C.c_double]
    L.oracle_gomath.restype = C.c_double
    L.oracle_lcg.argtypes = [C.c_uint64, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
    L.oracle_trace.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_uint32, C.POINTER(N.Hit)]
    L.oracle_render.argtypes = [C.c_void_p, C.POINTER(N.RenderReq), C.POINTER(C.c_double), C.POINTER(OracleStats),
                                C.c_int]
    L.oracle_firefly.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int]
    L.oracle_xyz_to_rgb.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int, C.c_int, C.c_double]
    L.oracle_postprocess.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_double), C.c_int]
    L.oracle_set_bvh.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
    L.oracle_quantize_bvh4.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    L.oracle_quantize_bvh4.restype = C.c_int
    L.oracle_prim_boxes.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    L.oracle_lbvh4.argtypes = [C.POINTER(C.c_double), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                               C.POINTER(C.c_uint32)]
    L.oracle_lbvh4.restype = C.c_uint32
    L.oracle_tiles.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32]
    L.oracle_tiles.restype = C.c_uint32
    L.oracle_sample_wavelength.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.oracle_cie_values.argtypes = [C.c_double, C.POINTER(C.c_double)]
    L.oracle_spectral_value.argtypes = [C.c_int, C.c_double, C.c_double, C.c_double, C.c_double]
    L.oracle_spectral_value.restype = C.c_double
    L.oracle_spd_tabulated_value.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_double]
    L.oracle_spd_tabulated_value.restype = C.c_double
    L.oracle_tbn_mul.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.oracle_path_length.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.oracle_path_length.restype = C.c_double
    _lib = L
    return L


def dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OracleScene:
    """The oracle's own construction of a scene (triangles, BVH4, lights, camera)."""

    def __init__(self, scene, aspect_override=0.0, bvh_seed=12345):
        L = lib()
        self._input = scene.to_input(aspect_override, bvh_seed)
        self.h = L.oracle_build(self._input.ref())
        err = L.oracle_error(self.h)
        if err:
            raise RuntimeError(err.decode())

    def nodes(self):
        L = lib()
        n = L.oracle_num_nodes(self.h)
        buf = np.zeros((n, 128), np.uint8)
        L.oracle_copy_nodes(self.h, buf.ctypes.data)
        return buf

    def prim_refs(self):
        L = lib()
        n = L.oracle_num_nodes(self.h)  # upper bound not needed: count from scene
        out = np.zeros(self._input.struct.num_tris + self._input.struct.num_spheres, np.uint32)
        L.oracle_copy_prim_refs(self.h, out.ctypes.data)
        return out

    def light_refs(self):
        L = lib()
        out = np.zeros(L.oracle_num_lights(self.h), np.uint32)
        if out.size:
            L.oracle_copy_light_refs(self.h, out.ctypes.data)
        return out

    def prim_boxes(self):
        out = np.zeros((self._input.struct.num_tris + self._input.struct.num_spheres, 6))
        lib().oracle_prim_boxes(self.h, dptr(out))
        return out

    def set_bvh(self, nodes, order):
        """Traverse an external tree: nodes (n, 128) uint8 BVH4Node records, order (leaf order)."""
        nodes = np.ascontiguousarray(nodes, np.uint8)
        order = np.ascontiguousarray(order, np.uint32)
        lib().oracle_set_bvh(self.h, nodes.ctypes.data, len(nodes), order.ctypes.data_as(C.POINTER(C.c_uint32)))

    def camera(self):
        from izpi_amd import _native as N
        c = N.Camera()
        lib().oracle_copy_camera(self.h, C.byref(c))
        return c

    def trace(self, rays):
        from izpi_amd import _native as N
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 8)
        out = (N.Hit * len(rays))()
        lib().oracle_trace(self.h, dptr(rays), len(rays), out)
        return out

    def render(self, req, canvas=None, threads=8):
        """Returns (canvas W*H*4 float64, stats dict)."""
        if canvas is None:
            canvas = np.zeros(req.width * req.height * 4, np.float64)
        st = OracleStats()
        lib().oracle_render(self.h, C.byref(req), dptr(canvas), C.byref(st), int(threads))
        return canvas, st.as_dict()

    def close(self):
        if self.h:
            lib().oracle_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def firefly(canvas, width, height):
    c = np.ascontiguousarray(canvas, np.float64).copy()
    lib().oracle_firefly(dptr(c), width, height)
    return c


def xyz_to_rgb(canvas, width, height, exposure):
    src = np.ascontiguousarray(canvas, np.float64)
    out = np.zeros_like(src)
    lib().oracle_xyz_to_rgb(dptr(src), dptr(out), width, height, float(exposure))
    return out


def postprocess(canvas, width, height, filters):
    """filters: [(kind, param)], kind 1 = Gamma, 2 = Clamp."""
    c = np.ascontiguousarray(canvas, np.float64).copy()
    k = np.array([f[0] for f in filters], np.uint32)
    p = np.array([f[1] for f in filters], np.float64)
    lib().oracle_postprocess(dptr(c), width, height, k.ctypes.data_as(C.POINTER(C.c_uint32)), dptr(p), len(filters))
    return c


def lbvh4(boxes, leaf_max=4, method=1):
    """Sequential restatement of the GPU BVH4 builder (method 0 LBVH, 1 PLOC; | 0x100 the
    surface-area-cost collapse):
    (nodes (m, 128) uint8, order)."""
    boxes = np.ascontiguousarray(boxes, np.float64).reshape(-1, 6)
    n = len(boxes)
    nodes = np.zeros((max(1, 2 * n), 128), np.uint8)
    order = np.zeros(max(1, n), np.uint32)
    m = lib().oracle_lbvh4(dptr(boxes), n, leaf_max, method, nodes.ctypes.data,
                           order.ctypes.data_as(C.POINTER(C.c_uint32)))
    return nodes[:m].copy(), order[:n].copy()


def quantize_bvh4(nodes):
    """IZPI_SCENE_QUANTIZED_BVH restated (oracle_quantize_bvh4): the tree with every inner
    node's slot boxes replaced by their decoded 8-bit quantisation and every leaf node's box
    by its parent slot's: (nodes (n, 128) uint8, applied)."""
    nodes = np.ascontiguousarray(nodes, np.uint8).reshape(-1, 128)
    out = np.zeros_like(nodes)
    ok = lib().oracle_quantize_bvh4(nodes.ctypes.data, len(nodes), out.ctypes.data)
    return out, bool(ok)


def tiles(width, height):
    buf = (C.c_uint32 * (4 * width * height))()
    n = lib().oracle_tiles(width, height, buf, width * height)
    return np.frombuffer(buf, np.uint32, count=4 * n).reshape(n, 4).copy()


def gomath(op, x, y=0.0):
    return lib().oracle_gomath(op, x, y)


def lcg(seed, n):
    out = np.zeros(n, np.float64)
    states = np.zeros(n, np.uint64)
    lib().oracle_lcg(seed, n, dptr(out), states.ctypes.data_as(C.POINTER(C.c_uint64)))
    return out, states
