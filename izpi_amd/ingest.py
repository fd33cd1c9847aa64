"""Scene ingestion: transport.Scene files and Wavefront OBJ meshes,
parsed by the C++ code in izpi_amd/csrc/scene_io.cpp (include/izpi_host.h).

``ProtoScene`` mirrors what izpi's leader does before ``render.New`` (leader.go:43-112):
read a ``.pbtxt`` (prototext) or ``.izpi`` (binary protobuf) scene, hand over the image
textures it names, optionally add streamed triangles, then ``transport.ToScene``. It
plugs into :class:`izpi_amd.scene.HostScene` / :class:`izpi_amd.renderer.GPURenderer`
exactly like the programmatic :class:`izpi_amd.scene.Scene`.

``WavefrontObj`` mirrors ``wavefront.WavefrontObj`` (wavefront.go:56-105): parse,
Scale/Rotate/Translate, GroupToTransportTrianglesWithMaterial.
"""
import ctypes as C
import os
from fractions import Fraction
from pathlib import Path

import numpy as np

from . import _native as N
from .scene import TRI_DTYPE

# math.Pi (Go's untyped constant, math/const.go)
_GO_PI = Fraction("3.14159265358979323846264338327950288419716939937510582097494459")


def go_radians(degrees):
    """``degrees * math.Pi / 180.0`` as a Go constant expression: exact, rounded once
    (e.g. scenes/spectral.go:645 passes -(60.0 * math.Pi / 180.0))."""
    return float(Fraction(degrees) * _GO_PI / 180)


def _err(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed (status %d): %s" % (what, rc, N.lib().izpi_host_last_error().decode()))


class _ProtoInput:
    """izpi_scene_input owned by the C++ scene (valid until the next conversion)."""

    def __init__(self, ptr, owner):
        self.struct = ptr.contents
        self._owner = owner

    def ref(self):
        return C.byref(self.struct)


class ProtoScene:
    def __init__(self, data, binary=False):
        L = N.lib()
        h = C.c_void_p()
        buf = bytes(data)
        fn = L.izpi_scene_parse_binary if binary else L.izpi_scene_parse_text
        _err(fn(buf, len(buf), C.byref(h)), "izpi_scene_parse_binary" if binary else "izpi_scene_parse_text")
        self.handle = h
        self._keep = []

    @classmethod
    def from_file(cls, path):
        """leader.go:54-75: the extension picks the decoder."""
        path = Path(path)
        ext = path.suffix
        if ext == ".pbtxt":
            return cls(path.read_bytes(), binary=False)
        if ext == ".izpi":
            return cls(path.read_bytes(), binary=True)
        raise ValueError("Unknown scene file extension: %s" % ext)

    def to_wire(self):
        """transport.Scene wire bytes (proto.Marshal's form, the .izpi file format)."""
        n = C.c_uint64()
        _err(N.lib().izpi_scene_serialize(self.handle, None, 0, C.byref(n)), "izpi_scene_serialize")
        buf = C.create_string_buffer(max(1, n.value))
        _err(N.lib().izpi_scene_serialize(self.handle, buf, n.value, C.byref(n)), "izpi_scene_serialize")
        return buf.raw[:n.value]

    def info(self):
        i = N.ProtoInfo()
        _err(N.lib().izpi_scene_info(self.handle, C.byref(i)), "izpi_scene_info")
        d = {k: getattr(i, k) for k, _ in i._fields_ if k != "pad"}
        for k in ("name", "version", "warnings"):
            d[k] = (d[k] or b"").decode()
        return d

    @property
    def sampler(self):
        """leader.go:77-81: a SPECTRAL scene renders with the spectral sampler."""
        return N.SAMPLER_SPECTRAL if self.info()["colour_representation"] == N.COLOUR_SPECTRAL else N.SAMPLER_COLOUR

    def image_files(self):
        L = N.lib()
        return [L.izpi_scene_image_file(self.handle, i).decode() for i in range(self.info()["num_image_textures"])]

    def set_image(self, filename, rgba):
        a = np.ascontiguousarray(rgba, np.float64)
        assert a.ndim == 3 and a.shape[2] == 4
        _err(N.lib().izpi_scene_set_image(self.handle, filename.encode(), a.shape[1], a.shape[0],
                                          a.ctypes.data_as(N.c_double_p)), "izpi_scene_set_image")

    def add_triangles(self, tris, material_name):
        t = np.ascontiguousarray(tris, TRI_DTYPE)
        _err(N.lib().izpi_scene_add_triangles(self.handle, t.ctypes.data if t.size else None, len(t),
                                              material_name.encode()), "izpi_scene_add_triangles")

    def spectral_background(self):
        L = N.lib()
        n = L.izpi_scene_background(self.handle, None, None, 0)
        wl, val = np.zeros(n), np.zeros(n)
        if n:
            L.izpi_scene_background(self.handle, wl.ctypes.data_as(N.c_double_p), val.ctypes.data_as(N.c_double_p), n)
        return wl, val

    def to_input(self, aspect_override=0.0, bvh_seed=12345):
        p = C.POINTER(N.SceneInput)()
        _err(N.lib().izpi_scene_to_input(self.handle, float(aspect_override), int(bvh_seed), C.byref(p)),
             "izpi_scene_to_input")
        return _ProtoInput(p, self)

    def material_names(self):
        L = N.lib()
        out = []
        while True:
            n = L.izpi_scene_material_name(self.handle, len(out))
            if n is None:
                return out
            out.append(n.decode())

    def close(self):
        if getattr(self, "handle", None):
            N.lib().izpi_scene_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def light_source(name):
    """lightsources.GetLightSource: the 75 values at the CIE wavelengths, or None."""
    v = np.zeros(75)
    n = N.lib().izpi_light_source(name.encode(), v.ctypes.data_as(N.c_double_p))
    return v if n else None


def light_source_names():
    L = N.lib()
    out = []
    while True:
        n = L.izpi_light_source_name(len(out))
        if n is None:
            return out
        out.append(n.decode())


class WavefrontObj:
    def __init__(self, text, container_dir=".", options=0):
        L = N.lib()
        h = C.c_void_p()
        buf = text.encode() if isinstance(text, str) else bytes(text)
        _err(L.izpi_obj_parse(buf, len(buf), str(container_dir).encode(), int(options), C.byref(h)), "izpi_obj_parse")
        self.handle = h

    @classmethod
    def from_file(cls, path, options=0):
        """NewObjFromReader(file, filepath.Dir(path)) (scenes/spectral.go:639)."""
        return cls(Path(path).read_bytes(), os.path.dirname(str(path)) or ".", options)

    def info(self):
        i = N.ObjInfo()
        _err(N.lib().izpi_obj_info_get(self.handle, C.byref(i)), "izpi_obj_info_get")
        d = {k: getattr(i, k) for k, _ in i._fields_ if k != "pad"}
        d["centre"] = tuple(i.centre)
        d["object_name"] = (i.object_name or b"").decode()
        return d

    def vertices(self):
        i = self.info()
        v, vn, vt = np.zeros((i["num_vertices"], 3)), np.zeros((i["num_normals"], 3)), np.zeros((i["num_uvs"], 2))
        N.lib().izpi_obj_copy_vertices(self.handle, v.ctypes.data_as(N.c_double_p), vn.ctypes.data_as(N.c_double_p),
                                       vt.ctypes.data_as(N.c_double_p))
        return v, vn, vt

    def groups(self):
        L = N.lib()
        out = []
        for g in range(self.info()["num_groups"]):
            gi = N.ObjGroup()
            _err(L.izpi_obj_group_get(self.handle, g, C.byref(gi)), "izpi_obj_group_get")
            sizes = np.zeros(gi.num_faces, np.uint32)
            idx = np.zeros((gi.num_face_vertices, 3), np.int64)
            L.izpi_obj_copy_faces(self.handle, g, sizes.ctypes.data_as(N.c_uint32_p),
                                  idx.ctypes.data_as(C.POINTER(C.c_int64)))
            faces, k = [], 0
            for s in sizes:
                faces.append([tuple(int(x) for x in idx[k + j]) for j in range(int(s))])
                k += int(s)
            out.append(None if gi.is_null else {"name": gi.name.decode(), "material": gi.material.decode(),
                                                "face_type": gi.face_type, "faces": faces})
        return out

    def materials(self):
        L = N.lib()
        out = {}
        for i in range(self.info()["num_materials"]):
            m = N.ObjMaterial()
            _err(L.izpi_obj_material_get(self.handle, i, C.byref(m)), "izpi_obj_material_get")
            out[m.name.decode()] = {"Kd": list(m.kd[:m.num_kd]), "Ka": list(m.ka[:m.num_ka]), "Ks": list(m.ks[:m.num_ks]),
                                    "Ns": m.ns, "Ni": m.ni, "D": m.d, "Sharpness": m.sharpness, "Illum": m.illum}
        return out

    def translate(self, x, y, z):
        N.lib().izpi_obj_translate(self.handle, x, y, z)

    def scale(self, x, y, z):
        N.lib().izpi_obj_scale(self.handle, x, y, z)

    def rotate(self, alpha, beta, gamma):
        N.lib().izpi_obj_rotate(self.handle, alpha, beta, gamma)

    def group_to_transport_triangles(self, group, without_uvs=False):
        L = N.lib()
        n = C.c_uint64()
        _err(L.izpi_obj_group_to_triangles(self.handle, group, int(without_uvs), None, 0, C.byref(n)),
             "izpi_obj_group_to_triangles")
        t = np.zeros(n.value, TRI_DTYPE)
        _err(L.izpi_obj_group_to_triangles(self.handle, group, int(without_uvs), t.ctypes.data if t.size else None,
                                           n.value, C.byref(n)), "izpi_obj_group_to_triangles")
        return t

    def close(self):
        if getattr(self, "handle", None):
            N.lib().izpi_obj_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
