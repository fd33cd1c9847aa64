"""Protobuf-level scene description (internal/proto/transport/transport.proto) for
the izpi GPU path.

A :class:`Scene` holds exactly what a ``transport.Scene`` message carries —
triangles, spheres, materials, textures, camera — and turns it into the
``izpi_scene_input`` struct of include/izpi_host.h. Every scalar that the proto
declares as ``float`` is rounded to float32 first (``f32``), as
``float64(proto.GetX())`` does in transport.go:606-627.
"""
import ctypes as C

import numpy as np

from . import _native as N

TRI_DTYPE = np.dtype([("v0", "<f8", 3), ("v1", "<f8", 3), ("v2", "<f8", 3), ("uv", "<f8", 6),
                      ("material", "<u4"), ("pad", "<u4")], align=True)
SPHERE_DTYPE = np.dtype([("center", "<f8", 3), ("radius", "<f8"), ("material", "<u4"), ("pad", "<u4")], align=True)
assert TRI_DTYPE.itemsize == C.sizeof(N.TriIn)
assert SPHERE_DTYPE.itemsize == C.sizeof(N.SphereIn)

# texture.NewSpectralNeutral's wavelength grid (spectral_constant.go:85)
NEUTRAL_WAVELENGTHS = [float(w) for w in range(380, 751, 10)]


def f32(x):
    """Round like a proto float field widened to float64."""
    return np.asarray(x, dtype=np.float32).astype(np.float64)


def _ptr(arr, ctype):
    return arr.ctypes.data_as(C.POINTER(ctype)) if arr is not None and arr.size else None


class Scene:
    def __init__(self, name="scene"):
        self.name = name
        self.textures = []
        self.materials = []
        self.texels = []            # list of float64 arrays (H, W, 4)
        self._texel_len = 0
        self.spd_wl = []
        self.spd_val = []
        self.tris = np.zeros(0, TRI_DTYPE)
        self.spheres = np.zeros(0, SPHERE_DTYPE)
        self.camera = None

    # ------------------------------------------------------------- textures
    def constant(self, rgb):
        t = N.Texture(kind=N.TEX_CONSTANT)
        t.value[:] = [float(v) for v in f32(rgb)]
        self.textures.append(t)
        return len(self.textures) - 1

    def image(self, rgba):
        """float64 NRGBA texture, rgba shape (H, W, 4), row 0 = top (image.go:73-101)."""
        a = np.ascontiguousarray(rgba, dtype=np.float64)
        assert a.ndim == 3 and a.shape[2] == 4
        t = N.Texture(kind=N.TEX_IMAGE, width=a.shape[1], height=a.shape[0], texel_offset=self._texel_len)
        self.texels.append(a.reshape(-1))
        self._texel_len += a.size
        self.textures.append(t)
        return len(self.textures) - 1

    def spectral_image(self, image_tex):
        """texture.SpectralImage of an image texture (NewSpectralImageFromImage,
        spectral_image.go:64-190): what transport.textureToSpectralTexture makes of a PBR
        image albedo for the Spectral sampler (transport.go:486-497). Shares its texels."""
        src = self.textures[image_tex]
        assert src.kind == N.TEX_IMAGE
        t = N.Texture(kind=N.TEX_SPECTRAL_IMAGE, width=src.width, height=src.height, texel_offset=src.texel_offset)
        self.textures.append(t)
        return len(self.textures) - 1

    def spectral_gaussian(self, peak, center, width):
        t = N.Texture(kind=N.TEX_SPECTRAL_GAUSSIAN, peak=float(f32(peak)), center=float(f32(center)),
                      width_nm=float(f32(width)))
        self.textures.append(t)
        return len(self.textures) - 1

    def spectral_tabulated(self, wavelengths, values, proto_float=True):
        wl = [float(v) for v in (f32(wavelengths) if proto_float else np.asarray(wavelengths, np.float64))]
        vl = [float(v) for v in (f32(values) if proto_float else np.asarray(values, np.float64))]
        assert len(wl) == len(vl)
        t = N.Texture(kind=N.TEX_SPECTRAL_TABULATED, spd_offset=len(self.spd_wl), spd_count=len(wl))
        self.spd_wl.extend(wl)
        self.spd_val.extend(vl)
        self.textures.append(t)
        return len(self.textures) - 1

    def spectral_neutral(self, reflectance):
        """texture.NewSpectralNeutral (spectral_constant.go:83-96)."""
        r = float(f32(reflectance))
        return self.spectral_tabulated(NEUTRAL_WAVELENGTHS, [r] * len(NEUTRAL_WAVELENGTHS), proto_float=False)

    def spectral_spd(self, wavelengths, values):
        """A float64 SPD from the light-source library (lightsources.go)."""
        return self.spectral_tabulated(wavelengths, values, proto_float=False)

    # ------------------------------------------------------------ materials
    def _mat(self, **kw):
        m = N.Material(albedo_tex=-1, spectral_tex=-1, normal_tex=-1, roughness_tex=-1, metalness_tex=-1,
                       absorb_tex=-1)
        for k, v in kw.items():
            if k == "rgb":
                m.rgb[:] = [float(x) for x in v]
            else:
                setattr(m, k, v)
        self.materials.append(m)
        return len(self.materials) - 1

    def lambert(self, albedo=-1, spectral=-1):
        return self._mat(kind=N.MAT_LAMBERT, albedo_tex=albedo, spectral_tex=spectral)

    def diffuse_light(self, emit=-1, spectral=-1):
        return self._mat(kind=N.MAT_DIFFUSE_LIGHT, albedo_tex=emit, spectral_tex=spectral)

    def dielectric(self, ref_idx=0.0, spectral_refidx=-1, absorb=(0.0, 0.0, 0.0), spectral_absorb=-1,
                   beer_lambert=False):
        """transport.toSceneDielectricMaterial (transport.go:306-360)."""
        absorb = [float(v) for v in f32(absorb)]
        flags = 0
        if spectral_refidx < 0 and any(a != 0 for a in absorb):
            flags = N.MATF_BEER_LAMBERT  # NewColoredDielectric
        elif spectral_refidx >= 0 and spectral_absorb < 0 and beer_lambert:
            flags = N.MATF_BEER_LAMBERT  # NewSpectralDielectric(refidx, computeBeerLambert)
        return self._mat(kind=N.MAT_DIELECTRIC, ref_idx=float(f32(ref_idx)), spectral_tex=spectral_refidx,
                         absorb_tex=spectral_absorb, rgb=absorb, flags=flags)

    def isotropic(self, albedo):
        """material.NewIsotropic (isotropic.go; transport.go:269-278): RGB albedo texture."""
        return self._mat(kind=N.MAT_ISOTROPIC, albedo_tex=albedo)

    def metal(self, albedo, fuzz):
        return self._mat(kind=N.MAT_METAL, rgb=[float(v) for v in f32(albedo)], fuzz=float(f32(fuzz)))

    def pbr(self, albedo, normal=-1, roughness=-1, metalness=-1, spectral=-1):
        return self._mat(kind=N.MAT_PBR, albedo_tex=albedo, normal_tex=normal, roughness_tex=roughness,
                         metalness_tex=metalness, spectral_tex=spectral)

    # -------------------------------------------------------------- objects
    def add_triangles(self, v0, v1, v2, material, uv=None):
        v0, v1, v2 = (f32(np.asarray(v, np.float64).reshape(-1, 3)) for v in (v0, v1, v2))
        n = v0.shape[0]
        t = np.zeros(n, TRI_DTYPE)
        t["v0"], t["v1"], t["v2"] = v0, v1, v2
        if uv is not None:
            t["uv"] = f32(np.asarray(uv, np.float64).reshape(n, 6))
        t["material"] = material
        self.tris = np.concatenate([self.tris, t])

    def add_sphere(self, center, radius, material):
        s = np.zeros(1, SPHERE_DTYPE)
        s["center"] = f32(center)
        s["radius"] = f32(radius)
        s["material"] = material
        self.spheres = np.concatenate([self.spheres, s])

    def set_camera(self, look_from, look_at, vup, vfov, aspect, aperture, focus_dist, time0, time1, exposure=1.0):
        c = N.CameraIn()
        c.look_from[:] = [float(v) for v in f32(look_from)]
        c.look_at[:] = [float(v) for v in f32(look_at)]
        c.vup[:] = [float(v) for v in f32(vup)]
        c.vfov, c.aspect, c.aperture, c.focus_dist, c.time0, c.time1, c.exposure = (
            float(f32(v)) for v in (vfov, aspect, aperture, focus_dist, time0, time1, exposure))
        self.camera = c

    # --------------------------------------------------------------- export
    def to_input(self, aspect_override=0.0, bvh_seed=12345):
        """izpi_scene_input; the returned object keeps every buffer alive."""
        keep = {}
        keep["tris"] = np.ascontiguousarray(self.tris)
        keep["spheres"] = np.ascontiguousarray(self.spheres)
        keep["mats"] = (N.Material * max(1, len(self.materials)))(*self.materials)
        keep["texs"] = (N.Texture * max(1, len(self.textures)))(*self.textures)
        keep["texels"] = np.concatenate(self.texels) if self.texels else np.zeros(0)
        keep["spd_wl"] = np.asarray(self.spd_wl, np.float64)
        keep["spd_val"] = np.asarray(self.spd_val, np.float64)
        si = N.SceneInput()
        si.num_tris = len(self.tris)
        si.num_spheres = len(self.spheres)
        si.num_materials = len(self.materials)
        si.num_textures = len(self.textures)
        si.num_spd = len(self.spd_wl)
        si.num_texels = keep["texels"].size
        si.tris = keep["tris"].ctypes.data if si.num_tris else None
        si.spheres = keep["spheres"].ctypes.data if si.num_spheres else None
        si.materials = C.cast(keep["mats"], C.POINTER(N.Material))
        si.textures = C.cast(keep["texs"], C.POINTER(N.Texture))
        si.texels = _ptr(keep["texels"], C.c_double)
        si.spd_wavelengths = _ptr(keep["spd_wl"], C.c_double)
        si.spd_values = _ptr(keep["spd_val"], C.c_double)
        si.camera = self.camera
        si.aspect_override = float(aspect_override)
        si.bvh_seed = int(bvh_seed)
        keep["input"] = si
        return _Input(si, keep)


class _Input:
    def __init__(self, si, keep):
        self.struct = si
        self._keep = keep

    def ref(self):
        return C.byref(self.struct)


class HostScene:
    """izpi_host_build_scene result: the flattened izpi_scene_desc (Go host's
    transport.ToScene + NewBVH4 output)."""

    def __init__(self, scene, aspect_override=0.0, bvh_seed=12345, skip_bvh=False):
        L = N.lib()
        self._input = scene.to_input(aspect_override, bvh_seed)
        h = C.c_void_p()
        rc = L.izpi_host_build_scene_ex(self._input.ref(), N.HOST_SKIP_BVH if skip_bvh else 0, C.byref(h))
        if rc != 0:
            raise RuntimeError("izpi_host_build_scene failed (%d): %s" % (rc, L.izpi_host_last_error().decode()))
        self.handle = h
        self.desc = L.izpi_host_scene_desc(h).contents
        self.stack_bound = L.izpi_host_scene_stack_bound(h)
        self.build_ms = L.izpi_host_scene_build_ms(h)

    def prim_boxes(self):
        """[num_tris + num_spheres][6] f64 boxes the BVH is built over."""
        d = self.desc
        out = np.zeros((d.num_tris + d.num_spheres, 6))
        N.lib().izpi_host_scene_prim_boxes(self.handle, out.ctypes.data_as(N.c_double_p))
        return out

    def set_bvh(self, nodes, order):
        """Attach a BVH4 built elsewhere (e.g. izpi_gpu_build_bvh4)."""
        nodes = np.ascontiguousarray(nodes, np.uint8).reshape(-1, 128)
        order = np.ascontiguousarray(order, np.uint32)
        self._bvh_keep = (nodes, order)  # the host scene copies them; kept for inspection
        rc = N.lib().izpi_host_scene_set_bvh(self.handle, nodes.ctypes.data_as(C.POINTER(N.BVH4Node)), len(nodes),
                                              order.ctypes.data_as(N.c_uint32_p))
        if rc != 0:
            raise RuntimeError("izpi_host_scene_set_bvh failed (%d): %s" % (rc, N.lib().izpi_host_last_error().decode()))
        self.desc = N.lib().izpi_host_scene_desc(self.handle).contents
        self.stack_bound = N.lib().izpi_host_scene_stack_bound(self.handle)

    def set_flags(self, flags):
        """izpi_host_scene_set_flags: the descriptor's IZPI_SCENE_* flags."""
        rc = N.lib().izpi_host_scene_set_flags(self.handle, int(flags))
        if rc != 0:
            raise RuntimeError("izpi_host_scene_set_flags failed (%d): %s" % (rc, N.lib().izpi_host_last_error().decode()))
        self.desc = N.lib().izpi_host_scene_desc(self.handle).contents

    def nodes(self):
        d = self.desc
        buf = (N.BVH4Node * d.num_nodes).from_address(C.addressof(d.nodes.contents))
        return np.frombuffer(buf, dtype=np.uint8).reshape(d.num_nodes, 128).copy()

    def prim_refs(self):
        d = self.desc
        return np.ctypeslib.as_array(d.prim_ref, shape=(d.num_prims,)).copy()

    def light_refs(self):
        d = self.desc
        return np.ctypeslib.as_array(d.light_ref, shape=(d.num_lights,)).copy() if d.num_lights else np.zeros(0, np.uint32)

    def close(self):
        if self.handle:
            N.lib().izpi_host_scene_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
