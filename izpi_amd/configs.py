"""The benchmark configurations of BASELINE.json, as deterministic
synthetic scenes (no files needed).

C1  Cornell box, Lambert walls + diffuse light, Colour sampler, 200x200x16
C2  same box, 1024^2 x 256
C3  box + synthetic ~820k-triangle "dragon" (displaced cube-sphere), 1024^2 x 512
C4  PBR box (procedural albedo / normal / roughness textures), 1920x1080 x 1024
C5  spectral glass scene of cmd/izpi/examples/cornell_box_transparent_pyramid_spectral.pbtxt,
    2048^2 x 4096

Geometry of the box: the 12 wall/light triangles of the example .pbtxt (consistent
inward winding, no duplicated floor: SURVEY.md appendix A12). RGB materials follow
scenes.CornellBoxRGB (scenes/scenes.go:934): White 0.73, Green (0,0.73,0),
Red (0.73,0,0), light 15. Camera (50,50,-140)->(50,50,0), vfov 40.
"""
import json
import math
from dataclasses import dataclass
from pathlib import Path

import numpy as np

from .scene import Scene, f32

DATA = Path(__file__).resolve().parent / "data"

# (v0, v1, v2, material, uv) from the example pbtxt, in file order
_BOX = [
    ((100, 0, 100), (0, 0, 100), (100, 100, 100), "White", ((0, 0), (1, 0), (1, 1))),
    ((100, 100, 100), (0, 0, 100), (0, 100, 100), "White", None),
    ((0, 0, 0), (0, 0, 100), (100, 0, 100), "White", None),
    ((0, 0, 0), (100, 0, 100), (100, 0, 0), "White", None),
    ((0, 100, 0), (100, 100, 0), (100, 100, 100), "White", None),
    ((0, 100, 100), (0, 100, 0), (100, 100, 100), "White", None),
    ((33, 99, 33), (66, 99, 33), (66, 99, 66), "light", None),
    ((33, 99, 33), (66, 99, 66), (33, 99, 66), "light", None),
    ((0, 100, 100), (0, 0, 0), (0, 100, 0), "Green", None),
    ((0, 100, 100), (0, 0, 100), (0, 0, 0), "Green", None),
    ((100, 0, 0), (100, 100, 100), (100, 100, 0), "Red", None),
    ((100, 0, 0), (100, 0, 100), (100, 100, 100), "Red", None),
]

# ten r=10 glass spheres of the example pbtxt
_GLASS = [(30, 15, 30), (50, 15, 30), (70, 15, 30), (40, 15, 50), (60, 15, 50), (50, 15, 70),
          (40, 28, 40), (60, 28, 40), (50, 28, 60), (50, 42, 50)]
_REFIDX_WL = [380, 400, 420, 440, 460, 480, 500, 520, 540, 560, 580, 600, 620, 640, 660, 680, 700, 720, 740, 750]
_REFIDX_V = [1.52, 1.51, 1.51, 1.5, 1.5, 1.49, 1.49, 1.48, 1.48, 1.47, 1.47, 1.46, 1.46, 1.45, 1.45, 1.44, 1.44,
             1.43, 1.43, 1.42]


def spectral_tables():
    return json.loads((DATA / "spectral_tables.json").read_text())


def add_box(scene, mats):
    for v0, v1, v2, m, uv in _BOX:
        uvs = None
        if uv is not None:
            uvs = [uv[0][0], uv[0][1], uv[1][0], uv[1][1], uv[2][0], uv[2][1]]
        scene.add_triangles([v0], [v1], [v2], mats[m], uv=[uvs] if uvs else None)


def rgb_box_materials(scene):
    return {
        "White": scene.lambert(albedo=scene.constant((0.73, 0.73, 0.73))),
        "Green": scene.lambert(albedo=scene.constant((0.0, 0.73, 0.0))),
        "Red": scene.lambert(albedo=scene.constant((0.73, 0.0, 0.0))),
        "light": scene.diffuse_light(emit=scene.constant((15.0, 15.0, 15.0))),
    }


def cornell_camera(scene, aspect):
    scene.set_camera((50, 50, -140), (50, 50, 0), (0, 1, 0), 40, aspect, 0, 10, 0, 1, 1.0)


def cornell_rgb(aspect=1.0):
    s = Scene("cornell_rgb")
    add_box(s, rgb_box_materials(s))
    cornell_camera(s, aspect)
    return s


def dragon_mesh(n=261, center=(50.0, 0.0, 60.0), radius=22.0, rot_y_deg=-60.0):
    """Deterministic closed stand-in for the Stanford dragon (the mesh is not in the
    reference checkout): a cube-sphere with 6*n*n quads (12*n*n triangles; n=261 ->
    817,452) radially displaced by smooth sum-of-sines bumps, rotated about Y as in
    scenes/spectral.go:644-646, resting on the box floor. Outward winding. Vertices
    are rounded to float32 like proto Vec3 fields."""
    g = np.linspace(-1.0, 1.0, n + 1)
    a, b = np.meshgrid(g, g, indexing="ij")
    one = np.ones_like(a)
    tris = []
    for axis in range(3):
        for sgn in (1.0, -1.0):
            p = [None, None, None]
            p[axis] = sgn * one
            p[(axis + 1) % 3] = a
            p[(axis + 2) % 3] = b
            d = np.stack(p, -1)
            d = d / np.linalg.norm(d, axis=-1, keepdims=True)
            bump = (0.08 * np.sin(5 * d[..., 0]) * np.sin(4 * d[..., 1] + 0.5) * np.sin(6 * d[..., 2])
                    + 0.05 * np.sin(11 * d[..., 0] + 3 * d[..., 2]) + 0.03 * np.cos(17 * d[..., 1]))
            pos = d * (radius * (1.0 + bump))[..., None]
            q00, q10, q01, q11 = pos[:-1, :-1], pos[1:, :-1], pos[:-1, 1:], pos[1:, 1:]
            tris.append(np.stack([q00, q10, q11], -2).reshape(-1, 3, 3))
            tris.append(np.stack([q00, q11, q01], -2).reshape(-1, 3, 3))
    T = np.concatenate(tris)
    nrm = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    inward = (nrm * T.mean(1)).sum(-1) < 0
    T[inward] = T[inward][:, [0, 2, 1]]
    th = math.radians(rot_y_deg)
    rot = np.array([[math.cos(th), 0.0, math.sin(th)], [0.0, 1.0, 0.0], [-math.sin(th), 0.0, math.cos(th)]])
    T = T @ rot.T
    T[..., 1] -= T[..., 1].min() - 0.05
    T += np.array([center[0], center[1], center[2]])
    T = f32(T)
    return T[:, 0], T[:, 1], T[:, 2]


def cornell_dragon(aspect=1.0, n=261):
    s = Scene("cornell_dragon")
    mats = rgb_box_materials(s)
    add_box(s, mats)
    v0, v1, v2 = dragon_mesh(n)
    s.add_triangles(v0, v1, v2, mats["White"])
    cornell_camera(s, aspect)
    return s


def _pbr_textures(scene, res=512, seed_phase=0.0):
    y, x = np.mgrid[0:res, 0:res] / float(res)
    checker = ((np.floor(x * 8) + np.floor(y * 8)) % 2)
    alb = np.stack([0.25 + 0.5 * checker, 0.3 + 0.4 * (1 - checker), 0.35 + 0.2 * np.sin(6.28 * x + seed_phase) ** 2,
                    np.ones_like(x)], -1)
    hx = 0.5 + 0.35 * np.cos(2 * math.pi * 6 * x)
    hy = 0.5 + 0.35 * np.cos(2 * math.pi * 6 * y)
    nrm = np.stack([hx, hy, np.full_like(x, 0.9), np.ones_like(x)], -1)
    rough = np.stack([0.2 + 0.6 * checker, 0.2 + 0.6 * checker, 0.2 + 0.6 * checker, np.ones_like(x)], -1)
    metal = np.stack([0.5 * (1 - checker)] * 3 + [np.ones_like(x)], -1)
    return (scene.image(alb), scene.image(nrm), scene.image(rough), scene.image(metal))


def cornell_pbr(aspect=1920.0 / 1080.0, res=512):
    """C4: PBR walls (albedo/normal/roughness/metalness image textures, nearest texel
    lookup of image.go:73-101) with UVs spanning each wall, RGB diffuse light."""
    s = Scene("cornell_pbr")
    a, n, r, m = _pbr_textures(s, res)
    a2, n2, r2, m2 = _pbr_textures(s, res, 1.0)
    mats = {
        "White": s.pbr(a, normal=n, roughness=r, metalness=m),
        "Green": s.pbr(s.constant((0.1, 0.6, 0.1)), normal=n2, roughness=r2),
        "Red": s.pbr(s.constant((0.6, 0.1, 0.1)), normal=n2, roughness=r2),
        "light": s.diffuse_light(emit=s.constant((15.0, 15.0, 15.0))),
    }
    for v0, v1, v2, mname, _ in _BOX:
        P = np.array([v0, v1, v2], np.float64)
        # planar UVs over the wall: pick the two varying axes
        span = P.max(0) - P.min(0)
        ax = [i for i in range(3) if span[i] > 0][:2]
        uv = [(P[k, ax[0]] / 100.0, P[k, ax[1]] / 100.0) for k in range(3)]
        s.add_triangles([v0], [v1], [v2], mats[mname], uv=[[c for p in uv for c in p]])
    s.add_sphere((30, 20, 40), 20, s.pbr(a2, normal=n, roughness=r2, metalness=m2))
    s.add_sphere((72, 15, 60), 15, s.metal((0.8, 0.8, 0.9), 0.05))
    cornell_camera(s, aspect)
    return s


def cornell_glass_spectral(aspect=1.0):
    """C5: cmd/izpi/examples/cornell_box_transparent_pyramid_spectral.pbtxt."""
    tabs = spectral_tables()
    s = Scene("cornell_glass_spectral")
    mats = {
        "Green": s.lambert(spectral=s.spectral_gaussian(0.9, 540, 40)),
        "Red": s.lambert(spectral=s.spectral_gaussian(0.9, 640, 40)),
        "White": s.lambert(spectral=s.spectral_neutral(0.73)),
        "light": s.diffuse_light(spectral=s.spectral_spd(tabs["cie_wavelengths"],
                                                          tabs["light_sources"]["cie_f1_daylight_fluorescent"])),
    }
    glass = s.dielectric(spectral_refidx=s.spectral_tabulated(_REFIDX_WL, _REFIDX_V),
                         spectral_absorb=s.spectral_neutral(0.01))
    add_box(s, mats)
    for c in _GLASS:
        s.add_sphere(c, 10, glass)
    s.set_camera((50, 50, -120), (50, 50, 50), (0, 1, 0), 35, aspect, 0, 10, 0, 1, 1.0)
    return s


def cornell_rgb_pbtxt(aspect=1.0):
    """The RGB Cornell box of C1 as transport.Scene text (the format the C++ ingestion
    reads; RGB materials of scenes.CornellBoxRGB, scenes.go:934)."""
    def v(name, p):
        return "%s { x: %r y: %r z: %r }" % (name, float(p[0]), float(p[1]), float(p[2]))
    out = ['name: "cornell_rgb"', "colour_representation: RGB",
           "camera { %s %s %s vfov: 40 aspect: %r focusdist: 10 time1: 1 exposure: 1 }"
           % (v("lookfrom", (50, 50, -140)), v("lookat", (50, 50, 0)), v("vup", (0, 1, 0)), float(aspect))]
    for name, rgb, kind in (("White", (0.73, 0.73, 0.73), "lambert"), ("Green", (0, 0.73, 0), "lambert"),
                            ("Red", (0.73, 0, 0), "lambert"), ("light", (15, 15, 15), "diffuselight")):
        prop = "lambert { albedo { constant { %s } } }" % v("value", rgb) if kind == "lambert" else \
            "diffuselight { emit { constant { %s } } }" % v("value", rgb)
        out.append('materials { key: "%s" value { name: "%s" type: %s %s } }'
                   % (name, name, "LAMBERT" if kind == "lambert" else "DIFFUSE_LIGHT", prop))
    tris = []
    for v0, v1, v2, m, uv in _BOX:
        t = "triangles { %s %s %s" % (v("vertex0", v0), v("vertex1", v1), v("vertex2", v2))
        if uv is not None:
            t += " uv0 { u: %r v: %r } uv1 { u: %r v: %r } uv2 { u: %r v: %r }" % tuple(float(c) for p in uv for c in p)
        tris.append(t + ' material_name: "%s" }' % m)
    out.append("objects {\n  %s\n}" % "\n  ".join(tris))
    return "\n".join(out) + "\n"


def cornell_obj(path, aspect=1.0):
    """C3 with a mesh from a Wavefront OBJ file (e.g. the Stanford dragon, which the
    reference loads from meshes/dragon_tri.obj and this checkout lacks): parsed and
    transformed as scenes/spectral.go:639-657 does (Scale 90, Rotate Y -60 deg,
    Translate (50, 25.1, 60), GroupToTransportTrianglesWithMaterial WITHOUT_UVS), then
    streamed into the RGB Cornell box with the White Lambert material."""
    from . import ingest
    mesh = ingest.WavefrontObj.from_file(path)
    mesh.scale(90.0, 90.0, 90.0)
    mesh.rotate(0.0, -ingest.go_radians(60), 0.0)
    mesh.translate(50.0, 25.1, 60.0)
    scene = ingest.ProtoScene(cornell_rgb_pbtxt(aspect).encode())
    for g in range(mesh.info()["num_groups"]):
        scene.add_triangles(mesh.group_to_transport_triangles(g, without_uvs=True), "White")
    return scene


@dataclass
class Config:
    name: str
    width: int
    height: int
    spp: int
    sampler: int
    build: object
    max_depth: int = 50


def configs():
    from ._native import SAMPLER_COLOUR, SAMPLER_SPECTRAL
    return {
        "C1": Config("C1 cornell 200x200x16", 200, 200, 16, SAMPLER_COLOUR, lambda: cornell_rgb(1.0)),
        "C2": Config("C2 cornell 1024x1024x256", 1024, 1024, 256, SAMPLER_COLOUR, lambda: cornell_rgb(1.0)),
        "C3": Config("C3 cornell+dragon 1024x1024x512", 1024, 1024, 512, SAMPLER_COLOUR, lambda: cornell_dragon(1.0)),
        "C4": Config("C4 PBR cornell 1920x1080x1024", 1920, 1080, 1024, SAMPLER_COLOUR,
                     lambda: cornell_pbr(1920.0 / 1080.0)),
        "C5": Config("C5 spectral glass 2048x2048x4096", 2048, 2048, 4096, SAMPLER_SPECTRAL,
                     lambda: cornell_glass_spectral(1.0)),
    }
