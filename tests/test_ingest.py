"""Scene ingestion: transport.Scene text/binary decoding,
transport.ToScene's conversion rules, the light-source library and the Wavefront OBJ
loader (izpi_amd/csrc/scene_io.cpp). CPU only.

Pinned by the reference's own fixtures where they exist:
  * wavefront_test.go:13-98 (testdata/cube.obj + cube.mtl, copied to tests/golden/wavefront/):
    the parsed WavefrontObj is transcribed below field by field;
  * cmd/izpi/examples/cornell_box_transparent_pyramid_spectral.pbtxt (izpi_amd/data/scenes/):
    must yield the same flattened scene and the same oracle image as the C5 restatement;
  * transport_test.go:140-191 (light-source library, CIE A fallback) and :12-117 (PBR in
    RGB and spectral representations).
The rest (prototext corner cases, wire format, transform arithmetic) is checked against
restatements in this file; transforms use the oracle's Go-math restatement.
"""
import ctypes as C
import struct
from fractions import Fraction
from pathlib import Path

import numpy as np
import pytest

from izpi_amd import _native as N
from izpi_amd import configs, ingest
from izpi_amd.scene import HostScene

ROOT = Path(__file__).resolve().parents[1]
CUBE = ROOT / "tests" / "golden" / "wavefront" / "cube.obj"
EXAMPLE = ROOT / "izpi_amd" / "data" / "scenes" / "cornell_box_transparent_pyramid_spectral.pbtxt"


# ----------------------------------------------------------------- Wavefront OBJ
def test_cube_obj_matches_reference_test():
    """wavefront_test.go:13-76 (TestNewObjFromReader, "A simple cube")."""
    o = ingest.WavefrontObj.from_file(CUBE)
    info = o.info()
    assert info["object_name"] == "Cube"
    assert info["has_normals"] == 1 and info["has_uv"] == 1
    assert info["centre"] == (0.0, 0.0, 0.0)
    v, vn, vt = o.vertices()
    assert v.tolist() == [[-0.5, -0.5, -0.5], [0.5, -0.5, -0.5], [0.5, -0.5, 0.5], [-0.5, -0.5, 0.5],
                          [-0.5, 0.5, -0.5], [0.5, 0.5, -0.5], [0.5, 0.5, 0.5], [-0.5, 0.5, 0.5]]
    assert vn.tolist() == [[0, -1, 0], [0, 0, -1], [1, 0, 0], [0, 0, 1], [-1, 0, 0], [0, 1, 0]]
    assert vt.tolist() == [[0.25, 0], [0.5, 0], [0.25, 0.333333], [0.5, 0.333333], [1, 0.666667], [0.75, 0.666667],
                           [1, 0.333333], [0.75, 0.333333], [0.5, 0.666667], [0.25, 0.666667], [0, 0.666667],
                           [0, 0.333333], [0.25, 1], [0.5, 1]]
    assert o.materials() == {"Material1": {"Kd": [0.48, 0.48, 0.48], "Ka": [0.0, 0.0, 0.0], "Ks": [0.04, 0.04, 0.04],
                                           "Ns": 256.0, "Ni": 0.0, "D": 1.0, "Sharpness": 0, "Illum": 2}}
    groups = o.groups()
    assert len(groups) == 1
    g = groups[0]
    assert g["name"] == "Cube1" and g["material"] == "Material1" and g["face_type"] == N.OBJ_FACE_POLYGON
    assert g["faces"] == [
        [(1, 1, 1), (2, 2, 1), (4, 3, 1)], [(2, 2, 1), (3, 4, 1), (4, 3, 1)],
        [(5, 5, 2), (6, 6, 2), (1, 7, 2)], [(6, 6, 2), (2, 8, 2), (1, 7, 2)],
        [(6, 6, 3), (7, 9, 3), (2, 8, 3)], [(7, 9, 3), (3, 4, 3), (2, 8, 3)],
        [(7, 9, 4), (8, 10, 4), (3, 4, 4)], [(8, 10, 4), (4, 3, 4), (3, 4, 4)],
        [(8, 10, 5), (5, 11, 5), (4, 3, 5)], [(5, 11, 5), (1, 12, 5), (4, 3, 5)],
        [(5, 13, 6), (8, 10, 6), (6, 14, 6)], [(8, 10, 6), (7, 9, 6), (6, 14, 6)]]


def test_obj_parse_options_and_quirks(tmp_path):
    text = CUBE.read_text()
    o = ingest.WavefrontObj(text, str(tmp_path), N.OBJ_IGNORE_MATERIALS)  # no cube.mtl there: skipped
    assert o.materials() == {} and o.info()["ignore_materials"] == 1
    # faces before any group go to "default"; usemtl after g does not change the group
    o = ingest.WavefrontObj("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1// 2// 3//\ng A\nusemtl M\nf 1/0/0 2/0/0 3/0/0\n")
    gs = o.groups()
    assert [g["name"] for g in gs] == ["default", "A"] and gs[1]["material"] == ""
    assert gs[0]["faces"] == [[(1, 0, 0), (2, 0, 0), (3, 0, 0)]]  # missing fields parse as 0
    # no faces, no groups: the trailing group is nil (wavefront.go:228)
    assert ingest.WavefrontObj("v 0 0 0\n").groups() == [None]
    # CRLF lines (bufio.Scanner drops the '\r')
    o = ingest.WavefrontObj("o X\r\nv 1 2 3\r\n")
    assert o.info()["object_name"] == "X" and o.vertices()[0].tolist() == [[1, 2, 3]]


@pytest.mark.parametrize("text", ["v 0 0 0\nf 1 2 3\n",          # parseFaceVertex wants a/b/c
                                  "v 0  0 0\n",                  # strings.Split(" ") yields "" -> ParseFloat error
                                  "v 0 0 x\n",
                                  "v 0 0\n"])                    # index out of range in Go
def test_obj_parse_errors(text):
    with pytest.raises(RuntimeError):
        ingest.WavefrontObj(text)


def _go(op, x):
    from oracle import oracle as O
    return O.gomath(op, x)


def test_obj_transforms_follow_reference_arithmetic():
    """Translate/Scale/Rotate (wavefront.go:418-474) against a restatement using the
    oracle's Go math; the centre moves with Translate only."""
    o = ingest.WavefrontObj.from_file(CUBE)
    o.scale(90.0, 90.0, 90.0)
    beta = -ingest.go_radians(60)
    o.rotate(0.0, beta, 0.0)
    o.translate(50.0, 25.1, 60.0)
    v0 = np.array(ingest.WavefrontObj.from_file(CUBE).vertices()[0])
    ca, sa, cb, sb, cg, sg = _go(1, 0.0), _go(0, 0.0), _go(1, beta), _go(0, beta), _go(1, 0.0), _go(0, 0.0)
    exp = []
    for x, y, z in v0:
        x, y, z = (x - 0.0) * 90.0 + 0.0, (y - 0.0) * 90.0 + 0.0, (z - 0.0) * 90.0 + 0.0
        x1, y1, z1 = x * cg - y * sg, x * sg + y * cg, z
        x2, y2, z2 = x1 * cb + z1 * sb, y1, -x1 * sb + z1 * cb
        x3, y3, z3 = x2, y2 * ca - z2 * sa, y2 * sa + z2 * ca
        exp.append([x3 + 50.0, y3 + 25.1, z3 + 60.0])
    got = o.vertices()[0]
    assert got.tobytes() == np.array(exp).tobytes()
    assert o.info()["centre"] == (50.0, 25.1, 60.0)


def test_go_radians_is_the_exact_constant():
    # -(60.0 * math.Pi / 180.0) rounds pi/3 once; math.pi / 3 in float64 rounds twice
    assert ingest.go_radians(60) == float(ingest._GO_PI / 3)
    assert abs(ingest.go_radians(60) - np.pi / 3) <= np.spacing(np.pi / 3)


def test_group_to_transport_triangles():
    """GroupToTransportTrianglesWithMaterial: first three vertices per face, float32."""
    o = ingest.WavefrontObj("v 0.1 0.2 0.3\nv 1 0 0\nv 0 1 0\nv 1 1 0\nvt 0.1 0.7\nvt 1 0\nvt 0 1\nvt 1 1\n"
                            "g G\nf 1/1/0 2/2/0 3/3/0 4/4/0\n")
    t = o.group_to_transport_triangles(0)
    assert len(t) == 1  # quads are not split on this path
    f32 = lambda x: float(np.float32(x))  # noqa: E731
    assert t[0]["v0"].tolist() == [f32(0.1), f32(0.2), f32(0.3)]
    assert t[0]["uv"].tolist() == [f32(0.1), f32(0.7), 1.0, 0.0, 0.0, 1.0]
    assert o.group_to_transport_triangles(0, without_uvs=True)[0]["uv"].tolist() == [0.0] * 6
    cube = ingest.WavefrontObj.from_file(CUBE)
    assert len(cube.group_to_transport_triangles(0, without_uvs=True)) == 12


# --------------------------------------------------------------- transport.Scene
def test_example_pbtxt_equals_the_c5_restatement():
    """The reference's example scene parsed by the C++ ingestion == configs.C5."""
    s = ingest.ProtoScene.from_file(EXAMPLE)
    info = s.info()
    assert info["name"] == "Cornell Box Transparent Pyramid Spectral" and info["version"] == "1.0.0"
    assert info["colour_representation"] == N.COLOUR_SPECTRAL and s.sampler == N.SAMPLER_SPECTRAL
    assert (info["num_triangles"], info["num_spheres"], info["num_materials"]) == (12, 10, 5)
    wl, val = s.spectral_background()
    assert wl.tolist() == list(range(380, 751, 10)) and not val.any()
    a, b = HostScene(s, 1.0), HostScene(configs.cornell_glass_spectral(1.0), 1.0)
    assert a.nodes().tobytes() == b.nodes().tobytes()
    assert (a.prim_refs() == b.prim_refs()).all() and (a.light_refs() == b.light_refs()).all()
    from oracle import oracle as O
    req = N.RenderReq(width=24, height=24, spp=2, max_depth=50, sampler=N.SAMPLER_SPECTRAL, seed=12345)
    ia, sa = O.OracleScene(s, aspect_override=1.0).render(req, threads=4)
    ib, sb = O.OracleScene(configs.cornell_glass_spectral(1.0), aspect_override=1.0).render(req, threads=4)
    assert ia.tobytes() == ib.tobytes() and sa["rays"] == sb["rays"]


_BOX_RGB = """
name: "t"  # a comment
colour_representation: RGB
camera < lookfrom { x: 50 y: 50 z: -140 } lookat { x: 50, y: 50; } vup { y: 1 } vfov: 40 aspect: 1 focusdist: 10 time1: 1 exposure: 1.0 >
materials { key: "k1" value { name: "White" type: LAMBERT lambert { albedo { constant { value { x: 0.73 y: 0.73 z: 0.73 } } } } } }
materials { key: "k2" value { name: "light" type: DIFFUSE_LIGHT diffuselight { emit { constant { value { x: 15 y: 15 z: 15 } } } } } }
objects {
  triangles { vertex0 { x: 0 } vertex1 { x: 100 } vertex2 { y: 100 } material_name: "White" }
  triangles { vertex0 { x: 33 y: 99 z: 33 } vertex1 { x: 66 y: 99 z: 33 } vertex2 { x: 66 y: 99 z: 66 } material_name: "light" }
  spheres { center: { x: 50 y: 20 z: 50 } radius: 1e1 material_name: 'Wh\\x69te' }
}
"""


def _input(scene):
    return scene.to_input(1.0, 12345).struct


def test_text_format_features_and_transport_rules():
    s = ingest.ProtoScene(_BOX_RGB.encode())
    si = _input(s)
    assert (si.num_tris, si.num_spheres, si.num_materials) == (2, 1, 2)
    assert s.material_names() == ["White", "light"]  # registered under Material.name, not the map key
    assert si.spheres and C.cast(si.spheres, C.POINTER(N.SphereIn))[0].radius == 10.0
    assert si.camera.look_at[1] == 50.0 and si.camera.vup[1] == 1.0 and si.camera.aperture == 0.0
    mats = [si.materials[i] for i in range(si.num_materials)]
    tex = [si.textures[i] for i in range(si.num_textures)]
    assert mats[0].kind == N.MAT_LAMBERT and tex[mats[0].albedo_tex].value[0] == float(np.float32(0.73))
    assert mats[1].kind == N.MAT_DIFFUSE_LIGHT and tex[mats[1].albedo_tex].value[2] == 15.0


@pytest.mark.parametrize("text,msg", [
    ('name: "a" name: "b"', "is repeated"),
    ("nosuchfield: 1", "unknown field"),
    ('materials { key: "m" value { name: "m" type: LAMBERT lambert { albedo { constant {} } spectral_albedo { neutral {} } } } }',
     "oneof"),
    ("colour_representation: PURPLE", "enum"),
    ('camera { vfov: "x" }', "expected a value"),
    ('camera { vfov: 1.5.5 }', "invalid value"),
])
def test_text_format_errors(text, msg):
    with pytest.raises(RuntimeError, match=msg):
        ingest.ProtoScene(text.encode())


@pytest.mark.parametrize("mat,msg", [
    ('name: "m" type: LAMBERT', "lambert material must have"),
    ('name: "m" type: DIELECTRIC dielectric { }', "dielectric material must have"),
    ('name: "m" type: DIFFUSE_LIGHT', "diffuse light material must have"),
    ('name: "m" type: LAMBERT lambert { albedo { checker { } } }', "unknown texture type"),
    ('name: "m" type: LAMBERT lambert { albedo { image { filename: "a.png" } } }', "texture a.png not found"),
    ('name: "m" type: PBR pbr { albedo { constant { } } roughness { constant { } } metalness { constant { } } '
     'normal_map { constant { } } }', "unknown texture type"),  # the reference requires sss too
])
def test_transport_material_errors(mat, msg):
    s = ingest.ProtoScene(("materials { key: \"m\" value { %s } }" % mat).encode())
    with pytest.raises(RuntimeError, match=msg):
        s.to_input()


def test_transport_material_conversions():
    pbr = ('pbr { albedo { constant { value { x: 1 y: 0.5 z: 0.2 } } } roughness { constant { value { x: 0.5 } } } '
           'metalness { constant { } } normal_map { constant { value { x: 0.5 y: 0.5 z: 1 } } } sss { constant { } } }')
    text = """
materials { key: "a" value { name: "pbr" type: PBR %s } }
materials { key: "b" value { name: "glass" type: DIELECTRIC dielectric { refidx: 1.5 absorption_coeff { x: 0.1 } } } }
materials { key: "c" value { name: "glass2" type: DIELECTRIC dielectric { refidx: 1.5 } } }
materials { key: "d" value { name: "sg" type: DIELECTRIC dielectric { spectral_refidx { neutral { reflectance: 1.5 } }
                                                                        compute_beer_lambert_attenuation: true } } }
materials { key: "e" value { name: "metal" type: METAL metal { albedo { x: 0.8 y: 0.8 z: 0.9 } fuzz: 0.05 } } }
materials { key: "f" value { name: "skipped" } }
materials { key: "g" value { name: "gauss" type: LAMBERT lambert { spectral_albedo { gaussian { peak_value: 0.9 center_wavelength: 540 width: 40 } } } } }
""" % pbr
    for rep in ("RGB", "SPECTRAL"):
        s = ingest.ProtoScene(("colour_representation: %s\n" % rep + text).encode())
        si = _input(s)
        names = s.material_names()
        assert names == ["pbr", "glass", "glass2", "sg", "metal", "gauss"]  # UNSPECIFIED type: not converted
        m = {n: si.materials[i] for i, n in enumerate(names)}
        tex = [si.textures[i] for i in range(si.num_textures)]
        p = m["pbr"]
        assert p.kind == N.MAT_PBR and min(p.albedo_tex, p.roughness_tex, p.metalness_tex, p.normal_tex) >= 0
        if rep == "SPECTRAL":  # textureToSpectralTexture: neutral(luminance) (transport.go:500-507)
            t = tex[p.spectral_tex]
            lum = 0.299 * 1.0 + 0.587 * 0.5 + 0.114 * float(np.float32(0.2))
            assert t.kind == N.TEX_SPECTRAL_TABULATED and t.spd_count == 38
            assert si.spd_values[t.spd_offset] == lum
        else:
            assert p.spectral_tex == -1
        assert m["glass"].flags == N.MATF_BEER_LAMBERT and m["glass"].rgb[0] == float(np.float32(0.1))
        assert m["glass2"].flags == 0 and m["glass2"].ref_idx == 1.5
        assert m["sg"].flags == N.MATF_BEER_LAMBERT and m["sg"].spectral_tex >= 0
        assert m["metal"].kind == N.MAT_METAL and m["metal"].fuzz == float(np.float32(0.05))
        g = tex[m["gauss"].spectral_tex]
        assert g.kind == N.TEX_SPECTRAL_GAUSSIAN and (g.peak, g.center, g.width_nm) == (float(np.float32(0.9)), 540.0, 40.0)


def test_isotropic_materials():
    """toSceneIsotropicMaterial (transport.go:269-289): an RGB albedo converts; a spectral
    albedo is the reference's own error."""
    s = ingest.ProtoScene(b'materials { key: "i" value { name: "i" type: ISOTROPIC isotropic '
                          b'{ albedo { constant { value { x: 0.5 y: 0.25 z: 1 } } } } } }')
    si = _input(s)
    m = si.materials[0]
    assert m.kind == N.MAT_ISOTROPIC
    t = si.textures[m.albedo_tex]
    assert t.kind == N.TEX_CONSTANT and list(t.value) == [0.5, 0.25, 1.0]
    s = ingest.ProtoScene(b'materials { key: "i" value { name: "i" type: ISOTROPIC isotropic '
                          b'{ spectral_albedo { neutral { reflectance: 0.5 } } } } }')
    with pytest.raises(RuntimeError, match="spectral isotropic materials not yet implemented"):
        s.to_input()


def test_spectral_pbr_image_albedo_becomes_a_spectral_image():
    """textureToSpectralTexture (transport.go:486-497): a PBR image albedo under the
    Spectral sampler is read through NewSpectralImageFromImage of the same texels."""
    text = ('colour_representation: SPECTRAL\n'
            'image_textures { key: "k" value { filename: "albedo.exr" } }\n'
            'materials { key: "m" value { name: "m" type: PBR pbr { albedo { image { filename: "albedo.exr" } } '
            'roughness { constant { } } metalness { constant { } } normal_map { constant { } } sss { constant { } } } } }')
    s = ingest.ProtoScene(text.encode())
    rgba = np.arange(2 * 3 * 4, dtype=np.float64).reshape(2, 3, 4) / 24.0
    s.set_image("albedo.exr", rgba)
    si = _input(s)
    m = si.materials[0]
    a, t = si.textures[m.albedo_tex], si.textures[m.spectral_tex]
    assert a.kind == N.TEX_IMAGE and t.kind == N.TEX_SPECTRAL_IMAGE
    assert (t.width, t.height, t.texel_offset) == (a.width, a.height, a.texel_offset)


def test_displacement_is_outside_the_gpu_path():
    s = ingest.ProtoScene(b'materials { key: "w" value { name: "w" type: METAL } }\n'
                          b'objects { triangles { material_name: "w" operator: DISPLACE } }')
    with pytest.raises(RuntimeError, match="DISPLACE"):
        s.to_input()
    s = ingest.ProtoScene(b'objects { spheres { material_name: "nope" } }')
    with pytest.raises(RuntimeError, match="material nope not found"):
        s.to_input()


def test_image_textures_are_handed_over_by_filename():
    s = ingest.ProtoScene(b'image_textures { key: "k" value { filename: "albedo.exr" } }\n'
                          b'materials { key: "m" value { name: "m" type: LAMBERT lambert { albedo { image { filename: "albedo.exr" } } } } }')
    assert s.image_files() == ["albedo.exr"]
    rgba = np.arange(2 * 3 * 4, dtype=np.float64).reshape(2, 3, 4) / 24.0
    s.set_image("albedo.exr", rgba)
    si = _input(s)
    t = si.textures[si.materials[0].albedo_tex]
    assert (t.kind, t.width, t.height) == (N.TEX_IMAGE, 3, 2)
    assert np.ctypeslib.as_array(si.texels, shape=(si.num_texels,)).tolist() == rgba.ravel().tolist()


def test_streamed_obj_triangles_follow_embedded_ones():
    s = ingest.ProtoScene(_BOX_RGB.encode())
    cube = ingest.WavefrontObj.from_file(CUBE)
    cube.scale(20, 20, 20)
    cube.translate(50, 20, 50)
    s.add_triangles(cube.group_to_transport_triangles(0, without_uvs=True), "White")
    si = _input(s)
    assert si.num_tris == 14 and s.info()["num_streamed_triangles"] == 12
    tris = np.ctypeslib.as_array(C.cast(si.tris, C.POINTER(C.c_double)), shape=(14 * 16,)).reshape(14, 16)
    assert tris[2, :3].tolist() == [float(np.float32(v)) for v in cube.group_to_transport_triangles(0)[0]["v0"]]
    HostScene(s, 1.0)  # builds


# ------------------------------------------------------------------- wire format
def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _key(num, wt):
    return _varint(num << 3 | wt)


def _ld(num, payload):
    return _key(num, 2) + _varint(len(payload)) + payload


def _f32(num, x):
    return _key(num, 5) + struct.pack("<f", x)


def _vec3(num, x, y, z):
    return _ld(num, _f32(1, x) + _f32(2, y) + _f32(3, z))


def test_binary_scene_equals_text_scene():
    """The same scene in the wire format (.izpi): equal izpi_scene_input; packed and
    unpacked repeated floats; unknown fields skipped."""
    cam = _vec3(1, 50, 50, -140) + _vec3(2, 50, 50, 0) + _vec3(3, 0, 1, 0) + _f32(4, 40) + _f32(5, 1) + _f32(7, 10) + \
        _f32(9, 1) + _f32(10, 1.0)
    white = _ld(1, b"White") + _key(2, 0) + _varint(4) + _ld(6, _ld(1, _ld(3, _vec3(1, 0.73, 0.73, 0.73))))
    light = _ld(1, b"light") + _key(2, 0) + _varint(2) + _ld(4, _ld(1, _ld(3, _vec3(1, 15, 15, 15))))
    tri1 = _vec3(1, 0, 0, 0) + _vec3(2, 100, 0, 0) + _vec3(3, 0, 100, 0) + _ld(10, b"White")
    tri2 = _vec3(1, 33, 99, 33) + _vec3(2, 66, 99, 33) + _vec3(3, 66, 99, 66) + _ld(10, b"light")
    sph = _vec3(1, 50, 20, 50) + _f32(2, 10) + _ld(3, b"White")
    bg = _ld(1, struct.pack("<3f", 380, 390, 400)) + _f32(2, 0) + _f32(2, 0) + _f32(2, 0)  # packed + unpacked
    msg = (_ld(1, b"t") + _key(3, 0) + _varint(1) + _ld(4, cam) + _ld(5, _ld(1, b"k1") + _ld(2, white)) +
           _ld(5, _ld(1, b"k2") + _ld(2, light)) + _ld(8, _ld(1, tri1) + _ld(1, tri2) + _ld(2, sph)) + _ld(11, bg) +
           _ld(99, b"unknown") + _key(98, 0) + _varint(7))
    b = ingest.ProtoScene(msg, binary=True)
    t = ingest.ProtoScene(_BOX_RGB.encode())
    assert b.info()["name"] == "t" and b.info()["num_background"] == 3
    assert b.spectral_background()[0].tolist() == [380.0, 390.0, 400.0]
    bi, ti = _input(b), _input(t)
    for f in ("num_tris", "num_spheres", "num_materials", "num_textures"):
        assert getattr(bi, f) == getattr(ti, f), f
    assert bytes(bi.camera) == bytes(ti.camera)
    n = bi.num_tris
    rd = lambda si: np.ctypeslib.as_array(C.cast(si.tris, C.POINTER(C.c_uint8)), shape=(n * C.sizeof(N.TriIn),)).tobytes()  # noqa: E731
    assert rd(bi) == rd(ti)
    assert HostScene(b, 1.0).nodes().tobytes() == HostScene(t, 1.0).nodes().tobytes()
    with pytest.raises(RuntimeError, match="truncated"):
        ingest.ProtoScene(msg[:-3] + b"\x0a\x05ab", binary=True)


def test_scene_file_extensions(tmp_path):
    p = tmp_path / "s.json"
    p.write_text("{}")
    with pytest.raises(ValueError, match="Unknown scene file extension"):
        ingest.ProtoScene.from_file(p)


# ------------------------------------------------------------ light-source library
def test_light_source_library():
    import json
    data = json.loads((ROOT / "izpi_amd" / "data" / "spectral_tables.json").read_text())
    lib = data["light_source_library"]
    names = ingest.light_source_names()
    assert sorted(names) == sorted(lib) and len(names) == 42
    for name in ("hy_cree_llf_tm_30_90", "cie_f4_warm_white_fluorescent", "cie_f1_daylight_fluorescent"):
        assert ingest.light_source(name).tolist() == lib[name]
    assert ingest.light_source("nonexistent_light_source") is None


def _blackbody(T):
    """spectral.NewBlackbodySPD (spectral.go:275-318): exact constants, float64 steps,
    Go's exp from the oracle restatement."""
    from oracle import oracle as O
    h, c, k = Fraction("6.62607015e-34"), Fraction("2.99792458e8"), Fraction("1.380649e-23")
    c1, c2 = float(2 * h * c * c), float((h * c) / k)
    vals = []
    for wl in range(380, 751, 5):
        wm = float(wl) * 1e-9
        w5 = wm * wm * wm * wm * wm
        ex = c2 / (wm * T)
        vals.append(0.0 if ex > 700 else c1 / (w5 * (O.gomath(3, ex) - 1.0)))
    m = max(vals)
    return [v / m for v in vals]


@pytest.mark.parametrize("name,T", [("incandescent_2800k", 2800.0), ("halogen_3200k", 3200.0),
                                    ("cie_illuminant_a_2856k", 2856.0)])
def test_blackbody_light_sources(name, T):
    v = ingest.light_source(name)
    assert v.tolist() == _blackbody(T)
    assert v.max() == 1.0 and (v >= 0).all() and (v <= 1).all()  # transport_test.go:177-183


def test_unknown_light_source_falls_back_to_cie_a():
    """transport.go:474-478 / transport_test.go:151."""
    s = ingest.ProtoScene(b'materials { key: "l" value { name: "l" type: DIFFUSE_LIGHT diffuselight { spectral_emit {'
                          b' from_light_source_library { light_source_name: "nonexistent_light_source" } } } } }')
    si = _input(s)
    assert "nonexistent_light_source" in s.info()["warnings"]
    t = si.textures[si.materials[0].spectral_tex]
    vals = np.ctypeslib.as_array(si.spd_values, shape=(si.num_spd,))[t.spd_offset:t.spd_offset + t.spd_count]
    assert vals.tolist() == ingest.light_source("cie_illuminant_a_2856k").tolist()


def test_rgb_box_pbtxt_equals_c1_restatement():
    from oracle import oracle as O
    s = ingest.ProtoScene(configs.cornell_rgb_pbtxt(1.0).encode())
    a, b = HostScene(s, 1.0), HostScene(configs.cornell_rgb(1.0), 1.0)
    assert a.nodes().tobytes() == b.nodes().tobytes() and (a.light_refs() == b.light_refs()).all()
    req = N.RenderReq(width=20, height=20, spp=4, max_depth=50, sampler=N.SAMPLER_COLOUR, seed=12345)
    ia, _ = O.OracleScene(s, aspect_override=1.0).render(req, threads=4)
    ib, _ = O.OracleScene(configs.cornell_rgb(1.0), aspect_override=1.0).render(req, threads=4)
    assert ia.tobytes() == ib.tobytes()


def test_cornell_obj_streams_a_transformed_mesh(tmp_path):
    """configs.cornell_obj: an OBJ mesh through the reference's dragon pipeline
    (scenes/spectral.go:639-657) into the RGB box."""
    v0, v1, v2 = configs.dragon_mesh(n=6, center=(0, 0, 0), radius=0.3)
    verts = np.concatenate([v0, v1, v2])
    lines = ["o Mesh"] + ["v %r %r %r" % tuple(float(c) for c in p) for p in verts] + ["g G"]
    n = len(v0)
    lines += ["f %d// %d// %d//" % (i + 1, n + i + 1, 2 * n + i + 1) for i in range(n)]
    p = tmp_path / "mesh.obj"
    p.write_text("\n".join(lines) + "\n")
    s = configs.cornell_obj(p)
    si = _input(s)
    assert si.num_tris == 12 + n
    tris = np.ctypeslib.as_array(C.cast(si.tris, C.POINTER(C.c_double)), shape=(si.num_tris * 16,)).reshape(-1, 16)
    mesh = ingest.WavefrontObj.from_file(p)
    mesh.scale(90.0, 90.0, 90.0)
    mesh.rotate(0.0, -ingest.go_radians(60), 0.0)
    mesh.translate(50.0, 25.1, 60.0)
    v = mesh.vertices()[0].astype(np.float32).astype(np.float64)
    assert tris[12:, 0:3].tobytes() == v[:n].tobytes() and tris[12:, 3:6].tobytes() == v[n:2 * n].tobytes()
    HostScene(s, 1.0)


def test_parsers_survive_malformed_input():
    """Mutated scene files, truncated wire data and random OBJ lines end in a status code,
    never in a crash (the C++ parsers sit behind the C ABI)."""
    rng = np.random.default_rng(3)
    text = EXAMPLE.read_bytes()
    for _ in range(300):
        b = bytearray(text)
        for _ in range(rng.integers(1, 6)):
            i = int(rng.integers(0, len(b)))
            b[i] = int(rng.integers(0, 256))
        try:
            s = ingest.ProtoScene(bytes(b))
            s.to_input()
        except RuntimeError:
            pass
    wire = _ld(1, b"t") + _ld(4, _vec3(1, 1, 2, 3)) + _ld(8, _ld(2, _vec3(1, 5, 5, 5) + _f32(2, 1) + _ld(3, b"m")))
    for cut in range(len(wire)):
        try:
            ingest.ProtoScene(wire[:cut], binary=True).to_input()
        except RuntimeError:
            pass
    for _ in range(200):
        junk = bytes(rng.integers(0, 256, int(rng.integers(0, 64)), dtype=np.uint8))
        try:
            ingest.ProtoScene(junk, binary=True)
        except RuntimeError:
            pass
    deep = (b'materials { value { lambert { albedo { ' + b"checker { odd { " * 50 + b"}" * 100 + b"} } } }")
    with pytest.raises(RuntimeError, match="nested"):
        ingest.ProtoScene(deep)
    tex = b""
    for _ in range(100):  # Texture.checker.odd.checker.odd... (CheckerTexture nests Textures)
        tex = _ld(4, _ld(1, tex))
    with pytest.raises(RuntimeError, match="nested"):
        ingest.ProtoScene(_ld(5, _ld(2, _ld(6, _ld(1, tex)))), binary=True)
    lines = ["v 1 2 3", "vt 0.5 0.5", "vn 0 0 1", "f 1/1/1 1/1/1 1/1/1", "g x", "usemtl m", "o y", "f 1//", "v", "f",
             "g", "mtllib none.mtl", "s off", "# c"]
    for _ in range(200):
        obj = "\n".join(lines[int(k)] for k in rng.integers(0, len(lines), int(rng.integers(1, 20))))
        try:
            o = ingest.WavefrontObj(obj, "/nonexistent", 0)
            for g in range(o.info()["num_groups"]):
                try:
                    o.group_to_transport_triangles(g)
                except RuntimeError:
                    pass
        except RuntimeError:
            pass


def test_cli_constant_and_cpu_behaviour(tmp_path):
    """izpi-render (the C++ host over the C ABI): its dragon rotation constant is Go's,
    and on a host without a GPU it reads the scene, then fails cleanly at izpi_gpu_open."""
    import re
    import subprocess
    src = (ROOT / "izpi_amd" / "csrc" / "izpi_render.cpp").read_text()
    m = re.search(r"kMinus60Deg = (-0x[0-9a-fp.+-]+);", src)
    assert float.fromhex(m.group(1)) == -ingest.go_radians(60)
    cli = ROOT / "izpi_amd" / "_lib" / "izpi-render"
    bad = tmp_path / "scene.json"
    bad.write_text("{}")
    r = subprocess.run([str(cli), "--scene", str(bad)], capture_output=True, text=True)
    assert r.returncode == 1 and "Unknown scene file extension" in r.stderr
    r = subprocess.run([str(cli), "--scene", str(EXAMPLE), "--x", "8", "--y", "8", "--samples", "1"],
                       capture_output=True, text=True)
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        assert r.returncode == 1 and "izpi_gpu_open failed" in r.stderr, r.stderr


def test_wire_serializer_round_trips_every_scene():
    """izpi_scene_serialize (proto.Marshal's form): text -> wire -> parse gives the same
    izpi_scene_input and BVH; wire -> wire is a fixed point; hand-encoded wire bytes
    re-serialize to an equivalent message."""
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    texts = [_BOX_RGB, configs.cornell_rgb_pbtxt(1.0),
             (root / "izpi_amd" / "data" / "scenes" / "cornell_box_transparent_pyramid_spectral.pbtxt").read_text()]
    for text in texts:
        t = ingest.ProtoScene(text.encode())
        w = t.to_wire()
        b = ingest.ProtoScene(w, binary=True)
        assert b.to_wire() == w
        assert b.info() == t.info()
        bi, ti = _input(b), _input(t)
        for f in ("num_tris", "num_spheres", "num_materials", "num_textures", "num_spd", "num_texels"):
            assert getattr(bi, f) == getattr(ti, f), f
        assert bytes(bi.camera) == bytes(ti.camera)
        assert HostScene(b, 1.0).nodes().tobytes() == HostScene(t, 1.0).nodes().tobytes()
        mats = lambda si: b"".join(bytes(si.materials[i]) for i in range(si.num_materials))  # noqa: E731
        assert mats(bi) == mats(ti)


def test_wire_serializer_encoding_rules():
    """Field-number order, packed repeated floats, zero scalars omitted, oneof members kept."""
    s = ingest.ProtoScene(b'spectral_background { values: 0 values: 1 wavelengths: 380 wavelengths: 390 } '
                          b'name: "" camera { vfov: 0 aspect: 2 } '
                          b'materials { key: "g" value { name: "g" type: DIELECTRIC dielectric { refidx: 0 } } }')
    w = s.to_wire()
    cam = _ld(4, _f32(5, 2))                             # vfov 0 omitted
    mat = _ld(5, _ld(1, b"g") + _ld(2, _ld(1, b"g") + _key(2, 0) + _varint(1) + _ld(3, _f32(1, 0))))  # oneof refidx kept
    bg = _ld(11, _ld(1, struct.pack("<2f", 380, 390)) + _ld(2, struct.pack("<2f", 0, 1)))
    assert w == cam + mat + bg
