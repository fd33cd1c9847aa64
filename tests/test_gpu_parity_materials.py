"""GPU parity of the material and camera branches no benchmark config reaches: the
gfx950 kernels against the CPU oracle, bit for bit, counters included.

* RGB Dielectric (dielectric.go:156-181): plain glass (no absorption: no path-length
  ray) and coloured glass (NewColoredDielectric: Beer-Lambert with the extra World.Hit
  of calculatePathLength, :118-153), on spheres (flipped / unflipped normals, A16) and on
  triangles (normals never flipped).
* Spectral PBR (pbr.go:158-263): a spectral albedo texture, and the RGB albedo's
  luminance fallback (SpectralAlbedo, pbr.go:285-293), both with the x1.5 specular
  boost; normal / roughness / metalness image textures; PBR spheres and triangles.
* Thin-lens camera (camera.go:61-89): aperture > 0, so randomInUnitDisc's draws from the
  camera stream move the ray origin (A3), with a time interval.
"""
import numpy as np
import pytest

from izpi_amd import _native as N
from izpi_amd import configs
from izpi_amd.renderer import GPURenderer
from izpi_amd.scene import Scene

from tests.test_gpu_parity import assert_parity, oracle_canvas

pytestmark = pytest.mark.gpu


def rgb_glass_box(coloured):
    s = Scene("rgb_glass")
    mats = configs.rgb_box_materials(s)
    configs.add_box(s, mats)
    glass = s.dielectric(ref_idx=1.5, absorb=(0.12, 0.05, 0.02) if coloured else (0.0, 0.0, 0.0))
    plain = s.dielectric(ref_idx=1.33)
    s.add_sphere((35, 20, 45), 18, glass)
    s.add_sphere((70, 15, 30), 12, plain)
    # a glass "pyramid" face pair (triangle normals are not flipped toward the ray)
    s.add_triangles([(40, 0, 20), (60, 45, 30)], [(80, 0, 20), (40, 0, 40)], [(60, 45, 30), (80, 0, 40)], glass)
    configs.cornell_camera(s, 1.0)
    return s


@pytest.mark.parametrize("coloured", [False, True])
def test_rgb_dielectric_bitwise(gpu, coloured):
    scene = rgb_glass_box(coloured)
    m = scene.materials[-2]
    assert bool(m.flags & N.MATF_BEER_LAMBERT) == coloured  # transport.go:306-360 mapping
    r = GPURenderer(scene, 48, 48, 8)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    # coloured glass traces path-length rays: more node visits per Sampler call than plain
    assert r.stats["sph_tests"] > 0
    r.close()


def spectral_pbr_box(spectral_albedo):
    """spectral_albedo: True = a Gaussian spectral albedo, "image" = the SpectralImage of the
    image albedo (transport.go:486-497), False = no spectral albedo (the luminance fallback)."""
    return _spectral_pbr_box(spectral_albedo)


def _spectral_pbr_box(spectral_albedo):
    tabs = configs.spectral_tables()
    s = Scene("spectral_pbr")
    alb, nrm, rough, metal = configs._pbr_textures(s, res=64)
    mats = {
        "Green": s.lambert(spectral=s.spectral_gaussian(0.9, 540, 40)),
        "Red": s.lambert(spectral=s.spectral_gaussian(0.9, 640, 40)),
        "light": s.diffuse_light(spectral=s.spectral_spd(tabs["cie_wavelengths"],
                                                          tabs["light_sources"]["cie_f1_daylight_fluorescent"])),
    }
    spec = (s.spectral_image(alb) if spectral_albedo == "image"
            else s.spectral_gaussian(0.8, 600, 60) if spectral_albedo else -1)
    # White walls: PBR with image textures and UVs (normal map through Triangle.Hit's TBN
    # and again in PBR.SpectralScatter, A19)
    mats["White"] = s.pbr(alb, normal=nrm, roughness=rough, metalness=metal, spectral=spec)
    for v0, v1, v2, mname, _ in configs._BOX:
        P = np.array([v0, v1, v2], np.float64)
        span = P.max(0) - P.min(0)
        ax = [i for i in range(3) if span[i] > 0][:2]
        uv = [(P[k, ax[0]] / 100.0, P[k, ax[1]] / 100.0) for k in range(3)]
        s.add_triangles([v0], [v1], [v2], mats[mname], uv=[[c for p in uv for c in p]])
    s.add_sphere((35, 20, 45), 18, s.pbr(s.constant((0.7, 0.5, 0.3)), roughness=rough, metalness=metal,
                                         spectral=spec))
    s.add_sphere((70, 15, 30), 12, s.pbr(alb, normal=nrm))
    configs.cornell_camera(s, 1.0)
    return s


@pytest.mark.parametrize("spectral_albedo", [True, False, "image"])
def test_spectral_pbr_bitwise(gpu, spectral_albedo):
    scene = spectral_pbr_box(spectral_albedo)
    r = GPURenderer(scene, 48, 48, 8, sampler=N.SAMPLER_SPECTRAL)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_SPECTRAL)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


@pytest.mark.parametrize("sampler", [N.SAMPLER_COLOUR, N.SAMPLER_SPECTRAL])
def test_thin_lens_camera_bitwise(gpu, sampler):
    if sampler == N.SAMPLER_COLOUR:
        scene = configs.cornell_dragon(1.0, n=30)
    else:
        scene = configs.cornell_glass_spectral()
    # aperture 4, focus at the box's middle, shutter [0.25, 0.75] (camera.go:28-89)
    scene.set_camera((50, 50, -140), (50, 50, 0), (0, 1, 0), 40, 1.0, 4.0, 190.0, 0.25, 0.75)
    r = GPURenderer(scene, 40, 40, 6, sampler=sampler)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 40, 40, 6, sampler)
    assert_parity(img, ref, r.stats, ostats)
    r.close()
    # the lens must matter: a pinhole render of the same scene differs
    scene.set_camera((50, 50, -140), (50, 50, 0), (0, 1, 0), 40, 1.0, 0.0, 190.0, 0.25, 0.75)
    pin, _ = oracle_canvas(scene, 40, 40, 6, sampler)
    assert pin.tobytes() != ref.tobytes()


def textured_lambert_box():
    """Lambert walls with an image albedo (image.go:73-101) and UVs, next to constant ones:
    Lambert + DiffuseLight only, so the MATSET_BASIC shader with full (colour) unwinding
    records runs; the all-constant scenes take MATSET_CONST's (material, s, p) records."""
    s = Scene("textured_lambert")
    alb, _, _, _ = configs._pbr_textures(s, res=32)
    mats = configs.rgb_box_materials(s)
    mats["White"] = s.lambert(albedo=alb)
    for v0, v1, v2, mname, _ in configs._BOX:
        P = np.array([v0, v1, v2], np.float64)
        span = P.max(0) - P.min(0)
        ax = [i for i in range(3) if span[i] > 0][:2]
        uv = [(P[k, ax[0]] / 100.0, P[k, ax[1]] / 100.0) for k in range(3)]
        s.add_triangles([v0], [v1], [v2], mats[mname], uv=[[c for p in uv for c in p]])
    s.add_sphere((35, 20, 45), 18, s.lambert(albedo=alb))
    configs.cornell_camera(s, 1.0)
    return s


@pytest.mark.parametrize("tune", [{}, {"rec_dense": 2, "pool_div": 100000}])
def test_textured_lambert_bitwise(gpu, tune):
    scene = textured_lambert_box()
    r = GPURenderer(scene, 48, 48, 8, tuning=N.tuning(**tune) if tune else None)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def isotropic_box(spectral):
    """Isotropic walls and spheres (isotropic.go): randomInUnitSphere draws, Cosine(N) in
    the mixture, ScatteringPDF 0 (so they pass on no light but keep every draw and ray);
    the Spectral sampler reads the RGB albedo's red (SpectralScatter)."""
    s = Scene("isotropic")
    alb, _, _, _ = configs._pbr_textures(s, res=32)
    if spectral:
        tabs = configs.spectral_tables()
        mats = {"White": s.lambert(spectral=s.spectral_neutral(0.73)),
                "Green": s.lambert(spectral=s.spectral_gaussian(0.9, 540, 40)),
                "Red": s.isotropic(s.constant((0.73, 0.2, 0.1))),
                "light": s.diffuse_light(spectral=s.spectral_spd(tabs["cie_wavelengths"],
                                                                  tabs["light_sources"]["cie_f1_daylight_fluorescent"]))}
    else:
        mats = configs.rgb_box_materials(s)
        mats["Red"] = s.isotropic(s.constant((0.73, 0.2, 0.1)))
    configs.add_box(s, mats)
    s.add_sphere((35, 20, 45), 18, s.isotropic(alb))
    s.add_sphere((70, 15, 30), 12, mats["White"])
    configs.cornell_camera(s, 1.0)
    return s


@pytest.mark.parametrize("sampler", [N.SAMPLER_COLOUR, N.SAMPLER_SPECTRAL])
def test_isotropic_bitwise(gpu, sampler):
    scene = isotropic_box(sampler == N.SAMPLER_SPECTRAL)
    r = GPURenderer(scene, 48, 48, 8, sampler=sampler)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, sampler)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def pbr_storage_box():
    """PBR textures in every device storage form: an RGBA image albedo, a gray image
    roughness (R = G = B in every texel: one double per texel on the device), a metalness
    image that is gray except in one texel (kept RGBA), and CONSTANT normal maps, which
    Triangle.Hit's TBN (triangle.go:250-264) and PBR.Scatter (pbr.go:65-91) apply like image
    ones; a Lambert wall keeps an image albedo next to them."""
    s = Scene("pbr_storage")
    res = 40
    y, x = np.mgrid[0:res, 0:res] / float(res)
    alb = np.stack([0.2 + 0.6 * x, 0.3 + 0.5 * y, 0.4 + 0.2 * x * y, np.ones_like(x)], -1)
    g = 0.1 + 0.8 * ((np.floor(x * 5) + np.floor(y * 5)) % 2)
    rough = np.stack([g, g, g, np.ones_like(x)], -1)
    m = 0.6 * x
    metal = np.stack([m, m, m, np.ones_like(x)], -1)
    metal[7, 11, 2] += 0.25  # one texel with B != R: the whole texture stays RGBA
    a_id, r_id, m_id = s.image(alb), s.image(rough), s.image(metal)
    nconst = s.constant((0.55, 0.45, 0.9))
    mats = configs.rgb_box_materials(s)
    mats["White"] = s.pbr(a_id, normal=nconst, roughness=r_id, metalness=m_id)
    mats["Green"] = s.lambert(albedo=a_id)
    for v0, v1, v2, mname, _ in configs._BOX:
        P = np.array([v0, v1, v2], np.float64)
        span = P.max(0) - P.min(0)
        ax = [i for i in range(3) if span[i] > 0][:2]
        uv = [(P[k, ax[0]] / 100.0, P[k, ax[1]] / 100.0) for k in range(3)]
        s.add_triangles([v0], [v1], [v2], mats[mname], uv=[[c for p in uv for c in p]])
    s.add_sphere((35, 20, 45), 18, s.pbr(s.constant((0.7, 0.5, 0.3)), normal=nconst, roughness=r_id))
    s.add_sphere((70, 15, 30), 12, s.pbr(a_id, normal=s.constant((0.5, 0.5, 1.0)), metalness=m_id))
    configs.cornell_camera(s, 1.0)
    return s


def test_pbr_texture_storage_forms_bitwise(gpu):
    scene = pbr_storage_box()
    r = GPURenderer(scene, 48, 48, 8)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


@pytest.mark.parametrize("albedo", [(-0.5, 0.7, -0.0), (0.9, float("inf"), 0.4), (-0.0, -0.0, -0.0)])
def test_zero_radiance_unwinding_signs_bitwise(gpu, albedo):
    """finish skips the record reads of a path whose terminal radiance is +0 when every
    level keeps a zero a zero (ZF_*): the sign each component ends with comes from the
    specular levels' attenuation signs below the first non-specular level. Metal spheres
    with negative, -0 and infinite albedo components (an infinite attenuation turns the
    zero into a NaN: those paths must unwind their records), glass, and an open box whose
    escaping paths meet the black background: bit-exact against the oracle's unwinding."""
    s = Scene("zero_signs")
    mats = configs.rgb_box_materials(s)
    configs.add_box(s, mats)
    m1 = s.metal(albedo, 0.05)
    m2 = s.metal((0.8, -0.3, 0.6), 0.0)
    s.add_sphere((35, 20, 45), 18, m1)
    s.add_sphere((70, 15, 30), 12, m2)
    s.add_sphere((55, 60, 40), 10, s.dielectric(ref_idx=1.5))
    configs.cornell_camera(s, 1.0)
    r = GPURenderer(s, 48, 48, 16)
    img = r.render()
    ref, ostats = oracle_canvas(s, 48, 48, 16, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    assert np.signbit(img[1:]).any()  # negative zeros reached the canvas
    r.close()


def test_zero_radiance_unwinding_spectral_signs_bitwise(gpu):
    """The Spectral sampler's zero-radiance shortcut (ZF_*): PBR surfaces with a negative
    spectral albedo (a Gaussian of scale -0.8) make specular levels that flip the sign of a
    zero radiance (att = albedo x 1.5, pbr.go:158-263), glass adds sign-keeping specular
    levels, the open box's escapes meet a black background: bit-exact against the oracle."""
    tabs = configs.spectral_tables()
    s = Scene("spectral_zero_signs")
    mats = {
        "Green": s.lambert(spectral=s.spectral_gaussian(0.9, 540, 40)),
        "Red": s.lambert(spectral=s.spectral_gaussian(0.9, 640, 40)),
        "light": s.diffuse_light(spectral=s.spectral_spd(tabs["cie_wavelengths"],
                                                          tabs["light_sources"]["cie_f1_daylight_fluorescent"])),
        "White": s.pbr(s.constant((0.7, 0.7, 0.7)), spectral=s.spectral_gaussian(-0.8, 560, 80)),
    }
    configs.add_box(s, mats)
    s.add_sphere((35, 20, 45), 18, s.pbr(s.constant((0.2, 0.5, 0.3)), spectral=s.spectral_gaussian(-0.5, 500, 50)))
    s.add_sphere((70, 15, 30), 12, s.dielectric(spectral_refidx=s.spectral_tabulated(configs._REFIDX_WL, configs._REFIDX_V)))
    configs.cornell_camera(s, 1.0)
    r = GPURenderer(s, 48, 48, 16, sampler=N.SAMPLER_SPECTRAL)
    img = r.render()
    ref, ostats = oracle_canvas(s, 48, 48, 16, N.SAMPLER_SPECTRAL)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def test_normal_map_tbn_kats_device(gpu):
    """mat3_test.go:10-54 on the device: each KAT's (t, b, n) as a normal-mapped PBR triangle
    (tests/test_oracle_kats.tbn_kat_scene); izpi_gpu_trace's hit normal (Triangle.Hit with
    its TBN, triangle.go:250-264) is the oracle's bit for bit and unit(MatrixVectorMul)."""
    import ctypes as C
    from oracle import oracle as O
    from tests.test_oracle_kats import KATS, tbn_kat_scene
    s, rays = tbn_kat_scene()
    r8 = np.zeros((len(rays), 8))
    r8[:, :6], r8[:, 6], r8[:, 7] = rays, 0.001, np.finfo(np.float64).max
    r = GPURenderer(s, 16, 16, 1)
    got = (N.Hit * len(r8))()
    assert N.lib().izpi_gpu_trace(r.ctx, r8.ctypes.data_as(C.POINTER(C.c_double)), len(r8), got) == 0
    o = O.OracleScene(s)
    want = o.trace(r8)
    for i, k in enumerate(KATS["mat3_tbn"]):
        assert got[i].hit and got[i].prim_ref == want[i].prim_ref
        assert bytes(got[i])[:72] == bytes(want[i])[:72], (i, list(got[i].normal), list(want[i].normal))
        w = np.array(k["want"], float)
        assert list(got[i].normal) == list(w / np.sqrt(np.dot(w, w)))
    o.close()
    r.close()



def test_dielectric_path_length_kat_device(gpu):
    """dielectric_test.go:47-84 on the device: calculatePathLength's length and clamps
    (dielectric.go:141-150, the code k_shade runs when a path-length ray returns) for the
    KAT's hit point and mock exit point (exactly 1.0), the clamps' ends and random pairs,
    bit for bit against the oracle's Dielectric.calculatePathLength (device op 14)."""
    import ctypes as C
    from oracle import oracle as O
    from tests.test_oracle_kats import KATS
    k = KATS["path_length"]
    rng = np.random.default_rng(14)
    hp = [k["hit_p"], k["hit_p"], k["hit_p"]] + list(rng.uniform(-20, 20, (200, 3)))
    ex = [k["mock_exit"], [0.5, 0.5, 0.55], [0.5, 0.5, 500.0]] + list(rng.uniform(-80, 80, (200, 3)))
    hp, ex = np.ascontiguousarray(hp, np.float64), np.ascontiguousarray(ex, np.float64)
    n = len(hp)
    r = GPURenderer(configs.cornell_rgb(), 8, 8, 1)
    out = np.zeros(n)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    assert N.lib().izpi_gpu_gomath(r.ctx, 14, dp(hp), dp(ex), n, dp(out)) == 0
    r.close()
    assert out[0] == k["expected"] and out[1] == 0.1 and out[2] == 100.0
    dirs = np.tile(np.array(k["hit_n"] + k["ray_o"] + k["ray_d"] + k["scattered_d"], np.float64), 1)
    for i in range(n):
        a = np.concatenate([hp[i], dirs])
        want = O.lib().oracle_path_length(O.dptr(a), O.dptr(np.ascontiguousarray(ex[i])))
        assert out[i].tobytes() == np.float64(want).tobytes(), (i, out[i], want)
